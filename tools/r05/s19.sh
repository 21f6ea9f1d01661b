#!/bin/bash
# REMOVE rounds the host knows of (first round of a gh_step call after a
# detection) on a full-grid IN 6: parity, then the bench with its crash leg
set -o pipefail
mkdir -p gpurun_out/r05
O=gpurun_out/r05
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_tier8.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "remove or nibble_variants or timing or crash or d7" > $O/s19_tests.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/s19_bench.json 2> $O/s19_bench.err || exit 1
