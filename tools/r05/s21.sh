#!/bin/bash
# REMOVE rounds the host knows of: IN 6 as the round's nibble launch (IN 2 not launched)
set -o pipefail
mkdir -p gpurun_out/r05
O=gpurun_out/r05
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_tier8.py tests/test_gpu_parity.py tests/test_gpu_remove_list.py -x -q --timeout 300 --timeout-method thread > $O/s21_tests.log 2>&1 || exit 1
timeout -k 10 300 python3 tools/r05/crash_rounds.py 30 > $O/s21_crash_rounds.jsonl 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/s21_bench.json 2> $O/s21_bench.err || exit 1
