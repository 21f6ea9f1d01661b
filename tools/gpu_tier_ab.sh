#!/bin/bash
# tier parity tests, then the tier A/B bench (tools/tier_ab.sh)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_tier8.py tests/test_gpu_plane.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_tier8.log 2>&1 &&
bash tools/tier_ab.sh "$@"
