#!/bin/bash
# The new tier-tombstone test, then the whole -m gpu suite and smoke.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 250 --timeout-method thread tests/test_gpu_tier8.py -k tombstones > gpurun_out/r03_s17_tomb_test.log 2>&1 &&
bash tools/r03_final_a.sh
