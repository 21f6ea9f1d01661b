#!/bin/bash
# Round 3 session 7: lane jobs of the nibble path. Tier / plane / narrow /
# parity tests, the full-size crash case against the oracle, then the crash
# leg of the bench (per-round variant, lane jobs and wall time).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_tier8.py tests/test_gpu_plane.py tests/test_gpu_narrow.py > gpurun_out/r03_s7_tier.log 2>&1 &&
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py > gpurun_out/r03_s7_parity.log 2>&1 &&
timeout -k 10 200 python -u -c "
import json, sys
sys.argv = ['bench.py']
import bench, gossipsim as gs
print(json.dumps(bench.crash_leg(gs, 65536)))
" > gpurun_out/r03_s7_crash_leg.json 2> gpurun_out/r03_s7_crash_leg.err &&
timeout -k 10 500 python -u -m pytest -x -v --timeout 450 --timeout-method thread -s tests/test_gpu_fullsize.py -k crash > gpurun_out/r03_s7_fullsize_crash.log 2>&1
