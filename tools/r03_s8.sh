#!/bin/bash
# Lane jobs v2: crash leg timing, then the tier tests and the full-size crash parity.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u -c "
import json, sys
sys.argv = ['bench.py']
import bench, gossipsim as gs
print(json.dumps(bench.crash_leg(gs, 65536)))
" > gpurun_out/r03_s8_crash_leg.json 2> gpurun_out/r03_s8_crash_leg.err &&
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_tier8.py tests/test_gpu_narrow.py > gpurun_out/r03_s8_tier.log 2>&1 &&
timeout -k 10 500 python -u -m pytest -x -v --timeout 450 --timeout-method thread -s tests/test_gpu_fullsize.py -k crash > gpurun_out/r03_s8_fullsize_crash.log 2>&1
