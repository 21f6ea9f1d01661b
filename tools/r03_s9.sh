#!/bin/bash
# Lane jobs v3 (rolled exact gathers): crash leg timing + rocprof kernel stats of it, tier tests.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python -u tools/crash_leg.py > gpurun_out/r03_s9_crash_leg.json 2> gpurun_out/r03_s9_crash_leg.err &&
timeout -s KILL 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03_s9_prof -o run -- python3 tools/crash_leg.py > gpurun_out/r03_s9_prof.log 2>&1 &&
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_tier8.py tests/test_gpu_narrow.py > gpurun_out/r03_s9_tier.log 2>&1
