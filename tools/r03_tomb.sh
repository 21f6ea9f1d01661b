#!/bin/bash
# Tier tombstones (code 15, age 1..14) on the nibble path: tier / plane /
# parity tests, the full-size 1% crash, the crash leg and a short bench.
set -o pipefail
mkdir -p gpurun_out/tomb
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_tier8.py tests/test_gpu_narrow.py tests/test_gpu_plane.py tests/test_gpu_parity.py > gpurun_out/tomb/tests.log 2>&1 &&
timeout -k 10 200 python -u tools/crash_leg.py > gpurun_out/tomb/crash_leg.json 2> gpurun_out/tomb/crash_leg.err &&
timeout -k 10 500 python -u -m pytest -x -v --timeout 450 --timeout-method thread -s tests/test_gpu_fullsize.py -k crash > gpurun_out/tomb/fullsize_crash.log 2>&1 &&
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/tomb/bench.json 2> gpurun_out/tomb/bench.err
