#!/bin/bash
# Round 3 session 5: the buffer-addressed nibble path (quick bench, tier and
# plane parity, smoke), then the access-pattern probe and PMC calibration.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-secondary --files 0 > gpurun_out/r03_s5_bench_quick.json 2> gpurun_out/r03_s5_bench_quick.err &&
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_tier8.py tests/test_gpu_plane.py > gpurun_out/r03_s5_tier_tests.log 2>&1 &&
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03_s5_smoke.log 2>&1 &&
bash tools/r03_probe.sh
