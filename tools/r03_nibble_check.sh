#!/bin/bash
# Round 3: the nibble path on the GPU box (tier parity diagnostic, smoke,
# tier/plane/narrow parity, a quick bench, the full-size steady state). Every
# GPU step is time-limited and chained with &&.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 python -u tools/tier_parity_diag.py 512 12 > gpurun_out/r03_tier_diag.log 2>&1 &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03_smoke.log 2>&1 &&
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_tier8.py tests/test_gpu_plane.py tests/test_gpu_narrow.py > gpurun_out/r03_tier_tests.log 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-secondary > gpurun_out/r03_bench_quick.json 2> gpurun_out/r03_bench_quick.err &&
timeout -k 10 600 python -u -m pytest -x -v --timeout 500 --timeout-method thread -s tests/test_gpu_fullsize.py -k steady > gpurun_out/r03_fullsize_nibble.log 2>&1
