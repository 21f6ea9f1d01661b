#!/bin/bash
# The nibble path (16-B lanes) and the row layout's ghost table: the tests
# after test_gpu_plane, the tier tests, the full-size steady state, a quick
# bench and the smoke test.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 python -u tools/tier_parity_diag.py 512 12 > gpurun_out/r03_tier_diag.log 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-secondary --files 0 > gpurun_out/r03_bench_quick.json 2> gpurun_out/r03_bench_quick.err &&
timeout -k 10 1200 python -u -m pytest -x -v --timeout 600 --timeout-method thread -s tests/test_gpu_rows.py tests/test_gpu_sharded.py tests/test_gpu_tier8.py tests/test_gpu_plane.py tests/test_gpu_narrow.py "tests/test_gpu_fullsize.py::test_c3_fullsize_steady_state" > gpurun_out/r03_pytest_rest.log 2>&1 &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03_smoke.log 2>&1
