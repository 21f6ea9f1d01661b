#!/bin/bash
# Round 3 session 6: the whole -m gpu suite, smoke, the driver's bench command
# and the PMC passes + kernel stats of the same bench (tools/pmc.sh). Every
# GPU step is time-limited and chained with &&.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread -s > gpurun_out/r03_s6_pytest_gpu.log 2>&1 &&
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03_s6_smoke.log 2>&1 &&
timeout -k 10 300 python -u bench.py > gpurun_out/r03_s6_bench.json 2> gpurun_out/r03_s6_bench.err &&
bash tools/pmc.sh 5 20
