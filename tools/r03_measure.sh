#!/bin/bash
# Round 3: smoke, the driver's bench command, then the PMC passes and the
# kernel-trace stats of the same bench (tools/pmc.sh). Every GPU step is
# time-limited and chained with &&.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03_smoke.log 2>&1 &&
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r03_bench.json 2> gpurun_out/r03_bench.err &&
bash tools/pmc.sh 5 20
