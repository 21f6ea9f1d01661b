#!/bin/bash
# Round 3 final tree, part B: the driver's bench command, the PMC passes and
# kernel stats of the same bench (tools/pmc.sh), the shard-layout exchange at
# N=65,536, G=8 on one GPU (in-process transport).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py > gpurun_out/r03_final_bench.json 2> gpurun_out/r03_final_bench.err &&
bash tools/pmc.sh 5 20 &&
timeout -k 10 300 python -u tools/shard_exchange.py 65536 8 3 > gpurun_out/r03_final_shard_exchange.log 2>&1
