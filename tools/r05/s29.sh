#!/bin/bash
# final tree (last source change): the driver's GPU test command, the smoke, the driver's bench command
set -o pipefail
mkdir -p gpurun_out/r05
O=gpurun_out/r05
( time timeout -k 10 900 python -m pytest tests/ -x -q -m gpu > $O/s29_gpu_suite.log 2>&1 ) 2> $O/s29_suite_time.txt || exit 1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/s29_smoke.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/s29_bench.json 2> $O/s29_bench.err || exit 1
