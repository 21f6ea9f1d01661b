#!/bin/bash
# final tree with sc1|nt nibble stores: the driver's GPU test command, smoke, PMC passes + stats, the driver's bench
set -o pipefail
mkdir -p gpurun_out/r05
O=gpurun_out/r05
export TMPDIR=/tmp
( time timeout -k 10 900 python -m pytest tests/ -x -q -m gpu > $O/s33_gpu_suite.log 2>&1 ) 2> $O/s33_suite_time.txt || exit 1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/s33_smoke.log 2>&1 || exit 1
tools/pmc.sh 5 20 || exit 1
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/s33_bench.json 2> $O/s33_bench.err || exit 1
