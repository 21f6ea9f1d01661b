#!/bin/bash
# the driver's GPU test command, then its bench command
set -o pipefail
mkdir -p gpurun_out/r05
O=gpurun_out/r05
S=${1:-s3}
( time timeout -k 10 900 python -m pytest tests/ -x -q -m gpu > $O/${S}_gpu_suite.log 2>&1 ) 2> $O/${S}_suite_time.txt || exit 1
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/${S}_bench.json 2> $O/${S}_bench.err || exit 1
