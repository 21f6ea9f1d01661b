#!/bin/bash
# final tree, part a: the driver's GPU test command, then the smoke
set -o pipefail
mkdir -p gpurun_out/r05
O=gpurun_out/r05
( time timeout -k 10 900 python -m pytest tests/ -x -q -m gpu > $O/s17_gpu_suite.log 2>&1 ) 2> $O/s17_suite_time.txt || exit 1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/s17_smoke.log 2>&1 || exit 1
