#!/bin/bash
# final tree, part b: PMC passes + kernel stats (tools/pmc.sh), one round's
# kernel timeline, the driver's bench command
set -o pipefail
mkdir -p gpurun_out/r05
O=gpurun_out/r05
export TMPDIR=/tmp
tools/pmc.sh 5 20 || exit 1
timeout -s KILL 300 rocprofv3 --kernel-trace --output-format csv -d $O/tl17 -o run -- \
  python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-secondary --files 0 > $O/tl17.txt 2>&1 || exit 1
python3 tools/r04/round_timeline.py $O/tl17 > $O/s17_timeline.txt || exit 1
python3 tools/r05/kernel_stats_active.py $O/tl17 > $O/s17_kernel_stats_active.csv || exit 1
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/s17_bench.json 2> $O/s17_bench.err || exit 1
