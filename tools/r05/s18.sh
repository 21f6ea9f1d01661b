#!/bin/bash
# the REMOVE-taking nibble path on a residency-sized grid: its parity, the
# bench with its crash leg, one steady round's timeline
set -o pipefail
mkdir -p gpurun_out/r05
O=gpurun_out/r05
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_tier8.py -x -q --timeout 300 --timeout-method thread -k "remove or nibble_variants or timing" > $O/s18_tier8.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/s18_bench.json 2> $O/s18_bench.err || exit 1
timeout -s KILL 300 rocprofv3 --kernel-trace --output-format csv -d $O/tl18 -o run -- \
  python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-secondary --files 0 > $O/tl18.txt 2>&1 || exit 1
python3 tools/r04/round_timeline.py $O/tl18 > $O/s18_timeline.txt || exit 1
