#!/bin/bash
# fixed cost: the driver bench (no secondary legs) and one steady round's timeline under rocprofv3
set -o pipefail
mkdir -p gpurun_out/r04/s15
export TMPDIR=/tmp
timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-secondary > gpurun_out/r04/s15/bench.json 2> gpurun_out/r04/s15/bench.err || { tail gpurun_out/r04/s15/bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/r04/s15/bench.json').read().strip().splitlines()[-1]); r=d['roofline']; print('value', d['value'], 'ms_per_step', d['ms_per_step'], 'k_round', r['avg_launch_ms'], 'fixed_ms', d['ms_per_step'] - r['avg_launch_ms'])"
timeout -s KILL 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r04/s15/prof -o run -- \
  python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-secondary --files 0 > gpurun_out/r04/s15/prof.log 2>&1 || exit 1
python3 tools/r04/round_timeline.py gpurun_out/r04/s15/prof
