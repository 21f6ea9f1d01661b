#!/bin/bash
# side stream vs in-line idle variants: the bench (no secondary legs), alternating, then one timeline each
set -o pipefail
mkdir -p gpurun_out/r04/s16
export TMPDIR=/tmp
for pass in 1 2; do for side in 1 0; do
  GH_SIDE=$side timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-secondary --steps 40 > gpurun_out/r04/s16/b_$side.json 2> gpurun_out/r04/s16/b.err || { tail gpurun_out/r04/s16/b.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/r04/s16/b_$side.json').read().strip().splitlines()[-1]); r=d['roofline']; print('side $side pass $pass: value %.1f ms_per_step %.4f k_round %.4f fixed_us %.1f' % (d['value'], d['ms_per_step'], r['avg_launch_ms'], 1e3*(d['ms_per_step'] - r['avg_launch_ms'])))"
done; done
for side in 1 0; do
  GH_SIDE=$side timeout -s KILL 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r04/s16/prof$side -o run -- \
    python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-secondary --files 0 > gpurun_out/r04/s16/prof$side.log 2>&1 || exit 1
  echo "== side $side"; python3 tools/r04/round_timeline.py gpurun_out/r04/s16/prof$side
done
