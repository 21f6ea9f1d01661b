#!/bin/bash
# idle variants in line (GH_SIDE=0) against the side stream, with the launch-stamped timing of the final tree
set -o pipefail
mkdir -p gpurun_out/r05
O=gpurun_out/r05
export TMPDIR=/tmp
for pass in 1 2 3; do
  for v in 1 0; do
    GH_SIDE=$v timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-secondary --no-cpu-baseline > $O/ab_side_f_${v}_p$pass.json 2> $O/ab_side_f_${v}_p$pass.err || exit 1
    python3 -c "import json,sys; d=json.load(open('$O/ab_side_f_${v}_p$pass.json')); r=d['roofline']; print('side=$v pass=$pass', round(d['value'],1), 'rounds/s', round(d['ms_per_step'],4), 'ms/step', round(r['avg_launch_ms'],4), 'ms', round(d['ms_per_step']-r['avg_launch_ms'],4))" | tee -a $O/ab_side_final.txt
  done
done
export GH_SIDE=0
timeout -s KILL 300 rocprofv3 --kernel-trace --output-format csv -d $O/tl27 -o run -- \
  python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-secondary --files 0 > $O/tl27.txt 2>&1 || exit 1
python3 tools/r04/round_timeline.py $O/tl27 > $O/s27_timeline_inline.txt || exit 1
