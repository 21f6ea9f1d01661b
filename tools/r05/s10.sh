#!/bin/bash
# idle side-stream variants: IN 6 on a 1/8 grid, one or two side streams
# (GH_SIDE=1/2): parity of the nibble variants, per-round time with the
# timing events off and on, one round's kernel timeline each, bench A/B
set -o pipefail
mkdir -p gpurun_out/r05
O=gpurun_out/r05
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_tier8.py -x -v --timeout 300 --timeout-method thread -k "nibble_variants or remove_on_nibble" > $O/s10_tier8.log 2>&1 || exit 1
for sd in 1 2; do
  GH_SIDE=$sd timeout -k 10 200 python3 tools/r05/fixed_cost.py 20 3 > $O/s10_fixed_side$sd.jsonl 2>&1 || exit 1
done
for sd in 1 2; do
  export GH_SIDE=$sd
  timeout -s KILL 300 rocprofv3 --kernel-trace --output-format csv -d $O/tl10_$sd -o run -- \
    python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-secondary --files 0 > $O/tl10_$sd.txt 2>&1 || exit 1
  python3 tools/r04/round_timeline.py $O/tl10_$sd > $O/s10_timeline_side$sd.txt || exit 1
done
unset GH_SIDE
for pass in 1 2; do
  for v in 1 2; do
    GH_SIDE=$v timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-secondary --no-cpu-baseline > $O/ab_side${v}_p$pass.json 2> $O/ab_side${v}_p$pass.err || exit 1
    python3 -c "import json,sys; d=json.load(open('$O/ab_side${v}_p$pass.json')); r=d['roofline']; print('side=$v pass=$pass', round(d['value'],1), 'rounds/s', d['ms_per_step'], 'ms/step', round(r['avg_launch_ms'],4), 'ms', round(r['frac'],3))" | tee -a $O/ab_side.txt
  done
done
