#!/bin/bash
# side stream forked at the nibble launch's start stamp; timing modes 0 / 1
set -o pipefail
mkdir -p gpurun_out/r05
O=gpurun_out/r05
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_tier8.py -x -q --timeout 300 --timeout-method thread > $O/s13_tier8.log 2>&1 || exit 1
for t in 0 1; do
  GH_TMODE=$t timeout -k 10 200 python3 tools/r05/fixed_cost.py 20 3 > $O/s13_fixed_t$t.jsonl 2>&1 || exit 1
done
for t in 1 0; do
  export GH_TMODE=$t
  timeout -s KILL 300 rocprofv3 --kernel-trace --output-format csv -d $O/tl13_$t -o run -- \
    python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-secondary --files 0 > $O/tl13_$t.txt 2>&1 || exit 1
  python3 tools/r04/round_timeline.py $O/tl13_$t > $O/s13_timeline_t$t.txt || exit 1
done
unset GH_TMODE
for pass in 1 2 3; do
  for t in 0 1; do
    GH_TMODE=$t timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-secondary --no-cpu-baseline > $O/ab_tc_${t}_p$pass.json 2> $O/ab_tc_${t}_p$pass.err || exit 1
    python3 -c "import json,sys; d=json.load(open('$O/ab_tc_${t}_p$pass.json')); r=d['roofline']; print('tmode=$t pass=$pass', round(d['value'],1), 'rounds/s', round(d['ms_per_step'],4), 'ms/step', round(r['avg_launch_ms'],4), 'ms', round(r['frac'],3))" | tee -a $O/ab_tmode_c.txt
  done
done
