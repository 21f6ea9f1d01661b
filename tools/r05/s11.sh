#!/bin/bash
# timing modes (GH_TMODE 0: events on every variant launch; 1: on the
# nibble launch only, the others bracketed, the device's variant log) with
# the idle variants on the side stream or in line (GH_SIDE 1 / 0)
set -o pipefail
mkdir -p gpurun_out/r05
O=gpurun_out/r05
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_tier8.py -x -v --timeout 300 --timeout-method thread -k "timing or nibble_variants or remove_on_nibble" > $O/s11_tier8.log 2>&1 || exit 1
for c in "1 0" "1 1" "0 1"; do
  set -- $c
  GH_SIDE=$1 GH_TMODE=$2 timeout -k 10 200 python3 tools/r05/fixed_cost.py 20 3 > $O/s11_fixed_side$1_t$2.jsonl 2>&1 || exit 1
done
for c in "1 1" "0 1"; do
  set -- $c
  export GH_SIDE=$1 GH_TMODE=$2
  timeout -s KILL 300 rocprofv3 --kernel-trace --output-format csv -d $O/tl11_$1$2 -o run -- \
    python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-secondary --files 0 > $O/tl11_$1$2.txt 2>&1 || exit 1
  python3 tools/r04/round_timeline.py $O/tl11_$1$2 > $O/s11_timeline_side$1_t$2.txt || exit 1
done
unset GH_SIDE GH_TMODE
for pass in 1 2; do
  for c in "1 0" "1 1" "0 1"; do
    set -- $c
    GH_SIDE=$1 GH_TMODE=$2 timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-secondary --no-cpu-baseline > $O/ab_t_$1$2_p$pass.json 2> $O/ab_t_$1$2_p$pass.err || exit 1
    python3 -c "import json,sys; d=json.load(open('$O/ab_t_$1$2_p$pass.json')); r=d['roofline']; print('side=$1 tmode=$2 pass=$pass', round(d['value'],1), 'rounds/s', round(d['ms_per_step'],4), 'ms/step', round(r['avg_launch_ms'],4), 'ms', round(r['frac'],3))" | tee -a $O/ab_tmode.txt
  done
done
