#!/bin/bash
# side stream order A/B (GH_SIDE_ORDER=1: the costliest idle variant, IN 1, first)
set -o pipefail
mkdir -p gpurun_out/r05
O=gpurun_out/r05
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_tier8.py -x -q --timeout 200 --timeout-method thread -k "timing or nibble_variants" > $O/s28_tier8.log 2>&1 || exit 1
for pass in 1 2 3; do
  for v in 0 1; do
    GH_SIDE_ORDER=$v timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-secondary --no-cpu-baseline > $O/ab_order_${v}_p$pass.json 2> $O/ab_order_${v}_p$pass.err || exit 1
    python3 -c "import json,sys; d=json.load(open('$O/ab_order_${v}_p$pass.json')); r=d['roofline']; print('order=$v pass=$pass', round(d['value'],1), 'rounds/s', round(d['ms_per_step'],4), 'ms/step', round(r['avg_launch_ms'],4), 'ms', round(d['ms_per_step']-r['avg_launch_ms'],4))" | tee -a $O/ab_order.txt
  done
done
