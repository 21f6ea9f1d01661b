#!/bin/bash
# A/B of the nibble path's LDS-DMA staging (GH_NIB_DMA) on the bench workload, two alternating passes
set -o pipefail
mkdir -p gpurun_out/r05
O=gpurun_out/r05
for pass in 1 2; do
  for v in 0 1; do
    GH_NIB_DMA=$v timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-secondary --no-cpu-baseline > $O/ab_dma${v}_p$pass.json 2> $O/ab_dma${v}_p$pass.err || exit 1
    python3 -c "import json,sys; d=json.load(open('$O/ab_dma${v}_p$pass.json')); r=d['roofline']; print('dma=$v pass=$pass', round(d['value'],1), 'rounds/s', round(r['avg_launch_ms'],4), 'ms', round(r['frac'],3))" | tee -a $O/ab_dma.txt
  done
done
