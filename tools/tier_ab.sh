#!/bin/bash
# A/B of the round kernel's table tier on one box: the bench line (no CPU
# baseline, no secondary legs, no placement) per environment setting.
set -o pipefail
mkdir -p gpurun_out/ab
i=0
for env in "GH_C8=0" "GH_C8=1" "$@"; do
  i=$((i+1))
  echo "== $env" >> gpurun_out/ab/summary.txt
  env $env timeout -k 10 120 python -u bench.py --no-cpu-baseline --no-secondary --files 0 > gpurun_out/ab/$i.json 2> gpurun_out/ab/$i.err || exit 1
  python3 -c "
import json,sys;d=json.loads(open('gpurun_out/ab/$i.json').read().strip().splitlines()[-1])
print(round(d['value'],1),'rounds/s  k_round',round(d['roofline']['avg_launch_ms'],3),'ms',d['layout'])" >> gpurun_out/ab/summary.txt
done
