#!/bin/bash
# two row steps per nibble-path iteration (GH_NIB_RS=2: 78 VGPRs, 6 waves, twice the loads in flight) A/B
set -o pipefail
mkdir -p gpurun_out/r05
O=gpurun_out/r05
V=$PWD/p2p-file-system-with-gossip-detect-failure-management_amd/lib/variants/libgossiphip_rs2.so
for pass in 1 2 3; do
  for v in rs1 rs2; do
    if [ $v = rs2 ]; then export GOSSIPHIP_LIB=$V; else unset GOSSIPHIP_LIB; fi
    timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-secondary --no-cpu-baseline > $O/ab_rs_${v}_p$pass.json 2> $O/ab_rs_${v}_p$pass.err || exit 1
    python3 -c "import json,sys; d=json.load(open('$O/ab_rs_${v}_p$pass.json')); r=d['roofline']; print('$v pass=$pass', round(d['value'],1), 'rounds/s', round(d['ms_per_step'],4), 'ms/step', round(r['avg_launch_ms'],4), 'ms')" | tee -a $O/ab_rs.txt
  done
done
