#!/bin/bash
# nibble-path store policy A/B: nt (default, keeps the written lines in the XCD's L2) against sc1 and sc1|nt (drop them)
set -o pipefail
mkdir -p gpurun_out/r05
O=gpurun_out/r05
L=$PWD/p2p-file-system-with-gossip-detect-failure-management_amd/lib/variants
for pass in 1 2 3; do
  for v in st2 st16 st18; do
    if [ $v = st2 ]; then unset GOSSIPHIP_LIB; else export GOSSIPHIP_LIB=$L/libgossiphip_$v.so; fi
    timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-secondary --no-cpu-baseline > $O/ab_st_${v}_p$pass.json 2> $O/ab_st_${v}_p$pass.err || exit 1
    python3 -c "import json,sys; d=json.load(open('$O/ab_st_${v}_p$pass.json')); r=d['roofline']; print('$v pass=$pass', round(d['value'],1), 'rounds/s', round(d['ms_per_step'],4), 'ms/step', round(r['avg_launch_ms'],4), 'ms')" | tee -a $O/ab_st.txt
  done
done
