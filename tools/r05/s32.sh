#!/bin/bash
# store policy sc1|nt (drop the written lines from the XCD's L2) against nt, alternating order, plus L2 hit counters for each
set -o pipefail
mkdir -p gpurun_out/r05
O=gpurun_out/r05
export TMPDIR=/tmp
L=$PWD/p2p-file-system-with-gossip-detect-failure-management_amd/lib/variants
run() {
  if [ $1 = st2 ]; then unset GOSSIPHIP_LIB; else export GOSSIPHIP_LIB=$L/libgossiphip_$1.so; fi
  timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-secondary --no-cpu-baseline > $O/ab_st2_${1}_p$2.json 2> $O/ab_st2_${1}_p$2.err || return 1
  python3 -c "import json,sys; d=json.load(open('$O/ab_st2_${1}_p$2.json')); r=d['roofline']; print('$1 pass=$2', round(d['value'],1), 'rounds/s', round(d['ms_per_step'],4), 'ms/step', round(r['avg_launch_ms'],4), 'ms')" | tee -a $O/ab_st2.txt
}
run st18 1 && run st2 1 && run st2 2 && run st18 2 && run st18 3 && run st2 3 && run st2 4 && run st18 4 || exit 1
for v in st2 st18; do
  if [ $v = st2 ]; then unset GOSSIPHIP_LIB; else export GOSSIPHIP_LIB=$L/libgossiphip_$v.so; fi
  timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-include-regex 'k_round' --output-format csv -d $O/pmc_st_$v -o run -- \
    python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-secondary --files 0 > $O/pmc_st_$v.log 2>&1 || exit 1
done
