#!/bin/bash
# split-sender gathers (round_block_nib SPL): parity suites, then bench A/B against a GH_NIB_SPLIT=0 build
set -o pipefail
mkdir -p gpurun_out/r05
O=gpurun_out/r05
export TMPDIR=/tmp
timeout -k 10 800 python -u -m pytest tests/test_gpu_tier8.py tests/test_gpu_parity.py tests/test_gpu_sharded.py tests/test_gpu_plane.py tests/test_gpu_narrow.py -x -q --timeout 300 --timeout-method thread > $O/s16_tests.log 2>&1 || exit 1
V=p2p-file-system-with-gossip-detect-failure-management_amd/lib/variants/libgossiphip_nosplit.so
for pass in 1 2 3; do
  for v in split nosplit; do
    if [ $v = nosplit ]; then export GOSSIPHIP_LIB=$PWD/$V; else unset GOSSIPHIP_LIB; fi
    timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-secondary --no-cpu-baseline > $O/ab_split_${v}_p$pass.json 2> $O/ab_split_${v}_p$pass.err || exit 1
    python3 -c "import json,sys; d=json.load(open('$O/ab_split_${v}_p$pass.json')); r=d['roofline']; print('$v pass=$pass', round(d['value'],1), 'rounds/s', round(d['ms_per_step'],4), 'ms/step', round(r['avg_launch_ms'],4), 'ms', round(r['frac'],3))" | tee -a $O/ab_split.txt
  done
done
