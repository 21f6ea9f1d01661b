#!/bin/bash
# row layout's nibble path (IN 4) with split-sender gathers: parity of the row tests, then G=8 row-shard pull rounds A/B
set -o pipefail
mkdir -p gpurun_out/r05
O=gpurun_out/r05
V=$PWD/p2p-file-system-with-gossip-detect-failure-management_amd/lib/variants/libgossiphip_splitrows.so
GOSSIPHIP_LIB=$V timeout -k 10 500 python -u -m pytest tests/test_gpu_rows.py -x -q --timeout 300 --timeout-method thread > $O/s22_rows_split.log 2>&1 || exit 1
export GH_EXCHANGE_ONLY=rows_pull
for pass in 1 2; do
  for v in default split; do
    if [ $v = split ]; then export GOSSIPHIP_LIB=$V; else unset GOSSIPHIP_LIB; fi
    timeout -k 10 300 python3 tools/shard_exchange.py 65536 8 4 > $O/s22_${v}_p$pass.txt 2>&1 || exit 1
    python3 -c "import json; l=[x for x in open('$O/s22_${v}_p$pass.txt') if x.startswith('rows pull')][0]; print('$v pass=$pass', json.loads(l.split(' ',2)[2])['ms_per_round'])" | tee -a $O/s22_ab.txt
  done
done
