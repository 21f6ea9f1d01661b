#!/bin/bash
# 16-B ghost plane pack, peers_pull loads issued together; split-sender probe
set -o pipefail
mkdir -p gpurun_out/r05
O=gpurun_out/r05
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_gpu_rows.py tests/test_gpu_tier8.py -x -q --timeout 300 --timeout-method thread > $O/s14_rows_tier8.log 2>&1 || exit 1
tools/r05/probe4.sh || exit 1
for lay in rows_pull columns_pull; do
  export GH_EXCHANGE_ONLY=$lay
  timeout -k 10 300 python3 tools/shard_exchange.py 65536 8 3 > $O/s14_$lay.txt 2>&1 || exit 1
done
export GH_EXCHANGE_ONLY=rows_pull
timeout -s KILL 400 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $O/tl14_rows_pull -o run -- \
  python3 tools/shard_exchange.py 65536 8 3 > $O/s14_rows_pull_prof.txt 2>&1 || exit 1
