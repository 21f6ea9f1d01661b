#!/bin/bash
# direct same-device collectives of the in-process transport: sharded parity, then the G=8 exchange legs
set -o pipefail
mkdir -p gpurun_out/r05
O=gpurun_out/r05
export TMPDIR=/tmp
timeout -k 10 800 python -u -m pytest tests/test_gpu_sharded.py tests/test_gpu_rows.py tests/test_gpu_list_order.py -x -q --timeout 300 --timeout-method thread > $O/s15_sharded_tests.log 2>&1 || exit 1
for lay in rows_pull columns_pull rows_ring columns_ring; do
  export GH_EXCHANGE_ONLY=$lay
  timeout -k 10 300 python3 tools/shard_exchange.py 65536 8 3 > $O/s15_$lay.txt 2>&1 || exit 1
done
export GH_EXCHANGE_ONLY=rows_pull
timeout -s KILL 400 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $O/tl15_rows_pull -o run -- \
  python3 tools/shard_exchange.py 65536 8 3 > $O/s15_rows_pull_prof.txt 2>&1 || exit 1
