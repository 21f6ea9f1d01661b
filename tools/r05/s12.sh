#!/bin/bash
# stream-ordered LOCAL transport: the sharded parity tests, then where the
# in-process G=8 shard round goes (kernel + copy traces of
# tools/shard_exchange.py for row and column shards)
set -o pipefail
mkdir -p gpurun_out/r05
O=gpurun_out/r05
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_gpu_sharded.py tests/test_gpu_rows.py tests/test_gpu_list_order.py -x -q --timeout 300 --timeout-method thread > $O/s12_sharded_tests.log 2>&1 || exit 1
for lay in rows_pull columns_pull; do
  export GH_EXCHANGE_ONLY=$lay
  timeout -k 10 300 python3 tools/shard_exchange.py 65536 8 3 > $O/s12_$lay.txt 2>&1 || exit 1
  timeout -s KILL 400 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $O/tl12_$lay -o run -- \
    python3 tools/shard_exchange.py 65536 8 3 > $O/s12_${lay}_prof.txt 2>&1 || exit 1
done
