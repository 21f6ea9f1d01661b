#!/bin/bash
# shard exchange at N=65,536, G=8 on one GPU: all six legs (row/column shards, pull/ring, and the single engine)
set -o pipefail
mkdir -p gpurun_out/r04/s17
timeout -k 10 600 python -u tools/shard_exchange.py 65536 8 5 > gpurun_out/r04/s17/exchange.log 2>&1; rc=$?
grep -v "^{" gpurun_out/r04/s17/exchange.log | cut -c1-220; exit $rc
