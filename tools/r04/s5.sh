#!/bin/bash
# the whole -m gpu suite but the full-size module, then the exchange timing
set -o pipefail
mkdir -p gpurun_out/r04
timeout -k 10 1500 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests \
  --deselect tests/test_gpu_fullsize.py > gpurun_out/r04/s5_suite.log 2>&1; rc=$?
tail -15 gpurun_out/r04/s5_suite.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/shard_exchange.py 65536 8 5 > gpurun_out/r04/s5_exchange.log 2>&1; rc=$?
tail -4 gpurun_out/r04/s5_exchange.log | cut -c1-600; exit $rc
