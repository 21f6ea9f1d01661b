#!/bin/bash
# row layout with device want lists: the row / sharded GPU suites, the exchange timing, then the full-size layouts
set -o pipefail
mkdir -p gpurun_out/r04
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_rows.py \
  > gpurun_out/r04/s4_rows.log 2>&1; rc=$?; tail -4 gpurun_out/r04/s4_rows.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/shard_exchange.py 65536 8 5 > gpurun_out/r04/s4_exchange.log 2>&1; rc=$?
tail -4 gpurun_out/r04/s4_exchange.log | cut -c1-400; [ $rc -eq 0 ] || exit $rc
timeout -k 10 1500 python -u -m pytest -x -v -s --timeout 900 --timeout-method thread -m gpu \
  "tests/test_gpu_fullsize.py::test_c3_fullsize_rows_g8" "tests/test_gpu_fullsize.py::test_c3_fullsize_columns_g8" \
  > gpurun_out/r04/s4_fullsize.log 2>&1; rc=$?; grep -E "PASS|FAIL|Error|equal|r=2[3-5]" gpurun_out/r04/s4_fullsize.log | cut -c1-200 | tail -20; exit $rc
