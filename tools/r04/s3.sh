#!/bin/bash
# GH_REMOVE_LIST on the GPU: KATs, churn, storms, crash, tier, then the full-size crash
set -o pipefail
mkdir -p gpurun_out/r04
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_remove_list.py "tests/test_gpu_parity.py::test_kats_gpu" > gpurun_out/r04/s3_remove.log 2>&1
rc=$?; tail -25 gpurun_out/r04/s3_remove.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 550 --timeout-method thread -m gpu \
  "tests/test_gpu_fullsize.py::test_c3_fullsize_crash_1pct_remove_list" > gpurun_out/r04/s3_fullsize.log 2>&1
rc=$?; tail -40 gpurun_out/r04/s3_fullsize.log; exit $rc
