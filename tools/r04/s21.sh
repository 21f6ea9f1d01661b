#!/bin/bash
# the full-size 1% crash test alone
set -o pipefail
mkdir -p gpurun_out/r04/s21
timeout -k 10 700 python -u -m pytest -x -v -s --timeout 650 --timeout-method thread -m gpu tests/test_gpu_fullsize.py::test_c3_fullsize_crash_1pct > gpurun_out/r04/s21/full.log 2>&1; rc=$?; grep -E "PASSED|FAILED|passed|failed|round 25" gpurun_out/r04/s21/full.log | cut -c1-300; exit $rc
