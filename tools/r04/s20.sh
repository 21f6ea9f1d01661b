#!/bin/bash
# batched lane-job gathers: the crash leg round by round, the GPU suite, the full-size crash tests
set -o pipefail
mkdir -p gpurun_out/r04/s20
timeout -k 10 300 python3 -u tools/r04/crash_probe.py > gpurun_out/r04/s20/crash.log 2>&1; rc=$?; sed -n 20,30p gpurun_out/r04/s20/crash.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests --deselect tests/test_gpu_fullsize.py > gpurun_out/r04/s20/suite.log 2>&1; rc=$?; tail -3 gpurun_out/r04/s20/suite.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 700 python -u -m pytest -x -v -s --timeout 650 --timeout-method thread -m gpu tests/test_gpu_fullsize.py::test_c3_fullsize_crash_1pct tests/test_gpu_fullsize.py::test_c3_fullsize_rows_g8 > gpurun_out/r04/s20/full.log 2>&1; rc=$?; grep -E "PASSED|FAILED|passed|failed" gpurun_out/r04/s20/full.log | cut -c1-200; exit $rc
