#!/bin/bash
# full-size oracle checks, in two halves: s8.sh a|b
set -o pipefail
mkdir -p gpurun_out/r04
if [ "$1" = a ]; then
  T="tests/test_gpu_fullsize.py::test_c3_fullsize_rows_g8 tests/test_gpu_fullsize.py::test_c3_fullsize_columns_g8 tests/test_gpu_fullsize.py::test_c3_fullsize_crash_1pct_quirk"
else
  T="tests/test_gpu_fullsize.py::test_c5_fullsize_files tests/test_gpu_fullsize.py::test_c3_fullsize_steady_state tests/test_gpu_fullsize.py::test_c3_fullsize_reference_timeouts tests/test_gpu_fullsize.py::test_c3_fullsize_crash_1pct"
fi
timeout -k 10 1150 python -u -m pytest -x -v -s --timeout 600 --timeout-method thread -m gpu $T > gpurun_out/r04/s8_$1.log 2>&1
rc=$?; grep -E "PASSED|FAILED|Error|passed|failed" gpurun_out/r04/s8_$1.log | tail -20; exit $rc
