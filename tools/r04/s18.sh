#!/bin/bash
# incremental row counts after events: event rounds, the GPU suite, the full-size C5 and crash tests
set -o pipefail
mkdir -p gpurun_out/r04/s18
timeout -k 10 300 python3 -u tools/r04/event_probe.py > gpurun_out/r04/s18/events.log 2>&1; rc=$?; cat gpurun_out/r04/s18/events.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests --deselect tests/test_gpu_fullsize.py > gpurun_out/r04/s18/suite.log 2>&1; rc=$?; tail -3 gpurun_out/r04/s18/suite.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 700 python -u -m pytest -x -v -s --timeout 650 --timeout-method thread -m gpu tests/test_gpu_fullsize.py::test_c5_fullsize_files > gpurun_out/r04/s18/c5.log 2>&1; rc=$?; tail -3 gpurun_out/r04/s18/c5.log | cut -c1-200; exit $rc
