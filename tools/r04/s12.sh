#!/bin/bash
# saturated guard-row tombstones on the packed storm path: the reference-timeouts leg, the GPU suite, the full-size reference-timeouts test
set -o pipefail
mkdir -p gpurun_out/r04/s12
timeout -k 10 300 python3 -u tools/r04/leg_probe.py ref 24 > gpurun_out/r04/s12/ref.log 2>&1; rc=$?; cut -c1-200 gpurun_out/r04/s12/ref.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u tools/r04/leg_probe.py ring 24 > gpurun_out/r04/s12/ring.log 2>&1; rc=$?; cut -c1-200 gpurun_out/r04/s12/ring.log | tail -8; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests --deselect tests/test_gpu_fullsize.py > gpurun_out/r04/s12/suite.log 2>&1; rc=$?; tail -5 gpurun_out/r04/s12/suite.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u -m pytest -x -v -s --timeout 450 --timeout-method thread -m gpu tests/test_gpu_fullsize.py::test_c3_fullsize_reference_timeouts > gpurun_out/r04/s12/full_ref.log 2>&1; rc=$?; tail -4 gpurun_out/r04/s12/full_ref.log | cut -c1-300; exit $rc
