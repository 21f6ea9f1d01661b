#!/bin/bash
# quiet tiles skipped whole: both collapsed legs, then the GPU suite
set -o pipefail
mkdir -p gpurun_out/r04/s13
timeout -k 10 300 python3 -u tools/r04/leg_probe.py ref 24 > gpurun_out/r04/s13/ref.log 2>&1; rc=$?; cut -c1-120 gpurun_out/r04/s13/ref.log | tail -14; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u tools/r04/leg_probe.py ring 24 > gpurun_out/r04/s13/ring.log 2>&1; rc=$?; cut -c1-120 gpurun_out/r04/s13/ring.log | tail -8; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests --deselect tests/test_gpu_fullsize.py > gpurun_out/r04/s13/suite.log 2>&1; rc=$?; tail -3 gpurun_out/r04/s13/suite.log; exit $rc
