#!/bin/bash
# event rounds after the per-wave tallies, parity + sharded suites, the D4 divergence at full size
set -o pipefail
mkdir -p gpurun_out/r04/s10
timeout -k 10 300 python3 -u tools/r04/event_probe.py > gpurun_out/r04/s10/events.log 2>&1; rc=$?; cat gpurun_out/r04/s10/events.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_sharded.py > gpurun_out/r04/s10/pytest.log 2>&1; rc=$?; tail -3 gpurun_out/r04/s10/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 -u tools/r04/d4_probe.py > gpurun_out/r04/s10/d4.log 2>&1; rc=$?; cut -c1-400 gpurun_out/r04/s10/d4.log; exit $rc
