#!/bin/bash
# REMOVE on the nibble path: its parity tests, the crash leg with and without it, the full-size crash
set -o pipefail
mkdir -p gpurun_out/r05
O=gpurun_out/r05
timeout -k 10 600 python -u -m pytest tests/test_gpu_tier8.py -x -v --timeout 300 --timeout-method thread -k remove > $O/s2_remove_tests.log 2>&1 || exit 1
timeout -k 10 120 python tools/crash_leg.py > $O/s2_crash_leg_rmv.json 2> $O/s2_crash_leg_rmv.err || exit 1
GH_NIB_RMV=0 timeout -k 10 120 python tools/crash_leg.py > $O/s2_crash_leg_norm.json 2> $O/s2_crash_leg_norm.err || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py -x -v -s --timeout 580 --timeout-method thread -k "test_c3_fullsize_crash_1pct and not quirk and not remove_list" > $O/s2_fullsize_crash.log 2>&1 || exit 1
