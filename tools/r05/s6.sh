#!/bin/bash
# full-size (gpu_fullsize) tests, part 1: literal REMOVE (1% crash, timed storm), reference timeouts, quirk crash, G=8 row shards
set -o pipefail
mkdir -p gpurun_out/r05
O=gpurun_out/r05
P="python -u -m pytest tests/test_gpu_fullsize.py --fullsize -x -v -s --timeout 900 --timeout-method thread"
timeout -k 10 300 $P -k "remove_list_timed" > $O/s6_fs_remove_list_storm_timed.log 2>&1 || exit 1
timeout -k 10 400 $P -k "crash_1pct_remove_list" > $O/s6_fs_remove_list.log 2>&1 || exit 1
timeout -k 10 300 $P -k "test_c3_fullsize_reference_timeouts and not remove_list" > $O/s6_fs_reference_timeouts.log 2>&1 || exit 1
timeout -k 10 450 $P -k "crash_1pct_quirk" > $O/s6_fs_quirk.log 2>&1 || exit 1
