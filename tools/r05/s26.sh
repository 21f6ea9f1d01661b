#!/bin/bash
# full-size tests on the final tree: config 5's 2^20 files, reference timeouts, the literal-REMOVE storm timed
set -o pipefail
mkdir -p gpurun_out/r05
O=gpurun_out/r05
P="python -u -m pytest tests/test_gpu_fullsize.py --fullsize -x -v -s --timeout 900 --timeout-method thread"
timeout -k 10 400 $P -k "c5_fullsize" > $O/s26_fs_c5_files.log 2>&1 || exit 1
timeout -k 10 300 $P -k "test_c3_fullsize_reference_timeouts and not remove_list" > $O/s26_fs_reference_timeouts.log 2>&1 || exit 1
timeout -k 10 300 $P -k "remove_list_timed" > $O/s26_fs_remove_list_storm_timed.log 2>&1 || exit 1
