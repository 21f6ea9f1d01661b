#!/bin/bash
# full-size REMOVE-round tests on the final tree (IN 6 as the round's nibble launch): literal REMOVE 1% crash, quirk 1% crash
set -o pipefail
mkdir -p gpurun_out/r05
O=gpurun_out/r05
P="python -u -m pytest tests/test_gpu_fullsize.py --fullsize -x -v -s --timeout 900 --timeout-method thread"
timeout -k 10 450 $P -k "crash_1pct_remove_list" > $O/s24_fs_remove_list.log 2>&1 || exit 1
timeout -k 10 500 $P -k "crash_1pct_quirk" > $O/s24_fs_quirk.log 2>&1 || exit 1
