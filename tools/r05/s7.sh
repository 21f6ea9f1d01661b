#!/bin/bash
# full-size tests, part 2: G=8 row and column shards, config 5's 2^20 files
set -o pipefail
mkdir -p gpurun_out/r05
O=gpurun_out/r05
P="python -u -m pytest tests/test_gpu_fullsize.py --fullsize -x -v -s --timeout 900 --timeout-method thread"
timeout -k 10 450 $P -k "rows_g8" > $O/s7_fs_rows_g8.log 2>&1 || exit 1
timeout -k 10 450 $P -k "columns_g8" > $O/s7_fs_columns_g8.log 2>&1 || exit 1
timeout -k 10 400 $P -k "c5_fullsize" > $O/s7_fs_c5_files.log 2>&1 || exit 1
