#!/bin/bash
# full-size G=8 shard tests on the final tree (direct in-process collectives, 16-B ghost pack)
set -o pipefail
mkdir -p gpurun_out/r05
O=gpurun_out/r05
P="python -u -m pytest tests/test_gpu_fullsize.py --fullsize -x -v -s --timeout 900 --timeout-method thread"
timeout -k 10 500 $P -k "rows_g8" > $O/s25_fs_rows_g8.log 2>&1 || exit 1
timeout -k 10 500 $P -k "columns_g8" > $O/s25_fs_columns_g8.log 2>&1 || exit 1
