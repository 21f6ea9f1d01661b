#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r05
O=gpurun_out/r05
timeout -k 10 600 python -u -m pytest tests/test_gpu_list_order.py tests/test_gpu_rows.py -x -v --timeout 300 --timeout-method thread > $O/s5_lists_rows.log 2>&1 || exit 1
