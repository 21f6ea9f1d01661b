#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r05
O=gpurun_out/r05
timeout -k 10 400 python -u -m pytest tests/test_gpu_tier8.py -x -v --timeout 300 --timeout-method thread > $O/s4_tier8.log 2>&1 || exit 1
tools/r05/ab_dma.sh || exit 1
tools/r05/s3.sh s4 || exit 1
