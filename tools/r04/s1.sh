#!/bin/bash
# session 1: parity of the job list + side-stream variants, then the cache-policy A/B
set -o pipefail
mkdir -p gpurun_out/r04
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_tier8.py tests/test_gpu_fullsize.py > gpurun_out/r04/s1_pytest.log 2>&1 || { tail -30 gpurun_out/r04/s1_pytest.log; exit 1; }
tail -3 gpurun_out/r04/s1_pytest.log
AB_PASSES="1 2" bash tools/r04/ab.sh default st16 st17 age18 st16age18 st0
