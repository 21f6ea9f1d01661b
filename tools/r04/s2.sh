#!/bin/bash
# A/B of 32-cell lanes (16-B accesses) vs 16, then the tier tests on the 32-cell build
set -o pipefail
AB_PASSES="1 2" bash tools/r04/ab.sh default cpl32 cpl32w4 || exit 1
GOSSIPHIP_LIB=p2p-file-system-with-gossip-detect-failure-management_amd/lib/variants/libgossiphip_cpl32.so \
  timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_tier8.py \
  > gpurun_out/r04/s2_tier8_cpl32.log 2>&1; rc=$?; tail -5 gpurun_out/r04/s2_tier8_cpl32.log; exit $rc
