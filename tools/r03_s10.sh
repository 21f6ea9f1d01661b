#!/bin/bash
# Lean lane jobs: the crash leg per job-kernel build (default / 4 / 5 waves),
# then tier, narrow, parity and the full-size crash parity on the default build.
set -o pipefail
mkdir -p gpurun_out/s10
L=p2p-file-system-with-gossip-detect-failure-management_amd/lib
for v in default jobw4 jobw5; do
  if [ $v = default ]; then lib=$L/libgossiphip.so; else lib=$L/variants/libgossiphip_$v.so; fi
  GOSSIPHIP_LIB=$lib timeout -k 10 200 python -u tools/crash_leg.py > gpurun_out/s10/crash_$v.json 2> gpurun_out/s10/crash_$v.err || exit 1
done
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_tier8.py tests/test_gpu_narrow.py tests/test_gpu_plane.py > gpurun_out/s10/tier.log 2>&1 &&
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_list_order.py > gpurun_out/s10/parity.log 2>&1 &&
timeout -k 10 500 python -u -m pytest -x -v --timeout 450 --timeout-method thread -s tests/test_gpu_fullsize.py -k crash > gpurun_out/s10/fullsize_crash.log 2>&1
