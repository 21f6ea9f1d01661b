#!/bin/bash
# Tier tombstones (GH_TIER_TOMB, gated per wave) vs the round-3 rule
# (lib/variants/libgossiphip_notomb.so) and the ungated rule (tombng): tier /
# plane / parity tests on the default build, the diagnostic schedule, the
# crash leg on both, the quick bench A/B, the full-size 1% crash.
set -o pipefail
mkdir -p gpurun_out/s14
V=p2p-file-system-with-gossip-detect-failure-management_amd/lib/variants
timeout -k 10 120 python -u tools/tomb_diag.py > gpurun_out/s14/diag.log 2>&1 &&
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_tier8.py tests/test_gpu_narrow.py tests/test_gpu_plane.py tests/test_gpu_parity.py > gpurun_out/s14/tests.log 2>&1 &&
timeout -k 10 200 python -u tools/crash_leg.py > gpurun_out/s14/crash_default.json 2> gpurun_out/s14/crash_default.err &&
GOSSIPHIP_LIB=$V/libgossiphip_notomb.so timeout -k 10 200 python -u tools/crash_leg.py > gpurun_out/s14/crash_notomb.json 2> gpurun_out/s14/crash_notomb.err &&
rm -f gpurun_out/nib_ab/summary.txt &&
bash tools/nib_ab.sh default notomb tombng &&
timeout -k 10 500 python -u -m pytest -x -v --timeout 450 --timeout-method thread -s tests/test_gpu_fullsize.py -k crash > gpurun_out/s14/fullsize_crash.log 2>&1
