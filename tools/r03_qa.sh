#!/bin/bash
# 32-B lane-job entries (own words carried) on the default build and the
# whole-word nibble rule variant: tier / parity tests and the full-size
# steady state on the variant, the crash leg on both, the quick bench A/B.
set -o pipefail
mkdir -p gpurun_out/qa
W=p2p-file-system-with-gossip-detect-failure-management_amd/lib/variants/libgossiphip_word.so
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_tier8.py tests/test_gpu_narrow.py > gpurun_out/qa/tests_default.log 2>&1 &&
GOSSIPHIP_LIB=$W timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_tier8.py tests/test_gpu_plane.py tests/test_gpu_narrow.py tests/test_gpu_parity.py > gpurun_out/qa/tests_word.log 2>&1 &&
timeout -k 10 200 python -u tools/crash_leg.py > gpurun_out/qa/crash_default.json 2> gpurun_out/qa/crash_default.err &&
GOSSIPHIP_LIB=$W timeout -k 10 200 python -u tools/crash_leg.py > gpurun_out/qa/crash_word.json 2> gpurun_out/qa/crash_word.err &&
bash tools/nib_ab.sh default word &&
GOSSIPHIP_LIB=$W timeout -k 10 500 python -u -m pytest -x -v --timeout 450 --timeout-method thread -s tests/test_gpu_fullsize.py -k steady > gpurun_out/qa/fullsize_word.log 2>&1
