#!/bin/bash
# Whole-word nibble rule (GH_NIB_WORD=1, lib/variants/libgossiphip_word.so)
# against the default build: tier / plane / narrow parity and the full-size
# steady state on the variant, then the quick bench of both, twice.
set -o pipefail
mkdir -p gpurun_out/word
W=p2p-file-system-with-gossip-detect-failure-management_amd/lib/variants/libgossiphip_word.so
GOSSIPHIP_LIB=$W timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_tier8.py tests/test_gpu_plane.py tests/test_gpu_narrow.py tests/test_gpu_parity.py > gpurun_out/word/tests.log 2>&1 &&
GOSSIPHIP_LIB=$W timeout -k 10 500 python -u -m pytest -x -v --timeout 450 --timeout-method thread -s tests/test_gpu_fullsize.py -k steady > gpurun_out/word/fullsize.log 2>&1 &&
bash tools/nib_ab.sh default word
