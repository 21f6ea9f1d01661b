#!/bin/bash
# Tier tombstones with only the tombstone masks gated per wave (default) vs
# ungated (tombng) vs the round-3 rule (notomb, steady state only): parity
# subset on the default build, then the 3-pass steady-state A/B.
set -o pipefail
mkdir -p gpurun_out/s16
timeout -k 10 120 python -u tools/tomb_diag.py > gpurun_out/s16/diag.log 2>&1 &&
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_tier8.py tests/test_gpu_parity.py > gpurun_out/s16/tests.log 2>&1 &&
rm -f gpurun_out/nib_ab/summary.txt &&
NIB_AB_PASSES="1 2 3" NIB_AB_STEPS=40 bash tools/nib_ab.sh default notomb tombng
