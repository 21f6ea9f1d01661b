#!/bin/bash
# Steady-state A/B, 3 passes x 40 timed rounds: tier tombstones gated per
# wave (default), ungated (tombng), the round-3 rule (notomb: steady state
# only, its gossiphip.o still sets the tier's tombstone offset); crash leg on
# tombng.
set -o pipefail
mkdir -p gpurun_out/s15
V=p2p-file-system-with-gossip-detect-failure-management_amd/lib/variants
rm -f gpurun_out/nib_ab/summary.txt &&
NIB_AB_PASSES="1 2 3" NIB_AB_STEPS=40 bash tools/nib_ab.sh default notomb tombng &&
GOSSIPHIP_LIB=$V/libgossiphip_tombng.so timeout -k 10 200 python -u tools/crash_leg.py > gpurun_out/s15/crash_tombng.json 2> gpurun_out/s15/crash_tombng.err
