#!/bin/bash
# Sender-plane A/B on one box: bench lines at TW=256 (plane), TW=64 (plane)
# and TW=64 without the plane, then the GPU parity suite.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
B="python -u bench.py --no-cpu-baseline --no-secondary --files 0"
timeout -k 10 240 $B > gpurun_out/pc_tw256.json 2> gpurun_out/pc_tw256.err &&
GH_TILE_W=64 timeout -k 10 240 $B > gpurun_out/pc_tw64.json 2> gpurun_out/pc_tw64.err &&
GH_PLANE=0 GH_TILE_W=64 timeout -k 10 240 $B > gpurun_out/pc_noplane.json 2> gpurun_out/pc_noplane.err &&
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
