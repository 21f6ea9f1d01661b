#!/bin/bash
# 8-bit tier session: its parity tests first, then the whole GPU suite and
# the bench line. Every GPU step has its own limit; the chain stops at the
# first failure.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_tier8.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_tier8.log 2>&1 &&
timeout -k 10 240 python -u bench.py --no-cpu-baseline --no-secondary --files 0 > gpurun_out/bench_quick.log 2>&1 &&
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
