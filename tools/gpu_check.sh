#!/bin/bash
# One GPU session: parity tests, bench line, kernel-trace profile, PMC passes.
# Every GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python -u bench.py > gpurun_out/bench.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 10 --warmup 4 --no-cpu-baseline > gpurun_out/prof.log 2>&1 &&
bash tools/pmc.sh > gpurun_out/pmc.log 2>&1
