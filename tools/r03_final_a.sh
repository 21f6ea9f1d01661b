#!/bin/bash
# Round 3 final tree, part A: the whole -m gpu suite (one process), then smoke.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread -s > gpurun_out/r03_final_pytest_gpu.log 2>&1 &&
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03_final_smoke.log 2>&1
