#!/bin/bash
# One measurement session on the GPU box: the default bench line (the
# driver's command), a kernel-trace --stats profile of the timed rounds, and
# the PMC traffic passes (tools/pmc.sh). Each GPU step has its own limit; the
# chain stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- \
  python3 bench.py --no-cpu-baseline --no-secondary --files 0 > gpurun_out/prof.log 2>&1 &&
bash tools/pmc.sh > gpurun_out/pmc.log 2>&1
