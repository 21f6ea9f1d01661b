#!/bin/bash
# the crash leg's rounds: k_round per round, and a kernel trace of them
set -o pipefail
mkdir -p gpurun_out/r05
O=gpurun_out/r05
export TMPDIR=/tmp
timeout -k 10 300 python3 tools/r05/crash_rounds.py 30 > $O/s20_crash_rounds.jsonl 2>&1 || exit 1
timeout -s KILL 300 rocprofv3 --kernel-trace --output-format csv -d $O/tl20 -o run -- \
  python3 tools/r05/crash_rounds.py 30 > $O/s20_crash_rounds_prof.txt 2>&1 || exit 1
