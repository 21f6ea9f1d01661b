#!/bin/bash
# split-sender gather probe (tools/r05/gprobe4.hip): modes 0 / 1, alternating three times
set -o pipefail
mkdir -p gpurun_out/r05
for pass in 1 2 3; do
  for m in 0 1; do
    timeout -k 10 60 tools/bin/gprobe4 $m | tee -a gpurun_out/r05/gprobe4.jsonl || exit 1
  done
done
