#!/bin/bash
# LDS-DMA staging probe (tools/r05/gprobe2.hip): modes 0..4, alternating twice
set -o pipefail
mkdir -p gpurun_out/r05
for pass in 1 2; do
  for m in 0 1 2 3 4; do
    timeout -k 10 60 tools/bin/gprobe2 $m 1 | tee -a gpurun_out/r05/gprobe2.jsonl || exit 1
  done
done
timeout -k 10 60 tools/bin/gprobe2 1 4 | tee -a gpurun_out/r05/gprobe2.jsonl || exit 1
timeout -k 10 60 tools/bin/gprobe2 0 4 | tee -a gpurun_out/r05/gprobe2.jsonl || exit 1
