#!/bin/bash
# two-round tile-group probe (tools/r05/gprobe3.hip): G = 256 (two whole passes) against 8/16/32/64-tile groups, alternating twice
set -o pipefail
mkdir -p gpurun_out/r05
for pass in 1 2; do
  for g in 256 0 8 16 32 64; do
    timeout -k 10 60 tools/bin/gprobe3 $g | tee -a gpurun_out/r05/gprobe3.jsonl || exit 1
  done
done
