#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r04
for args in "16 0 1 1 0" "16 0 1 1 1" "16 1 1 1 0" "16 1 1 1 1" "32 0 1 1 1" "32 1 1 1 1" "16 1 4 1 1" "16 0 1 1 0" "16 0 1 1 1" "16 1 1 1 0" "16 1 1 1 1"; do
  timeout -k 10 60 tools/bin/gprobe $args | tee -a gpurun_out/r04/gprobe2.jsonl || exit 1
done
