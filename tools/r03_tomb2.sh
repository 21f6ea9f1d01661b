#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/tomb
timeout -k 10 120 python -u tools/tomb_diag.py > gpurun_out/tomb/diag.log 2>&1 &&
bash tools/r03_tomb.sh
