#!/bin/bash
# PMC passes for k_round (one counter group per run, kernel trace only; the
# guide's rules: FETCH_SIZE and WRITE_SIZE in separate passes).
set -o pipefail
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
i=0
for ctr in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $ctr --output-format csv -d gpurun_out/pmc/p$i -o run -- \
    python3 bench.py --steps 3 --warmup 2 --no-cpu-baseline > gpurun_out/pmc/p$i.log 2>&1 || exit 1
done
python3 tools/pmc_summary.py gpurun_out/pmc > gpurun_out/pmc/summary.json
