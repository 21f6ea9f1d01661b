#!/bin/bash
# PMC passes for k_round at the bench's own steady state (one counter group
# per run, kernel trace only; the guide's rules: FETCH_SIZE and WRITE_SIZE in
# separate passes), then a kernel-trace --stats run of the same command.
#   tools/pmc.sh [warmup] [steps]   -> gpurun_out/pmc/summary.json, gpurun_out/pmc/stats/
set -o pipefail
W=${1:-5}
S=${2:-20}
CMD="python3 bench.py --steps $S --warmup $W --no-cpu-baseline --no-secondary --files 0"
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
i=0
for ctr in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum" \
  "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
  "TA_TA_BUSY_sum TD_TD_BUSY_sum" "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $ctr --kernel-include-regex 'k_round' --output-format csv -d gpurun_out/pmc/p$i -o run -- \
    $CMD > gpurun_out/pmc/p$i.log 2>&1 || exit 1
done
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pmc/stats -o run -- \
  $CMD > gpurun_out/pmc/stats.log 2>&1 || exit 1
python3 tools/pmc_summary.py gpurun_out/pmc 65536 4 $W $S > gpurun_out/pmc/summary.json
