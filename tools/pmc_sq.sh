#!/bin/bash
# SQ instruction mix / occupancy counters for k_round at the bench's steady
# state (one pass each), kernel trace only.
set -o pipefail
mkdir -p gpurun_out/pmcsq
export TMPDIR=/tmp
CMD="python3 bench.py --steps 3 --warmup 12 --no-cpu-baseline --no-secondary --files 0"
i=0
for ctr in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
           "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM_RD SQ_INSTS_SMEM GRBM_GUI_ACTIVE" \
           "SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_SALU SQ_WAVE_CYCLES"; do
  i=$((i+1))
  timeout -s KILL 180 rocprofv3 --pmc $ctr --output-format csv -d gpurun_out/pmcsq/p$i -o run -- \
    $CMD > gpurun_out/pmcsq/p$i.log 2>&1 || exit 1
done
python3 tools/pmc_summary.py gpurun_out/pmcsq 65536 4 12 3 > gpurun_out/pmcsq/summary.json
