#!/bin/bash
# Round 3: the nibble path's access-pattern floor and a FETCH_SIZE calibration
# at 4-B lanes (tools/nib_probe.hip, built in-tree as tools/bin/nib_probe),
# then SQ instruction-mix counters of the bench's k_round at warm-up 5.
# Every GPU step is time-limited; the script stops at the first failure.
set -o pipefail
mkdir -p gpurun_out/probe
export TMPDIR=/tmp
for m in 0 1 2 3 4; do
  timeout -k 10 60 tools/bin/nib_probe $m 10 >> gpurun_out/probe/times.jsonl || exit 1
done
for m in 1 2 3 4; do
  i=0
  for ctr in "FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_BUBBLE_sum" \
             "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum" "TCC_EA0_RDREQ_DRAM_sum TCC_REQ_sum"; do
    i=$((i+1))
    timeout -s KILL 60 rocprofv3 --pmc $ctr --output-format csv -d gpurun_out/probe/m$m/p$i -o run -- \
      tools/bin/nib_probe $m 3 > gpurun_out/probe/m$m.p$i.log 2>&1 || exit 1
  done
done
CMD="python3 bench.py --steps 5 --warmup 5 --no-cpu-baseline --no-secondary --files 0"
i=0
for ctr in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
           "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM_RD SQ_INSTS_SMEM GRBM_GUI_ACTIVE" \
           "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_BUBBLE_sum" "TCC_EA0_RDREQ_DRAM_sum TCC_REQ_sum"; do
  i=$((i+1))
  timeout -s KILL 180 rocprofv3 --pmc $ctr --output-format csv -d gpurun_out/probe/sq/p$i -o run -- \
    $CMD > gpurun_out/probe/sq.p$i.log 2>&1 || exit 1
done
