#!/bin/bash
# PMC passes (one counter group per run, kernel trace only) of the nibble
# path at tile widths TWS, bench steady state; counters absent from
# rocprofv3 -L are dropped from a pass. -> gpurun_out/r04/pmc_tw/
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04/pmc_tw
mkdir -p $O
timeout -s KILL 60 rocprofv3 -L > $O/avail.txt 2>&1 || exit 1
CMD="python3 bench.py --steps ${STEPS:-10} --warmup 5 --no-cpu-baseline --no-secondary --files 0"
PASSES=("FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum"
  "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"
  "TA_TA_BUSY_sum TA_BUFFER_READ_WAVEFRONTS_sum TD_TD_BUSY_sum TD_SPI_STALL_sum"
  "TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum"
  "GRBM_GUI_ACTIVE GRBM_COUNT")
for tw in ${TWS:-256 128}; do
  i=0
  for pass in "${PASSES[@]}"; do
    i=$((i+1))
    ok=""
    for c in $pass; do
      base=${c%_sum}
      if grep -qw -- "$base" $O/avail.txt || grep -qw -- "$c" $O/avail.txt; then ok="$ok $c"; fi
    done
    [ -z "$ok" ] && continue
    echo "tw $tw pass $i:$ok"
    GH_TILE_W=$tw timeout -s KILL 120 rocprofv3 --pmc $ok --kernel-include-regex 'k_round' --output-format csv \
      -d $O/tw${tw}_p$i -o run -- $CMD > $O/tw${tw}_p$i.log 2>&1 || { echo "pass failed rc=$?"; tail -5 $O/tw${tw}_p$i.log; exit 1; }
  done
done
echo done
