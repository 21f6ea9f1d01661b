#!/bin/bash
# k_round ablations / layout sweep (timing only; results are wrong by design
# when ABLATE != 0):  ABLATE=1 every peer load reads the own row segment
# (cache hits), ABLATE=2 no peer loads at all.  CONFIGS="ablate:tw:tpw[:xmap] ..."
set -o pipefail
mkdir -p gpurun_out
for cfg in ${CONFIGS:-0:64:4 1:64:4 2:64:4 0:64:1 0:64:8 0:128:2 0:128:4 0:256:1 0:256:2 2:128:4}; do
  IFS=: read -r ab tw tpw xm <<< "$cfg"
  GH_ROUND_ABLATE=$ab GH_TILE_W=$tw GH_ROUND_TPW=$tpw GH_ROUND_XMAP=${xm:-0} timeout -k 10 120 python -u bench.py --steps 6 --warmup 4 \
    --no-cpu-baseline > gpurun_out/ablate_$cfg.json 2> gpurun_out/ablate_$cfg.err || exit 1
  python -c "import json; d=json.load(open('gpurun_out/ablate_$cfg.json')); print('ablate=$ab tw=$tw tpw=$tpw xmap=${xm:-0}', round(d['roofline']['avg_launch_ms'],2), 'ms')"
done
