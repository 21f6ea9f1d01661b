#!/bin/bash
# k_round layout sweep (timing only): tile width x tiles per workgroup x
# XCD-aware map, through the engine's environment knobs.
#   CONFIGS="tw:tpw:xmap ..." bash tools/ablate.sh
set -o pipefail
mkdir -p gpurun_out
for cfg in ${CONFIGS:-64:1:1 64:1:0 128:1:1 64:2:1 32:1:1}; do
  IFS=: read -r tw tpw xm <<< "$cfg"
  GH_TILE_W=$tw GH_ROUND_TPW=$tpw GH_ROUND_XMAP=${xm:-1} timeout -k 10 120 python -u bench.py --steps 6 --warmup 4 \
    --no-cpu-baseline > gpurun_out/layout_$cfg.json 2> gpurun_out/layout_$cfg.err || exit 1
  python -c "import json; d=json.load(open('gpurun_out/layout_$cfg.json')); print('tw=$tw tpw=$tpw xmap=${xm:-1}', round(d['roofline']['avg_launch_ms'],2), 'ms')"
done
