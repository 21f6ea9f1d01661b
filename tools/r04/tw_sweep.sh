#!/bin/bash
# Tile-width sweep of the nibble path on one box: bench line per TW (HIP-event k_round mean).
set -o pipefail
mkdir -p gpurun_out/r04
B="python -u bench.py --steps 20 --warmup 5 --no-secondary --no-cpu-baseline --files 0"
for tw in ${TWS:-256 128 64 256}; do
  GH_TILE_W=$tw timeout -k 10 240 $B > gpurun_out/r04/tw_$tw.json 2> gpurun_out/r04/tw_$tw.err || exit $?
  python - "$tw" <<'PY'
import json, sys
d = json.loads(open(f"gpurun_out/r04/tw_{sys.argv[1]}.json").read().strip().splitlines()[-1])
r = d["roofline"]
print("TW", sys.argv[1], "value", round(d["value"], 1), "k_round_ms", round(r["avg_launch_ms"], 4),
      "variant", d["layout"]["last_variant"], "tw", d["layout"]["tile_width"], flush=True)
PY
done
