#!/bin/bash
# kernel breakdown of the row-shard ring round and the column round (8 shards, one GPU)
set -o pipefail
mkdir -p gpurun_out/r04/s7
export TMPDIR=/tmp
for l in rows_ring columns_pull; do
  GH_EXCHANGE_ONLY=$l timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04/s7/$l -o run -- \
    python3 tools/shard_exchange.py 65536 8 10 > gpurun_out/r04/s7/$l.log 2>&1 || exit 1
done
python3 - <<'PY'
import csv, glob
for l in ("rows_ring", "columns_pull"):
    f = glob.glob(f"gpurun_out/r04/s7/{l}/**/*kernel_stats.csv", recursive=True)[0]
    rows = list(csv.DictReader(open(f)))
    rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
    print("==", l)
    for r in rows[:25]:
        print(f'{float(r["TotalDurationNs"])/1e6:10.2f} ms {int(r["Calls"]):7d} {float(r["AverageNs"])/1e3:9.1f} us  {r["Name"][:110]}')
PY
