#!/bin/bash
# kernel stats of the two collapsed legs (40 rounds: 27+ quiet)
set -o pipefail
mkdir -p gpurun_out/r04/s14
export TMPDIR=/tmp
for leg in ref ring; do
  timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04/s14/$leg -o run -- \
    python3 -u tools/r04/leg_probe.py $leg 40 > gpurun_out/r04/s14/$leg.log 2>&1 || exit 1
done
python3 - <<'PY'
import csv, glob
for leg in ("ref", "ring"):
    f = glob.glob(f"gpurun_out/r04/s14/{leg}/**/*kernel_stats.csv", recursive=True)[0]
    rows = sorted(csv.DictReader(open(f)), key=lambda r: -float(r["TotalDurationNs"]))
    print("==", leg)
    for r in rows[:22]:
        print(f'{float(r["TotalDurationNs"])/1e6:10.2f} ms {int(r["Calls"]):7d} {float(r["AverageNs"])/1e3:9.1f} us  {r["Name"][:100]}')
PY
