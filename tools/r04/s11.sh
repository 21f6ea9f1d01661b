#!/bin/bash
# the reference-timeouts leg round by round, then its kernel stats
set -o pipefail
mkdir -p gpurun_out/r04/s11
export TMPDIR=/tmp
timeout -k 10 300 python3 -u tools/r04/leg_probe.py ref 24 > gpurun_out/r04/s11/ref.log 2>&1; rc=$?; cut -c1-300 gpurun_out/r04/s11/ref.log; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04/s11/prof -o run -- \
  python3 -u tools/r04/leg_probe.py ref 24 > gpurun_out/r04/s11/prof.log 2>&1 || exit 1
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/r04/s11/prof/**/*kernel_stats.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:25]:
    print(f'{float(r["TotalDurationNs"])/1e6:10.2f} ms {int(r["Calls"]):7d} {float(r["AverageNs"])/1e3:9.1f} us  {r["Name"][:110]}')
PY
