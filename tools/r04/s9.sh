#!/bin/bash
# event rounds at full size: wall times, then the kernel stats of the same run
set -o pipefail
mkdir -p gpurun_out/r04/s9
export TMPDIR=/tmp
timeout -k 10 300 python3 -u tools/r04/event_probe.py > gpurun_out/r04/s9/probe.log 2>&1; rc=$?; cat gpurun_out/r04/s9/probe.log; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04/s9/prof -o run -- \
  python3 -u tools/r04/event_probe.py > gpurun_out/r04/s9/prof.log 2>&1 || exit 1
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/r04/s9/prof/**/*kernel_stats.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:25]:
    print(f'{float(r["TotalDurationNs"])/1e6:10.2f} ms {int(r["Calls"]):7d} {float(r["AverageNs"])/1e3:9.1f} us  {r["Name"][:110]}')
PY
