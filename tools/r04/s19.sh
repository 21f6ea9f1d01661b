#!/bin/bash
# the crash leg's heavy rounds under a kernel trace
set -o pipefail
mkdir -p gpurun_out/r04/s19
export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r04/s19/prof -o run -- \
  python3 -u tools/r04/crash_probe.py > gpurun_out/r04/s19/probe.log 2>&1 || exit 1
cat gpurun_out/r04/s19/probe.log
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/r04/s19/prof/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
st = [i for i, r in enumerate(rows) if "k_prologue" in r["Kernel_Name"]]
for rr in (23, 24, 25, 26):  # round rr starts at prologue index rr - 1
    a, b = st[rr - 1], st[rr]
    t0 = int(rows[a]["Start_Timestamp"])
    print("== round", rr, (int(rows[b]["Start_Timestamp"]) - t0) / 1e3, "us")
    for r in rows[a:b]:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        if d > 8: print(f"   {(int(r['Start_Timestamp']) - t0) / 1e3:8.1f} {d:8.1f}  {r['Kernel_Name'][:90]}")
PY
