"""Per-kernel stats from a rocprofv3 kernel trace with the idle k_round
variants separated out. Every round launches all k_round variants; the one
the device selected does the round and the others return at once, but an
idle launch on the side stream is dispatched between the running variant's
workgroups, so its duration spans that variant's (rocprof's --stats then
counts it as a second ~2 ms kernel). Here, in each round (k_prologue to
k_prologue), the k_round launch with the longest duration is the one that
ran; the others are listed as "<name> (idle)".
  python tools/r05/kernel_stats_active.py <rocprof output dir> > stats.csv"""
import csv
import glob
import sys
from collections import defaultdict

f = glob.glob(f"{sys.argv[1]}/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
agg = defaultdict(list)
cur = []


def flush(group):
    kr = [r for r in group if r["Kernel_Name"].lstrip().startswith("void (anonymous namespace)::k_round<")]
    run = max(kr, key=lambda r: int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) if kr else None
    for r in group:
        name = r["Kernel_Name"]
        if r in kr and r is not run:
            name += " (idle)"
        agg[name].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)


for r in rows:
    if "k_prologue" in r["Kernel_Name"] and cur:
        flush(cur)
        cur = []
    cur.append(r)
if cur:
    flush(cur)
w = csv.writer(sys.stdout)
w.writerow(["Name", "Calls", "TotalDurationUs", "AverageUs", "MinUs", "MaxUs"])
for name, d in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
    w.writerow([name, len(d), round(sum(d), 1), round(sum(d) / len(d), 2), round(min(d), 2), round(max(d), 2)])
