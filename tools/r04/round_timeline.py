"""One steady round's kernels (start, end, duration in us from the round's
k_prologue) from a rocprofv3 kernel trace directory, and per-kernel medians."""
import csv
import glob
import statistics
import sys

f = glob.glob(f"{sys.argv[1]}/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
st = [i for i, r in enumerate(rows) if "k_prologue" in r["Kernel_Name"]]
a, b = st[-3], st[-2]
t0 = int(rows[a]["Start_Timestamp"])
for r in rows[a:b + 1]:
    s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
    print(f"{s / 1e3:8.1f} {e / 1e3:8.1f} {(e - s) / 1e3:7.1f}  {r['Kernel_Name'][:90]}")
print("round length", (int(rows[b]["Start_Timestamp"]) - t0) / 1e3, "us")
lens = [(int(rows[st[k + 1]]["Start_Timestamp"]) - int(rows[st[k]]["Start_Timestamp"])) / 1e3 for k in range(5, len(st) - 1)]
print("median round length", statistics.median(lens), "us")
