"""GPU busy time by kernel class over the last rounds of a rocprofv3 kernel
trace: the union of the launches' [start, end) intervals per class and over
all, so that launches of concurrent streams (in-process shards) are not
counted twice. The window runs from the end of the (rounds * shards + 1)-th
last k_finish to the end of the last one.
  python tools/r05/busy_union.py <rocprof dir> [rounds] [shards]"""
import csv
import glob
import sys
from collections import defaultdict


def union(iv):
    tot, end = 0, None
    for s, e in sorted(iv):
        if end is None or s > end:
            tot += e - s
            end = e
        elif e > end:
            tot += e - end
            end = e
    return tot


d = sys.argv[1]
nr = int(sys.argv[2]) if len(sys.argv) > 2 else 3
ns = int(sys.argv[3]) if len(sys.argv) > 3 else 8
rows = []
for f in glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True) + glob.glob(f"{d}/**/*memory_copy_trace.csv",
                                                                              recursive=True):
    for r in csv.DictReader(open(f)):
        name = r.get("Kernel_Name") or ("copy " + r.get("Direction", ""))
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name))
fin = sorted(e for s, e, n in rows if "k_finish" in n)
lo, t1 = fin[-(nr * ns + 1)], fin[-1]
win = [(max(s, lo), min(e, t1), n) for s, e, n in rows if e > lo and s < t1]


def cls(n):
    for key in ("k_round_jobs", "k_round_slow", "k_round_redo", "k_round<", "k_ghost_pack", "copyBuffer", "fillBuffer",
                "k_copy_segs", "k_reduce", "k_want", "k_gx", "k_ghost", "k_peers", "k_inbox", "k_active", "k_base",
                "k_finish", "copy "):
        if key in n:
            return key
    return "other"


per = defaultdict(list)
for s, e, n in win:
    per[cls(n)].append((s, e))
span = (t1 - lo) / 1e6
print(f"window {span:.2f} ms ({nr} rounds, {span / nr:.2f} ms each), busy (any) {union([(s, e) for s, e, _ in win]) / 1e6:.2f} ms")
for k, iv in sorted(per.items(), key=lambda kv: -union(kv[1])):
    print(f"  {k:14s} {union(iv) / 1e6:8.2f} ms busy, {len(iv)} launches")
