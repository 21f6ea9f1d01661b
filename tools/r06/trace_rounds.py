"""Split a rocprofv3 kernel trace into rounds and list each chosen round's
kernels by total time.
  python tools/r06/trace_rounds.py TRACE_DIR MARKER PER_ROUND ROUND [ROUND ...]
MARKER: a kernel name substring that starts every round (k_prologue for one
engine, k_base for shards); PER_ROUND: its launches per round (1, or the
shard count); ROUND: 1-based round numbers of the run."""
import collections
import csv
import glob
import re
import sys


def short(name):
    """k_round<4, 256, 1, true, false, 2> from the demangled kernel name"""
    name = re.sub(r"\(anonymous namespace\)::", "", name)
    name = re.sub(r"^void ", "", name)
    depth, out = 0, []
    for ch in name:
        if ch == "(" and depth == 0:
            break
        depth += ch == "<"
        depth -= ch == ">"
        out.append(ch)
    return "".join(out)[:80]

d, marker, per = sys.argv[1], sys.argv[2], int(sys.argv[3])
want = [int(x) for x in sys.argv[4:]]
f = glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
marks = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]][::per]
print(f"{len(marks)} rounds found")
for r in want:
    if r > len(marks):
        continue
    a = marks[r - 1]
    b = marks[r] if r < len(marks) else len(rows)
    t0 = int(rows[a]["Start_Timestamp"])
    t1 = int(rows[b]["Start_Timestamp"]) if b < len(rows) else int(rows[b - 1]["End_Timestamp"])
    tot = collections.defaultdict(lambda: [0, 0.0])
    for x in rows[a:b]:
        name = short(x["Kernel_Name"])
        tot[name][0] += 1
        tot[name][1] += (int(x["End_Timestamp"]) - int(x["Start_Timestamp"])) / 1e3
    busy = sum(v[1] for v in tot.values())
    print(f"round {r}: span {(t1 - t0) / 1e3:.1f} us, kernel time {busy:.1f} us, {b - a} launches")
    for name, (c, us) in sorted(tot.items(), key=lambda kv: -kv[1][1])[:12]:
        print(f"  {us:9.1f} us  x{c:<4d} {name}")
