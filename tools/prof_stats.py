"""Kernel statistics (rocprofv3 --stats equivalent) from a rocprofv3 .db:
  python tools/prof_stats.py gpurun_out/prof/run_results.db > profiles/x.csv"""
import sqlite3
import sys

con = sqlite3.connect(sys.argv[1])
rows = con.execute(
    "select name, count(*), sum(end-start), avg(end-start), min(end-start), max(end-start) "
    "from kernels group by name order by sum(end-start) desc").fetchall()
total = sum(r[2] for r in rows) or 1
print('"Name","Calls","TotalDurationNs","AverageNs","Percentage","MinNs","MaxNs"')
for name, calls, tot, avg, mn, mx in rows:
    print(f'"{name}",{calls},{tot},{avg:.1f},{100.0 * tot / total:.3f},{mn},{mx}')
