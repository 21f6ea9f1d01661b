"""Host-side probe for the CPU baseline plan (BASELINE.md "CPU baseline plan"):
prints nproc / lscpu model / memory and times oracle/tablesim.c whole-cluster
rounds at a few sizes and thread counts. Test infrastructure (loads the
oracle); not part of the product."""
import os
import subprocess
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import oracle as om  # noqa: E402


def host():
    model = "?"
    for line in subprocess.run(["lscpu"], capture_output=True, text=True).stdout.splitlines():
        if line.startswith("Model name"):
            model = line.split(":", 1)[1].strip()
    mem = "?"
    for line in open("/proc/meminfo"):
        if line.startswith("MemTotal"):
            mem = line.split()[1]
    aff = len(os.sched_getaffinity(0))
    nproc = subprocess.run(["nproc"], capture_output=True, text=True).stdout.strip()
    print(f"nproc={nproc} cpu_count={os.cpu_count()} affinity={aff} model={model} MemTotal_kB={mem}", flush=True)


def rate(n, threads, rounds, t_fail=16, k=4):
    cfg = om.default_config(n, fanout=k, seed=0x5EED0003, t_fail=t_fail, t_cleanup=t_fail)
    o = om.Oracle(cfg, threads=threads)
    o.init_full(2, 0, 0)
    o.step(1)
    t0 = time.perf_counter()
    o.step(rounds)
    el = time.perf_counter() - t0
    o.close()
    print(f"N={n} k={k} threads={threads}: {rounds / el:.4f} rounds/s ({el / rounds:.2f} s/round)", flush=True)


if __name__ == "__main__":
    om.build()
    host()
    for spec in sys.argv[1:]:
        n, th, r = (int(x) for x in spec.split(":"))
        rate(n, th, r)
