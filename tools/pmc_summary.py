"""Per-dispatch averages of the PMC passes of tools/pmc.sh for k_round:
  python tools/pmc_summary.py gpurun_out/pmc [N K] > summary.json
(N, K = the bench configuration the passes ran, recorded for bench.py)."""
import csv
import glob
import json
import sys
from collections import defaultdict

root = sys.argv[1]
# per k_round variant (lean / storm: both are launched every round, the one
# not selected returns at once); the summary is the variant that ran
byk = defaultdict(lambda: defaultdict(list))
for f in glob.glob(f"{root}/p*/**/*counter_collection.csv", recursive=True):
    for row in csv.DictReader(open(f)):
        name = row.get("Kernel_Name", "")
        if "::k_round<" not in name:  # the round kernel, not k_round_slow
            continue
        byk[name][row["Counter_Name"]].append(float(row["Counter_Value"]))
kern = max(byk, key=lambda k: sum(sum(v) for v in byk[k].values())) if byk else None
acc = byk[kern] if kern else {}
out = {k: {"per_dispatch": sum(v) / len(v), "dispatches": len(v)} for k, v in acc.items()}
out["kernel"] = kern
if "FETCH_SIZE" in out:  # KB; gfx950 counts half of a wide streaming read (MI355X_MICROARCH.md)
    out["read_bytes_corrected"] = out["FETCH_SIZE"]["per_dispatch"] * 1024 * 2
if "WRITE_SIZE" in out:
    out["write_bytes"] = out["WRITE_SIZE"]["per_dispatch"] * 1024
if "TCC_HIT_sum" in out and "TCC_MISS_sum" in out:
    h, m = out["TCC_HIT_sum"]["per_dispatch"], out["TCC_MISS_sum"]["per_dispatch"]
    out["l2_hit_rate"] = h / (h + m)
if "read_bytes_corrected" in out and "write_bytes" in out:
    out["traffic_bytes"] = out["read_bytes_corrected"] + out["write_bytes"]
n, k = (int(x) for x in sys.argv[2:4]) if len(sys.argv) >= 4 else (65536, 4)
out["config"] = {"n": n, "k": k, "world": 1, "cell_bytes": 2,
                 "command": "python3 bench.py --steps 3 --warmup 2 --no-cpu-baseline"}
out["algorithmic_bytes"] = 2.0 * n * n * (k + 2)  # narrow cells: own in + out, k peers in
print(json.dumps(out, indent=1))
