"""Per-dispatch averages of the PMC passes of tools/pmc.sh for k_round, over
the timed (last `steps`) dispatches of the variant that ran:
  python tools/pmc_summary.py gpurun_out/pmc N K WARMUP STEPS > summary.json"""
import csv
import glob
import json
import sys
from collections import defaultdict

root = sys.argv[1]
n, k, warmup, steps = (int(x) for x in sys.argv[2:6]) if len(sys.argv) >= 6 else (65536, 4, 12, 5)
# per k_round variant (lean / storm: both are launched every round, the one
# not selected returns at once) and counter: (dispatch id, value)
byk = defaultdict(lambda: defaultdict(list))
for f in glob.glob(f"{root}/p*/**/*counter_collection.csv", recursive=True):
    for row in csv.DictReader(open(f)):
        name = row.get("Kernel_Name", "")
        if "::k_round<" not in name:  # the round kernel, not k_round_slow
            continue
        byk[name][row["Counter_Name"]].append((int(row.get("Dispatch_Id", 0)), float(row["Counter_Value"])))
kern = max(byk, key=lambda kk: sum(v for lst in byk[kk].values() for _, v in lst)) if byk else None
out = {}
for ctr, lst in (byk[kern].items() if kern else []):
    lst = sorted(lst)[-steps:]  # the timed rounds (steady state), not the warm-up
    out[ctr] = {"per_dispatch": sum(v for _, v in lst) / len(lst), "dispatches": len(lst)}
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
import os  # noqa: E402
# the layout the pass ran with (bench.py matches it): pull with 3 <= k <= 4
# at N >= 16,384 keeps the sender plane at TW=256 unless GH_PLANE / GH_TILE_W
# say otherwise
plane = int(3 <= k <= 4 and (os.environ["GH_PLANE"] != "0" if "GH_PLANE" in os.environ else n >= 16384))
tw = int(os.environ.get("GH_TILE_W", "256" if plane else "64"))
# the 4-bit tier comes with the plane (column layout, one tile per workgroup)
tier4 = int(plane and os.environ.get("GH_C8", "1") != "0" and os.environ.get("GH_ROUND_TPW", "1") == "1")
enc = "t4" if tier4 else "u16"
out["config"] = {"n": n, "k": k, "world": 1, "encoding": enc, "warmup": warmup, "steps": steps,
                 "plane": plane, "tile_width": tw,
                 "command": f"python3 bench.py --steps {steps} --warmup {warmup} --no-cpu-baseline --no-secondary "
                            "--files 0"}
# compulsory bytes: t4 = lag + age nibbles in and out (the lag nibbles are the
# plane); u16 = 2-B cells in and out, the plane out and in
out["compulsory_bytes"] = (2.0 if tier4 else (4.0 + (1.0 if plane else 0.0))) * n * n
out["prev_model_bytes"] = 3.0 * n * n  # round 2's 8-bit tier model (1-B cells + the plane)
out["gather_bytes"] = (0.5 if (tier4 or plane) else 2.0) * n * n * k  # 4-bit plane codes per sender cell
# SQ / TA / TD / GRBM passes (if captured): per-dispatch figures
if "SQ_WAVE_CYCLES" in out:
    w = out["SQ_WAVE_CYCLES"]["per_dispatch"]
    out["sq"] = {c: out[c]["per_dispatch"] for c in list(out) if c.startswith("SQ_")}
    out["sq"]["wait_any_frac"] = out["SQ_WAIT_ANY"]["per_dispatch"] / w if "SQ_WAIT_ANY" in out else None
    out["sq"]["active_inst_frac"] = out["SQ_ACTIVE_INST_ANY"]["per_dispatch"] / w if "SQ_ACTIVE_INST_ANY" in out else None
    out["sq"]["wait_inst_frac"] = out["SQ_WAIT_INST_ANY"]["per_dispatch"] / w if "SQ_WAIT_INST_ANY" in out else None
if "GRBM_GUI_ACTIVE" in out:
    out["gpu_cycles_per_xcd"] = out["GRBM_GUI_ACTIVE"]["per_dispatch"] / 8
    if "SQ_INSTS_VALU" in out:  # VALU issue share: wave64 VALU = 2 cycles on a SIMD, 1,024 SIMDs
        out["valu_busy_frac"] = 2.0 * out["SQ_INSTS_VALU"]["per_dispatch"] / (1024 * out["gpu_cycles_per_xcd"])
if "TA_TA_BUSY_sum" in out and "GRBM_GUI_ACTIVE" in out:
    out["ta_busy_frac"] = out["TA_TA_BUSY_sum"]["per_dispatch"] / (256 * out["GRBM_GUI_ACTIVE"]["per_dispatch"] / 8)
if "TD_TD_BUSY_sum" in out and "GRBM_GUI_ACTIVE" in out:
    out["td_busy_frac"] = out["TD_TD_BUSY_sum"]["per_dispatch"] / (256 * out["GRBM_GUI_ACTIVE"]["per_dispatch"] / 8)
if "traffic_bytes" in out:
    out["traffic_over_compulsory"] = out["traffic_bytes"] / out["compulsory_bytes"]
print(json.dumps(out, indent=1))
