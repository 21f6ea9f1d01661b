"""Per-round time of the bench workload (N=65,536, k=4 pull, T_fail =
T_cleanup = 16) with the kernel timing events off and on, alternating, to
show what the per-launch start/stop events add to a round.
  python tools/r05/fixed_cost.py [rounds] [passes]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..",
                                "p2p-file-system-with-gossip-detect-failure-management_amd"))
import gossipsim as gs  # noqa: E402

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 20
passes = int(sys.argv[2]) if len(sys.argv) > 2 else 3
n = 65536
eng = gs.Engine(gs.default_config(n, fanout=4, seed=0x5EED0003, t_fail=16, t_cleanup=16))
eng.init_full(2, 0, 0)
eng.step(5)
out = []
for p in range(passes):
    for timing in (False, True):
        eng.set_timing(timing)
        eng.sync()
        t0 = time.perf_counter()
        eng.step(rounds)
        eng.sync()
        dt = (time.perf_counter() - t0) / rounds * 1e3
        rec = {"pass": p, "timing": timing, "ms_per_round": round(dt, 4)}
        if timing:
            k, l = eng.read_timing()
            rec["k_round_ms"] = round(k / max(l, 1), 4)
        eng.set_timing(False)
        out.append(rec)
        print(json.dumps(rec), flush=True)
eng.close()
