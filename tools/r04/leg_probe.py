"""Per-round wall time of a bench secondary leg at N=65,536 (ref: T_fail =
T_cleanup = 5 pull; ring: the same with ring push), for profiling."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "p2p-file-system-with-gossip-detect-failure-management_amd"))
import gossipsim as gs  # noqa: E402

leg = sys.argv[1] if len(sys.argv) > 1 else "ref"
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 24
kw = dict(peer_mode=gs.GH_PEER_RING) if leg == "ring" else dict(fanout=4)
eng = gs.Engine(gs.default_config(65536, seed=0x5EED0003, t_fail=5, t_cleanup=5, **kw))
eng.init_full(2, 0, 0)
for r in range(1, rounds + 1):
    eng.sync()
    t0 = time.perf_counter()
    s = eng.step(1)
    eng.sync()
    print(f"r={r}: {1e3 * (time.perf_counter() - t0):.2f} ms variant {eng.tier_info(full=True)[3]} "
          f"enc {eng.encoding_info(full=True)} active {s['active_rows']} det {s['detections']} rel {s['released']} "
          f"tomb {s['tombstoned']} unk {s['remove_unknown']}", flush=True)
eng.close()
