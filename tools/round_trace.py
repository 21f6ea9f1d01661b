"""Per-round trace at N=65,536 (MI355X): variant, k_round ms, active rows,
detections, slow segments.  python tools/round_trace.py [ring|pull] [T_fail] [rounds]"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "p2p-file-system-with-gossip-detect-failure-management_amd"))
import gossipsim as gs  # noqa: E402

mode = sys.argv[1] if len(sys.argv) > 1 else "ring"
tf = int(sys.argv[2]) if len(sys.argv) > 2 else 5
rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 32
n = 65536
cfg = gs.default_config(n, fanout=4, seed=0x5EED0003, t_fail=tf, t_cleanup=tf,
                        peer_mode=gs.GH_PEER_RING if mode == "ring" else gs.GH_PEER_PULL)
eng = gs.Engine(cfg)
eng.init_full(2, 0, 0)
eng.set_timing(True)
prev = 0.0
for r in range(1, rounds + 1):
    t0 = time.perf_counter()
    st = eng.step(1)
    wall = (time.perf_counter() - t0) * 1e3
    ms, _ = eng.read_timing()
    enc = eng.encoding_info(full=True)
    print(f"r={r:2d} k_round {ms - prev:6.3f} ms  wall {wall:6.2f} ms  variant {'storm' if enc[2] else 'lean '} "
          f"slow {enc[1]:8d} active {st['active_rows']:6d} det {st['detections']:10d} merged {st['merged_cells']}",
          flush=True)
    prev = ms
