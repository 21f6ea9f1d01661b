"""Sender-plane diagnostic (MI355X): the bench's configuration round by round,
with the plane's validity, its fallback waves and the k_round time.
  python tools/plane_diag.py [N] [rounds]"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "p2p-file-system-with-gossip-detect-failure-management_amd"))
import gossipsim as gs  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 16
eng = gs.Engine(gs.default_config(n, fanout=4, seed=0x5EED0003, t_fail=16, t_cleanup=16))
eng.init_full(2, 0, 0)
eng.set_timing(True)
print("plane", eng.plane_info(), "mem", eng.memory_info(), flush=True)
for r in range(1, rounds + 1):
    t0 = time.perf_counter()
    st = eng.step(1)
    dt = time.perf_counter() - t0
    print(r, "plane", eng.plane_info(), "enc", eng.encoding_info(full=True), "timing", eng.read_timing(),
          "%.2f ms" % (dt * 1e3), "merged", st["merged_cells"], flush=True)
