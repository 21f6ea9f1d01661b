"""Cost of GH_ORDER_APPEND (list order kept per row) against GH_ORDER_ID on
the same cluster: rounds/s for pull and ring mode at a given N
(python tools/order_probe.py [n] [rounds])."""
import pathlib
import sys
import time

REPO = pathlib.Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO), str(REPO / "p2p-file-system-with-gossip-detect-failure-management_amd")]

import gossipsim as gs  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 5
for mode in ("pull", "ring"):
    for order in (0, 1):
        cfg = gs.default_config(n, fanout=4, seed=0x5EED0003, t_fail=16, t_cleanup=16, list_order=order,
                                peer_mode=gs.GH_PEER_RING if mode == "ring" else gs.GH_PEER_PULL)
        eng = gs.Engine(cfg)
        eng.init_full()
        eng.step(4)
        eng.sync()
        t = time.perf_counter()
        st = eng.step(rounds)
        eng.sync()
        el = time.perf_counter() - t
        print(f"{mode:4s} order={'append' if order else 'id':6s} n={n} {rounds / el:8.2f} rounds/s "
              f"({1e3 * el / rounds:.2f} ms/round) merged={st['merged_cells']}", flush=True)
        eng.close()
