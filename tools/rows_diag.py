"""Row-layout diagnostic: import a full state into a world-G ShardGroup and
print every rank's outcome (no close on failure: a rank stuck in a barrier
keeps its engine).  python tools/rows_diag.py [G] [N]"""
import os
import sys
from concurrent.futures import wait

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "p2p-file-system-with-gossip-detect-failure-management_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import gossipsim as gs  # noqa: E402
import scenarios as sc  # noqa: E402

G = int(sys.argv[1]) if len(sys.argv) > 1 else 4
n = int(sys.argv[2]) if len(sys.argv) > 2 else 257
grp = gs.ShardGroup(gs.default_config(n, fanout=3, seed=0x7D, shard_layout=1), G)
init = sc.full_state(n)
futs = [grp.pool.submit(e.import_state, *init, 0) for e in grp.engines]
done, pend = wait(futs, timeout=30)
for r, f in enumerate(futs):
    print(r, "done" if f.done() else "PENDING", f.exception() if f.done() else "", flush=True)
os._exit(0)
