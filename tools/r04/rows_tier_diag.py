"""Row shards with the 4-bit tier vs one engine: first round and cells that differ."""
import os, sys
os.environ["GH_PLANE"] = "1"
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "p2p-file-system-with-gossip-detect-failure-management_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))
import numpy as np
import gossipsim as gs
import scenarios as sc
n, G = int(sys.argv[1]) if len(sys.argv) > 1 else 1100, int(sys.argv[2]) if len(sys.argv) > 2 else 2
cfg = dict(fanout=4, seed=0x5EED0600 + G, t_fail=6, t_cleanup=8)
sched = sc.random_churn(n, 24, 0xB0 + G, p_crash=0.01, p_leave=0.01, p_join=0.03) if "churn" in sys.argv else {}
one = gs.Engine(gs.default_config(n, **cfg))
grp = gs.ShardGroup(gs.default_config(n, shard_layout=1, **cfg), G)
init = sc.full_state(n)
one.import_state(*init, 0)
grp.import_state(*init, 0)
for r in range(1, 8):
    if r in sched:
        print("  events", sched[r][:6], len(sched[r]))
        one.apply_events(sched[r])
        grp.apply_events(sched[r])
    a, b = one.step(1), grp.step(1)
    ti = grp.run("tier_info", full=True)
    print("round", r, "single", a["merged_cells"], "rows", b["merged_cells"], "tier", ti, one.tier_info(full=True), flush=True)
    h1, t1, _ = one.export_state()
    h2, t2, _ = grp.export_state()
    bad = np.argwhere((h1 != h2) | (t1 != t2))
    if len(bad):
        print("  differing cells", len(bad), "rows with diffs per shard", np.bincount(bad[:, 0] // ((n + G - 1) // G)))
        ex = grp.run("exchange_info")
        print("  exchange", ex)
        for i, c in bad[:8]:
            print("   ", i, c, "single", h1[i, c], t1[i, c], "rows", h2[i, c], t2[i, c])
        break
