"""How far SPEC D4 (REMOVE delivered to every running member, GH_REMOVE_ALL)
departs from the reference's literal recipients (the detector's list at the
moment of Remove, GH_REMOVE_LIST) at the reference's own timeouts at full
size: N=65,536, k=4 pull, T_fail = T_cleanup = 5 (slave/slave.go:24-25).
Per round: both engines' counters; at a few rounds the number of cells whose
exported (hb, ts) differ."""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "p2p-file-system-with-gossip-detect-failure-management_amd"))
import gossipsim as gs  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 14
eng = {m: gs.Engine(gs.default_config(N, fanout=4, seed=0x5EED0003, t_fail=5, t_cleanup=5, remove_mode=m))
       for m in (gs.GH_REMOVE_ALL, gs.GH_REMOVE_LIST)}
for e in eng.values():
    e.init_full(2, 0, 0)
out = []
for r in range(1, rounds + 1):
    st = {m: e.step(1) for m, e in eng.items()}
    rec = {"r": r, "all": st[gs.GH_REMOVE_ALL], "list": st[gs.GH_REMOVE_LIST]}
    if r in (6, 7, 8, 10, rounds):
        dh = dt = 0
        for r0 in range(0, N, 4096):
            a = eng[gs.GH_REMOVE_ALL].export_state(r0, min(4096, N - r0))
            b = eng[gs.GH_REMOVE_LIST].export_state(r0, min(4096, N - r0))
            dh += int((a[0] != b[0]).sum())
            dt += int(((a[1] != b[1]) & (a[0] == b[0])).sum())
        rec["cells_hb_differ"] = dh
        rec["cells_ts_differ"] = dt
        fa, fl = eng[gs.GH_REMOVE_ALL].read_failed(), eng[gs.GH_REMOVE_LIST].read_failed()
        rec["failed_set_equal"] = bool((fa == fl).all())
    print(json.dumps(rec), flush=True)
    out.append(rec)
for e in eng.values():
    e.close()
