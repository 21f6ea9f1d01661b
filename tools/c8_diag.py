"""How much of the benched steady state an 8-bit cell tier could hold
(DESIGN.md "Next"): after the bench's warm-up at N (default 16,384; pull,
k=4, T_fail=16), the share of 8-cell chunks whose every cell is visible and
unflagged with a lag in [-2, 12] behind the member's own counter and an age
<= 15, absent, or a tombstone aged <= 13 (python tools/c8_diag.py [n])."""
import pathlib
import sys

import numpy as np

REPO = pathlib.Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO), str(REPO / "p2p-file-system-with-gossip-detect-failure-management_amd")]

import gossipsim as gs  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
eng = gs.Engine(gs.default_config(n, fanout=4, seed=0x5EED0003, t_fail=16, t_cleanup=16))
eng.init_full()
for r in range(1, 21):
    eng.step(1)
    if r in (12, 16, 20):
        hb, ts, _ = eng.export_state()
        now = eng.round + 1
        own = np.diag(hb).astype(np.int64)
        lag = own[None, :] - hb
        age = now - ts.astype(np.int64)
        vis = (hb >= 0) & (lag >= -2) & (lag <= 12) & (age <= 15) & (age > 16 - 17)  # unflagged: age <= T_fail
        ok = vis | (hb == -1) | ((hb == -2) & (age <= 13))
        ch = ok.reshape(n, n // 8, 8).all(axis=2)
        print(f"r={r} cells ok {ok.mean():.6f} chunks ok {ch.mean():.6f} "
              f"lag max {int(lag[hb >= 0].max())} age max {int(age[hb >= 0].max())}", flush=True)
eng.close()
