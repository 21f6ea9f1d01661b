"""8-bit tier diagnostics: runs one scenario with the tier (GH_C8 unset) and
without it (GH_C8=0), prints per round the kernel variant, the tier of the
current table and escaped chunks, and at the first round whose tables differ
the differing cells of both (python tools/tier_diag.py)."""
import os
import pathlib
import sys

import numpy as np

REPO = pathlib.Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO), str(REPO / "tests"), str(REPO / "p2p-file-system-with-gossip-detect-failure-management_amd")]
os.environ["GH_PLANE"] = "1"

import gossipsim as gs  # noqa: E402
import scenarios as sc  # noqa: E402

n = 2048
cfg = dict(fanout=4, seed=0x5EED0007, t_fail=16, t_cleanup=16)
sched = {14: [(sc.CRASH, 7), (sc.LEAVE, 1500)], 18: [(sc.JOIN, 1500), (sc.JOIN, 7)]}
rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 34


def run(c8):
    if c8:
        os.environ.pop("GH_C8", None)
    else:
        os.environ["GH_C8"] = "0"
    eng = gs.Engine(gs.default_config(n, **cfg))
    eng.import_state(*sc.full_state(n), 0)
    out = []
    for r in range(1, rounds + 1):
        if r in sched:
            eng.apply_events(sched[r])
        st = eng.step(1)
        out.append((st, eng.export_state(), eng.encoding_info(full=True), eng.tier_info()))
    eng.close()
    return out


a, b = run(True), run(False)
for r, (x, y) in enumerate(zip(a, b), 1):
    same = x[0] == y[0] and all(np.array_equal(p, q) for p, q in zip(x[1], y[1]))
    print(r, "same" if same else "DIFF", "enc", x[2], "tier", x[3], "| 16-bit enc", y[2], flush=True)
    if not same:
        print("  stats", x[0], y[0])
        for name, p, q in zip(("hb", "ts"), x[1][:2], y[1][:2]):
            bad = np.argwhere(p != q)
            print(f"  {name}: {len(bad)} cells differ; rows {np.unique(bad[:, 0])[:20].tolist()} "
                  f"cols {np.unique(bad[:, 1])[:20].tolist()}")
            for i, c in bad[:12].tolist():
                print(f"    ({i},{c}) tier hb={x[1][0][i, c]} ts={x[1][1][i, c]}  16-bit hb={y[1][0][i, c]} "
                      f"ts={y[1][1][i, c]}")
        break
