"""Writes tests/golden/kats.json: the hand-derived known-answer tests of
SURVEY.md Appendix B, embedded in whole-round scenarios so that every engine
(listsim, tablesim, libgossiphip) can run them through its public API.

Each expected value below is derived by hand from the reference source (the
comment names the line); the script only lays the inputs out as dense tables
and checks them against the literal list replay (oracle/listsim.py) before
writing. Run: python tests/golden/gen_kats.py
"""
import json
import pathlib
import sys

HERE = pathlib.Path(__file__).resolve().parent
sys.path.insert(0, str(HERE.parents[1]))

from oracle import philox  # noqa: E402
from oracle.listsim import ListSim  # noqa: E402

A, T = -1, -2  # absent, tombstone


def blank(n):
    return [[A] * n for _ in range(n)], [[0] * n for _ in range(n)], [0] * n


kats = []

# KAT-2 detect (slave/slave.go:460-477). now=1000, PERIOD=5 -> stale <=> ts<995.
# Row 0 = S (self), list [S, A(2,990), B(3,994), C(1,0), D(4,999), E(5,900),
# F(6,901), G(2,100)]; every other row crashed, so no gossip reaches row 0.
# Candidates {A,B,E,F,G} (C: hb<=1; D: fresh). Quirk: runs [A,B],[E,F,G] ->
# A, E, G detected (Go range over the shifted slice). Canonical: all five.
# Step 5 releases each new tombstone at once (ts < 995 = now-COOLDOWN).
hb, ts, alive = blank(8)
hb[0] = [10, 2, 3, 1, 4, 5, 6, 2]
ts[0] = [999, 990, 994, 0, 999, 900, 901, 100]
alive[0] = 1
for quirk, det, row in (
    (True, [1, 5, 7], [11, A, 3, 1, 4, A, 6, A]),
    (False, [1, 2, 5, 6, 7], [11, A, A, 1, 4, A, A, A]),
):
    kats.append(dict(
        name=f"kat2_detect_{'quirk' if quirk else 'canonical'}", n=8, round=999, detect_mode=int(quirk),
        peer_mode=0, fanout=3, seed=1, t_fail=5, t_cleanup=5,
        hb=hb, ts=ts, alive=alive, events=[],
        expect_row=0, expect_hb=row,
        expect_ts=[1000, 990, 994, 0, 999, 900, 901, 100],  # own ts=now (:445); others kept
        expect_failed=det, expect_detectors=[0], expect_stats=dict(detections=len(det), released=len(det))))

# KAT-3 clean (slave/slave.go:484-497). now=1000, COOLDOWN=5: tombstones with
# ts {994, 995, 996} -> only 994 released (strict <). Row 0 has 4 fresh
# members so it is active and detects nothing.
hb, ts, alive = blank(8)
hb[0] = [7, 3, 3, 3, A, T, T, T]
ts[0] = [999, 999, 998, 997, 0, 994, 995, 996]
alive[0] = 1
kats.append(dict(
    name="kat3_clean", n=8, round=999, detect_mode=0, peer_mode=0, fanout=3, seed=1, t_fail=5, t_cleanup=5,
    hb=hb, ts=ts, alive=alive, events=[], expect_row=0,
    expect_hb=[8, 3, 3, 3, A, A, T, T], expect_ts=[1000, 999, 998, 997, 0, 994, 995, 996],
    expect_failed=[], expect_detectors=[], expect_stats=dict(detections=0, released=1)))

# KAT-4 guard (slave/slave.go:504-509). Row 0 holds 3 members at now=7: every
# ts becomes 7, hb unchanged (no hb++), no detection although entry 1 is stale.
hb, ts, alive = blank(6)
hb[0] = [5, 3, 2, A, A, A]
ts[0] = [1, 0, 3, 0, 0, 0]
alive[0] = 1
kats.append(dict(
    name="kat4_guard", n=6, round=6, detect_mode=0, peer_mode=0, fanout=3, seed=1, t_fail=5, t_cleanup=5,
    hb=hb, ts=ts, alive=alive, events=[], expect_row=0,
    expect_hb=[5, 3, 2, A, A, A], expect_ts=[7, 7, 7, 0, 0, 0],
    expect_failed=[], expect_detectors=[], expect_stats=dict(detections=0, active_rows=0)))

# KAT-1 merge (slave/slave.go:414-440), end to end. now=200. Receiver row 0
# holds [0(self,50,199), A=1(5,100), B=2(3,90), C=3(7,95)], tombstone D=4.
# Sender row 6 holds [0:40, A:4, B:4, C:7, D:9, E=5:2, 6(self):60]; members
# 1..5 crashed. T_fail/T_cleanup = 1000 so nothing is detected or released.
# Row 0's pull peers (k=8, Philox) must include 6 for this seed (checked).
# Merge: A remote 4<5 kept (ts 100); B 3<4 -> (4,200); C equal -> ts 95 kept;
# D tombstoned -> ignored; E absent -> added (2,200); 6 absent -> added with
# the sender's post-heartbeat hb 61 (:443-446), ts 200; self 0: own hb++ ->
# 51, remote 40 lower.
hb, ts, alive = blank(7)
hb[0] = [50, 5, 3, 7, T, A, A]
ts[0] = [199, 100, 90, 95, 80, 0, 0]
hb[6] = [40, 4, 4, 7, 9, 2, 60]
ts[6] = [199] * 7
alive[0] = alive[6] = 1
seed = None
for cand in range(1, 200):
    if 6 in [philox.peer(cand, 0, 200, t, 7) for t in range(8)]:
        seed = cand
        break
assert seed is not None
kats.append(dict(
    name="kat1_merge", n=7, round=199, detect_mode=0, peer_mode=0, fanout=8, seed=seed, t_fail=1000,
    t_cleanup=1000, hb=hb, ts=ts, alive=alive, events=[], expect_row=0,
    expect_hb=[51, 5, 4, 7, T, 2, 61], expect_ts=[200, 100, 200, 95, 80, 200, 200],
    expect_failed=[], expect_detectors=[], expect_stats=dict(detections=0)))

# KAT-8 REMOVE / unknown-member (slave/slave.go:236-240, 276-286), two rounds.
# Members 5, 6, 7 are crashed but fresh (ts 19), so alive rows stay active
# without listing each other: no alive row is in another's list, so nothing is
# gossiped (a sender only sends to its list). Lists: row 0 [0, 3(fresh), 5, 6,
# 7]; rows 1, 2 [i, 3(stale), 5, 6, 7]; row 4 [4, 5, 6, 7].
# Round 20: rows 1 and 2 detect 3 (ts 10, 12 < 15) and release it at once.
# Round 21: two detectors, so every alive row gets REMOVE(3): row 0 tombstones
# it (tombstoned=1, ts 19 kept); rows 1, 2 (released) and 4 (never knew it)
# would panic in the reference -> remove_unknown = 3.
hb, ts, alive = blank(8)
for i in (0, 1, 2, 4):
    alive[i] = 1
    for c in (i, 5, 6, 7):
        hb[i][c] = 5
        ts[i][c] = 19
hb[0][3], ts[0][3] = 6, 19
hb[1][3], ts[1][3] = 6, 10
hb[2][3], ts[2][3] = 6, 12
kats.append(dict(
    name="kat8_remove_unknown", n=8, round=19, detect_mode=0, peer_mode=0, fanout=3, seed=1, t_fail=5,
    t_cleanup=5, hb=hb, ts=ts, alive=alive, events=[], rounds=2, expect_row=0,
    expect_hb=[7, A, A, T, A, 5, 5, 5], expect_ts=[21, 0, 0, 19, 0, 19, 19, 19],
    expect_failed=[], expect_detectors=[],
    expect_stats=dict(remove_unknown=3, tombstoned=1, detections=2, failed_members=1)))


def check_with_listsim(k):
    import oracle.listsim as L
    L.T_FAIL, L.T_CLEANUP = k["t_fail"], k["t_cleanup"]
    sim = ListSim.from_dense(k["hb"], k["ts"], k["alive"], k["round"], seed=k["seed"],
                             peer_mode="ring" if k["peer_mode"] else "pull", fanout=k["fanout"],
                             quirk=bool(k["detect_mode"]))
    st = sim.step(k.get("rounds", 1))
    hb, ts, _ = sim.dense()
    i = k["expect_row"]
    if k["expect_hb"] is not None:
        assert list(hb[i]) == k["expect_hb"], (k["name"], list(hb[i]))
        for c, v in enumerate(k["expect_hb"]):
            if v != A:
                assert ts[i][c] == k["expect_ts"][c], (k["name"], c, list(ts[i]))
    for key, v in k["expect_stats"].items():
        assert st[key] == v, (k["name"], key, st[key], v)
    if k.get("rounds", 1) == 1:
        assert sim.last_failed == k["expect_failed"], (k["name"], sim.last_failed)
        assert sim.last_detectors == k["expect_detectors"]
    L.T_FAIL, L.T_CLEANUP = 5, 5


for k in kats:
    check_with_listsim(k)


(HERE / "kats.json").write_text(json.dumps(kats, indent=1))
print(f"wrote {len(kats)} KATs")
