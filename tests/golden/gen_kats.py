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


# ---- round 3: ring neighbours, JOIN broadcast, LEAVE lifetime, sole detector

def ring_kat(name, sender, lst, own_hb, fresh_col, fresh_hb, targets, n=8):
    """HeartBeat's ring (slave/slave.go:515-524): row `sender` holds `lst`
    (ID order = list order) and is the only active row; every other alive
    row holds 2 members (itself and `fresh_col`, stale hb 10), so it sits
    under the <4 guard (:504-509): it stamps ts = now and sends nothing, but
    still merges what it receives. The sender's snapshot carries `fresh_hb`
    in column `fresh_col`; exactly the 3 neighbours `targets` take it."""
    hb, ts, alive = blank(n)
    for j in range(n):
        alive[j] = 1
        if j == sender:
            continue
        hb[j][j], ts[j][j] = 5, 99
        hb[j][fresh_col], ts[j][fresh_col] = 10, 99
    hb[sender] = [A] * n
    for c in lst:
        hb[sender][c], ts[sender][c] = 5, 99
    if sender in lst:
        hb[sender][sender] = own_hb
    hb[sender][fresh_col] = fresh_hb - (1 if fresh_col == sender else 0)  # own hb++ first (:443-448)
    more = []
    for j in range(n):
        if j == sender:
            continue
        got = j in targets
        row_hb = [A] * n
        row_ts = [0] * n
        row_hb[j], row_ts[j] = 5, 100  # guard: ts = now, no hb++
        row_hb[fresh_col], row_ts[fresh_col] = (fresh_hb, 100) if got else (10, 100)
        if got:  # absent members of the snapshot are appended with ts = now (:430-439)
            for c in lst:
                if row_hb[c] == A:
                    row_hb[c], row_ts[c] = (fresh_hb if c == fresh_col else (own_hb + 1 if c == sender else 5)), 100
        more.append(dict(row=j, hb=row_hb, ts=row_ts))
    return dict(name=name, n=n, round=99, detect_mode=0, peer_mode=1, fanout=3, seed=1, t_fail=1000,
                t_cleanup=1000, hb=hb, ts=ts, alive=alive, events=[], expect_row=more[0]["row"],
                expect_hb=more[0]["hb"], expect_ts=more[0]["ts"], expect_more=more[1:], expect_failed=[],
                expect_detectors=[], expect_stats=dict(detections=0, active_rows=1))


# KAT-9 ring, self at index 0: list [0, 2, 4, 6], idx 0 -> list[(0-1) mod 4]
# = 6, list[1] = 2, list[2] = 4. Member 0's hb 50 -> 51 reaches rows 6, 2, 4
# only.
kats.append(ring_kat("kat9_ring_self_first", 0, [0, 2, 4, 6], 50, 0, 51, {6, 2, 4}))
# KAT-10 ring, self at the last slot: list [1, 2, 3, 5, 6], idx 4 ->
# list[3] = 5, list[5 mod 5] = 1, list[6 mod 5] = 2; row 3 is not a target.
kats.append(ring_kat("kat10_ring_self_last", 6, [1, 2, 3, 5, 6], 50, 6, 51, {5, 1, 2}))
# KAT-11 ring, self absent (removed from its own list): idx = -1 -> Go's
# (-2) % 5 = -2, fixed to 3 (:520-522): list[3] = 4, list[0] = 0, list[1] = 1.
# No own hb++; the sender's fresh view of member 7 (hb 40) reaches 4, 0, 1.
kats.append(ring_kat("kat11_ring_self_absent", 6, [0, 1, 3, 4, 7], None, 7, 40, {4, 0, 1}))

# KAT-12 JOIN broadcast (slave/slave.go:224-231, 250-272). Round 10: member 6
# (a fresh process, empty list) joins through introducer 0, whose list is
# [0(5), 1(5)]: 0 appends (6, hb 0, ts now) and sends its whole list to every
# member of it, itself and the joiner included. Row 1 [1(7)] appends 0 (5)
# and 6 (0); its own 7 > 5 stays. Row 2 [2(8), 0(5)] is not in 0's
# list: it gets nothing. Row 6 takes the whole list with ts = now. After the
# adds every row holds < 4 members, so the round itself only stamps ts = now
# (guard, :504-509): no hb++, nothing sent.
hb, ts, alive = blank(8)
hb[0][0], hb[0][1] = 5, 5
hb[1][1] = 7
hb[2][2], hb[2][0] = 8, 5
for j in (0, 1, 2):
    alive[j] = 1
    for c in range(8):
        if hb[j][c] != A:
            ts[j][c] = 9
kats.append(dict(
    name="kat12_join_broadcast", n=8, round=9, detect_mode=0, peer_mode=1, fanout=3, seed=1, t_fail=1000,
    t_cleanup=1000, hb=hb, ts=ts, alive=alive, events=[[1, 6]], expect_row=1,
    expect_hb=[5, 7, A, A, A, A, 0, A], expect_ts=[10, 10, 0, 0, 0, 0, 10, 0],
    expect_more=[dict(row=6, hb=[5, 5, A, A, A, A, 0, A], ts=[10, 10, 0, 0, 0, 0, 10, 0]),
                 dict(row=2, hb=[5, A, 8, A, A, A, A, A], ts=[10, 0, 10, 0, 0, 0, 0, 0]),
                 dict(row=0, hb=[5, 5, A, A, A, A, 0, A], ts=[10, 10, 0, 0, 0, 0, 10, 0])],
    expect_failed=[], expect_detectors=[], expect_stats=dict(detections=0, active_rows=0)))

# KAT-13 LEAVE tombstone lifetime (slave/slave.go:232-235, 276-286, 484-497).
# Members 0..4 fully connected and fresh (ts 19); member 4 leaves in round 20:
# every other alive row tombstones it with its last ts 19 (removeMember keeps
# the Member). cleanFailList drops it once ts < now - COOLDOWN (5): it lives
# through rounds 20..24 and is released in round 25. Nothing re-adds it (a
# tombstoned cell ignores merges; no snapshot lists it). T_fail = 1000.
hb, ts, alive = blank(5)
for j in range(5):
    alive[j] = 1
    for c in range(5):
        hb[j][c], ts[j][c] = 5, 19
for rounds, col4, t4, rel in ((5, T, 19, 0), (6, A, 0, 4)):
    kats.append(dict(
        name=f"kat13_leave_tombstone_{rounds}r", n=5, round=19, detect_mode=0, peer_mode=0, fanout=3, seed=3,
        t_fail=1000, t_cleanup=5, hb=hb, ts=ts, alive=alive, events=[[2, 4]], rounds=rounds, expect_row=0,
        expect_hb=[5 + rounds, None, None, None, col4], expect_ts=[19 + rounds, None, None, None, t4],
        expect_failed=[], expect_detectors=[], expect_stats=dict(tombstoned=4, released=rel, detections=0)))

# KAT-14 REMOVE sole-detector exception (slave/slave.go:338-363, 344-346):
# KAT-8's layout, but only row 1 holds member 3 stale (ts 10; rows 0 and 2
# hold it fresh, ts 19). Round 20: row 1 alone detects 3 and releases it at
# once. Round 21: REMOVE(3) reaches every alive row except its only detector
# (the detector does not message itself): rows 0 and 2 tombstone it (ts 19
# kept), row 4 never knew it (remove_unknown 1), row 1 gets nothing (KAT-8,
# with two detectors: remove_unknown 3).
hb, ts, alive = blank(8)
for i in (0, 1, 2, 4):
    alive[i] = 1
    for c in (i, 5, 6, 7):
        hb[i][c] = 5
        ts[i][c] = 19
hb[0][3], ts[0][3] = 6, 19
hb[1][3], ts[1][3] = 6, 10
hb[2][3], ts[2][3] = 6, 19
kats.append(dict(
    name="kat14_remove_sole_detector", n=8, round=19, detect_mode=0, peer_mode=0, fanout=3, seed=1, t_fail=5,
    t_cleanup=5, hb=hb, ts=ts, alive=alive, events=[], rounds=2, expect_row=1,
    expect_hb=[A, 7, A, A, A, 5, 5, 5], expect_ts=[0, 21, 0, 0, 0, 19, 19, 19],
    expect_more=[dict(row=2, hb=[A, A, 7, T, A, 5, 5, 5], ts=[0, 0, 21, 19, 0, 19, 19, 19]),
                 dict(row=0, hb=[7, A, A, T, A, 5, 5, 5], ts=[21, 0, 0, 19, 0, 19, 19, 19])],
    expect_failed=[], expect_detectors=[],
    expect_stats=dict(remove_unknown=1, tombstoned=2, detections=1, failed_members=1)))

# KAT-14L: KAT-14 with the reference's REMOVE recipients (GH_REMOVE_LIST,
# slave/slave.go:344, 472-473). Row 1's list is [1, 3, 5, 6, 7]; Remove(3)
# runs right after removeMember(3), so it messages 5, 6 and 7 (not itself,
# :344-346) - all crashed. Rows 0 and 2 are outside row 1's list: they keep
# member 3 (hb 6, ts 19: fresh, nobody gossips a higher count), row 4 gets no
# REMOVE of a member it never knew.
hb, ts, alive = blank(8)
for i in (0, 1, 2, 4):
    alive[i] = 1
    for c in (i, 5, 6, 7):
        hb[i][c] = 5
        ts[i][c] = 19
hb[0][3], ts[0][3] = 6, 19
hb[1][3], ts[1][3] = 6, 10
hb[2][3], ts[2][3] = 6, 19
kats.append(dict(
    name="kat14L_remove_outside_list", n=8, round=19, detect_mode=0, peer_mode=0, fanout=3, seed=1, t_fail=5,
    t_cleanup=5, remove_mode=1, hb=hb, ts=ts, alive=alive, events=[], rounds=2, expect_row=1,
    expect_hb=[A, 7, A, A, A, 5, 5, 5], expect_ts=[0, 21, 0, 0, 0, 19, 19, 19],
    expect_more=[dict(row=2, hb=[A, A, 7, 6, A, 5, 5, 5], ts=[0, 0, 21, 19, 0, 19, 19, 19]),
                 dict(row=0, hb=[7, A, A, 6, A, 5, 5, 5], ts=[21, 0, 0, 19, 0, 19, 19, 19])],
    expect_failed=[], expect_detectors=[],
    expect_stats=dict(remove_unknown=0, tombstoned=0, detections=1, failed_members=1)))

# KAT-15 a false positive's victim (slave/slave.go:338-363 with :443-448).
# Five alive members know each other (hb 5, ts 19); only row 1 holds member 2
# stale (ts 10). Round 20: row 1 alone detects 2 (and releases it at once);
# member 2 is alive and counts to 6. Round 21, the REMOVE(2) delivery:
#  * reference recipients (remove_mode 1): Remove(2) runs after
#    removeMember(2), so row 1 messages 0, 3 and 4 only. They tombstone 2;
#    the victim never hears of it and counts on: its own cell is 7 at 21.
#  * SPEC D4 (remove_mode 0): every alive row but the sole detector, the
#    victim included: row 2 tombstones itself (ts 20 kept) and stops counting.
# Rows 0, 3 and 4 hold member 2 as a tombstone either way (its ts depends on
# the round-20 merges, not checked).
hb, ts, alive = blank(5)
for i in range(5):
    alive[i] = 1
    for c in range(5):
        hb[i][c], ts[i][c] = 5, 19
ts[1][2] = 10
for mode, own, own_ts, tomb in ((1, 7, 21, 3), (0, T, 20, 4)):
    kats.append(dict(
        name=f"kat15_victim_{'list' if mode else 'all'}", n=5, round=19, detect_mode=0, peer_mode=0, fanout=3,
        seed=5, t_fail=5, t_cleanup=5, remove_mode=mode, hb=hb, ts=ts, alive=alive, events=[], rounds=2,
        expect_row=2, expect_hb=[None, None, own, None, None], expect_ts=[None, None, own_ts, None, None],
        expect_tomb=[[0, 2], [3, 2], [4, 2]],
        expect_failed=[], expect_detectors=[],
        expect_stats=dict(tombstoned=tomb, detections=1, failed_members=1, remove_unknown=0)))


# KAT-16 a JOIN of a member the introducer holds tombstoned (SPEC D7,
# slave/slave.go:224-231, 250-255, 276-286, 484-497). Members 0..5 know each
# other (hb 5, ts 19); T_fail = 1000, COOLDOWN 5; introducer 0.
#  * Round 20: 4 LEAVEs: rows 0, 1, 2, 3, 5 tombstone it with its last ts 19
#    (tombstoned 5).
#  * Round 22: 4 JOINs (a fresh process). At 0, MemberInList reads MemberList
#    only, so addNewMember appends (4, hb 0, ts 22) while RecentFailList keeps
#    (4, ts 19). The broadcast reaches 1, 2, 3, 5, whose tombstones block the
#    re-add (:430-433), and the fresh row 4.
#  * Round 23 (the "leave" cases): 4 LEAVEs again. At 0, removeMember finds 4
#    in RecentFailList, appends nothing (tombstoned stays 5) and drops it from
#    MemberList: 0's tombstone of 4 is the old entry, ts 19. Rows 1, 2, 3, 5
#    hold only the tombstone: a no-op (not a panic, :278-281).
#  * cleanFailList releases every ts-19 entry in round 25 (19 < 25 - 5): after
#    rounds 20..24 row 0 still holds the tombstone (ts 19, not the 22 of its
#    present entry); after round 25 it is gone, with rows 1, 2, 3, 5's
#    (released 5).
#  * The "stay" case (no second LEAVE): round 25 releases 0's RecentFailList
#    entry too, while 4 stays in its MemberList (released 5: four tombstones
#    and the shadow entry).
hb, ts, alive = blank(6)
for j in range(6):
    alive[j] = 1
    for c in range(6):
        hb[j][c], ts[j][c] = 5, 19
for name, sched, rounds, col4, t4, rel in (
        ("kat16_d7_rejoin_leave_5r", {"20": [[2, 4]], "22": [[1, 4]], "23": [[2, 4]]}, 5, T, 19, 0),
        ("kat16_d7_rejoin_leave_6r", {"20": [[2, 4]], "22": [[1, 4]], "23": [[2, 4]]}, 6, A, 0, 5),
        ("kat16_d7_rejoin_stay_6r", {"20": [[2, 4]], "22": [[1, 4]]}, 6, None, None, 5)):
    kats.append(dict(
        name=name, n=6, round=19, detect_mode=0, peer_mode=0, fanout=3, seed=7, t_fail=1000, t_cleanup=5,
        hb=hb, ts=ts, alive=alive, events=[], sched=sched, rounds=rounds, expect_row=0,
        expect_hb=[None, None, None, None, col4, None], expect_ts=[None, None, None, None, t4, None],
        expect_more=[dict(row=j, hb=[None] * 4 + [T if rounds == 5 else A, None], ts=[None] * 4 + [19, None])
                     for j in (1, 2, 3, 5)] if "leave" in name else [],
        expect_failed=[], expect_detectors=[], expect_stats=dict(tombstoned=5, released=rel, detections=0,
                                                                remove_unknown=0)))


def row_matches(name, hb, ts, i, exp_hb, exp_ts):
    """hb of row i equals exp_hb (None = any), ts where present"""
    for c, v in enumerate(exp_hb):
        if v is None:
            continue
        assert hb[i][c] == v, (name, i, c, list(hb[i]))
        if v != A:
            assert ts[i][c] == exp_ts[c], (name, i, c, list(ts[i]))


def check_with_listsim(k):
    import oracle.listsim as L
    L.T_FAIL, L.T_CLEANUP = k["t_fail"], k["t_cleanup"]
    sim = ListSim.from_dense(k["hb"], k["ts"], k["alive"], k["round"], seed=k["seed"],
                             peer_mode="ring" if k["peer_mode"] else "pull", fanout=k["fanout"],
                             quirk=bool(k["detect_mode"]), remove="list" if k.get("remove_mode") else "all")
    if k["events"]:
        sim.apply_events([tuple(e) for e in k["events"]])
    sys.path.insert(0, str(HERE.parent))
    from kat_util import run_rounds
    st = run_rounds(sim, k)
    hb, ts, _ = sim.dense()
    if k["expect_hb"] is not None:
        row_matches(k["name"], hb, ts, k["expect_row"], k["expect_hb"], k["expect_ts"])
    for m in k.get("expect_more", []):
        row_matches(k["name"], hb, ts, m["row"], m["hb"], m["ts"])
    for i, c in k.get("expect_tomb", []):
        assert hb[i][c] == T, (k["name"], i, c, list(hb[i]))
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
