"""GPU parity of GH_ORDER_APPEND (SPEC.md §7 D1) against oracle/listsim.py's
literal Go-slice replay in append order (slave/slave.go:255, 437 append;
:283 removal closes the gap): every round the counters, the dense hb/ts
tables, the failed set, the detectors AND every row's list order (gh_lsm)
must match, in ring and pull mode, canonical and quirk detection, under
crash / leave / join churn with re-adds. Placement candidates, MemberList[0]
and external datagrams follow the same order. Run on a MI355X: pytest -m gpu."""
import numpy as np
import pytest

import scenarios as sc
from oracle import listsim as L
from oracle.listsim import ListSim, Member

pytestmark = pytest.mark.gpu

APPEND = 1  # GH_ORDER_APPEND


@pytest.fixture(scope="module")
def gs():
    import gossipsim
    return gossipsim


def make_pair(gs, n, peer_mode, quirk, fanout=3, seed=0x5EED0001, init_full=False, max_files=0, **kw):
    cfg = gs.default_config(n, peer_mode=gs.GH_PEER_RING if peer_mode == "ring" else gs.GH_PEER_PULL,
                            fanout=fanout, detect_mode=int(quirk), seed=seed, list_order=APPEND,
                            max_files=max_files, **kw)
    eng = gs.Engine(cfg)
    if init_full:
        hb, ts, alive = sc.full_state(n)
        eng.import_state(hb, ts, alive, 0)
        ls = ListSim.from_dense(hb, ts, alive, 0, seed=seed, peer_mode=peer_mode, fanout=fanout, quirk=quirk,
                                order="append")
    else:
        ls = ListSim(n, seed=seed, peer_mode=peer_mode, fanout=fanout, quirk=quirk, order="append")
    return eng, ls


def lists_gpu(eng, n):
    return [list(eng.lsm(i)[0]) for i in range(n)]


def lists_ref(ls):
    return [[m.addr for m in nd.members] for nd in ls.nodes]


def compare(eng, ls, n, r):
    from test_gpu_parity import check_counts
    check_counts(eng, r)
    h1, t1, a1 = eng.export_state()
    h2, t2, a2 = ls.dense()
    np.testing.assert_array_equal(a1, a2, err_msg=f"alive r={r}")
    np.testing.assert_array_equal(h1, h2, err_msg=f"hb r={r}")
    np.testing.assert_array_equal(t1, sc.export_view(h2, t2, r, L.T_CLEANUP)[1], err_msg=f"ts r={r}")
    g, w = lists_gpu(eng, n), lists_ref(ls)
    bad = [i for i in range(n) if g[i] != w[i]]
    assert not bad, f"r={r}: list order of rows {bad[:4]}: gpu {g[bad[0]]} ref {w[bad[0]]}"


def run_pair(eng, ls, n, rounds, sched):
    reordered = 0
    for r in range(1, rounds + 1):
        ev = sched.get(r, [])
        if ev:
            eng.apply_events(ev)
            ls.apply_events(ev)
        s1, s2 = eng.step(1), ls.step(1)
        assert s1 == s2, f"round {r}: gpu {s1} != ref {s2}"
        bm = eng.read_failed()
        assert [c for c in range(n) if bm[c >> 5] >> (c & 31) & 1] == ls.last_failed, r
        assert sorted(eng.read_detectors()) == sorted(ls.last_detectors), r
        compare(eng, ls, n, ls.round)
        reordered = max(reordered, sum(1 for x in lists_ref(ls) if x != sorted(x)))
    return reordered


@pytest.mark.parametrize("seed", [1, 2, 3])
@pytest.mark.parametrize("peer_mode,quirk", [("ring", False), ("ring", True), ("pull", True), ("pull", False)])
def test_append_churn_matches_listsim(gs, peer_mode, quirk, seed):
    """Seeded churn with re-adds (released tombstones come back at the end of
    the list): the orders the ID-order engine misses (tests/test_list_order.py)."""
    n = 24
    sched = sc.random_churn(n, 80, seed, p_crash=0.03, p_leave=0.02, p_join=0.08)
    eng, ls = make_pair(gs, n, peer_mode, quirk, init_full=True)
    try:
        reordered = run_pair(eng, ls, n, 80, sched)
    finally:
        eng.close()
    assert reordered > 0  # the lists did leave ID order


@pytest.mark.parametrize("peer_mode", ["ring", "pull"])
@pytest.mark.parametrize("quirk", [False, True], ids=["canonical", "quirk"])
def test_append_c1_bootstrap(gs, peer_mode, quirk):
    """BASELINE config 1: 10 members join one per round through the
    introducer (its broadcast appends in its list order), 7 crashes at r=30."""
    n = 10
    sched = {r: [(sc.JOIN, r - 1)] for r in range(1, 11)}
    sched.setdefault(30, []).append((sc.CRASH, 7))
    eng, ls = make_pair(gs, n, peer_mode, quirk)
    try:
        run_pair(eng, ls, n, 60, sched)
    finally:
        eng.close()


@pytest.mark.parametrize("seed", [11, 12])
def test_append_heavy_churn_ring_quirk(gs, seed):
    n = 36
    sched = sc.random_churn(n, 60, seed, p_crash=0.06, p_leave=0.03, p_join=0.12)
    eng, ls = make_pair(gs, n, "ring", True, init_full=True, seed=0x7000 + seed)
    try:
        run_pair(eng, ls, n, 60, sched)
    finally:
        eng.close()


def test_append_short_timeouts(gs):
    """T_fail / T_cleanup off the defaults: tombstones outlive detection, so a
    member can be removed, kept out, and re-added rounds later."""
    n = 20
    sched = sc.random_churn(n, 60, 21, p_crash=0.05, p_leave=0.02, p_join=0.1)
    eng, ls = make_pair(gs, n, "ring", False, init_full=True, t_fail=3, t_cleanup=7)
    L.T_FAIL, L.T_CLEANUP = 3, 7
    try:
        run_pair(eng, ls, n, 60, sched)
    finally:
        L.T_FAIL, L.T_CLEANUP = 5, 5
        eng.close()


def test_append_placement_and_first_member(gs):
    """Member_list = the master's list in list order (master/master.go:46):
    put draws index it (:135); repair refills from it; MemberList[0]
    (slave/slave.go:936) is the list's head."""
    n = 24
    sched = sc.random_churn(n, 50, 2, p_crash=0.03, p_leave=0.02, p_join=0.08)
    eng, ls = make_pair(gs, n, "ring", False, init_full=True, max_files=64)
    try:
        run_pair(eng, ls, n, 50, sched)
        assert lists_ref(ls)[0] != sorted(lists_ref(ls)[0])  # the master's list is out of ID order
        files = list(range(40))
        rep, ver, st = eng.put(np.array(files, np.int32))
        for k, f in enumerate(files):
            nodes, v, s = ls.put(f)
            assert st[k] == s and ver[k] == v, f
            assert [x for x in rep[k] if x >= 0] == nodes, f
        first, ln, _ = eng.vote_scan(np.zeros(n, np.int32))
        want = [nd.members[0].addr if nd.members else -1 for nd in ls.nodes]
        assert list(first) == want
        assert list(ln) == [len(nd.members) for nd in ls.nodes]
        # crash two replicas' worth of members, detect, then repair from row 0
        ev = [(sc.CRASH, c) for c in [c for c in lists_ref(ls)[0] if c != 0][:2]]
        eng.apply_events(ev)
        ls.apply_events(ev)
        run_pair(eng, ls, n, 8, {})
        assert eng.repair(0) == ls.repair(0)
    finally:
        eng.close()


def test_append_merge_list_datagram_order(gs):
    """MergeMemberList (slave/slave.go:433-437) appends the members it lacks
    in the received list's order."""
    n = 40
    eng, ls = make_pair(gs, n, "ring", False)
    try:
        ev = [(sc.JOIN, c) for c in (0, 5, 9)]
        eng.apply_events(ev)
        ls.apply_events(ev)
        run_pair(eng, ls, n, 1, {})
        rng = np.random.default_rng(5)
        for obs in (5, 9, 0):
            ids = rng.permutation(n)[:17].astype(np.int32)
            hb = rng.integers(0, 50, len(ids)).astype(np.int32)
            eng.merge_list(obs, ids, hb)
            ls.nodes[obs].merge([Member(int(a), int(b), 0) for a, b in zip(ids, hb)], ls.round)
            assert list(eng.lsm(obs)[0]) == [m.addr for m in ls.nodes[obs].members], obs
        run_pair(eng, ls, n, 6, {})
    finally:
        eng.close()


def test_append_refused_on_column_shards(gs):
    """A row's order spans every column: column shards refuse it."""
    with pytest.raises(gs.GossipError):
        gs.ShardGroup(gs.default_config(64, list_order=APPEND), 2)


def make_rows_pair(gs, n, world, peer_mode, quirk, fanout=3, seed=0x5EED0001, init_full=False, max_files=0, **kw):
    """GH_ORDER_APPEND on G row shards (every shard keeps a replica of every
    list, the owners' changes are copied each round) against listsim."""
    cfg = gs.default_config(n, peer_mode=gs.GH_PEER_RING if peer_mode == "ring" else gs.GH_PEER_PULL,
                            fanout=fanout, detect_mode=int(quirk), seed=seed, list_order=APPEND,
                            max_files=max_files, shard_layout=gs.GH_LAYOUT_ROWS, **kw)
    eng = gs.ShardGroup(cfg, world)
    if init_full:
        hb, ts, alive = sc.full_state(n)
        eng.import_state(hb, ts, alive, 0)
        ls = ListSim.from_dense(hb, ts, alive, 0, seed=seed, peer_mode=peer_mode, fanout=fanout, quirk=quirk,
                                order="append")
    else:
        ls = ListSim(n, seed=seed, peer_mode=peer_mode, fanout=fanout, quirk=quirk, order="append")
    return eng, ls


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("peer_mode,quirk", [("ring", False), ("ring", True), ("pull", False), ("pull", True)])
def test_append_row_shards_churn(gs, world, peer_mode, quirk):
    """The reference topology on row shards (ring + append order, the
    Cluster default; slave/slave.go:255, 437, 515-524): seeded churn with
    re-adds, every round's counters, tables, failed set, detectors and every
    row's list order equal listsim's."""
    n = 24
    sched = sc.random_churn(n, 60, 40 + world, p_crash=0.03, p_leave=0.02, p_join=0.08)
    eng, ls = make_rows_pair(gs, n, world, peer_mode, quirk, init_full=True, seed=0x7100 + world)
    try:
        reordered = run_pair(eng, ls, n, 60, sched)
    finally:
        eng.close()
    assert reordered > 0


@pytest.mark.parametrize("world", [2, 4])
def test_append_row_shards_bootstrap_placement(gs, world):
    """BASELINE config 1 on row shards in append order: 10 members join one
    per round through the introducer (its broadcast appends in its list
    order, shipped to every shard), 7 crashes at r=30; then placement from
    the master's list order, MemberList[0] of every row and a datagram
    merge."""
    n = 10
    sched = {r: [(sc.JOIN, r - 1)] for r in range(1, 11)}
    sched.setdefault(30, []).append((sc.CRASH, 7))
    eng, ls = make_rows_pair(gs, n, world, "ring", False, max_files=32)
    try:
        run_pair(eng, ls, n, 40, sched)
        files = list(range(12))
        rep, ver, st = eng.put(np.array(files, np.int32))
        for k, f in enumerate(files):
            nodes, v, s_ = ls.put(f)
            assert st[k] == s_ and ver[k] == v, f
            assert [x for x in rep[k] if x >= 0] == nodes, f
        first, ln, _ = eng.vote_scan(np.zeros(n, np.int32))
        assert list(first) == [nd.members[0].addr if nd.members else -1 for nd in ls.nodes]
        ids = np.array([9, 7, 3], np.int32)
        hb = np.array([99, 98, 97], np.int32)
        eng.merge_list(4, ids, hb)
        ls.nodes[4].merge([Member(int(a), int(b), 0) for a, b in zip(ids, hb)], ls.round)
        assert list(eng.lsm(4)[0]) == [m.addr for m in ls.nodes[4].members]
        run_pair(eng, ls, n, 6, {})
    finally:
        eng.close()


def test_id_order_unchanged_lsm(gs):
    """GH_ORDER_ID keeps member-ID order in lsm."""
    eng = gs.Engine(gs.default_config(32, fanout=3, seed=0x99))
    try:
        eng.init_full()
        eng.step(3)
        ids = list(eng.lsm(4)[0])
        assert ids == sorted(ids)
    finally:
        eng.close()


def test_append_at_scale_matches_id_order(gs):
    """Pull mode with canonical detection is order-free (tests/test_list_order.py):
    at N=20,000 (sender plane, 256-member tiles) with a crash wave, a join
    batch and leaves, the append-order engine gives the ID-order engine's
    tables and counters every round, and every list holds exactly its row's
    present members."""
    n = 20000
    cfg = dict(fanout=4, seed=0x5EED0900, t_fail=8, t_cleanup=8)
    sched = {3: [(sc.CRASH, c) for c in sc.crash_ids(n, 0.01, 0x5EED0901)],
             14: [(sc.LEAVE, 17), (sc.LEAVE, 4000)],
             16: [(sc.JOIN, c) for c in sc.crash_ids(n, 0.01, 0x5EED0901)[:40]]}
    a = gs.Engine(gs.default_config(n, list_order=APPEND, **cfg))
    b = gs.Engine(gs.default_config(n, **cfg))
    try:
        for e in (a, b):
            e.init_full()
        for r in range(1, 25):
            for e in (a, b):
                if r in sched:
                    e.apply_events(sched[r])
            assert a.step(1) == b.step(1), r
            if r % 6 == 0 or r in (4, 15, 17):
                ha, ta, _ = a.export_state(0, 64)
                hb, tb, _ = b.export_state(0, 64)
                np.testing.assert_array_equal(ha, hb)
                np.testing.assert_array_equal(ta, tb)
                for i in (0, 17, 33, 63):
                    ids = a.lsm(i)[0]
                    assert sorted(ids) == list(np.flatnonzero(ha[i] >= 0)), (r, i)
        assert a.plane_info()[0] == 1
    finally:
        a.close()
        b.close()
