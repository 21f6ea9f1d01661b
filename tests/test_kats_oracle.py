"""App. B known-answer tests on the C oracle (tablesim) and the placement
KATs (KAT-5/6) on both CPU restatements."""
import numpy as np
import pytest

from oracle import philox
from oracle.listsim import ListSim

from kat_util import KATS, kat_config, run_kat


@pytest.mark.parametrize("k", KATS, ids=[k["name"] for k in KATS])
def test_kat_tablesim(oracle_mod, k):
    run_kat(oracle_mod.Oracle(kat_config(oracle_mod, k)), k)


def _master_with(om, n, present, files=64, seed=0x5EED0001, replicas=4):
    """Master row 0 holding `present` (others absent); everyone else crashed."""
    cfg = om.default_config(n, max_files=files, seed=seed, replicas=replicas)
    o = om.Oracle(cfg)
    hb = np.full((n, n), -1, np.int32)
    ts = np.zeros((n, n), np.int32)
    alive = np.zeros(n, np.uint8)
    hb[0, present] = 3
    alive[0] = 1
    o.import_state(hb, ts, alive, 20)
    ls = ListSim.from_dense(hb, ts, alive, 20, seed=seed, replicas=replicas)
    return o, ls


def test_kat5_last_candidate_never_drawn(oracle_mod):
    """master/master.go:135: Intn(len-1) never returns the last index."""
    o, ls = _master_with(oracle_mod, 12, list(range(10)), files=400)
    rep, ver, st = o.put(np.arange(400))
    assert (st == 0).all() and (ver == 1).all()
    assert 9 not in rep  # m9 = last of Member_list [m0..m9]
    assert set(np.unique(rep)) == set(range(9))
    for f in range(400):
        assert len(set(rep[f])) == 4
        nodes, v, s = ls.put(f)
        assert nodes == list(rep[f]) and v == 1 and s == 0


def test_kat5_draw_order_and_existing_kept(oracle_mod):
    """Existing replicas stay first; draws fill in draw order (:130-141)."""
    o, ls = _master_with(oracle_mod, 10, list(range(10)), files=8)
    seed = 0x5EED0001
    cand = list(range(10))
    # hand replay of the draw loop for file 3
    nodes, d = [], 0
    while len(nodes) < 4:
        a = cand[philox.place_index(seed, 3, d, 10)]
        d += 1
        if a not in nodes:
            nodes.append(a)
    rep, ver, st = o.put([3])
    assert list(rep[0]) == nodes and ver[0] == 1
    # a second put keeps the list and bumps the version (:152-160)
    rep2, ver2, _ = o.put([3])
    assert list(rep2[0]) == nodes and ver2[0] == 2
    # delete then get -> absent (-1) (:177-185, :249-259)
    old = o.delete_files([3])
    assert list(old[0]) == nodes
    r3, v3 = o.get_files([3])
    assert v3[0] == -1 and (r3 == -1).all()


def test_kat5_starvation(oracle_mod):
    """M=4 candidates: only 3 choosable -> reference loops forever (:130)."""
    o, ls = _master_with(oracle_mod, 8, [0, 1, 2, 3], files=4)
    rep, ver, st = o.put([0])
    assert st[0] == oracle_mod.GH_EPLACEMENT_STARVED and ver[0] == 0
    assert ls.put(0)[2] == -5
    o2, _ = _master_with(oracle_mod, 8, [0], files=4)  # M=1: Intn(0) panics
    assert o2.put([1])[2][0] == oracle_mod.GH_EPLACEMENT_STARVED


def test_kat6_rereplication(oracle_mod):
    """master/master.go:93-123: replicas [a,b,c,d], b unavailable ->
    working [a,c,d], Node_list [a,c,d,x], plan {a, v, [x]}."""
    n = 12
    o, ls = _master_with(oracle_mod, n, list(range(10)), files=4)
    rep, ver, _ = o.put([1])
    ls.put(1)
    a, b, c, d = rep[0]
    # observer row 5 knows everything except b
    hb, ts, alive = o.export_state()
    hb[5, :10] = 3
    hb[5, b] = -1
    alive[5] = 1
    o.import_state(hb, ts, alive, 20)
    ls2 = ListSim.from_dense(hb, ts, alive, 20, seed=0x5EED0001)
    ls2.files, ls2.draws = ls.files, ls.draws
    plan = o.repair(5)
    assert len(plan) == 1
    f, node1, v, status, new = plan[0]
    assert (f, node1, v, status) == (1, a, 1, 0) and len(new) == 1 and new[0] not in (a, c, d)
    rep2, _ = o.get_files([1])
    assert list(rep2[0]) == [a, c, d, new[0]]
    assert ls2.repair(5) == plan
    # everything available now -> empty plan
    assert o.repair(0) == [] or all(p[4] == () for p in o.repair(0))
