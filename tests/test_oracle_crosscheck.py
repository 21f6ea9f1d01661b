"""Cross-check the two independent CPU restatements of the reference:
oracle/listsim.py (literal Go list semantics) and oracle/tablesim.c (dense
tables), round by round on seeded churn scenarios (SPEC.md)."""
import numpy as np
import pytest

from oracle.listsim import ListSim

import scenarios as sc


def run_pair(om, n, rounds, sched, peer_mode, fanout=3, quirk=False, seed=0x5EED0001,
             init_full=False, t_fail=5, t_cleanup=5, remove="all", per_round=None):
    cfg = om.default_config(n, peer_mode=om.GH_PEER_RING if peer_mode == "ring" else om.GH_PEER_PULL,
                            fanout=fanout, detect_mode=int(quirk), seed=seed, t_fail=t_fail,
                            t_cleanup=t_cleanup,
                            remove_mode=om.GH_REMOVE_LIST if remove == "list" else om.GH_REMOVE_ALL)
    orc = om.Oracle(cfg)
    if init_full:
        hb, ts, alive = sc.full_state(n)
        orc.import_state(hb, ts, alive, 0)
        ls = ListSim.from_dense(hb, ts, alive, 0, seed=seed, peer_mode=peer_mode, fanout=fanout,
                                quirk=quirk, remove=remove)
    else:
        ls = ListSim(n, seed=seed, peer_mode=peer_mode, fanout=fanout, quirk=quirk, remove=remove)
    import oracle.listsim as L
    L.T_FAIL, L.T_CLEANUP = t_fail, t_cleanup
    try:
        for r in range(1, rounds + 1):
            ev = sched.get(r, [])
            if ev:
                orc.apply_events(ev)
                ls.apply_events(ev)
            s1 = orc.step(1)
            s2 = ls.step(1)
            assert s1 == s2, f"round {r}: stats {s1} != {s2}"
            h1, t1, a1 = orc.export_state()
            h2, t2, a2 = ls.dense()
            np.testing.assert_array_equal(a1, a2, err_msg=f"alive r={r}")
            np.testing.assert_array_equal(h1, h2, err_msg=f"hb r={r}")
            np.testing.assert_array_equal(t1, sc.export_view(h2, t2, r, t_cleanup)[1], err_msg=f"ts r={r}")
            bm = orc.read_failed()
            failed = [c for c in range(n) if bm[c >> 5] >> (c & 31) & 1]
            assert failed == ls.last_failed
            assert list(orc.read_detectors()) == ls.last_detectors
            if per_round:
                per_round(orc, ls, r)
    finally:
        L.T_FAIL, L.T_CLEANUP = 5, 5
    return orc, ls


@pytest.mark.parametrize("peer_mode", ["ring", "pull"])
@pytest.mark.parametrize("quirk", [False, True])
def test_bootstrap_crash_c1(oracle_mod, peer_mode, quirk):
    """BASELINE config 1 shape: 10 joins, member 7 crashes at r=30, to r=60."""
    n = 10
    sched = sc.bootstrap_schedule(n)
    sched.setdefault(30, []).append((sc.CRASH, 7))
    orc, ls = run_pair(oracle_mod, n, 60, sched, peer_mode, quirk=quirk)
    hb, ts, alive = orc.export_state()
    assert alive[7] == 0


@pytest.mark.parametrize("seed", [1, 2, 3])
@pytest.mark.parametrize("peer_mode", ["ring", "pull"])
def test_random_churn(oracle_mod, seed, peer_mode):
    n = 16
    sched = sc.random_churn(n, 50, seed)
    run_pair(oracle_mod, n, 50, sched, peer_mode, fanout=2, init_full=True, seed=0x1000 + seed)


@pytest.mark.parametrize("seed", [4, 5])
def test_random_churn_quirk(oracle_mod, seed):
    n = 14
    sched = sc.random_churn(n, 40, seed, p_crash=0.08)
    run_pair(oracle_mod, n, 40, sched, "ring", init_full=True, quirk=True, seed=0x2000 + seed)


def test_fast_fail_short_cooldown(oracle_mod):
    """T_fail/T_cleanup off their defaults (tombstones survive detection)."""
    n = 12
    sched = sc.random_churn(n, 40, 9, p_crash=0.1)
    run_pair(oracle_mod, n, 40, sched, "pull", fanout=3, init_full=True, t_fail=3, t_cleanup=6)


# ---- the reference's REMOVE recipients (GH_REMOVE_LIST, slave/slave.go:344) ----

@pytest.mark.parametrize("seed", [1, 2, 3])
@pytest.mark.parametrize("peer_mode", ["ring", "pull"])
@pytest.mark.parametrize("quirk", [False, True])
def test_random_churn_remove_list(oracle_mod, seed, peer_mode, quirk):
    """listsim's literal Remove (recipients = the detector's list right after
    removeMember in the sweep) against tablesim's column-wise form."""
    n = 16
    sched = sc.random_churn(n, 50, seed, p_crash=0.06)
    run_pair(oracle_mod, n, 50, sched, peer_mode, fanout=2, init_full=True, quirk=quirk,
             seed=0x3000 + seed, remove="list")


@pytest.mark.parametrize("quirk", [False, True])
def test_collapse_remove_list(oracle_mod, quirk):
    """The reference's constants at a size where dissemination outruns them
    not: the round-6 detection storm and the collapse, literal recipients."""
    n = 48
    run_pair(oracle_mod, n, 14, {}, "pull", fanout=3, init_full=True, quirk=quirk, seed=0x5EED0002,
             remove="list")


@pytest.mark.parametrize("seed", [7, 8])
def test_bootstrap_churn_remove_list(oracle_mod, seed):
    n = 12
    sched = sc.bootstrap_schedule(n)
    for r, ev in sc.random_churn(n, 50, seed, p_crash=0.05).items():
        sched.setdefault(r + n, []).extend(ev)
    run_pair(oracle_mod, n, 60, sched, "ring", init_full=False, seed=0x4000 + seed, remove="list")


@pytest.mark.parametrize("peer_mode", ["ring", "pull"])
@pytest.mark.parametrize("quirk", [False, True])
@pytest.mark.parametrize("seed", [11, 12])
def test_rejoin_while_tombstoned(oracle_mod, peer_mode, quirk, seed):
    """SPEC D7 under churn: members leave or crash and rejoin while the
    introducer still holds their tombstone, so its list holds them twice
    (MemberList and RecentFailList, slave/slave.go:228-230, 250-255); later
    LEAVEs, REMOVEs and detections meet the double entry
    (:276-286) and cleanFailList releases the old entry (:484-497).
    listsim (the literal lists) = tablesim (the shadow entries) every round,
    and double entries do occur."""
    n = 12
    sched = sc.rejoin_churn(n, 45, seed)
    seen = []

    def per_round(orc, ls, r):
        sh = orc.debug_shadow()
        I = ls.nodes[0]
        dual = sorted(m.addr for m in I.members if any(f.addr == m.addr for f in I.recent_fail))
        assert sorted(np.nonzero(sh != np.iinfo(np.int32).min)[0].tolist()) == dual, (r, sh, dual)
        for f in I.recent_fail:  # the entry's own ts (removeMember kept the Member, :280)
            if f.addr in dual:
                assert sh[f.addr] == f.ts, (r, f.addr, sh[f.addr], f.ts)
        seen.append(len(dual))

    run_pair(oracle_mod, n, 45, sched, peer_mode, quirk=quirk, init_full=True, seed=0x3000 + seed,
             t_fail=4, t_cleanup=6, per_round=per_round)
    assert max(seen) > 0, seen
