"""SPEC D1 (list order), measured: the reference appends members to its
MemberList (slave/slave.go:255 addNewMember, :437 MergeMemberList) while the
engine and the tablesim oracle keep member-ID order. oracle/listsim.py runs
both orders with the literal Go list semantics; these tests pin where the
two coincide and where they part (CPU, seconds).

Measured (tools-free, this file):
  * BASELINE config 1 (10 members joining one per round through the
    introducer, member 7 crashing at r=30, 60 rounds): identical in ring and
    pull mode, canonical and quirk detection -- joins arrive in ID order and
    nothing is re-added.
  * Pull mode with canonical detection: identical under any churn -- the
    merge, detection and cleanup rules act on the list as a SET.
  * Ring mode and quirk detection under churn with re-adds (a member whose
    tombstone was released comes back through a merge and is appended at
    the END of the list): the orders part within a few rounds, because ring
    targets are list neighbours (slave/slave.go:515-519) and quirk runs are
    list runs (:464-477)."""
import numpy as np
import pytest

import scenarios as sc
from oracle.listsim import ListSim


def run(n, rounds, sched, peer_mode, quirk, order, init_full=False, fanout=3, seed=0x5EED0001):
    if init_full:
        hb, ts, alive = sc.full_state(n)
        sim = ListSim.from_dense(hb, ts, alive, 0, seed=seed, peer_mode=peer_mode, fanout=fanout, quirk=quirk,
                                 order=order)
    else:
        sim = ListSim(n, seed=seed, peer_mode=peer_mode, fanout=fanout, quirk=quirk, order=order)
    out = []
    for r in range(1, rounds + 1):
        if r in sched:
            sim.apply_events(sched[r])
        st = sim.step(1)
        hb, ts, _ = sim.dense()
        out.append((st, hb, ts, tuple(sim.last_failed)))
    return out, sim


def differing_rounds(n, rounds, sched, peer_mode, quirk, **kw):
    a, sa = run(n, rounds, sched, peer_mode, quirk, "append", **kw)
    b, _ = run(n, rounds, sched, peer_mode, quirk, "id", **kw)
    diff = [r for r, (x, y) in enumerate(zip(a, b), 1)
            if not (x[0] == y[0] and np.array_equal(x[1], y[1]) and np.array_equal(x[2], y[2]) and x[3] == y[3])]
    reordered = sum(1 for nd in sa.nodes if nd.alive and [m.addr for m in nd.members] != sorted(m.addr for m in nd.members))
    return diff, reordered


def c1_schedule():
    sched = {r: [(sc.JOIN, r - 1)] for r in range(1, 11)}
    sched.setdefault(30, []).append((sc.CRASH, 7))
    return sched


@pytest.mark.parametrize("peer_mode", ["ring", "pull"])
@pytest.mark.parametrize("quirk", [False, True], ids=["canonical", "quirk"])
def test_c1_orders_identical(peer_mode, quirk):
    diff, reordered = differing_rounds(10, 60, c1_schedule(), peer_mode, quirk)
    assert diff == [] and reordered == 0


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_pull_canonical_order_free(seed):
    sched = sc.random_churn(24, 80, seed, p_crash=0.03, p_leave=0.02, p_join=0.08)
    diff, reordered = differing_rounds(24, 80, sched, "pull", False, init_full=True)
    assert diff == []
    assert reordered > 0  # the lists themselves did leave ID order


@pytest.mark.parametrize("peer_mode,quirk", [("ring", False), ("ring", True), ("pull", True)])
def test_order_matters_under_readds(peer_mode, quirk):
    """Seeded churn with re-adds: ring targets and quirk runs follow list
    order, so the append-order replay leaves the ID-order one."""
    sched = sc.random_churn(24, 80, 3, p_crash=0.03, p_leave=0.02, p_join=0.08)
    diff, reordered = differing_rounds(24, 80, sched, peer_mode, quirk, init_full=True)
    assert reordered > 0 and len(diff) > 0
