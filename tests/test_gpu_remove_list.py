"""GPU parity of the reference's REMOVE recipients (GH_REMOVE_LIST,
slave/slave.go:338-363 with :472-473: Remove messages the detector's list as
it stands right after removeMember, itself excluded): libgossiphip's
column-bitmap form (csrc/remove.hip) against tablesim's per-detector
restatement (oracle/tablesim.c), bit for bit every round, on churn in both
detection modes and peer modes, the reference's 5-round timeouts (detection
storm: the recipient sets need explicit bitmap intersections), BASELINE
config 2's crash and the 4-bit tier's nibble path. The hand-derived KATs
(kat14L, kat15) run in test_gpu_parity.py::test_kats_gpu."""
import os

import numpy as np
import pytest

import scenarios as sc
from test_gpu_parity import run_parity

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gs():
    import gossipsim
    return gossipsim


@pytest.mark.parametrize("quirk", [0, 1])
@pytest.mark.parametrize("n,peer_mode,seed", [(16, 0, 1), (16, 1, 2), (64, 0, 3), (64, 1, 4), (300, 0, 5),
                                              (257, 1, 6)])
def test_churn_remove_list(gs, oracle_mod, n, peer_mode, seed, quirk):
    sched = sc.random_churn(n, 40, seed, p_crash=0.06, p_leave=0.02, p_join=0.05)
    run_parity(gs, oracle_mod, dict(peer_mode=peer_mode, fanout=3, seed=0x3300 + seed, detect_mode=quirk,
                                    t_fail=3, t_cleanup=5, remove_mode=1), n, 40, sched, init=sc.full_state(n))


@pytest.mark.parametrize("quirk", [0, 1])
def test_collapse_remove_list_n4096(gs, oracle_mod, quirk):
    """T_fail = T_cleanup = 5 at N=4,096: the round-6 storm, where most
    (receiver, member) pairs are settled by the counts and the rest by
    intersecting the detectors' and the survivors' column bitmaps."""
    n = 4096
    run_parity(gs, oracle_mod, dict(fanout=3, seed=0x5EED0002, detect_mode=quirk, remove_mode=1), n, 12, {},
               init=sc.full_state(n), every=2)


def test_c2_crash_remove_list(gs, oracle_mod):
    """BASELINE config 2 (N=4,096, k=3, 1% crash at r=8) with the reference's
    recipients, 40 rounds."""
    n = 4096
    sched = {8: [(sc.CRASH, c) for c in sc.crash_ids(n, 0.01, 0x5EED0002)]}
    run_parity(gs, oracle_mod, dict(fanout=3, seed=0x5EED0002, remove_mode=1), n, 40, sched,
               init=sc.full_state(n), every=4)


def test_tier_crash_remove_list(gs, oracle_mod, monkeypatch):
    """The 4-bit tier (nibble path + lane jobs: REMOVE'd lanes are jobs,
    whose per-cell rule asks the recipient bitmaps) at N=1,024, T_fail=12,
    a 2% crash with false positives from a short cleanup."""
    monkeypatch.setenv("GH_PLANE", "1")
    n = 1024
    sched = {6: [(sc.CRASH, c) for c in sc.crash_ids(n, 0.02, 0x5EED0009)]}
    eng, _ = run_parity(gs, oracle_mod, dict(fanout=4, seed=0x5EED0009, t_fail=12, t_cleanup=12, remove_mode=1),
                        n, 40, sched, init=sc.full_state(n), every=2)
    assert eng.tier_info()[0] == 1
