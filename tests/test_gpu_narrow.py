"""GPU parity of the narrow/wide table encoding (gh_internal.h, DESIGN.md
"Data layout in HBM"): states whose heartbeats do not fit a 16-bit narrow cell
(spread beyond the 1,022-round window of the column base, stale outliers,
base jumps, saturated ages, timeouts past the age cap) must give the oracle's
results bit for bit while segments move between the narrow and the wide
encoding. Run on a MI355X: pytest -m gpu."""
import numpy as np
import pytest

import scenarios as sc
from test_gpu_parity import compare


pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gs():
    import gossipsim
    return gossipsim


def spread_state(n, seed, lo=0, hi=5_000_000, p_absent=0.1, p_tomb=0.05, round0=0):
    """Every cell an independent heartbeat in [lo, hi) (most segments wide),
    with absent and tombstoned cells; ts within the T window of round0."""
    rng = np.random.default_rng(seed)
    hb = rng.integers(lo, hi, (n, n), dtype=np.int64).astype(np.int32)
    u = rng.random((n, n))
    hb[u < p_absent] = -1
    hb[(u >= p_absent) & (u < p_absent + p_tomb)] = -2
    ts = rng.integers(round0 - 3, round0 + 2, (n, n)).astype(np.int32)
    alive = np.ones(n, np.uint8)
    return hb, ts, alive


def run_cov(gs, om, cfg_kw, n, rounds, sched, init, every=1):
    """run_parity with the encoding read-outs: returns (wide segments right
    after the import, max wide over the rounds, total slow-list segments)."""
    eng = gs.Engine(gs.default_config(n, **cfg_kw))
    orc = om.Oracle(om.default_config(n, **cfg_kw), threads=8)
    eng.import_state(*init, 0)
    orc.import_state(*init, 0)
    wide0 = eng.encoding_info()[0]
    wmax, slow = wide0, 0
    for r in range(1, rounds + 1):
        ev = sched.get(r, [])
        if ev:
            eng.apply_events(ev)
            orc.apply_events(ev)
        s1, s2 = eng.step(1), orc.step(1)
        assert s1 == s2, f"round {r}: gpu {s1} != cpu {s2}"
        w, sl = eng.encoding_info()
        wmax, slow = max(wmax, w), slow + sl
        if r % every == 0 or r == rounds or ev:
            compare(eng, orc, r)
    eng.close()
    return wide0, wmax, slow


@pytest.mark.parametrize("n,peer_mode,seed", [(64, 0, 1), (200, 1, 2), (300, 0, 3)])
def test_wide_spread_import(gs, oracle_mod, n, peer_mode, seed):
    """Heartbeats spread over millions: wide segments everywhere, narrowed as
    the gossip pulls each column's views within the base window."""
    sched = sc.random_churn(n, 24, 100 + seed, p_crash=0.03, p_leave=0.01, p_join=0.04)
    wide0, _, slow = run_cov(gs, oracle_mod, dict(peer_mode=peer_mode, fanout=3, seed=0x9100 + seed, t_fail=6,
                                                  t_cleanup=8), n, 24, sched, spread_state(n, seed))
    assert wide0 > 0 and slow > 0


@pytest.mark.parametrize("n,seed", [(128, 4), (257, 5)])
def test_stale_outliers(gs, oracle_mod, n, seed):
    """Columns near their member's own heartbeat (narrow) with a few views
    more than 1,022 rounds stale (below the base): mixed narrow and wide
    segments in one column, and the outliers' merges."""
    rng = np.random.default_rng(seed)
    own = rng.integers(5_000, 50_000, n).astype(np.int64)
    hb = (own[None, :] - rng.integers(0, 4, (n, n))).astype(np.int32)
    stale = rng.random((n, n)) < 0.03
    hb[stale] = (own[None, :] - 1500 - rng.integers(0, 3000, (n, n)))[stale].astype(np.int32)
    np.fill_diagonal(hb, own.astype(np.int32))
    ts = np.zeros((n, n), np.int32)
    alive = np.ones(n, np.uint8)
    sched = sc.random_churn(n, 20, 200 + seed, p_crash=0.03, p_leave=0.01, p_join=0.03)
    wide0, wmax, slow = run_cov(gs, oracle_mod, dict(fanout=4, seed=0x9200 + seed, t_fail=5, t_cleanup=7), n, 20,
                                sched, (hb, ts, alive))
    assert wmax > 0 and slow > 0


def test_base_jump_by_merge(gs, oracle_mod):
    """External lists that raise members' heartbeats by far more than 1,023
    (gh_merge_list): the column base jumps and the rows catch up."""
    n = 150
    cfg = dict(fanout=3, seed=0x9301, t_fail=6, t_cleanup=8)
    eng = gs.Engine(gs.default_config(n, **cfg))
    orc = oracle_mod.Oracle(oracle_mod.default_config(n, **cfg), threads=8)
    init = sc.full_state(n, hb0=7)
    eng.import_state(*init, 0)
    orc.import_state(*init, 0)
    rng = np.random.default_rng(13)
    wmax = 0
    for r in range(1, 21):
        assert eng.step(1) == orc.step(1), r
        if r % 3 == 0:
            ids = rng.permutation(n)[:40].astype(np.int32)
            hb = (rng.integers(0, 3, 40) * 700_000 + rng.integers(0, 5_000, 40)).astype(np.int32)
            obs = int(rng.integers(0, n))
            assert eng.merge_list(obs, ids, hb) == orc.merge_list(obs, ids, hb)
            wmax = max(wmax, eng.encoding_info()[0])
        compare(eng, orc, r)
    eng.close()
    assert wmax > 0


@pytest.mark.parametrize("t_fail,t_cleanup", [(20, 25), (29, 30), (40, 45)])
def test_age_saturation(gs, oracle_mod, t_fail, t_cleanup):
    """Ages past the narrow age field (cap 31): heartbeats 0/1 are never
    detected, so their ages saturate and the exact ts goes to the ts table;
    timeouts at or past the cap run every cell by the exact rule."""
    n = 96
    hb, ts, alive = sc.full_state(n, hb0=1)
    hb[:, ::7] = 0
    sched = sc.random_churn(n, 48, 300 + t_fail, p_crash=0.02, p_leave=0.01, p_join=0.02)
    _, _, slow = run_cov(gs, oracle_mod, dict(fanout=2, seed=0x9400 + t_fail, t_fail=t_fail, t_cleanup=t_cleanup),
                         n, 48, sched, (hb, ts, alive), every=4)
    assert slow > 0


@pytest.mark.parametrize("world", [2, 3])
def test_wide_spread_sharded(gs, oracle_mod, world):
    """The wide-spread start over column shards (bases are per local column)."""
    from test_gpu_sharded import run_group
    n = 200
    sched = sc.random_churn(n, 20, 400 + world, p_crash=0.03, p_leave=0.01, p_join=0.04)
    run_group(gs, oracle_mod, world, dict(fanout=3, seed=0x9500 + world, t_fail=6, t_cleanup=8), n, 20, sched,
              init=spread_state(n, 40 + world))


def test_steady_state_stays_narrow(gs):
    """The bench regime (full start, healthy gossip): after the first rounds
    every segment is narrow and no segment needs the per-cell rule."""
    n = 4096
    eng = gs.Engine(gs.default_config(n, fanout=4, seed=0x9600, t_fail=16, t_cleanup=16))
    eng.init_full(2, 0, 0)
    eng.step(6)
    assert eng.encoding_info() == (0, 0)
    eng.close()


@pytest.mark.parametrize("peer_mode", [0, 1])
def test_storm_variant_collapse(gs, oracle_mod, peer_mode):
    """A failure storm and the collapse under the <4 guard (BASELINE config
    2's regime, T_fail=5 at N=4,096): the storm variant of the round kernel
    (detections, REMOVE, releases and guard rows in the packed path) runs and
    matches the oracle every round."""
    n = 4096
    cfg = dict(peer_mode=peer_mode, fanout=3, seed=0x9700 + peer_mode, t_fail=5, t_cleanup=5)
    eng = gs.Engine(gs.default_config(n, **cfg))
    orc = oracle_mod.Oracle(oracle_mod.default_config(n, **cfg), threads=8)
    init = sc.full_state(n)
    eng.import_state(*init, 0)
    orc.import_state(*init, 0)
    sched = {4: [(sc.CRASH, c) for c in sc.crash_ids(n, 0.01, 0x9701)]}
    storm_rounds = 0
    for r in range(1, 17):
        if r in sched:
            eng.apply_events(sched[r])
            orc.apply_events(sched[r])
        assert eng.step(1) == orc.step(1), r
        storm_rounds += eng.encoding_info(full=True)[2]
        if r % 4 == 0 or r > 5:
            compare(eng, orc, r)
    eng.close()
    assert storm_rounds > 0
