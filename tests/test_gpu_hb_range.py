"""GPU parity over the full heartbeat range and the sparse wide store.

The reference's HeartbeatCount is a Go int (master/master.go:18) incremented
without a bound (slave/slave.go:446). libgossiphip keeps int32 heartbeats:
any value 0..INT32_MAX is held exactly (narrow 16-bit cells relative to a
per-column base, or the wide arena), and a round that would increment
INT32_MAX is refused with GH_ERANGE by both the HIP path and the oracle
(SPEC.md §2), after the same rounds, with the same state.

Also: the wide arena growing between calls, an arena overflow inside a round
losing the state loudly (GH_ENOMEM) until a full import, and the HBM
footprint at the headline N=65,536. Run on a MI355X: pytest -m gpu."""
import numpy as np
import pytest

import scenarios as sc
from test_gpu_parity import compare

pytestmark = pytest.mark.gpu

I32MAX = 2**31 - 1


@pytest.fixture(scope="module")
def gs():
    import gossipsim
    return gossipsim


def pair(gs, om, n, **cfg):
    return gs.Engine(gs.default_config(n, **cfg)), om.Oracle(om.default_config(n, **cfg), threads=8)


def wide_range_state(n, seed):
    """Own heartbeats at 2^23 - 3 (crossing 2^23 in the first rounds), near
    2^31 and small, views lagging each owner by 0..3 rounds."""
    rng = np.random.default_rng(seed)
    own = np.where(np.arange(n) % 3 == 0, 2**23 - 3, np.where(np.arange(n) % 3 == 1, I32MAX - 400, 5))
    own = own - rng.integers(0, 4, n)
    hb = (own[None, :] - rng.integers(0, 4, (n, n))).astype(np.int64)
    np.fill_diagonal(hb, own)
    hb = hb.astype(np.int32)
    ts = np.zeros((n, n), np.int32)
    alive = np.ones(n, np.uint8)
    return hb, ts, alive


@pytest.mark.parametrize("peer_mode,seed", [(0, 1), (1, 2)])
def test_heartbeats_across_2p23_and_near_2p31(gs, oracle_mod, peer_mode, seed):
    n = 96
    eng, orc = pair(gs, oracle_mod, n, peer_mode=peer_mode, fanout=3, seed=0xA100 + seed, t_fail=6, t_cleanup=8)
    init = wide_range_state(n, seed)
    eng.import_state(*init, 0)
    orc.import_state(*init, 0)
    sched = sc.random_churn(n, 30, 500 + seed, p_crash=0.03, p_leave=0.01, p_join=0.04)
    rng = np.random.default_rng(seed)
    for r in range(1, 31):
        if r in sched:
            eng.apply_events(sched[r])
            orc.apply_events(sched[r])
        assert eng.step(1) == orc.step(1), r
        if r % 4 == 0:
            # received lists raising members far beyond the column base:
            # values near 2^31, just past 2^23, and small
            ids = rng.permutation(n)[:30].astype(np.int32)
            hb = np.concatenate([I32MAX - 300 + rng.integers(0, 100, 10), 2**23 + rng.integers(0, 50, 10),
                                 rng.integers(0, 20, 10)]).astype(np.int32)
            obs = int(rng.integers(0, n))
            assert eng.merge_list(obs, ids, hb) == orc.merge_list(obs, ids, hb)
        compare(eng, orc, r)
    h, _, _ = eng.export_state()
    assert h.max() > I32MAX - 400 and (h == 2**23 + 2).any()  # the ranges were exercised
    eng.close()


def test_int32_overflow_refused_like_the_oracle(gs, oracle_mod):
    """Member 5's own heartbeat reaches INT32_MAX; the next round is refused
    by both (GH_ERANGE), after the same rounds and with the same state."""
    n = 24
    eng, orc = pair(gs, oracle_mod, n, fanout=3, seed=0xA201, t_fail=6, t_cleanup=6)
    hb, ts, alive = sc.full_state(n, hb0=7)
    hb[:, 5] = I32MAX - 6
    hb[5, 5] = I32MAX - 3
    eng.import_state(hb, ts, alive, 0)
    orc.import_state(hb, ts, alive, 0)
    rc1, s1 = eng.step_rc(10)
    rc2, s2 = orc.step_rc(10)
    assert rc1 == rc2 == gs._abi.GH_ERANGE
    assert s1 == s2 and s1["rounds"] == 3
    compare(eng, orc, 3)
    h, _, _ = eng.export_state()
    assert h[5, 5] == I32MAX
    # refused again, nothing runs, and a refused round's events stay pending
    # (member 9's leave); member 5 crashing in the same round lets it run
    eng.apply_events([(sc.LEAVE, 9)])
    orc.apply_events([(sc.LEAVE, 9)])
    rc1, s1 = eng.step_rc(1)
    rc2, s2 = orc.step_rc(1)
    assert rc1 == rc2 == gs._abi.GH_ERANGE and s1 == s2 and s1["rounds"] == 0
    compare(eng, orc, 3)
    eng.apply_events([(sc.CRASH, 5)])
    orc.apply_events([(sc.CRASH, 5)])
    assert eng.step(4) == orc.step(4)
    compare(eng, orc, 7)
    h, _, al = eng.export_state()
    assert not al[5] and not al[9] and h[0, 9] == -2  # both events ran in round 4
    eng.close()


def test_import_range_matches_oracle(gs, oracle_mod):
    """Both accept every int32 >= -2 and any ts; both reject -3 (GH_ERANGE)."""
    n = 16
    eng, orc = pair(gs, oracle_mod, n)
    hb, ts, alive = sc.full_state(n)
    hb[0, 1], hb[2, 3], ts[4, 5], ts[6, 7] = I32MAX, 0, -2**31, 2**31 - 1
    eng.import_state(hb, ts, alive, 10)
    orc.import_state(hb, ts, alive, 10)
    compare(eng, orc, 10)
    assert eng.step(3) == orc.step(3)
    compare(eng, orc, 13)
    hb[1, 1] = -3
    with pytest.raises(gs.GossipError) as ex:
        eng.import_state(hb, ts, alive, 0)
    assert ex.value.code == gs._abi.GH_ERANGE
    with pytest.raises(RuntimeError, match="-6"):
        orc.import_state(hb, ts, alive, 0)
    eng.close()


def test_arena_grows_between_calls(gs, oracle_mod):
    """A 4-slot arena and a state whose segments are nearly all wide: the
    import grows the arena and the rounds stay bit-exact."""
    from test_gpu_narrow import spread_state
    n = 200
    eng, orc = pair(gs, oracle_mod, n, fanout=3, seed=0xA301, t_fail=6, t_cleanup=8, wide_segments=4)
    init = spread_state(n, 7)
    eng.import_state(*init, 0)
    orc.import_state(*init, 0)
    m0 = eng.memory_info()
    assert m0["wide_cap"] > 4 and m0["wide_used"] > 0
    for r in range(1, 16):
        assert eng.step(1) == orc.step(1), r
        compare(eng, orc, r)
    eng.close()


def test_arena_overflow_in_a_round_loses_state_loudly(gs, oracle_mod):
    """Every cell of heartbeat <= 1 is 31 rounds old (narrow): in round 1 all
    age past the narrow field at once and need the wide arena, which has one
    slot: gh_step fails with GH_ENOMEM, the state is refused until a full
    import, after which the engine matches the oracle again."""
    n = 128
    eng, orc = pair(gs, oracle_mod, n, fanout=3, seed=0xA401, t_fail=40, t_cleanup=40, wide_segments=1)
    hb, ts, alive = sc.full_state(n, hb0=1)
    ts[:] = 10 - 31  # age 31 in round 10 (the oldest a narrow cell holds)
    eng.import_state(hb, ts, alive, 9)
    with pytest.raises(gs.GossipError) as ex:
        eng.step(1)
    assert ex.value.code == gs._abi.GH_ENOMEM
    with pytest.raises(gs.GossipError):
        eng.export_state()
    init = sc.full_state(n)
    eng.import_state(*init, 0)
    orc.import_state(*init, 0)
    assert eng.step(5) == orc.step(5)
    compare(eng, orc, 5)
    eng.close()


def test_long_collapse_stays_narrow(gs, oracle_mod):
    """The reference's 5-round timeouts at N=2,048: the round-6 storm, the
    collapse under the <4 guard, then 40 more rounds in which every guard
    row's tombstones age past T_cleanup (saturated at T_cleanup + 1 = 6,
    exported as 6 rounds old by both; the rows then stop changing)."""
    n = 2048
    eng, orc = pair(gs, oracle_mod, n, fanout=3, seed=0xA501)
    eng.init_full(2, 0, 0)
    orc.init_full(2, 0, 0)
    for r in range(1, 49):
        assert eng.step(1) == orc.step(1), r
        if r in (6, 7, 30, 37, 48):
            compare(eng, orc, r)
    assert eng.memory_info()["wide_used"] == 0
    eng.close()


def test_footprint_n65536(gs):
    """The headline configuration's tables in HBM: <= 31 GiB (the narrow
    table x2 is 16 GiB, the 8-bit tier x2 8 GiB, the sender plane x2 4 GiB,
    the wide arenas 2 GiB and the rest < 1 GiB; GH_PLANE=0 drops the plane and
    the tier, GH_C8=0 the tier), measured with hipMemGetInfo around the
    engine's creation and first rounds."""
    import ctypes as C
    hip = C.CDLL("libamdhip64.so")

    def free():
        f, t = C.c_size_t(), C.c_size_t()
        assert hip.hipMemGetInfo(C.byref(f), C.byref(t)) == 0
        return f.value

    eng0 = gs.Engine(gs.default_config(64))  # the HIP context exists before the first reading
    free0 = free()
    eng = gs.Engine(gs.default_config(65536, fanout=4, seed=0x5EED0003, t_fail=16, t_cleanup=16))
    eng.init_full(2, 0, 0)
    eng.step(3)
    used = free0 - free()
    info = eng.memory_info()
    eng.close()
    eng0.close()
    print(f"N=65536: {used / 2**30:.2f} GiB by hipMemGetInfo, tables {info['device_bytes'] / 2**30:.2f} GiB")
    assert used <= 31 * 2**30 and info["device_bytes"] <= used
