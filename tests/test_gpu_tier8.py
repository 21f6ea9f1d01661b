"""4-bit tier (csrc/gh_internal.h `c4_dec` / `c4_enc`, DESIGN.md "Cell
encoding"): in plane mode every cell of a healthy chunk is a 4-bit lag code
(which is also the sender plane) and a 4-bit age, run by the nibble path
(k_round IN 2 / 4) and its lane jobs; chunks the tier cannot hold -- flags,
young tombstones, wide and frozen markers, lags past the window, ages past
min(T_fail, 15) -- are escaped to 16-bit codes. These tests pin that the tier is in use
where it should be, that escapes happen and stay bit-exact against the
oracle, that events, imports, quirk flag clears, list merges, storms and
quiet rows cross it, and that it changes no result against the 16-bit table
(GH_C8=0). Small clusters keep the plane (and so the tier) through
GH_PLANE=1. Run on a MI355X: pytest -m gpu."""
import numpy as np
import pytest

import scenarios as sc
from test_gpu_parity import compare, run_parity

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gs():
    import gossipsim
    return gossipsim


@pytest.fixture(autouse=True)
def tier_on(monkeypatch):
    monkeypatch.setenv("GH_PLANE", "1")
    monkeypatch.delenv("GH_C8", raising=False)


def test_tier_steady_state(gs, oracle_mod):
    """N=2,048, k=4 pull from full membership with the bench's timeouts: the
    lean rounds write the 8-bit tier from round 1 on, the healthy rounds
    escape no chunk, crash / leave / join events write into 8-bit buffers, the
    detection wave's storm rounds switch to 16 bits and back; bit-exact every
    round."""
    n = 2048
    cfg = dict(fanout=4, seed=0x5EED0007, t_fail=16, t_cleanup=16)
    eng = gs.Engine(gs.default_config(n, **cfg))
    orc = oracle_mod.Oracle(oracle_mod.default_config(n, **cfg), threads=8)
    hb, ts, alive = sc.full_state(n)
    eng.import_state(hb, ts, alive, 0)
    orc.import_state(hb, ts, alive, 0)
    assert eng.tier_info()[:2] == (1, 0)  # an import leaves a 16-bit table
    sched = {14: [(sc.CRASH, 7), (sc.LEAVE, 1500)], 18: [(sc.JOIN, 1500), (sc.JOIN, 7)]}
    esc, tiers = [], []
    for r in range(1, 56):
        ev = sched.get(r, [])
        if ev:
            eng.apply_events(ev)
            orc.apply_events(ev)
        s1, s2 = eng.step(1), orc.step(1)
        assert s1 == s2, f"round {r}: gpu {s1} != cpu {s2}"
        compare(eng, orc, r)
        en, cur8, e = eng.tier_info()
        assert en == 1
        esc.append(e)
        tiers.append(cur8)
    # 8-bit from the first round on; the crash's detection and tombstones
    # (rounds ~31-48) run the storm variant (16-bit), the healthy rounds after
    # them return to 8 bits
    assert tiers[:13] == [1] * 13 and 0 in tiers and tiers[-1] == 1, tiers
    assert esc[7:13] == [0] * 6, esc


def ranged_state(n, seed):
    """Views lagging their owners by 0..40 rounds (past the 14-round byte
    window), ages up to 24 (past 15), ahead-of-owner views (offsets above
    the byte reference) and a few tombstones: every kind of escape, all
    within the 16-bit narrow window and rare enough (tombstones in ~1% of the
    segments) for the lean variant to run."""
    rng = np.random.default_rng(seed)
    own = 1000 + rng.integers(0, 5, n)
    hb = own[None, :] - rng.integers(0, 41, (n, n))
    ahead = np.arange(n) % 97 == 3
    hb[:, ahead] = own[ahead][None, :] + rng.integers(1, 9, (n, int(ahead.sum())))
    tomb = rng.random((n, n)) < 0.00004
    hb[tomb] = -2
    np.fill_diagonal(hb, own)
    ts = rng.integers(16, 41, (n, n)).astype(np.int32)
    np.fill_diagonal(ts, 40)
    return hb.astype(np.int32), ts, np.ones(n, np.uint8)


@pytest.mark.parametrize("k", [3, 4])
def test_tier_escapes_exact(gs, oracle_mod, k):
    """Lags, ages and tombstones outside the byte codes: the lean rounds
    escape chunks (escaped > 0) and every round stays bit-exact."""
    n = 1024
    cfg = dict(fanout=k, seed=0x5EED0110 + k, t_fail=60, t_cleanup=60)
    eng = gs.Engine(gs.default_config(n, **cfg))
    orc = oracle_mod.Oracle(oracle_mod.default_config(n, **cfg), threads=8)
    hb, ts, alive = ranged_state(n, k)
    eng.import_state(hb, ts, alive, 40)
    orc.import_state(hb, ts, alive, 40)
    esc = []
    for r in range(1, 16):
        s1, s2 = eng.step(1), orc.step(1)
        assert s1 == s2, f"round {r}: gpu {s1} != cpu {s2}"
        compare(eng, orc, r)
        esc.append(eng.tier_info()[2])
    assert sum(esc) > 0, esc


def run_states(gs, n, cfg, sched, rounds, init, merges=None):
    eng = gs.Engine(gs.default_config(n, **cfg))
    eng.import_state(*init, 0)
    out = []
    for r in range(1, rounds + 1):
        ev = sched.get(r, [])
        if ev:
            eng.apply_events(ev)
        if merges and r in merges:
            obs, ids, hbs = merges[r]
            eng.merge_list(obs, ids, hbs)
        st = eng.step(1)
        out.append((st, eng.export_state(), eng.read_failed(), eng.read_detectors(), eng.lsm(3)))
    info = eng.tier_info()
    eng.close()
    return out, info


def assert_same(base, other):
    for r, (a, b) in enumerate(zip(base, other), 1):
        assert a[0] == b[0], (r, a[0], b[0])
        for x, y in zip(a[1], b[1]):
            np.testing.assert_array_equal(x, y, err_msg=f"round {r}")
        np.testing.assert_array_equal(a[2], b[2])
        np.testing.assert_array_equal(a[3], b[3])
        for x, y in zip(a[4], b[4]):
            np.testing.assert_array_equal(x, y, err_msg=f"lsm round {r}")


@pytest.mark.parametrize("detect_mode", [0, 1], ids=["canonical", "quirk"])
@pytest.mark.parametrize("order", [0, 1], ids=["id_order", "append_order"])
def test_tier_matches_16bit(gs, monkeypatch, detect_mode, order):
    """Seeded churn with detection waves (T_fail 6: storm rounds write 16-bit
    tables, lean rounds 8-bit ones), quirk flag clears and datagram merges
    into 8-bit buffers: the tier gives the same tables, counters, failed
    sets, detectors and lists every round as the 16-bit table (GH_C8=0)."""
    n = 1536
    cfg = dict(fanout=4, seed=0x5EED0210 + 2 * detect_mode + order, t_fail=6, t_cleanup=8,
               detect_mode=detect_mode, list_order=order)
    sched = sc.random_churn(n, 40, 0x78 + detect_mode, p_crash=0.01, p_leave=0.005, p_join=0.02)
    rng = np.random.default_rng(5)
    merges = {r: (int(rng.integers(0, n)), np.arange(0, n, 7, dtype=np.int32),
                  rng.integers(0, 60, len(range(0, n, 7))).astype(np.int32)) for r in (9, 21, 33)}
    init = sc.full_state(n)
    base, info = run_states(gs, n, cfg, sched, 40, init, merges)
    assert info[0] == 1
    monkeypatch.setenv("GH_C8", "0")
    other, info2 = run_states(gs, n, cfg, sched, 40, init, merges)
    assert info2[0] == 0
    assert_same(base, other)


def test_tier_quiet_rows_collapse(gs, oracle_mod):
    """The reference's 5-round timeouts at N=2,048: the detection storm runs
    the storm variant (16-bit), the collapsed cluster's lean rounds switch
    the tables back to the 8-bit tier while rows are quiet, a join rewrites
    rows. Bit-exact against the oracle, with quiet rows skipped."""
    n = 2048
    cfg = dict(fanout=4, seed=0x5EED0810)
    eng = gs.Engine(gs.default_config(n, **cfg))
    orc = oracle_mod.Oracle(oracle_mod.default_config(n, **cfg), threads=8)
    hb, ts, alive = sc.full_state(n)
    eng.import_state(hb, ts, alive, 0)
    orc.import_state(hb, ts, alive, 0)
    quiet, tiers = [], []
    for r in range(1, 61):
        if r == 48:
            ev = [(sc.JOIN, 5)]
            eng.apply_events(ev)
            orc.apply_events(ev)
        s1, s2 = eng.step(1), orc.step(1)
        assert s1 == s2, f"round {r}: gpu {s1} != cpu {s2}"
        quiet.append(eng.encoding_info(full=True)[4])
        tiers.append(eng.tier_info()[1])
        if r % 3 == 0 or r in (47, 48, 49):
            compare(eng, orc, r)
    assert max(quiet) > 0, quiet
    assert 0 in tiers and 1 in tiers, tiers


@pytest.mark.parametrize("world", [2, 3])
def test_tier_sharded_parity(gs, oracle_mod, world):
    """Column shards (in-process transport) each keep the tier of their own
    columns; seeded churn is bit-exact against the oracle every round."""
    from test_gpu_sharded import run_group
    n = 1100
    sched = sc.random_churn(n, 30, 0xB0 + world, p_crash=0.01, p_leave=0.01, p_join=0.03)
    run_group(gs, oracle_mod, world, dict(fanout=4, seed=0x5EED0410 + world, t_fail=9, t_cleanup=9), n, 30, sched,
              init=sc.full_state(n))


def test_tier_placement(gs, oracle_mod):
    """Placement and repair read the master / observer rows from 8-bit tables:
    churn with files, bit-exact against the oracle."""
    n = 640
    sched = {5: [(sc.CRASH, 3), (sc.CRASH, 200)], 12: [(sc.JOIN, 3)], 20: [(sc.LEAVE, 9)]}
    files = {r: np.arange(r * 40, r * 40 + 40) for r in (2, 8, 15, 24)}
    eng, orc = run_parity(gs, oracle_mod, dict(fanout=4, seed=0x5EED0910, t_fail=7, t_cleanup=7, max_files=2048),
                          n, 28, sched, init=sc.full_state(n), files=files)
    assert eng.tier_info()[0] == 1


def test_tier_plane_kept_across_events(gs, oracle_mod):
    """Crashes, a join and a datagram merge between rounds keep the sender
    plane valid (every chunk writer rewrites its plane word), so the round
    after them runs the byte path: only the rows the events touched go to the
    per-cell kernel. Bit-exact against the oracle every round."""
    n = 2048
    cfg = dict(fanout=4, seed=0x5EED0A10, t_fail=16, t_cleanup=16)
    eng = gs.Engine(gs.default_config(n, **cfg))
    orc = oracle_mod.Oracle(oracle_mod.default_config(n, **cfg), threads=8)
    hb, ts, alive = sc.full_state(n)
    eng.import_state(hb, ts, alive, 0)
    orc.import_state(hb, ts, alive, 0)
    # (a LEAVE tombstones its column in every row: the storm variant's case)
    sched = {10: [(sc.CRASH, 33), (sc.CRASH, 900)], 12: [(sc.JOIN, 33)]}
    slow_after = []
    for r in range(1, 16):
        ev = sched.get(r, [])
        if ev:
            eng.apply_events(ev)
            orc.apply_events(ev)
            assert eng.plane_info()[1] == 1, r  # still valid before the round
        if r == 11:
            ids = np.arange(0, n, 5, dtype=np.int32)
            vals = np.full(len(ids), 9, np.int32)
            assert eng.merge_list(7, ids, vals) == orc.merge_list(7, ids, vals)
            assert eng.plane_info()[1] == 1
        s1, s2 = eng.step(1), orc.step(1)
        assert s1 == s2, f"round {r}: gpu {s1} != cpu {s2}"
        compare(eng, orc, r)
        if r in (10, 11, 12):
            slow_after.append(eng.encoding_info()[1])
            assert eng.tier_info(full=True)[3] == 3, r  # the byte path ran
        assert eng.tier_info()[1] == 1, r
    # the rounds after the events list a few rows' segments, not the table
    segs = (n // 256) * n
    assert max(slow_after) < segs // 4, (slow_after, segs)


@pytest.mark.parametrize("case", ["wide_spread", "stale_outliers", "base_jump"])
def test_tier_wide_segments(gs, oracle_mod, case):
    """The 16-bit table's wide segments (heartbeats spread over millions,
    views stale by more than 1,022, base jumps by external lists) under the
    8-bit tier: their chunks are escaped, the per-cell kernel writes them into
    8-bit buffers, the rows narrow back into bytes; bit-exact against the
    oracle (tests/test_gpu_narrow.py's scenarios with the tier kept)."""
    import test_gpu_narrow as tn
    if case == "wide_spread":
        n = 300
        sched = sc.random_churn(n, 24, 103, p_crash=0.03, p_leave=0.01, p_join=0.04)
        wide0, _, slow = tn.run_cov(gs, oracle_mod, dict(fanout=4, seed=0x9103, t_fail=6, t_cleanup=8), n, 24, sched,
                                    tn.spread_state(n, 3))
        assert wide0 > 0 and slow > 0
    elif case == "stale_outliers":
        tn.test_stale_outliers(gs, oracle_mod, 257, 5)
    else:
        tn.test_base_jump_by_merge(gs, oracle_mod)


@pytest.mark.parametrize("t_cleanup", [3, 13, 16, 29, 30])
def test_tier_tombstones(gs, oracle_mod, t_cleanup):
    """Tombstones in the 4-bit tier (GH_TIER_TOMB, gh_internal.h gh_tier_toff):
    a tombstone's last 14 ages before release are tier cells (age nibble 1..14
    with the offset T_cleanup - 13, nibble 14 = released this round). Crashes,
    a LEAVE and a rejoin at N=2,048 with T_cleanup from below the offset's
    zero (3) to past the tier's range (30: no tombstone in the tier), so the
    offset is negative, zero, positive and absent; bit-exact every round."""
    n = 2048
    cfg = dict(fanout=4, seed=0x5EED0B10, t_fail=12, t_cleanup=t_cleanup)
    sched = {3: [(sc.CRASH, 17), (sc.CRASH, 900), (sc.CRASH, 1500)], 14: [(sc.LEAVE, 40)],
             30: [(sc.JOIN, 17)]}
    eng = gs.Engine(gs.default_config(n, **cfg))
    orc = oracle_mod.Oracle(oracle_mod.default_config(n, **cfg), threads=8)
    hb, ts, alive = sc.full_state(n)
    eng.import_state(hb, ts, alive, 0)
    orc.import_state(hb, ts, alive, 0)
    import ctypes as C
    eng.lib.gh_debug_tier.argtypes = [C.c_void_p, C.c_int32, C.c_int64, C.c_int64, C.c_void_p]
    nib = np.zeros(8, np.uint8)
    rel, tier_tombs, rel_variants, rel_jobs, trace = 0, 0, set(), [], []
    for r in range(1, 34 + t_cleanup // 2):
        ev = sched.get(r, [])
        if ev:
            eng.apply_events(ev)
            orc.apply_events(ev)
        s1, s2 = eng.step(1), orc.step(1)
        assert s1 == s2, f"round {r}: gpu {s1} != cpu {s2}"
        rel += s1["released"]
        compare(eng, orc, r)
        # a pure release round: no detection wave, no events, before the
        # rejoin at r=30 (whose column's base jump makes its lanes jobs)
        if s1["released"] and r > 3 and not s1["detections"] and not s1["tombstoned"] and r < 30 and r not in sched:
            rel_variants.add(eng.tier_info(full=True)[3])
            rel_jobs.append(eng.job_info()[0])
        trace.append((r, s1["released"], s1["detections"], s1["tombstoned"], eng.tier_info(full=True)[3], eng.job_info()[0]))
        # the crashed members' columns in a few rows: a tier tombstone is
        # lag code 15 with an age nibble 1..14 (gh_debug_tier)
        for row in (0, 511, 1023, 2047):
            for col in (17, 40, 900, 1500):  # the crashed members and the leaver
                assert eng.lib.gh_debug_tier(eng.h, row, col & ~7, 8, nib.ctypes.data_as(C.c_void_p)) == 0
                v = int(nib[col & 7])
                tier_tombs += v != 0xFF and (v >> 4) == 15 and 1 <= (v & 15) <= 14
    assert rel > 0
    assert eng.tier_info()[0] == 1
    # rounds that released tombstones ran the nibble path, with few lane jobs
    # (the tombstones age and release inside it, not as jobs)
    assert rel_variants <= {3}, trace
    assert max(rel_jobs, default=0) * 100 <= n * n // 16, rel_jobs
    if t_cleanup < 30:  # the tier holds tombstones (gh_tier_toff)
        assert tier_tombs > 0
    else:
        assert tier_tombs == 0


def remove_run(gs, om, n, cfg, sched, rounds, world=1, layout=0, check=True):
    """Runs the crash wave; returns per round (stats, tier variant, lane
    jobs) and, for one engine, the final exported state."""
    if world > 1:
        eng = gs.ShardGroup(gs.default_config(n, shard_layout=layout, **cfg), world)
    else:
        eng = gs.Engine(gs.default_config(n, **cfg))
    orc = om.Oracle(om.default_config(n, **cfg), threads=8) if check else None
    hb, ts, alive = sc.full_state(n)
    eng.import_state(hb, ts, alive, 0)
    if orc:
        orc.import_state(hb, ts, alive, 0)
    trace = []
    try:
        for r in range(1, rounds + 1):
            ev = sched.get(r, [])
            if ev:
                eng.apply_events(ev)
                if orc:
                    orc.apply_events(ev)
            s1 = eng.step(1)
            if orc:
                s2 = orc.step(1)
                assert s1 == s2, f"round {r}: gpu {s1} != cpu {s2}"
                compare(eng, orc, r)
            var, jobs = (eng.tier_info(full=True)[3], eng.job_info()[0]) if world == 1 else (None, None)
            trace.append((s1, var, jobs))
        final = eng.export_state() if world == 1 else None
    finally:
        eng.close()
        if orc:
            orc.close()
    return trace, final


@pytest.mark.parametrize("case", ["canonical", "quirk", "t_cleanup20", "cols2", "rows3"])
def test_tier_remove_on_nibble_path(gs, oracle_mod, monkeypatch, case):
    """REMOVE delivery on the nibble path (round.hip nib_word RMV,
    slave/slave.go:236-240, 276-286, 338-363): a 1% crash wave at N=2,048
    with T_fail = 16 and T_cleanup >= 15, bit-exact against the oracle every
    round. In the REMOVE rounds the REMOVE'd members' present cells become
    tier tombstones inside the nibble path: one engine runs it (variant 3)
    with at most a quarter of the lane jobs GH_NIB_RMV=0 (every lane holding a
    REMOVE'd member a job) leaves, and both give the same tables and
    counters. Quirk detection, an age offset of 7 (T_cleanup 20), 2 column
    shards and 3 row shards run the same wave."""
    n = 2048
    t_cleanup = 20 if case == "t_cleanup20" else 16
    cfg = dict(fanout=4, seed=0x5EED0C10, t_fail=16, t_cleanup=t_cleanup, detect_mode=1 if case == "quirk" else 0)
    crashed = sc.crash_ids(n, 0.01, 0x5EED0C11)
    sched = {8: [(sc.CRASH, int(c)) for c in crashed]}
    rounds = 34
    world, layout = {"cols2": (2, 0), "rows3": (3, 1)}.get(case, (1, 0))
    trace, final = remove_run(gs, oracle_mod, n, cfg, sched, rounds, world, layout)
    tomb_rounds = [r for r, (s, _, _) in enumerate(trace, 1) if s["tombstoned"]]
    assert tomb_rounds, trace
    if world > 1:
        return
    # the REMOVE rounds ran the nibble path, with few lane jobs
    assert all(trace[r - 1][1] == 3 for r in tomb_rounds), [(r, trace[r - 1]) for r in tomb_rounds]
    monkeypatch.setenv("GH_NIB_RMV", "0")
    off, final_off = remove_run(gs, oracle_mod, n, cfg, sched, rounds, check=False)
    for r, (a, b) in enumerate(zip(trace, off), 1):
        assert a[0] == b[0], (r, a[0], b[0])
    for x, y in zip(final, final_off):
        np.testing.assert_array_equal(x, y)
    on_jobs = sum(trace[r - 1][2] for r in tomb_rounds)
    off_jobs = sum(off[r - 1][2] for r in tomb_rounds)
    assert on_jobs * 4 <= off_jobs, (on_jobs, off_jobs, [(r, trace[r - 1][2], off[r - 1][2]) for r in tomb_rounds])


@pytest.mark.parametrize("case", ["steady_crash", "remove_quirk"])
def test_tier_lds_dma_staging(gs, oracle_mod, monkeypatch, case):
    """The nibble path with its lines staged by LDS-DMA (GH_NIB_DMA=1,
    round.hip round_block_nib DMA: buffer_load_dwordx4 ... lds, 8 rows per
    wave step) at N=2,048, k=4, T_fail=16: a crash wave with its detection,
    REMOVE and release rounds (canonical, then quirk detection), bit-exact
    against the oracle every round, the nibble path in the healthy rounds."""
    monkeypatch.setenv("GH_NIB_DMA", "1")
    n = 2048
    cfg = dict(fanout=4, seed=0x5EED0D10, t_fail=16, t_cleanup=16, detect_mode=1 if case == "remove_quirk" else 0)
    crashed = sc.crash_ids(n, 0.01, 0x5EED0D11)
    sched = {8: [(sc.CRASH, int(c)) for c in crashed], 30: [(sc.JOIN, int(crashed[0]))]}
    trace, _ = remove_run(gs, oracle_mod, n, cfg, sched, 36)
    assert sum(v == 3 for _, v, _ in trace) >= 30, trace
    assert any(s["tombstoned"] for s, _, _ in trace)


@pytest.mark.parametrize("env", [("GH_ROUND_XMAP", "2"), ("GH_NIB_RMV", "2")])
def test_tier_nibble_variants(gs, oracle_mod, monkeypatch, env):
    """Two nibble-path options on the crash wave of test_tier_lds_dma_staging,
    bit-exact against the oracle every round: GH_ROUND_XMAP=2 (odd rounds
    sweep the tiles from the other end, round.hip nib_region; the lane jobs
    walk the same regions) and GH_NIB_RMV=2 (the REMOVE-taking
    instantiation, k_round IN 6, in every round instead of only the rounds
    after a detection)."""
    monkeypatch.setenv(*env)
    n = 2048
    cfg = dict(fanout=4, seed=0x5EED0D20, t_fail=16, t_cleanup=16)
    crashed = sc.crash_ids(n, 0.01, 0x5EED0D21)
    sched = {8: [(sc.CRASH, int(c)) for c in crashed], 30: [(sc.JOIN, int(crashed[0]))]}
    trace, _ = remove_run(gs, oracle_mod, n, cfg, sched, 36)
    assert sum(v == 3 for _, v, _ in trace) >= 30, trace
    assert any(s["tombstoned"] for s, _, _ in trace)


@pytest.mark.parametrize("tmode", ["0", "1"])
def test_round_timing_modes(gs, monkeypatch, tmode):
    """gh_read_timing (the bench's k_round time): with GH_TMODE=1 only the
    nibble launch carries its own HIP events, the other variants are timed
    together and the device logs which variant ran (vlog); GH_TMODE=0 times
    every launch. Through a crash wave at N=2,048 (nibble, storm-free REMOVE
    and release rounds) every round is counted once with a positive time, and
    the nibble rounds' times agree between the modes within a factor 3."""
    monkeypatch.setenv("GH_TMODE", tmode)
    n = 2048
    cfg = gs.default_config(n, fanout=4, seed=0x5EED0D30, t_fail=16, t_cleanup=16)
    crashed = sc.crash_ids(n, 0.01, 0x5EED0D31)
    eng = gs.Engine(cfg)
    try:
        hb, ts, alive = sc.full_state(n)
        eng.import_state(hb, ts, alive, 0)
        eng.set_timing(True)
        prev, per = 0.0, []
        for r in range(1, 41):
            if r == 8:
                eng.apply_events([(sc.CRASH, int(c)) for c in crashed])
            eng.step(1)
            ms, launches = eng.read_timing()
            assert launches == r
            assert ms > prev, (r, ms, prev)
            per.append((eng.tier_info(full=True)[3], ms - prev))
            prev = ms
        eng.set_timing(True)
        eng.step(10)  # several rounds in one call
        ms, launches = eng.read_timing()
        assert launches == 10 and ms > 0
    finally:
        eng.close()
    nib = [t for v, t in per[1:] if v == 3]
    assert len(nib) >= 30
    med = sorted(nib)[len(nib) // 2]
    assert all(t < 3 * med + 0.5 for t in nib), (med, nib)
