"""GPU parity at the headline configuration (BASELINE config 3, SURVEY §8d
C3): N=65,536 members, k=4 Philox pull, full-membership start (hb=2, ts=0),
seed 0x5EED0003 — the HIP path against the CPU oracle (oracle/tablesim.c,
48 GiB of host tables, OpenMP on the box's host cores), bit for bit.

Two regimes:
  * the bench's healthy steady state (T_fail = T_cleanup = 16 rounds);
  * the reference's own PERIOD = COOLDOWN = 5 s (slave/slave.go:24-25): the
    round-6 detection storm, the REMOVE wave and the round-7 collapse under
    the <4 guard (slave/slave.go:460-497, 504-509), which runs k_round's
    storm variant at full scale.

  * the bench's steady state with a 1% crash (BASELINE config 2's crash rate
    at the config-3 size): 655 Philox-drawn members stop at r=8; they are
    detected once their views age past T_fail (slave/slave.go:460-482), the
    REMOVE wave follows (:338-363) and the tombstones age out (:484-497).

Counters, the failed set and the detectors are compared every round; the
whole hb and ts tables (65,536 x 65,536 each) row block by row block at the
rounds listed. The steady-state test also asserts, from round 8 on, that the
round ran the nibble path (gh_tier_info variant 3) with at most one in a
million lanes handed to the lane-job kernel: the path the bench times is the
path checked here. The crash case runs on the nibble path and its lane jobs
throughout (no storm round)."""
import os
import time

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

N = 65536
BLOCK = 4096
THREADS = int(os.environ.get("GH_ORACLE_THREADS", "16"))


@pytest.fixture(scope="module")
def gs():
    import gossipsim
    return gossipsim


def shard_sample(n=N, g=8, nb=256):
    """Row ranges for a sharded group's bit-for-bit table check: the first
    rows and nb rows across each of the g - 1 inner shard boundaries (a
    group's export assembles every row on every rank and takes ~80 s for the
    whole N=65,536 table; this sample takes ~3 s)."""
    out = [(0, nb)]
    for k in range(1, g):
        out.append((k * (n // g) - nb // 2, nb))
    return out


def compare_blocks(engs, orc, r, n=N):
    """full hb / ts tables and alive vector of every single engine against
    the oracle's row block by row block, and of every ShardGroup the rows of
    shard_sample (the oracle block exported once per range)"""
    t0 = time.perf_counter()
    full = [(row0, min(BLOCK, n - row0)) for row0 in range(0, n, BLOCK)]
    sample = shard_sample(n)
    for row0, nb in sorted(set(full) | set(sample)):
        who = [(name, eng) for name, eng in engs
               if ((row0, nb) in sample if hasattr(eng, "engines") else (row0, nb) in full)]
        if not who:
            continue
        h2, t2, a2 = orc.export_state(row0, nb)
        for name, eng in who:
            if hasattr(eng, "engines"):  # a ShardGroup: every rank assembles the same rows; rank 0's copy
                h1, t1, a1 = eng.run("export_state", row0, nb)[0]
            else:
                h1, t1, a1 = eng.export_state(row0, nb)
            np.testing.assert_array_equal(a1, a2, err_msg=f"{name}: alive r={r} rows {row0}+")
            if not np.array_equal(h1, h2):
                bad = np.argwhere(h1 != h2)
                i, c = bad[0]
                raise AssertionError(f"{name}: hb r={r}: {len(bad)} cells differ in rows {row0}+, first "
                                     f"({row0 + i}, {c}) gpu={h1[i, c]} cpu={h2[i, c]}")
            if not np.array_equal(t1, t2):
                bad = np.argwhere(t1 != t2)
                i, c = bad[0]
                raise AssertionError(f"{name}: ts r={r}: {len(bad)} cells differ in rows {row0}+, first "
                                     f"({row0 + i}, {c}) gpu={t1[i, c]} cpu={t2[i, c]} hb={h2[i, c]}")
    names = "/".join(nm + (" (sampled rows)" if hasattr(e, "engines") else "") for nm, e in engs)
    print(f"  r={r}: tables equal, {names} ({time.perf_counter() - t0:.1f} s)", flush=True)


LAYOUT_NAMES = {(1, 0): "single", (8, 0): "columns_g8", (8, 1): "rows_g8"}


class Lockstep:
    """One engine (or G in-process shards of layout `layout`) and tablesim
    stepped round by round from the full-membership start; `lockstep` adds
    more (world, layout) groups stepped beside it against the SAME oracle
    run (one 48 GiB tablesim pass checks every layout). advance(r) runs to
    round r, checking counters, failed sets and detectors of every engine
    each round and full tables at the rounds in full_at (of the engines in
    full_all, else only the first); per_round / after_round see the first
    engine. A test can advance in parts, so that no single test runs longer
    than a few minutes without reporting."""

    def __init__(self, gs, om, t_fail, full_at=(), sched=None, per_round=None, remove_mode=0, world=1, layout=0,
                 extra=None, after_round=None, lockstep=(), full_all=None):
        cfg = dict(fanout=4, seed=0x5EED0003, t_fail=t_fail, t_cleanup=t_fail, remove_mode=remove_mode,
                   **(extra or {}))
        self.engs, self.orc = [], None
        self.sched, self.per_round, self.after_round = sched or {}, per_round, after_round
        self.world = world
        self.full_at, self.full_all = set(full_at), full_all
        self.r = 0
        self.seen = {"detections": 0, "storm": False, "variants": {}, "first_detection": None}
        try:
            for w, lay in ((world, layout),) + tuple(lockstep):
                if w > 1:  # G in-process shards of one cluster on this GPU (GH_COMM_LOCAL)
                    e = gs.ShardGroup(gs.default_config(N, shard_layout=lay, **cfg), w)
                else:
                    e = gs.Engine(gs.default_config(N, **cfg))
                self.engs.append((LAYOUT_NAMES.get((w, lay), f"g{w}l{lay}"), e))
            self.orc = om.Oracle(om.default_config(N, **cfg), threads=THREADS)
            for _, e in self.engs:
                e.init_full(2, 0, 0)
            self.orc.init_full(2, 0, 0)
        except BaseException:
            self.close()
            raise

    def advance(self, to_r):
        eng, orc, seen = self.engs[0][1], self.orc, self.seen
        while self.r < to_r:
            r = self.r = self.r + 1
            if r in self.sched:
                for _, e in self.engs:
                    e.apply_events(self.sched[r])
                orc.apply_events(self.sched[r])
            t0 = time.perf_counter()
            s2 = orc.step(1)
            t1 = time.perf_counter()
            ms = []
            for name, e in self.engs:
                ta = time.perf_counter()
                s1 = e.step(1)
                ms.append(f"{name} {1e3 * (time.perf_counter() - ta):.1f} ms")
                assert s1 == s2, f"{name} round {r}: gpu {s1} != cpu {s2}"
                np.testing.assert_array_equal(e.read_failed(), orc.read_failed(), err_msg=f"{name}: failed r={r}")
                np.testing.assert_array_equal(e.read_detectors(), orc.read_detectors(),
                                              err_msg=f"{name}: detectors r={r}")
            print(f"  r={r}: oracle {t1 - t0:.1f} s, gpu {', '.join(ms)}, {s2}", flush=True)
            seen["detections"] += s2["detections"]
            if self.world == 1:  # (per-shard diagnostics differ between shards)
                seen["storm"] |= eng.encoding_info(full=True)[2] == 1
                var = eng.tier_info(full=True)[3]
                seen["variants"][var] = seen["variants"].get(var, 0) + 1
            if self.after_round:
                self.after_round(eng, orc, r)
            if self.per_round:
                self.per_round(eng, r, s2)
            if s2["detections"] and seen["first_detection"] is None:
                seen["first_detection"] = r
                if self.full_all is None:
                    self.full_at |= {r, r + 1}  # the detection round and the REMOVE round after it
            if r in self.full_at:
                all_ = self.full_all is None or r in self.full_all
                compare_blocks(self.engs if all_ else self.engs[:1], orc, r)
        return seen

    def close(self):
        for _, e in self.engs:
            e.close()
        self.engs = []
        if self.orc is not None:
            self.orc.close()
            self.orc = None


def run(gs, om, t_fail, rounds, full_at, expect, **kw):
    ls = Lockstep(gs, om, t_fail, full_at, **kw)
    try:
        seen = ls.advance(rounds)
        print(f"  variants (round counts by gh_tier_info variant): {seen['variants']}", flush=True)
        expect(seen)
    finally:
        ls.close()


def byte_path_from(r0, r_var=None):
    """per-round check: from round r_var (default r0) on, the round ran the
    nibble path (tier variant 3); from round r0 on, the lanes it handed to the
    lane-job kernel and the chunks written escaped also stay below one in a
    million (stragglers: a view not refreshed for 16 rounds leaves the tier's
    15-round age window; the job kernel writes it escaped, bit-exact)"""
    r_var = r0 if r_var is None else r_var

    def check(eng, r, st):
        kept, current, escaped, variant = eng.tier_info(full=True)
        if r >= r_var:
            assert (kept, current, variant) == (1, 1, 3), f"round {r}: tier_info {kept, current, escaped, variant}"
        if r >= r0:
            jobs, redo = eng.job_info()
            n = eng.cfg.n_members
            assert escaped * 10**6 <= n * n // 8 and jobs * 10**6 <= n * n // 16 and redo == 0, \
                f"round {r}: {escaped} escaped chunks, {jobs} lane jobs, {redo} redos"
    return check


def test_c3_fullsize_steady_state(gs, oracle_mod):
    """The bench's workload (T_fail = 16) through the rounds the bench times
    (the driver's --warmup 5 --steps 20 covers rounds 6-25): no detections,
    full tables equal at r = 6, 12 and 25, the nibble path in every timed
    round (from round 6), with its lane jobs below one in a million lanes from
    round 8."""
    run(gs, oracle_mod, 16, 25, {6, 12, 25}, lambda s: s["detections"] == 0 or pytest.fail("unexpected detections"),
        per_round=byte_path_from(8, r_var=6))


@pytest.fixture(scope="module")
def crash_lockstep(gs, oracle_mod):
    """1% crash in the bench's workload: 655 members (Philox, seed
    0x5EED0003, tag CRASH) stop at r=8; detected at r=23, REMOVE'd at r=24.
    Three layouts in lockstep against the one tablesim run: one engine,
    north_star's 8 row shards (each owns 8,192 observer rows; the other
    shards' sender plane rows arrive by alltoallv into its ghost table) and 8
    column shards (O(N) exchanges), all on this GPU through the in-process
    transport (~150 GB of HBM). Counters, failed sets and detectors of all
    three every round; at the detection round, the round after it and the
    last round the engine's full tables and the shard groups' rows around
    every shard boundary (shard_sample). Advanced by the four tests below in
    order; the last one frees the ~150 GB of HBM."""
    from scenarios import crash_ids
    crashed = crash_ids(N, 0.01, 0x5EED0003)
    assert len(crashed) == 655
    sched = {8: [(gs.GH_EV_CRASH, int(c)) for c in crashed]}

    def fast(eng, r, st):
        # the crash wave stays on the nibble path: REMOVE delivery turns the
        # removed members' cells into tier tombstones inside it (round.hip
        # nib_word RMV), so no round hands more than 1% of the lanes to the
        # lane-job kernel (round 4: 38 M = 14% in the REMOVE round)
        if r >= 6:
            assert eng.tier_info(full=True)[3] == 3, (r, eng.tier_info(full=True))
            jobs, _ = eng.job_info()
            assert jobs * 100 <= N * N // 16, (r, jobs)

    ls = Lockstep(gs, oracle_mod, 16, {23, 24, 32}, sched=sched, per_round=fast, lockstep=((8, 1), (8, 0)),
                  full_all={23, 24, 32})
    yield ls
    ls.close()


def test_c3_fullsize_crash_1pct(crash_lockstep):
    """Rounds 1-16 of the crash (crash_lockstep): the crash at r=8."""
    s = crash_lockstep.advance(16)
    assert s["detections"] == 0


def test_c3_fullsize_crash_1pct_detection(crash_lockstep):
    """Rounds 17-23: the crashed members' views age past T_fail, the
    detection round; tables of all three layouts at r=23."""
    s = crash_lockstep.advance(23)
    assert s["first_detection"] == 23, s


def test_c3_fullsize_crash_1pct_remove(crash_lockstep):
    """Round 24: the REMOVE wave of the 655 members; tables of all three
    layouts."""
    crash_lockstep.advance(24)


def test_c3_fullsize_crash_1pct_release(crash_lockstep):
    """Rounds 25-32: tombstones age out; tables of all three layouts at
    r=32. Frees the three groups' HBM for the tests after it."""
    try:
        s = crash_lockstep.advance(32)
        assert s["detections"] > 0
    finally:
        crash_lockstep.close()


@pytest.mark.gpu_fullsize
def test_c3_fullsize_crash_1pct_remove_list(gs, oracle_mod):
    """The 1% crash with the reference's REMOVE recipients (GH_REMOVE_LIST:
    each detector's list right after removeMember, slave/slave.go:344,
    472-473): the recipient sets of all 655 crashed members are decided at
    full size (remove.hip) and the REMOVE wave matches tablesim's literal
    per-detector restatement."""
    from scenarios import crash_ids
    crashed = crash_ids(N, 0.01, 0x5EED0003)
    sched = {8: [(gs.GH_EV_CRASH, int(c)) for c in crashed]}

    def expect(s):
        assert s["detections"] > 0 and s["first_detection"] is not None, s

    run(gs, oracle_mod, 16, 28, {28}, expect, sched=sched, remove_mode=1)


@pytest.mark.gpu_fullsize
def test_c3_fullsize_reference_timeouts(gs, oracle_mod):
    """T_fail = T_cleanup = 5 (slave/slave.go:24-25) through the round-6
    detection storm and the collapse: the storm variant runs at N=65,536."""
    def expect(s):
        assert s["detections"] > 0 and s["storm"]
    run(gs, oracle_mod, 5, 9, {6, 7, 9}, expect)


def crash_sched(gs):
    from scenarios import crash_ids
    crashed = crash_ids(N, 0.01, 0x5EED0003)
    return {8: [(gs.GH_EV_CRASH, int(c)) for c in crashed]}


def expect_detection(s):
    assert s["detections"] > 0 and s["first_detection"] is not None, s


@pytest.mark.gpu_fullsize
def test_c3_fullsize_crash_1pct_quirk(gs, oracle_mod):
    """Quirk-mode detection (Go's range over the slice removeMember shifts,
    slave/slave.go:464-477) through the 1% crash at N=65,536: the crashed
    members' runs of candidates in every row, the skipped ones detected a
    round later."""
    run(gs, oracle_mod, 16, 28, {28}, expect_detection, sched=crash_sched(gs), extra=dict(detect_mode=1))


@pytest.mark.gpu_fullsize
def test_c5_fullsize_files(gs, oracle_mod):
    """SURVEY C5's shape at N=65,536 with 2^20 files (master/master.go:74-175):
    every file put at r=3 (Init_replica over the master's list), a 1% crash
    wave at r=4, 1% leaves at r=8, the r=4 crashed members rejoining at r=12,
    re-replication from the first detectors' views at detection + 8
    (Fail_recover, slave/slave.go:1122-1133), then Get_file_replica_list /
    Get_file_version of every file."""
    from scenarios import crash_ids
    F = 1 << 20
    crashed = crash_ids(N, 0.01, 0x5EED0005)
    leavers = [c for c in crash_ids(N, 0.02, 0x5EED0006) if c not in set(crashed)][: N // 100]
    sched = {4: [(gs.GH_EV_CRASH, int(c)) for c in crashed],
             8: [(gs.GH_EV_LEAVE, int(c)) for c in leavers],
             12: [(gs.GH_EV_JOIN, int(c)) for c in crashed]}
    files = np.arange(F, dtype=np.int32)
    repair_at = {}

    def after_round(eng, orc, r):
        if r == 3:
            a, b = eng.put(files), orc.put(files)
            for x, y in zip(a, b):
                np.testing.assert_array_equal(x, y)
        dets = orc.read_detectors()
        if len(dets) and r + 8 not in repair_at:
            repair_at[r + 8] = [int(x) for x in dets[:2]]
        for obs in repair_at.get(r, []):
            pa, pb = eng.repair(obs), orc.repair(obs)
            assert pa == pb, f"repair at r={r} from {obs}: {len(pa)} vs {len(pb)} plan entries"
            print(f"  r={r}: repair from {obs}: {len(pa)} plan entries equal", flush=True)
        if r == 40:
            for x, y in zip(eng.get_files(files), orc.get_files(files)):
                np.testing.assert_array_equal(x, y)
            print("  r=40: get_files of 2^20 files equal", flush=True)

    run(gs, oracle_mod, 16, 40, {40}, expect_detection, sched=sched, extra=dict(max_files=F),
        after_round=after_round)


@pytest.mark.gpu_fullsize
def test_c3_fullsize_reference_timeouts_remove_list_timed(gs):
    """GH_REMOVE_LIST (the reference's REMOVE recipients, csrc/remove.hip)
    through the reference timeouts' detection storm at N=65,536, timed: the
    round-6 storm detects nearly every cell, so D_r holds nearly every member
    with nearly every row as a detector -- the worst case of the recipient
    decision (k_rm_recv: counts and the pigeonhole rule settle the pairs,
    the nonzero words of det(c) the rest). Every round must finish within 5 s
    (ADVICE round 4); the engine runs alone (tablesim's literal recipients
    are O(|det(c)| * N / 32) per member, hours in a storm of this size), and
    the rounds up to the storm equal the D4 engine's counters (the two rules
    only part once a REMOVE is delivered)."""
    cfg = dict(fanout=4, seed=0x5EED0003, t_fail=5, t_cleanup=5)
    lit = gs.Engine(gs.default_config(N, remove_mode=1, **cfg))
    d4 = gs.Engine(gs.default_config(N, **cfg))
    try:
        lit.init_full(2, 0, 0)
        d4.init_full(2, 0, 0)
        storm = False
        for r in range(1, 13):
            t0 = time.perf_counter()
            s1 = lit.step(1)
            ms = 1e3 * (time.perf_counter() - t0)
            s2 = d4.step(1)
            print(f"  r={r}: literal REMOVE {ms:.1f} ms, {s1}", flush=True)
            assert ms < 5000, f"round {r}: {ms:.0f} ms"
            storm |= s1["detections"] > N * N // 4
            if r <= 6:  # before the first REMOVE delivery
                assert s1 == s2, (r, s1, s2)
        assert storm
    finally:
        lit.close()
        d4.close()


# ---- beyond N = 65,536 -------------------------------------------------------
# Every other test stays at N <= 65,536. These two run what only larger
# clusters reach: ring receivers with more than 65,535 senders, and a single
# engine plus 8 column shards at N = 131,072 (config 4's per-GPU column count
# is 32,768 of 262,144 rows; this is the largest N one MI355X holds twice).


def _mix(i, c):
    """a fixed spread of heartbeats 2..18 per (row, member) cell"""
    h = (i.astype(np.uint32) * np.uint32(0x9E3779B1)) ^ (c.astype(np.uint32) * np.uint32(0x85EBCA77))
    h ^= h >> np.uint32(15)
    return (2 + (h % np.uint32(17))).astype(np.int32)


def test_ring_receiver_65537_senders(gs, oracle_mod):
    """Ring mode at N = 65,600 with rows 1..65,537 holding every member but
    themselves: a sender whose own cell is absent sends to list[len-2],
    list[0] and list[1] (self index -1 in slave/slave.go:515-524), so member
    0 receives from 65,537 senders, member 1 from 65,536 and member 65,598
    from 65,537. The kernels pack a receiver's sender count into the row
    record (round.hip nmeta / s_meta, bits 2..29); a 16-bit unpack had read
    these counts as 1, 0 and 1, merged at most one sender and skipped
    k_round_slow. Two rounds against tablesim: counters every round, the
    many-sender rows at round 1, the full tables at round 2."""
    n = 65600
    nabs = 65537  # rows 1..nabs have their own cell absent
    cfg = dict(fanout=4, seed=0x5EED0007, t_fail=16, t_cleanup=16, peer_mode=gs.GH_PEER_RING)
    eng = gs.Engine(gs.default_config(n, **cfg))
    orc = oracle_mod.Oracle(oracle_mod.default_config(n, **cfg), threads=THREADS)
    try:
        cols = np.arange(n, dtype=np.int64)
        alive = np.ones(BLOCK, np.uint8)
        for row0 in range(0, n, BLOCK):
            nb = min(BLOCK, n - row0)
            rows = np.arange(row0, row0 + nb, dtype=np.int64)
            hb = _mix(rows[:, None], cols[None, :])
            hb[rows == 0, :] = 2  # the receiver starts low: every sender's view beats it
            own = (rows >= 1) & (rows <= nabs)
            hb[np.nonzero(own)[0], rows[own]] = -1
            ts = np.zeros_like(hb)
            eng.import_state(hb, ts, alive[:nb], 0, row0)
            orc.import_state(hb, ts, alive[:nb], 0, row0)
        print("  imported", flush=True)
        for r in (1, 2):
            t0 = time.perf_counter()
            s2 = orc.step(1)
            t1 = time.perf_counter()
            s1 = eng.step(1)
            print(f"  r={r}: oracle {t1 - t0:.1f} s, gpu {1e3 * (time.perf_counter() - t1):.1f} ms, {s2}", flush=True)
            assert s1 == s2, f"round {r}: gpu {s1} != cpu {s2}"
            np.testing.assert_array_equal(eng.read_failed(), orc.read_failed())
            if r == 1:
                for i in (0, 1, 2, n - 2, n - 1):
                    a, b = eng.export_state(i, 1), orc.export_state(i, 1)
                    for x, y in zip(a, b):
                        np.testing.assert_array_equal(x, y, err_msg=f"row {i} r=1")
                h0 = orc.export_state(0, 1)[0][0]
                # the max over 65,537 senders' views: 18 nearly everywhere (one sender: ~10 on average)
                assert (h0 == 18).mean() > 0.99, np.bincount(h0[h0 >= 0])
        compare_blocks([("single", eng)], orc, 2, n=n)
    finally:
        eng.close()
        orc.close()


def _single_vs_group(gs, n, layout, world, seed):
    """One engine and `world` in-process shards of layout `layout` of the same
    N-member cluster (k = 4 pull, T_fail = 16) in lockstep: 12 healthy
    rounds (properties of any size: every member stays everywhere, the own
    heartbeat advances one per round, no view runs ahead of its owner, the
    epidemic reaches every cell, the nibble path runs), then a 1% crash
    detected everywhere; the group's counters, failed sets and detectors
    equal the engine's every round, sampled rows bit for bit."""
    from scenarios import crash_ids
    rounds = 12
    cfg = dict(fanout=4, seed=seed, t_fail=16, t_cleanup=16)
    one = gs.Engine(gs.default_config(n, **cfg))
    grp = None
    try:
        grp = gs.ShardGroup(gs.default_config(n, shard_layout=layout, **cfg), world)
        sample = (0, 1, 4095, n // 2 - 1, n // 2, n - 2, n - 1)

        def same_rows(r):
            for i in sample:
                a, b = one.export_state(i, 1), grp.run("export_state", i, 1)[0]
                for x, y in zip(a, b):
                    np.testing.assert_array_equal(x, y, err_msg=f"row {i} r={r}")

        one.init_full(2, 0, 0)
        grp.init_full(2, 0, 0)
        merged = 0
        for r in range(1, rounds + 1):
            t0 = time.perf_counter()
            s1 = one.step(1)
            t1 = time.perf_counter()
            s2 = grp.step(1)
            print(f"  r={r}: engine {1e3 * (t1 - t0):.1f} ms, {world} shards {1e3 * (time.perf_counter() - t1):.1f} ms, "
                  f"{s1}", flush=True)
            assert s1 == s2, (r, s1, s2)
            assert s1["detections"] == 0 and s1["active_rows"] == n
            merged += s1["merged_cells"]
        assert merged > n * n  # the epidemic has reached every cell
        assert one.tier_info(full=True)[3] == 3  # the nibble path at this size
        same_rows(rounds)
        for i in sample:
            hb, ts, _ = one.export_state(i, 1)
            assert hb[0, i] == 2 + rounds
            assert (hb[0] >= 2).all() and (hb[0] <= 2 + rounds).all()
            assert (ts[0] <= rounds).all()
        crashed = crash_ids(n, 0.01, seed)
        ev = [(gs.GH_EV_CRASH, int(c)) for c in crashed]
        one.apply_events(ev)
        grp.apply_events(ev)
        seen = set()
        for r in range(rounds + 1, rounds + 41):
            s1, s2 = one.step(1), grp.step(1)
            assert s1 == s2, (r, s1, s2)
            bm = one.read_failed()
            np.testing.assert_array_equal(bm, grp.read_failed(), err_msg=f"failed r={r}")
            np.testing.assert_array_equal(one.read_detectors(), grp.read_detectors(), err_msg=f"detectors r={r}")
            seen |= {int(c) for c in crashed if bm[c >> 5] >> (c & 31) & 1}
            if s1["detections"]:
                print(f"  r={r}: {s1}", flush=True)
        assert seen == {int(c) for c in crashed}
        same_rows(rounds + 40)
    finally:
        if grp is not None:
            grp.close()
        one.close()


def test_n98304_single_vs_rows_g8(gs):
    """North_star's layout above N=65,536: N = 98,304, one engine (73 GB)
    and 8 in-process row shards (12,288 observer rows each, the other
    shards' sender plane rows by alltoallv into ghost tables; 166 GB) on this
    GPU, in lockstep through the healthy rounds and a 1% crash
    (_single_vs_group). The largest N at which one MI355X holds both."""
    _single_vs_group(gs, 98304, 1, 8, 0x5EED0008)


def test_n131072_single_vs_columns_g8(gs):
    """N = 131,072, k = 4 pull, T_fail = 16: one engine (~130 GB) and 8
    in-process column shards of the same cluster (~130 GB) on this GPU in
    lockstep (_single_vs_group) -- the sizes where a (row, 128-B line)
    offset no longer fits 31 bits in a (row x ld / 8) word index."""
    _single_vs_group(gs, 131072, 0, 8, 0x5EED0004)
