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


def compare_blocks(eng, orc, r):
    t0 = time.perf_counter()
    for row0 in range(0, N, BLOCK):
        h1, t1, a1 = eng.export_state(row0, BLOCK)
        h2, t2, a2 = orc.export_state(row0, BLOCK)
        np.testing.assert_array_equal(a1, a2, err_msg=f"alive r={r} rows {row0}+")
        if not np.array_equal(h1, h2):
            bad = np.argwhere(h1 != h2)
            i, c = bad[0]
            raise AssertionError(f"hb r={r}: {len(bad)} cells differ in rows {row0}+, first ({row0 + i}, {c}) "
                                 f"gpu={h1[i, c]} cpu={h2[i, c]}")
        if not np.array_equal(t1, t2):
            bad = np.argwhere(t1 != t2)
            i, c = bad[0]
            raise AssertionError(f"ts r={r}: {len(bad)} cells differ in rows {row0}+, first ({row0 + i}, {c}) "
                                 f"gpu={t1[i, c]} cpu={t2[i, c]} hb={h2[i, c]}")
    print(f"  r={r}: full tables equal ({time.perf_counter() - t0:.1f} s)", flush=True)


def run(gs, om, t_fail, rounds, full_at, expect, sched=None, per_round=None, remove_mode=0, world=1, layout=0,
        extra=None, after_round=None):
    cfg = dict(fanout=4, seed=0x5EED0003, t_fail=t_fail, t_cleanup=t_fail, remove_mode=remove_mode, **(extra or {}))
    if world > 1:  # G in-process shards of one cluster on this GPU (GH_COMM_LOCAL)
        eng = gs.ShardGroup(gs.default_config(N, shard_layout=layout, **cfg), world)
    else:
        eng = gs.Engine(gs.default_config(N, **cfg))
    orc = om.Oracle(om.default_config(N, **cfg), threads=THREADS)
    try:
        eng.init_full(2, 0, 0)
        orc.init_full(2, 0, 0)
        seen = {"detections": 0, "storm": False, "variants": {}, "first_detection": None}
        pending_full = set(full_at)
        for r in range(1, rounds + 1):
            if sched and r in sched:
                eng.apply_events(sched[r])
                orc.apply_events(sched[r])
            t0 = time.perf_counter()
            s2 = orc.step(1)
            t1 = time.perf_counter()
            s1 = eng.step(1)
            t2 = time.perf_counter()
            print(f"  r={r}: oracle {t1 - t0:.1f} s, gpu {1e3 * (t2 - t1):.1f} ms, {s2}", flush=True)
            assert s1 == s2, f"round {r}: gpu {s1} != cpu {s2}"
            np.testing.assert_array_equal(eng.read_failed(), orc.read_failed(), err_msg=f"failed r={r}")
            np.testing.assert_array_equal(eng.read_detectors(), orc.read_detectors(), err_msg=f"detectors r={r}")
            seen["detections"] += s1["detections"]
            if world == 1:  # (per-shard diagnostics differ between shards)
                seen["storm"] |= eng.encoding_info(full=True)[2] == 1
                var = eng.tier_info(full=True)[3]
                seen["variants"][var] = seen["variants"].get(var, 0) + 1
            if after_round:
                after_round(eng, orc, r)
            if per_round:
                per_round(eng, r, s1)
            if s1["detections"] and seen["first_detection"] is None:
                seen["first_detection"] = r
                pending_full |= {r, r + 1}  # the detection round and the REMOVE round after it
            if r in pending_full:
                compare_blocks(eng, orc, r)
        print(f"  variants (round counts by gh_tier_info variant): {seen['variants']}", flush=True)
        expect(seen)
    finally:
        eng.close()
        orc.close()


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


def test_c3_fullsize_crash_1pct(gs, oracle_mod):
    """1% crash in the bench's workload: 655 members (Philox, seed
    0x5EED0003, tag CRASH) stop at r=8; run through their detection and the
    REMOVE wave, full tables equal at r=12, the detection round, the round
    after it and the last round."""
    from scenarios import crash_ids
    crashed = crash_ids(N, 0.01, 0x5EED0003)
    assert len(crashed) == 655
    sched = {8: [(gs.GH_EV_CRASH, int(c)) for c in crashed]}

    def expect(s):
        assert s["detections"] > 0 and s["first_detection"] is not None, s

    def fast(eng, r, st):
        # the crash wave stays on the nibble path: REMOVE delivery turns the
        # removed members' cells into tier tombstones inside it (round.hip
        # nib_word RMV), so no round hands more than 1% of the lanes to the
        # lane-job kernel (round 4: 38 M = 14% in the REMOVE round)
        if r >= 6:
            assert eng.tier_info(full=True)[3] == 3, (r, eng.tier_info(full=True))
            jobs, _ = eng.job_info()
            assert jobs * 100 <= N * N // 16, (r, jobs)

    run(gs, oracle_mod, 16, 32, {12, 32}, expect, sched=sched, per_round=fast)


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
def test_c3_fullsize_rows_g8(gs, oracle_mod):
    """North_star's layout at the largest size one MI355X holds: 8 row shards
    (each owns 8,192 observer rows; the senders' plane rows of other shards
    arrive by alltoallv into its ghost table, the want lists built on the
    device), N=65,536, k=4, T_fail=16, the 1% crash at r=8, 25 rounds: full
    tables at r=6, 25, the detection round and the one after."""
    run(gs, oracle_mod, 16, 25, {6, 25}, expect_detection, sched=crash_sched(gs), world=8, layout=1)


@pytest.mark.gpu_fullsize
def test_c3_fullsize_columns_g8(gs, oracle_mod):
    """The default multi-GPU layout at full size: 8 column shards (each holds
    every row of 8,192 member columns, O(N) exchanges), the same workload
    against tablesim (not against one engine)."""
    run(gs, oracle_mod, 16, 25, {6, 25}, expect_detection, sched=crash_sched(gs), world=8, layout=0)


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
