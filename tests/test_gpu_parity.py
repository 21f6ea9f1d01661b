"""GPU parity: libgossiphip's HIP path (through the C-ABI) against the CPU
oracle (oracle/tablesim.c), bit for bit — hb, ts, alive, failed set,
detectors, per-round counters and placement results — on the App. B KATs,
BASELINE config shapes and seeded churn. Run on a MI355X: pytest -m gpu."""
import numpy as np
import pytest

import scenarios as sc
from kat_util import KATS, kat_config, run_kat

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gs():
    import gossipsim
    return gossipsim


def check_counts(eng, r):
    """The maintained per-row present counts (cntl: the rounds, events and
    list merges keep them by deltas; the <4 guard reads them) equal a full
    recount on every engine (gh_debug_counts)."""
    for e in getattr(eng, "engines", [eng]):
        nm, first = e.debug_counts()
        assert nm == 0, f"r={r}: {nm} rows' maintained present counts differ from a recount, first row {first}"


def compare(eng, orc, r, full=True):
    check_counts(eng, r)
    h1, t1, a1 = eng.export_state()
    h2, t2, a2 = orc.export_state()
    np.testing.assert_array_equal(a1, a2, err_msg=f"alive r={r}")
    if full:
        bad = np.argwhere(h1 != h2)
        assert bad.size == 0, f"hb r={r}: {len(bad)} cells differ, first {bad[:5].tolist()} " \
                              f"gpu={h1[tuple(bad[0])]} cpu={h2[tuple(bad[0])]}"
        np.testing.assert_array_equal(t1, t2, err_msg=f"ts r={r}")
    np.testing.assert_array_equal(eng.read_failed(), orc.read_failed(), err_msg=f"failed r={r}")
    np.testing.assert_array_equal(eng.read_detectors(), orc.read_detectors(), err_msg=f"detectors r={r}")


def run_parity(gs, om, cfg_kw, n, rounds, sched, init=None, threads=8, every=1, files=None):
    eng = gs.Engine(gs.default_config(n, **cfg_kw))
    orc = om.Oracle(om.default_config(n, **cfg_kw), threads=threads)
    if init is not None:
        hb, ts, alive = init
        eng.import_state(hb, ts, alive, 0)
        orc.import_state(hb, ts, alive, 0)
    for r in range(1, rounds + 1):
        ev = sched.get(r, [])
        if ev:
            eng.apply_events(ev)
            orc.apply_events(ev)
        s1, s2 = eng.step(1), orc.step(1)
        assert s1 == s2, f"round {r}: gpu {s1} != cpu {s2}"
        if files is not None and r in files:
            f = np.asarray(files[r], np.int32)
            a, b = eng.put(f), orc.put(f)
            for x, y in zip(a, b):
                np.testing.assert_array_equal(x, y)
            for obs in orc.read_detectors()[:2]:
                assert eng.repair(int(obs)) == orc.repair(int(obs))
        if r % every == 0 or r == rounds or ev:
            compare(eng, orc, r)
    return eng, orc


@pytest.mark.parametrize("k", KATS, ids=lambda k: k["name"])
def test_kats_gpu(gs, k):
    run_kat(gs.Engine(kat_config(gs, k)), k)


@pytest.mark.parametrize("n,peer_mode,t_fail,seed", [(14, 1, 5, 4), (64, 1, 3, 5), (64, 0, 3, 6), (300, 0, 2, 7),
                                                     (257, 1, 3, 8)])
def test_quirk_detection_churn(gs, oracle_mod, n, peer_mode, t_fail, seed):
    """Quirk-mode detection (slave/slave.go:464-477 range over the slice that
    removeMember shifts): runs of candidates, skipped candidates staying in
    the senders' snapshots, the last list entry, under crash/leave/join."""
    sched = sc.random_churn(n, 40, seed, p_crash=0.08, p_leave=0.02, p_join=0.05)
    run_parity(gs, oracle_mod, dict(peer_mode=peer_mode, fanout=3, seed=0x2000 + seed, detect_mode=1,
                                    t_fail=t_fail, t_cleanup=t_fail + 2), n, 40, sched, init=sc.full_state(n))


@pytest.mark.parametrize("tw", [8, 16, 32, 64, 128, 256])
def test_quirk_detection_tile_widths(gs, oracle_mod, tw):
    """Quirk-mode detection under churn at every tile width: the pre-pass
    sums 8 cells per lane below 32-member tiles and 32 cells per lane from
    32 on (k_quirk_sum / k_quirk_sum32), runs crossing tile boundaries."""
    n = 600
    sched = sc.random_churn(n, 30, 0x71 + tw, p_crash=0.08, p_leave=0.02, p_join=0.05)
    run_parity(gs, oracle_mod, dict(fanout=3, seed=0x2100 + tw, detect_mode=1, t_fail=4, t_cleanup=6, tile_width=tw),
               n, 30, sched, init=sc.full_state(n))


def test_quirk_c2_collapse(gs, oracle_mod):
    """N=4,096 with the reference's 5-round timeouts in quirk mode: the
    round-6 detection storm with long candidate runs in every row."""
    n = 4096
    sched = {8: [(sc.CRASH, c) for c in sc.crash_ids(n, 0.01, 0x5EED0002)]}
    run_parity(gs, oracle_mod, dict(fanout=3, seed=0x5EED0002, detect_mode=1), n, 12, sched,
               init=sc.full_state(n), every=3)


@pytest.mark.parametrize("peer_mode", [0, 1])
def test_c1_bootstrap_crash_places(gs, oracle_mod, peer_mode):
    """BASELINE config 1: 10 members join one per round, 10 files put at r=20,
    member 7 crashes at r=30, run to r=60 with repairs."""
    n = 10
    sched = sc.bootstrap_schedule(n)
    sched.setdefault(30, []).append((sc.CRASH, 7))
    files = {20: list(range(10))}
    for r in range(31, 61):
        files[r] = []
    run_parity(gs, oracle_mod, dict(peer_mode=peer_mode, max_files=16, seed=0x5EED0001), n, 60, sched,
               files=files)


@pytest.mark.parametrize("n,peer_mode,seed", [(16, 0, 1), (16, 1, 2), (64, 0, 3), (64, 1, 4), (300, 0, 5),
                                              (257, 1, 6)])
def test_random_churn(gs, oracle_mod, n, peer_mode, seed):
    sched = sc.random_churn(n, 40, seed, p_crash=0.03, p_leave=0.01, p_join=0.05)
    run_parity(gs, oracle_mod, dict(peer_mode=peer_mode, fanout=3, seed=0x77 + seed), n, 40, sched,
               init=sc.full_state(n))


@pytest.mark.parametrize("fanout", [1, 4, 5, 8])
def test_fanouts_short_timeouts(gs, oracle_mod, fanout):
    n = 200
    sched = sc.random_churn(n, 30, 11, p_crash=0.05)
    run_parity(gs, oracle_mod, dict(fanout=fanout, t_fail=3, t_cleanup=7, seed=0x99), n, 30, sched,
               init=sc.full_state(n))


def test_c2_n4096_crash_1pct(gs, oracle_mod):
    """BASELINE config 2: N=4,096, k=3, full tables (hb=2, ts=0), 1% crash
    drawn by Philox(0x5EED0002) at r=8, 64 rounds; full-state compare every 8
    rounds, counters and failed sets every round."""
    n = 4096
    sched = {8: [(sc.CRASH, c) for c in sc.crash_ids(n, 0.01, 0x5EED0002)]}
    eng, orc = run_parity(gs, oracle_mod, dict(fanout=3, seed=0x5EED0002), n, 64, sched,
                          init=sc.full_state(n), every=8)


def test_c2_steady_state_crash(gs, oracle_mod):
    """N=4,096, k=3 in the healthy regime (T_fail = T_cleanup = 12 rounds,
    above the ~6-round dissemination time): ~55% of cells merge every round;
    a 1% crash at r=8 is detected and REMOVE'd everywhere."""
    n = 4096
    sched = {8: [(sc.CRASH, c) for c in sc.crash_ids(n, 0.01, 0x5EED0012)]}
    eng, orc = run_parity(gs, oracle_mod, dict(fanout=3, seed=0x5EED0012, t_fail=12, t_cleanup=12), n, 48,
                          sched, init=sc.full_state(n), every=8)
    assert eng.step(0)["rounds"] == 0


def test_placement_parity_many_files(gs, oracle_mod):
    n, F = 512, 20000
    cfg = dict(max_files=F, seed=0x5EED0005)
    eng = gs.Engine(gs.default_config(n, **cfg))
    orc = oracle_mod.Oracle(oracle_mod.default_config(n, **cfg))
    hb, ts, alive = sc.full_state(n)
    eng.import_state(hb, ts, alive, 3)
    orc.import_state(hb, ts, alive, 3)
    f = np.random.default_rng(0).permutation(F)[: F // 2].astype(np.int32)
    for x, y in zip(eng.put(f), orc.put(f)):
        np.testing.assert_array_equal(x, y)
    # crash 5% and let the failure be detected, then repair from two observers
    sched = {1: [(sc.CRASH, c) for c in sc.crash_ids(n, 0.05, 0x5EED0005)]}
    for r in range(1, 12):
        if r in sched:
            eng.apply_events(sched[r])
            orc.apply_events(sched[r])
        assert eng.step(1) == orc.step(1)
    for obs in (0, 5):
        assert eng.repair(obs) == orc.repair(obs)
    for x, y in zip(eng.get_files(np.arange(F)), orc.get_files(np.arange(F))):
        np.testing.assert_array_equal(x, y)
    g = np.arange(0, F, 7, dtype=np.int32)
    np.testing.assert_array_equal(eng.delete_files(g), orc.delete_files(g))
    for x, y in zip(eng.put(g[:100]), orc.put(g[:100])):
        np.testing.assert_array_equal(x, y)


def test_starvation_gpu(gs, oracle_mod):
    n = 8
    eng = gs.Engine(gs.default_config(n, max_files=4))
    hb = np.full((n, n), -1, np.int32)
    hb[0, :4] = 3
    alive = np.zeros(n, np.uint8)
    alive[0] = 1
    eng.import_state(hb, np.zeros((n, n), np.int32), alive, 20)
    rep, ver, st = eng.put([0])
    assert st[0] == gs.GH_EPLACEMENT_STARVED and ver[0] == 0


def test_n65536_invariants(gs):
    """BASELINE config 3 scale (N=65,536, k=4, 48 GiB of tables): properties
    that hold at any size — with no failures every member stays everywhere,
    the own heartbeat advances by one per round, no cell runs ahead of its
    owner, nothing is detected; then a 1% crash is detected by every live
    observer's failed set within T_fail + the dissemination time."""
    n, rounds = 65536, 12
    eng = gs.Engine(gs.default_config(n, fanout=4, seed=0x5EED0003, t_fail=16, t_cleanup=16))
    eng.init_full(2, 0, 0)
    st = eng.step(rounds)
    assert st["detections"] == 0 and st["active_rows"] == n * rounds
    assert st["merged_cells"] > n * n  # the epidemic has reached every cell
    rows = np.array([0, 1, 4095, 32768, 65535])
    for i in rows:
        hb, ts, _ = eng.export_state(int(i), 1)
        assert hb[0, i] == 2 + rounds
        assert (hb[0] >= 2).all() and (hb[0] <= 2 + rounds).all()
        assert (ts[0] <= rounds).all()
    crashed = sc.crash_ids(n, 0.01, 0x5EED0003)
    eng.apply_events([(sc.CRASH, c) for c in crashed])
    seen = set()
    for _ in range(40):
        eng.step(1)
        bm = eng.read_failed()
        seen |= {c for c in crashed if bm[c >> 5] >> (c & 31) & 1}
    assert seen == set(crashed)


@pytest.mark.parametrize("tw,nt,xmap", [(64, 1, 0), (64, 0, 1), (32, 1, 1), (128, 1, 0), (256, 0, 0),
                                         (256, 1, 1), (16, 1, 1), (8, 1, 1), (16, 0, 0)])
def test_layout_variants_identical(gs, oracle_mod, tw, nt, xmap):
    """Every table tile width and k_round stream policy gives the oracle's
    results (layout/tuning knobs), including N not a multiple of the tile."""
    n = 700
    sched = sc.random_churn(n, 24, 21, p_crash=0.04, p_leave=0.01, p_join=0.05)
    eng = gs.Engine(gs.default_config(n, fanout=4, seed=0x31, t_fail=4, t_cleanup=6, tile_width=tw))
    eng.set_round_variant(nt, xmap)
    orc = oracle_mod.Oracle(oracle_mod.default_config(n, fanout=4, seed=0x31, t_fail=4, t_cleanup=6), threads=8)
    hb, ts, alive = sc.full_state(n)
    eng.import_state(hb, ts, alive, 0)
    orc.import_state(hb, ts, alive, 0)
    for r in range(1, 25):
        if r in sched:
            eng.apply_events(sched[r])
            orc.apply_events(sched[r])
        assert eng.step(1) == orc.step(1), r
    compare(eng, orc, 24)
    for obs in (0, 3, 699):
        a, b = eng.lsm(obs), orc.lsm(obs)
        for x, y in zip(a, b):
            np.testing.assert_array_equal(x, y)


def test_merge_list_external_datagrams(gs, oracle_mod):
    """Reference datagrams (gossipsim.codec, slave/slave.go:365-385) merged
    into members' rows between rounds (GetMsg -> decode -> MergeMemberList,
    :241-245) through gh_merge_list, then more rounds: bit-exact vs the
    oracle. Lists carry raised, equal, lower and tombstoned entries."""
    from gossipsim import codec
    n = 48
    cfg = dict(fanout=3, seed=0x4D, t_fail=4, t_cleanup=6)
    eng = gs.Engine(gs.default_config(n, **cfg))
    orc = oracle_mod.Oracle(oracle_mod.default_config(n, **cfg))
    init = sc.full_state(n)
    eng.import_state(*init, 0)
    orc.import_state(*init, 0)
    sched = sc.random_churn(n, 20, 17, p_crash=0.05, p_leave=0.02, p_join=0.05)
    addr = [f"10.1.0.{i}" for i in range(n)]
    rng = np.random.default_rng(5)
    for r in range(1, 21):
        if r in sched:
            eng.apply_events(sched[r])
            orc.apply_events(sched[r])
        assert eng.step(1) == orc.step(1), r
        for _ in range(3):
            src, dst = (int(x) for x in rng.integers(0, n, 2))
            ids, hb, ts = orc.lsm(src)
            if len(ids) == 0:  # empty lists are never sent (HeartBeat's <4 guard); decode would panic
                continue
            hb = hb + rng.integers(-2, 4, len(hb)).clip(-hb)  # some raised, some lowered
            dg = codec.encode((addr[i], int(h), int(t)) for i, h, t in zip(ids, hb, ts))
            got = codec.decode(dg, read_buf=1 << 20)
            ids2 = [addr.index(a) for a, _, _ in got]
            hb2 = [h for _, h, _ in got]
            assert eng.merge_list(dst, ids2, hb2) == orc.merge_list(dst, ids2, hb2)
        compare(eng, orc, r)


def test_cluster_datagram_roundtrip(gs):
    """Cluster.datagram/receive: a member's list in the reference's wire
    format merged at another member (10 VMs, config 1 shape)."""
    cl = gs.Cluster(10, max_files=16)
    assert cl.engine.cfg.peer_mode == gs.GH_PEER_RING  # the facade gossips the reference's ring
    for m in range(10):
        cl.join(m)
        cl.tick()
    cl.tick(3)
    dg = cl.datagram(3)
    assert dg.count(b"<#ENTRY#>") == len(cl.lsm(3)) - 1 and len(dg) <= 1024
    assert cl.receive(5, dg) >= 0
    assert {i for i, _, _ in cl.lsm(5)} >= {i for i, _, _ in cl.lsm(3)}


def test_put_conflicts_and_cluster_ops(gs, oracle_mod):
    """The write-write window on the GPU against the oracle for 3,000 files
    put at different rounds, and Cluster.put/get: conflicts go ahead only
    when confirmed; acks count live replicas against the quorum."""
    n, F = 64, 3000
    cfg = dict(max_files=F, seed=0x5EED0006)
    eng = gs.Engine(gs.default_config(n, **cfg))
    orc = oracle_mod.Oracle(oracle_mod.default_config(n, **cfg))
    init = sc.full_state(n)
    eng.import_state(*init, 0)
    orc.import_state(*init, 0)
    rng = np.random.default_rng(1)
    for r in range(1, 80):
        assert eng.step(1) == orc.step(1)
        if r % 7 == 0:
            f = rng.permutation(F)[:200].astype(np.int32)
            for x, y in zip(eng.put(f), orc.put(f)):
                np.testing.assert_array_equal(x, y)
        if r % 13 == 0:
            f = np.arange(F, dtype=np.int32)
            np.testing.assert_array_equal(eng.put_conflicts(f), orc.put_conflicts(f))
    eng.close()

    cl = gs.Cluster(10, max_files=8)
    for m in range(10):
        cl.join(m)
        cl.tick()
    res = cl.put([0, 1])
    assert all(p.put_or_not and p.version == 1 and p.quorum_met for p in res)
    again = cl.put([0, 1], confirm=[1])  # file 0 clashes (0 rounds ago), 1 is confirmed
    assert (again[0].put_or_not, again[1].put_or_not, again[1].version) == (False, True, 2)
    # Get's copy source (slave/slave.go:857-878): every live replica holds
    # version 2 of file 1, so the first one in arrival (= replica) order
    g = cl.get([1])[0]
    assert (g.source, g.source_version) == (again[1].replicas[0], 2)
    for a in again[1].replicas[:3]:
        cl.crash(a)
    cl.tick()
    g = cl.get([1, 5])[0]
    assert g.acks == 1 and g.quorum_met is False and cl.get([5])[0].version == -1
    assert g.source == again[1].replicas[3] and g.source_version == 2  # the only live replica
    # a crashed replica that restarts is a fresh process: no Local_files, so
    # it answers version 0, which is <= 2, and is picked when it answers first
    first = again[1].replicas[0]
    cl.join(first)
    cl.tick()
    g = cl.get([1])[0]
    assert cl.local_version(first, 1) == 0 and (g.source, g.source_version) == (first, 0)


def c5_run(eng, orc, n, F, rounds=32):
    """BASELINE config 5 shape at 1-GPU scale: 2^20 files placed, then waves
    at r=4/8/12 (join 1% new IDs, leave 1%, crash 1%), and every detecting
    row's repair pass 8 rounds after its detection (Fail_recover,
    slave/slave.go:1122-1133; here the first two detectors per round)."""
    files = np.arange(F, dtype=np.int32)
    for lo in range(0, F, 1 << 18):
        for x, y in zip(eng.put(files[lo:lo + (1 << 18)]), orc.put(files[lo:lo + (1 << 18)])):
            np.testing.assert_array_equal(x, y)
    newcomers = list(range(n - n // 100, n))
    rng = np.random.default_rng(55)
    pool = [c for c in range(1, n - n // 100)]
    rng.shuffle(pool)
    waves = {4: [(sc.JOIN, c) for c in newcomers],
             8: [(sc.LEAVE, c) for c in pool[: n // 100]],
             12: [(sc.CRASH, c) for c in pool[n // 100: 2 * (n // 100)]]}
    due = {}
    plans = 0
    for r in range(1, rounds + 1):
        if r in waves:
            eng.apply_events(waves[r])
            orc.apply_events(waves[r])
        assert eng.step(1) == orc.step(1), r
        det = list(orc.read_detectors())
        np.testing.assert_array_equal(eng.read_detectors(), det)
        if det:
            due.setdefault(r + 8, []).extend(int(x) for x in det[:2])
        for obs in due.pop(r, []):
            p1, p2 = eng.repair(obs), orc.repair(obs)
            assert p1 == p2, (r, obs)
            plans += len(p1)
    for lo in range(0, F, 1 << 18):
        for x, y in zip(eng.get_files(files[lo:lo + (1 << 18)]), orc.get_files(files[lo:lo + (1 << 18)])):
            np.testing.assert_array_equal(x, y)
    return plans


def test_c5_churn_rereplication_1m_files(gs, oracle_mod):
    n, F = 2048, 1 << 20
    cfg = dict(fanout=4, seed=0x5EED0005, max_files=F, t_fail=8, t_cleanup=8)
    eng = gs.Engine(gs.default_config(n, **cfg))
    orc = oracle_mod.Oracle(oracle_mod.default_config(n, **cfg), threads=8)
    hb, ts, alive = sc.full_state(n)
    alive[n - n // 100:] = 0
    hb[:, n - n // 100:] = -1
    hb[n - n // 100:, :] = -1
    eng.import_state(hb, ts, alive, 0)
    orc.import_state(hb, ts, alive, 0)
    assert c5_run(eng, orc, n, F) > 0


def test_quirk_repair_plan_last_file_only(gs, oracle_mod):
    """Quirk mode: Update_metadata re-makes its plan map per repaired file
    (master/master.go:118) and returns the last one only, while every file's
    metadata is repaired (SPEC D5)."""
    n, F = 64, 300
    cfg = dict(max_files=F, seed=0x5EED0007, detect_mode=1, t_fail=4, t_cleanup=4)
    eng = gs.Engine(gs.default_config(n, **cfg))
    orc = oracle_mod.Oracle(oracle_mod.default_config(n, **cfg))
    init = sc.full_state(n)
    eng.import_state(*init, 0)
    orc.import_state(*init, 0)
    f = np.arange(F, dtype=np.int32)
    for x, y in zip(eng.put(f), orc.put(f)):
        np.testing.assert_array_equal(x, y)
    ev = [(sc.CRASH, c) for c in sc.crash_ids(n, 0.1, 0x5EED0007)]
    eng.apply_events(ev)
    orc.apply_events(ev)
    for r in range(1, 10):
        assert eng.step(1) == orc.step(1), r
    p1, p2 = eng.repair(0), orc.repair(0)
    assert p1 == p2 and len(p1) == 1
    for x, y in zip(eng.get_files(f), orc.get_files(f)):
        np.testing.assert_array_equal(x, y)
    eng.close()


def test_quiet_rows_after_collapse(gs, oracle_mod):
    """The reference's 5-round timeouts at N=2,048, k=4: the round-6
    detection storm collapses the cluster; once the inactive rows'
    tombstones saturate (age 30) their rows stop changing and the round
    skips them (neither read nor rewritten). Bit-exact against the oracle
    through round 64, a join at round 52 (a host write: every row is a
    candidate again), and the skip did happen."""
    n = 2048
    cfg = dict(fanout=4, seed=0x5EED0800)
    eng = gs.Engine(gs.default_config(n, **cfg))
    orc = oracle_mod.Oracle(oracle_mod.default_config(n, **cfg), threads=8)
    hb, ts, alive = sc.full_state(n)
    eng.import_state(hb, ts, alive, 0)
    orc.import_state(hb, ts, alive, 0)
    quiet = []
    for r in range(1, 65):
        if r == 52:
            ev = [(sc.JOIN, 5)]
            eng.apply_events(ev)
            orc.apply_events(ev)
        s1, s2 = eng.step(1), orc.step(1)
        assert s1 == s2, f"round {r}: gpu {s1} != cpu {s2}"
        quiet.append(eng.encoding_info(full=True)[4])
        if r % 4 == 0 or r in (51, 52, 53):
            compare(eng, orc, r)
    assert max(quiet) > 0, quiet


@pytest.mark.parametrize("n", [9, 1500])
def test_ring_whole_lists(gs, oracle_mod, n):
    """Ring mode with long timeouts: most rounds have no flag and no REMOVE,
    so every sender's targets come from its whole list by the outward scan
    (k_ring_fast); a crash wave, leaves and re-joins (own member absent from
    a list, short lists, the wrap-around) switch rounds back to the counting
    path. Bit-exact against the oracle every round."""
    crash = sc.crash_ids(n, 0.2, 0x5EED0A00)
    sched = {4: [(sc.CRASH, c) for c in crash],
             30: [(sc.LEAVE, (n // 2) | 1)],
             36: [(sc.JOIN, c) for c in crash[: max(1, len(crash) // 2)]]}
    run_parity(gs, oracle_mod, dict(peer_mode=1, seed=0x5EED0A01 + n, t_fail=20, t_cleanup=20), n, 50, sched,
               init=sc.full_state(n))


def shadows_of(eng, n):
    """int32[n]: the engine's (or shard group's) D7 shadow entries by member"""
    out = np.full(n, np.iinfo(np.int32).min, np.int32)
    cnt = 0
    for e in getattr(eng, "engines", [eng]):
        c0, sh, k = e.debug_shadow()
        out[c0:c0 + len(sh)] = np.where(sh != np.iinfo(np.int32).min, sh, out[c0:c0 + len(sh)])
        cnt += k
    assert cnt == int((out != np.iinfo(np.int32).min).sum()), (cnt, out)
    return out


@pytest.mark.parametrize("layout", ["single", "cols3", "rows2"])
@pytest.mark.parametrize("peer_mode", [0, 1], ids=["pull", "ring"])
def test_rejoin_while_tombstoned_d7(gs, oracle_mod, layout, peer_mode):
    """SPEC D7 as the reference does it (slave/slave.go:228-230, 250-255,
    276-286, 484-497): members leave or crash and rejoin while the
    introducer still holds their tombstone, so it holds them twice; LEAVEs,
    REMOVEs and detections of such a member at the introducer keep the old
    RecentFailList entry (its ts), cleanFailList releases it. Bit-exact
    against tablesim every round, the shadow entries included, with double
    entries occurring; one engine, 3 column shards and 2 row shards."""
    n = 300
    cfg = dict(fanout=3, seed=0x5EED0E10 + peer_mode, t_fail=4, t_cleanup=6, peer_mode=peer_mode)
    sched = sc.rejoin_churn(n, 40, 0xD7 + peer_mode)
    if layout == "single":
        eng = gs.Engine(gs.default_config(n, **cfg))
    else:
        world, lay = (3, 0) if layout == "cols3" else (2, 1)
        eng = gs.ShardGroup(gs.default_config(n, shard_layout=lay, **cfg), world)
    orc = oracle_mod.Oracle(oracle_mod.default_config(n, **cfg), threads=8)
    hb, ts, alive = sc.full_state(n)
    eng.import_state(hb, ts, alive, 0)
    orc.import_state(hb, ts, alive, 0)
    dual = 0
    try:
        for r in range(1, 41):
            ev = sched.get(r, [])
            if ev:
                eng.apply_events(ev)
                orc.apply_events(ev)
            s1, s2 = eng.step(1), orc.step(1)
            assert s1 == s2, f"round {r}: gpu {s1} != cpu {s2}"
            compare(eng, orc, r)
            a, b = shadows_of(eng, n), orc.debug_shadow()
            np.testing.assert_array_equal(a, b, err_msg=f"shadow entries r={r}")
            dual = max(dual, int((b != np.iinfo(np.int32).min).sum()))
    finally:
        eng.close()
        orc.close()
    assert dual > 0
