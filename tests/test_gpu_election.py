"""Master re-election on the GPU (SPEC §9): gh_vote_scan and
gh_rebuild_meta against oracle/election.py on the oracle's tables, single and
sharded, and gossipsim.Cluster's election against the oracle Tally round by
round (slave/slave.go:451-457, 930-1051)."""
import numpy as np
import pytest

import scenarios as sc
from oracle import election as el

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gs():
    import gossipsim
    return gossipsim


def _scan_check(eng, hb, rng, n):
    for mv in (np.zeros(n, np.int32), rng.integers(0, n, n).astype(np.int32)):
        got = eng.vote_scan(mv)
        exp = el.vote_scan(hb, mv)
        for g, e, name in zip(got, exp, ("first", "list_len", "has_master")):
            np.testing.assert_array_equal(g, e, err_msg=name)


@pytest.mark.parametrize("detect_mode", [0, 1])
@pytest.mark.parametrize("peer_mode", [0, 1])
def test_vote_scan_churn(gs, oracle_mod, peer_mode, detect_mode):
    """Seeded churn at N=300 (crashes, leaves, joins; tombstones and empty
    rows), canonical and quirk detection, the scan checked every 3 rounds
    against the oracle's table."""
    n, rounds = 300, 30
    cfg = dict(peer_mode=peer_mode, detect_mode=detect_mode, t_fail=3, t_cleanup=3, seed=0x5EED0F31)
    eng = gs.Engine(gs.default_config(n, **cfg))
    orc = oracle_mod.Oracle(oracle_mod.default_config(n, **cfg))
    sched = sc.random_churn(n, rounds, seed=31)
    rng = np.random.default_rng(7)
    _scan_check(eng, orc.export_state()[0], rng, n)  # empty table: first = -1
    for r in range(1, rounds + 1):
        ev = sched.get(r, [])
        if ev:
            eng.apply_events(ev)
            orc.apply_events(ev)
        assert eng.step(1) == orc.step(1)
        if r % 3 == 0:
            _scan_check(eng, orc.export_state()[0], rng, n)
    eng.close()


@pytest.mark.parametrize("world", [2, 3])
def test_vote_scan_sharded(gs, world):
    """G shards (in-process transport) agree with the single engine: the
    first member may sit on any shard, the master's column on one."""
    n = 500
    cfg = gs.default_config(n, t_fail=4, t_cleanup=4, seed=0x5EED0F32)
    one = gs.Engine(gs.Config.from_buffer_copy(cfg))
    grp = gs.ShardGroup(cfg, world)
    init = sc.full_state(n)
    one.import_state(*init, 0)
    grp.import_state(*init, 0)
    crash = [(gs.GH_EV_CRASH, c) for c in range(0, 300, 7)]
    one.apply_events(crash)
    grp.apply_events(crash)
    rng = np.random.default_rng(3)
    for _ in range(8):
        assert one.step(1) == grp.step(1)
        mv = rng.integers(0, n, n).astype(np.int32)
        for a, b in zip(one.vote_scan(mv), grp.vote_scan(mv)):
            np.testing.assert_array_equal(a, b)
    grp.close()
    one.close()


def _meta(eng, F):
    return eng.get_files(np.arange(F, dtype=np.int32))


@pytest.mark.parametrize("world", [1, 3])
def test_rebuild_meta(gs, world):
    """rebuild_file_meta at several new masters after placement, crashes and
    repairs: the file table equals the oracle's literal rebuild."""
    n, F = 64, 3000
    cfg = gs.default_config(n, max_files=F, seed=0x5EED0F33, t_fail=8, t_cleanup=8)
    eng = gs.Engine(cfg) if world == 1 else gs.ShardGroup(cfg, world)
    eng.import_state(*sc.full_state(n), 0)
    eng.step(2)
    eng.put(np.arange(0, F, 2, dtype=np.int32))
    eng.apply_events([(gs.GH_EV_CRASH, c) for c in (3, 9, 17, 40)])
    eng.step(1)
    eng.put(np.arange(1, F, 4, dtype=np.int32))
    eng.step(9)
    eng.repair(5)
    eng.step(1)
    for m in (0, 2, 33):  # 0: its own MemberList[0]; 2, 33: f0 = another member
        rep, ver = _meta(eng, F)
        ids = [int(x) for x in eng.lsm(m)[0]]
        assert len(ids) == 60  # the 4 crashed members detected and removed
        er, ev, _ = el.rebuild(rep, ver, np.zeros(F, np.int32), m, ids, now=eng.round)
        f0, nf = eng.rebuild_meta(m)
        assert f0 == ids[0] and nf == int((ev >= 0).sum())
        r2, v2 = _meta(eng, F)
        np.testing.assert_array_equal(v2, ev)
        np.testing.assert_array_equal(r2, er)
        # the new master's list is the placement candidate list from now on
        rp, _, st = eng.put(np.array([F - 1], np.int32))
        assert st[0] == gs.GH_OK and all(x in ids for x in rp[0] if x >= 0)
    eng.close()


@pytest.mark.parametrize("peer_mode", [0, 1])
def test_cluster_master_crash_election(gs, peer_mode):
    """Cluster(elect=True), 32 members, master 0 crashes: the votes go to
    member 1 (everyone's MemberList[0]) and elect it the round its majority
    arrives; it rebuilds two rounds later (its own MemberList[0], so every
    listed member reports its store); the detectors' Fail_recover 8 rounds
    after detection dials the dead master and log.Fatal's. Checked round by
    round against the oracle Tally on the exported table. Pull and the
    reference's ring (there only the ring neighbours of 0 detect it; the
    rest get the REMOVE and vote a round later)."""
    n, F = 32, 400
    tf = 8 if peer_mode == 0 else 16  # ring dissemination needs the longer timeout to stay healthy
    cl = gs.Cluster(n, elect=True, max_files=F, seed=0x5EED0F34, t_fail=tf, t_cleanup=tf, peer_mode=peer_mode)
    eng = cl.engine
    eng.import_state(*sc.full_state(n), 0)
    cl.tick(2)
    cl.put(range(F))
    cl.crash(0)
    tally = el.Tally(n, master=0)
    pending, det_round, detectors = {}, None, None
    prev = _meta(eng, F)
    for _ in range(30):
        cl.tick(1)
        r = eng.round
        hb, _, alive = eng.export_state()
        if det_round is None and len(eng.read_detectors()):
            det_round, detectors = r, set(eng.read_detectors().tolist())
        for m in pending.pop(r, []):
            lst = [int(c) for c in np.flatnonzero(hb[m] >= 0)]
            tally.finish_rebuild(m, lst[0])
            er, ev, _ = el.rebuild(prev[0], prev[1], np.zeros(F, np.int32), m, lst, now=r)
            rep, ver = _meta(eng, F)
            np.testing.assert_array_equal(ver, ev)
            np.testing.assert_array_equal(rep, er)
        for m in tally.round(alive, *el.vote_scan(hb, tally.mview), dead=cl.dead):
            pending[r + 2] = pending.get(r + 2, []) + [m]
        np.testing.assert_array_equal(cl.mview, tally.mview, err_msg=f"r={r}")
        prev = _meta(eng, F)
    assert [m for _, m in cl.elections] == [1] and cl.master == 1
    assert not pending
    # Fail_recover at det_round + 8: every detector but the new master dies
    assert det_round is not None
    fatal = {m for r, m, why in cl.fatal if why.startswith("Fail_recover") and r == det_round + cl.repair_delay}
    assert fatal == detectors - {1}
    eng.close()


def test_cluster_rebuild_fatal_and_self_votes(gs):
    """A hand-built table (member ids 0..7, master 0 crashed and tombstoned
    everywhere; member 1 tombstoned in rows 3..7):
      row 1 = {1..7}: votes for itself (counted, no check);
      row 2 = {1..7}: votes for 1;  rows 3..7 = {2..7}: vote for 2.
    Round 1: Vote_num[1] = 2, not > 7 // 2; Vote_num[2] reaches 4 > 3 at
    row 6, so 2 is elected (row 7's vote still counts: 5). Member 1 then crashes; at round 3 the rebuild
    dials MemberList_2[0] = 1, which is gone: 2 log.Fatal's (:996-999) and
    the master stays 0."""
    n = 8
    hb = np.full((n, n), -1, np.int32)
    hb[:, 0] = -2
    hb[1, 1:] = 5
    hb[2, 1:] = 5
    hb[3:, 2:] = 5
    hb[3:, 1] = -2
    hb[0, :] = 5
    ts = np.zeros((n, n), np.int32)
    alive = np.ones(n, np.uint8)
    alive[0] = 0
    cl = gs.Cluster(n, elect=True, t_fail=8, t_cleanup=30, fanout=2, peer_mode=gs.GH_PEER_PULL)
    cl.engine.import_state(hb, ts, alive, 0)
    cl.dead.add(0)
    cl.tick(1)
    assert cl.elections == [(1, 2)] and cl.mview[2] == 2
    assert cl.vote_num[1] == 2 and cl.voters[1] == {2} and cl.vote_num[2] == 5
    cl.crash(1)
    cl.tick(2)
    assert (3, 2, "rebuild_file_meta: MemberList[0] unreachable") in cl.fatal
    assert cl.master == 0
    cl.engine.close()


def test_rebuild_master_not_in_own_list(gs):
    """A new master whose own list lacks itself (its self entry tombstoned):
    the rebuild loop never reaches member == M (:991-992), so M's own store
    is never read, and a file only M holds is dropped."""
    n, F = 8, 64
    hb = np.full((n, n), 5, np.int32)
    hb[5, 5] = -2
    ts = np.zeros((n, n), np.int32)
    eng = gs.Engine(gs.default_config(n, max_files=F, seed=0x5EED0F35, t_fail=8, t_cleanup=8))
    eng.import_state(hb, ts, np.ones(n, np.uint8), 0)
    eng.put(np.arange(F, dtype=np.int32))
    rep, ver = _meta(eng, F)
    ids = [int(x) for x in eng.lsm(5)[0]]
    assert 5 not in ids and ids[0] == 0
    er, ev, _ = el.rebuild(rep, ver, np.zeros(F, np.int32), 5, ids, now=eng.round)
    only_m = [f for f in range(F) if 5 in rep[f] and 0 not in rep[f]]
    assert only_m and all(ev[f] == -1 for f in only_m)
    f0, nf = eng.rebuild_meta(5)
    r2, v2 = _meta(eng, F)
    assert f0 == 0 and nf == int((ev >= 0).sum())
    np.testing.assert_array_equal(v2, ev)
    np.testing.assert_array_equal(r2, er)
    eng.close()


def test_crash_join_then_master_crash(gs):
    """A member that crashed and joins again is a fresh process
    (new_slave, slave/slave.go:99-112): out of the gone set, master = the
    configured one, VoteStatus off; when the master then crashes it votes
    like everyone else and is not taken for a dead process."""
    n = 32
    cl = gs.Cluster(n, elect=True, max_files=64, seed=0x5EED0F36, t_fail=8, t_cleanup=8, peer_mode=gs.GH_PEER_PULL)
    cl.engine.import_state(*sc.full_state(n), 0)
    cl.tick(2)
    cl.put(range(64))
    cl.crash(5)
    cl.vote_on[5], cl.vote_num[5] = True, 3  # stale state the dead process held
    cl.tick(20)
    assert 5 in cl.dead
    cl.join(5)
    assert 5 not in cl.dead and cl.mview[5] == 0 and not cl.vote_on[5] and cl.vote_num[5] == 0
    cl.tick(12)
    cl.crash(0)
    cl.tick(30)
    assert [m for _, m in cl.elections] == [1] and cl.master == 1
    # its vote reaches member 1 (no log.Fatal on the vote path for it)
    assert all(not (m == 5 and why.startswith("revote")) for _, m, why in cl.fatal)
    g = cl.get([0, 1])
    assert all(x.source == next((a for a in x.replicas if a not in cl.dead), -1) for x in g)


@pytest.mark.gpu
def test_repair_at_stale_running_master(gs):
    """Fail_recover (slave/slave.go:1122-1142) dials the observer's own idea
    of the master. Master 0 crashes, 1 is elected and rebuilds; 0 restarts as
    a fresh process (Join, :288-308), believing the configured master -- itself
    -- is the master. A repair it runs goes to its own SDFSMaster, which a
    fresh process holds empty (master/master.go:38): Update_metadata returns
    nothing and Fail_recover returns at once (:1139-1142). The same repair
    from a member that follows the new master gets the master's plan."""
    n, F = 32, 400
    cl = gs.Cluster(n, elect=True, max_files=F, seed=0x5EED0F34, t_fail=8, t_cleanup=8, peer_mode=gs.GH_PEER_PULL)
    cl.engine.import_state(*sc.full_state(n), 0)
    cl.tick(2)
    cl.put(range(F))
    cl.crash(0)
    for _ in range(40):
        cl.tick(1)
        if cl.master != 0:
            break
    assert cl.master == 1
    cl.join(0)
    cl.tick(1)
    assert cl.mview[0] == 0 and 0 not in cl.dead
    alive = cl.engine.alive()
    obs = next(i for i in range(1, n) if alive[i] and i not in cl.dead and cl.mview[i] == cl.master)
    r = cl.engine.round
    cl.scheduled[r + 1] = [0, obs]
    cl.tick(1)
    got = {o: plan for rr, o, plan in cl.plans if rr == r + 1}
    assert got[0] == () and obs in got
    cl.engine.close()


@pytest.mark.parametrize("world", [1, 2])
def test_cluster_demoted_master_keeps_running(gs, oracle_mod, world):
    """A master demoted while its process keeps running answers from its
    own maps (slave/slave.go:1122-1136 -> master/master.go:74-127): 16
    members, master 0 stale in rows 2..15 (not crashed). Round 21 those rows
    detect 0 and vote for their MemberList[0] = 1, which is elected and
    rebuilds at round 23; the REMOVE of 0 reaches every row, 0's own too. Most
    members never learn the new master (only MemberList_1[0] gets
    Assign_new_master), so their Fail_recover calls go to 0, whose process
    still runs: it runs Update_metadata on the maps it had when it was
    demoted (gh_export_files / gh_import_files swap them into the engine,
    with its own list as Member_list, gh_set_master), while 1 answers from
    the rebuilt table. A crash of member 5 at round 23 gives more repairs
    (0's own included). Every plan, and both masters' tables at the end,
    against the oracle's Update_metadata on the same tables, routed by the
    oracle Tally's self.master; world 2: the engine's file table sharded
    by file ID."""
    n, F = 16, 64
    cfg = dict(max_files=F, seed=0x5EED0F37, t_fail=4, t_cleanup=6, fanout=3, peer_mode=gs.GH_PEER_PULL)
    hb, ts, alive = sc.full_state(n, 2, 20)
    ts[2:, 0] = 10  # rows 2..15 last heard of 0 ten rounds ago: detected at round 21
    if world == 1:
        cl = gs.Cluster(n, elect=True, **cfg)
    else:  # the Cluster over 2 column shards (ID list order: the same lists here, no joins)
        cl = gs.Cluster(n, elect=True, **cfg)
        cl.engine.close()
        cl.engine = gs.ShardGroup(gs.default_config(n, list_order=gs.GH_ORDER_ID, **cfg), world)
    eng = cl.engine
    orc = oracle_mod.Oracle(oracle_mod.default_config(n, **cfg))
    try:
        eng.import_state(hb, ts, alive, 20)
        orc.import_state(hb, ts, alive, 20)
        files = np.arange(F, dtype=np.int32)
        cl.put(files)
        orc.put(files)
        tally = el.Tally(n, master=0)
        master, demoted, dead = 0, {}, set()
        due, pending, expect = {}, {}, []
        for r in range(21, 45):
            if r == 23:
                cl.crash(5)
                orc.apply_events([(gs.GH_EV_CRASH, 5)])
                dead.add(5)
            cl.tick(1)
            s2 = orc.step(1)
            assert eng.round == r
            if s2["detections"]:
                due.setdefault(r + cl.repair_delay, []).extend(int(x) for x in orc.read_detectors())
            hbo, _, alo = orc.export_state()
            for m in pending.pop(r, []):  # rebuild_file_meta at the new master m
                lst = [int(c) for c in np.flatnonzero(hbo[m] >= 0)]
                tally.finish_rebuild(m, lst[0])
                old = orc.export_files()
                if master != m and master not in dead:
                    demoted[master] = old
                demoted.pop(m, None)
                er, ev, ef = el.rebuild(old[0], old[1], old[2], m, lst, now=r)
                orc.import_files(er, ev, ef, old[3])
                orc.set_master(m)
                master = m
                due.setdefault(r + cl.repair_delay, []).append(m)
            for m in tally.round(alo, *el.vote_scan(hbo, tally.mview), dead=dead):
                pending[r + 2] = pending.get(r + 2, []) + [m]
            np.testing.assert_array_equal(cl.mview, tally.mview, err_msg=f"r={r}")
            for obs in due.pop(r, []):
                if obs in dead:
                    continue
                m = int(tally.mview[obs])
                assert m not in dead  # (no Fail_recover log.Fatal in this scenario)
                if m == master:
                    expect.append((r, obs, tuple(orc.repair(obs))))
                elif m in demoted:  # the demoted master's own maps and list
                    cur = orc.export_files()
                    orc.import_files(*demoted[m])
                    orc.set_master(m)
                    expect.append((r, obs, tuple(orc.repair(obs))))
                    demoted[m] = orc.export_files()
                    orc.import_files(*cur)
                    orc.set_master(master)
                else:
                    expect.append((r, obs, ()))
        assert cl.elections and cl.elections[0][1] == 1 and cl.master == 1 == master
        assert 0 in cl._demoted and 0 in demoted
        routed = [(r, o) for r, o, _ in expect if int(tally.mview[o]) == 0]
        assert len(routed) >= 10, routed  # the stale master answered most repairs
        assert any(p for r, o, p in expect if int(tally.mview[o]) == 0)  # ... with real plans
        assert cl.plans == expect
        for a, b in zip(eng.export_files(), orc.export_files()):
            np.testing.assert_array_equal(a, b)
        for a, b in zip(cl._demoted[0][1], demoted[0]):
            np.testing.assert_array_equal(a, b)
    finally:
        eng.close()
        orc.close()
