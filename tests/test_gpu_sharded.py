"""GPU parity of the column-sharded engine (DESIGN.md "Multi-GPU"): one
cluster split over G shards must give the oracle's results bit for bit —
hb, ts, alive, failed set, detectors, per-round counters, placement — for
every G, in pull and ring mode, under churn. The shards run as threads of
this process on one MI355X (GH_COMM_LOCAL: same code path as RCCL, the
collectives are in-process copies); the RCCL transport itself is checked at
world 1 (one rank, real communicator). Run on a MI355X: pytest -m gpu."""
import numpy as np
import pytest

import scenarios as sc
from kat_util import KATS_SHARDED, kat_config, run_kat

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gs():
    import gossipsim
    return gossipsim


def compare(eng, orc, r):
    from test_gpu_parity import check_counts
    check_counts(eng, r)
    h1, t1, a1 = eng.export_state()
    h2, t2, a2 = orc.export_state()
    np.testing.assert_array_equal(a1, a2, err_msg=f"alive r={r}")
    bad = np.argwhere(h1 != h2)
    assert bad.size == 0, f"hb r={r}: {len(bad)} cells differ, first {bad[:5].tolist()}"
    np.testing.assert_array_equal(t1, t2, err_msg=f"ts r={r}")
    np.testing.assert_array_equal(eng.read_failed(), orc.read_failed(), err_msg=f"failed r={r}")
    np.testing.assert_array_equal(eng.read_detectors(), orc.read_detectors(), err_msg=f"detectors r={r}")


def run_group(gs, om, world, cfg_kw, n, rounds, sched, init=None, every=1, files=None, per_round=None):
    grp = gs.ShardGroup(gs.default_config(n, **cfg_kw), world)
    orc = om.Oracle(om.default_config(n, **cfg_kw), threads=8)
    try:
        if init is not None:
            grp.import_state(*init, 0)
            orc.import_state(*init, 0)
        for r in range(1, rounds + 1):
            ev = sched.get(r, [])
            if ev:
                grp.apply_events(ev)
                orc.apply_events(ev)
            s1, s2 = grp.step(1), orc.step(1)
            assert s1 == s2, f"G={world} round {r}: gpu {s1} != cpu {s2}"
            if files is not None and r in files:
                f = np.asarray(files[r], np.int32)
                for x, y in zip(grp.put(f), orc.put(f)):
                    np.testing.assert_array_equal(x, y)
                for obs in orc.read_detectors()[:2]:
                    assert grp.repair(int(obs)) == orc.repair(int(obs))
            if r % every == 0 or r == rounds or ev:
                compare(grp, orc, r)
            if per_round:
                per_round(grp, r)
    finally:
        grp.close()


def test_shard_layout(gs):
    grp = gs.ShardGroup(gs.default_config(100), 3)
    try:
        info = grp.run("shard_info")
        assert [x[:2] for x in info] == [(0, 3), (1, 3), (2, 3)]
        assert [x[2] for x in info] == [0, 64, 128] and [x[3] for x in info] == [64, 36, 0]
    finally:
        grp.close()


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("k", KATS_SHARDED, ids=lambda k: k["name"])
def test_kats_sharded(gs, k, world):
    grp = gs.ShardGroup(kat_config(gs, k), world)
    try:
        run_kat(grp, k)
    finally:
        grp.close()


@pytest.mark.parametrize("world,peer_mode", [(2, 0), (3, 1), (4, 0), (2, 1)])
def test_c1_bootstrap_crash_places_sharded(gs, oracle_mod, world, peer_mode):
    """BASELINE config 1 over G shards: joins, 10 files, crash, repairs."""
    n = 10
    sched = sc.bootstrap_schedule(n)
    sched.setdefault(30, []).append((sc.CRASH, 7))
    files = {20: list(range(10))}
    for r in range(31, 61):
        files[r] = []
    run_group(gs, oracle_mod, world, dict(peer_mode=peer_mode, max_files=16, seed=0x5EED0001), n, 60, sched,
              files=files)


@pytest.mark.parametrize("world,n,peer_mode,seed", [(2, 64, 0, 3), (2, 64, 1, 4), (3, 300, 0, 5), (4, 257, 1, 6),
                                                    (5, 200, 0, 7), (8, 300, 0, 8)])
def test_random_churn_sharded(gs, oracle_mod, world, n, peer_mode, seed):
    sched = sc.random_churn(n, 30, seed, p_crash=0.03, p_leave=0.01, p_join=0.05)
    run_group(gs, oracle_mod, world, dict(peer_mode=peer_mode, fanout=3, seed=0x77 + seed), n, 30, sched,
              init=sc.full_state(n))


@pytest.mark.parametrize("world,n,peer_mode", [(2, 64, 1), (3, 300, 0), (4, 257, 1)])
def test_quirk_detection_sharded(gs, oracle_mod, world, n, peer_mode):
    """Quirk-mode run parity carried across shard boundaries (the runs of
    candidates continue from one shard's columns into the next)."""
    sched = sc.random_churn(n, 30, 40 + world, p_crash=0.08, p_leave=0.02, p_join=0.05)
    run_group(gs, oracle_mod, world, dict(peer_mode=peer_mode, fanout=3, seed=0x3000 + n, detect_mode=1, t_fail=3,
                                          t_cleanup=5), n, 30, sched, init=sc.full_state(n))


@pytest.mark.parametrize("world", [2, 4])
def test_storm_short_timeouts_sharded(gs, oracle_mod, world):
    """Short timeouts at N=700: failure storms (|D| above the recount list),
    the guard flipping rows, tombstones surviving detection."""
    n = 700
    sched = sc.random_churn(n, 24, 21, p_crash=0.04, p_leave=0.01, p_join=0.05)
    run_group(gs, oracle_mod, world, dict(fanout=4, seed=0x31, t_fail=2, t_cleanup=6), n, 24, sched,
              init=sc.full_state(n), every=4)


def test_c2_n4096_sharded(gs, oracle_mod):
    """BASELINE config 2 (N=4,096, k=3, 1% crash at r=8) over 4 shards."""
    n = 4096
    sched = {8: [(sc.CRASH, c) for c in sc.crash_ids(n, 0.01, 0x5EED0002)]}
    run_group(gs, oracle_mod, 4, dict(fanout=3, seed=0x5EED0002), n, 24, sched, init=sc.full_state(n), every=8)


def test_placement_sharded(gs, oracle_mod):
    n, F = 512, 5000
    cfg = dict(max_files=F, seed=0x5EED0005)
    grp = gs.ShardGroup(gs.default_config(n, **cfg), 3)
    orc = oracle_mod.Oracle(oracle_mod.default_config(n, **cfg))
    try:
        hb, ts, alive = sc.full_state(n)
        grp.import_state(hb, ts, alive, 3)
        orc.import_state(hb, ts, alive, 3)
        f = np.random.default_rng(0).permutation(F)[: F // 2].astype(np.int32)
        for x, y in zip(grp.put(f), orc.put(f)):
            np.testing.assert_array_equal(x, y)
        sched = {1: [(sc.CRASH, c) for c in sc.crash_ids(n, 0.05, 0x5EED0005)]}
        for r in range(1, 12):
            if r in sched:
                grp.apply_events(sched[r])
                orc.apply_events(sched[r])
            assert grp.step(1) == orc.step(1)
        for obs in (0, 5, 300):
            assert grp.repair(obs) == orc.repair(obs)
        for x, y in zip(grp.get_files(np.arange(F)), orc.get_files(np.arange(F))):
            np.testing.assert_array_equal(x, y)
        for obs in (0, 511):
            for x, y in zip(grp.lsm(obs), orc.lsm(obs)):
                np.testing.assert_array_equal(x, y)
    finally:
        grp.close()


def test_rccl_transport_world1(gs, oracle_mod):
    """The RCCL transport (dlopen'd librccl, real communicator of one rank)
    gives the oracle's results."""
    n = 300
    uid = gs.comm_unique_id()
    assert len(uid) == 128
    cfg = dict(fanout=3, seed=0x44, peer_mode=1)
    eng = gs.Engine(gs.default_config(n, **cfg), rank=0, world=1, transport=gs.GH_COMM_RCCL, comm_id=uid)
    orc = oracle_mod.Oracle(oracle_mod.default_config(n, **cfg))
    init = sc.full_state(n)
    eng.import_state(*init, 0)
    orc.import_state(*init, 0)
    sched = sc.random_churn(n, 16, 9, p_crash=0.03)
    for r in range(1, 17):
        if r in sched:
            eng.apply_events(sched[r])
            orc.apply_events(sched[r])
        assert eng.step(1) == orc.step(1)
    compare(eng, orc, 16)
    eng.close()


def test_n65536_sharded_matches_single(gs):
    """N=65,536 (BASELINE config 3 scale) over 2 shards on one GPU
    (2 x 24 GiB) against the single-engine run: identical counters every
    round and identical sampled rows."""
    n, rounds = 65536, 6
    cfg = gs.default_config(n, fanout=4, seed=0x5EED0003, t_fail=16, t_cleanup=16)
    crashed = sc.crash_ids(n, 0.01, 0x5EED0003)
    grp = gs.ShardGroup(cfg, 2)
    grp.init_full(2, 0, 0)
    res_g = []
    for r in range(rounds):
        if r == 2:
            grp.apply_events([(sc.CRASH, c) for c in crashed])
        res_g.append(grp.step(1))
    rows_g = [grp.export_state(int(i), 1) for i in (0, 777, 65535)]
    grp.close()
    eng = gs.Engine(cfg)
    eng.init_full(2, 0, 0)
    for r in range(rounds):
        if r == 2:
            eng.apply_events([(sc.CRASH, c) for c in crashed])
        assert eng.step(1) == res_g[r], r
    for i, rg in zip((0, 777, 65535), rows_g):
        for x, y in zip(eng.export_state(i, 1), rg):
            np.testing.assert_array_equal(x, y)
    eng.close()


def test_merge_list_sharded(gs, oracle_mod):
    """gh_merge_list over 3 shards: each shard merges the members of its
    columns; counts summed over ranks."""
    n = 150
    cfg = dict(fanout=3, seed=0x4E)
    grp = gs.ShardGroup(gs.default_config(n, **cfg), 3)
    orc = oracle_mod.Oracle(oracle_mod.default_config(n, **cfg))
    try:
        init = sc.full_state(n)
        grp.import_state(*init, 0)
        orc.import_state(*init, 0)
        rng = np.random.default_rng(9)
        for r in range(1, 9):
            assert grp.step(1) == orc.step(1)
            ids = rng.permutation(n)[:60].astype(np.int32)
            hb = rng.integers(0, 3 * r + 4, 60).astype(np.int32)
            obs = int(rng.integers(0, n))
            assert grp.merge_list(obs, ids, hb) == orc.merge_list(obs, ids, hb)
            compare(grp, orc, r)
    finally:
        grp.close()


def test_c5_churn_rereplication_sharded(gs, oracle_mod):
    """Config 5 shape (2^20 files, join/leave/crash waves, repairs at
    detection + 8) over 2 shards, the file table sharded by file ID (file f on
    shard f % 2, master/master.go:74-150 is per file): each shard holds and
    places 2^19 files, the puts, repair plans and lookups equal the oracle's."""
    from test_gpu_parity import c5_run
    n, F = 1024, 1 << 20
    cfg = dict(fanout=4, seed=0x5EED0015, max_files=F, t_fail=8, t_cleanup=8)
    grp = gs.ShardGroup(gs.default_config(n, **cfg), 2)
    orc = oracle_mod.Oracle(oracle_mod.default_config(n, **cfg), threads=8)
    try:
        hb, ts, alive = sc.full_state(n)
        alive[n - n // 100:] = 0
        hb[:, n - n // 100:] = -1
        hb[n - n // 100:, :] = -1
        grp.import_state(hb, ts, alive, 0)
        orc.import_state(hb, ts, alive, 0)
        assert c5_run(grp, orc, n, F) > 0
        info = grp.run("file_info")
        assert [x["slots"] for x in info] == [F // 2, F // 2]
        assert [x["shards"] for x in info] == [2, 2]
        assert [x["held"] for x in info] == [F // 2, F // 2]
    finally:
        grp.close()


@pytest.mark.parametrize("world", [3, 5])
def test_file_shards_uneven(gs, oracle_mod, world):
    """File-ID sharding with a file count no shard count divides (1,000
    files): puts in two batches with repeats of earlier files, a crash wave,
    repairs from two observers, gets, conflicts and deletes equal the
    oracle's; every shard holds ceil(1000 / G) slots and its own files."""
    n, F = 96, 1000
    cfg = dict(fanout=3, seed=0x5EED0019, max_files=F, t_fail=4, t_cleanup=6)
    grp = gs.ShardGroup(gs.default_config(n, **cfg), world)
    orc = oracle_mod.Oracle(oracle_mod.default_config(n, **cfg))
    try:
        hb, ts, alive = sc.full_state(n)
        grp.import_state(hb, ts, alive, 0)
        orc.import_state(hb, ts, alive, 0)
        f1 = np.arange(0, 700, dtype=np.int32)
        f2 = np.arange(500, F, dtype=np.int32)  # 500..699 put again
        for batch in (f1, f2):
            for x, y in zip(grp.put(batch), orc.put(batch)):
                np.testing.assert_array_equal(x, y)
        ev = [(sc.CRASH, c) for c in sc.crash_ids(n, 0.1, 0x5EED0019)]
        grp.apply_events(ev)
        orc.apply_events(ev)
        for r in range(1, 13):
            assert grp.step(1) == orc.step(1), r
        for obs in (0, 7):
            assert grp.repair(obs) == orc.repair(obs), obs
        allf = np.arange(F, dtype=np.int32)
        for x, y in zip(grp.get_files(allf), orc.get_files(allf)):
            np.testing.assert_array_equal(x, y)
        np.testing.assert_array_equal(grp.put_conflicts(allf), orc.put_conflicts(allf))
        gone = np.arange(0, F, 7, dtype=np.int32)
        np.testing.assert_array_equal(grp.delete_files(gone), orc.delete_files(gone))
        for x, y in zip(grp.get_files(allf), orc.get_files(allf)):
            np.testing.assert_array_equal(x, y)
        info = grp.run("file_info")
        slots = -(-F // world)
        kept = set(range(F)) - set(gone.tolist())
        for g, x in enumerate(info):
            assert (x["slots"], x["shards"]) == (slots, world)
            assert x["held"] == sum(1 for f in kept if f % world == g)
    finally:
        grp.close()
        orc.close()
