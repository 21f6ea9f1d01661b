"""GPU parity of the ROW-sharded engine (GH_LAYOUT_ROWS, north_star; DESIGN.md
"Multi-GPU"): rank g owns observer rows [g*nrs, (g+1)*nrs) with every member
column, and each round the rows its receivers pull from other shards arrive
by one alltoallv (ncclAllToAllv under RCCL; peer copies under the in-process
transport used here) into ghost slots. One cluster over G shards must give
the oracle's results bit for bit: hb, ts, alive, failed set, detectors,
per-round counters, placement. Run on a MI355X: pytest -m gpu."""
import numpy as np
import pytest

import scenarios as sc
from kat_util import KATS_SHARDED, kat_config, run_kat
from test_gpu_sharded import run_group

pytestmark = pytest.mark.gpu

ROWS = 1  # GH_LAYOUT_ROWS


@pytest.fixture(scope="module")
def gs():
    import gossipsim
    return gossipsim


def rows_cfg(**kw):
    return dict(shard_layout=ROWS, **kw)


def test_row_layout_shapes(gs):
    """Shards own contiguous row ranges, every column, in pull and ring mode."""
    for pm in (gs.GH_PEER_PULL, gs.GH_PEER_RING):
        grp = gs.ShardGroup(gs.default_config(100, shard_layout=ROWS, peer_mode=pm), 3)
        try:
            assert [x[2:] for x in grp.run("shard_info")] == [(0, 100)] * 3
        finally:
            grp.close()


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("k", KATS_SHARDED, ids=lambda k: k["name"])
def test_kats_rows(gs, k, world):
    cfg = kat_config(gs, k)
    cfg.shard_layout = ROWS
    grp = gs.ShardGroup(cfg, world)
    try:
        run_kat(grp, k)
    finally:
        grp.close()


@pytest.mark.parametrize("world,n,seed", [(1, 64, 1), (2, 64, 3), (3, 300, 5), (4, 257, 6), (5, 200, 7),
                                          (8, 300, 8)])
def test_random_churn_rows(gs, oracle_mod, world, n, seed):
    """Crash / leave / join churn (freezes of owned rows, LEAVE bitmaps from
    the leaver's owner, the introducer's row broadcast as a ghost)."""
    sched = sc.random_churn(n, 30, seed, p_crash=0.03, p_leave=0.01, p_join=0.05)
    run_group(gs, oracle_mod, world, rows_cfg(fanout=3, seed=0x77 + seed), n, 30, sched, init=sc.full_state(n))


@pytest.mark.parametrize("world,n", [(2, 64), (3, 300), (4, 257)])
def test_quirk_detection_rows(gs, oracle_mod, world, n):
    """Quirk-mode runs never cross shards in the row layout (whole rows)."""
    sched = sc.random_churn(n, 30, 40 + world, p_crash=0.08, p_leave=0.02, p_join=0.05)
    run_group(gs, oracle_mod, world, rows_cfg(fanout=3, seed=0x3000 + n, detect_mode=1, t_fail=3, t_cleanup=5), n,
              30, sched, init=sc.full_state(n))


@pytest.mark.parametrize("world", [2, 4])
def test_storm_short_timeouts_rows(gs, oracle_mod, world):
    """Failure storms: D_r's counts and first detectors summed / minimised
    over the shards that detected them, REMOVE from every shard."""
    n = 700
    sched = sc.random_churn(n, 24, 21, p_crash=0.04, p_leave=0.01, p_join=0.05)
    run_group(gs, oracle_mod, world, rows_cfg(fanout=4, seed=0x31, t_fail=2, t_cleanup=6), n, 24, sched,
              init=sc.full_state(n), every=4)


def test_c1_bootstrap_crash_places_rows(gs, oracle_mod):
    """BASELINE config 1 over 3 row shards: joins through the introducer,
    10 files, a crash, repairs from the master's and the detectors' rows."""
    n = 10
    sched = sc.bootstrap_schedule(n)
    sched.setdefault(30, []).append((sc.CRASH, 7))
    files = {20: list(range(10))}
    for r in range(31, 61):
        files[r] = []
    run_group(gs, oracle_mod, 3, rows_cfg(max_files=16, seed=0x5EED0001), n, 60, sched, files=files)


def wide_state(n, seed):
    """Views far ahead of some owners' counters (restarted members): wide
    segments in every sender row, shipped with their exact cells."""
    rng = np.random.default_rng(seed)
    own = 5000 + rng.integers(0, 5, n)
    hb = own[None, :] - rng.integers(0, 4, (n, n))
    ahead = np.arange(n) % 37 == 5
    own[ahead] = 7
    hb[:, ahead] = 6000 + rng.integers(0, 5, (n, int(ahead.sum())))
    np.fill_diagonal(hb, own)
    return hb.astype(np.int32), np.zeros((n, n), np.int32), np.ones(n, np.uint8)


@pytest.mark.parametrize("world", [2, 3])
def test_wide_ghosts_rows(gs, oracle_mod, world):
    run_group(gs, oracle_mod, world, rows_cfg(fanout=4, seed=0x5EED0500 + world, t_fail=40, t_cleanup=40), 600, 12,
              {}, init=wide_state(600, world))


@pytest.mark.parametrize("world", [2, 3])
def test_plane_rows(gs, oracle_mod, monkeypatch, world):
    """The sender plane travels with the ghost rows (plane words beside the
    narrow codes) and stays exact under churn."""
    monkeypatch.setenv("GH_PLANE", "1")
    n = 1100
    sched = sc.random_churn(n, 24, 0xB0 + world, p_crash=0.01, p_leave=0.01, p_join=0.03)
    run_group(gs, oracle_mod, world, rows_cfg(fanout=4, seed=0x5EED0600 + world, t_fail=6, t_cleanup=8), n, 24,
              sched, init=sc.full_state(n))


def test_c2_n4096_rows(gs, oracle_mod):
    """BASELINE config 2 (N=4,096, k=3, 1% crash at r=8) over 4 row shards."""
    n = 4096
    sched = {8: [(sc.CRASH, c) for c in sc.crash_ids(n, 0.01, 0x5EED0002)]}
    run_group(gs, oracle_mod, 4, rows_cfg(fanout=3, seed=0x5EED0002), n, 24, sched, init=sc.full_state(n), every=8)


@pytest.mark.parametrize("direct", [1, 0])
def test_rows_match_columns_and_single(gs, monkeypatch, direct):
    """N=8,192 with the plane, 16 rounds from full membership and a crash
    wave: row shards, column shards and one engine agree every round. The
    row shards' ghost planes either gathered from their owners' tables
    (same-device shards, the default) or packed and moved by the transport's
    alltoallv (GH_GX_DIRECT=0: what RCCL ranks do)."""
    monkeypatch.setenv("GH_GX_DIRECT", str(direct))
    n = 8192
    cfg = dict(fanout=4, seed=0x5EED0700, t_fail=10, t_cleanup=10)
    sched = {5: [(sc.CRASH, c) for c in sc.crash_ids(n, 0.005, 0x5EED0701)]}

    def states(make):
        eng = make()
        try:
            eng.import_state(*sc.full_state(n), 0)
            out = []
            for r in range(1, 17):
                if r in sched:
                    eng.apply_events(sched[r])
                st = eng.step(1)
                out.append((st, eng.read_failed(), eng.export_state()[0][::97]))
            return out
        finally:
            eng.close()

    single = states(lambda: gs.Engine(gs.default_config(n, **cfg)))
    rows = states(lambda: gs.ShardGroup(gs.default_config(n, shard_layout=ROWS, **cfg), 4))
    cols = states(lambda: gs.ShardGroup(gs.default_config(n, **cfg), 4))
    for r, (a, b, c) in enumerate(zip(single, rows, cols), 1):
        assert a[0] == b[0] == c[0], (r, a[0], b[0], c[0])
        np.testing.assert_array_equal(a[1], b[1])
        np.testing.assert_array_equal(a[2], b[2])
        np.testing.assert_array_equal(a[2], c[2])


@pytest.mark.parametrize("world,n,seed", [(2, 64, 1), (3, 300, 2), (5, 200, 3), (8, 300, 4)])
def test_ring_rows(gs, oracle_mod, world, n, seed):
    """The reference's ring push (slave/slave.go:515-524) over row shards:
    each sender's owner finds its 3 targets in its own row, the targets are
    reduced, and the senders' rows travel to their receivers' owners; churn
    makes lists differ, so targets jump across shards."""
    sched = sc.random_churn(n, 30, 0x60 + seed, p_crash=0.03, p_leave=0.01, p_join=0.05)
    run_group(gs, oracle_mod, world, rows_cfg(peer_mode=gs.GH_PEER_RING, seed=0x5EED0900 + seed, t_fail=5,
                                              t_cleanup=5), n, 30, sched, init=sc.full_state(n))


def test_ring_rows_quirk(gs, oracle_mod):
    """Ring push and the reference's quirk detection over 3 row shards."""
    n = 120
    sched = sc.random_churn(n, 30, 0x6A, p_crash=0.06, p_leave=0.02, p_join=0.05)
    run_group(gs, oracle_mod, 3, rows_cfg(peer_mode=gs.GH_PEER_RING, detect_mode=1, seed=0x5EED0910, t_fail=3,
                                          t_cleanup=5), n, 30, sched, init=sc.full_state(n))


def test_ring_rows_halo(gs, oracle_mod):
    """in a healthy ring the targets of a sender are its adjacent
    members, so each row shard needs only the few rows across its two
    boundaries (a halo), not k * rows / G ghost rows."""
    n, world = 4096, 4
    cfg = rows_cfg(peer_mode=gs.GH_PEER_RING, seed=0x5EED0920, t_fail=40, t_cleanup=40)
    grp = gs.ShardGroup(gs.default_config(n, **cfg), world)
    orc = oracle_mod.Oracle(oracle_mod.default_config(n, **cfg), threads=8)
    try:
        init = sc.full_state(n)
        grp.import_state(*init, 0)
        orc.import_state(*init, 0)
        for r in range(1, 9):
            assert grp.step(1) == orc.step(1)
            for x in grp.run("exchange_info"):
                assert 0 < x["ghost_rows"] <= 4, x
        h1, t1, _ = grp.export_state()
        h2, t2, _ = orc.export_state()
        assert np.array_equal(h1, h2) and np.array_equal(t1, t2)
    finally:
        grp.close()
        orc.close()


def test_plane_only_ghosts(gs, oracle_mod, monkeypatch):
    """A healthy pull round moves only the ghosts' sender plane (0.5 B per
    cell): the 16-bit codes follow only when a segment needs the per-cell
    rule, so a storm round still moves them; parity either way."""
    monkeypatch.setenv("GH_PLANE", "1")
    n, world = 2048, 4
    cfg = rows_cfg(fanout=4, seed=0x5EED0930, t_fail=16, t_cleanup=16)
    grp = gs.ShardGroup(gs.default_config(n, **cfg), world)
    orc = oracle_mod.Oracle(oracle_mod.default_config(n, **cfg), threads=8)
    try:
        init = sc.full_state(n)
        grp.import_state(*init, 0)
        orc.import_state(*init, 0)
        ld = n  # padded columns (n is a multiple of 8 * 256)
        plane_only = 0
        for r in range(1, 21):
            if r == 12:
                ev = [(sc.CRASH, c) for c in sc.crash_ids(n, 0.02, 0x5EED0931)]
                grp.apply_events(ev)
                orc.apply_events(ev)
            assert grp.step(1) == orc.step(1), r
            for x in grp.run("exchange_info"):
                if x["ghost_rows"] and x["bytes_in"] == x["ghost_rows"] * ld // 2:
                    plane_only += 1
        h1, t1, _ = grp.export_state()
        h2, t2, _ = orc.export_state()
        assert np.array_equal(h1, h2) and np.array_equal(t1, t2)
        assert plane_only >= world * 5, plane_only  # the healthy rounds moved planes only
    finally:
        grp.close()
        orc.close()


@pytest.mark.parametrize("world,peer_mode", [(2, 0), (4, 0), (3, 1)])
def test_tier_rows(gs, oracle_mod, monkeypatch, world, peer_mode):
    """The 4-bit tier on row shards: the nibble path runs on every shard
    (tier_info variant 3) with its ghost senders' lag nibbles gathered from
    the ghost table; lane jobs that gather their senders' codes pull the
    ghosts' 16-bit codes first. A 1% crash through detection and REMOVE,
    bit-exact against the oracle every round."""
    monkeypatch.setenv("GH_PLANE", "1")
    n = 2048
    sched = {4: [(sc.CRASH, c) for c in sc.crash_ids(n, 0.01, 0x5EED0880 + world)]}
    seen = {}

    def check(grp, r):
        info = grp.run("tier_info", full=True)
        if r >= 3:
            for g, (kept, current, escaped, variant) in enumerate(info):
                assert kept == 1, (r, g, info)
                seen.setdefault(variant, set()).add(r)

    if peer_mode == 0:
        run_group(gs, oracle_mod, world, rows_cfg(fanout=4, seed=0x5EED0880 + world, t_fail=8, t_cleanup=8), n, 24,
                  sched, init=sc.full_state(n), per_round=check)
        assert seen.get(3) and len(seen[3]) >= 10, seen  # the nibble path ran on the row shards
    else:  # ring mode has no sender plane: the tier is off, the ghosts carry 16-bit codes
        run_group(gs, oracle_mod, world, rows_cfg(peer_mode=1, seed=0x5EED0890, t_fail=8, t_cleanup=8), n, 16,
                  sched, init=sc.full_state(n))
