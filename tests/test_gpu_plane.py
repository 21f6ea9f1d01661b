"""Sender snapshot plane (csrc/gh_internal.h `pl`, DESIGN.md "Sender plane"):
pull-mode rounds with 3 <= k <= 4 gather 4-bit lag codes of the senders'
snapshots instead of their 16-bit segments, and fall back to the 16-bit
gathers per wave when a code is outside the plane's window. These tests pin
that the plane is in use where it should be, that its fallbacks happen and
stay bit-exact against the oracle, and that it changes no result against the
16-bit gather path (GH_PLANE=0) or another tile width. Run on a MI355X:
pytest -m gpu."""
import numpy as np
import pytest

import scenarios as sc
from test_gpu_parity import compare

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gs():
    import gossipsim
    return gossipsim


@pytest.fixture(autouse=True)
def plane_on(monkeypatch):
    """The plane is kept from N=16,384 on by default; these small clusters
    keep it through GH_PLANE=1."""
    monkeypatch.setenv("GH_PLANE", "1")


def test_plane_steady_state_used(gs, oracle_mod):
    """N=2,048, k=4 pull from full membership with the bench's timeouts:
    the plane is kept, valid from the second round on except after events,
    and the healthy rounds take no fallback; bit-exact every round."""
    n = 2048
    cfg = dict(fanout=4, seed=0x5EED0007, t_fail=16, t_cleanup=16)
    eng = gs.Engine(gs.default_config(n, **cfg))
    orc = oracle_mod.Oracle(oracle_mod.default_config(n, **cfg), threads=8)
    hb, ts, alive = sc.full_state(n)
    eng.import_state(hb, ts, alive, 0)
    orc.import_state(hb, ts, alive, 0)
    assert eng.plane_info()[:2] == (1, 0)  # an import leaves no valid plane
    sched = {14: [(sc.CRASH, 7), (sc.LEAVE, 1500)], 18: [(sc.JOIN, 1500)]}
    fb_steady = []
    for r in range(1, 31):
        ev = sched.get(r, [])
        if ev:
            eng.apply_events(ev)
            orc.apply_events(ev)
        s1, s2 = eng.step(1), orc.step(1)
        assert s1 == s2, f"round {r}: gpu {s1} != cpu {s2}"
        compare(eng, orc, r)
        en, valid, fb = eng.plane_info()
        assert en == 1 and valid == 1, (r, en, valid)
        if 8 <= r < 14:
            fb_steady.append(fb)
    assert fb_steady == [0] * len(fb_steady), fb_steady


def lagging_state(n, seed):
    """Owners at 1,000 + small; views lagging by 0..40 rounds (outside the
    plane's 13-round window: "older" codes), and members whose own counter
    sits a few below everyone's view of it (a restart: views ahead of the
    owner, "unknown" codes), all within the narrow window so the lean
    variant runs."""
    rng = np.random.default_rng(seed)
    own = 1000 + rng.integers(0, 5, n)
    hb = own[None, :] - rng.integers(0, 41, (n, n))
    ahead = np.arange(n) % 97 == 3
    hb[:, ahead] = own[ahead][None, :] + rng.integers(1, 9, (n, int(ahead.sum())))
    np.fill_diagonal(hb, own)
    ts = np.zeros((n, n), np.int32)
    return hb.astype(np.int32), ts, np.ones(n, np.uint8)


@pytest.mark.parametrize("k", [3, 4])
def test_plane_fallback_exact(gs, oracle_mod, k, monkeypatch):
    """Views far outside the plane's window force 16-bit gathers (fallback
    waves > 0) while the plane is valid; every round stays bit-exact. (The
    8-bit tier's byte path sends such rows to the per-cell kernel instead:
    GH_C8=0 here; tests/test_gpu_tier8.py covers the tier.)"""
    monkeypatch.setenv("GH_C8", "0")
    n = 1024
    cfg = dict(fanout=k, seed=0x5EED0100 + k, t_fail=60, t_cleanup=60)
    eng = gs.Engine(gs.default_config(n, **cfg))
    orc = oracle_mod.Oracle(oracle_mod.default_config(n, **cfg), threads=8)
    hb, ts, alive = lagging_state(n, k)
    eng.import_state(hb, ts, alive, 0)
    orc.import_state(hb, ts, alive, 0)
    fbs = []
    for r in range(1, 16):
        s1, s2 = eng.step(1), orc.step(1)
        assert s1 == s2, f"round {r}: gpu {s1} != cpu {s2}"
        compare(eng, orc, r)
        en, valid, fb = eng.plane_info()
        assert en == 1 and valid == 1
        fbs.append((fb, eng.encoding_info(full=True)))
    assert fbs[0][0] == 0, fbs  # round 1 read no plane (the import invalidated it)
    assert sum(f for f, _ in fbs[1:]) > 0, fbs


def run_states(gs, n, cfg, sched, rounds, init):
    eng = gs.Engine(gs.default_config(n, **cfg))
    eng.import_state(*init, 0)
    out = []
    for r in range(1, rounds + 1):
        ev = sched.get(r, [])
        if ev:
            eng.apply_events(ev)
        st = eng.step(1)
        out.append((st, eng.export_state(), eng.read_failed(), eng.read_detectors()))
    info = eng.plane_info()
    eng.close()
    return out, info


@pytest.mark.parametrize("env", [{"GH_PLANE": "0", "GH_TILE_W": "256"}, {"GH_TILE_W": "64"}],
                         ids=["gather16_tw256", "plane_tw64"])
def test_plane_matches_gather_path(gs, monkeypatch, env):
    """Seeded churn with detections (T_fail 6): the plane at TW=256 gives the
    same tables, counters, failed sets and detectors every round as the
    16-bit gathers at the same layout and as the plane at TW=64."""
    n = 1536
    cfg = dict(fanout=4, seed=0x5EED0200, t_fail=6, t_cleanup=8)
    sched = sc.random_churn(n, 36, 0x77, p_crash=0.01, p_leave=0.005, p_join=0.02)
    init = sc.full_state(n)
    monkeypatch.setenv("GH_TILE_W", "256")
    base, info = run_states(gs, n, cfg, sched, 36, init)
    assert info[0] == 1
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    other, info2 = run_states(gs, n, cfg, sched, 36, init)
    assert info2[0] == (0 if env.get("GH_PLANE") == "0" else 1)
    for r, (a, b) in enumerate(zip(base, other), 1):
        assert a[0] == b[0], (r, a[0], b[0])
        for x, y in zip(a[1], b[1]):
            np.testing.assert_array_equal(x, y, err_msg=f"round {r}")
        np.testing.assert_array_equal(a[2], b[2])
        np.testing.assert_array_equal(a[3], b[3])


@pytest.mark.parametrize("detect_mode", [0, 1], ids=["canonical", "quirk"])
def test_plane_churn_parity(gs, oracle_mod, detect_mode):
    """Seeded crash/leave/join churn with detections in both detection modes
    (quirk mode's pre-pass clears flags in place and invalidates the plane):
    bit-exact against the oracle every round with the plane kept."""
    from test_gpu_parity import run_parity
    n = 700
    sched = sc.random_churn(n, 40, 0x99 + detect_mode, p_crash=0.02, p_leave=0.01, p_join=0.04)
    eng, _ = run_parity(gs, oracle_mod, dict(fanout=4, seed=0x5EED0300 + detect_mode, t_fail=4, t_cleanup=6,
                                             detect_mode=detect_mode), n, 40, sched, init=sc.full_state(n))
    assert eng.plane_info()[0] == 1


@pytest.mark.parametrize("world", [2, 3])
def test_plane_sharded_parity(gs, oracle_mod, world):
    """Column shards (in-process transport) each keep the plane of their own
    columns; seeded churn is bit-exact against the oracle every round."""
    from test_gpu_sharded import run_group
    n = 1100
    sched = sc.random_churn(n, 30, 0xA0 + world, p_crash=0.01, p_leave=0.01, p_join=0.03)
    run_group(gs, oracle_mod, world, dict(fanout=3, seed=0x5EED0400 + world, t_fail=5, t_cleanup=7), n, 30, sched,
              init=sc.full_state(n))
