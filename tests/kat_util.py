"""Run the App. B KAT fixtures (tests/golden/kats.json) on any engine with the
gh_* call shapes (oracle.Oracle or gossipsim.Engine)."""
import json
import pathlib

import numpy as np

KATS = json.loads((pathlib.Path(__file__).parent / "golden" / "kats.json").read_text())
# the reference's REMOVE recipients (GH_REMOVE_LIST) is a one-engine mode
KATS_SHARDED = [k for k in KATS if not k.get("remove_mode")]


def kat_config(mod, k):
    return mod.default_config(k["n"], peer_mode=k["peer_mode"], fanout=k["fanout"],
                              detect_mode=k["detect_mode"], seed=k["seed"], t_fail=k["t_fail"],
                              t_cleanup=k["t_cleanup"], remove_mode=k.get("remove_mode", 0))


def check_row(k, hb, ts, i, exp_hb, exp_ts):
    """row i of (hb, ts) equals exp_hb (None = not checked), ts where present"""
    for c, v in enumerate(exp_hb):
        if v is None:
            continue
        assert hb[i][c] == v, (k["name"], i, c, list(hb[i]))
        if v != -1:
            assert ts[i][c] == exp_ts[c], (k["name"], i, c, list(ts[i]))


def run_rounds(engine, k):
    """k["rounds"] rounds; events of k["sched"] ({round: [[kind, member]]})
    before their round; the stats summed over the rounds"""
    rounds = k.get("rounds", 1)
    if "sched" not in k:
        return engine.step(rounds)
    tot = None
    for r in range(k["round"] + 1, k["round"] + rounds + 1):
        ev = k["sched"].get(str(r), [])
        if ev:
            engine.apply_events([tuple(e) for e in ev])
        st = engine.step(1)
        tot = dict(st) if tot is None else {key: (v if key == "last_round" else tot[key] + v) for key, v in st.items()}
    return tot


def run_kat(engine, k):
    engine.import_state(np.array(k["hb"], np.int32), np.array(k["ts"], np.int32),
                        np.array(k["alive"], np.uint8), k["round"])
    if k["events"]:  # applied at the first round (its events phase)
        engine.apply_events([tuple(e) for e in k["events"]])
    st = run_rounds(engine, k)
    hb, ts, _ = engine.export_state()
    if k["expect_hb"] is not None:
        check_row(k, hb, ts, k["expect_row"], k["expect_hb"], k["expect_ts"])
    for m in k.get("expect_more", []):
        check_row(k, hb, ts, m["row"], m["hb"], m["ts"])
    for i, c in k.get("expect_tomb", []):
        assert hb[i][c] == -2, (k["name"], i, c, list(hb[i]))
    for key, v in k["expect_stats"].items():
        assert st[key] == v, (k["name"], key, st[key], v)
    if k.get("rounds", 1) == 1:
        bm = engine.read_failed()
        failed = [c for c in range(k["n"]) if bm[c >> 5] >> (c & 31) & 1]
        assert failed == k["expect_failed"], (k["name"], failed)
        assert list(engine.read_detectors()) == k["expect_detectors"]
    return st
