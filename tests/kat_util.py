"""Run the App. B KAT fixtures (tests/golden/kats.json) on any engine with the
gh_* call shapes (oracle.Oracle or gossipsim.Engine)."""
import json
import pathlib

import numpy as np

KATS = json.loads((pathlib.Path(__file__).parent / "golden" / "kats.json").read_text())


def kat_config(mod, k):
    return mod.default_config(k["n"], peer_mode=k["peer_mode"], fanout=k["fanout"],
                              detect_mode=k["detect_mode"], seed=k["seed"], t_fail=k["t_fail"],
                              t_cleanup=k["t_cleanup"])


def run_kat(engine, k):
    engine.import_state(np.array(k["hb"], np.int32), np.array(k["ts"], np.int32),
                        np.array(k["alive"], np.uint8), k["round"])
    st = engine.step(k.get("rounds", 1))
    hb, ts, _ = engine.export_state()
    i = k["expect_row"]
    if k["expect_hb"] is not None:
        assert list(hb[i]) == k["expect_hb"], (k["name"], list(hb[i]))
        exp_ts = np.array(k["expect_ts"])
        keep = np.array(k["expect_hb"]) != -1
        assert list(ts[i][keep]) == list(exp_ts[keep]), (k["name"], list(ts[i]))
    for key, v in k["expect_stats"].items():
        assert st[key] == v, (k["name"], key, st[key], v)
    if k.get("rounds", 1) == 1:
        bm = engine.read_failed()
        failed = [c for c in range(k["n"]) if bm[c >> 5] >> (c & 31) & 1]
        assert failed == k["expect_failed"], (k["name"], failed)
        assert list(engine.read_detectors()) == k["expect_detectors"]
    return st
