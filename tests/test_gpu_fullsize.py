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

Counters, the failed set and the detectors are compared every round; the
whole hb and ts tables (65,536 x 65,536 each) row block by row block at the
rounds listed."""
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


def run(gs, om, t_fail, rounds, full_at, expect):
    cfg = dict(fanout=4, seed=0x5EED0003, t_fail=t_fail, t_cleanup=t_fail)
    eng = gs.Engine(gs.default_config(N, **cfg))
    orc = om.Oracle(om.default_config(N, **cfg), threads=THREADS)
    try:
        eng.init_full(2, 0, 0)
        orc.init_full(2, 0, 0)
        seen = {"detections": 0, "storm": False}
        for r in range(1, rounds + 1):
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
            seen["storm"] |= eng.encoding_info(full=True)[2] == 1
            if r in full_at:
                compare_blocks(eng, orc, r)
        expect(seen)
    finally:
        eng.close()
        orc.close()


def test_c3_fullsize_steady_state(gs, oracle_mod):
    """The bench's workload (T_fail = 16): 6 rounds, no detections."""
    run(gs, oracle_mod, 16, 6, {3, 6}, lambda s: s["detections"] == 0 or pytest.fail("unexpected detections"))


def test_c3_fullsize_reference_timeouts(gs, oracle_mod):
    """T_fail = T_cleanup = 5 (slave/slave.go:24-25) through the round-6
    detection storm and the collapse: the storm variant runs at N=65,536."""
    def expect(s):
        assert s["detections"] > 0 and s["storm"]
    run(gs, oracle_mod, 5, 9, {6, 7, 9}, expect)
