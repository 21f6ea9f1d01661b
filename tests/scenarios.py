"""Deterministic churn scenarios shared by the CPU (oracle cross-check) and GPU
(parity) tests. A scenario is a list of per-round event batches; engines expose
apply_events(list[(kind, member)]) and step(1)."""
from __future__ import annotations

import numpy as np

from oracle import philox

JOIN, LEAVE, CRASH = 1, 2, 3


def bootstrap_schedule(n, start=1):
    """C1-style start: member r-start joins in round r (0 first: the
    introducer joins through itself, slave/slave.go:288 + :228)."""
    return {start + c: [(JOIN, c)] for c in range(n)}


def random_churn(n, rounds, seed, p_crash=0.04, p_leave=0.02, p_join=0.05, start_full=True):
    """Per-round batches of crash/leave/join events on a seeded stream."""
    rng = np.random.default_rng(seed)
    alive = np.ones(n, bool) if start_full else np.zeros(n, bool)
    sched = {}
    for r in range(1, rounds + 1):
        ev = []
        for c in range(1, n):  # keep the introducer alive so joins can happen
            u = rng.random()
            if alive[c] and u < p_crash:
                ev.append((CRASH, c))
                alive[c] = False
            elif alive[c] and u < p_crash + p_leave:
                ev.append((LEAVE, c))
                alive[c] = False
            elif not alive[c] and u < p_join:
                ev.append((JOIN, c))
                alive[c] = True
        if ev:
            sched[r] = ev
    return sched


def rejoin_churn(n, rounds, seed, p_out=0.06, p_back=0.5):
    """Members leave (or crash) and come back within a few rounds, again and
    again: the introducer (member 0) still holds the tombstone of a member
    when it rejoins, so its list holds the member twice (SPEC D7), and a
    later LEAVE, REMOVE or detection meets that double entry."""
    rng = np.random.default_rng(seed)
    alive = np.ones(n, bool)
    sched = {}
    for r in range(1, rounds + 1):
        ev = []
        for c in range(1, n):
            u = rng.random()
            if alive[c] and u < p_out:
                ev.append((LEAVE if rng.random() < 0.6 else CRASH, c))
                alive[c] = False
            elif not alive[c] and u < p_back:
                ev.append((JOIN, c))
                alive[c] = True
        if ev:
            sched[r] = ev
    return sched


def crash_ids(n, frac, seed):
    """BASELINE configs: crash `frac` of N, IDs drawn by Philox(seed, CRASH);
    the introducer/master (0) is excluded."""
    count = max(1, int(round(n * frac)))
    return philox.sample_distinct(seed, philox.TAG_CRASH, count, n, exclude=(0,))


def full_state(n, hb0=2, ts0=0):
    hb = np.full((n, n), hb0, np.int32)
    ts = np.full((n, n), ts0, np.int32)
    alive = np.ones(n, np.uint8)
    return hb, ts, alive


def masked(hb, ts):
    """ts of absent cells carries no meaning in the list model (listsim keeps
    no Member for them); compare it only where hb != -1."""
    t = ts.copy()
    t[hb == -1] = 0
    return hb, t


def export_view(hb, ts, round_, t_cleanup):
    """A dense (hb, ts) state as gh_export_state / or_export_state present it
    (SPEC.md §1): ts 0 for absent cells, and with T_cleanup < 30 a tombstone
    older than T_cleanup + 1 rounds at exactly T_cleanup + 1 rounds (round_ =
    last completed)."""
    t = ts.astype(np.int64).copy()
    t[hb == -1] = 0
    if t_cleanup < 30:
        now = round_ + 1
        old = (hb == -2) & (now - t > t_cleanup + 1)
        t[old] = now - (t_cleanup + 1)
    return hb, t.astype(np.int32)
