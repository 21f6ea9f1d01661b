"""gossipsim — host facade of the MI355X gossip-membership engine.

`Engine` is a thin, 1:1 wrapper of the libgossiphip C-ABI (include/gossiphip.h).
`Cluster` keeps the reference's command vocabulary on top of it — the REPL of
slave/slave.go:546-613 (join, leave, lsm, put, get, delete, ls, store) plus
crash ("CTRL+C", README.md:30) — and the Fail_recover schedule
(slave/slave.go:1122-1133: a repair pass 8 rounds after a detection).

Every call runs on a gfx950 GPU through the HIP kernels; there is no CPU
fallback. Construction fails with GossipError(GH_ENODEV) without a device.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _abi
from ._abi import (GH_DETECT_CANONICAL, GH_DETECT_QUIRK, GH_EPLACEMENT_STARVED, GH_EV_CRASH,  # noqa: F401
                   GH_EV_JOIN, GH_EV_LEAVE, GH_OK, GH_PEER_PULL, GH_PEER_RING, Config, PlanEntry)

__all__ = ["Engine", "Cluster", "GossipError", "default_config", "Config"]


class GossipError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"{_abi.ERRORS.get(code, code)}: {msg}")
        self.code = code


def default_config(n, **kw) -> Config:
    cfg = Config()
    _abi.load().gh_config_default(C.byref(cfg))
    cfg.n_members = n
    for k, v in kw.items():
        setattr(cfg, k, v)
    return cfg


def _p(a: np.ndarray):
    return a.ctypes.data_as(C.c_void_p)


class Engine:
    """One libgossiphip handle: N members' tables resident in HBM."""

    def __init__(self, cfg: Config):
        self.lib = _abi.load()
        self.cfg = cfg
        self.n = cfg.n_members
        self.R = cfg.replicas
        h = C.c_void_p()
        rc = self.lib.gh_create(C.byref(cfg), C.byref(h))
        if rc != GH_OK:
            raise GossipError(rc, "gh_create failed (a gfx950 device is required; no CPU fallback)")
        self.h = h

    def close(self):
        if getattr(self, "h", None):
            self.lib.gh_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def _chk(self, rc, ok=(GH_OK,)):
        if rc not in ok:
            raise GossipError(rc, self.lib.gh_last_error(self.h).decode())
        return rc

    # ---- state -----------------------------------------------------------
    def import_state(self, hb, ts, alive, round_=0, row0=0):
        hb = np.ascontiguousarray(hb, dtype=np.int32)
        ts = np.ascontiguousarray(ts, dtype=np.int32)
        alive = np.ascontiguousarray(alive, dtype=np.uint8)
        self._chk(self.lib.gh_import_state(self.h, _p(hb), _p(ts), _p(alive), row0, hb.shape[0], round_))

    def export_state(self, row0=0, n_rows=None):
        n_rows = self.n - row0 if n_rows is None else n_rows
        hb = np.empty((n_rows, self.n), np.int32)
        ts = np.empty((n_rows, self.n), np.int32)
        alive = np.empty(n_rows, np.uint8)
        self._chk(self.lib.gh_export_state(self.h, _p(hb), _p(ts), _p(alive), row0, n_rows))
        return hb, ts, alive

    def init_full(self, hb0=2, ts0=0, round_=0):
        self._chk(self.lib.gh_init_full(self.h, hb0, ts0, round_))

    @property
    def round(self):
        r = C.c_int32()
        self._chk(self.lib.gh_get_round(self.h, C.byref(r)))
        return r.value

    # ---- rounds ----------------------------------------------------------
    def apply_events(self, events):
        arr = (_abi.Event * max(len(events), 1))(*[_abi.Event(k, m) for k, m in events])
        self._chk(self.lib.gh_apply_events(self.h, arr, len(events)))

    def step(self, rounds=1):
        st = _abi.RoundStats()
        self._chk(self.lib.gh_step(self.h, rounds, C.byref(st)))
        return st.as_dict()

    def read_failed(self):
        words = (self.n + 31) // 32
        bm = np.zeros(words, np.uint32)
        self._chk(self.lib.gh_read_failed(self.h, _p(bm), words))
        return bm

    def read_detectors(self):
        out = np.zeros(self.n, np.int32)
        n = C.c_int64()
        self._chk(self.lib.gh_read_detectors(self.h, _p(out), self.n, C.byref(n)))
        return out[: n.value]

    def lsm(self, observer):
        ids = np.zeros(self.n, np.int32)
        hb = np.zeros(self.n, np.int32)
        ts = np.zeros(self.n, np.int32)
        n = C.c_int64()
        self._chk(self.lib.gh_lsm(self.h, observer, _p(ids), _p(hb), _p(ts), self.n, C.byref(n)))
        k = n.value
        return ids[:k], hb[:k], ts[:k]

    # ---- files -----------------------------------------------------------
    def put(self, files):
        f = np.ascontiguousarray(files, dtype=np.int32)
        rep = np.zeros((len(f), self.R), np.int32)
        ver = np.zeros(len(f), np.int32)
        st = np.zeros(len(f), np.int32)
        self._chk(self.lib.gh_put(self.h, _p(f), len(f), _p(rep), _p(ver), _p(st)),
                  ok=(GH_OK, GH_EPLACEMENT_STARVED))
        return rep, ver, st

    def repair(self, observer, cap=None):
        cap = cap if cap is not None else max(int(self.cfg.max_files), 1)
        plan = (PlanEntry * cap)()
        n = C.c_int64()
        self._chk(self.lib.gh_repair(self.h, observer, plan, cap, C.byref(n)), ok=(GH_OK, GH_EPLACEMENT_STARVED))
        return [(e.file, e.node1, e.version, e.status, tuple(e.new_nodes[: e.n_new]))
                for e in plan[: min(n.value, cap)]]

    def get_files(self, files):
        f = np.ascontiguousarray(files, dtype=np.int32)
        rep = np.zeros((len(f), self.R), np.int32)
        ver = np.zeros(len(f), np.int32)
        self._chk(self.lib.gh_get_files(self.h, _p(f), len(f), _p(rep), _p(ver)))
        return rep, ver

    def delete_files(self, files):
        f = np.ascontiguousarray(files, dtype=np.int32)
        rep = np.zeros((len(f), self.R), np.int32)
        self._chk(self.lib.gh_delete_files(self.h, _p(f), len(f), _p(rep)))
        return rep

    # ---- tuning / timing -------------------------------------------------
    def set_round_variant(self, nontemporal=True, xcd_map=False):
        self._chk(self.lib.gh_set_round_variant(self.h, int(nontemporal), int(xcd_map)))

    def set_timing(self, enable=True):
        self._chk(self.lib.gh_set_timing(self.h, int(enable)))

    def read_timing(self):
        ms = C.c_double()
        k = C.c_int64()
        self._chk(self.lib.gh_read_timing(self.h, C.byref(ms), C.byref(k)))
        return ms.value, k.value

    def sync(self):
        self._chk(self.lib.gh_sync(self.h))


class Cluster:
    """The reference's per-node commands over one Engine (member IDs stand in
    for the VM addresses). Repairs follow Fail_recover: every row that detects
    a failure in round r triggers Update_metadata with its own list as
    `available` at round r + repair_delay (slave/slave.go:1122-1133)."""

    def __init__(self, n, repair_delay=8, **cfg_kw):
        self.engine = Engine(default_config(n, **cfg_kw))
        self.n = n
        self.repair_delay = repair_delay
        self.scheduled: dict[int, list[int]] = {}
        self.plans: list[tuple[int, int, tuple]] = []  # (round, observer, plan)

    # REPL vocabulary (slave/slave.go:546-613)
    def join(self, member):
        self.engine.apply_events([(GH_EV_JOIN, member)])

    def leave(self, member):
        self.engine.apply_events([(GH_EV_LEAVE, member)])

    def crash(self, member):
        self.engine.apply_events([(GH_EV_CRASH, member)])

    def lsm(self, member):
        ids, hb, ts = self.engine.lsm(member)
        return list(zip(ids.tolist(), hb.tolist(), ts.tolist()))

    def put(self, files):
        return self.engine.put(files)

    def get(self, files):
        return self.engine.get_files(files)

    ls = get

    def delete(self, files):
        return self.engine.delete_files(files)

    def store(self, member):
        """Files with a replica on `member` (sdfs_slave Local_files)."""
        f = np.arange(self.engine.cfg.max_files, dtype=np.int32)
        rep, ver = self.engine.get_files(f)
        return f[(ver >= 0) & (rep == member).any(axis=1)].tolist()

    def tick(self, rounds=1):
        """Run rounds one at a time, running due repair passes after each."""
        total = {}
        for _ in range(rounds):
            st = self.engine.step(1)
            for k, v in st.items():
                total[k] = total.get(k, 0) + v if k not in ("last_round",) else v
            r = self.engine.round
            if st["detections"]:
                self.scheduled.setdefault(r + self.repair_delay, []).extend(self.engine.read_detectors().tolist())
            for obs in self.scheduled.pop(r, []):
                if self.engine.cfg.max_files > 0:
                    self.plans.append((r, obs, tuple(self.engine.repair(obs))))
        return total
