"""ORACLE / TEST INFRASTRUCTURE ONLY.

ctypes wrapper around oracle/_build/liboracle.so (tablesim.c, the C
restatement of the reference's gossip/detect/placement logic, SPEC.md).
Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this module; the product package never does.
"""
from __future__ import annotations

import ctypes as C
import os
import pathlib
import subprocess

import numpy as np

HERE = pathlib.Path(__file__).resolve().parent
LIB_PATH = HERE / "_build" / "liboracle.so"

GH_OK = 0
GH_EINVAL = -1
GH_EPLACEMENT_STARVED = -5
GH_ERANGE = -6
GH_PEER_PULL, GH_PEER_RING = 0, 1
GH_DETECT_CANONICAL, GH_DETECT_QUIRK = 0, 1
GH_REMOVE_ALL, GH_REMOVE_LIST = 0, 1
GH_EV_JOIN, GH_EV_LEAVE, GH_EV_CRASH = 1, 2, 3


class Config(C.Structure):
    _fields_ = [
        ("n_members", C.c_int32), ("fanout", C.c_int32), ("peer_mode", C.c_int32),
        ("detect_mode", C.c_int32), ("t_fail", C.c_int32), ("t_cleanup", C.c_int32),
        ("min_members", C.c_int32), ("replicas", C.c_int32), ("introducer", C.c_int32),
        ("master", C.c_int32), ("device", C.c_int32), ("tile_width", C.c_int32),
        ("seed", C.c_uint64), ("max_files", C.c_int64), ("wide_segments", C.c_int64),
        ("shard_layout", C.c_int32), ("list_order", C.c_int32), ("remove_mode", C.c_int32),
        ("reserved", C.c_int32 * 3),
    ]


class Event(C.Structure):
    _fields_ = [("kind", C.c_int32), ("member", C.c_int32)]


class Stats(C.Structure):
    _fields_ = [(n, C.c_int64) for n in (
        "rounds", "last_round", "detections", "failed_members", "remove_unknown",
        "ring_empty", "active_rows", "merged_cells", "released", "tombstoned")]

    def as_dict(self):
        return {n: getattr(self, n) for n, _ in self._fields_}


class PlanEntry(C.Structure):
    _fields_ = [("file", C.c_int32), ("node1", C.c_int32), ("version", C.c_int32),
                ("n_new", C.c_int32), ("status", C.c_int32), ("new_nodes", C.c_int32 * 8)]


def default_config(n, **kw) -> Config:
    cfg = Config()
    cfg.n_members = n
    cfg.fanout = 3
    cfg.peer_mode = GH_PEER_PULL
    cfg.detect_mode = GH_DETECT_CANONICAL
    cfg.t_fail = 5
    cfg.t_cleanup = 5
    cfg.min_members = 4
    cfg.replicas = 4
    cfg.introducer = 0
    cfg.master = 0
    cfg.device = 0
    cfg.seed = 0x5EED0001
    cfg.max_files = 0
    for k, v in kw.items():
        setattr(cfg, k, v)
    return cfg


def build() -> None:
    subprocess.run(["make", "-s", "-C", str(HERE)], check=True)


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not LIB_PATH.exists():
            build()
        L = C.CDLL(str(LIB_PATH))
        vp, i32, i64 = C.c_void_p, C.c_int32, C.c_int64
        P = C.POINTER
        L.or_create.argtypes = [P(Config), i64, P(vp)]
        L.or_destroy.argtypes = [vp]
        L.or_last_error.argtypes = [vp]
        L.or_last_error.restype = C.c_char_p
        L.or_set_threads.argtypes = [vp, C.c_int]
        L.or_import_state.argtypes = [vp, vp, vp, vp, i64, i64, i32]
        L.or_export_state.argtypes = [vp, vp, vp, vp, i64, i64]
        L.or_init_full.argtypes = [vp, i32, i32, i32]
        L.or_get_round.argtypes = [vp, P(i32)]
        L.or_apply_events.argtypes = [vp, P(Event), i64]
        L.or_step.argtypes = [vp, i32, P(Stats)]
        L.or_read_failed.argtypes = [vp, vp, i64]
        L.or_read_detectors.argtypes = [vp, vp, i64, P(i64)]
        L.or_lsm.argtypes = [vp, i32, vp, vp, vp, i64, P(i64)]
        L.or_merge_list.argtypes = [vp, i32, vp, vp, i64, P(i64)]
        L.or_put.argtypes = [vp, vp, i64, vp, vp, vp]
        L.or_repair.argtypes = [vp, i32, P(PlanEntry), i64, P(i64)]
        L.or_put_conflicts.argtypes = [vp, vp, i64, i32, vp]
        L.or_get_files.argtypes = [vp, vp, i64, vp, vp]
        L.or_delete_files.argtypes = [vp, vp, i64, vp]
        L.or_export_files.argtypes = [vp, vp, vp, vp, vp]
        L.or_import_files.argtypes = [vp, vp, vp, vp, vp]
        L.or_set_master.argtypes = [vp, i32]
        L.or_philox.argtypes = [vp, vp, vp]
        L.or_debug_shadow.argtypes = [vp, vp]
        _lib = L
    return _lib


def _p(a: np.ndarray):
    return a.ctypes.data_as(C.c_void_p)


def philox(ctr, key):
    c = np.asarray(ctr, dtype=np.uint32)
    k = np.asarray(key, dtype=np.uint32)
    out = np.zeros(4, dtype=np.uint32)
    lib().or_philox(_p(c), _p(k), _p(out))
    return out


class Oracle:
    """Table-semantics CPU replay (tablesim.c) with the gh_* call shapes."""

    def __init__(self, cfg: Config, rows: int | None = None, threads: int = 1):
        self.cfg = cfg
        self.n = cfg.n_members
        self.rows = rows if rows is not None else cfg.n_members
        self.R = cfg.replicas
        h = C.c_void_p()
        rc = lib().or_create(C.byref(cfg), self.rows, C.byref(h))
        if rc != 0:
            raise RuntimeError(f"or_create failed: {rc}")
        self.h = h
        lib().or_set_threads(self.h, threads)

    def close(self):
        if self.h:
            lib().or_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _chk(self, rc, ok=(0,)):
        if rc not in ok:
            raise RuntimeError(f"oracle error {rc}: {lib().or_last_error(self.h)!r}")
        return rc

    def import_state(self, hb, ts, alive, round_=0, row0=0):
        hb = np.ascontiguousarray(hb, dtype=np.int32)
        ts = np.ascontiguousarray(ts, dtype=np.int32)
        alive = np.ascontiguousarray(alive, dtype=np.uint8)
        self._chk(lib().or_import_state(self.h, _p(hb), _p(ts), _p(alive), row0, hb.shape[0], round_))

    def export_state(self, row0=0, n_rows=None):
        n_rows = self.rows - row0 if n_rows is None else n_rows
        hb = np.empty((n_rows, self.n), np.int32)
        ts = np.empty((n_rows, self.n), np.int32)
        alive = np.empty(n_rows, np.uint8)
        self._chk(lib().or_export_state(self.h, _p(hb), _p(ts), _p(alive), row0, n_rows))
        return hb, ts, alive

    def init_full(self, hb0=2, ts0=0, round_=0):
        self._chk(lib().or_init_full(self.h, hb0, ts0, round_))

    @property
    def round(self):
        r = C.c_int32()
        lib().or_get_round(self.h, C.byref(r))
        return r.value

    def apply_events(self, events):
        arr = (Event * len(events))(*[Event(k, m) for k, m in events])
        self._chk(lib().or_apply_events(self.h, arr, len(events)))

    def step(self, rounds=1):
        st = Stats()
        self._chk(lib().or_step(self.h, rounds, C.byref(st)))
        return st.as_dict()

    def step_rc(self, rounds=1):
        """(return code, stats of the rounds run): GH_ERANGE stops at the
        round that would pass INT32_MAX."""
        st = Stats()
        rc = lib().or_step(self.h, rounds, C.byref(st))
        return rc, st.as_dict()

    def read_failed(self):
        words = (self.n + 31) // 32
        bm = np.zeros(words, np.uint32)
        self._chk(lib().or_read_failed(self.h, _p(bm), words))
        return bm

    def read_detectors(self):
        out = np.zeros(self.rows, np.int32)
        n = C.c_int64()
        self._chk(lib().or_read_detectors(self.h, _p(out), self.rows, C.byref(n)))
        return out[: n.value]

    def lsm(self, observer):
        ids = np.zeros(self.n, np.int32)
        hb = np.zeros(self.n, np.int32)
        ts = np.zeros(self.n, np.int32)
        n = C.c_int64()
        self._chk(lib().or_lsm(self.h, observer, _p(ids), _p(hb), _p(ts), self.n, C.byref(n)))
        k = n.value
        return ids[:k], hb[:k], ts[:k]

    def debug_shadow(self):
        """int32[n]: the ts of the introducer's RecentFailList entry beside
        its present member c (SPEC D7), INT32_MIN where there is none."""
        out = np.empty(self.cfg.n_members, np.int32)
        self._chk(lib().or_debug_shadow(self.h, _p(out)))
        return out

    def merge_list(self, observer, ids, hb):
        ids = np.ascontiguousarray(ids, dtype=np.int32)
        hb = np.ascontiguousarray(hb, dtype=np.int32)
        n = C.c_int64()
        self._chk(lib().or_merge_list(self.h, observer, _p(ids), _p(hb), len(ids), C.byref(n)))
        return n.value

    def put(self, files):
        f = np.ascontiguousarray(files, dtype=np.int32)
        rep = np.zeros((len(f), self.R), np.int32)
        ver = np.zeros(len(f), np.int32)
        st = np.zeros(len(f), np.int32)
        self._chk(lib().or_put(self.h, _p(f), len(f), _p(rep), _p(ver), _p(st)), ok=(0, GH_EPLACEMENT_STARVED))
        return rep, ver, st

    def put_conflicts(self, files, window=60):
        f = np.ascontiguousarray(files, dtype=np.int32)
        out = np.zeros(len(f), np.uint8)
        self._chk(lib().or_put_conflicts(self.h, _p(f), len(f), window, _p(out)))
        return out

    def repair(self, observer, cap=None):
        cap = cap if cap is not None else max(int(self.cfg.max_files), 1)
        plan = (PlanEntry * cap)()
        n = C.c_int64()
        self._chk(lib().or_repair(self.h, observer, plan, cap, C.byref(n)), ok=(0, GH_EPLACEMENT_STARVED))
        return [plan_tuple(plan[x]) for x in range(min(n.value, cap))]

    def get_files(self, files):
        f = np.ascontiguousarray(files, dtype=np.int32)
        rep = np.zeros((len(f), self.R), np.int32)
        ver = np.zeros(len(f), np.int32)
        self._chk(lib().or_get_files(self.h, _p(f), len(f), _p(rep), _p(ver)))
        return rep, ver

    def delete_files(self, files):
        f = np.ascontiguousarray(files, dtype=np.int32)
        rep = np.zeros((len(f), self.R), np.int32)
        self._chk(lib().or_delete_files(self.h, _p(f), len(f), _p(rep)))
        return rep

    def export_files(self):
        """The master's file metadata as flat arrays (gh_export_files)."""
        F = int(self.cfg.max_files)
        rep = np.empty((F, self.R), np.int32)
        ver = np.empty(F, np.int32)
        ts = np.empty(F, np.int32)
        dr = np.empty(F, np.uint32)
        self._chk(lib().or_export_files(self.h, _p(rep), _p(ver), _p(ts), _p(dr)))
        return rep, ver, ts, dr

    def import_files(self, rep, ver, ts, dr):
        a = [np.ascontiguousarray(rep, dtype=np.int32), np.ascontiguousarray(ver, dtype=np.int32),
             np.ascontiguousarray(ts, dtype=np.int32), np.ascontiguousarray(dr, dtype=np.uint32)]
        self._chk(lib().or_import_files(self.h, *[_p(x) for x in a]))

    def set_master(self, master):
        self._chk(lib().or_set_master(self.h, int(master)))
        self.cfg.master = int(master)


def plan_tuple(e: PlanEntry):
    return (e.file, e.node1, e.version, e.status, tuple(e.new_nodes[: e.n_new]))
