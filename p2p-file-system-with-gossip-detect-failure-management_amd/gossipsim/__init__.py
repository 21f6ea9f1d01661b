"""gossipsim — host facade of the MI355X gossip-membership engine.

`Engine` is a thin, 1:1 wrapper of the libgossiphip C-ABI (include/gossiphip.h).
`Cluster` keeps the reference's command vocabulary on top of it — the REPL of
slave/slave.go:546-613 (join, leave, lsm, put, get, delete, ls, store) plus
crash ("CTRL+C", README.md:30) — and the Fail_recover schedule
(slave/slave.go:1122-1133: a repair pass 8 rounds after a detection).

A cluster can be column-sharded over G GPUs (DESIGN.md "Multi-GPU"): one
`Engine(cfg, rank, world, GH_COMM_RCCL, comm_unique_id-from-rank-0)` per
process and GPU, every rank making the same calls (SPMD); or all G shards
driven from one process by `ShardGroup` (threads, GH_COMM_LOCAL transport, any
devices including G shards on one GPU: the sharded-path parity harness).

Every call runs on a gfx950 GPU through the HIP kernels; there is no CPU
fallback. Construction fails with GossipError(GH_ENODEV) without a device.
"""
from __future__ import annotations

import ctypes as C
import itertools
from collections import namedtuple
import os
from concurrent.futures import FIRST_EXCEPTION, ThreadPoolExecutor, wait

import numpy as np

from . import _abi, codec
from ._abi import (GH_COMM_LOCAL, GH_COMM_RCCL, GH_DETECT_CANONICAL, GH_DETECT_QUIRK,  # noqa: F401
                   GH_LAYOUT_COLUMNS, GH_LAYOUT_ROWS, GH_ORDER_APPEND, GH_ORDER_ID, GH_REMOVE_ALL, GH_REMOVE_LIST,
                   GH_EPLACEMENT_STARVED, GH_EV_CRASH, GH_EV_JOIN, GH_EV_LEAVE, GH_OK, GH_PEER_PULL,
                   GH_PEER_RING, Config, PlanEntry)

__all__ = ["Engine", "ShardGroup", "Cluster", "GossipError", "default_config", "comm_unique_id", "Config"]


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


def footprint(cfg: Config, rank: int = 0, world: int = 1, transport: int = GH_COMM_RCCL) -> dict:
    """HBM one shard of `cfg` would hold (gh_footprint: a dry walk of
    gh_create's allocations, no device needed): create_bytes (tables, plane,
    tier, arenas, per-row / per-column vectors, files) and exchange_bytes
    (the row layout's ghost-row buffers at the expected distinct senders of
    a healthy pull round; 0 for column shards)."""
    cb, xb = C.c_int64(), C.c_int64()
    rc = _abi.load().gh_footprint(C.byref(cfg), rank, world, transport, C.byref(cb), C.byref(xb))
    if rc != GH_OK:
        raise GossipError(rc, "gh_footprint failed")
    return {"create_bytes": cb.value, "exchange_bytes": xb.value, "total_bytes": cb.value + xb.value}


def comm_unique_id() -> bytes:
    """RCCL unique id for a sharded cluster (rank 0 makes it, every rank uses it)."""
    buf = (C.c_uint8 * _abi.GH_COMM_ID_BYTES)()
    rc = _abi.load().gh_comm_unique_id(buf)
    if rc != GH_OK:
        raise GossipError(rc, "gh_comm_unique_id failed (RCCL missing?)")
    return bytes(buf)


def _p(a: np.ndarray):
    return a.ctypes.data_as(C.c_void_p)


class Engine:
    """One libgossiphip handle: N members' tables resident in HBM, or rank
    `rank` of `world` column shards of them (then every rank makes the same
    calls and gets the same results)."""

    def __init__(self, cfg: Config, rank: int = 0, world: int = 1, transport: int | None = None,
                 comm_id: bytes | None = None):
        self.lib = _abi.load()
        self.cfg = cfg
        self.n = cfg.n_members
        self.R = cfg.replicas
        self.rank, self.world = rank, world
        h = C.c_void_p()
        if world == 1 and comm_id is None:
            rc = self.lib.gh_create(C.byref(cfg), C.byref(h))
        else:
            if comm_id is None or len(comm_id) > _abi.GH_COMM_ID_BYTES:
                raise ValueError("a sharded engine needs a comm id of <= 128 bytes")
            buf = (C.c_uint8 * _abi.GH_COMM_ID_BYTES).from_buffer_copy(
                comm_id.ljust(_abi.GH_COMM_ID_BYTES, b"\0"))
            tr = GH_COMM_LOCAL if transport is None else transport
            rc = self.lib.gh_create_sharded(C.byref(cfg), rank, world, tr, buf, C.byref(h))
        if rc != GH_OK:
            raise GossipError(rc, "gh_create failed (a gfx950 device is required; no CPU fallback)")
        self.h = h

    def shard_info(self):
        """(rank, world, first member column, member columns) of this engine."""
        r, w = C.c_int32(), C.c_int32()
        c0, nc = C.c_int64(), C.c_int64()
        self._chk(self.lib.gh_shard_info(self.h, C.byref(r), C.byref(w), C.byref(c0), C.byref(nc)))
        return r.value, w.value, c0.value, nc.value

    def encoding_info(self, full=False):
        """(wide segments of the current table, segments the last round ran
        by the per-cell rule) of this engine's shard; full=True adds the last
        round's kernel variant (0 lean, 1 storm), its storm measure and the
        row segments it skipped as quiet (diagnostic)."""
        w, sl, ns, nq = C.c_int64(), C.c_int64(), C.c_int64(), C.c_int64()
        mode = C.c_int32()
        self._chk(self.lib.gh_encoding_info(self.h, C.byref(w), C.byref(sl), C.byref(mode), C.byref(ns),
                                            C.byref(nq)))
        return (w.value, sl.value, mode.value, ns.value, nq.value) if full else (w.value, sl.value)

    def plane_info(self):
        """(plane kept, plane valid for the next round, waves of the last
        round that gathered 16-bit sender codes although it was valid) --
        the sender snapshot plane of pull mode (gh_plane_info, diagnostic)."""
        en, va, fb = C.c_int32(), C.c_int32(), C.c_int64()
        self._chk(self.lib.gh_plane_info(self.h, C.byref(en), C.byref(va), C.byref(fb)))
        return en.value, va.value, fb.value

    def tier_info(self, full=False):
        """(4-bit tier kept, current table held in it, chunks the last round
        wrote escaped) -- gh_tier_info, diagnostic; full=True adds the last
        round's kernel variant (0 lean on a 16-bit input, 1 storm, 2 lean on
        a tier input widened, 3 the nibble path)."""
        en, cu, esc, var = C.c_int32(), C.c_int32(), C.c_int64(), C.c_int32()
        self._chk(self.lib.gh_tier_info(self.h, C.byref(en), C.byref(cu), C.byref(esc), C.byref(var)))
        return (en.value, cu.value, esc.value, var.value) if full else (en.value, cu.value, esc.value)

    def job_info(self):
        """(lane jobs, of them redone wide) of the last round's nibble path
        (gh_job_info, diagnostic)."""
        nj, nr = C.c_int64(), C.c_int64()
        self._chk(self.lib.gh_job_info(self.h, C.byref(nj), C.byref(nr)))
        return nj.value, nr.value

    def debug_counts(self):
        """(rows whose maintained present count differs from a full recount,
        the first such row or -1): the invariant the <4 guard relies on
        (gh_debug_counts, test-only and not in the header, like
        gh_debug_tier; the maintained counts are left unchanged)."""
        fn = self.lib.gh_debug_counts
        fn.argtypes = [C.c_void_p, C.POINTER(C.c_int64), C.POINTER(C.c_int32)]
        fn.restype = C.c_int
        nm, fr = C.c_int64(), C.c_int32()
        self._chk(fn(self.h, C.byref(nm), C.byref(fr)))
        return nm.value, fr.value

    def debug_shadow(self):
        """(col0, int32[ncols], count): the D7 shadow entries of this engine's
        member columns -- the ts of the introducer's RecentFailList entry
        beside its present member c, or INT32_MIN (none) -- and the count the
        engine keeps (gh_debug_shadow, test-only and not in the header)."""
        fn = self.lib.gh_debug_shadow
        fn.argtypes = [C.c_void_p, C.c_void_p, C.c_int64, C.POINTER(C.c_int32)]
        fn.restype = C.c_int
        _, _, c0, nc = self.shard_info()
        out = np.empty(max(nc, 1), np.int32)
        cnt = C.c_int32()
        self._chk(fn(self.h, out.ctypes.data_as(C.c_void_p), len(out), C.byref(cnt)))
        out = out[:nc]
        out[out == np.int32(-2139062144)] = np.iinfo(np.int32).min  # GH_NO_SHADOW (0x80808080)
        return c0, out, cnt.value

    def exchange_info(self):
        """dict(ghost_rows, bytes_out, bytes_in) of this shard's last ghost-row
        exchange (row layout; gh_exchange_info)."""
        v = [C.c_int64() for _ in range(3)]
        self._chk(self.lib.gh_exchange_info(self.h, *[C.byref(x) for x in v]))
        return dict(zip(("ghost_rows", "bytes_out", "bytes_in"), (x.value for x in v)))

    def memory_info(self):
        """dict(device_bytes, wide_used, wide_cap, frozen_rows) of this
        engine's tables (gh_memory_info)."""
        v = [C.c_int64() for _ in range(4)]
        self._chk(self.lib.gh_memory_info(self.h, *[C.byref(x) for x in v]))
        return dict(zip(("device_bytes", "wide_used", "wide_cap", "frozen_rows"), (x.value for x in v)))

    def file_info(self):
        """dict(slots, shards, held): this shard's file-table slots
        (ceil(max_files / G), files sharded by ID, file f on shard f % G),
        the shard count and the files it holds (gh_file_info)."""
        sl, sh, hd = C.c_int64(), C.c_int32(), C.c_int64()
        self._chk(self.lib.gh_file_info(self.h, C.byref(sl), C.byref(sh), C.byref(hd)))
        return {"slots": sl.value, "shards": sh.value, "held": hd.value}

    def export_files(self):
        """(replicas [F][R], versions [F], timestamps [F], draws [F]): the
        master's file metadata (gh_export_files)."""
        F = int(self.cfg.max_files)
        rep = np.empty((F, self.R), np.int32)
        ver = np.empty(F, np.int32)
        ts = np.empty(F, np.int32)
        dr = np.empty(F, np.uint32)
        self._chk(self.lib.gh_export_files(self.h, _p(rep), _p(ver), _p(ts), _p(dr)))
        return rep, ver, ts, dr

    def import_files(self, rep, ver, ts, dr):
        """Replace the file metadata (gh_import_files; export_files' arrays)."""
        rep = np.ascontiguousarray(rep, dtype=np.int32)
        ver = np.ascontiguousarray(ver, dtype=np.int32)
        ts = np.ascontiguousarray(ts, dtype=np.int32)
        dr = np.ascontiguousarray(dr, dtype=np.uint32)
        self._chk(self.lib.gh_import_files(self.h, _p(rep), _p(ver), _p(ts), _p(dr)))

    def set_master(self, master):
        """The member whose list is the placement candidate list (gh_set_master)."""
        self._chk(self.lib.gh_set_master(self.h, int(master)))
        self.cfg.master = int(master)

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

    def step_rc(self, rounds=1):
        """(return code, stats of the rounds run) without raising on
        GH_ERANGE: a round that would push a heartbeat past INT32_MAX is
        refused and stats["rounds"] tells how many ran."""
        st = _abi.RoundStats()
        rc = self.lib.gh_step(self.h, rounds, C.byref(st))
        self._chk(rc, ok=(GH_OK, _abi.GH_ERANGE))
        return rc, st.as_dict()

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

    def merge_list(self, observer, ids, hb):
        """MergeMemberList (slave/slave.go:414-440) of a received list into
        `observer`'s row now; returns the number of cells changed."""
        ids = np.ascontiguousarray(ids, dtype=np.int32)
        hb = np.ascontiguousarray(hb, dtype=np.int32)
        n = C.c_int64()
        self._chk(self.lib.gh_merge_list(self.h, observer, _p(ids), _p(hb), len(ids), C.byref(n)))
        return n.value

    # ---- files -----------------------------------------------------------
    def put(self, files):
        f = np.ascontiguousarray(files, dtype=np.int32)
        rep = np.zeros((len(f), self.R), np.int32)
        ver = np.zeros(len(f), np.int32)
        st = np.zeros(len(f), np.int32)
        self._chk(self.lib.gh_put(self.h, _p(f), len(f), _p(rep), _p(ver), _p(st)),
                  ok=(GH_OK, GH_EPLACEMENT_STARVED))
        return rep, ver, st

    def put_conflicts(self, files, window=60):
        """If_file_updated_recent (master/master.go:214-229): 1 where the
        file was put less than `window` rounds (60 s at 1 s rounds) ago."""
        f = np.ascontiguousarray(files, dtype=np.int32)
        out = np.zeros(len(f), np.uint8)
        self._chk(self.lib.gh_put_conflicts(self.h, _p(f), len(f), window, _p(out)))
        return out

    def alive(self):
        a = np.empty(self.n, np.uint8)
        self._chk(self.lib.gh_export_state(self.h, None, None, _p(a), 0, self.n))
        return a

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

    # ---- master re-election (SPEC §9) -------------------------------------
    def vote_scan(self, mview):
        """Per row: MemberList[0] (-1 if empty), len(MemberList), and whether
        the row's master mview[i] is in its list (slave/slave.go:451-457,
        930-948)."""
        mv = np.ascontiguousarray(mview, dtype=np.int32)
        first = np.empty(self.n, np.int32)
        ln = np.empty(self.n, np.int32)
        has = np.empty(self.n, np.uint8)
        self._chk(self.lib.gh_vote_scan(self.h, _p(mv), _p(first), _p(ln), _p(has)))
        return first, ln, has

    def rebuild_meta(self, new_master):
        """rebuild_file_meta (slave/slave.go:986-1043) at `new_master`, which
        becomes the master row. Returns (f0 = the member that gets
        Assign_new_master, files left)."""
        f0 = C.c_int32()
        nf = C.c_int64()
        self._chk(self.lib.gh_rebuild_meta(self.h, int(new_master), C.byref(f0), C.byref(nf)))
        return f0.value, nf.value

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


def _same(a, b):
    if isinstance(a, np.ndarray):
        return isinstance(b, np.ndarray) and a.shape == b.shape and np.array_equal(a, b)
    if isinstance(a, (tuple, list)):
        return type(a) is type(b) and len(a) == len(b) and all(_same(x, y) for x, y in zip(a, b))
    if isinstance(a, dict):
        return isinstance(b, dict) and a.keys() == b.keys() and all(_same(a[k], b[k]) for k in a)
    return a == b


class ShardGroup:
    """One cluster column-sharded over `world` engines driven from this
    process, one thread per rank (GH_COMM_LOCAL). Methods mirror Engine's;
    each call runs on every rank concurrently (the SPMD contract) and
    returns rank 0's result after checking that every rank agrees."""

    _ids = itertools.count()

    def __init__(self, cfg: Config, world: int, devices=None):
        self.world = world
        self.n = cfg.n_members
        self.cfg = cfg
        self.pool = ThreadPoolExecutor(max_workers=world)
        key = f"gossipsim-{os.getpid()}-{next(self._ids)}".encode()
        devices = devices or [cfg.device] * world

        def make(r):
            c = Config.from_buffer_copy(cfg)
            c.device = devices[r]
            return Engine(c, rank=r, world=world, transport=GH_COMM_LOCAL, comm_id=key)

        self.engines = list(self.pool.map(make, range(world)))

    def run(self, name, *args, **kw):
        """Every rank's result of Engine.<name>(*args, **kw). A rank that
        raises is reported at once (the others may still wait in a collective
        until the transport's barrier gives up)."""
        futs = [self.pool.submit(getattr(e, name), *args, **kw) for e in self.engines]
        done, _ = wait(futs, return_when=FIRST_EXCEPTION)
        for f in done:
            if f.exception() is not None:
                raise f.exception()
        return [f.result() for f in futs]

    def __getattr__(self, name):
        if name.startswith("_") or not callable(getattr(Engine, name, None)):
            raise AttributeError(name)

        def call(*args, **kw):
            res = self.run(name, *args, **kw)
            for r, x in enumerate(res[1:], 1):
                if not _same(res[0], x):
                    raise AssertionError(f"rank {r} disagrees with rank 0 on {name}")
            return res[0]
        return call

    @property
    def round(self):
        return self.engines[0].round

    def close(self):
        self.run("close")
        self.pool.shutdown()


PutResult = namedtuple("PutResult", "file put_or_not replicas version status acks quorum_met")
GetResult = namedtuple("GetResult", "file replicas version acks quorum_met source source_version",
                       defaults=(None,))


class Cluster:
    """The reference's per-node commands over one Engine (member IDs stand in
    for the VM addresses). Repairs follow Fail_recover: every row that detects
    a failure in round r triggers Update_metadata with its own list as
    `available` at round r + repair_delay (slave/slave.go:1122-1133). The
    defaults are the reference's own topology: gossip is the 3-neighbour ring
    push (GH_PEER_RING, slave/slave.go:515-542) unless peer_mode is given,
    and lists keep the reference's append order (GH_ORDER_APPEND) unless
    list_order is given: lsm, ring targets, quirk runs, MemberList[0] and the
    placement candidates read them as the reference's slices do (SPEC D1).
    (Engine / gh_config_default keep Philox pull: the batched bench mode.)"""

    def __init__(self, n, repair_delay=8, addresses=None, elect=False, **cfg_kw):
        cfg_kw.setdefault("peer_mode", GH_PEER_RING)
        cfg_kw.setdefault("list_order", GH_ORDER_APPEND)
        self.engine = Engine(default_config(n, **cfg_kw))
        self.n = n
        self.repair_delay = repair_delay
        # master re-election (SPEC §9, slave/slave.go:930-1051), when `elect`:
        # each member's self.master, VoteStatus, the pending rebuilds and the
        # members whose process is gone (crash; log.Fatal)
        self.elect = elect
        self.master = int(self.engine.cfg.master)
        self._configured_master = self.master  # INTRODUCER_ADDR: what a fresh process believes
        self.mview = np.full(n, self.master, np.int32)
        self.vote_on = np.zeros(n, bool)
        self.vote_num = np.zeros(n, np.int64)
        self.voters: list[set] = [set() for _ in range(n)]
        self.rebuilds: dict[int, list[int]] = {}
        self.dead: set[int] = set()
        self.elections: list[tuple[int, int]] = []  # (round, new master)
        self.fatal: list[tuple[int, int, str]] = []  # (round, member, why)
        # member id <-> address (the reference's identity, slave/slave.go:145-159)
        self.addresses = list(addresses) if addresses is not None else [f"10.0.{i >> 8}.{i & 255}" for i in range(n)]
        self.ids = {a: i for i, a in enumerate(self.addresses)}
        self.scheduled: dict[int, list[int]] = {}
        self.plans: list[tuple[int, int, tuple]] = []  # (round, observer, plan)
        # each member's SDFSInfo.Local_files (sdfs_slave/sdfs_slave.go:20-41):
        # file -> {member: (version, process epoch)}, written when a put or a
        # repair copies the file to the member; a restarted process (join
        # after a crash) starts with an empty map, so entries of an older
        # epoch read as Go's zero value
        self._local: dict[int, dict[int, tuple[int, int]]] = {}
        self._epoch = np.zeros(n, np.int64)
        # the process epoch in which a member last held the file metadata as
        # master (SDFSMaster's maps live in the process, master/master.go:38):
        # any other running member's metadata is empty
        self._meta_epoch = {self.master: 0}
        # masters demoted by an election while their process kept running:
        # member -> (process epoch, its maps as export_files arrays). Members
        # whose self.master still names it send their Update_metadata there
        # (Fail_recover, slave/slave.go:1122-1136), and it answers from these
        self._demoted: dict[int, tuple[int, tuple]] = {}

    # REPL vocabulary (slave/slave.go:546-613)
    def join(self, member):
        """A (re)started process joins (Join, slave/slave.go:288-308): it is
        a fresh Slave (new_slave, :99-112), so a member whose process was
        gone runs again with self.master = the configured master and its
        VoteStatus off."""
        member = int(member)
        self.engine.apply_events([(GH_EV_JOIN, member)])
        if member in self.dead:
            self._epoch[member] += 1  # a fresh process: empty Local_files
            self.dead.discard(member)
            self.mview[member] = self._configured_master
            self.vote_on[member] = False
            self.vote_num[member] = 0
            self.voters[member] = set()

    def leave(self, member):
        self.engine.apply_events([(GH_EV_LEAVE, member)])

    def crash(self, member):
        self.engine.apply_events([(GH_EV_CRASH, member)])
        self.dead.add(int(member))

    def local_version(self, member, file):
        """SDFSInfo.Get_file_version at `member` (sdfs_slave/sdfs_slave.go:39-41):
        the version its process stored, 0 (Go's zero value) if it holds none."""
        v = self._local.get(int(file), {}).get(int(member))
        return v[0] if v is not None and v[1] == self._epoch[int(member)] else 0

    def _store(self, file, members, version):
        loc = self._local.setdefault(int(file), {})
        for m in members:
            loc[int(m)] = (int(version), int(self._epoch[int(m)]))

    def lsm(self, member):
        ids, hb, ts = self.engine.lsm(member)
        return list(zip(ids.tolist(), hb.tolist(), ts.tolist()))

    # wire format of the gossip datagrams (slave/slave.go:365-385, 527-542)
    def datagram(self, member) -> bytes:
        """What `member` sends its ring neighbours: its list, encoded. The
        update time is the member's local tick (the reference sends UnixNano,
        which receivers ignore, :426, :437)."""
        return codec.encode((self.addresses[i], hb, ts) for i, hb, ts in self.lsm(member))

    def receive(self, member, datagram: bytes):
        """GetMsg's gossip branch (:241-245) at `member`: decode (raises
        codec.DecodePanic where the reference's goroutine would panic), then
        MergeMemberList. Returns the number of cells changed. Addresses must
        be cluster members; the first entry of a repeated address is the one
        MergeMemberList compares (GetIndex, :396-403)."""
        entries = codec.decode(datagram)
        seen, ids, hbs = set(), [], []
        for addr, hb, _ in entries:
            if addr in seen:
                continue
            seen.add(addr)
            ids.append(self.ids[addr])
            hbs.append(hb)
        return self.engine.merge_list(member, ids, hbs)

    # SDFS ops (slave/slave.go:661-928 over master/master.go:74-259)
    WRITE_WINDOW = 60  # If_file_updated_recent: 60 s (master/master.go:225) at 1 s rounds

    @staticmethod
    def quorum(n_replicas):
        """cal_quorum_num (slave/slave.go:717-722): int(math.Ceil(float64((n+1)/2)))
        with Go's integer division inside: 1, 1, 2, 2, 3 for n = 1..5."""
        return (n_replicas + 1) // 2

    def put(self, files, confirm=()):
        """put for each file (slave/slave.go:668 -> Get_put_info,
        server/server.go:74-121): a file put less than WRITE_WINDOW rounds ago
        is a write-write conflict and goes ahead only if the requester
        confirms (file in `confirm`, the interactive "yes"); otherwise
        Handle_put_request places it and bumps the version. acks = replicas
        whose process is alive; the reference waits for
        quorum(len(replicas)) of them (:698-714, forever if they never come).
        Returns PutResult per file, in input order."""
        files = [int(f) for f in files]
        conf = set(int(f) for f in confirm)
        clash = self.engine.put_conflicts(files, self.WRITE_WINDOW) if files else []
        go = [f for f, c in zip(files, clash) if not c or f in conf]
        placed = {}
        if go:
            rep, ver, st = self.engine.put(go)
            alive = self._running()
            for x, f in enumerate(go):
                r = [int(a) for a in rep[x] if a >= 0]
                placed[f] = (r, int(ver[x]), int(st[x]), sum(int(alive[a]) for a in r))
                if int(st[x]) == GH_OK:  # Put_file at every live replica (slave/slave.go:724-760)
                    self._store(f, [a for a in r if alive[a]], int(ver[x]))
        out = []
        for f in files:
            if f not in placed:
                out.append(PutResult(f, False, [], -1, GH_OK, 0, False))
                continue
            r, v, st, acks = placed[f]
            out.append(PutResult(f, True, r, v, st, acks, st == GH_OK and acks >= self.quorum(len(r))))
        return out

    @staticmethod
    def get_source(responses, version):
        """Get's copy source (slave/slave.go:857-878) over the replicas'
        responses [(member, local_version), ...] in arrival order: the first
        whose local version is <= the master's `version`, or the only
        response; None when no response qualifies (nothing is copied). A
        replica without the file answers Go's zero value 0, which qualifies:
        the reference can copy from a replica that holds no file."""
        for m, lv in responses:
            if lv <= version or len(responses) == 1:
                return m, lv
        return None

    def get(self, files):
        """get (slave/slave.go:815-890): the master's replica list and
        version (-1: "No File Found"), whether a read quorum of replicas is
        alive to answer, and the copy source: every live replica answers
        Get_file_data with its local version (:799-810; arrival order is
        taken as replica order) and get_source picks among the answers."""
        rep, ver = self.engine.get_files(files)
        alive = self._running()
        out = []
        for x, f in enumerate(files):
            r = [int(a) for a in rep[x] if a >= 0]
            acks = sum(int(alive[a]) for a in r)
            src, sv = -1, None
            if int(ver[x]) >= 0:
                pick = self.get_source([(a, self.local_version(a, f)) for a in r if alive[a]], int(ver[x]))
                if pick is not None:
                    src, sv = pick
            out.append(GetResult(int(f), r, int(ver[x]), acks, int(ver[x]) >= 0 and acks >= self.quorum(len(r)),
                                 src, sv))
        return out

    def _running(self):
        """The engine's alive vector with the members whose process already
        ended in a log.Fatal this round masked out (their crash event is
        applied by the next round)."""
        alive = self.engine.alive().copy()
        if self.dead:
            alive[list(self.dead)] = 0
        return alive

    def ls(self, files):
        """ls (slave/slave.go:892-917): replica list and version per file."""
        return self.engine.get_files(files)

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
            if self.elect:
                self._election_step(r)
            for obs in self.scheduled.pop(r, []):
                if self.elect:
                    if obs in self.dead:
                        continue
                    if self.mview[obs] in self.dead:  # Fail_recover dials a dead master (:1125-1127)
                        self._fatal(r, obs, "Fail_recover: master unreachable")
                        continue
                    m = int(self.mview[obs])
                    if m != self.master:
                        # a stale but running master answers from its own
                        # SDFSMaster: the maps it kept when an election
                        # demoted it, else (this process was never master)
                        # empty maps, an empty plan: Fail_recover returns at
                        # once (slave/slave.go:1139-1142)
                        kept = self._demoted.get(m)
                        if kept is not None and kept[0] == self._epoch[m] and self.engine.cfg.max_files > 0:
                            plan = self._repair_at_demoted(m, obs)
                            self.plans.append((r, obs, plan))
                            self._copy_repairs(plan)
                        elif self._meta_epoch.get(m) != self._epoch[m]:
                            self.plans.append((r, obs, ()))
                        continue
                if self.engine.cfg.max_files > 0:
                    plan = tuple(self.engine.repair(obs))
                    self.plans.append((r, obs, plan))
                    self._copy_repairs(plan)
        return total

    def _copy_repairs(self, plan):
        alive = self._running()
        for f, node1, v, st, new in plan:  # Re_put / Remote_reput copy the file (:1148-1170)
            if node1 >= 0:
                self._store(f, [a for a in new if alive[a]], v)

    def _repair_at_demoted(self, m, obs):
        """Update_metadata (master/master.go:74-127) run by the demoted but
        running master m on its own maps, with its own list as Member_list:
        m's maps and master row are swapped into the engine for the call and
        the current master's swapped back."""
        cur = self.engine.export_files()
        self.engine.import_files(*self._demoted[m][1])
        self.engine.set_master(m)
        try:
            plan = tuple(self.engine.repair(obs))
            self._demoted[m] = (self._demoted[m][0], self.engine.export_files())
        finally:
            self.engine.import_files(*cur)
            self.engine.set_master(self.master)
        return plan

    # ---- master re-election (SPEC §9) -----------------------------------
    def _touch(self, x):  # `if self.VoteStatus.Vote == false {...}` (slave/slave.go:931-935, 969-973)
        if not self.vote_on[x]:
            self.vote_on[x] = True
            self.vote_num[x] = 0
            self.voters[x] = set()

    def _fatal(self, r, member, why):
        """log.Fatal ends the member's process: a crash."""
        self.fatal.append((r, int(member), why))
        self.crash(member)

    def _election_step(self, r):
        """After round r: every running row whose master left its list calls
        revote_master (slave/slave.go:451-457, 930-948); the votes are
        Receive_vote'd in ID order (:968-984); an elected member rebuilds the
        metadata two rounds later (:987, `time.Sleep(HEARTBEAT_PERIOD * 2)`)."""
        for m in self.rebuilds.pop(r, []):
            if m in self.dead:
                continue
            ids, _, _ = self.engine.lsm(m)
            f0 = int(ids[0]) if len(ids) else m
            if f0 != m and f0 in self.dead:  # rpc.Dial to MemberList[0] fails (:996-999)
                self._fatal(r, m, "rebuild_file_meta: MemberList[0] unreachable")
                continue
            if self.engine.cfg.max_files > 0:
                old = self.master
                if old != m and old not in self.dead and self._meta_epoch.get(old) == self._epoch[old]:
                    # the old master's process runs on with its maps
                    self._demoted[old] = (int(self._epoch[old]), self.engine.export_files())
                self._demoted.pop(m, None)  # m's maps are the rebuilt ones now
                f0, _ = self.engine.rebuild_meta(m)
            self.master = m
            self._meta_epoch[m] = int(self._epoch[m])
            self.mview[f0] = m  # Assign_New_Master (:1045-1048)
            self.vote_on[f0] = False
            self.vote_on[m] = False  # :1039-1040
            self.voters[m] = set()
            self.scheduled.setdefault(r + self.repair_delay, []).append(m)  # go Fail_recover (:1042)
        first, ln, has = self.engine.vote_scan(self.mview)
        alive = self.engine.alive()
        run = (alive != 0) & (ln >= self.engine.cfg.min_members) & (has == 0)
        self._tally(r, np.flatnonzero(run), first, ln)

    def _tally(self, r, idx, first, ln):
        """The votes of one round, in voter-ID order, as array operations
        (the same result as running revote_master / Receive_vote voter by
        voter; oracle/election.py's Tally is that loop). idx: the voting
        rows, ascending."""
        if len(idx) == 0:
            return
        tgt = first[idx].astype(np.int64)
        remote = tgt != idx
        # log.Fatal when the target's process is gone: already dead, or a
        # voter that died earlier in this round's order (its own vote failed)
        dead = np.zeros(self.n, bool)
        if self.dead:
            dead[list(self.dead)] = True
        fatal = remote & dead[tgt]
        while True:
            fdead = np.zeros(self.n, bool)
            fdead[idx[fatal]] = True
            more = remote & ~fatal & fdead[tgt] & (tgt < idx)
            if not more.any():
                break
            fatal |= more
        ok = remote & ~fatal
        # touch (slave/slave.go:931-935, 969-973): every voter, and every target of a vote that arrives
        touched = np.unique(np.concatenate([idx, tgt[ok]]))
        fresh = touched[~self.vote_on[touched]]
        self.vote_on[fresh] = True
        self.vote_num[fresh] = 0
        for x in fresh.tolist():
            if self.voters[x]:
                self.voters[x] = set()
        selfv = idx[~remote]
        self.vote_num[selfv] += 1  # self votes: counted, no majority check (:936-939)
        events = []
        if ok.any():
            selfset = set(selfv.tolist())
            vs, ts = idx[ok], tgt[ok]
            for t in np.unique(ts).tolist():
                who = vs[ts == t]  # ascending
                old = self.voters[t]
                new = np.array([v not in old for v in who.tolist()]) if old else np.ones(len(who), bool)
                sv = int(t in selfset)
                # Vote_num as each remote vote is checked: the count after the
                # touch, + the new voters so far, + t's own vote if t came first
                start = int(self.vote_num[t]) - sv
                cum = start + np.cumsum(new) + (sv & (who > t)).astype(np.int64)
                self.voters[t].update(who[new].tolist())
                self.vote_num[t] = start + int(new.sum()) + sv
                if self.mview[t] != t:
                    hit = np.flatnonzero(cum > ln[t] // 2)
                    if len(hit):
                        events.append((int(who[hit[0]]), t))
        for _, t in sorted(events):
            self.mview[t] = t
            self.elections.append((r, t))
            self.rebuilds.setdefault(r + 2, []).append(t)
        for i in idx[fatal].tolist():
            self._fatal(r, i, "revote_master: MemberList[0] unreachable")
