"""ctypes declarations of include/gossiphip.h (the libgossiphip C-ABI).

This is the binding a Python host uses; the cgo equivalent for the
reference's Go world is in INTEGRATION.md. The library is loaded from the
in-tree build (lib/libgossiphip.so); there is no fallback implementation.
"""
from __future__ import annotations

import ctypes as C
import os
import pathlib

PKG_ROOT = pathlib.Path(__file__).resolve().parents[1]
LIB_PATH = pathlib.Path(os.environ.get("GOSSIPHIP_LIB", PKG_ROOT / "lib" / "libgossiphip.so"))

GH_OK = 0
GH_EINVAL = -1
GH_ENODEV = -2
GH_ENOMEM = -3
GH_EHIP = -4
GH_EPLACEMENT_STARVED = -5
GH_ERANGE = -6
ERRORS = {GH_EINVAL: "GH_EINVAL", GH_ENODEV: "GH_ENODEV", GH_ENOMEM: "GH_ENOMEM", GH_EHIP: "GH_EHIP",
          GH_EPLACEMENT_STARVED: "GH_EPLACEMENT_STARVED", GH_ERANGE: "GH_ERANGE"}

GH_ABSENT, GH_TOMBSTONE = -1, -2
GH_PEER_PULL, GH_PEER_RING = 0, 1
GH_DETECT_CANONICAL, GH_DETECT_QUIRK = 0, 1
GH_EV_JOIN, GH_EV_LEAVE, GH_EV_CRASH = 1, 2, 3
GH_COMM_RCCL, GH_COMM_LOCAL = 0, 1
GH_COMM_ID_BYTES = 128
GH_LAYOUT_COLUMNS, GH_LAYOUT_ROWS = 0, 1
GH_ORDER_ID, GH_ORDER_APPEND = 0, 1
GH_REMOVE_ALL, GH_REMOVE_LIST = 0, 1


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


class RoundStats(C.Structure):
    _fields_ = [(n, C.c_int64) for n in (
        "rounds", "last_round", "detections", "failed_members", "remove_unknown",
        "ring_empty", "active_rows", "merged_cells", "released", "tombstoned")]

    def as_dict(self):
        return {n: getattr(self, n) for n, _ in self._fields_}


class PlanEntry(C.Structure):
    _fields_ = [("file", C.c_int32), ("node1", C.c_int32), ("version", C.c_int32),
                ("n_new", C.c_int32), ("status", C.c_int32), ("new_nodes", C.c_int32 * 8)]


# (name, restype, argtypes) for every symbol include/gossiphip.h declares.
_vp, _i32, _i64 = C.c_void_p, C.c_int32, C.c_int64
_P = C.POINTER
SYMBOLS = [
    ("gh_abi_version", C.c_int, []),
    ("gh_config_default", None, [_P(Config)]),
    ("gh_create", C.c_int, [_P(Config), _P(_vp)]),
    ("gh_destroy", None, [_vp]),
    ("gh_last_error", C.c_char_p, [_vp]),
    ("gh_import_state", C.c_int, [_vp, _vp, _vp, _vp, _i64, _i64, _i32]),
    ("gh_export_state", C.c_int, [_vp, _vp, _vp, _vp, _i64, _i64]),
    ("gh_init_full", C.c_int, [_vp, _i32, _i32, _i32]),
    ("gh_get_round", C.c_int, [_vp, _P(_i32)]),
    ("gh_apply_events", C.c_int, [_vp, _P(Event), _i64]),
    ("gh_step", C.c_int, [_vp, _i32, _P(RoundStats)]),
    ("gh_read_failed", C.c_int, [_vp, _vp, _i64]),
    ("gh_read_detectors", C.c_int, [_vp, _vp, _i64, _P(_i64)]),
    ("gh_lsm", C.c_int, [_vp, _i32, _vp, _vp, _vp, _i64, _P(_i64)]),
    ("gh_merge_list", C.c_int, [_vp, _i32, _vp, _vp, _i64, _P(_i64)]),
    ("gh_put", C.c_int, [_vp, _vp, _i64, _vp, _vp, _vp]),
    ("gh_put_conflicts", C.c_int, [_vp, _vp, _i64, _i32, _vp]),
    ("gh_repair", C.c_int, [_vp, _i32, _P(PlanEntry), _i64, _P(_i64)]),
    ("gh_get_files", C.c_int, [_vp, _vp, _i64, _vp, _vp]),
    ("gh_delete_files", C.c_int, [_vp, _vp, _i64, _vp]),
    ("gh_vote_scan", C.c_int, [_vp, _vp, _vp, _vp, _vp]),
    ("gh_rebuild_meta", C.c_int, [_vp, _i32, _P(_i32), _P(_i64)]),
    ("gh_set_round_variant", C.c_int, [_vp, _i32, _i32]),
    ("gh_set_timing", C.c_int, [_vp, _i32]),
    ("gh_read_timing", C.c_int, [_vp, _P(C.c_double), _P(_i64)]),
    ("gh_sync", C.c_int, [_vp]),
    ("gh_comm_unique_id", C.c_int, [_vp]),
    ("gh_create_sharded", C.c_int, [_P(Config), _i32, _i32, _i32, _vp, _P(_vp)]),
    ("gh_shard_info", C.c_int, [_vp, _P(_i32), _P(_i32), _P(_i64), _P(_i64)]),
    ("gh_encoding_info", C.c_int, [_vp, _P(_i64), _P(_i64), _P(_i32), _P(_i64), _P(_i64)]),
    ("gh_plane_info", C.c_int, [_vp, _P(_i32), _P(_i32), _P(_i64)]),
    ("gh_tier_info", C.c_int, [_vp, _P(_i32), _P(_i32), _P(_i64), _P(_i32)]),
    ("gh_exchange_info", C.c_int, [_vp, _P(_i64), _P(_i64), _P(_i64)]),
    ("gh_job_info", C.c_int, [_vp, _P(_i64), _P(_i64)]),
    ("gh_memory_info", C.c_int, [_vp, _P(_i64), _P(_i64), _P(_i64), _P(_i64)]),
    ("gh_file_info", C.c_int, [_vp, _P(_i64), _P(C.c_int32), _P(_i64)]),
    ("gh_export_files", C.c_int, [_vp, _vp, _vp, _vp, _vp]),
    ("gh_import_files", C.c_int, [_vp, _vp, _vp, _vp, _vp]),
    ("gh_set_master", C.c_int, [_vp, C.c_int32]),
    ("gh_footprint", C.c_int, [_P(Config), _i32, _i32, _i32, _P(_i64), _P(_i64)]),
]

_lib = None


def load() -> C.CDLL:
    """Load the in-tree libgossiphip; raise if it is missing (no fallback)."""
    global _lib
    if _lib is None:
        if not LIB_PATH.exists():
            raise ImportError(f"libgossiphip not built: {LIB_PATH} missing (run `make -C {PKG_ROOT}`)")
        lib = C.CDLL(str(LIB_PATH))
        for name, res, args in SYMBOLS:
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _lib = lib
    return _lib
