"""CPU checks of the drop-in boundary: libgossiphip loads, exports every symbol
include/gossiphip.h declares, the ctypes structs match the header's layout,
and without a gfx950 device it refuses to run (no CPU fallback)."""
import ctypes as C
import re

import pytest

from conftest import PKG_DIR, REPO

HEADER = (REPO / "include" / "gossiphip.h").read_text()


def declared_functions():
    body = re.sub(r"/\*.*?\*/", "", HEADER, flags=re.S)
    return sorted(set(re.findall(r"\b(gh_[a-z_]+)\s*\(", body)))


@pytest.fixture(scope="module")
def abi():
    from gossipsim import _abi
    if not _abi.LIB_PATH.exists():
        import subprocess
        subprocess.run(["make", "-s", "-C", str(PKG_DIR)], check=True)
    _abi.load()
    return _abi


def test_every_declared_symbol_is_exported(abi):
    lib = C.CDLL(str(abi.LIB_PATH))
    names = declared_functions()
    assert len(names) >= 20
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing
    bound = {n for n, _, _ in abi.SYMBOLS}
    assert set(names) == bound, set(names) ^ bound


def test_struct_layouts(abi):
    # sizes implied by the header (int32 x 12 + u64 + i64 x 2 + int32 x 6)
    assert C.sizeof(abi.Config) == 12 * 4 + 8 + 8 + 8 + 6 * 4
    assert C.sizeof(abi.Event) == 8
    assert C.sizeof(abi.RoundStats) == 10 * 8
    assert C.sizeof(abi.PlanEntry) == 13 * 4


def test_abi_version_and_defaults(abi):
    lib = abi.load()
    assert lib.gh_abi_version() == 7
    cfg = abi.Config()
    lib.gh_config_default(C.byref(cfg))
    # reference constants: PERIOD/COOLDOWN 5 s at 1 s rounds, 4 replicas, literal 4
    assert (cfg.t_fail, cfg.t_cleanup, cfg.min_members, cfg.replicas) == (5, 5, 4, 4)
    assert cfg.remove_mode == abi.GH_REMOVE_ALL


def test_remove_list_validation(abi):
    """GH_REMOVE_LIST is a one-engine, ID-order mode: gh_create and
    gh_footprint refuse it sharded, in append order, or an unknown mode,
    before looking for a device; a valid one plans its recipient bitmaps."""
    from gossipsim import default_config, footprint, GossipError, GH_ORDER_APPEND
    lib = abi.load()
    h = C.c_void_p()
    for kw in (dict(remove_mode=2), dict(remove_mode=1, list_order=GH_ORDER_APPEND)):
        cfg = default_config(64, **kw)
        assert lib.gh_create(C.byref(cfg), C.byref(h)) == abi.GH_EINVAL
    with pytest.raises(GossipError):
        footprint(default_config(64, remove_mode=1), rank=0, world=2)
    base = footprint(default_config(4096))["create_bytes"]
    lit = footprint(default_config(4096, remove_mode=1))["create_bytes"]
    assert lit - base >= 5 * 4096 * 4096 // 8  # two recipient sets + three column bitmaps of N x N bits


def test_no_cpu_fallback(abi):
    """Without a gfx950 device gh_create must fail (GH_ENODEV), never emulate."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    lib = abi.load()
    cfg = abi.Config()
    lib.gh_config_default(C.byref(cfg))
    h = C.c_void_p()
    assert lib.gh_create(C.byref(cfg), C.byref(h)) == abi.GH_ENODEV
    from gossipsim import Engine, GossipError, default_config
    with pytest.raises(GossipError):
        Engine(default_config(8))
