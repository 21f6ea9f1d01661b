"""Per-GPU HBM plans from gh_footprint (a dry walk of gh_create's
allocations: no device needed), for BASELINE config 4 (N = 262,144 members
over 8 MI355X, 288 GB of HBM each) in both shard layouts, and the single-GPU
headline configuration."""
import pytest

GB = 1e9
CAP = 270 * GB  # of the 288 GB per MI355X: headroom for RCCL and staging


@pytest.fixture(scope="module")
def gs():
    import gossipsim
    return gossipsim


def plan(gs, n, world, layout, **kw):
    cfg = gs.default_config(n, fanout=4, shard_layout=layout, **kw)
    return [gs.footprint(cfg, g, world) for g in range(world)]


@pytest.mark.parametrize("layout", ["columns", "rows"])
def test_config4_fits_every_rank(gs, layout):
    lay = gs.GH_LAYOUT_ROWS if layout == "rows" else gs.GH_LAYOUT_COLUMNS
    ranks = plan(gs, 262144, 8, lay)
    worst = max(r["total_bytes"] for r in ranks)
    print(f"config 4, {layout}: {worst / GB:.1f} GB per GPU (create {max(r['create_bytes'] for r in ranks) / GB:.1f}, "
          f"exchange staging {max(r['exchange_bytes'] for r in ranks) / GB:.1f})")
    assert worst <= CAP, f"{layout}: {worst / GB:.1f} GB per GPU"


def test_headline_single_gpu(gs):
    """N = 65,536 on one GPU: the 16-bit table x2 (16 GiB), the sender plane
    x2 and the 4-bit tier's age plane x2 (4 GiB each), the wide arenas, the
    nibble path's lane-job regions (4 GiB: 512 jobs of 32 B per wave), 2^20
    files."""
    (r,) = plan(gs, 65536, 1, gs.GH_LAYOUT_COLUMNS, max_files=1 << 20)
    assert r["exchange_bytes"] == 0
    assert 28 * 2**30 <= r["create_bytes"] <= 31 * 2**30, r


def test_row_shards_hold_no_ghost_slots_in_the_tables(gs):
    """Row layout: ghost rows live in one single-buffered ghost table sized
    to a pull round's expected distinct remote senders, not in both table
    buffers: the plan grows with N^2 / G, not N^2 k / G."""
    small = max(r["total_bytes"] for r in plan(gs, 65536, 8, gs.GH_LAYOUT_ROWS))
    cols = max(r["total_bytes"] for r in plan(gs, 65536, 8, gs.GH_LAYOUT_COLUMNS))
    assert small < 4 * cols, (small / GB, cols / GB)


def test_footprint_rejects_bad_configs(gs):
    with pytest.raises(gs.GossipError):
        gs.footprint(gs.default_config(0), 0, 1)
    with pytest.raises(gs.GossipError):
        gs.footprint(gs.default_config(1024), 3, 2)
