"""A/B of k_round layout/stream variants at N=65,536 (steady state). One
engine per tile width (64 GiB each at N=65,536, up to 3 alive at once), rounds
interleaved across variants in one process (guide §5.4 rule 24); kernel time
from HIP events on each engine's stream.
  python tools/round_variants.py [--n 65536] [--iters 4] [--rounds 3]
         [--variants 64:1:0,16:1:1]   (tile_width:nontemporal:xcd_map)"""
import argparse
import json
import pathlib
import statistics
import sys

REPO = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO / "p2p-file-system-with-gossip-detect-failure-management_amd"))
import gossipsim as gs  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=65536)
ap.add_argument("--k", type=int, default=4)
ap.add_argument("--iters", type=int, default=4)
ap.add_argument("--rounds", type=int, default=3)
ap.add_argument("--variants", default="64:1:0,64:1:1,16:1:1,16:1:0,8:1:1,32:1:1")
a = ap.parse_args()
variants = [tuple(int(x) for x in v.split(":")) for v in a.variants.split(",")]
engines = {}
for tw in sorted({v[0] for v in variants}):
    e = gs.Engine(gs.default_config(a.n, fanout=a.k, seed=0x5EED0003, t_fail=16, t_cleanup=16, tile_width=tw))
    e.init_full(2, 0, 0)
    e.step(12)
    engines[tw] = e
res = {v: [] for v in variants}
for it in range(a.iters):
    for v in variants:
        e = engines[v[0]]
        e.set_round_variant(v[1], v[2])
        e.set_timing(True)
        e.step(a.rounds)
        ms, k = e.read_timing()
        res[v].append(ms / k)
    print(f"iter {it}: " + " ".join(f"{v[0]}:{v[1]}:{v[2]}={res[v][-1]:.2f}" for v in variants), flush=True)
bytes_alg = 4.0 * a.n * a.n * (a.k + 4)
out = {f"tw{v[0]}_nt{v[1]}_x{v[2]}": {"median_ms": statistics.median(t), "min_ms": min(t),
                             "alg_GBps": bytes_alg / (statistics.median(t) / 1e3) / 1e9} for v, t in res.items()}
print(json.dumps(out, indent=1))
