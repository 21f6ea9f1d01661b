"""bench.py — gossip rounds/sec at N=65,536 members (BASELINE.json metric).

One "step" = one synchronous gossip round of the whole simulated cluster
(SPEC.md §2: REMOVE delivery, <4 guard, own heartbeat, T_fail detection,
T_cleanup sweep, k=4 Philox-peer max-merge) over the N x N int32 heartbeat and
timestamp tables resident in HBM (BASELINE config 3, SURVEY.md §8d C3:
full membership hb=2 ts=0, seed 0x5EED0003).

  python bench.py [--gpus N] [--steps K] [--warmup W]

N>1 is launched by the driver under torch.distributed.run, one rank per GPU:
the SAME cluster (N=65,536 by default) is column-sharded over the N GPUs
(DESIGN.md "Multi-GPU"; rank g owns member columns [g*N/G, (g+1)*N/G) of all
rows, RCCL over xGMI carries the O(N) per-round exchanges), so total work is
fixed ("scaling": "strong") and value = rounds / max-over-ranks time. The RCCL
unique id travels from rank 0 over a gloo (CPU) process group.

Timeouts: the reference's PERIOD = COOLDOWN = 5 s at 1 s rounds
(slave/slave.go:24-25) was sized for ~10 VMs. A heartbeat needs ~log5(N) ~ 7
rounds to reach everyone at N=65,536, so T_fail=5 detects ~95% of all cells in
round 6 and every row falls under the <4 guard in round 7 (measured with the
oracle at N=4,096/16,384, DESIGN.md "Workload"); the bench therefore times the
healthy steady state with T_fail = T_cleanup = 16 rounds (--t-fail). Parity
tests cover both regimes.

The JSON line also carries
  roofline: the round kernel (k_round) — achieved = its COMPULSORY bytes per
            launch / its mean duration from HIP events on the engine's stream;
            peak 8.0 TB/s (MI355X_MICROARCH.md), so frac <= 1 is the share of
            the HBM peak the round moves. Compulsory bytes on the 4-bit tier:
            2*N*ncols (each cell's lag nibble and age nibble read once and
            written once; the lag nibbles ARE the sender plane the k gathers
            read; DESIGN.md "Kernels"); on the 16-bit table 5*N*ncols (cells
            in and out, the plane out and in). frac_prev_model restates the
            same time on round 2's 8-bit-tier model (3*N*ncols) so a model
            change cannot pass for a speed-up. The k sender gathers are
            gather_bytes_per_launch, SURVEY.md §8d's int32 model
            4*N^2*(k+4) survey_bytes_per_launch; traffic = fabric-side bytes
            per launch from the rocprofv3 PMC passes of tools/pmc.sh for this
            configuration, encoding and warm-up (profiles/, FETCH_SIZE x2 +
            WRITE_SIZE, the guide's gfx950 correction; Infinity-Cache hits
            included), null if none was captured at this warm-up.
  cpu_baseline: the CPU restatement (oracle/tablesim.c, "port") timed on this
            host's cores (nproc threads and 1 thread) on the full benched
            configuration, plus N=4,096 and N=10 rates and the literal list
            replay (oracle/listsim.py) at N <= 256 (rank 0, N=1 only).
  secondary: the same engine at the reference's own PERIOD = COOLDOWN = 5
            rounds (slave/slave.go:24-25; the cluster collapses under the <4
            guard in round 7), the reference's ring push, BASELINE config 2
            (N=4,096, k=3, 1% crash at r=8, 64 rounds: the launch-gap regime),
            and the benched configuration with a 1% crash (655 Philox-drawn
            members at r=8, through detection, REMOVE and the tombstones'
            release: rounds/s and the round count of each kernel variant).
"""
from __future__ import annotations

import argparse
import json
import os
import pathlib
import sys
import time

REPO = pathlib.Path(__file__).resolve().parent
PKG_DIR = REPO / "p2p-file-system-with-gossip-detect-failure-management_amd"
sys.path.insert(0, str(PKG_DIR))
sys.path.insert(0, str(REPO))

HBM_PEAK_GBS = 8000.0        # MI355X_MICROARCH.md: 8.0 TB/s spec
HBM_MEASURED_GBS = 6290.0    # MI355X_MICROARCH.md: 6.29 TB/s float4 copy


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--n", type=int, default=65536)
    ap.add_argument("--fanout", type=int, default=4)
    ap.add_argument("--peer-mode", choices=("pull", "ring"), default="pull",
                    help="pull: k Philox peers (BASELINE configs 2-4); ring: the reference's ring push")
    ap.add_argument("--detect", choices=("canonical", "quirk"), default="canonical")
    ap.add_argument("--layout", choices=("columns", "rows"), default="columns",
                    help="shard layout for --gpus > 1: member columns (O(N) exchanges, default) or observer "
                         "rows with the senders' rows by ncclAllToAllv (north_star)")
    ap.add_argument("--seed", type=lambda s: int(s, 0), default=0x5EED0003)
    ap.add_argument("--t-fail", type=int, default=16,
                    help="T_fail = T_cleanup in rounds (reference: 5; see module doc)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=6.0, help="timed CPU rounds per rate (at least 1 round)")
    ap.add_argument("--cpu-threads", type=int, default=0, help="0 = nproc (OMP_NUM_THREADS, else the CPU count)")
    ap.add_argument("--no-secondary", action="store_true", help="skip the reference-constant / ring / C2 legs")
    ap.add_argument("--c4", action="store_true", help="world > 1: add the N=262,144 column-layout leg (on by "
                    "default at 8 GPUs)")
    ap.add_argument("--files", type=int, default=1 << 20,
                    help="placement leg (SURVEY.md §8d C5 files, after the timed rounds; 0 = skip)")
    return ap.parse_args()


def pmc_traffic(n, k, world, warmup, plane, tw, encoding):
    """Fabric-side bytes per k_round launch from the committed PMC summary of
    the same configuration, layout (sender plane, tile width), table encoding
    and warm-up (tools/pmc.sh -> profiles/*k_round_pmc*.json); a profile taken
    at another warm-up is refused (its timed rounds are another regime)."""
    import re

    def order(f):  # the latest round and session win: r03_s12 after r03_s6
        m = re.match(r"r(\d+)(?:_s(\d+))?", f.name)
        return (int(m.group(1)), int(m.group(2) or 0), f.name) if m else (0, 0, f.name)

    best = None
    for f in sorted((REPO / "profiles").glob("*k_round_pmc*.json"), key=order):
        try:
            d = json.loads(f.read_text())
        except (OSError, ValueError):
            continue
        c = d.get("config", {})
        enc = c.get("encoding", {4: "int32", 2: "u16", 1: "u8"}.get(c.get("cell_bytes", 4)))
        if (c.get("n") == n and c.get("k") == k and c.get("world", 1) == world and enc == encoding
                and c.get("warmup") == warmup and "traffic_bytes" in d
                and c.get("plane", 0) == plane and c.get("tile_width", 64) == tw):
            best = {"traffic_bytes": d["traffic_bytes"], "source": f"profiles/{f.name}",
                    "l2_hit_rate": d.get("l2_hit_rate")}
    return best


def progress(msg):
    print(f"[bench] {msg}", file=sys.stderr, flush=True)


def host_info():
    import subprocess
    model = "unknown"
    try:
        for line in subprocess.run(["lscpu"], capture_output=True, text=True).stdout.splitlines():
            if line.startswith("Model name"):
                model = line.split(":", 1)[1].strip()
    except OSError:
        pass
    try:
        nproc = int(subprocess.run(["nproc"], capture_output=True, text=True).stdout.strip())
    except (OSError, ValueError):
        nproc = os.cpu_count() or 1
    return {"nproc": nproc, "cpu_count": os.cpu_count(), "lscpu_model": model}


def oracle_rate(om, n, fanout, seed, t_fail, threads, seconds, peer_mode=0):
    """Whole-cluster rounds/s of the C oracle on the full N x N tables (full
    membership start, one untimed round, then >= 1 timed round and at least
    `seconds` of them)."""
    cfg = om.default_config(n, fanout=fanout, seed=seed, t_fail=t_fail, t_cleanup=t_fail, peer_mode=peer_mode)
    o = om.Oracle(cfg, threads=threads)
    o.init_full(2, 0, 0)
    o.step(1)
    done, t0 = 0, time.perf_counter()
    while True:
        o.step(1)
        done += 1
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    o.close()
    return done / el, done, el


def cpu_baseline(n, fanout, seed, seconds, threads, t_fail):
    """BASELINE.md "CPU baseline plan": the oracle (the same semantics as the
    GPU path) on this host: the benched configuration in full with nproc
    threads and with 1, N=4,096 (k=3) both ways, BASELINE config 1 (N=10,
    ring push, bootstrap + crash), and the literal list replay at N <= 256."""
    import numpy as np
    from oracle import oracle as om
    from oracle.listsim import ListSim
    om.build()
    host = host_info()
    threads = threads or int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or host["nproc"]
    b_round = 4.0 * n * n * (fanout + 4)  # SURVEY.md §8d int32 bytes per round
    progress(f"cpu baseline: tablesim N={n}, {threads} threads")
    full, done, el = oracle_rate(om, n, fanout, seed, t_fail, threads, seconds)
    progress("cpu baseline: 1 thread")
    one, done1, el1 = oracle_rate(om, n, fanout, seed, t_fail, 1, 0.0)
    progress("cpu baseline: N=4096, N=10, listsim")
    c2, _, _ = oracle_rate(om, 4096, 3, 0x5EED0002, 5, threads, 1.0)
    c2_1, _, _ = oracle_rate(om, 4096, 3, 0x5EED0002, 5, 1, 1.0)
    # BASELINE config 1: 10 members join one per round, ring push, member 7
    # crashes at r=30, 60 rounds (tablesim and the literal list replay)
    cfg1 = om.default_config(10, peer_mode=om.GH_PEER_RING, seed=0x5EED0001)
    o1 = om.Oracle(cfg1)
    t0 = time.perf_counter()
    for r in range(1, 61):
        ev = ([(om.GH_EV_JOIN, r - 1)] if r <= 10 else []) + ([(om.GH_EV_CRASH, 7)] if r == 30 else [])
        if ev:
            o1.apply_events(ev)
        o1.step(1)
    c1 = 60 / (time.perf_counter() - t0)
    o1.close()
    ls = {}
    for m in (64, 128, 256):
        hb = np.full((m, m), 2, np.int32)
        sim = ListSim.from_dense(hb, np.zeros((m, m), np.int32), np.ones(m, np.uint8), 0, seed=seed,
                                 peer_mode="pull", fanout=fanout)
        t0 = time.perf_counter()
        sim.step(1)
        ls[str(m)] = time.perf_counter() - t0
    return {
        "value": full, "unit": "rounds/s", "cores": threads, "kind": "port",
        "sample": f"oracle/tablesim.c (C, OpenMP, {threads} threads = nproc) on the full benched configuration: "
                  f"N={n} x {n} int32 hb/ts tables, k={fanout} Philox pull, full membership start, "
                  f"T_fail={t_fail}; {done} timed rounds in {el:.1f} s after one untimed round",
        "host": host,
        "host_gbs": b_round * full / 1e9,
        "host_gbs_note": "SURVEY.md §8d bytes per round 4*N^2*(k+4) x rounds/s",
        "value_1core": one,
        "sample_1core": f"the same on 1 thread: {done1} round(s) in {el1:.1f} s",
        "c2_n4096_k3_rounds_per_s": c2, "c2_n4096_k3_rounds_per_s_1core": c2_1,
        "c1_n10_ring_rounds_per_s": c1,
        "listsim_s_per_round": ls,
        "listsim_note": "oracle/listsim.py, the literal Go-list replay (pure Python, O(N^3) per round), "
                        "full membership, one round at each N",
    }


def secondary_legs(gs):
    """The engine at the reference's constants and on BASELINE config 2 (one
    engine at a time; outside the main timed region)."""
    out = {}

    def timed(cfg, warmup, steps, sched=None):
        eng = gs.Engine(cfg)
        eng.init_full(2, 0, 0)
        if warmup:
            eng.step(warmup)
        eng.set_timing(True)
        eng.sync()
        t0 = time.perf_counter()
        st = {}
        if sched:
            for r in range(1, steps + 1):
                if r in sched:
                    eng.apply_events(sched[r])
                s1 = eng.step(1)
                for k, v in s1.items():
                    st[k] = st.get(k, 0) + v
        else:
            st = eng.step(steps)
        eng.sync()
        el = time.perf_counter() - t0
        ms, launches = eng.read_timing()
        mode = eng.encoding_info(full=True)[2]
        eng.close()
        return {"rounds_per_s": steps / el, "k_round_ms": ms / max(launches, 1), "last_variant": "storm" if mode else
                "lean", "detections": st["detections"], "active_rows": st["active_rows"]}

    n = 65536
    progress("secondary legs")
    out["reference_timeouts"] = dict(
        workload=f"N={n}, k=4 pull, T_fail=T_cleanup=5 (slave/slave.go:24-25), full start, 12 warm-up rounds "
                 "(the round-6 detection storm and the round-7 collapse under the <4 guard), 20 timed rounds",
        **timed(gs.default_config(n, fanout=4, seed=0x5EED0003, t_fail=5, t_cleanup=5), 12, 20))
    out["ring_reference"] = dict(
        workload=f"N={n}, the reference's ring push (3 targets, slave/slave.go:515-524), T_fail=T_cleanup=5, "
                 "full start, 12 warm-up rounds, 20 timed rounds",
        **timed(gs.default_config(n, seed=0x5EED0003, t_fail=5, t_cleanup=5, peer_mode=gs.GH_PEER_RING), 12, 20))
    import numpy as np
    crash = np.random.default_rng(0x5EED0002).choice(np.arange(1, 4096), size=41, replace=False)
    out["c2_n4096"] = dict(
        workload="BASELINE config 2: N=4096, k=3 pull, T_fail=T_cleanup=5, full start, 1% crash (41 members) "
                 "at r=8, 64 rounds timed one gh_step call per round",
        **timed(gs.default_config(4096, fanout=3, seed=0x5EED0002), 0, 64,
                sched={8: [(gs.GH_EV_CRASH, int(c)) for c in crash]}))
    out["c3_crash_1pct"] = crash_leg(gs, n)
    return out


def crash_leg(gs, n, rounds=40):
    """The benched configuration (N=65,536, k=4 pull, T_fail = T_cleanup = 16,
    full start) with 1% of the members (655, Philox seed 0x5EED0003, tag
    CRASH: the set tests/test_gpu_fullsize.py checks against the oracle)
    crashing at r=8, rounds 1..40 timed one gh_step call per round: the
    healthy rounds, the crashed members' views ageing past T_fail, the
    detection round, the REMOVE wave and the tombstones' release. Reports
    rounds/s over all of them and, per k_round variant (gh_tier_info: 3 the
    nibble path, 1 storm, 2 / 0 lean 16-bit rule), its round count, mean
    k_round time (HIP events) and mean whole-round wall time (the gh_step
    call: every kernel of the round, the lane jobs included), plus a per-round
    trace (variant, lane jobs of the nibble path, wall ms)."""
    from gossipsim.scenario import crash_ids
    crashed = crash_ids(n, 0.01, 0x5EED0003)
    eng = gs.Engine(gs.default_config(n, fanout=4, seed=0x5EED0003, t_fail=16, t_cleanup=16))
    eng.init_full(2, 0, 0)
    eng.set_timing(True)
    names = {0: "lean_16bit_input", 1: "storm", 2: "lean_tier_input_16bit_rule", 3: "nibble_path"}
    per = {}
    tot = {"detections": 0, "tombstoned": 0, "released": 0, "remove_unknown": 0}
    first_det = None
    eng.sync()
    t0 = time.perf_counter()
    ms_prev = 0.0
    trace = []
    for r in range(1, rounds + 1):
        if r == 8:
            eng.apply_events([(gs.GH_EV_CRASH, int(c)) for c in crashed])
        t1 = time.perf_counter()
        st = eng.step(1)
        ms, _ = eng.read_timing()  # (synchronises)
        wall = (time.perf_counter() - t1) * 1e3
        v = names.get(eng.tier_info(full=True)[3], "?")
        jobs, redo = eng.job_info()
        e = per.setdefault(v, {"rounds": 0, "k_round_ms_sum": 0.0, "round_wall_ms_sum": 0.0, "lane_jobs": 0})
        e["rounds"] += 1
        e["k_round_ms_sum"] += ms - ms_prev
        e["round_wall_ms_sum"] += wall
        e["lane_jobs"] += jobs if v == "nibble_path" else 0
        trace.append([r, v, jobs if v == "nibble_path" else 0, round(wall, 3)])
        ms_prev = ms
        for key in tot:
            tot[key] += st[key]
        if st["detections"] and first_det is None:
            first_det = r
    eng.sync()
    el = time.perf_counter() - t0
    eng.close()
    for e in per.values():
        e["k_round_ms"] = e.pop("k_round_ms_sum") / max(e["rounds"], 1)
        e["round_wall_ms"] = e.pop("round_wall_ms_sum") / max(e["rounds"], 1)
    return {"workload": f"N={n}, k=4 pull, T_fail=T_cleanup=16, full start, 655 members (1%, Philox seed "
                        f"0x5eed0003) crash at r=8, rounds 1..{rounds} timed one gh_step call per round "
                        "(host round trips included)",
            "rounds_per_s": rounds / el, "first_detection_round": first_det, "variants": per, **tot,
            "trace": trace, "trace_fields": ["round", "variant", "lane_jobs", "round_wall_ms"]}


def placement_leg(gs, eng, n, files, t_fail):
    """SURVEY.md §8d placement figure, on the benched cluster after its timed
    rounds (outside them): put `files` files through gh_put (Init_replica /
    Handle_put_request, master/master.go:129-175), crash 1% of the members,
    run the rounds until they are detected and REMOVE'd, then one repair pass
    gh_repair (Update_metadata, master/master.go:74-127) from the master's
    view. Host-buffer calls: the times include the PCIe copies of the file
    ids, replicas and plan."""
    import ctypes as C
    import numpy as np
    f = np.arange(files, dtype=np.int32)
    eng.sync()
    t0 = time.perf_counter()
    rep, ver, st = eng.put(f)
    t_put = time.perf_counter() - t0
    rng = np.random.default_rng(0x5EED0005)
    crashed = rng.choice(np.arange(1, n), size=max(1, n // 100), replace=False)
    eng.apply_events([(gs.GH_EV_CRASH, int(c)) for c in crashed])
    # rounds until the detections stop (the last round's REMOVE is applied
    # in the round that reports none)
    rounds, det = 0, 0
    while rounds < 4 * t_fail + 8:
        d = eng.step(1)["detections"]
        rounds += 1
        if d == 0 and det:
            break
        det += d
    cap = files
    plan = (gs.PlanEntry * cap)()
    nout = C.c_int64()
    eng.sync()
    t0 = time.perf_counter()
    rc = eng.lib.gh_repair(eng.h, 0, plan, cap, C.byref(nout))
    t_rep = time.perf_counter() - t0
    if rc not in (gs.GH_OK, gs.GH_EPLACEMENT_STARVED):
        raise RuntimeError(f"gh_repair: {rc}")
    hit = np.isin(rep, crashed).any(axis=1)
    return {
        "files": files,
        "put_files_per_s": files / t_put,
        "put_ms": t_put * 1e3,
        "crashed_members": int(len(crashed)),
        "detections": int(det),
        "rounds_to_detection_and_remove": rounds,
        "files_with_crashed_replica": int(hit.sum()),
        "repair_plan_entries": int(min(nout.value, cap)),
        "repair_ms": t_rep * 1e3,
        "repair_files_per_s": files / t_rep,
        "replaced_files_per_s": int(min(nout.value, cap)) / t_rep,
        "note": "host-buffer C-ABI calls (PCIe copies included); files checked per second = files / repair time",
    }


def election_leg(gs, eng, n, t_fail):
    """SURVEY.md §8f f3 figure, after the placement leg (outside the timed
    rounds): crash the master (member 0), run the rounds until it is detected
    and REMOVE'd, then the per-round election scan gh_vote_scan over all N
    rows (updateMemberList's master check + revote_master's MemberList[0],
    slave/slave.go:451-457, 930-948), and gh_rebuild_meta
    (rebuild_file_meta, :986-1043) over the file table at the member the
    votes elect. Host-buffer calls, PCIe copies included."""
    import numpy as np
    eng.apply_events([(gs.GH_EV_CRASH, 0)])
    rounds, det = 0, 0
    while rounds < 4 * t_fail + 8:
        d = eng.step(1)["detections"]
        rounds += 1
        if d == 0 and det:
            break
        det += d
    mview = np.zeros(n, np.int32)
    eng.vote_scan(mview)  # first call allocates; time the second
    eng.sync()
    t0 = time.perf_counter()
    first, ln, has = eng.vote_scan(mview)
    t_scan = time.perf_counter() - t0
    alive = eng.alive()
    voters = (alive != 0) & (ln >= eng.cfg.min_members) & (has == 0)
    votes = np.bincount(first[voters & (first >= 0)], minlength=n)
    # Vote_num (self vote included) against the candidate's own list; the
    # check runs only when a remote vote arrives (Receive_vote :974-978)
    self_v = np.bincount(first[voters & (first == np.arange(n))], minlength=n)
    elected = np.flatnonzero((votes > ln // 2) & (votes - self_v > 0))
    out = {"rounds_to_detection_and_remove": rounds, "voters": int(voters.sum()),
           "vote_scan_ms": t_scan * 1e3, "rows_scanned_per_s": n / t_scan,
           "elected": int(elected[0]) if len(elected) else None}
    if len(elected) and eng.cfg.max_files > 0:
        eng.sync()
        t0 = time.perf_counter()
        f0, kept = eng.rebuild_meta(int(elected[0]))
        t_rb = time.perf_counter() - t0
        out.update({"rebuild_ms": t_rb * 1e3, "rebuild_files_per_s": eng.cfg.max_files / t_rb,
                    "files_kept": int(kept), "assign_new_master_to": int(f0)})
    out["note"] = "host-buffer C-ABI calls (PCIe copies included)"
    return out


def make_engine(gs, cfg, rank, world, dist):
    """One engine: the whole cluster (world 1) or rank `rank`'s shard of it
    over RCCL, the unique id broadcast from rank 0 over the gloo group."""
    if world > 1:
        box = [gs.comm_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(box, src=0)
        return gs.Engine(cfg, rank=rank, world=world, transport=gs.GH_COMM_RCCL, comm_id=box[0])
    return gs.Engine(cfg)


def rank_bytes(n, world, layout, ncols, tier4, plane, k):
    """Algorithmic bytes of one k_round launch on this rank: compulsory (each
    cell of the rank's rows x columns read once and written once: on the
    4-bit tier a lag nibble -- the sender plane itself -- and an age nibble,
    1 B in and 1 B out; on the 16-bit table 2 B in and out plus the 4-bit
    plane out and in), round 2's 8-bit model, the k sender gathers and
    SURVEY.md §8d's int32 model."""
    nrows_r = -(-n // world) if layout == "rows" else n
    if tier4:
        b_table, b_plane = 2.0 * nrows_r * ncols, 0.0
    else:
        b_table = 4.0 * nrows_r * ncols
        b_plane = 1.0 * nrows_r * ncols if plane else 0.0
    return {"rows": nrows_r, "cols": ncols, "compulsory": b_table + b_plane, "table": b_table, "plane": b_plane,
            "prev_model": 3.0 * nrows_r * ncols,
            "gather": (0.5 if (tier4 or plane) else 2.0) * nrows_r * ncols * k,
            "survey": 4.0 * nrows_r * ncols * (k + 4)}


def rank_roofline(rank, b, kern_ms, launches):
    """This rank's k_round: mean launch time (HIP events on its stream) and
    compulsory bytes / that time against the HBM peak."""
    avg_s = (kern_ms / 1e3) / max(launches, 1)
    ach = b["compulsory"] / avg_s / 1e9 if avg_s > 0 else 0.0
    return {"rank": rank, "rows": b["rows"], "cols": b["cols"], "avg_launch_ms": avg_s * 1e3, "launches": launches,
            "bytes_per_launch": b["compulsory"], "achieved": ach, "frac": ach / HBM_PEAK_GBS}


def gather_ranks(dist, obj):
    if dist is None:
        return [obj]
    out = [None] * dist.get_world_size()
    dist.all_gather_object(out, obj)
    return out


def max_over_ranks(dist, x):
    if dist is None:
        return x
    return max(gather_ranks(dist, x))


def timed_rounds(eng, dist, warmup, steps):
    """init_full, `warmup` untimed rounds, then `steps` rounds bracketed by a
    barrier and a device sync on both sides; returns (max-over-ranks seconds,
    stats, k_round ms, launches) with the engine's launch timing on."""
    eng.init_full(2, 0, 0)
    if warmup:
        eng.step(warmup)
    eng.set_timing(True)
    if dist is not None:
        dist.barrier()
    eng.sync()
    t0 = time.perf_counter()
    st = eng.step(steps)  # blocks until the device is done
    eng.sync()
    t1 = time.perf_counter()
    if dist is not None:
        dist.barrier()
    kern_ms, launches = eng.read_timing()
    eng.set_timing(False)
    return max_over_ranks(dist, t1 - t0), st, kern_ms, launches


def shard_leg(gs, args, rank, world, local, dist, n, layout, warmup, steps):
    """One more sharded configuration at world > 1 (outside the main timed
    region): rounds/s over all ranks, each rank's k_round roofline and, for
    the row layout, its ghost-row exchange (gh_exchange_info: the bytes the
    last round's ncclAllToAllv moved out of and into this rank, over xGMI on
    one node)."""
    cfg = gs.default_config(n, fanout=args.fanout, seed=args.seed, device=local, t_fail=args.t_fail,
                            t_cleanup=args.t_fail, max_files=0, peer_mode=gs.GH_PEER_PULL,
                            shard_layout=gs.GH_LAYOUT_ROWS if layout == "rows" else gs.GH_LAYOUT_COLUMNS)
    eng = make_engine(gs, cfg, rank, world, dist)
    try:
        ncols = eng.shard_info()[3]
        b = rank_bytes(n, world, layout, ncols, eng.tier_info()[0], eng.plane_info()[0], args.fanout)
        el, st, kern_ms, launches = timed_rounds(eng, dist, warmup, steps)
        mine = rank_roofline(rank, b, kern_ms, launches)
        if layout == "rows":
            x = eng.exchange_info()
            mine["exchange"] = x
            mine["xgmi_in_gbs"] = x["bytes_in"] / (el / steps) / 1e9
        mem = eng.memory_info()["device_bytes"]
    finally:
        eng.close()
    per_rank = gather_ranks(dist, mine)
    return {"workload": f"N={n}, k={args.fanout} Philox pull, T_fail=T_cleanup={args.t_fail}, full start, "
                        f"{warmup} warm-up rounds, {steps} timed rounds, {layout} layout over {world} GPUs",
            "n_members": n, "layout": layout, "rounds_per_s": steps / el, "ms_per_step": el / steps * 1e3,
            "detections": st["detections"], "table_bytes_per_rank": mem,
            "roofline_per_rank": per_rank,
            "frac_min": min(r["frac"] for r in per_rank), "frac_max": max(r["frac"] for r in per_rank)}


def multi_gpu_legs(gs, args, rank, world, local, dist):
    """world > 1: the other shard layout at the benched N (north_star's row
    layout when the main line times columns), and on 8 GPUs BASELINE config
    4's size, N=262,144, column layout (56 GB of tables per GPU)."""
    out = {}
    other = "rows" if args.layout == "columns" else "columns"
    progress(f"multi-GPU leg: {other} layout, N={args.n}")
    out[other] = shard_leg(gs, args, rank, world, local, dist, args.n, other, args.warmup, args.steps)
    if world == 8 or args.c4:
        progress("multi-GPU leg: config 4, N=262144, column layout")
        # (10 warm-up rounds: a heartbeat needs ~log5(262,144) ~ 8 rounds to reach every member)
        out["c4_n262144"] = shard_leg(gs, args, rank, world, local, dist, 262144, "columns", 10, 10)
    return out


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    import gossipsim as gs

    n, k = args.n, args.fanout
    cfg = gs.default_config(n, fanout=k, seed=args.seed, device=local, t_fail=args.t_fail, t_cleanup=args.t_fail,
                            max_files=args.files if world == 1 else 0,
                            peer_mode=gs.GH_PEER_RING if args.peer_mode == "ring" else gs.GH_PEER_PULL,
                            detect_mode=gs.GH_DETECT_QUIRK if args.detect == "quirk" else gs.GH_DETECT_CANONICAL,
                            shard_layout=gs.GH_LAYOUT_ROWS if args.layout == "rows" else gs.GH_LAYOUT_COLUMNS)
    if world > 1:
        import torch.distributed as dist  # noqa: F811
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo", rank=rank, world_size=world)
    eng = make_engine(gs, cfg, rank, world, dist)
    _, _, _, ncols = eng.shard_info()
    plane = eng.plane_info()[0]
    tier4 = eng.tier_info()[0]  # steady-state cells: a lag nibble (the plane) + an age nibble (escapes: 16-bit)
    tile_w = int(os.environ.get("GH_TILE_W", "256" if plane else "64"))
    b = rank_bytes(n, world, args.layout, ncols, tier4, plane, k)
    elapsed, st, kern_ms, launches = timed_rounds(eng, dist, args.warmup, args.steps)
    exch = eng.exchange_info() if args.layout == "rows" else None
    plane_fb = eng.plane_info()[2]
    tier_last = eng.tier_info()
    tier_last_var = eng.tier_info(full=True)[3]
    placement = None
    if world == 1 and args.files > 0:
        progress("placement and election legs")
        placement = placement_leg(gs, eng, n, args.files, args.t_fail)
        placement["election"] = election_leg(gs, eng, n, args.t_fail)
    mem = eng.memory_info()
    eng.close()
    per_rank = gather_ranks(dist, rank_roofline(rank, b, kern_ms, launches))
    secondary = None
    if not args.no_secondary:
        secondary = secondary_legs(gs) if world == 1 else multi_gpu_legs(gs, args, rank, world, local, dist)

    if rank != 0:
        return
    line = build_line(args, world, elapsed, st, b, kern_ms, launches, per_rank, tier4, plane, tile_w, exch, plane_fb,
                      tier_last, tier_last_var, mem, secondary, placement)
    if world == 1 and not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline(n, k, args.seed, args.cpu_seconds, args.cpu_threads, args.t_fail)
    print(json.dumps(line), flush=True)


def build_line(args, world, elapsed, st, b, kern_ms, launches, per_rank, tier4, plane, tile_w, exch, plane_fb,
               tier_last, tier_last_var, mem, secondary, placement):
    """The one JSON line (rank 0): value = rounds / max-over-ranks seconds of
    the timed region; roofline = rank 0's k_round (roofline_per_rank: every
    rank's)."""
    n, k = args.n, args.fanout
    value = args.steps / elapsed
    encoding = "t4" if tier4 else "u16"
    traffic = pmc_traffic(n, k, world, args.warmup, plane, tile_w, encoding)
    tier_cur, tier_esc = tier_last[1], tier_last[2]
    avg_s = (kern_ms / 1e3) / max(launches, 1)
    b_compulsory, b_prev_model, b_gather = b["compulsory"], b["prev_model"], b["gather"]
    achieved = b_compulsory / avg_s / 1e9
    nrows_r, ncols = b["rows"], b["cols"]
    line = {
        "metric": "gossip rounds/sec at N=65,536 members (achieved HBM GB/s, % of peak)",
        "value": value,
        "unit": "rounds/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        # the arithmetic is int32-exact (heartbeats over the full int32 range
        # through the 16-bit escapes and the int32 wide arena); "storage" is
        # the steady-state encoding the round streams
        "dtype": "int32",
        "storage": ("4-bit lag + 4-bit age per cell (the lag nibbles are the sender plane); escaped chunks "
                    "16-bit, wide segments int32") if tier4 else "16-bit narrow codes, wide segments int32",
        "data": "synthetic",
        "config": {
            "workload": f"BASELINE config 3: N={n} members, "
                        + (f"fanout k={k} Philox pull" if args.peer_mode == "pull" else "reference ring push (3 targets)")
                        + (", quirk detection" if args.detect == "quirk" else "") + ", full membership "
                        f"start (hb=2, ts=0), {args.warmup} warm-up rounds to the steady state, "
                        f"T_fail=T_cleanup={args.t_fail} rounds, seed {hex(args.seed)}",
            "t_fail": args.t_fail,
            "n_members": n, "fanout": k, "global_batch": n, "seq_len": n,
            "parallelism": (f"row-shard x{world} (RCCL alltoallv)" if args.layout == "rows" else
                            f"column-shard x{world} (RCCL)") if world > 1 else "single",
            "rows_per_gpu": nrows_r,
            "columns_per_gpu": ncols,
            "rounds_checked": {"detections": st["detections"], "active_rows": st["active_rows"]},
        },
        "roofline": {
            "bound": "hbm", "kernel": "k_round", "achieved": achieved, "peak": HBM_PEAK_GBS,
            "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
            "traffic": traffic["traffic_bytes"] if traffic else None,
            "traffic_source": traffic["source"] if traffic else None,
            "bytes_per_launch": b_compulsory,
            "bytes_model": ("compulsory: 2*N*ncols (4-bit tier: lag nibble + age nibble per cell read + written "
                            "once; the lag nibbles are the sender plane the gathers read)" if tier4 else
                            "compulsory: " + ("5" if plane else "4") + "*N*ncols (2-byte cells read + written once"
                            + (", 4-bit sender plane written + read once" if plane else "") + ")"),
            "table_bytes_per_launch": b["table"], "plane_bytes_per_launch": b["plane"],
            "prev_model_bytes_per_launch": b_prev_model,
            "frac_prev_model": b_prev_model / avg_s / 1e9 / HBM_PEAK_GBS,
            "avg_launch_ms": avg_s * 1e3, "launches": launches,
            "gather_bytes_per_launch": b_gather, "gather_achieved": b_gather / avg_s / 1e9,
            "survey_bytes_per_launch": b["survey"],
            "frac_of_measured_copy_peak": achieved / HBM_MEASURED_GBS,
            # fabric-side bytes (FETCH_SIZE x2 + WRITE_SIZE; Infinity-Cache
            # hits included) over the same duration; traffic / compulsory =
            # the sender gathers that missed L2
            "traffic_achieved": traffic["traffic_bytes"] / avg_s / 1e9 if traffic else None,
            "traffic_over_compulsory": traffic["traffic_bytes"] / b_compulsory if traffic else None,
            "l2_hit_rate": traffic["l2_hit_rate"] if traffic else None,
        },
        "cpu_baseline": None,
        "memory": {"table_bytes": mem["device_bytes"], "wide_slots_per_buffer": mem["wide_cap"],
                   "wide_slots_used": mem["wide_used"]},
        "exchange": exch,
        "layout": {"tile_width": tile_w, "sender_plane": bool(plane), "shards": args.layout,
                   "plane_fallback_waves_last_round": plane_fb, "tier4": bool(tier4),
                   "tier4_current": bool(tier_cur), "tier4_escaped_chunks_last_round": tier_esc,
                   "last_variant": {0: "lean_16bit_input", 1: "storm", 2: "lean_tier_input_16bit_rule",
                                    3: "nibble_path"}.get(tier_last_var, "?")},
        "roofline_per_rank": per_rank,
        "secondary": secondary,
        "placement": placement,
    }
    return line


if __name__ == "__main__":
    main()
