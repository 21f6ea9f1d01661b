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
  roofline: the round kernel (k_round) — algorithmic bytes per launch
            2*N*ncols*(k+2): own segment in, k peer segments in, own segment
            out, 2-byte narrow cells (DESIGN.md "Kernels"; SURVEY.md §8d's
            4*N^2*(k+4) counted int32 hb and ts streams, which the narrow
            age-encoded cells no longer move, reported as
            survey_bytes_per_launch) / its mean duration from HIP events on
            the engine's stream; peak 8.0 TB/s (MI355X_MICROARCH.md);
            traffic = HBM-side bytes per launch from the rocprofv3 PMC passes of
            tools/pmc.sh for this configuration (profiles/, null if none).
  cpu_baseline: the CPU restatement (oracle/tablesim.c, "port") timed on this
            host on a bounded sample (rank 0, N=1 only).
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
    ap.add_argument("--warmup", type=int, default=12)
    ap.add_argument("--n", type=int, default=65536)
    ap.add_argument("--fanout", type=int, default=4)
    ap.add_argument("--peer-mode", choices=("pull", "ring"), default="pull",
                    help="pull: k Philox peers (BASELINE configs 2-4); ring: the reference's ring push")
    ap.add_argument("--detect", choices=("canonical", "quirk"), default="canonical")
    ap.add_argument("--seed", type=lambda s: int(s, 0), default=0x5EED0003)
    ap.add_argument("--t-fail", type=int, default=16,
                    help="T_fail = T_cleanup in rounds (reference: 5; see module doc)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-rows", type=int, default=2048, help="observer rows in the CPU sample")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--cpu-threads", type=int, default=0, help="0 = min(16, cores)")
    ap.add_argument("--files", type=int, default=1 << 20,
                    help="placement leg (SURVEY.md §8d C5 files, after the timed rounds; 0 = skip)")
    return ap.parse_args()


def pmc_traffic(n, k, world):
    """HBM-side bytes per k_round launch from the committed PMC summary of
    the same configuration (tools/pmc.sh -> profiles/*k_round_pmc*.json)."""
    best = None
    for f in sorted((REPO / "profiles").glob("*k_round_pmc*.json")):
        try:
            d = json.loads(f.read_text())
        except (OSError, ValueError):
            continue
        c = d.get("config", {})
        if (c.get("n") == n and c.get("k") == k and c.get("world", 1) == world and c.get("cell_bytes", 4) == 2
                and "traffic_bytes" in d):
            best = {"traffic_bytes": d["traffic_bytes"], "source": f"profiles/{f.name}"}
    return best


def cpu_rate(n, fanout, seed, rows, seconds, threads, t_fail):
    """Whole-cluster rounds/s of the C oracle on `rows` observer rows of an
    N-column table (peers drawn among the sampled rows), scaled by rows/N."""
    from oracle import oracle as om
    cfg = om.default_config(n, fanout=fanout, seed=seed, t_fail=t_fail, t_cleanup=t_fail)
    o = om.Oracle(cfg, rows=rows, threads=threads)
    o.init_full(2, 0, 0)
    o.step(1)  # first touch
    done, t0 = 0, time.perf_counter()
    while True:
        o.step(1)
        done += 1
        el = time.perf_counter() - t0
        if el >= seconds or done >= 50:
            break
    o.close()
    return (rows / n) / (el / done), done, el


def cpu_baseline(n, fanout, seed, rows, seconds, threads, t_fail):
    """Time the C oracle (same semantics) on `rows` observer rows of an
    N-column table; peers are drawn among the sampled rows. Also one core on
    the same sample (the parallel run plus a 1-core run)."""
    from oracle import oracle as om
    om.build()
    threads = threads or min(16, os.cpu_count() or 1)
    rows_per_s, done, el = cpu_rate(n, fanout, seed, rows, seconds, threads, t_fail)
    rows1 = rows
    one, done1, el1 = cpu_rate(n, fanout, seed, rows1, seconds / 2, 1, t_fail)
    rounds_per_s = rows_per_s
    cpu = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                cpu = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return {
        "value": rounds_per_s, "unit": "rounds/s", "cores": threads, "kind": "port",
        "sample": f"oracle/tablesim.c (OpenMP, {threads} threads) on {rows} of {n} observer rows x {n} columns, "
                  f"k={fanout} peers drawn among the sampled rows, {done} rounds in {el:.1f} s, scaled by "
                  f"rows/N to whole-cluster rounds/s; host CPU: {cpu}",
        "value_1core": one,
        "sample_1core": f"the same on 1 thread, {rows1} observer rows, {done1} rounds in {el1:.1f} s",
    }


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
                            detect_mode=gs.GH_DETECT_QUIRK if args.detect == "quirk" else gs.GH_DETECT_CANONICAL)
    if world > 1:
        import torch.distributed as dist  # noqa: F811
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo", rank=rank, world_size=world)
        box = [gs.comm_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(box, src=0)
        eng = gs.Engine(cfg, rank=rank, world=world, transport=gs.GH_COMM_RCCL, comm_id=box[0])
    else:
        eng = gs.Engine(cfg)
    _, _, _, ncols = eng.shard_info()
    eng.init_full(2, 0, 0)
    if args.warmup:
        eng.step(args.warmup)
    eng.set_timing(True)

    def barrier():
        if dist is not None:
            dist.barrier()

    barrier()
    eng.sync()
    t0 = time.perf_counter()
    st = eng.step(args.steps)  # blocks until the device is done
    eng.sync()
    t1 = time.perf_counter()
    barrier()
    elapsed = t1 - t0
    if dist is not None:
        import torch
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    kern_ms, launches = eng.read_timing()
    eng.set_timing(False)
    placement = None
    if world == 1 and args.files > 0:
        placement = placement_leg(gs, eng, n, args.files, args.t_fail)
        placement["election"] = election_leg(gs, eng, n, args.t_fail)
    eng.close()

    if rank != 0:
        return
    value = args.steps / elapsed
    # algorithmic bytes of one k_round launch (this rank's columns)
    b_round = 2.0 * n * ncols * (k + 2)        # narrow cells: own in + out, k peers in
    b_survey = 4.0 * n * ncols * (k + 4)       # SURVEY.md §8d (int32 hb + a ts stream)
    b_compulsory = 4.0 * n * ncols             # each narrow cell read and written once
    traffic = pmc_traffic(n, k, world)
    avg_s = (kern_ms / 1e3) / max(launches, 1)
    achieved = b_round / avg_s / 1e9
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
        "dtype": "int16",
        "data": "synthetic",
        "config": {
            "workload": f"BASELINE config 3: N={n} members, "
                        + (f"fanout k={k} Philox pull" if args.peer_mode == "pull" else "reference ring push (3 targets)")
                        + (", quirk detection" if args.detect == "quirk" else "") + ", full membership "
                        f"start (hb=2, ts=0), {args.warmup} warm-up rounds to the steady state, "
                        f"T_fail=T_cleanup={args.t_fail} rounds, seed {hex(args.seed)}",
            "t_fail": args.t_fail,
            "n_members": n, "fanout": k, "global_batch": n, "seq_len": n,
            "parallelism": f"column-shard x{world} (RCCL)" if world > 1 else "single",
            "columns_per_gpu": ncols,
            "rounds_checked": {"detections": st["detections"], "active_rows": st["active_rows"]},
        },
        "roofline": {
            "bound": "hbm", "kernel": "k_round", "achieved": achieved, "peak": HBM_PEAK_GBS,
            "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
            "traffic": traffic["traffic_bytes"] if traffic else None,
            "traffic_source": traffic["source"] if traffic else None,
            "bytes_per_launch": b_round, "survey_bytes_per_launch": b_survey,
            "avg_launch_ms": avg_s * 1e3, "launches": launches,
            "compulsory_bytes_per_launch": b_compulsory,
            "compulsory_achieved": b_compulsory / avg_s / 1e9,
            "frac_of_measured_copy_peak": achieved / HBM_MEASURED_GBS,
            # the measured HBM-side bytes over the same duration: above 1 the
            # algorithmic frac counts sender re-reads the on-die caches serve
            "traffic_achieved": traffic["traffic_bytes"] / avg_s / 1e9 if traffic else None,
            "traffic_frac": traffic["traffic_bytes"] / avg_s / 1e9 / HBM_PEAK_GBS if traffic else None,
        },
        "cpu_baseline": None,
        "placement": placement,
    }
    if world == 1 and not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline(n, k, args.seed, args.cpu_rows, args.cpu_seconds, args.cpu_threads,
                                            args.t_fail)
    print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
