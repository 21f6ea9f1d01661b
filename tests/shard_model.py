"""TEST INFRASTRUCTURE: a numpy model of the column-sharded round protocol of
libgossiphip (DESIGN.md "Multi-GPU", csrc/gossiphip.cpp process_events /
decide_active / build_inboxes, csrc/round.hip), run as one torch.distributed
(gloo, CPU) rank per shard.

Each rank holds all N rows for its member columns [col0, col0+ncol) with
ncs = roundup(ceil(N/G), 32), exactly like the HIP engine, computes only
column-local work and exchanges only what the HIP host code exchanges, with
the same collectives:
  leave / join / placement  all_gather of the leavers' / introducer's /
                            master's presence bits over the local columns
  join                      all_reduce(sum) of the introducer adds
  guard                     all_reduce(sum) of local present counts + |D|,
                            then of the post-REMOVE counts of undecided rows
  pull                      all_gather of the local receivers' draw-validity bytes
  ring                      all_gather of (local list length, sender position),
                            all_reduce(max) of the targets
  read-outs                 all_gather of the D bitmap, all_reduce(max) of
                            det_any, all_reduce(sum) of the counters
Per-column work (REMOVE delivery, heartbeat, detection, cleanup, merge) is the
SPEC §2 rule applied to the slice. Comparing every rank's slice with the full
oracle/tablesim state each round shows that the decomposition and the
exchange set are complete — the property the GPU code relies on at N>1.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.distributed as dist

from oracle import philox

ABSENT, TOMB = -1, -2
NOSH = -(1 << 40)


def _gather_rows_bool(local: np.ndarray, ncs: int, n: int) -> np.ndarray:
    """[nr][ncol] local bits -> [nr][n] global (pads each slice to ncs)."""
    nr = local.shape[0]
    pad = np.zeros((nr, ncs), np.int64)
    pad[:, : local.shape[1]] = local
    parts = [torch.zeros((nr, ncs), dtype=torch.int64) for _ in range(dist.get_world_size())]
    dist.all_gather(parts, torch.from_numpy(pad))
    return torch.cat(parts, dim=1).numpy()[:, :n].astype(bool)


def _allreduce(x: np.ndarray, op=dist.ReduceOp.SUM) -> np.ndarray:
    t = torch.from_numpy(np.ascontiguousarray(x, dtype=np.int64))
    dist.all_reduce(t, op=op)
    return t.numpy()


class ShardModel:
    def __init__(self, n, fanout=3, peer_mode=0, seed=1, t_fail=5, t_cleanup=5, min_members=4, introducer=0):
        self.rank, self.world = dist.get_rank(), dist.get_world_size()
        self.n, self.k, self.pm, self.seed = n, fanout, peer_mode, seed
        self.t_fail, self.t_cleanup, self.minm, self.I = t_fail, t_cleanup, min_members, introducer
        self.ncs = ((n + self.world - 1) // self.world + 31) // 32 * 32
        self.col0 = self.rank * self.ncs
        self.ncol = max(0, min(self.ncs, n - self.col0))
        self.hb = np.full((n, self.ncol), ABSENT, np.int64)
        self.ts = np.zeros((n, self.ncol), np.int64)
        self.alive = np.zeros(n, bool)
        self.dcnt = np.zeros(self.ncol, np.int64)
        self.dmin = np.full(self.ncol, np.iinfo(np.int64).max, np.int64)
        self.det_any = np.zeros(n, bool)
        self.round = 0
        self.pending = []
        # SPEC D7: per local column the ts of the introducer's RecentFailList
        # entry beside its present member (a join of a tombstoned member)
        self.shadow = np.full(self.ncol, NOSH, np.int64)

    # ---- state -------------------------------------------------------------
    def import_full(self, hb, ts, alive, round_):
        sl = slice(self.col0, self.col0 + self.ncol)
        self.hb = np.array(hb, np.int64)[:, sl].copy()
        self.ts = np.array(ts, np.int64)[:, sl].copy()
        self.alive = np.array(alive, bool)
        self.round = round_
        self.dcnt[:] = 0
        self.dmin[:] = np.iinfo(np.int64).max
        self.shadow[:] = NOSH

    def apply_events(self, ev):
        self.pending.extend(ev)

    def _remove(self, j, lc, st):  # removeMember, slave/slave.go:276-286
        x = self.hb[j, lc]
        if x >= 0 and j == self.I and self.shadow[lc] != NOSH:  # D7: the RecentFailList entry stays
            self.hb[j, lc] = TOMB
            self.ts[j, lc] = self.shadow[lc]
            self.shadow[lc] = NOSH
        elif x >= 0:
            self.hb[j, lc] = TOMB
            st["tombstoned"] += 1
        elif x == ABSENT:
            st["remove_unknown"] += 1

    def _local(self, c):
        lc = c - self.col0
        return lc if 0 <= lc < self.ncol else None

    def _events(self, r, st):
        ev, self.pending = self.pending, []
        for kind, c in ev:
            if kind == 3:
                self.alive[c] = False
        leavers = []
        for kind, c in ev:
            if kind == 2 and self.alive[c]:
                self.alive[c] = False
                leavers.append(c)
        if leavers:
            bits = _gather_rows_bool(self.hb[leavers] >= 0, self.ncs, self.n)
            for q, c in enumerate(leavers):
                lc = self._local(c)
                if lc is None:
                    continue
                for j in range(self.n):
                    if j != c and self.alive[j] and bits[q, j]:
                        self._remove(j, lc, st)
        joiners = [c for kind, c in ev if kind == 1]
        for c in joiners:
            if not self.alive[c]:
                self.hb[c, :] = ABSENT
                self.ts[c, :] = 0
                if c == self.I:
                    self.shadow[:] = NOSH
                self.alive[c] = True
        I = self.I
        if joiners and self.alive[I]:
            added = 0
            for c in joiners:
                lc = self._local(c)
                if lc is not None and self.hb[I, lc] < 0:
                    if self.hb[I, lc] == TOMB:  # D7: its tombstone stays beside it
                        self.shadow[lc] = self.ts[I, lc]
                    self.hb[I, lc] = 0
                    self.ts[I, lc] = r
                    added += 1
            added = int(_allreduce(np.array([added]))[0])
            bits = _gather_rows_bool((self.hb[[I]] >= 0), self.ncs, self.n)[0]
            if added:
                msg = self.hb[I].copy()
                for j in range(self.n):
                    if j == I or not self.alive[j] or not bits[j]:
                        continue
                    upd = (msg >= 0) & (self.hb[j] >= ABSENT) & (msg > self.hb[j])
                    self.hb[j, upd] = msg[upd]
                    self.ts[j, upd] = r
                    st["merged_cells"] += int(upd.sum())

    def _removes_at(self, j):
        """bool[ncol]: REMOVE of each local column is delivered at row j."""
        return (self.dcnt > 0) & ~((self.dcnt == 1) & (self.dmin == j))

    def _decide_active(self):
        cntl = (self.hb >= 0).sum(axis=1)
        ndl = int((self.dcnt > 0).sum())
        g = _allreduce(np.concatenate([cntl, [ndl]]))
        cntg, ndg = g[: self.n], g[self.n]
        active = np.zeros(self.n, bool)
        und = np.zeros(self.n, bool)
        post = np.zeros(self.n, np.int64)
        for i in range(self.n):
            if not self.alive[i] or cntg[i] < self.minm:
                continue
            if cntg[i] - ndg >= self.minm:
                active[i] = True
            else:
                und[i] = True
                post[i] = int(((self.hb[i] >= 0) & ~self._removes_at(i)).sum())
        post = _allreduce(post)
        active[und] = post[und] >= self.minm
        return active

    def step(self):
        r = self.round + 1
        st = dict(rounds=1, last_round=r, detections=0, failed_members=0, remove_unknown=0, ring_empty=0,
                  active_rows=0, merged_cells=0, released=0, tombstoned=0)
        self._events(r, st)
        active = self._decide_active()
        if self.rank == 0:
            st["active_rows"] = int(active.sum())
        self.det_any[:] = False
        ndcnt = np.zeros(self.ncol, np.int64)
        ndmin = np.full(self.ncol, np.iinfo(np.int64).max, np.int64)
        gcols = np.arange(self.col0, self.col0 + self.ncol)
        for i in range(self.n):
            if not self.alive[i]:
                continue
            rm = self._removes_at(i)
            sh = (self.shadow != NOSH) if i == self.I else np.zeros(self.ncol, bool)
            dual = rm & (self.hb[i] >= 0) & sh  # D7: the RecentFailList entry (and its ts) stays
            self.ts[i, dual] = self.shadow[dual]
            self.shadow[dual] = NOSH
            sh &= ~dual
            st["tombstoned"] += int((rm & (self.hb[i] >= 0) & ~dual).sum())
            st["remove_unknown"] += int((rm & (self.hb[i] == ABSENT)).sum())
            self.hb[i, rm & (self.hb[i] >= 0)] = TOMB
            if not active[i]:
                self.ts[i, self.hb[i] >= 0] = r
                continue
            own = gcols == i
            up = own & (self.hb[i] >= 0)
            self.hb[i, up] += 1
            self.ts[i, up] = r
            det = (~own) & (self.hb[i] > 1) & (self.ts[i] < r - self.t_fail)
            if det.any():
                self.hb[i, det] = TOMB
                dd = det & sh
                self.ts[i, dd] = self.shadow[dd]
                self.shadow[dd] = NOSH
                sh &= ~dd
                st["detections"] += int(det.sum())
                ndcnt[det] += 1
                ndmin[det] = np.minimum(ndmin[det], i)
                self.det_any[i] = True
            rel = (self.hb[i] == TOMB) & (self.ts[i] < r - self.t_cleanup)
            self.hb[i, rel] = ABSENT
            st["released"] += int(rel.sum())
            old = sh & (self.shadow < r - self.t_cleanup)
            self.shadow[old] = NOSH
            st["released"] += int(old.sum())
        snap = self.hb.copy()
        inbox = self._inbox_pull(snap, active, r) if self.pm == 0 else self._inbox_ring(snap, active, st)
        for i in range(self.n):
            if not self.alive[i] or not inbox[i]:
                continue
            m = np.full(self.ncol, -1, np.int64)
            for s in set(inbox[i]):
                m = np.maximum(m, np.where(snap[s] >= 0, snap[s], -1))
            upd = (self.hb[i] >= ABSENT) & (m > self.hb[i])
            self.hb[i, upd] = m[upd]
            self.ts[i, upd] = r
            st["merged_cells"] += int(upd.sum())
        self.dcnt, self.dmin = ndcnt, ndmin
        st["failed_members"] = int((ndcnt > 0).sum())
        keys = sorted(st)
        tot = _allreduce(np.array([st[k] for k in keys]))
        out = dict(zip(keys, (int(x) for x in tot)))
        out["rounds"], out["last_round"] = 1, r
        self.round = r
        return out

    def _inbox_pull(self, snap, active, r):
        """Receivers in the local columns draw and validate their peers
        (k_peers_pull); one byte per receiver, the validity bits of its k
        draws, is all_gathered, and every shard redraws the peers of every
        receiver and keeps the valid ones in draw order (k_inbox_bits)."""
        loc = np.zeros(self.ncs, np.uint8)
        for t in range(self.ncol):
            i = self.col0 + t
            if not self.alive[i] or self.n < 2:
                continue
            for q in range(self.k):
                s = philox.peer(self.seed, i, r, q, self.n)
                if self.alive[s] and active[s] and snap[s, t] >= 0:
                    loc[t] |= 1 << q
        parts = [torch.zeros(self.ncs, dtype=torch.uint8) for _ in range(self.world)]
        dist.all_gather(parts, torch.from_numpy(loc))
        bits = torch.cat(parts).numpy()[: self.n]
        return [[philox.peer(self.seed, i, r, q, self.n) for q in range(self.k) if (int(bits[i]) >> q) & 1]
                for i in range(self.n)]

    def _inbox_ring(self, snap, active, st):
        """k_ring_count / all_gather / k_ring_select / all_reduce(max)."""
        gcols = np.arange(self.col0, self.col0 + self.ncol)
        loc = np.zeros((self.n, 2), np.int64)
        for s in range(self.n):
            loc[s] = (0, -1)
            if not (self.alive[s] and active[s]):
                continue
            pres = snap[s] >= 0
            loc[s, 0] = int(pres.sum())
            ls = s - self.col0
            if 0 <= ls < self.ncol and pres[ls]:
                loc[s, 1] = int(pres[:ls].sum())
        parts = [torch.zeros((self.n, 2), dtype=torch.int64) for _ in range(self.world)]
        dist.all_gather(parts, torch.from_numpy(loc))
        allc = torch.stack(parts).numpy()  # [world][n][2]
        tg = np.full((self.n, 3), -1, np.int64)
        for s in range(self.n):
            if not (self.alive[s] and active[s]):
                continue
            L = int(allc[:, s, 0].sum())
            if L == 0:
                if self.rank == 0:
                    st["ring_empty"] += 1
                continue
            owner = s // self.ncs
            lp = allc[owner, s, 1]
            idx = int(allc[:owner, s, 0].sum() + lp) if lp >= 0 else -1
            before = int(allc[: self.rank, s, 0].sum())
            present_cols = gcols[snap[s] >= 0]
            for q, w in enumerate((idx - 1, idx + 1, idx + 2)):
                v = int(np.fmod(w, L))
                v = v + L if v < 0 else v
                if before <= v < before + len(present_cols):
                    tg[s, q] = present_cols[v - before]
        tg = _allreduce(tg, dist.ReduceOp.MAX)
        inbox = [[] for _ in range(self.n)]
        for s in range(self.n):
            for t in tg[s]:
                if t >= 0 and self.alive[t]:
                    inbox[t].append(s)
        return inbox

    # ---- read-outs (collective) -------------------------------------------
    def read_failed(self):
        bits = _gather_rows_bool((self.dcnt > 0)[None, :], self.ncs, self.n)[0]
        return [c for c in range(self.n) if bits[c]]

    def read_detectors(self):
        anyd = _allreduce(self.det_any.astype(np.int64), dist.ReduceOp.MAX)
        return [i for i in range(self.n) if anyd[i]]

    def vote_scan(self, mview):
        """gh_vote_scan's exchange (csrc/elect.hip k_vote_scan + gossiphip.cpp):
        per row, n - (first present local member) and (mview[i] present
        locally) reduced with MAX, the local present counts with SUM."""
        pres = self.hb >= 0
        n = self.n
        loc_first = np.where(pres.any(axis=1), n - (self.col0 + pres.argmax(axis=1)), 0) if self.ncol else np.zeros(n)
        lc = np.asarray(mview) - self.col0
        ok = (lc >= 0) & (lc < self.ncol)
        has = np.zeros(n, np.int64)
        rows = np.flatnonzero(ok)
        has[rows] = pres[rows, lc[rows]]
        red = _allreduce(np.concatenate([loc_first, has]).astype(np.int64), dist.ReduceOp.MAX)
        ln = _allreduce(pres.sum(axis=1).astype(np.int64))
        first = np.where(red[:n] > 0, n - red[:n], -1)
        return first, ln, red[n:]

    def master_list(self, master=0):
        """Placement candidates (k_candidates) from the gathered master row."""
        bits = _gather_rows_bool(self.hb[[master]] >= 0, self.ncs, self.n)[0]
        return [c for c in range(self.n) if bits[c]]


def worker(rank, world, port, n, rounds, cfg, churn_seed, files_at):
    """One gloo rank: replay a churn scenario on the model and check this
    rank's column slice, the counters and the read-outs against the full
    oracle every round."""
    import os
    import sys
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import scenarios as sc
        from oracle import oracle as om
        ocfg = om.default_config(n, peer_mode=cfg["peer_mode"], fanout=cfg["fanout"], seed=cfg["seed"],
                                 t_fail=cfg["t_fail"], t_cleanup=cfg["t_cleanup"], max_files=64)
        orc = om.Oracle(ocfg)
        m = ShardModel(n, fanout=cfg["fanout"], peer_mode=cfg["peer_mode"], seed=cfg["seed"],
                       t_fail=cfg["t_fail"], t_cleanup=cfg["t_cleanup"])
        init = sc.full_state(n)
        orc.import_state(*init, 0)
        m.import_full(*init, 0)
        sched = sc.random_churn(n, rounds, churn_seed, p_crash=0.05, p_leave=0.03, p_join=0.08)
        sl = slice(m.col0, m.col0 + m.ncol)
        for r in range(1, rounds + 1):
            ev = sched.get(r, [])
            orc.apply_events(ev)
            m.apply_events(ev)
            s_cpu, s_mod = orc.step(1), m.step()
            assert s_cpu == s_mod, f"rank {rank} round {r}: oracle {s_cpu} != model {s_mod}"
            hb, ts, alive = orc.export_state()
            assert np.array_equal(hb[:, sl], m.hb), f"rank {rank} round {r}: hb slice differs"
            mts = sc.export_view(m.hb, m.ts, r, cfg["t_cleanup"])[1]
            assert np.array_equal(ts[:, sl], mts), f"rank {rank} round {r}: ts slice differs"
            assert np.array_equal(alive.astype(bool), m.alive)
            bm = orc.read_failed()
            assert m.read_failed() == [c for c in range(n) if bm[c >> 5] >> (c & 31) & 1]
            assert m.read_detectors() == list(orc.read_detectors())
            if r in files_at:
                assert m.master_list() == [c for c in range(n) if hb[0, c] >= 0]
            from oracle import election as el
            mv = np.random.default_rng(r).integers(0, n, n)
            for a, b in zip(m.vote_scan(mv), el.vote_scan(hb, mv)):
                assert np.array_equal(a, b), f"rank {rank} round {r}: vote scan differs"
        sys.stdout.flush()
    finally:
        dist.destroy_process_group()
