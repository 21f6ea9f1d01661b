"""TEST INFRASTRUCTURE: a numpy model of the ROW-sharded round protocol of
libgossiphip (GH_LAYOUT_ROWS, the north_star layout; DESIGN.md "Multi-GPU",
csrc/gossiphip.cpp process_events / decide_active / build_inboxes /
round_ghosts / ghost_setup + ghost_move, csrc/rows.hip), run as one
torch.distributed (gloo, CPU) rank per shard.

Rank g holds observer rows [g*nrs, g*nrs + nrows) (nrs = ceil(N/G)) for ALL
member columns, exactly like the HIP engine, and exchanges only what the HIP
host code exchanges:
  leave / join          the leavers' / introducer's rows from their owners
                        (slice sums: every other rank adds 0)
  guard                 all_reduce(sum) of the owned rows' present counts +
                        |D| (rank 0), then of the post-REMOVE counts of the
                        undecided rows (owners)
  pull                  the sender's owner validates each draw against the
                        sender's row (k_peers_rows); all_reduce(sum) of the
                        N*k flags, then every rank builds every inbox
  ring                  the sender's owner finds its 3 targets in its list
                        (slave/slave.go:515-524); all_reduce(max) of the 3N
                        targets, then every rank builds every inbox
  ghost rows            from the replicated inboxes every rank derives the
                        same want lists; each owner sends the requested rows
                        as they stand before the round (the alltoallv, here
                        pairwise send / recv: gloo has no alltoall); the
                        receiver derives the sender's snapshot itself (REMOVE
                        of D_{r-1} at the sender, the sender's own hb + 1, its
                        detections excluded: SPEC §2 A.3's single-pass form)
  D_r                   all_reduce(sum) of the detection counts per column,
                        all_reduce(max) of the negated first detectors
  read-outs             the failed set is replicated; all_reduce(max) of
                        det_any, all_reduce(sum) of the counters
Comparing every rank's rows with the full oracle/tablesim state each round
shows the row decomposition and its exchange set are complete.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.distributed as dist

from oracle import philox

ABSENT, TOMB = -1, -2
NOSH = -(1 << 40)
BIG = np.iinfo(np.int64).max


def _allreduce(x, op=dist.ReduceOp.SUM):
    t = torch.from_numpy(np.ascontiguousarray(x, dtype=np.int64))
    dist.all_reduce(t, op=op)
    return t.numpy()


class RowModel:
    def __init__(self, n, fanout=3, peer_mode=0, seed=1, t_fail=5, t_cleanup=5, min_members=4, introducer=0):
        self.rank, self.world = dist.get_rank(), dist.get_world_size()
        self.n, self.k, self.pm, self.seed = n, fanout, peer_mode, seed
        self.t_fail, self.t_cleanup, self.minm, self.I = t_fail, t_cleanup, min_members, introducer
        self.nrs = -(-n // self.world)
        self.row0 = min(self.rank * self.nrs, n)
        self.nrows = min(self.nrs, n - self.row0)
        self.hb = np.full((self.nrows, n), ABSENT, np.int64)
        self.ts = np.zeros((self.nrows, n), np.int64)
        self.alive = np.zeros(n, bool)
        self.dcnt = np.zeros(n, np.int64)  # D_{r-1}: detectors per column (replicated)
        self.dmin = np.full(n, BIG, np.int64)
        self.det_any = np.zeros(n, bool)
        self.round = 0
        self.pending = []
        self.ghost_rows_in = 0
        # SPEC D7: the ts of the introducer's RecentFailList entry beside its
        # present member c (a join of a tombstoned member), NOSH where none;
        # meaningful on the owner of row I
        self.shadow = np.full(n, NOSH, np.int64)

    def owner(self, i):
        return i // self.nrs

    def owned(self, i):
        return self.row0 <= i < self.row0 + self.nrows

    # ---- state -------------------------------------------------------------
    def import_full(self, hb, ts, alive, round_):
        sl = slice(self.row0, self.row0 + self.nrows)
        self.hb = np.array(hb, np.int64)[sl].copy()
        self.ts = np.array(ts, np.int64)[sl].copy()
        self.alive = np.array(alive, bool)
        self.round = round_
        self.dcnt[:] = 0
        self.dmin[:] = BIG
        self.shadow[:] = NOSH

    def apply_events(self, ev):
        self.pending.extend(ev)

    def _rows(self, rows, what="hb"):
        """the full rows `rows` from their owners (slice sums, like k_rowbits
        into slice 0 + allreduce)"""
        out = np.zeros((len(rows), self.n), np.int64)
        for q, i in enumerate(rows):
            if self.owned(i):
                src = self.hb if what == "hb" else self.ts
                out[q] = src[i - self.row0] - (ABSENT if what == "hb" else 0)  # absent -> 0 for the sum
        out = _allreduce(out)
        return out + ABSENT if what == "hb" else out

    def _remove(self, j, c, st):  # removeMember, slave/slave.go:276-286
        x = self.hb[j - self.row0, c]
        if x >= 0 and j == self.I and self.shadow[c] != NOSH:  # D7: the RecentFailList entry stays
            self.hb[j - self.row0, c] = TOMB
            self.ts[j - self.row0, c] = self.shadow[c]
            self.shadow[c] = NOSH
        elif x >= 0:
            self.hb[j - self.row0, c] = TOMB
            st["tombstoned"] += 1
        elif x == ABSENT:
            st["remove_unknown"] += 1

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
            lists = self._rows(leavers) >= 0  # each leaver's list (slave/slave.go:316-319)
            for q, c in enumerate(leavers):
                for j in range(self.row0, self.row0 + self.nrows):
                    if j != c and self.alive[j] and lists[q, j]:
                        self._remove(j, c, st)
        joiners = [c for kind, c in ev if kind == 1]
        for c in joiners:
            if not self.alive[c]:
                if self.owned(c):
                    self.hb[c - self.row0, :] = ABSENT
                    self.ts[c - self.row0, :] = 0
                if c == self.I:
                    self.shadow[:] = NOSH
                self.alive[c] = True
        I = self.I
        if joiners and self.alive[I]:
            added = 0
            if self.owned(I):
                for c in joiners:
                    if self.hb[I - self.row0, c] < 0:
                        if self.hb[I - self.row0, c] == TOMB:  # D7: its tombstone stays beside it
                            self.shadow[c] = self.ts[I - self.row0, c]
                        self.hb[I - self.row0, c] = 0
                        self.ts[I - self.row0, c] = r
                        added += 1
            added = int(_allreduce(np.array([added]))[0])
            msg = self._rows([I])[0]  # the introducer's row, shipped to every shard
            if added:
                for j in range(self.row0, self.row0 + self.nrows):
                    if j == I or not self.alive[j] or msg[j] < 0:
                        continue
                    row = self.hb[j - self.row0]
                    upd = (msg >= 0) & (row >= ABSENT) & (msg > row)
                    row[upd] = msg[upd]
                    self.ts[j - self.row0, upd] = r
                    st["merged_cells"] += int(upd.sum())

    def _removes_at(self, j):
        """bool[n]: REMOVE of each column of D_{r-1} is delivered at row j"""
        return (self.dcnt > 0) & ~((self.dcnt == 1) & (self.dmin == j))

    def _decide_active(self):
        cntl = np.zeros(self.n + 1, np.int64)
        cntl[self.row0:self.row0 + self.nrows] = (self.hb >= 0).sum(axis=1)
        if self.rank == 0:
            cntl[self.n] = int((self.dcnt > 0).sum())
        g = _allreduce(cntl)
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
                if self.owned(i):
                    post[i] = int(((self.hb[i - self.row0] >= 0) & ~self._removes_at(i)).sum())
        post = _allreduce(post)
        active[und] = post[und] >= self.minm
        return active

    def _snapshot_raw(self, s, hb, ts, active, r):
        """the snapshot sender s sends this round, from its row as it stood
        before the round (a ghost): REMOVE'd and detected members dropped, its
        own heartbeat + 1"""
        x = hb.copy()
        x[(x >= 0) & self._removes_at(s)] = TOMB
        if x[s] >= 0:
            x[s] += 1
        cand = (np.arange(self.n) != s) & (x > 1) & (ts < r - self.t_fail)
        x[cand] = TOMB
        return np.where(x >= 0, x, -1)

    def step(self):
        r = self.round + 1
        st = dict(rounds=1, last_round=r, detections=0, failed_members=0, remove_unknown=0, ring_empty=0,
                  active_rows=0, merged_cells=0, released=0, tombstoned=0)
        self._events(r, st)
        active = self._decide_active()
        if self.rank == 0:
            st["active_rows"] = int(active.sum())
        pre_hb, pre_ts = self.hb.copy(), self.ts.copy()  # what the ghosts carry
        # steps 1-5 on the owned rows
        self.det_any[:] = False
        ndcnt = np.zeros(self.n, np.int64)
        ndmin = np.full(self.n, BIG, np.int64)
        cols = np.arange(self.n)
        for i in range(self.row0, self.row0 + self.nrows):
            if not self.alive[i]:
                continue
            row, tsr = self.hb[i - self.row0], self.ts[i - self.row0]
            rm = self._removes_at(i)
            sh = (self.shadow != NOSH) if i == self.I else np.zeros(self.n, bool)
            dual = rm & (row >= 0) & sh  # D7: the RecentFailList entry (and its ts) stays
            tsr[dual] = self.shadow[dual]
            self.shadow[dual] = NOSH
            sh &= ~dual
            st["tombstoned"] += int((rm & (row >= 0) & ~dual).sum())
            st["remove_unknown"] += int((rm & (row == ABSENT)).sum())
            row[rm & (row >= 0)] = TOMB
            if not active[i]:
                tsr[row >= 0] = r
                continue
            if row[i] >= 0:
                row[i] += 1
                tsr[i] = r
            det = (cols != i) & (row > 1) & (tsr < r - self.t_fail)
            if det.any():
                row[det] = TOMB
                dd = det & sh
                tsr[dd] = self.shadow[dd]
                self.shadow[dd] = NOSH
                sh &= ~dd
                st["detections"] += int(det.sum())
                ndcnt[det] += 1
                ndmin[det] = np.minimum(ndmin[det], i)
                self.det_any[i] = True
            rel = (row == TOMB) & (tsr < r - self.t_cleanup)
            row[rel] = ABSENT
            st["released"] += int(rel.sum())
            old = sh & (self.shadow < r - self.t_cleanup)
            self.shadow[old] = NOSH
            st["released"] += int(old.sum())
        snap_own = {i: np.where(self.hb[i - self.row0] >= 0, self.hb[i - self.row0], -1)
                    for i in range(self.row0, self.row0 + self.nrows)}
        inbox = self._inbox_pull(pre_hb, pre_ts, active, r) if self.pm == 0 else \
            self._inbox_ring(snap_own, active, st)
        ghosts = self._ghost_exchange(inbox, pre_hb, pre_ts)
        for i in range(self.row0, self.row0 + self.nrows):
            if not self.alive[i] or not inbox[i]:
                continue
            m = np.full(self.n, -1, np.int64)
            for s in set(inbox[i]):
                sn = snap_own[s] if self.owned(s) else self._snapshot_raw(s, *ghosts[s], active, r)
                m = np.maximum(m, sn)
            row = self.hb[i - self.row0]
            upd = (row >= ABSENT) & (m > row)
            row[upd] = m[upd]
            self.ts[i - self.row0, upd] = r
            st["merged_cells"] += int(upd.sum())
        # D_r: counts summed, first detectors MIN (as the MAX of negations)
        self.dcnt = _allreduce(ndcnt)
        neg = _allreduce(np.where(ndmin == BIG, -BIG, -ndmin), dist.ReduceOp.MAX)
        self.dmin = np.where(neg == -BIG, BIG, -neg)
        if self.rank == 0:
            st["failed_members"] = int((self.dcnt > 0).sum())
        keys = sorted(st)
        tot = _allreduce(np.array([st[k] for k in keys]))
        out = dict(zip(keys, (int(x) for x in tot)))
        out["rounds"], out["last_round"] = 1, r
        self.round = r
        return out

    def _inbox_pull(self, pre_hb, pre_ts, active, r):
        """k_peers_rows: the owner of each drawn sender checks the receiver's
        cell in the sender's row; the N*k flags are summed over the shards."""
        pvf = np.zeros((self.n, self.k), np.int64)
        for i in range(self.n):
            if not self.alive[i] or self.n < 2:
                continue
            for q in range(self.k):
                s = philox.peer(self.seed, i, r, q, self.n)
                if not (self.owned(s) and self.alive[s] and active[s]):
                    continue
                x, t = pre_hb[s - self.row0, i], pre_ts[s - self.row0, i]
                flagged = i != s and x > 1 and t < r - self.t_fail
                removed = self.dcnt[i] > 0 and not (self.dcnt[i] == 1 and self.dmin[i] == s)
                pvf[i, q] = int(x >= 0 and not flagged and not removed)
        pvf = _allreduce(pvf)
        return [[philox.peer(self.seed, i, r, q, self.n) for q in range(self.k) if pvf[i, q]] for i in range(self.n)]

    def _inbox_ring(self, snap_own, active, st):
        """The owner of each sender finds its targets list[(idx-1) mod L],
        list[(idx+1) mod L], list[(idx+2) mod L] in its snapshot list
        (slave/slave.go:515-524); all_reduce(max) of the 3N targets."""
        tg = np.full((self.n, 3), -1, np.int64)
        for s in range(self.row0, self.row0 + self.nrows):
            if not (self.alive[s] and active[s]):
                continue
            lst = np.flatnonzero(snap_own[s] >= 0)
            L = len(lst)
            if L == 0:
                st["ring_empty"] += 1
                continue
            hit = np.flatnonzero(lst == s)
            idx = int(hit[0]) if len(hit) else -1
            for q, w in enumerate((idx - 1, idx + 1, idx + 2)):
                v = int(np.fmod(w, L))
                tg[s, q] = lst[v + L if v < 0 else v]
        tg = _allreduce(tg, dist.ReduceOp.MAX)
        inbox = [[] for _ in range(self.n)]
        for s in range(self.n):
            for t in tg[s]:
                if t >= 0 and self.alive[t]:
                    inbox[t].append(s)
        return inbox

    def _ghost_exchange(self, inbox, pre_hb, pre_ts):
        """want lists from the replicated inboxes; each owner sends the rows
        others want (pairwise send / recv in rank order)."""
        want = [sorted({s for i in range(g * self.nrs, min((g + 1) * self.nrs, self.n)) for s in inbox[i]
                        if self.owner(s) != g}) for g in range(self.world)]
        got = {}
        for a in range(self.world):
            for b in range(self.world):
                if a == b:
                    continue
                rows = [s for s in want[b] if self.owner(s) == a]  # a sends these to b
                if not rows:
                    continue
                if self.rank == a:
                    idx = np.array(rows) - self.row0
                    dist.send(torch.from_numpy(np.ascontiguousarray(pre_hb[idx])), dst=b)
                    dist.send(torch.from_numpy(np.ascontiguousarray(pre_ts[idx])), dst=b)
                elif self.rank == b:
                    h = torch.zeros((len(rows), self.n), dtype=torch.int64)
                    t = torch.zeros((len(rows), self.n), dtype=torch.int64)
                    dist.recv(h, src=a)
                    dist.recv(t, src=a)
                    for q, s in enumerate(rows):
                        got[s] = (h[q].numpy(), t[q].numpy())
        self.ghost_rows_in = len(got)
        return got

    # ---- read-outs (collective) -------------------------------------------
    def read_failed(self):
        return [c for c in range(self.n) if self.dcnt[c] > 0]

    def read_detectors(self):
        anyd = _allreduce(self.det_any.astype(np.int64), dist.ReduceOp.MAX)
        return [i for i in range(self.n) if anyd[i]]


def worker(rank, world, port, n, rounds, cfg, churn_seed):
    """One gloo rank: replay a churn scenario on the model and check this
    rank's rows, the counters and the read-outs against the full oracle every
    round."""
    import os
    import sys
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import scenarios as sc
        from oracle import oracle as om
        ocfg = om.default_config(n, peer_mode=cfg["peer_mode"], fanout=cfg["fanout"], seed=cfg["seed"],
                                 t_fail=cfg["t_fail"], t_cleanup=cfg["t_cleanup"])
        orc = om.Oracle(ocfg)
        m = RowModel(n, fanout=cfg["fanout"], peer_mode=cfg["peer_mode"], seed=cfg["seed"],
                     t_fail=cfg["t_fail"], t_cleanup=cfg["t_cleanup"])
        init = sc.full_state(n)
        orc.import_state(*init, 0)
        m.import_full(*init, 0)
        sched = sc.random_churn(n, rounds, churn_seed, p_crash=0.05, p_leave=0.03, p_join=0.08)
        sl = slice(m.row0, m.row0 + m.nrows)
        ghosts = 0
        for r in range(1, rounds + 1):
            ev = sched.get(r, [])
            orc.apply_events(ev)
            m.apply_events(ev)
            s_cpu, s_mod = orc.step(1), m.step()
            assert s_cpu == s_mod, f"rank {rank} round {r}: oracle {s_cpu} != model {s_mod}"
            hb, ts, alive = orc.export_state()
            assert np.array_equal(hb[sl], m.hb), f"rank {rank} round {r}: hb rows differ"
            mts = sc.export_view(m.hb, m.ts, r, cfg["t_cleanup"])[1]
            assert np.array_equal(ts[sl], mts), f"rank {rank} round {r}: ts rows differ"
            assert np.array_equal(alive.astype(bool), m.alive)
            bm = orc.read_failed()
            assert m.read_failed() == [c for c in range(n) if bm[c >> 5] >> (c & 31) & 1]
            assert m.read_detectors() == list(orc.read_detectors())
            ghosts += m.ghost_rows_in
        assert world == 1 or ghosts > 0, "no ghost row ever crossed shards"
        sys.stdout.flush()
    finally:
        dist.destroy_process_group()
