"""ORACLE / TEST INFRASTRUCTURE ONLY.

listsim — a literal, list-based replay of the reference's membership code for
small clusters (pure Python, O(N^3) per round). Each method follows the Go
function it names line by line, on `Member` objects held in Python lists, with
member addresses as ints. Go slice semantics are emulated where they change
behaviour: `detectfailure` ranges over the slice that `removeMember` shifts in
place (slave/slave.go:464-477 with :283), which yields quirk-mode detection.

The network is replaced by the synchronous delivery schedule of SPEC.md §2
(gossip delivered in the round it is sent, REMOVEs at the start of the next
round). Its purpose: cross-check oracle/tablesim.c (dense table semantics)
and pin the hand-derived KATs of SURVEY.md App. B (tests/golden/).
"""
from __future__ import annotations

from dataclasses import dataclass

from . import philox

T_FAIL = 5      # PERIOD = 5e9 ns / HEARTBEAT_PERIOD 1e9 ns (slave/slave.go:24,27)
T_CLEANUP = 5   # COOLDOWN (slave/slave.go:25)
MIN_NODES = 4   # literal 4 at slave/slave.go:504,511


@dataclass
class Member:  # master/master.go:16-20
    addr: int
    hb: int
    ts: int


class Panic(Exception):
    pass


def get_index(addr, lst):  # slave/slave.go:405-412
    for i, m in enumerate(lst):
        if m.addr == addr:
            return i
    return -1


def is_member_exist(m, lst):  # slave/slave.go:387-394
    return any(m.addr == x.addr for x in lst)


class Node:
    """One SDFS process's membership state (slave/slave.go:59-72)."""

    def __init__(self, addr, order="id"):
        self.addr = addr
        self.alive = False
        self.sent: dict[int, set[int]] = {}   # the last sweep's REMOVE recipients per member
        self.members: list[Member] = []      # MemberList
        self.recent_fail: list[Member] = []  # RecentFailList
        self.order = order
        self.stats = None

    # ---- list helpers ---------------------------------------------------
    def _append(self, m: Member):
        if self.order == "append":
            self.members.append(m)  # slave/slave.go:255, 437
        else:  # SPEC D1: member-ID order
            k = 0
            while k < len(self.members) and self.members[k].addr < m.addr:
                k += 1
            self.members.insert(k, m)

    def remove_member(self, addr):  # slave/slave.go:276-286
        remove_index = get_index(addr, self.members)
        index = get_index(addr, self.recent_fail)
        if index == -1:
            if remove_index == -1:
                # self.MemberList[-1] -> Go index-out-of-range panic (:280)
                self.stats["remove_unknown"] += 1
                return
            self.recent_fail.append(self.members[remove_index])
            return_tomb = True
        else:
            return_tomb = False
        if remove_index != -1:
            del self.members[remove_index]  # append(s[:i], s[i+1:]...) (:283)
        return return_tomb

    def merge(self, s, now):  # MergeMemberList, slave/slave.go:414-440
        changed = set()
        if len(s) == 0:
            return changed
        for local in self.members:
            if not is_member_exist(local, s):
                continue
            idx = get_index(local.addr, s)
            if local.hb < s[idx].hb:
                local.hb = s[idx].hb
                local.ts = now
                changed.add(local.addr)
        for remote in s:
            judge2 = is_member_exist(remote, self.members)
            judge3 = is_member_exist(remote, self.recent_fail)
            if judge2:
                continue
            if not judge2 and not judge3:
                self._append(Member(remote.addr, remote.hb, now))
                changed.add(remote.addr)
        return changed

    def update_member_list(self, now, quirk):  # slave/slave.go:442-458
        for m in self.members:
            if m.addr == self.addr:
                m.ts = now
                m.hb += 1
        detected = self.detect_failure(now, quirk)
        self.clean_fail_list(now)
        return detected  # revote_master (:452-457) is out of scope

    def _remove_msg(self, c, live):
        # Remove (slave/slave.go:338-363): REMOVE c to every member of the
        # list as it stands when the call is made (after removeMember(c) and
        # the removals before it in the sweep), self excluded (:344-346)
        self.sent.setdefault(c, set()).update(m.addr for m in live if m.addr != self.addr)

    def detect_failure(self, now, quirk):  # slave/slave.go:460-482
        current = now
        detected = []
        self.sent = {}  # c -> recipients of this sweep's REMOVE(c) messages
        if not quirk:
            # canonical: every candidate of the list is detected
            cands = [m for m in self.members
                     if m.addr != self.addr and m.hb > 1 and m.ts < current - T_FAIL]
            for m in cands:
                self.remove_member(m.addr)
                detected.append(m.addr)
                self._remove_msg(m.addr, self.members)
            return detected
        # literal Go: `for _, member := range self.MemberList` captures the
        # header (array, len); removeMember shifts the same array in place.
        backing = list(self.members)
        length = len(backing)
        for j in range(len(backing)):
            member = backing[j]
            if member.addr == self.addr:
                continue
            if member.hb <= 1:
                continue
            if member.hb > 1 and member.ts < current - T_FAIL:
                # removeMember on the live slice backing[:length]
                live = backing[:length]
                ri = get_index(member.addr, live)
                ti = get_index(member.addr, self.recent_fail)
                panicked = False
                if ti == -1:
                    if ri == -1:
                        self.stats["remove_unknown"] += 1
                        panicked = True  # :280 panics before Remove is reached
                    else:
                        self.recent_fail.append(live[ri])
                if ri != -1:
                    for q in range(ri, length - 1):
                        backing[q] = backing[q + 1]
                    length -= 1  # backing[length] keeps the stale last entry
                    detected.append(member.addr)
                # self.Remove(member.Address), sent again on a stale re-read
                if not panicked:
                    self._remove_msg(member.addr, backing[:length])
        self.members = backing[:length]
        return detected

    def clean_fail_list(self, now):  # slave/slave.go:484-497
        if len(self.recent_fail) < 1:
            return
        current = now
        i = 0
        while i < len(self.recent_fail):
            if self.recent_fail[i].ts < current - T_CLEANUP:
                del self.recent_fail[i]
                self.stats["released"] += 1
            else:
                i += 1

    def snapshot(self):  # encode (slave/slave.go:365-373), hb only is used
        return [Member(m.addr, m.hb, m.ts) for m in self.members]


class ListSim:
    """N nodes run in synchronous rounds (SPEC.md §2) with reference logic."""

    def __init__(self, n, seed=0x5EED0001, peer_mode="ring", fanout=3, quirk=False,
                 order="id", introducer=0, master=0, replicas=4, population=None, remove="all"):
        self.n = n
        self.nodes = [Node(a, order) for a in range(n)]
        self.seed = seed
        self.peer_mode = peer_mode
        self.k = fanout
        self.quirk = quirk
        self.introducer = introducer
        self.master = master
        self.R = replicas
        # REMOVE recipients: "list" = the reference's (every member of the
        # detector's list when Remove runs, slave/slave.go:344, 472-473);
        # "all" = SPEC D4 (every alive row but a sole detector)
        assert remove in ("all", "list")
        self.remove = remove
        self.round = 0
        self.pending_remove: dict[int, list[int]] = {}  # c -> detectors (D_{r-1})
        self.pending_recv: dict[int, set[int]] = {}     # c -> recipients of REMOVE(c) ("list")
        self.events: list[tuple[int, int]] = []
        self.files: dict[int, dict] = {}  # File_matadata (master/master.go:23)
        self.draws: dict[int, int] = {}
        self.last_detectors: list[int] = []
        self.last_failed: list[int] = []
        self._zero()

    def _zero(self):
        self.stats = dict(rounds=0, last_round=0, detections=0, failed_members=0, remove_unknown=0,
                          ring_empty=0, active_rows=0, merged_cells=0, released=0, tombstoned=0)
        for nd in self.nodes:
            nd.stats = self.stats

    # ---- events (SPEC §5) -------------------------------------------------
    def apply_events(self, events):
        self.events.extend(events)

    def _remove_at(self, j, c):
        nd = self.nodes[j]
        if nd.remove_member(c):
            self.stats["tombstoned"] += 1

    def _do_events(self, now):
        ev, self.events = self.events, []
        for kind, c in ev:
            if kind == 3:
                self.nodes[c].alive = False
        leavers = []
        for kind, c in ev:
            if kind == 2 and self.nodes[c].alive:
                self.nodes[c].alive = False
                leavers.append(c)
        for c in leavers:  # Leave (slave/slave.go:310-336)
            for m in list(self.nodes[c].members):
                if m.addr == c:
                    continue
                if self.nodes[m.addr].alive:
                    self._remove_at(m.addr, c)  # LEAVE handler (:232-235)
        joiners = [c for kind, c in ev if kind == 1]
        for c in joiners:
            nd = self.nodes[c]
            if not nd.alive:
                nd.members, nd.recent_fail = [], []
                nd.alive = True
        I = self.nodes[self.introducer]
        if joiners and I.alive:
            added = 0
            for c in joiners:
                if get_index(c, I.members) == -1:  # MemberInList reads MemberList only (:198-205)
                    # SPEC D7: a joiner the introducer holds tombstoned is
                    # appended and keeps its RecentFailList entry too
                    I._append(Member(c, 0, now))  # addNewMember (:250-255)
                    added += 1
            if added:
                msg = I.snapshot()
                for m in msg:  # send to every member, self and joiner included (:257-272)
                    rcv = self.nodes[m.addr]
                    if rcv.alive:
                        self.stats["merged_cells"] += len(rcv.merge(msg, now))

    # ---- one synchronous round --------------------------------------------
    def step(self, rounds=1):
        self._zero()
        for _ in range(rounds):
            self._one_round()
        return dict(self.stats)

    def _one_round(self):
        r = self.round + 1
        nodes = self.nodes
        self._do_events(r)
        # step 1: REMOVE delivery of D_{r-1}
        for c, dets in sorted(self.pending_remove.items()):
            for j, nd in enumerate(nodes):
                if not nd.alive:
                    continue
                if self.remove == "list":
                    if j not in self.pending_recv.get(c, ()):
                        continue  # no detector had j in its list (:344)
                elif dets == [j]:
                    continue  # the sole detector does not message itself (:344-346)
                self._remove_at(j, c)
        # steps 2-5 per node (HeartBeat, slave/slave.go:499-511)
        active = [False] * self.n
        detected_by: dict[int, list[int]] = {}
        recv: dict[int, set[int]] = {}
        self.last_detectors = []
        for i, nd in enumerate(nodes):
            if not nd.alive:
                continue
            if len(nd.members) < MIN_NODES:
                for m in nd.members:
                    m.ts = r  # :505-507
                continue
            active[i] = True
            self.stats["active_rows"] += 1
            det = nd.update_member_list(r, self.quirk)
            self.stats["detections"] += len(det)
            for c in det:
                detected_by.setdefault(c, []).append(i)
            for c, to in nd.sent.items():
                recv.setdefault(c, set()).update(to)
            if det:
                self.last_detectors.append(i)
        snaps = {i: nodes[i].snapshot() for i in range(self.n) if active[i]}
        inbox: dict[int, list[int]] = {}
        if self.peer_mode == "ring":
            for s, snap in snaps.items():  # slave/slave.go:515-542
                L = len(snap)
                if L == 0:
                    self.stats["ring_empty"] += 1
                    continue
                self_index = get_index(s, snap)
                neigh = [(self_index - 1), (self_index + 1), (self_index + 2)]
                neigh = [int(_go_mod(v, L)) for v in neigh]
                for v in neigh:
                    tgt = snap[v].addr
                    if nodes[tgt].alive:
                        inbox.setdefault(tgt, []).append(s)
        else:
            for i, nd in enumerate(nodes):
                if not nd.alive:
                    continue
                for t in range(self.k):
                    p = philox.peer(self.seed, i, r, t, self.n)
                    if p in snaps and get_index(i, snaps[p]) != -1:
                        inbox.setdefault(i, []).append(p)
        for i in sorted(inbox):
            changed = set()
            for s in sorted(set(inbox[i])):
                changed |= nodes[i].merge(snaps[s], r)
            self.stats["merged_cells"] += len(changed)
        self.pending_remove = detected_by
        self.pending_recv = recv
        self.last_failed = sorted(detected_by)
        self.stats["failed_members"] += len(detected_by)
        self.round = r
        self.stats["rounds"] += 1
        self.stats["last_round"] = r

    # ---- dense views ------------------------------------------------------
    @classmethod
    def from_dense(cls, hb, ts, alive, round_, **kw):
        sim = cls(len(alive), **kw)
        sim.round = round_
        for i, nd in enumerate(sim.nodes):
            nd.alive = bool(alive[i])
            for c in range(sim.n):  # ID order
                if hb[i][c] >= 0:
                    nd.members.append(Member(c, int(hb[i][c]), int(ts[i][c])))
                elif hb[i][c] == -2:
                    nd.recent_fail.append(Member(c, -2, int(ts[i][c])))
        return sim

    def dense(self):
        import numpy as np
        hb = np.full((self.n, self.n), -1, np.int32)
        ts = np.zeros((self.n, self.n), np.int32)
        alive = np.zeros(self.n, np.uint8)
        for i, nd in enumerate(self.nodes):
            alive[i] = nd.alive
            for m in nd.recent_fail:
                hb[i, m.addr] = -2
                ts[i, m.addr] = m.ts
            for m in nd.members:
                hb[i, m.addr] = m.hb
                ts[i, m.addr] = m.ts
        return hb, ts, alive

    # ---- placement (master/master.go) -------------------------------------
    def _member_list(self):  # Update_member aliasing (master/master.go:46)
        return [m.addr for m in self.nodes[self.master].members]

    def _init_replica(self, f, cand):  # master/master.go:129-150
        info = self.files[f]
        need = self.R - len(info["nodes"])
        if need <= 0:
            return 0
        M = len(cand)
        if M <= 1:
            return -5  # Intn(<=0) panics
        pool = set(cand[:-1]) - set(info["nodes"])
        if len(pool) < need:
            return -5  # infinite loop
        d = self.draws.get(f, 0)
        nodes = list(info["nodes"])
        budget = 1 << 20
        while len(nodes) < self.R:
            if budget == 0:
                return -5
            budget -= 1
            num = philox.place_index(self.seed, f, d, M)
            d += 1
            a = cand[num]
            if a not in nodes:
                nodes.append(a)
        self.draws[f] = d
        info["nodes"] = nodes
        return 0

    def put(self, f):  # Handle_put_request (master/master.go:152-175)
        if f not in self.files:
            self.files[f] = {"nodes": [], "version": 0, "ts": self.round}
        self.files[f]["ts"] = self.round
        st = self._init_replica(f, self._member_list())
        if st == 0:
            self.files[f]["version"] += 1
        info = self.files[f]
        return list(info["nodes"]), info["version"], st

    def repair(self, observer):  # Update_metadata (master/master.go:74-127)
        available = []
        for m in self.nodes[observer].members:
            if m.addr not in available:
                available.append(m.addr)
        cand = self._member_list()
        plan = []
        for f in sorted(self.files):
            info = self.files[f]
            working = [x for x in info["nodes"] if x in available]
            if len(working) < self.R:
                ver = info["version"]
                info["nodes"] = list(working)
                st = self._init_replica(f, cand)
                new = [x for x in info["nodes"] if x not in working]
                plan.append((f, working[0] if working else -1, ver, st, tuple(new)))
        if self.quirk and len(plan) > 1:
            plan = plan[-1:]  # the plan map is re-made per file (master/master.go:118)
        return plan

    def get(self, f):
        if f not in self.files:
            return [], -1
        return list(self.files[f]["nodes"]), self.files[f]["version"]

    def delete(self, f):
        info = self.files.pop(f, None)
        return list(info["nodes"]) if info else []


def _go_mod(a, n):
    """Go's % truncates toward zero; negative results are then +n (:520-523)."""
    r = abs(a) % n
    r = -r if a < 0 else r
    return r + n if r < 0 else r
