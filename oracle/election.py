"""ORACLE / TEST INFRASTRUCTURE ONLY.

election — a CPU restatement of the reference's master re-election (SURVEY
§8f f3, SPEC.md §9) used as the checker for `gh_vote_scan`, `gh_rebuild_meta`
and gossipsim.Cluster's vote tally. Only tests import it.

  vote_scan   updateMemberList's master check (slave/slave.go:451-457) and
              revote_master's target MemberList[0] (:930-948), on a dense
              external hb table (>= 0 present, -1 absent, -2 tombstone).
  Tally       revote_master (:930-948) + Receive_vote (:968-984) +
              Assign_New_Master (:1045-1051) as plain per-member state.
  rebuild     rebuild_file_meta (:986-1043): builds the reference's
              tmp_file_meta literally (one (member, version) entry per store
              read, the remote reads all going to MemberList[0], :994), then
              sortByValue (:131-143, ascending; ties kept in list order, SPEC
              D10) and the first-4 cut (:1028-1035).

Parity is unpinned against the reference itself (no fixtures, no Go
toolchain); the hand-derived cases in tests/test_election.py pin it.
"""
from __future__ import annotations

import numpy as np


def vote_scan(hb: np.ndarray, mview: np.ndarray):
    """Per row i: MemberList_i[0] (lowest present id, SPEC D1; -1 if empty),
    len(MemberList_i), and whether mview[i] is in the list."""
    pres = hb >= 0
    ln = pres.sum(axis=1).astype(np.int32)
    first = np.where(ln > 0, pres.argmax(axis=1), -1).astype(np.int32)
    has = pres[np.arange(hb.shape[0]), mview].astype(np.uint8)
    return first, ln, has


class Tally:
    """Per-member VoteStatus (slave/slave.go:930-984) and self.master."""

    def __init__(self, n: int, master: int, min_members: int = 4):
        self.mview = np.full(n, master, np.int32)
        self.on = np.zeros(n, bool)
        self.num = np.zeros(n, np.int64)
        self.voters = [set() for _ in range(n)]
        self.min_members = min_members

    def _touch(self, x):  # `if self.VoteStatus.Vote == false {...}` (:931-935, :969-973)
        if not self.on[x]:
            self.on[x] = True
            self.num[x] = 0
            self.voters[x] = set()

    def round(self, alive, first, ln, has, dead=()):
        """One election step on the end-of-round table: every running row
        (alive, list >= min_members: HeartBeat's gate :504-511) whose master is
        not in its list votes, in ID order. A vote to a member whose process is
        gone (`dead`) is rpc.Dial's log.Fatal (:941-944): the voter is listed
        in self.fatal and does not vote. Returns the members elected."""
        elected = []
        self.fatal = []
        for i in np.flatnonzero((alive != 0) & (ln >= self.min_members) & (has == 0)):
            i = int(i)
            t = int(first[i])
            self._touch(i)
            if t == i:  # self vote: counted, no majority check (:936-939)
                self.num[i] += 1
                continue
            if t in dead:
                self.fatal.append(i)
                continue
            # TCPServer.Vote -> Receive_vote(i) at t (:968-984)
            self._touch(t)
            if i not in self.voters[t]:
                self.voters[t].add(i)
                self.num[t] += 1
            if self.mview[t] != t and self.num[t] > ln[t] // 2:
                self.mview[t] = t
                elected.append(t)
        return elected

    def finish_rebuild(self, m, f0):
        """Assign_New_Master at f0 (:1045-1048), then the rebuild's reset (:1039-1041)."""
        self.mview[f0] = m
        self.on[f0] = False
        self.on[m] = False
        self.voters[m] = set()


def rebuild(rep: np.ndarray, ver: np.ndarray, fts: np.ndarray, m: int, lst: list[int], now: int):
    """rebuild_file_meta at new master m with list `lst` (ID order). A
    member's store = the files whose metadata lists it, at the file's version
    (SPEC §9). Returns new (rep, ver, fts); R = rep.shape[1]."""
    nf, R = rep.shape
    store = {}
    for f in range(nf):
        if ver[f] >= 0:
            for x in rep[f]:
                if x >= 0:
                    store.setdefault(int(x), {})[f] = int(ver[f])
    f0 = lst[0]
    tmp: dict[int, list[tuple[int, int]]] = {}
    for member in lst:
        files = store.get(m if member == m else f0, {})
        for f, v in files.items():
            tmp.setdefault(f, []).append((member, v))
    out_rep = np.full_like(rep, -1)
    out_ver = np.full_like(ver, -1)
    out_fts = fts.copy()
    for f, ent in tmp.items():
        sl = sorted(ent, key=lambda e: e[1])  # stable: ties in list order
        nodes = [k for k, _ in sl[:4]][:R]
        out_rep[f, : len(nodes)] = nodes
        out_ver[f] = sl[0][1]
        out_fts[f] = now
    return out_rep, out_ver, out_fts
