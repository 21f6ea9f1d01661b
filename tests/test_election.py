"""Master re-election oracle (oracle/election.py, SPEC §9) against cases
derived by hand from slave/slave.go:930-1043. CPU only."""
import numpy as np

from oracle import election as el


def test_vote_scan_kat():
    # rows: 0 = master's own row; row 1 lost the master (tombstone), row 2 has
    # nobody, row 3 keeps the master; rows list members in ID order (SPEC D1)
    hb = np.array([[3, 2, -1, 1],
                   [-2, 4, 1, -1],
                   [-1, -1, -1, -1],
                   [1, -2, -1, 2]], np.int32)
    first, ln, has = el.vote_scan(hb, np.zeros(4, np.int32))
    assert first.tolist() == [0, 1, -1, 0]
    assert ln.tolist() == [3, 2, 0, 2]
    assert has.tolist() == [1, 0, 0, 1]


def test_tally_majority_on_remote_votes():
    """N=6, master 0 crashed and gone from every list: rows 1..5 hold
    [1..5] (len 5). Row 1 votes for itself (counted, no check, :936-939);
    rows 2, 3 vote remotely: after row 3, Vote_num = 3 > 5 // 2 -> elected
    (:978). Rows 4, 5 still count but 1 is already master."""
    n = 6
    t = el.Tally(n, master=0)
    alive = np.array([0, 1, 1, 1, 1, 1], np.uint8)
    first = np.array([-1, 1, 1, 1, 1, 1], np.int32)
    ln = np.array([0, 5, 5, 5, 5, 5], np.int32)
    has = np.zeros(n, np.uint8)
    assert t.round(alive, first, ln, has) == [1]
    assert t.num[1] == 5 and t.voters[1] == {2, 3, 4, 5} and t.mview[1] == 1
    # next round: the same voters re-vote (their master is still 0): the
    # voter map dedups them, the self vote adds again, nobody new is elected
    assert t.round(alive, first, ln, has) == []
    assert t.num[1] == 6
    t.finish_rebuild(1, 1)  # M is its own MemberList[0]
    assert not t.on[1] and t.voters[1] == set()
    # voters still think 0 is master and keep voting; 1 is master -> no re-election
    assert t.round(alive, first, ln, has) == [] and t.num[1] == 5


def test_tally_no_majority_small_lists_and_gate():
    """Rows with fewer than 4 members do not run updateMemberList (:504);
    self votes alone never elect (no check on the self path)."""
    n = 5
    t = el.Tally(n, master=4)
    alive = np.ones(n, np.uint8)
    first = np.array([0, 0, 0, 0, 0], np.int32)
    ln = np.array([4, 3, 3, 3, 4], np.int32)
    has = np.array([0, 0, 0, 0, 1], np.uint8)
    assert t.round(alive, first, ln, has) == []
    assert t.num[0] == 1 and t.mview[0] == 4


def test_tally_fatal_vote_to_dead_member():
    t = el.Tally(5, master=0)
    alive = np.array([0, 1, 1, 1, 1], np.uint8)
    first = np.array([-1, 1, 1, 1, 1], np.int32)
    ln = np.full(5, 4, np.int32)
    assert t.round(alive, first, ln, np.zeros(5, np.uint8), dead={1}) == []
    assert t.fatal == [2, 3, 4]


def test_rebuild_kat():
    """M = 2 with list [1, 2, 3, 4, 5]: f0 = 1 answers every remote store
    query (:994). R = 4.
      a: on 1,3,4 -> f0 has it, M not: every member but M -> [1, 3, 4, 5]
      b: on 2,5,6,7 -> only M's own store -> [2]
      c: on 1,2,6,7 -> both -> [1, 2, 3, 4]
      d: on 6,7,8 -> in neither store read -> dropped
      e: absent -> stays absent"""
    rep = np.array([[1, 3, 4, -1], [2, 5, 6, 7], [1, 2, 6, 7], [6, 7, 8, -1], [-1, -1, -1, -1]], np.int32)
    ver = np.array([3, 1, 2, 5, -1], np.int32)
    fts = np.array([10, 11, 12, 13, 0], np.int32)
    r2, v2, t2 = el.rebuild(rep, ver, fts, 2, [1, 2, 3, 4, 5], now=40)
    assert r2.tolist() == [[1, 3, 4, 5], [2, -1, -1, -1], [1, 2, 3, 4], [-1] * 4, [-1] * 4]
    assert v2.tolist() == [3, 1, 2, -1, -1]
    assert t2.tolist() == [40, 40, 40, 13, 0]
    # M its own MemberList[0]: every member of the list reports M's store
    r3, v3, _ = el.rebuild(rep, ver, fts, 1, [1, 2, 3], now=40)
    assert r3.tolist() == [[1, 2, 3, -1], [-1] * 4, [1, 2, 3, -1], [-1] * 4, [-1] * 4]
    assert v3.tolist() == [3, -1, 2, -1, -1]


class _NoEngine:
    """Stands in for the engine in Cluster._tally (only crash events reach it)."""

    def __init__(self):
        self.events = []

    def apply_events(self, ev):
        self.events.extend(ev)


def test_cluster_tally_matches_oracle_loop():
    """gossipsim.Cluster._tally (array form) against the oracle's voter-by-
    voter Tally on random vote patterns over many rounds: several
    candidates, self votes before and after remote ones, repeat voters,
    dead targets and chains of log.Fatal, candidates that are voters."""
    import gossipsim as gs
    rng = np.random.default_rng(11)
    for trial in range(40):
        n = int(rng.integers(6, 60))
        cl = object.__new__(gs.Cluster)
        cl.n, cl.engine = n, _NoEngine()
        cl.mview = np.zeros(n, np.int32)
        cl.vote_on = np.zeros(n, bool)
        cl.vote_num = np.zeros(n, np.int64)
        cl.voters = [set() for _ in range(n)]
        cl.rebuilds, cl.elections, cl.fatal = {}, [], []
        cl.dead = set(rng.choice(n, size=int(rng.integers(0, 3)), replace=False).tolist())
        t = el.Tally(n, master=0)
        for r in range(1, 6):
            # voters: running members only (Cluster never lets a gone
            # process vote); every target keeps its own list length, voter
            # or not, so majorities reached by remote votes alone are covered
            dead_before = set(cl.dead)
            gone = np.zeros(n, bool)
            gone[list(dead_before)] = True
            idx = np.flatnonzero((rng.random(n) < 0.7) & ~gone)
            cands = rng.choice(n, size=int(rng.integers(1, 4)), replace=False)
            first = np.where(rng.random(n) < 0.2, np.arange(n), rng.choice(cands, size=n)).astype(np.int32)
            ln_run = rng.integers(0, 2 * n, size=n).astype(np.int32)
            idx = idx[ln_run[idx] >= 4]  # HeartBeat's gate (slave/slave.go:504-511)
            has = np.zeros(n, np.uint8)
            # the oracle loop, with log.Fatal deaths taking effect in voter order
            elected, fatal, dead = [], [], set(dead_before)
            for i in idx.tolist():
                e = t.round(np.eye(1, n, i, dtype=np.uint8)[0], first, ln_run, has, dead=dead)
                elected += e
                if t.fatal:
                    fatal += t.fatal
                    dead |= set(t.fatal)
            n_el = len(cl.elections)
            cl._tally(r, idx, first, ln_run)
            assert [m for _, m in cl.elections[n_el:]] == elected, (trial, r)
            assert [m for rr, m, _ in cl.fatal if rr == r] == fatal, (trial, r)
            np.testing.assert_array_equal(cl.vote_num, t.num)
            np.testing.assert_array_equal(cl.mview, t.mview)
            np.testing.assert_array_equal(cl.vote_on, t.on)
            assert cl.voters == t.voters
            assert cl.dead == dead
