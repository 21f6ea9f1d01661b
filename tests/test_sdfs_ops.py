"""SDFS op semantics around placement: the quorum size
(slave/slave.go:717-722), the 60 s write-write window
(master/master.go:214-229) on the oracle, hand-derived from the Go source."""
import numpy as np

import scenarios as sc


def test_quorum_kat7():
    """KAT-7: int(math.Ceil(float64((num+1)/2))) with Go's integer division
    inside the float64(): n = 1..5 -> 1, 1, 2, 2, 3 (the report's 3-of-4 is
    not what the code computes)."""
    from gossipsim import Cluster
    assert [Cluster.quorum(n) for n in range(1, 6)] == [1, 1, 2, 2, 3]
    assert Cluster.quorum(4) == 2


def test_write_window_oracle(oracle_mod):
    """If_file_updated_recent: now - ts < 60 s; strict, so a put 60 rounds
    later is not a conflict; absent files never conflict."""
    n = 12
    o = oracle_mod.Oracle(oracle_mod.default_config(n, max_files=8))
    hb, ts, alive = sc.full_state(n)
    o.import_state(hb, ts, alive, 20)
    assert list(o.put_conflicts([0, 1])) == [0, 0]
    o.put([0])
    assert list(o.put_conflicts([0, 1])) == [1, 0]
    o.step(59)  # round 79: 79 - 20 = 59 < 60
    assert list(o.put_conflicts([0])) == [1]
    o.step(1)   # round 80: 60 is not < 60
    assert list(o.put_conflicts([0])) == [0]
    o.put([0])  # Update_timestamp refreshes the window (:231-238)
    assert list(o.put_conflicts([0])) == [1]
    assert list(o.put_conflicts([0], window=0)) == [0]


def test_get_source_kats():
    """Get's copy source, hand-derived from slave/slave.go:857-878: the first
    response (arrival order) whose local version is <= the master's, or the
    only response; a replica without the file answers Go's zero value 0."""
    from gossipsim import Cluster
    src = Cluster.get_source
    assert src([(4, 3), (7, 2)], 2) == (7, 2)   # 3 > 2 is skipped
    assert src([(4, 2), (7, 2)], 2) == (4, 2)   # the first qualifying response
    assert src([(4, 7)], 5) == (4, 7)           # the only response, even if newer
    assert src([(4, 7), (7, 9)], 5) is None     # nothing qualifies: no copy
    assert src([(4, 0), (7, 5)], 5) == (4, 0)   # an empty replica is picked first
    assert src([], 5) is None
