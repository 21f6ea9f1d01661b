"""The reference's gossip wire format (slave/slave.go:365-385) and the
MergeMemberList of a received list (:414-440) on the CPU oracle against the
literal list replay. Hand-derived expectations from the Go source."""
import numpy as np

import scenarios as sc
import pytest

from gossipsim import codec
from oracle.listsim import ListSim


def test_encode_matches_go_sprint_trim_replace():
    # fmt.Sprint([]string{"a<#INFO#>1<#INFO#>2", "b<#INFO#>3<#INFO#>4"}) = "[a.. b..]"
    e = codec.encode([("10.0.0.1", 5, 100), ("10.0.0.2", 7, 200)])
    assert e == b"10.0.0.1<#INFO#>5<#INFO#>100<#ENTRY#>10.0.0.2<#INFO#>7<#INFO#>200"
    assert codec.encode([]) == b""                     # Sprint([]) = "[]" -> trimmed
    assert codec.encode([("x", 0, 0)]) == b"x<#INFO#>0<#INFO#>0"


def test_roundtrip_and_go_parse_errors():
    ent = [("10.0.0.%d" % i, i * 3, 1700000000000000000 + i) for i in range(5)]
    assert codec.decode(codec.encode(ent)) == ent
    # strconv errors are ignored -> 0; overflow clamps (ParseInt bitSize 64)
    d = codec.decode(b"a<#INFO#>12x<#INFO#>99999999999999999999999")
    assert d == [("a", 0, (1 << 63) - 1)]
    assert codec.decode(b"a<#INFO#>+7<#INFO#>-3") == [("a", 7, -3)]
    # an address keeps everything before the first <#INFO#>, the ts field the rest
    assert codec.decode(b"a<#INFO#>1<#INFO#>2<#INFO#>3") == [("a", 1, 0)]


def test_decode_panics_where_the_reference_does():
    with pytest.raises(codec.DecodePanic):
        codec.decode(b"")                              # Split("") = [""] -> sentence[1]
    with pytest.raises(codec.DecodePanic):
        codec.decode(b"a<#INFO#>1")
    # 16 UnixNano-stamped members fit the 1,024-byte read buffer (:210)
    ok = [("172.22.157.%d" % i, 1000 + i, 1700000000000000000 + i) for i in range(16)]
    assert len(codec.encode(ok)) <= codec.UDP_READ_BUF and codec.decode(codec.encode(ok)) == ok


@pytest.mark.parametrize("addr_len", [12, 13, 40, 60])  # 13: the cut lands in a ts field
def test_read_buffer_cut(addr_len):
    """A list over 1,024 bytes is cut by ReadFromUDP: entries after the cut
    are lost; an entry cut inside its ts field parses the digits that
    arrived; one cut before its second <#INFO#> panics the reference."""
    ent = [(("m%d-" % i).ljust(addr_len, "x"), 1000 + i, 1700000000000000000 + i) for i in range(40)]
    big = codec.encode(ent)
    assert len(big) > codec.UDP_READ_BUF
    text = big[: codec.UDP_READ_BUF].decode()
    whole = text.split(codec.ENTRY)
    last = whole[-1]
    if last.count(codec.INFO) < 2:
        with pytest.raises(codec.DecodePanic):
            codec.decode(big)
    else:
        got = codec.decode(big)
        assert got[:-1] == ent[: len(whole) - 1]
        addr, hb, ts = got[-1]
        assert (addr, hb) == ent[len(whole) - 1][:2] and ts == int(last.split(codec.INFO)[2])


def test_merge_list_oracle_vs_listsim(oracle_mod):
    """KAT-1 through the external-list path: local [A(5,100),
    B(3,90), C(7,95)], tombstone D; message [B:4, C:7, D:9, E:2, A:4] at now=200
    -> [A(5,100), B(4,200), C(7,95), E(2,200)]."""
    n = 6
    hb = np.full((n, n), -1, np.int32)
    ts = np.zeros((n, n), np.int32)
    alive = np.zeros(n, np.uint8)
    hb[0, :4], ts[0, :4] = [50, 5, 3, 7], [199, 100, 90, 95]
    hb[0, 4], ts[0, 4] = -2, 80
    alive[0] = 1
    o = oracle_mod.Oracle(oracle_mod.default_config(n))
    o.import_state(hb, ts, alive, 200)
    msg = codec.decode(codec.encode([("B", 4, 1), ("C", 7, 1), ("D", 9, 1), ("E", 2, 1), ("A", 4, 1)]))
    ids = {"A": 1, "B": 2, "C": 3, "D": 4, "E": 5}
    assert o.merge_list(0, [ids[a] for a, _, _ in msg], [h for _, h, _ in msg]) == 2
    h2, t2, _ = o.export_state()
    assert list(h2[0]) == [50, 5, 4, 7, -2, 2] and list(t2[0][[1, 2, 3, 5]]) == [100, 200, 95, 200]
    ls = ListSim.from_dense(hb, ts, alive, 200)
    node = ls.nodes[0]
    from oracle.listsim import Member
    changed = node.merge([Member(ids[a], h, 0) for a, h, _ in msg], 200)
    assert len(changed) == 2
    lh, lt, _ = ls.dense()
    assert np.array_equal(lh[0], h2[0])
    assert np.array_equal(sc.export_view(lh, lt, 200, 5)[1][0], t2[0])
