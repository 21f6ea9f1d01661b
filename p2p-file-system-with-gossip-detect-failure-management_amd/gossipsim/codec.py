"""The reference's gossip datagram format (slave/slave.go:365-385), byte for
byte, so the engine can emit and ingest real reference messages.

  encode  entries "addr<#INFO#>hb<#INFO#>ts" joined by "<#ENTRY#>" — Go builds
          fmt.Sprint([]string) = "[e1 e2 ...]", trims "[]" and turns every
          space into "<#ENTRY#>" (:365-373)
  decode  split on "<#ENTRY#>", SplitN(e, "<#INFO#>", 3), strconv.Atoi /
          ParseInt with their errors ignored (:375-385), after GetMsg's
          1,024-byte read buffer (:210) has cut longer datagrams

An entry with fewer than three fields makes the reference index out of range
(a panic that ends its GetMsg goroutine); decode raises DecodePanic there —
which is also what a datagram over 1,024 bytes usually does, so a list of
more than ~16 members never reaches MergeMemberList in the reference.
"""
from __future__ import annotations

INFO = "<#INFO#>"
ENTRY = "<#ENTRY#>"
UDP_READ_BUF = 1024  # buf := make([]byte, 1024), slave/slave.go:210
_I64 = (1 << 63) - 1


class DecodePanic(ValueError):
    """The reference's decode would panic on this datagram."""


def encode(entries) -> bytes:
    """entries: iterable of (address, heartbeat, update_time)."""
    d = [f"{addr}{INFO}{hb}{INFO}{ts}" for addr, hb, ts in entries]
    s = "[" + " ".join(d) + "]"          # fmt.Sprint of a []string
    s = s.strip("[]")                     # strings.Trim(.., "[]")
    return s.replace(" ", ENTRY).encode("latin-1")


def _parse_int(s: str, bits: int = 64) -> int:
    """strconv.ParseInt(s, 10, 64) with the error ignored: 0 on a syntax
    error, the clamped extreme on overflow."""
    if not s:
        return 0
    body = s[1:] if s[0] in "+-" else s
    if not body or not all("0" <= ch <= "9" for ch in body):
        return 0
    v = int(s)
    lim = (1 << (bits - 1))
    return max(-lim, min(lim - 1, v))


def decode(data: bytes, read_buf: int = UDP_READ_BUF):
    """-> list of (address, heartbeat, update_time) as the reference sees it."""
    vv = data[:read_buf].decode("latin-1")  # Go string(buf[:n]) keeps raw bytes
    out = []
    for ss in vv.split(ENTRY):
        sentence = ss.split(INFO, 2)
        if len(sentence) < 3:
            raise DecodePanic(f"index out of range in decode (slave/slave.go:379): {ss[:40]!r}")
        out.append((sentence[0], _parse_int(sentence[1]), _parse_int(sentence[2])))
    return out
