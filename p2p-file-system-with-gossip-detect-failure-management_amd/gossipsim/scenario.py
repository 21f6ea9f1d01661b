"""Workload generation for the BASELINE configurations: the
crash sets drawn by Philox4x32-10 (Salmon et al., SC'11) keyed by (seed;
draw index, tag CRASH), vectorised over draws with numpy. The same stream as
SPEC.md §6's scenario draws, so bench legs and parity tests crash the same
members."""
from __future__ import annotations

import numpy as np

TAG_CRASH = 0x43525348  # 'CRSH'
_M0, _M1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57)
_W0, _W1 = 0x9E3779B9, 0xBB67AE85
_LO = np.uint64(0xFFFFFFFF)


def philox_words(seed: int, a: np.ndarray, b: int, tag: int, blk: int) -> np.ndarray:
    """Word 0 of Philox4x32-10 at counters (a[x], b, tag, blk), key = seed
    (64-bit: low word k0, high word k1), for every x."""
    c0 = np.asarray(a, np.uint64) & _LO
    c1 = np.full_like(c0, b & 0xFFFFFFFF)
    c2 = np.full_like(c0, tag & 0xFFFFFFFF)
    c3 = np.full_like(c0, blk & 0xFFFFFFFF)
    k0, k1 = seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF
    for rnd in range(10):
        if rnd:
            k0 = (k0 + _W0) & 0xFFFFFFFF
            k1 = (k1 + _W1) & 0xFFFFFFFF
        p0 = _M0 * c0
        p1 = _M1 * c2
        n0 = (p1 >> np.uint64(32)) ^ c1 ^ np.uint64(k0)
        n2 = (p0 >> np.uint64(32)) ^ c3 ^ np.uint64(k1)
        c1, c3 = p1 & _LO, p0 & _LO
        c0, c2 = n0 & _LO, n2 & _LO
    return c0


def crash_ids(n: int, frac: float, seed: int) -> list[int]:
    """`round(frac * n)` distinct members (at least 1) drawn in order by
    Philox(seed; draw d, 0, CRASH, 0) -> floor(u * n / 2^32); the introducer
    / master 0 is never drawn."""
    count = max(1, int(round(n * frac)))
    out, seen, d = [], {0}, 0
    while len(out) < count:
        u = philox_words(seed, np.arange(d, d + 4 * count, dtype=np.uint64), 0, TAG_CRASH, 0)
        d += 4 * count
        for x in ((u * np.uint64(n)) >> np.uint64(32)).tolist():
            if x not in seen:
                seen.add(x)
                out.append(x)
                if len(out) == count:
                    break
    return out
