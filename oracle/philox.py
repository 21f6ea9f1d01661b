"""ORACLE / TEST INFRASTRUCTURE ONLY.

Pure-Python Philox4x32-10 (same stream as oracle/philox.h), used by the
literal list replay (oracle/listsim.py) and by scenario generators in tests
and bench.py (crash-ID draws). Pinned against rocRAND and the Random123 KATs in
tests/test_philox.py.
"""
M0, M1 = 0xD2511F53, 0xCD9E8D57
W0, W1 = 0x9E3779B9, 0xBB67AE85
MASK = 0xFFFFFFFF

TAG_PEER = 0x50454552   # 'PEER'
TAG_PLACE = 0x504C4143  # 'PLAC'
TAG_CRASH = 0x43525348  # 'CRSH' (scenario generation only)
TAG_CHURN = 0x43485552  # 'CHUR' (scenario generation only)


def philox4x32_10(ctr, key):
    c0, c1, c2, c3 = (x & MASK for x in ctr)
    k0, k1 = (x & MASK for x in key)
    for rnd in range(10):
        if rnd:
            k0 = (k0 + W0) & MASK
            k1 = (k1 + W1) & MASK
        p0 = M0 * c0
        p1 = M1 * c2
        c0, c1, c2, c3 = ((p1 >> 32) ^ c1 ^ k0) & MASK, p1 & MASK, ((p0 >> 32) ^ c3 ^ k1) & MASK, p0 & MASK
    return c0, c1, c2, c3


def word(seed, a, b, tag, blk, t):
    return philox4x32_10((a, b, tag, blk), (seed & MASK, (seed >> 32) & MASK))[t & 3]


def peer(seed, i, r, t, population):
    """SPEC §2 step 6: the t-th pull peer of receiver i in round r."""
    u = word(seed, i, r, TAG_PEER, t >> 2, t & 3)
    q = (u * (population - 1)) >> 32
    return q + (1 if q >= i else 0)


def place_index(seed, f, d, m):
    """SPEC §6: Intn(M-1) replacement for draw d of file f."""
    u = word(seed, f, d, TAG_PLACE, 0, 0)
    return (u * (m - 1)) >> 32


def sample_distinct(seed, tag, count, population, exclude=()):
    """Deterministic draw of `count` distinct IDs (scenario generation)."""
    out, seen, d = [], set(exclude), 0
    while len(out) < count:
        u = word(seed, d, 0, tag, 0, 0)
        d += 1
        x = (u * population) >> 32
        if x not in seen:
            seen.add(x)
            out.append(x)
    return out
