/*
 * ORACLE / TEST INFRASTRUCTURE ONLY — never linked into libgossiphip.
 *
 * Philox4x32-10 (Salmon et al., "Parallel random numbers: as easy as 1, 2, 3",
 * SC'11), hand-written. Round constants cross-checked against
 * /opt/rocm/include/rocrand/rocrand_philox4x32_10.h:62-65 and pinned by
 * tests/test_philox.py against rocRAND's engine and the Random123 KATs.
 *
 * Replaces the reference's time-seeded math/rand draws
 * (master/master.go:134-135) with a counter-based stream (SPEC.md §6, D6).
 */
#ifndef ORACLE_PHILOX_H_
#define ORACLE_PHILOX_H_
#include <stdint.h>

#define OR_PHILOX_M0 0xD2511F53u
#define OR_PHILOX_M1 0xCD9E8D57u
#define OR_PHILOX_W0 0x9E3779B9u
#define OR_PHILOX_W1 0xBB67AE85u

#define OR_TAG_PEER 0x50454552u  /* 'PEER' */
#define OR_TAG_PLACE 0x504C4143u /* 'PLAC' */

static inline void or_philox4x32_10_raw(const uint32_t ctr_in[4], const uint32_t key_in[2],
                                        uint32_t out[4]) {
  uint32_t c0 = ctr_in[0], c1 = ctr_in[1], c2 = ctr_in[2], c3 = ctr_in[3];
  uint32_t k0 = key_in[0], k1 = key_in[1];
  for (int round = 0; round < 10; ++round) {
    if (round > 0) {
      k0 += OR_PHILOX_W0;
      k1 += OR_PHILOX_W1;
    }
    uint64_t p0 = (uint64_t)OR_PHILOX_M0 * c0;
    uint64_t p1 = (uint64_t)OR_PHILOX_M1 * c2;
    uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    uint32_t n0 = hi1 ^ c1 ^ k0;
    uint32_t n2 = hi0 ^ c3 ^ k1;
    c0 = n0;
    c1 = lo1;
    c2 = n2;
    c3 = lo0;
  }
  out[0] = c0;
  out[1] = c1;
  out[2] = c2;
  out[3] = c3;
}

/* Draw word `t` (0..3) of the block at counter (a, b, tag, blk). */
static inline uint32_t or_philox_word(uint64_t seed, uint32_t a, uint32_t b, uint32_t tag,
                                      uint32_t blk, int t) {
  uint32_t ctr[4] = {a, b, tag, blk};
  uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
  uint32_t out[4];
  or_philox4x32_10_raw(ctr, key, out);
  return out[t & 3];
}

#endif
