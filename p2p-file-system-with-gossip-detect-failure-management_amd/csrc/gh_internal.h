// Internal definitions shared by libgossiphip's HIP translation units.
//
// Column sharding (DESIGN.md "Multi-GPU"): an engine (rank g of world G)
// holds ALL N observer rows for its member columns
//   [col0, col0 + ncol),  col0 = g * ncs,  ncs = roundup(ceil(N / G), 32),
// so merge, detection, cleanup and REMOVE delivery of a column never leave
// its owner; only O(N) per-row / per-column vectors cross ranks (comm.h).
// G = 1 is the same code with ncol = N.
//
// Device layout (SPEC.md §1/§3, DESIGN.md "Data layout in HBM"):
//   The N x ld local membership tables are stored in column TILES of TW
//   members:
//     cell(i, c) = (c / TW) * (N * TW) + i * TW + c % TW     (c local)
//   i.e. tile t holds local members [t*TW, (t+1)*TW) of every observer row,
//   rows contiguous. One tile of the narrow table is N*TW*2 bytes (8 MiB at
//   N=65,536, TW=64): the round kernel sweeps tile by tile, so its own-row
//   streams are sequential and every peer gather of a tile stays inside
//   that slice.
//   Each cell has one 32-bit meaning (the "wide" encoding):
//                    present    0 <= v:  heartbeat in bits 0..22, age in
//                                        23..29, flag in bit 30
//                    tombstone  v < -1:  INT_MIN | age << 23
//                    absent     v == -1
//                  age = (last completed round + 1) - ts, the cell's age in the
//                  round about to run, saturating at GH_AGE_CAP. flag = the
//                  row's process detects the member in that round (SPEC §2
//                  step 4: hb > 1, member != observer, ts < r - T_fail),
//                  decided when the cell is written, so neither the row nor
//                  the peers reading it as a snapshot re-derive it. Every
//                  decision of a round on ts is a flag test or an age
//                  comparison: a round reads and writes one table, not two.
//   hn[2]  uint16  double-buffered NARROW table, where the round streams: a
//                  heartbeat is stored as an offset from a per-column base
//                  (base[buf][c]):
//                    present    H<<15 | off<<5 | age   off 0..1022, H = flag
//                    tombstone  0xFFE0 | age           age 0..30
//                    absent     0xFFFF
//                  Visible (present, unflagged) cells are the non-negative
//                  int16 values and compare like their heartbeats, so a
//                  snapshot merge is a packed 16-bit max.
//   hw[2]  int32   the wide encoding, for (tile, row) segments that a narrow
//                  cell cannot hold (heartbeat outside [base, base+1022],
//                  saturated tombstone) and for stopped rows (kept wide and
//                  identical in both buffers: the round never touches them).
//                  Every narrow cell of such a segment holds GH_N_WIDE, a code
//                  no narrow cell has, so any reader finds the segment's
//                  encoding from the cell it reads.
//   base[2] int32  per local column: base of buf's narrow cells. The round
//                  sets base[next][c] = (member c's own heartbeat) - GH_BASE_LAG
//                  (k_base), so every view of c within GH_BASE_LAG rounds of
//                  its own counter is narrow.
//   Local columns are padded to ld (multiple of 8*TW and 256); padding cells
//   stay -1.
//   per row (global): alive, active, und (u8), cntl / cntg (local / global
//            present count, [N] = |D|; the rounds keep cntl current by
//            per-segment deltas), post, det_any, inboxes: pull mode
//            inbox[i*(k+1)] = count, then the senders; ring mode inbox_cnt,
//            inbox_beg into inbox.
//   per local column: det_cnt / det_min (x2: pending D_{r-1} and current
//            D_r), dbits (bitmap of pending D_{r-1}), dlist.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/gossiphip.h"

#define GH_HB_BITS 23
#define GH_HB_MAX ((1 << GH_HB_BITS) - 1)  // largest heartbeat a cell holds (saturates)
#define GH_AGE_CAP 31                      // age saturates here; exact ts is then in ts[]
#define GH_N_ABSENT 0xFFFFu                // narrow absent
#define GH_N_TOMB 0xFFE0u                  // narrow tombstone | age
#define GH_N_WIDE 0x7FFFu                  // narrow cell of a wide segment
#define GH_N_OFFMAX 1022                   // largest narrow heartbeat offset
#define GH_BASE_LAG 1000                   // base = own heartbeat - GH_BASE_LAG
#define GH_FLAG (1 << 30)                  // detected next round (present cells)
#define GH_PAD 256               // column padding granule (ld % 256 == 0)
#ifndef GH_WG_CELLS
#define GH_WG_CELLS 16384        // round kernel: cells per workgroup tile (rows = GH_WG_CELLS / TW)
#endif
#define GH_MAXK 8                // max pull fanout
#define GH_DLIST_MAX 1024        // local |D| above which undecided rows are recounted in full
#define GH_TW_DEFAULT 64         // default tile width (members per tile)
#define GH_TAG_PEER 0x50454552u
#define GH_TAG_PLACE 0x504C4143u
#define GH_MAX_DRAWS (1u << 20)

enum {
  ST_DETECTIONS = 0,
  ST_FAILED,
  ST_REMOVE_UNKNOWN,
  ST_RING_EMPTY,  // counted by rank 0 only (replicated computation)
  ST_ACTIVE_ROWS, // counted by rank 0 only
  ST_MERGED,
  ST_RELEASED,
  ST_TOMBSTONED,
  ST_COUNT
};

// Philox4x32-10 (Salmon et al. SC'11), the same stream as SPEC.md §2/§6.
__host__ __device__ inline uint32_t gh_philox_word(uint64_t seed, uint32_t a, uint32_t b,
                                                   uint32_t tag, uint32_t blk, int t) {
  uint32_t c0 = a, c1 = b, c2 = tag, c3 = blk;
  uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
#pragma unroll
  for (int rnd = 0; rnd < 10; ++rnd) {
    if (rnd) {
      k0 += 0x9E3779B9u;
      k1 += 0xBB67AE85u;
    }
    const uint64_t p0 = (uint64_t)0xD2511F53u * c0;
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
    const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0;
    const uint32_t n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
    c1 = (uint32_t)p1;
    c3 = (uint32_t)p0;
    c0 = n0;
    c2 = n2;
  }
  const uint32_t o[4] = {c0, c1, c2, c3};
  return o[t & 3];
}

struct GhDev {
  int32_t n;        // members N (= observer rows = global columns)
  int64_t ld;       // padded LOCAL columns
  int32_t tw;       // tile width (power of two)
  int32_t lgtw;     // log2(tw)
  int64_t tstride;  // cells per tile = n * tw
  int64_t col0;     // global member id of local column 0
  int32_t ncol;     // valid local columns
  int32_t ncs;      // columns per rank (multiple of 32): rank g owns [g*ncs, g*ncs + ncol_g)
  int32_t ncsw;     // ncs / 32 (bitmap words per rank)
  int32_t rank, world;
  int64_t ntiles;   // ld / tw
  uint16_t *hn[2];  // narrow double buffer
  int32_t *hw[2];   // wide double buffer
  int32_t *base[2]; // [ld] narrow base per buffer
  int32_t *colq;    // [ld] scratch: per local column event index / merged value
  int64_t *slow;    // [ntiles * n] round: segments for k_round_slow, tile << 32 | row
  int32_t *slow_n;  // their count
  int32_t *mode;    // k_round variant of the round: 0 lean, 1 storm (k_base)
  int32_t *nstorm;  // storm variant: segments holding flagged or tombstoned cells
  int32_t *nflag;   // [2]: segments written into buffer b holding flagged cells (quirk pre-pass gate)
  int32_t *ts;
  uint8_t *alive, *active, *det_any, *und;
  int32_t *cntl, *cntg;  // [n + 8]: per-row present counts (local / allreduced), [n] = |D|, [n + 1] = nflag[cur]
  int32_t *post;         // [n]: post-REMOVE present counts of undecided rows (allreduced)
  int32_t *det_cnt[2], *det_min[2];
  uint32_t *dbits;
  int32_t *dlist;
  int32_t *nd;      // [0..1] local |D| per parity, [2..3] dlist fill, [4] join adds, [5] list merges
  int32_t *inbox_beg, *inbox_cnt, *inbox, *inbox_fill, *targets;
  int32_t *ring;    // ring mode: [world][n][2] (local snapshot count, local position of the sender)
  uint16_t *rcnt;   // ring mode: [ld/tw][n] snapshot-list members per (tile, sender row)
  uint32_t *rbits;  // gathered presence bitmaps of some rows: [world][nr][ncsw]
  // quirk-mode detection (SPEC §4): per-(tile,row) run summaries / prefixes,
  // per-row totals of every shard, carry-in and last present tile
  uint8_t *qsum;    // [ld/tw][n]
  uint8_t *qall;    // [world][n]
  uint8_t *qcarry;  // [n]: bit0 run state entering this shard, bit1 shard holds the row's last list entry
  int32_t *qlast;   // [n]: local tile of the row's last present cell (-1 none)
  unsigned long long *stats;  // ST_COUNT
  // files (replicated on every rank)
  int64_t fcap;
  int32_t *rep, *ver, *fts;
  uint32_t *draws;
  int32_t *cand, *ncand;
  int32_t *io_a, *io_b, *io_c, *io_d;  // per-call scratch (files, outputs)
  gh_plan_entry *plan;
  int32_t *nplan;
  int64_t io_cap;
};

// ---- cell encoding --------------------------------------------------------
__host__ __device__ __forceinline__ int gh_age(int32_t v) { return (v >> GH_HB_BITS) & 0x7F; }
__host__ __device__ __forceinline__ int32_t gh_hbv(int32_t v) { return v & GH_HB_MAX; }
__host__ __device__ __forceinline__ int32_t gh_present(int32_t hb, int age, bool flag = false) {
  return hb | (age << GH_HB_BITS) | (flag ? GH_FLAG : 0);
}
__host__ __device__ __forceinline__ int32_t gh_tomb(int age) {
  return (int32_t)(0x80000000u | ((uint32_t)age << GH_HB_BITS));
}
// age one round later (saturating)
__host__ __device__ __forceinline__ int gh_inc(int a) { return a < GH_AGE_CAP ? a + 1 : GH_AGE_CAP; }
// external value (>= 0 heartbeat, -1 absent, -2 tombstone)
__host__ __device__ __forceinline__ int32_t gh_ext(int32_t v) {
  return v >= 0 ? gh_hbv(v) : (v == GH_ABSENT ? GH_ABSENT : GH_TOMBSTONE);
}

// Linear index of cell (observer i, LOCAL member column c) in the tiled layout.
__host__ __device__ __forceinline__ int64_t gh_cell(const GhDev& d, int64_t i, int64_t c) {
  return (c >> d.lgtw) * d.tstride + (i << d.lgtw) + (c & (d.tw - 1));
}

// ---- narrow <-> wide --------------------------------------------------
__host__ __device__ __forceinline__ int32_t gh_dec16(uint32_t x, int32_t base) {
  if (x == GH_N_ABSENT) return GH_ABSENT;
  const int a = x & 31, f = (x >> 5) & 1023;
  if (f == 1023) return gh_tomb(a);
  return gh_present(base + f, a, (x >> 15) != 0);
}
// narrow code of wide value v; fit &= it has one
__host__ __device__ __forceinline__ uint32_t gh_enc16(int32_t v, int32_t base, bool& fit) {
  if (v == GH_ABSENT) return GH_N_ABSENT;
  const int a = gh_age(v);
  if (v < 0) {
    fit &= a < 31;
    return GH_N_TOMB | (a & 31);
  }
  const int64_t off = (int64_t)gh_hbv(v) - base;
  fit &= off >= 0 && off <= GH_N_OFFMAX && a <= 31;
  return ((v & GH_FLAG) ? 0x8000u : 0u) | ((uint32_t)(off & 1023) << 5) | (uint32_t)(a & 31);
}

// Cell (i, local c) of buffer buf, wide encoding.
__device__ __forceinline__ int32_t gh_get(const GhDev& d, int buf, int64_t i, int64_t c) {
  const int64_t off = gh_cell(d, i, c);
  const uint32_t x = d.hn[buf][off];
  return x == GH_N_WIDE ? d.hw[buf][off] : gh_dec16(x, d.base[buf][c]);
}

typedef int v4i __attribute__((ext_vector_type(4)));
// Cells (i, c..c+3) of buffer buf (c % 4 == 0), wide encoding.
__device__ __forceinline__ v4i gh_load4(const GhDev& d, int buf, int64_t i, int64_t c) {
  const int64_t off = gh_cell(d, i, c);
  const uint2 x = *reinterpret_cast<const uint2*>(d.hn[buf] + off);
  if ((x.x & 0xFFFFu) == GH_N_WIDE) return *reinterpret_cast<const v4i*>(d.hw[buf] + off);
  const v4i b = *reinterpret_cast<const v4i*>(d.base[buf] + c);
  v4i v;
  v.x = gh_dec16(x.x & 0xFFFFu, b.x);
  v.y = gh_dec16(x.x >> 16, b.y);
  v.z = gh_dec16(x.y & 0xFFFFu, b.z);
  v.w = gh_dec16(x.y >> 16, b.w);
  return v;
}
// Presence and flag bits of cells (i, c..c+7) of buffer buf (c % 8 == 0):
// bit j = present, bit 8 + j = present and flagged. Narrow codes answer
// directly (no base).
__device__ __forceinline__ uint32_t gh_pf8(const GhDev& d, int buf, int64_t i, int64_t c) {
  const int64_t off = gh_cell(d, i, c);
  const uint4 x = *reinterpret_cast<const uint4*>(d.hn[buf] + off);
  uint32_t out = 0;
  if ((x.x & 0xFFFFu) == GH_N_WIDE) {
    const v4i a = *reinterpret_cast<const v4i*>(d.hw[buf] + off);
    const v4i b = *reinterpret_cast<const v4i*>(d.hw[buf] + off + 4);
    const int32_t v[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if (v[j] >= 0) out |= (1u << j) | ((v[j] & GH_FLAG) ? 1u << (8 + j) : 0u);
  } else {
    const uint32_t w[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const uint32_t h = (w[j >> 1] >> (16 * (j & 1))) & 0xFFFFu;
      if (h < GH_N_TOMB) out |= (1u << j) | (h >= 0x8000u ? 1u << (8 + j) : 0u);
    }
  }
  return out;
}
// Clears the flag of present cells (i, c + j) for the bits j of m (c % 8 == 0).
__device__ __forceinline__ void gh_clearflags8(const GhDev& d, int buf, int64_t i, int64_t c, uint32_t m) {
  const int64_t off = gh_cell(d, i, c);
  uint4* np = reinterpret_cast<uint4*>(d.hn[buf] + off);
  uint4 x = *np;
  if ((x.x & 0xFFFFu) == GH_N_WIDE) {
    v4i* wp = reinterpret_cast<v4i*>(d.hw[buf] + off);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      v4i v = wp[h];
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if ((m >> (4 * h + j)) & 1u) v[j] &= ~GH_FLAG;
      wp[h] = v;
    }
    return;
  }
  uint32_t w[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
  for (int j = 0; j < 8; ++j)
    if ((m >> j) & 1u) w[j >> 1] &= ~(0x8000u << (16 * (j & 1)));
  *np = uint4{w[0], w[1], w[2], w[3]};
}

// ts < r - T for a present or tombstoned cell (stored v at table offset off)
// in round r: the age decides, except for a saturated age when T itself
// reaches the cap (then the exact ts is in d.ts).
// EXACT = false is the form for T < GH_AGE_CAP (every realistic timeout):
// pure register arithmetic, no conditional load in the streaming loops.
template <bool EXACT = true>
__device__ __forceinline__ bool gh_stale(const GhDev& d, int32_t v, int64_t off, int32_t r, int32_t T) {
  const int a = gh_age(v);
  if constexpr (!EXACT) {
    return a > T;
  } else {
    if (a < GH_AGE_CAP || T < GH_AGE_CAP) return a > T;
    return d.ts[off] < r - T;
  }
}

// The flag of a present cell written for round rn (member cg of row i, exact
// ts: age < cap ? rn - age : ts[off]).
template <bool EXACT>
__device__ __forceinline__ bool gh_flag_for(const GhDev& d, int32_t hb, int age, int64_t cg, int64_t i, int64_t off,
                                           int32_t rn, int32_t t_fail) {
  if (hb <= 1 || cg == i) return false;
  if constexpr (!EXACT) {
    return age > t_fail;
  } else {
    if (age < GH_AGE_CAP || t_fail < GH_AGE_CAP) return age > t_fail;
    return d.ts[off] < rn - t_fail;
  }
}

// Bit of GLOBAL member j in row q of a gathered bitmap [world][nr][ncsw].
__device__ __forceinline__ bool gh_gbit(const GhDev& d, const uint32_t* bits, int nr, int q, int64_t j) {
  const int64_t o = j / d.ncs;
  const int64_t lc = j - o * d.ncs;
  return (bits[(o * nr + q) * d.ncsw + (lc >> 5)] >> (lc & 31)) & 1u;
}

// Receiver i's inbox: sender count and the offset of the first sender in
// d.inbox (pull: count in slot 0 of a (k+1)-int row, so a shard's receivers
// are one contiguous slice for the allgather; ring: CSR).
__device__ __forceinline__ int gh_in_cnt(const GhDev& d, bool pull, int k, int64_t i) {
  return pull ? d.inbox[i * (k + 1)] : d.inbox_cnt[i];
}
__device__ __forceinline__ int64_t gh_in_beg(const GhDev& d, bool pull, int k, int64_t i) {
  return pull ? i * (k + 1) + 1 : (int64_t)d.inbox_beg[i];
}

// Parameters of one round, passed by value to the kernels.
struct GhRound {
  int32_t r;          // now
  int32_t n;
  int64_t ld;
  int32_t t_fail, t_cleanup, min_members;
  int32_t k;
  uint64_t seed;
  int32_t peer_mode;
  int32_t xmap;       // k_round block->tile map: 0 tile-major, 1 XCD-aware
  int32_t tpw;        // k_round tiles per workgroup (1, 2, 4, 8)
  int32_t exact;      // T_fail or T_cleanup >= GH_AGE_CAP: every cell by the slow rule (exact ts)
  int32_t qgate;      // quirk pre-pass: 1 = return at once when cntg[n + 1] (flagged segments, all shards) is 0
  int32_t force_storm;  // diagnostics (GH_FORCE_STORM): run the storm variant every round
};

// ---- launchers (kernels in round.hip / events.hip / place.hip) ----------
// round.hip
void launch_active_pre(const GhDev& d, int cur, int dcur, const GhRound& p, hipStream_t s);
void launch_active_post(const GhDev& d, const GhRound& p, hipStream_t s);
void launch_peers_pull(const GhDev& d, int cur, int dcur, const GhRound& p, hipStream_t s);
void launch_ring_count(const GhDev& d, int cur, int dcur, const GhRound& p, hipStream_t s);
void launch_ring_select(const GhDev& d, int cur, int dcur, const GhRound& p, hipStream_t s);
void launch_inbox(const GhDev& d, const GhRound& p, hipStream_t s);
// nt = non-temporal hints on the once-touched streams of k_round
// storm: the storm variant (else the lean one); both are launched every
// round and only the one k_base selected runs
void launch_round(const GhDev& d, int cur, int dcur, const GhRound& p, hipStream_t s, bool nt, bool storm);
// the segments k_round listed, by the per-cell rule (after launch_round)
void launch_round_slow(const GhDev& d, int cur, int dcur, const GhRound& p, hipStream_t s);
void launch_finish(const GhDev& d, int dcur, const GhRound& p, hipStream_t s);
// base[cur ^ 1] from buffer cur (member c's own heartbeat - GH_BASE_LAG),
// |D_{r-1}| next to the local counts, empty slow list
void launch_base(const GhDev& d, int cur, int dcur, const GhRound& p, hipStream_t s);
// quirk-mode detection: summaries + per-row prefix (then allgather qall), and
// carry-in + flag rewrite of the current table
void launch_quirk_scan(const GhDev& d, int cur, int dcur, const GhRound& p, hipStream_t s);
void launch_quirk_apply(const GhDev& d, int cur, int dcur, const GhRound& p, hipStream_t s);
// events.hip
void launch_count(const GhDev& d, int cur, const GhRound& p, hipStream_t s);
void launch_fill(const GhDev& d, int cur, int32_t hb0, int32_t ts0, const GhRound& p,
                 hipStream_t s);
// full host rows (hb, ts: [nrows][n]) -> encoded tiled local columns; p.r is
// the round about to run
void launch_pack(const GhDev& d, int cur, const int32_t* hb_rows, const int32_t* ts_rows, int64_t row0,
                 int64_t nrows, const GhRound& p, hipStream_t s);
// tiled local columns -> [nrows][ncs] (local column order) of the external hb
// (what = 0) or the exact ts (what = 1); p.r is the round about to run
void launch_unpack(const GhDev& d, int cur, int32_t* dst_rows, int64_t row0, int64_t nrows, int what,
                   const GhRound& p, hipStream_t s);
// rows that stop (crash / leave): exact ts of their cells into ts[], rows
// stored wide in both buffers
void launch_freeze(const GhDev& d, int cur, const int32_t* rows, int32_t nr, const GhRound& p, hipStream_t s);
// number of wide segments of buffer buf -> *out (device)
void launch_count_wide(const GhDev& d, int buf, unsigned long long* out, hipStream_t s);
// presence bitmaps of rows[0..nr) over the local columns -> rbits + rank*nr*ncsw
void launch_rowbits(const GhDev& d, int cur, const int32_t* rows, int32_t nr, hipStream_t s);
// leavers[0..nl) (global ids); tiles[0..ntl): the distinct local tiles of
// the local ones
void launch_leave(const GhDev& d, int cur, const int32_t* leavers, const int32_t* tiles, int32_t ntl, int32_t nl,
                  const GhRound& p, hipStream_t s);
void launch_join_add(const GhDev& d, int cur, const int32_t* joiners, int32_t nj, int32_t introducer,
                     const GhRound& p, hipStream_t s);
void launch_join_bcast(const GhDev& d, int cur, int32_t introducer, const GhRound& p, hipStream_t s);
// MergeMemberList of an external list into one row (nd[5] counts merges)
void launch_merge_list(const GhDev& d, int cur, int32_t obs, const int32_t* ids, const int32_t* hb, int64_t n,
                       const GhRound& p, hipStream_t s);
void launch_join_reset(const GhDev& d, int cur, const int32_t* rows, int32_t nr, const GhRound& p,
                       hipStream_t s);
// place.hip (rbits holds the master row [q=0] and, for repair, the observer row [q=1])
void launch_candidates(const GhDev& d, int32_t nr, hipStream_t s);
void launch_put(const GhDev& d, int32_t nr, int64_t n, int32_t R, int32_t now, uint64_t seed, hipStream_t s);
void launch_repair(const GhDev& d, int32_t nr, int32_t R, uint64_t seed, hipStream_t s);
void launch_get(const GhDev& d, int64_t n, int32_t R, int del, hipStream_t s);
void launch_conflicts(const GhDev& d, int64_t n, int32_t now, int32_t window, hipStream_t s);
// master re-election (elect.hip): out [2n] = per-row (n - first local present
// member, 0 none) and (mview[i] present locally), both MAX-reducible
void launch_vote_scan(const GhDev& d, int cur, const int32_t* mview, int32_t* out, hipStream_t s);
// rebuild_file_meta at new master M with its list's first nl (<= 5) members L
void launch_rebuild(const GhDev& d, int32_t R, int32_t M, const int32_t* L, int32_t nl, int32_t m_listed,
                    int32_t now, hipStream_t s);
