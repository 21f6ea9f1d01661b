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
//   rows contiguous. One tile of one table is N*TW*4 bytes (16 MiB at
//   N=65,536, TW=64): the round kernel sweeps tile by tile, so its own-row
//   streams are sequential and every peer gather of a tile stays inside
//   that slice.
//   hb[2]  int32   double-buffered heartbeat table; bit 30 of a present cell =
//                  next-round detection eligibility; -1 absent, -2 tombstone.
//   ts     int32   local-clock tick of each cell, updated in place.
//   Local columns are padded to ld (multiple of 8*TW and 256); padding cells
//   stay -1.
//   per row (global): alive, active, und (u8), cntl / cntg (local / global
//            present count, [N] = |D|), post, det_any, inbox_cnt, inbox[].
//   per local column: det_cnt / det_min (x2: pending D_{r-1} and current
//            D_r), dbits (bitmap of pending D_{r-1}), dlist.
//   part[ld/TW][N] uint16  per-(tile,row) present counts of the last pass.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/gossiphip.h"

#define GH_FLAG (1 << 30)        // eligibility bit inside a present hb cell
#define GH_HBMASK (GH_FLAG - 1)  // heartbeat value bits
#define GH_PAD 256               // column padding granule (ld % 256 == 0)
#define GH_RB 64                 // rows per workgroup tile in the round kernel
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
  int32_t *hb[2];   // double buffer
  int32_t *ts;
  uint8_t *alive, *active, *det_any, *und;
  int32_t *cntl, *cntg;  // [n + 8]: per-row present counts (local / allreduced), [n] = |D|
  int32_t *post;         // [n]: post-REMOVE present counts of undecided rows (allreduced)
  int32_t *det_cnt[2], *det_min[2];
  uint32_t *dbits;
  int32_t *dlist;
  int32_t *nd;      // [0..1] local |D| per parity, [2..3] dlist fill, [4] join adds
  uint16_t *part;
  int32_t *inbox_beg, *inbox_cnt, *inbox, *inbox_fill, *targets;
  int32_t *ring;    // ring mode: [world][n][2] (local snapshot count, local position of the sender)
  uint32_t *rbits;  // gathered presence bitmaps of some rows: [world][nr][ncsw]
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

// Linear index of cell (observer i, LOCAL member column c) in the tiled layout.
__host__ __device__ __forceinline__ int64_t gh_cell(const GhDev& d, int64_t i, int64_t c) {
  return (c >> d.lgtw) * d.tstride + (i << d.lgtw) + (c & (d.tw - 1));
}

// Bit of GLOBAL member j in row q of a gathered bitmap [world][nr][ncsw].
__device__ __forceinline__ bool gh_gbit(const GhDev& d, const uint32_t* bits, int nr, int q, int64_t j) {
  const int64_t o = j / d.ncs;
  const int64_t lc = j - o * d.ncs;
  return (bits[(o * nr + q) * d.ncsw + (lc >> 5)] >> (lc & 31)) & 1u;
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
  int32_t ablate;     // timing-only experiments (results wrong): 1 = every
                      // peer load reads the own row, 2 = no peer loads. 0 always
                      // in production (set only through GH_ROUND_ABLATE).
};

// ---- launchers (kernels in round.hip / events.hip / place.hip) ----------
// round.hip
void launch_prep(const GhDev& d, int dcur, hipStream_t s);
void launch_active_pre(const GhDev& d, int cur, int dcur, const GhRound& p, hipStream_t s);
void launch_active_post(const GhDev& d, const GhRound& p, hipStream_t s);
void launch_peers_pull(const GhDev& d, int cur, int dcur, const GhRound& p, hipStream_t s);
void launch_ring_count(const GhDev& d, int cur, int dcur, const GhRound& p, hipStream_t s);
void launch_ring_select(const GhDev& d, int cur, int dcur, const GhRound& p, hipStream_t s);
void launch_inbox(const GhDev& d, const GhRound& p, hipStream_t s);
// nt = non-temporal hints on the once-touched streams of k_round
void launch_round(const GhDev& d, int cur, int dcur, const GhRound& p, hipStream_t s, bool nt);
void launch_finish(const GhDev& d, int dcur, const GhRound& p, hipStream_t s);
// events.hip
void launch_count(const GhDev& d, int cur, const GhRound& p, hipStream_t s);
void launch_flags(const GhDev& d, int cur, int64_t row0, int64_t nrows, const GhRound& p,
                  hipStream_t s);
void launch_fill(const GhDev& d, int cur, int32_t hb0, int32_t ts0, const GhRound& p,
                 hipStream_t s);
// full rows [nrows][n] (host order) -> tiled local columns
void launch_pack(const GhDev& d, int32_t* dst_tiled, const int32_t* src_rows, int64_t row0,
                 int64_t nrows, hipStream_t s);
// tiled local columns -> [nrows][ncs] (local column order)
void launch_unpack(const GhDev& d, int32_t* dst_rows, const int32_t* src_tiled, int64_t row0,
                   int64_t nrows, int strip_flag, hipStream_t s);
// presence bitmaps of rows[0..nr) over the local columns -> rbits + rank*nr*ncsw
void launch_rowbits(const GhDev& d, int cur, const int32_t* rows, int32_t nr, hipStream_t s);
void launch_leave(const GhDev& d, int cur, const int32_t* leavers, int32_t nl, const GhRound& p,
                  hipStream_t s);
void launch_join_add(const GhDev& d, int cur, const int32_t* joiners, int32_t nj, int32_t introducer,
                     const GhRound& p, hipStream_t s);
void launch_join_bcast(const GhDev& d, int cur, int32_t introducer, const GhRound& p, hipStream_t s);
void launch_join_reset(const GhDev& d, int cur, const int32_t* rows, int32_t nr, const GhRound& p,
                       hipStream_t s);
// place.hip (rbits holds the master row [q=0] and, for repair, the observer row [q=1])
void launch_candidates(const GhDev& d, int32_t nr, hipStream_t s);
void launch_put(const GhDev& d, int32_t nr, int64_t n, int32_t R, int32_t now, uint64_t seed, hipStream_t s);
void launch_repair(const GhDev& d, int32_t nr, int32_t R, uint64_t seed, hipStream_t s);
void launch_get(const GhDev& d, int64_t n, int32_t R, int del, hipStream_t s);
