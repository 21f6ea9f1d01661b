// Internal definitions shared by libgossiphip's HIP translation units.
//
// Device layout (SPEC.md §1/§3, DESIGN.md "Data layout in HBM"):
//   The N x N membership tables are stored in column TILES of TW members:
//     cell(i, c) = (c / TW) * (N * TW) + i * TW + c % TW
//   i.e. tile t holds members [t*TW, (t+1)*TW) of every observer row, rows
//   contiguous. One tile of one table is N*TW*4 bytes (16 MiB at N=65,536,
//   TW=64): the round kernel sweeps tile by tile, so its own-row streams are
//   sequential and every peer gather of a tile stays inside that slice.
//   hb[2]  int32   double-buffered heartbeat table; bit 30 of a present cell =
//                  next-round detection eligibility; -1 absent, -2 tombstone.
//   ts     int32   local-clock tick of each cell, updated in place.
//   Columns are padded to ld = N rounded up to 256 (padding cells stay -1).
//   per row: alive, active (u8), cnt (present count), det_any (u8),
//            inbox_beg / inbox_cnt (int32), inbox[] (sender rows).
//   per column: det_cnt / det_min (x2: pending D_{r-1} and current D_r),
//            dbits (bitmap of pending D_{r-1}).
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
#define GH_DLIST_MAX 1024        // |D| above which k_active_exact recounts whole rows
#define GH_TW_DEFAULT 64         // default tile width (members per tile)
#define GH_TAG_PEER 0x50454552u
#define GH_TAG_PLACE 0x504C4143u
#define GH_MAX_DRAWS (1u << 20)

enum {
  ST_DETECTIONS = 0,
  ST_FAILED,
  ST_REMOVE_UNKNOWN,
  ST_RING_EMPTY,
  ST_ACTIVE_ROWS,
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
  int32_t n;        // members (= observer rows)
  int64_t ld;       // padded columns (multiple of GH_PAD)
  int32_t tw;       // tile width (power of two, divides GH_PAD)
  int32_t lgtw;     // log2(tw)
  int64_t tstride;  // cells per tile = n * tw
  int32_t *hb[2];   // double buffer
  int32_t *ts;
  uint8_t *alive, *active, *det_any;
  int32_t *cnt;
  int32_t *det_cnt[2], *det_min[2];
  uint32_t *dbits;
  int32_t *dlist;
  int32_t *nd;      // [0..1] |D| per parity, [2..3] dlist fill, [4] join adds
  uint16_t *part;
  int32_t *inbox_beg, *inbox_cnt, *inbox, *inbox_fill, *targets;
  unsigned long long *stats;  // ST_COUNT
  // files
  int64_t fcap;
  int32_t *rep, *ver, *fts;
  uint32_t *draws;
  int32_t *cand, *ncand;
  int32_t *io_a, *io_b, *io_c, *io_d;  // per-call scratch (files, outputs)
  gh_plan_entry *plan;
  int32_t *nplan;
  int64_t io_cap;
};

// Linear index of cell (observer i, member c) in the tiled layout.
__host__ __device__ __forceinline__ int64_t gh_cell(const GhDev& d, int64_t i, int64_t c) {
  return (c >> d.lgtw) * d.tstride + (i << d.lgtw) + (c & (d.tw - 1));
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
void launch_active(const GhDev& d, int cur, int dcur, const GhRound& p, hipStream_t s);
void launch_peers_pull(const GhDev& d, int cur, int dcur, const GhRound& p, hipStream_t s);
void launch_ring(const GhDev& d, int cur, int dcur, const GhRound& p, hipStream_t s);
// nt = non-temporal hints on the once-touched streams of k_round
void launch_round(const GhDev& d, int cur, int dcur, const GhRound& p, hipStream_t s, bool nt);
void launch_finish(const GhDev& d, int dcur, const GhRound& p, hipStream_t s);
void launch_count(const GhDev& d, int cur, const GhRound& p, hipStream_t s);
void launch_flags(const GhDev& d, int cur, int64_t row0, int64_t nrows, const GhRound& p,
                  hipStream_t s);
void launch_fill(const GhDev& d, int cur, int32_t hb0, int32_t ts0, const GhRound& p,
                 hipStream_t s);
// row-major staging [nrows][n] <-> tiled tables (import/export/lsm)
void launch_pack(const GhDev& d, int32_t* dst_tiled, const int32_t* src_rows, int64_t row0,
                 int64_t nrows, hipStream_t s);
void launch_unpack(const GhDev& d, int32_t* dst_rows, const int32_t* src_tiled, int64_t row0,
                   int64_t nrows, int strip_flag, hipStream_t s);
void launch_leave(const GhDev& d, int cur, const int32_t* leavers, int32_t nl, const GhRound& p,
                  hipStream_t s);
void launch_join(const GhDev& d, int cur, const int32_t* joiners, int32_t nj, int32_t introducer,
                 const GhRound& p, hipStream_t s);
void launch_join_reset(const GhDev& d, int cur, const int32_t* rows, int32_t nr, const GhRound& p,
                       hipStream_t s);
void launch_candidates(const GhDev& d, int cur, int32_t master, const GhRound& p, hipStream_t s);
// placement reads the master's (and the observer's) row of the current hb
void launch_put(const GhDev& d, const int32_t* hb, int32_t master, int64_t n, int32_t R, int32_t now,
                uint64_t seed, hipStream_t s);
void launch_repair(const GhDev& d, const int32_t* hb, int32_t master, int32_t observer, int32_t R,
                   uint64_t seed, hipStream_t s);
void launch_get(const GhDev& d, int64_t n, int32_t R, int del, hipStream_t s);
