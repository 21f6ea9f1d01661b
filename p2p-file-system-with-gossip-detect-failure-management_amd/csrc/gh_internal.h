// Internal definitions shared by libgossiphip's HIP translation units.
//
// Column sharding (DESIGN.md "Multi-GPU"): an engine (rank g of world G)
// holds ALL N observer rows for its member columns
//   [col0, col0 + ncol),  col0 = g * ncs,  ncs = roundup(ceil(N / G), 32),
// so merge, detection, cleanup and REMOVE delivery of a column never leave
// its owner; only O(N) per-row / per-column vectors cross ranks (comm.h).
// G = 1 is the same code with ncol = N.
//
// Row sharding (GH_LAYOUT_ROWS, north_star; DESIGN.md "Multi-GPU"): rank g
// holds observer rows [row0, row0 + nrows) for ALL member columns (col0 = 0,
// ncol = N), plus GHOST rows: the snapshots of the senders its receivers pull
// this round, received from their owners by alltoallv before the round. Row
// SLOTS: owned row i at slot i - row0 of the (tiled, double-buffered) table;
// ghost j at slot nrows + j, held in the single ghost table gcodes / gplane
// (row-major, [gcap][ld], written by the alltoallv itself); rslot[i] maps a
// global row to its slot (-1: not held). Column layout: row0 = 0, nrows =
// nslots = N, rslot = null (slot = row id), no ghosts.
//
// Device layout (SPEC.md §1/§3, DESIGN.md "Data layout in HBM"):
//   The N x ld local membership tables are stored in column TILES of TW
//   members:
//     cell(i, c) = (c / TW) * (N * TW) + i * TW + c % TW     (c local)
//   i.e. tile t holds local members [t*TW, (t+1)*TW) of every observer row,
//   rows contiguous. One tile of the narrow table is N*TW*2 bytes (8 MiB at
//   N=65,536, TW=64): the round kernel sweeps tile by tile, so its own-row
//   streams are sequential and every peer gather of a tile stays inside
//   that slice. A (tile, row) SEGMENT is TW cells; a CHUNK is 8 consecutive
//   cells (one 16-B lane load).
//   A cell's meaning is (x, ts, flag): x >= 0 present with heartbeat x (full
//   int32 range, Go's HeartbeatCount, master/master.go:18), -1 absent, -2
//   tombstone; ts its exact UpdateTime tick (present / tombstone); flag (on
//   present cells) = the row's process detects the member in the round the
//   buffer is for (SPEC §2 step 4: x > 1, member != observer,
//   ts < r - T_fail), decided when the cell is written, so neither the row
//   nor the peers reading it as a snapshot re-derive it.
//   hn[2]  uint16  double-buffered NARROW table, where the round streams;
//                  buffer b is "for" round r (its ages count to r):
//                    present    H<<15 | off<<5 | age   off = x - base 0..1022,
//                                                      age = r - ts 0..31 exact
//                    tombstone  0xFFE0 | age           age 0..30 (tsa =
//                                                      T_cleanup + 1: "tsa or
//                                                      more")
//                    absent     0xFFFF
//                  Visible (present, unflagged) cells are the non-negative
//                  int16 values and compare like their heartbeats, so a
//                  snapshot merge is a packed 16-bit max.
//                  A segment that a narrow code cannot hold (x outside
//                  [base, base + 1022], age past the field, a future ts) is
//                  WIDE: cell 0 of each of its chunks holds GH_N_WIDE and
//                  cells 1, 2 the segment's slot in the buffer's wide arena;
//                  the segment of a stopped (crashed / left) row holds
//                  GH_N_FROZEN in every cell: its exact cells are in the
//                  frozen store, identical for both buffers (the round never
//                  touches a stopped row).
//   base[2] int32  per local column: base of buf's narrow cells. The round
//                  sets base[next][c] = (member c's own heartbeat) - GH_BASE_LAG
//                  (k_base), so every view of c within GH_BASE_LAG rounds of
//                  its own counter is narrow.
//   wide arena (per buffer b): slot s holds a segment's TW cells: wh[b] x,
//            wt[b] exact ts, wf[b] flags (one byte per chunk, bit j = cell j).
//            wn[b] = slots in use; the round resets the arena of the buffer
//            it writes (nothing of a running row survives a round in it).
//   frozen store: fzh / fzt [slot][ld] exact x / ts of stopped rows, slot =
//            frow[i] (-1 for running rows); host-managed (events stop and
//            restart rows between rounds).
//   pl[2]  uint32  SENDER SNAPSHOT PLANE beside each narrow buffer, 4 bits per
//                  cell in the narrow table's tiled order: word gh_cell(i, c)
//                  >> 3 holds cells c..c+7 of row i, cell c+2j in bits 4j..
//                  4j+3 and cell c+2j+1 in bits 16+4j.. (one field per 16-bit
//                  half, so packed 16-bit min/shift work on it). The code is
//                  what row i contributes as a sender in the round buffer b is
//                  for (visible cells, +1 on the diagonal), as u = GH_P_REF +
//                  1 - offset in base[b]'s frame:
//                    0      unknown (offset above GH_P_REF, wide segment)
//                    1..13  visible, offset = GH_P_REF + 1 - code exactly
//                    14     visible, offset below GH_P_REF - 12
//                    15     not in the snapshot (absent, tombstone, flagged)
//                  so the min over senders is the freshest entry, and any
//                  unknown sender shows as a 0. Written by every round kernel
//                  for the segments it writes (pull mode, 3 <= k <= 4, N >=
//                  GH_PLANE_MIN_N); read by
//                  k_round's lean variant, whose sender gathers become one 128-B
//                  line per 256 members at TW = 256. A wave falls back to the
//                  16-bit gathers when a min is 0 or 14. Every writer of a
//                  chunk keeps its plane word (gh_put8, gh_clearflags8; a
//                  stopped row's words are 0); pvalid[b] = 0 after whole-table
//                  rewrites (imports, fill) and the list-order quirk pass.
//   a4[2]  uint32  4-BIT TIER beside each narrow buffer (tiered engines: plane
//                  mode, column layout): the AGE plane, one nibble per cell in
//                  the sender plane's word and nibble order (word gh_cell(i,
//                  c) >> 3). Together with the sender plane pl[b] it IS the
//                  table while m8[b] = 1: the cell's plane code u (0..15, see
//                  pl) and its age a. A chunk whose age word has a zero cell-0
//                  nibble is ESCAPED: its cells are hn[b]'s 16-bit codes (its
//                  plane word is their plane_word, as for any chunk). Any
//                  other chunk holds only
//                    visible cells  u = GH_P_REF + 1 - offset (exact, 2..13;
//                                   on the row's own member, u = GH_P_REF -
//                                   offset, 1..12: the plane's diagonal code)
//                                   with age 1..15
//                    absent cells   u = 15, age nibble 15
//                    tombstones     u = 15, age nibble s = 1..14: age toff + s
//                                   (GH_TIER_TOMB; toff = gh_tier_toff(T_cleanup))
//                  so the plane word a round writes for its senders is the
//                  row's own lag code as well: the steady state streams one
//                  nibble of lag and one of age per cell each way, and the
//                  senders gather the same lag nibbles. Flags, tombstones,
//                  wide and frozen markers, lags or ages outside the window
//                  keep their 16-bit chunk (escaped). m8[b] = 0: hn[b] alone
//                  holds the buffer (a4[b] is ignored, except that stopped
//                  rows' chunks are escaped in both buffers at all times).
//                  The round that writes buffer b picks its tier (k_base: the
//                  lean variants write tier chunks); every other reader and
//                  writer goes through gh_ld16 / gh_put8 / gh_st16, which
//                  follow m8.
//   tsa = T_cleanup + 1 when T_cleanup < 30: a tombstone's age is only ever
//            compared with T_cleanup (cleanFailList, slave/slave.go:490), so
//            every age past T_cleanup decides the same; tombstones saturate
//            at tsa and the exported ts of an older tombstone is round + 1 -
//            tsa (SPEC §1; the oracle exports the same). A row under the <4
//            guard (:504-509) never cleans, so its tombstones age without
//            bound: saturated, they stop changing and the row goes quiet.
//   Local columns are padded to ld (multiple of 8*TW and 256); padding cells
//   stay absent.
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

#define GH_NO_SHADOW ((int32_t)0x80808080)  // no D7 shadow entry (GhDev.shadow; a byte fill of 0x80)
#define GH_N_ABSENT 0xFFFFu                // narrow absent
#define GH_N_TOMB 0xFFE0u                  // narrow tombstone | age
#define GH_N_WIDE 0x7FFFu                  // chunk marker of a wide segment (cells 1, 2: arena slot)
#define GH_N_FROZEN 0x7FFEu                // every cell of a stopped row (frozen store)
#define GH_N_OFFMAX 1022                   // largest narrow heartbeat offset
#define GH_N_AGEMAX 31                     // largest narrow age of a present cell
#define GH_N_TAGEMAX 30                    // largest narrow age of a tombstone (saturates at GhDev.tsa)
#define GH_TSAT_T 30                       // tsat = T_cleanup < GH_TSAT_T
#define GH_BASE_LAG 1000                   // base = own heartbeat - GH_BASE_LAG
#define GH_P_REF (GH_BASE_LAG + 2)         // plane: an active member's own snapshot offset
#define GH_P_UNK 0u                        // plane: unknown (read the narrow table)
#define GH_P_OLD 14u                       // plane: visible, offset below GH_P_REF - 12
#define GH_P_NONE 15u                      // plane: not in the snapshot
#define GH_C8_REF (GH_BASE_LAG + 1)        // 4-bit tier: offset of lag l = 0 (an active member's own cell)
#define GH_PAD 256               // column padding granule (ld % 256 == 0)
#ifndef GH_WG_CELLS
#define GH_WG_CELLS 16384        // round kernel: cells per workgroup tile (rows = GH_WG_CELLS / TW)
#endif
#ifndef GH_WG_ROWS_WIDE
#define GH_WG_ROWS_WIDE 256      // round kernel: rows per workgroup at TW >= 128
#endif
#ifndef GH_NIB_CPL
#define GH_NIB_CPL 16           // nibble path: cells per lane (8, 16, 32: 4-, 8-, 16-B lane accesses; 16 measured best)
#endif
#define GH_JOB_CPL 16           // a lane job covers 16 cells (a 32-cell lane of the nibble path writes two)
#ifndef GH_NIB_SPLIT
#define GH_NIB_SPLIT 0          // nibble path, 16-cell lanes, 256-member tiles: the sender gathers split over
                                // lane halves (round.hip round_block_nib SPL; parity green, measured slower)
#endif
#ifndef GH_NIB_SPLIT_ROWS
#define GH_NIB_SPLIT_ROWS 0     // the same for the row layout's nibble path (IN 4)
#endif
#ifndef GH_NIB_RS
#define GH_NIB_RS 1             // nibble path: row steps per iteration (1 measured best at CPL 8 and 16)
#endif
#ifndef GH_NIB_WAVES
#define GH_NIB_WAVES 1          // nibble path: min waves per SIMD it is compiled for (1: the compiler picks)
#endif
#ifndef GH_RMV_WAVES
#define GH_RMV_WAVES 1          // k_round IN 7 (IN 6 on a full grid): min waves per SIMD (1: the compiler picks)
#endif
#ifndef GH_RMV_FULL7
#define GH_RMV_FULL7 1          // 0: the host's full-grid REMOVE launch is IN 6 with its block loop (A/B build)
#endif
// nibble path cache policies (gfx950 buffer aux bits: 1 sc0, 2 nt, 16 sc1):
// the own age words (read once), the own lag words (also gathered by the
// tile's receivers), the sender gathers, and the stores of both planes
#ifndef GH_NIB_AGE_AUX
#define GH_NIB_AGE_AUX 2
#endif
#ifndef GH_NIB_OWN_AUX
#define GH_NIB_OWN_AUX 0
#endif
#ifndef GH_NIB_GAT_AUX
#define GH_NIB_GAT_AUX 0
#endif
#ifndef GH_NIB_ST_AUX
#define GH_NIB_ST_AUX 18  // sc1 | nt: the next round's lines leave the XCD's L2 instead of displacing this
                          // round's sender lines (2, nt, keeps them: 2.08 against 2.04 ms, profiles/r05_s32_*)
#endif
#ifndef GH_JOBF_WAVES
#define GH_JOBF_WAVES 3         // the flat lane-job kernel (k_round_jobs_flat): at 4 its rule spilled
#endif
#ifndef GH_JOB_WAVES
#define GH_JOB_WAVES 4          // lane-job kernel: min waves per SIMD it is compiled for (A/B: 4 beats 3 and 5)
#endif
#ifndef GH_TIER_TOMB
#define GH_TIER_TOMB 1          // 4-bit tier: tombstones in their last 14 ages before release are tier cells
#endif
#ifndef GH_TIER_TOMB_GATE
#define GH_TIER_TOMB_GATE 1     // nibble path: the tombstone rule only in waves whose own cells include code 15
#endif
#ifndef GH_STORM_WAVES
#define GH_STORM_WAVES 5         // storm variant: waves per SIMD it is compiled for (96 VGPRs, SGPR spills only)
#endif
#define GH_MAXK 8                // max pull fanout
#define GH_JOB_CAP 512           // nibble path: lane jobs per wave (half of its lanes at 16 cells per lane); beyond: whole segments to the slow list
#define GH_REDO_CAP 65536        // lane jobs per round whose segment must go wide (beyond: the engine state is lost, GH_ENOMEM)
#define GH_DLIST_MAX 1024        // local |D| above which undecided rows are recounted in full
#define GH_TW_DEFAULT 64         // default tile width (members per tile)
#define GH_TW_PLANE 256          // default tile width with the sender plane (pull, 3 <= k <= 4)
#define GH_PLANE_MIN_N 16384     // the sender plane from this many members on
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
  int32_t rowlay;   // GH_LAYOUT_ROWS
  int64_t row0, nrows;  // rows this engine owns (column layout: 0, n)
  int64_t nslots;   // table rows per tile: the owned rows (column layout: n)
  int32_t *rslot;   // row layout: [n] table slot of a global row, -1 = not held
  uint16_t *gcodes; // row layout: ghost rows' narrow codes [gcap][ld], row-major (null: no ghosts)
  uint32_t *gplane; // ... their sender plane words [gcap][ld / 8] (null without the plane)
  int64_t gcap;     // ghost rows the ghost table holds
  int32_t *pvf;     // row layout: [n][k] validity of each receiver's draws (summed over shards)
  // row layout, G > 1: per local column c REMOVE'd with a single detector j
  // (D_{r-1}: det_cnt == 1, det_min == j; SPEC §2 step 1), j's merge
  // candidate for c -- its exact heartbeat when present and unflagged, else
  // -1 -- from j's owner, max-allreduced (k_sole_vals). j is the only sender
  // that still carries c, so a lane job of a REMOVE'd column reads this
  // instead of a ghost sender's 16-bit codes (which then need not travel).
  int32_t *soleval;
  uint8_t *pvb;     // column layout, G > 1, pull: [G * ncs] per receiver the validity bits of its k draws
                    // (its column's owner decides them; allgathered, then every shard rebuilds every inbox)
  uint16_t *hn[2];  // narrow double buffer
  uint32_t *a4[2];  // 4-bit tier: age plane per buffer (null: tier off); with pl[b] it holds buffer b
  int32_t *m8;      // [0..1] buffer b is in the 4-bit tier; [2] this round switches the next buffer's tier;
                    // [3] escaped chunks the round wrote; [4] the round variant that ran (gh_tier_info)
  uint32_t *pl[2];  // sender snapshot plane per buffer (null: plane off)
  int32_t *pvalid;  // [2]: plane of buffer b written by the round that wrote b
  int32_t *pfb;     // waves of the last round that gathered 16-bit codes with a valid plane
  // quiet rows (by round parity r & 1): stab[r & 1][i] = row i was inactive
  // in round r - 1 and none of its segments changed (k_active_post sets it
  // for the inactive rows, k_round / k_round_slow clear it). Round r skips
  // such a row when it is still inactive with no senders, no REMOVE is
  // pending and no base of the tile moved: its output equals its input,
  // which the next buffer already holds (written two rounds ago, unchanged
  // one round ago). A collapsed cluster stops rewriting its tables.
  uint8_t *stab[2];
  int32_t *nquiet;  // row segments the last round skipped as quiet
  // one engine, column layout: aq[0] != 0 when a running row of this round
  // is not a quiet candidate or a column base moved (k_peers_pull /
  // k_inbox_fill, base_col; reset by k_finish); else k_round has nothing to
  // read or write and every variant returns at once
  int32_t *aq;
  // one tiered engine, column layout: each row's nibble-path record, written
  // by k_peers_pull: nmeta[i] (alive | active << 1 | senders << 2 | quiet
  // candidate << 30) and nsnd[4 i .. 4 i + 3] (the senders, unused slots the
  // row itself), so a nibble workgroup stages its rows with two coalesced
  // loads per row instead of five scattered ones per (row, slot)
  int32_t *nmeta, *nsnd;
  // a tiered column-layout engine: this round's base move per 8-column
  // chunk as one nibble word (dnw, the nibble path's order) and whether any
  // of its columns moves outside 0..15 (dbad), written by base_col
  uint32_t *dnw;
  uint8_t *dbad;
  // MemberList order (GH_ORDER_APPEND, order.hip; null under GH_ORDER_ID).
  // Generation g (the host's lcur) of row i: the list is lord[lsel[g][i]] +
  // i * ld (member at each position), llen[g][i] entries, the row's own
  // member at lself[g][i] (-1 not listed). Two buffers per row: a rewrite
  // goes to the other one while the senders read the current one.
  int32_t *lord[2], *llen[2], *lself[2];
  uint8_t *lsel[2];
  int32_t *lchg;    // row shards: [n] rows whose list this shard rebuilt (copied to every shard, then cleared)
  int32_t *base[2]; // [ld] narrow base per buffer
  // wide arena per buffer: [wcap][tw] x / exact ts, [wcap][tw/8] flag bytes
  int32_t *wh[2], *wt[2];
  uint8_t *wf[2];
  int32_t *wn;      // [2] slots in use per buffer
  int64_t wcap;     // slots per buffer
  int32_t *err;     // device-side error (GH_ENOMEM: arena full; GH_ERANGE), 0 = none
  // frozen store of stopped rows: [fzcap][ld] exact x / ts; frow[i] = slot or -1
  int32_t *frow, *fzh, *fzt;
  int32_t tsa;      // tombstone ages saturate here: T_cleanup + 1 when T_cleanup < GH_TSAT_T, else 0 (none; SPEC §1)
  int32_t toff;     // 4-bit tier: a tombstone of age toff + s is the tier cell (15, s), s = 1..14 (gh_tier_toff)
  int32_t *colq;    // [ld] scratch: per local column event index / merged value
  int64_t *slow;    // [ntiles * n] round: segments for k_round_slow, tile << 32 | row
  int32_t *slow_n;  // their count
  // nibble path LANE JOBS (tiered engines): a lane of an active row whose
  // cells leave the tier (escaped input, flag, tombstone, age or code out of
  // the window), hold a REMOVE'd member, a base move outside 0..15, an
  // unknown or old sender code, or the row's own member needing the per-cell
  // rule goes to k_round_jobs instead of sending its whole segment to the
  // slow list. Wave w of nibble workgroup b writes its jobs to
  // jobs[2 (4 b + w) * GH_JOB_CAP ..], two uint4 each (row, tile << 8 |
  // lane, the minimum plane words; the lane's own lag words and age words)
  // and their count to jobn[4 b + w], with no atomics. Results that need the
  // wide arena go to redo (the redo pass redo_all in k_round_slow, the first uint4).
  uint4 *jobs;
  int32_t *jobn;    // [4 * nibble workgroups]
  int32_t *njobs;   // [0] jobs of the last round (k_base's variant choice), [1] redo entries, [2] jobs of the round before,
                    // [3] nibble workgroups listed in jlist this round
  int32_t *jlist;   // [jobw] the nibble workgroups that wrote lane jobs this round (k_round_jobs walks only these)
  uint4 *redo;      // [GH_REDO_CAP] lane jobs whose cells need a wide segment
  int64_t jobw;     // nibble workgroups (jobn entries / 4)
  int32_t *mode;    // k_round variant of the round: 0 lean, 1 storm (k_base)
  int32_t *nstorm;  // storm variant: segments holding flagged or tombstoned cells
  int32_t *nflag;   // [2]: segments written into buffer b holding flagged cells (quirk pre-pass gate)
  uint8_t *alive, *active, *det_any, *und;
  int32_t *cntl, *cntg;  // [n + 8]: per-row present counts (local / allreduced), [n] = |D|, [n + 1] = nflag[cur]
  int32_t *post;         // [n]: post-REMOVE present counts of undecided rows (allreduced)
  int32_t *det_cnt[2], *det_min[2];
  uint32_t *dbits;
  uint32_t *sbits;  // [ld/32 + 2]: the columns of dbits with exactly one detector (k_finish)
  // GH_REMOVE_LIST (the reference's REMOVE recipients, slave/slave.go:344;
  // one engine, member-ID list order): rcv[b] holds, per column c of the
  // REMOVE set of parity b, bit j of word c * nw + j / 32 = row j receives
  // REMOVE(c). Built after each detection round (remove.hip) from column
  // bitmaps over the rows that ran the sweep: cdet (the row detected the
  // member), csurv (listed and not detected), clst (listed; self excluded)
  // and their counts ccnt [0, ld) survivors, [ld, 2 ld) listed, [2 ld] rows
  int32_t rlist;
  int64_t nw;       // words of a column bitmap over the rows, ceil(n / 32)
  uint32_t *rcv[2];
  uint32_t *cdet, *csurv, *clst;
  int32_t *ccnt;
  int32_t *dlist;
  // SPEC D7 (slave/slave.go:228-230, 250-255, 276-286): a JOIN of a member the
  // introducer holds tombstoned appends it to MemberList while the
  // RecentFailList entry stays. shadow[c] (local column) = that entry's ts
  // beside the introducer's present member c, GH_NO_SHADOW when none;
  // nshadow[0] = entries held. A LEAVE, REMOVE or detection of c at the
  // introducer leaves the old entry (its ts, no new tombstone counted);
  // cleanFailList releases it like any tombstone. The introducer's segments
  // run the per-cell rule (k_round_slow) while any entry may exist.
  int32_t *shadow, *nshadow;
  // timing (gh_set_timing, tmode 1): vlog[q] = the host variant number
  // (launch_round's 0..4) of the k_round launch that ran in round q of the
  // current gh_step call; null when not timing
  int32_t* vlog;
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
  // files, sharded by file ID (master/master.go:74-175 is per
  // file): file f lives on shard f % fsh, at local slot f / fsh; fcap = this
  // shard's slots (ceil(max_files / fsh)). One engine: fsh = 1, frank = 0.
  int64_t fcap;
  int32_t fsh, frank;
  int32_t *rep, *ver, *fts;
  uint32_t *draws;
  int32_t *cand, *ncand;
  int32_t *io_a, *io_b, *io_c, *io_d;  // per-call scratch (files, outputs)
  gh_plan_entry *plan;
  int32_t *nplan;
  int64_t io_cap;
};

// ---- cells -----------------------------------------------------------
// One cell: x (>= 0 heartbeat, GH_ABSENT, GH_TOMBSTONE), exact ts (present
// and tombstone; 0 for absent), flag (present cells).
struct GhCell {
  int32_t x, ts;
  bool f;
};
__host__ __device__ __forceinline__ GhCell gh_absent() { return GhCell{GH_ABSENT, 0, false}; }

// The flag a present cell (x, ts) of member cg in row i gets when written for
// round r: a step-4 candidate (slave/slave.go:468-470).
__host__ __device__ __forceinline__ bool gh_flag_for(int32_t x, int32_t ts, int64_t cg, int64_t i, int32_t r,
                                                     int32_t t_fail) {
  return x > 1 && cg != i && (int64_t)ts < (int64_t)r - t_fail;
}

// File f's local slot on this shard, or -1 when another shard holds it.
__host__ __device__ __forceinline__ int64_t gh_fslot(const GhDev& d, int64_t f) {
  return (f % d.fsh) == d.frank ? f / d.fsh : -1;
}

// Linear index of cell (table slot s, LOCAL member column c) in the tiled layout.
__host__ __device__ __forceinline__ int64_t gh_cell_slot(const GhDev& d, int64_t s, int64_t c) {
  return (c >> d.lgtw) * d.tstride + (s << d.lgtw) + (c & (d.tw - 1));
}
// Table slot of global row i (device; the row must be held: owned or ghost).
__device__ __forceinline__ int64_t gh_slot(const GhDev& d, int64_t i) { return d.rslot ? d.rslot[i] : i; }
// Row i is one this engine owns (and rounds / events write).
__host__ __device__ __forceinline__ bool gh_owned(const GhDev& d, int64_t i) {
  return i >= d.row0 && i < d.row0 + d.nrows;
}
// Linear index of cell (observer i, LOCAL member column c) in the tiled layout.
__device__ __forceinline__ int64_t gh_cell(const GhDev& d, int64_t i, int64_t c) {
  return gh_cell_slot(d, gh_slot(d, i), c);
}
// Arena index of cell (slot s, local column c) (the segment's column offset).
__host__ __device__ __forceinline__ int64_t gh_wcell(const GhDev& d, int64_t s, int64_t c) {
  return (s << d.lgtw) + (c & (d.tw - 1));
}

// ---- packed 16-bit (two narrow cells per dword) ------------------------
typedef uint32_t v4u __attribute__((ext_vector_type(4)));
typedef short s16x2 __attribute__((ext_vector_type(2)));
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ s16x2 as_s(uint32_t x) { return __builtin_bit_cast(s16x2, x); }
__device__ __forceinline__ u16x2 as_us(uint32_t x) { return __builtin_bit_cast(u16x2, x); }
__device__ __forceinline__ uint32_t as_u(s16x2 x) { return __builtin_bit_cast(uint32_t, x); }
__device__ __forceinline__ uint32_t as_u(u16x2 x) { return __builtin_bit_cast(uint32_t, x); }
__device__ __forceinline__ uint32_t pk_max_i16(uint32_t a, uint32_t b) {
  return as_u(__builtin_elementwise_max(as_s(a), as_s(b)));
}
__device__ __forceinline__ uint32_t pk_subs_i16(uint32_t a, uint32_t b) {  // saturating a - b
  return as_u(__builtin_elementwise_sub_sat(as_s(a), as_s(b)));
}
__device__ __forceinline__ uint32_t pk_adds_u16(uint32_t a, uint32_t b) {  // saturating a + b
  return as_u(__builtin_elementwise_add_sat(as_us(a), as_us(b)));
}
__device__ __forceinline__ uint32_t pk_add_u16(uint32_t a, uint32_t b) { return as_u(as_us(a) + as_us(b)); }
__device__ __forceinline__ uint32_t pk_sub_u16(uint32_t a, uint32_t b) { return as_u(as_us(a) - as_us(b)); }
// 0xFFFF per negative half. Opaque to the compiler: as a plain shift its
// result feeds selects that get rewritten into per-half compares and
// v_cndmask (7 instructions where and/or take 2).
__device__ __forceinline__ uint32_t pk_sra15(uint32_t a) {
  uint32_t r;
  asm("v_pk_ashrrev_i16 %0, 15, %1 op_sel_hi:[0,1]" : "=v"(r) : "v"(a));  // both halves by 15
  return r;
}
__device__ __forceinline__ uint32_t pk_min_u16(uint32_t a, uint32_t b) {
  return as_u(__builtin_elementwise_min(as_us(a), as_us(b)));
}
// 0xFFFF in each half that is zero
__device__ __forceinline__ uint32_t pk_zero_mask(uint32_t a) {
  return pk_sub_u16(pk_min_u16(a, 0x00010001u), 0x00010001u);
}
__device__ __forceinline__ uint32_t pk_lshr16(uint32_t a, int k) { return as_u(as_us(a) >> (unsigned short)k); }
__device__ __forceinline__ uint32_t pk_shl16(uint32_t a, int k) { return as_u(as_us(a) << (unsigned short)k); }

// ---- sender snapshot plane (pl) ---------------------------------------------
// The plane word of 8 written narrow codes o (an all-narrow chunk); jd = the
// row's own member in the chunk (0..7) or -1: its snapshot entry carries
// hb + 1 (the heartbeat the row sends with next round).
__device__ __forceinline__ uint32_t plane_word(const v4u& o, int jd) {
  uint32_t wd = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const uint32_t y = o[j];
    // u = REF + 1 - offset, clamped to [0, 14]; not visible (bit 15): 15
    const uint32_t u = pk_sub_u16((uint32_t)(GH_P_REF + 1) * 0x10001u, pk_lshr16(y, 5));
    uint32_t code = pk_min_u16(pk_max_i16(u, 0u), GH_P_OLD * 0x10001u);
    code |= pk_sra15(y) & (GH_P_NONE * 0x10001u);
    wd |= code << (4 * j);
  }
  if (jd >= 0) {
    // offset + 1 on the diagonal: an exact code moves one down (1 = at the
    // reference becomes unknown); unknown, old and not-visible stay
    const int pos = 4 * (jd >> 1) + 16 * (jd & 1);
    const uint32_t c = (wd >> pos) & 0xFu;
    const uint32_t c2 = (c >= 2u && c <= 13u) ? c - 1u : (c == 1u ? 0u : c);
    wd = (wd & ~(0xFu << pos)) | (c2 << pos);
  }
  return wd;
}
// ---- 4-bit tier (a4 + pl) -------------------------------------------------
// Nibble of cell j (0..7) of a chunk in the plane's order: cell 2m in bits
// 4m, cell 2m + 1 in bits 16 + 4m (one field per 16-bit half of pair m).
__host__ __device__ __forceinline__ int gh_nib(int j) { return 4 * (j >> 1) + 16 * (j & 1); }
// the escape test of a tier chunk's age word
__host__ __device__ __forceinline__ bool gh_t4_esc(uint32_t age) { return (age & 0xFu) == 0u; }
// Tombstone age offset of the 4-bit tier for T_cleanup tc: the tier holds a
// tombstone's last 14 ages before its release, tc - 12 .. tc + 1, as age
// nibbles 1..14, so the age the release reads (tc + 1) is always nibble 14;
// GH_TOFF_NONE (no tombstone in the tier) when tc + 1 passes the 16-bit
// tombstone's 30 (GH_N_TAGEMAX)
#define GH_TOFF_NONE (-128)
__host__ __device__ __forceinline__ int gh_tier_toff(int tc) {
  return !GH_TIER_TOMB || tc < 0 || tc + 1 > 30 ? GH_TOFF_NONE : tc - 13;
}
// The 16-bit codes of a tier chunk (not escaped): lag plane word u, age word
// a; jd = the row's own member in the chunk (0..7, its code is the plane's
// diagonal code) or -1; toff = GhDev::toff. Invariant: a code-15 cell with an
// age nibble 1..14 (a tier tombstone) is written only when toff !=
// GH_TOFF_NONE, and then toff + nibble lies in 0..30 (gh_tier_toff); the
// decode relies on it, gh_debug_raw reports a cell that breaks it.
__device__ __forceinline__ v4u c4_dec(uint32_t u, uint32_t a, int jd, int toff) {
  v4u o;
  const uint32_t TO = (uint32_t)(toff & 0xFFFF) * 0x00010001u;  // (modulo 2^16 per half)
#pragma unroll
  for (int m = 0; m < 4; ++m) {
    const uint32_t U = (u >> (4 * m)) & 0x000F000Fu, A = (a >> (4 * m)) & 0x000F000Fu;
    // offset = GH_P_REF + 1 - u; no borrow crosses the halves (u <= 15)
    const uint32_t code = ((uint32_t)((GH_P_REF + 1) << 5) * 0x10001u - (U << 5)) | A;
    const uint32_t nv = pk_sub_u16(0u, ((U + 0x00010001u) >> 4) & 0x00010001u);  // 0xFFFF per half with u = 15
    // u = 15: absent (age nibble 15: 0xFFFF) or a tombstone of age toff + A
    const uint32_t ab = pk_zero_mask(A ^ 0x000F000Fu);
    const uint32_t tb = 0xFFE0FFE0u | (pk_add_u16(A, TO) & ~ab) | (0x001F001Fu & ab);
    o[m] = (code & ~nv) | (tb & nv);
  }
  if (jd >= 0) {  // the diagonal's code is one offset lower: offset = GH_P_REF - u
    const int m = jd >> 1, sh = 16 * (jd & 1);
#pragma unroll
    for (int q = 0; q < 4; ++q)
      if (q == m && ((o[q] >> sh) & 0x8000u) == 0u) o[q] -= 0x20u << sh;
  }
  return o;
}
// The age word of 16-bit codes o whose plane word is u = plane_word(o, jd),
// when the chunk has a tier encoding (every cell absent, visible with an
// exact plane code in the window and age 1..15, or a tombstone of age
// toff + 1..14); else false.
__device__ __forceinline__ bool c4_enc(const v4u& o, int jd, uint32_t& age, int toff) {
  uint32_t a = 0, bad = 0;
  const uint32_t TO = (uint32_t)(toff & 0xFFFF) * 0x00010001u;  // (modulo 2^16 per half)
  const uint32_t tno = toff == GH_TOFF_NONE ? 0x80008000u : 0u;  // no tombstone in the tier
#pragma unroll
  for (int m = 0; m < 4; ++m) {
    const uint32_t y = o[m];
    const uint32_t ab = pk_zero_mask(pk_add_u16(y, 0x00010001u));  // absent halves
    const uint32_t ta = pk_zero_mask(pk_lshr16(pk_add_u16(y, 0x00200020u), 5));  // tombstone or absent
    // raw plane code GH_P_REF + 1 - offset in 2..13 (the diagonal's 1..12 is
    // the same range before its - 1); flagged, tombstone and marker codes
    // have bit 15 or an offset far above the window
    const uint32_t ur = pk_sub_u16((uint32_t)(GH_P_REF + 1) * 0x10001u, pk_lshr16(y, 5));
    const uint32_t ag = pk_sub_u16(y & 0x001F001Fu, TO & ta & ~ab);  // a tombstone's age - toff
    // visible halves: bit 15 of (y), (ur - 2), (13 - ur), (ag - 1), (15 - ag);
    // tombstones: (ag - 1), (14 - ag) (15 is the absent code)
    const uint32_t b = y | pk_sub_u16(ur, 0x00020002u) | pk_sub_u16(0x000D000Du, ur) | pk_sub_u16(ag, 0x00010001u) |
                       pk_sub_u16(0x000F000Fu, ag);
    const uint32_t bt = pk_sub_u16(ag, 0x00010001u) | pk_sub_u16(0x000E000Eu, ag) | tno;
    bad |= ((b & ~ta) | (bt & ta & ~ab)) & 0x80008000u;
    a |= ((ag | ab) & 0x000F000Fu) << (4 * m);  // absent: age nibble 15
  }
  (void)jd;
  age = a;
  return bad == 0;
}
#define GH_T4_ESC 0u  // the age word of an escaped chunk

// buffer buf is in the 4-bit tier
__device__ __forceinline__ bool gh_m8(const GhDev& d, int buf) { return d.a4[0] != nullptr && d.m8[buf] != 0; }
// own-member position of row i in the chunk at local column c: 0..7 or -1
__device__ __forceinline__ int gh_jd(const GhDev& d, int64_t i, int64_t c) {
  const int64_t jd = i - (d.col0 + c);
  return (uint64_t)jd < 8u ? (int)jd : -1;
}
// The 16-bit chunk of table slot s, local column c (c % 8 == 0) of buffer
// buf: its tier codes decoded, or hn's chunk when escaped or the buffer is
// 16-bit. jd: the row's own member in the chunk (gh_jd) or -1.
__device__ __forceinline__ uint4 gh_ld16s(const GhDev& d, int buf, int64_t s, int64_t c, int jd) {
  if (d.gcodes && s >= d.nrows)  // a ghost row (row layout: 16-bit, single-buffered)
    return *reinterpret_cast<const uint4*>(d.gcodes + (s - d.nrows) * d.ld + c);
  const int64_t cell = gh_cell_slot(d, s, c);
  if (gh_m8(d, buf)) {
    // both words at once (one memory latency, not two)
    const uint32_t a = d.a4[buf][cell >> 3], u = d.pl[buf][cell >> 3];
    if (!gh_t4_esc(a)) {
      const v4u w = c4_dec(u, a, jd, d.toff);
      return uint4{w[0], w[1], w[2], w[3]};
    }
  }
  return *reinterpret_cast<const uint4*>(d.hn[buf] + cell);
}
// ... of global row i (held by this engine)
__device__ __forceinline__ uint4 gh_ld16(const GhDev& d, int buf, int64_t i, int64_t c) {
  return gh_ld16s(d, buf, gh_slot(d, i), c, gh_jd(d, i, c));
}
// Stores the 16-bit chunk x (narrow codes or a marker) of row i, local
// column c of buffer buf whose plane word the caller writes (gh_put8): in the
// 4-bit tier as its age word when the chunk has a tier encoding (t4 =
// allowed), else escaped with x in hn.
__device__ __forceinline__ void gh_st16(const GhDev& d, int buf, int64_t i, int64_t c, const uint4& x, bool t4 = true) {
  const int64_t cell = gh_cell(d, i, c);
  if (gh_m8(d, buf)) {
    uint32_t a = 0;
    if (t4 && c4_enc(v4u{x.x, x.y, x.z, x.w}, gh_jd(d, i, c), a, d.toff)) {
      d.a4[buf][cell >> 3] = a;
      return;
    }
    d.a4[buf][cell >> 3] = GH_T4_ESC;
  }
  *reinterpret_cast<uint4*>(d.hn[buf] + cell) = x;
}

// ---- narrow codes ---------------------------------------------------------
// Decodes a narrow (non-marker) code of a column with base b in a buffer for
// round r.
__host__ __device__ __forceinline__ GhCell gh_dec16(uint32_t h, int32_t b, int32_t r) {
  if (h == GH_N_ABSENT) return gh_absent();
  const int a = h & 31, off = (h >> 5) & 1023;
  if (off == 1023) return GhCell{GH_TOMBSTONE, r - a, false};
  return GhCell{b + off, r - a, (h >> 15) != 0};
}
// Narrow code of cell v in a buffer for round r with column base b; fit &= it
// has one. tsa: tombstone ages past tsa saturate (SPEC §1; 0: none).
__host__ __device__ __forceinline__ uint32_t gh_enc16(const GhCell& v, int32_t b, int32_t r, int32_t tsa, bool& fit) {
  if (v.x == GH_ABSENT) return GH_N_ABSENT;
  int64_t a = (int64_t)r - v.ts;
  if (v.x < 0) {
    if (tsa && a > tsa) a = tsa;
    fit &= a >= 0 && a <= GH_N_TAGEMAX;
    return GH_N_TOMB | (uint32_t)(a & 31);
  }
  const int64_t off = (int64_t)v.x - b;
  fit &= off >= 0 && off <= GH_N_OFFMAX && a >= 0 && a <= GH_N_AGEMAX;
  return (v.f ? 0x8000u : 0u) | ((uint32_t)(off & 1023) << 5) | (uint32_t)(a & 31);
}
// The 16-B chunk of a wide segment (slot s): marker, slot, markers.
__host__ __device__ __forceinline__ uint4 gh_wide_chunk(int64_t s) {
  const uint32_t lo = (uint32_t)s & 0xFFFFu, hi = ((uint32_t)s >> 16) & 0xFFFFu;
  const uint32_t m = GH_N_WIDE | (GH_N_WIDE << 16);
  return uint4{GH_N_WIDE | (lo << 16), hi | (GH_N_WIDE << 16), m, m};
}
__host__ __device__ __forceinline__ int64_t gh_wide_slot(uint32_t w0, uint32_t w1) {
  return (int64_t)((w0 >> 16) | ((w1 & 0xFFFFu) << 16));
}

// The 8 cells (i, c..c+7), c % 8 == 0, of buffer buf (for round r); the
// chunk's narrow codes are x (already loaded).
// A marker whose slot is out of range (never written by a correct engine)
// decodes as absent rather than reading outside the arena / store.
__device__ __forceinline__ void gh_dec8(const GhDev& d, int buf, int64_t i, int64_t c, int32_t r, const uint4& x,
                                        GhCell out[8]) {
  const uint32_t h0 = x.x & 0xFFFFu;
  if ((h0 == GH_N_WIDE && gh_wide_slot(x.x, x.y) >= d.wcap) || (h0 == GH_N_FROZEN && d.frow[i] < 0)) {
#pragma unroll
    for (int j = 0; j < 8; ++j) out[j] = gh_absent();
  } else if (h0 == GH_N_WIDE) {
    const int64_t w = gh_wcell(d, gh_wide_slot(x.x, x.y), c);
    const int4 a = *reinterpret_cast<const int4*>(d.wh[buf] + w);
    const int4 b = *reinterpret_cast<const int4*>(d.wh[buf] + w + 4);
    const int4 ta = *reinterpret_cast<const int4*>(d.wt[buf] + w);
    const int4 tb = *reinterpret_cast<const int4*>(d.wt[buf] + w + 4);
    const uint32_t fl = d.wf[buf][w >> 3];
    const int32_t xs[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
    const int32_t tss[8] = {ta.x, ta.y, ta.z, ta.w, tb.x, tb.y, tb.z, tb.w};
#pragma unroll
    for (int j = 0; j < 8; ++j) out[j] = GhCell{xs[j], xs[j] == GH_ABSENT ? 0 : tss[j], ((fl >> j) & 1u) != 0};
  } else if (h0 == GH_N_FROZEN) {
    const int64_t w = (int64_t)d.frow[i] * d.ld + c;
    const int4 a = *reinterpret_cast<const int4*>(d.fzh + w);
    const int4 b = *reinterpret_cast<const int4*>(d.fzh + w + 4);
    const int4 ta = *reinterpret_cast<const int4*>(d.fzt + w);
    const int4 tb = *reinterpret_cast<const int4*>(d.fzt + w + 4);
    const int32_t xs[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
    const int32_t tss[8] = {ta.x, ta.y, ta.z, ta.w, tb.x, tb.y, tb.z, tb.w};
#pragma unroll
    for (int j = 0; j < 8; ++j) out[j] = GhCell{xs[j], xs[j] == GH_ABSENT ? 0 : tss[j], false};
  } else {
    const int32_t* bp = d.base[buf] + c;
    const uint32_t w[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
    for (int j = 0; j < 8; ++j) out[j] = gh_dec16((w[j >> 1] >> (16 * (j & 1))) & 0xFFFFu, bp[j], r);
  }
}
__device__ __forceinline__ void gh_get8(const GhDev& d, int buf, int64_t i, int64_t c, int32_t r, GhCell out[8]) {
  const uint4 x = gh_ld16(d, buf, i, c);
  gh_dec8(d, buf, i, c, r, x, out);
}

// Cell (i, local c) of buffer buf (for round r).
__device__ __forceinline__ GhCell gh_get(const GhDev& d, int buf, int64_t i, int64_t c, int32_t r) {
  const int64_t c8 = c & ~(int64_t)7;
  const int32_t b = d.base[buf][c];  // (issued beside the cell's loads)
  const uint4 hd = gh_ld16(d, buf, i, c8);
  const uint32_t h0 = hd.x & 0xFFFFu;
  if (h0 == GH_N_WIDE) {
    if (gh_wide_slot(hd.x, hd.y) >= d.wcap) return gh_absent();
    const int64_t w = gh_wcell(d, gh_wide_slot(hd.x, hd.y), c);
    const int32_t x = d.wh[buf][w];
    return GhCell{x, x == GH_ABSENT ? 0 : d.wt[buf][w], ((d.wf[buf][w >> 3] >> (c & 7)) & 1u) != 0};
  }
  if (h0 == GH_N_FROZEN) {
    if (d.frow[i] < 0) return gh_absent();
    const int64_t w = (int64_t)d.frow[i] * d.ld + c;
    const int32_t x = d.fzh[w];
    return GhCell{x, x == GH_ABSENT ? 0 : d.fzt[w], false};
  }
  const uint32_t hw[4] = {hd.x, hd.y, hd.z, hd.w};
  return gh_dec16((hw[(c & 7) >> 1] >> (16 * (c & 1))) & 0xFFFFu, b, r);
}

// Presence and flag bits of cells (i, c..c+7) of buffer buf (c % 8 == 0):
// bit j = present, bit 8 + j = present and flagged. Narrow codes answer
// directly (no base, no round).
// (x: the chunk's 16 B of narrow cells, loaded by the caller)
__device__ __forceinline__ uint32_t gh_pf8x(const GhDev& d, int buf, int64_t i, int64_t c, const uint4& x) {
  const uint32_t h0 = x.x & 0xFFFFu;
  uint32_t out = 0;
  if (h0 == GH_N_WIDE || h0 == GH_N_FROZEN) {
    GhCell v[8];
    gh_dec8(d, buf, i, c, 0, x, v);
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if (v[j].x >= 0) out |= (1u << j) | (v[j].f ? 1u << (8 + j) : 0u);
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
__device__ __forceinline__ uint32_t gh_pf8(const GhDev& d, int buf, int64_t i, int64_t c) {
  return gh_pf8x(d, buf, i, c, gh_ld16(d, buf, i, c));
}
// The present cells of a tier chunk (bit j = cell j) from its lag word
// alone: a code other than 15. A tier chunk holds no flag (a flagged cell is
// always escaped), so whole-table sweeps (the quirk pre-pass) need no decode.
__host__ __device__ __forceinline__ uint32_t gh_t4_present8(uint32_t lag) {
  const uint32_t e = ~lag;
  uint32_t t = e | (e >> 2);
  t = (t | (t >> 1)) & 0x11111111u;  // bit 0 of each nibble: the code is not 15
  uint32_t P = 0;
#pragma unroll
  for (int j = 0; j < 8; ++j) P |= ((t >> gh_nib(j)) & 1u) << j;  // nibble gh_nib(j) -> bit j
  return P;
}
// Clears the flag of present cells (i, c + j) for the bits j of m (c % 8 == 0).
// A stopped row has no flags.
__device__ __forceinline__ void gh_clearflags8(const GhDev& d, int buf, int64_t i, int64_t c, uint32_t m) {
  const int64_t cell = gh_cell(d, i, c);
  // a tier chunk holds no flag; an escaped one is hn's
  if (gh_m8(d, buf) && !gh_t4_esc(d.a4[buf][cell >> 3])) return;
  uint4* np = reinterpret_cast<uint4*>(d.hn[buf] + cell);
  uint4 x = *np;
  const uint32_t h0 = x.x & 0xFFFFu;
  if (h0 == GH_N_FROZEN) return;
  if (h0 == GH_N_WIDE) {
    if (gh_wide_slot(x.x, x.y) >= d.wcap) return;
    uint8_t* fp = d.wf[buf] + (gh_wcell(d, gh_wide_slot(x.x, x.y), c) >> 3);
    *fp = (uint8_t)(*fp & ~m);
    return;
  }
  uint32_t w[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
  for (int j = 0; j < 8; ++j)
    if ((m >> j) & 1u) w[j >> 1] &= ~(0x8000u << (16 * (j & 1)));
  *np = uint4{w[0], w[1], w[2], w[3]};
  if (d.pl[buf]) {  // cleared flags make cells visible to the row's peers
    const int64_t jd = i - (d.col0 + c);
    d.pl[buf][cell >> 3] = plane_word(v4u{w[0], w[1], w[2], w[3]}, (uint64_t)jd < 8u ? (int)jd : -1);
  }
}

// Writes 8 cells of one chunk (i, c..c+7) of buffer buf: narrow codes nx
// when the whole segment is narrow (narrow = the segment-wide decision),
// else the cells into arena slot `slot` and the chunk's marker.
__device__ __forceinline__ void gh_put8(const GhDev& d, int buf, int64_t i, int64_t c, bool narrow, const uint4& nx,
                                        int64_t slot, const GhCell v[8]) {
  const int64_t cell = gh_cell(d, i, c);
  // the chunk's sender plane word follows it (a wide chunk: unknown), so a
  // host write leaves the plane valid
  if (d.pl[buf]) {
    const int64_t jd = i - (d.col0 + c);
    d.pl[buf][cell >> 3] = narrow ? plane_word(v4u{nx.x, nx.y, nx.z, nx.w}, (uint64_t)jd < 8u ? (int)jd : -1) : 0u;
  }
  if (narrow) {
    gh_st16(d, buf, i, c, nx);
    return;
  }
  if (gh_m8(d, buf)) d.a4[buf][cell >> 3] = GH_T4_ESC;
  uint4* np = reinterpret_cast<uint4*>(d.hn[buf] + cell);
  const int64_t w = gh_wcell(d, slot, c);
  *reinterpret_cast<int4*>(d.wh[buf] + w) = int4{v[0].x, v[1].x, v[2].x, v[3].x};
  *reinterpret_cast<int4*>(d.wh[buf] + w + 4) = int4{v[4].x, v[5].x, v[6].x, v[7].x};
  *reinterpret_cast<int4*>(d.wt[buf] + w) = int4{v[0].ts, v[1].ts, v[2].ts, v[3].ts};
  *reinterpret_cast<int4*>(d.wt[buf] + w + 4) = int4{v[4].ts, v[5].ts, v[6].ts, v[7].ts};
  uint32_t fl = 0;
#pragma unroll
  for (int j = 0; j < 8; ++j) fl |= (v[j].x >= 0 && v[j].f) ? 1u << j : 0u;
  d.wf[buf][w >> 3] = (uint8_t)fl;
  *np = gh_wide_chunk(slot);
}
// Narrow codes of 8 cells for buffer buf (for round r); fit &= all have one.
__device__ __forceinline__ uint4 gh_enc8(const GhDev& d, int buf, int64_t c, int32_t r, const GhCell v[8], bool& fit) {
  const int32_t* bp = d.base[buf] + c;
  uint32_t w[4] = {0u, 0u, 0u, 0u};
#pragma unroll
  for (int j = 0; j < 8; ++j) w[j >> 1] |= gh_enc16(v[j], bp[j], r, d.tsa, fit) << (16 * (j & 1));
  return uint4{w[0], w[1], w[2], w[3]};
}
// A fresh arena slot of buffer buf (one lane per segment calls it); on
// overflow the engine's state is lost: err = GH_ENOMEM and -1.
__device__ __forceinline__ int64_t gh_wide_alloc(const GhDev& d, int buf) {
  const int64_t s = atomicAdd(&d.wn[buf], 1);
  if (s >= d.wcap) {
    atomicExch(d.err, GH_ENOMEM);
    return -1;
  }
  return s;
}

// The exported ts of a cell (SPEC §1): 0 for absent; a tombstone older than
// tsa = T_cleanup + 1 rounds (T_cleanup < 30) as tsa rounds old (r = the
// round the buffer is for).
__host__ __device__ __forceinline__ int32_t gh_export_ts(const GhCell& v, int32_t r, int32_t tsa) {
  if (v.x == GH_ABSENT) return 0;
  if (v.x == GH_TOMBSTONE && tsa && (int64_t)r - v.ts > tsa) return r - tsa;
  return v.ts;
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
  int32_t xmap;       // k_round block->tile map: 0 tile-major, 1 XCD-aware, 2 XCD-aware with odd rounds reversed (nibble path)
  int32_t tpw;        // k_round tiles per workgroup (1, 2, 4, 8)
  int32_t qgate;      // quirk pre-pass: 1 = return at once when cntg[n + 1] (flagged segments, all shards) is 0
  int32_t force_storm;  // diagnostics (GH_FORCE_STORM): run the storm variant every round
  int32_t force_slow;   // diagnostics (GH_FORCE_SLOW): every segment by the per-cell rule
  int32_t nib_rmv;      // nibble path: REMOVE'd members with >= 2 detectors stay on it (GH_NIB_RMV=0: lane jobs;
                        // 2: k_round IN 6 every round, else only in rounds with a detection)
  int32_t nib_dma;      // nibble path: LDS-DMA staging of the own and sender lines (GH_NIB_DMA; column layout, TW 256)
  int32_t shadow_row;   // the introducer while it may hold D7 shadow entries (its segments take k_round_slow), else -1
  int32_t vslot;        // the round's index in its gh_step call (vlog: which k_round variant ran)
  int32_t rmv_full;     // k_round IN 6 on a full grid: the host knows a REMOVE is pending this round
  int32_t plane;        // the round writes the next buffer's sender plane (and may read cur's)
  int32_t ring_whole;   // ring mode: one engine and a current flag count, so the targets may come
                        // from whole lists when no REMOVE / flag is pending (k_ring_fast)
  int32_t gpo;          // row layout: this round's ghost rows carry only their sender plane (the
                        // 16-bit codes arrive after k_round, before k_round_slow, if any segment needs them)
};

// ---- launchers (kernels in round.hip / events.hip / place.hip) ----------
// round.hip
// Row j receives REMOVE(c) of the REMOVE set of parity dcur (c in that set):
// the reference's recipients under GH_REMOVE_LIST, else every row but a sole
// detector (SPEC D4; the detector does not message itself, :344-346).
__device__ __forceinline__ bool gh_rm_at(const GhDev& d, int dcur, int64_t c, int64_t j) {
  if (d.rlist) return (d.rcv[dcur][c * d.nw + (j >> 5)] >> (j & 31)) & 1u;
  return !(d.det_cnt[dcur][c] == 1 && d.det_min[dcur][c] == j);
}

void launch_active_pre(const GhDev& d, int cur, int dcur, const GhRound& p, hipStream_t s);
void launch_active_post(const GhDev& d, const GhRound& p, hipStream_t s);
// one engine (world 1): launch_base + the guard of every row, decided in
// place (no count exchange, no launch_active_post)
void launch_prologue(const GhDev& d, int cur, int dcur, const GhRound& p, hipStream_t s);
void launch_peers_pull(const GhDev& d, int cur, int dcur, const GhRound& p, hipStream_t s);
// row layout: draw validity at the senders' owners (pvf, then SUM over
// shards), then every receiver's inbox
void launch_peers_rows(const GhDev& d, int cur, int dcur, const GhRound& p, hipStream_t s);
void launch_inbox_bits(const GhDev& d, const GhRound& p, hipStream_t s);
void launch_inbox_rows(const GhDev& d, const GhRound& p, hipStream_t s);
void launch_negate(int32_t* x, int64_t n, hipStream_t s);
// row layout: soleval of every local column from the owners of the single detectors (then max-allreduced)
void launch_sole_vals(const GhDev& d, int cur, int dcur, const GhRound& p, hipStream_t s);
void launch_ring_count(const GhDev& d, int cur, int dcur, const GhRound& p, hipStream_t s);
void launch_ring_select(const GhDev& d, int cur, int dcur, const GhRound& p, hipStream_t s);
void launch_inbox(const GhDev& d, const GhRound& p, hipStream_t s);
// nt = non-temporal hints on the once-touched streams of k_round
// variant: 0 the lean one on a 16-bit input, 1 the storm one, 2 the lean one
// on a 4-bit-tier input by the 16-bit rule, 3 the nibble path (2 and 3:
// tiered engines; the nibble path's row-layout form is k_round IN = 4); all
// are launched every round (0-2 on the side stream) and only the one k_base,
// the input's tier and the plane select runs
// t0 / t1: timing events stamped by the launch itself (hipExtLaunchKernel:
// the dispatch packet's start and end, no separate event packets), or null
bool launch_round(const GhDev& d, int cur, int dcur, const GhRound& p, hipStream_t s, bool nt, int variant,
                  hipEvent_t t0 = nullptr, hipEvent_t t1 = nullptr);
// the nibble path's lane jobs (tiered engines; after launch_round, before
// launch_round_slow): k_round_jobs, then the wide redo of the rare lanes
// whose cells leave the 16-bit window
void launch_round_jobs(const GhDev& d, int cur, int dcur, const GhRound& p, hipStream_t s);
// the segments k_round listed, by the per-cell rule (after launch_round)
void launch_round_slow(const GhDev& d, int cur, int dcur, const GhRound& p, hipStream_t s);
void launch_finish(const GhDev& d, int dcur, const GhRound& p, hipStream_t s);
// GH_REMOVE_LIST: the column bitmaps of the round's sweep (before
// launch_finish) and the recipients of D_r (after it); remove.hip
void launch_rm_cols(const GhDev& d, int cur, int dcur, const GhRound& p, hipStream_t s);
void launch_rm_recv(const GhDev& d, int dnew, const GhRound& p, hipStream_t s);
// base[cur ^ 1] from buffer cur (member c's own heartbeat - GH_BASE_LAG),
// |D_{r-1}| next to the local counts, empty slow list
void launch_base(const GhDev& d, int cur, int dcur, const GhRound& p, hipStream_t s);
// quirk-mode detection: summaries + per-row prefix (then allgather qall), and
// carry-in + flag rewrite of the current table
void launch_quirk_scan(const GhDev& d, int cur, int dcur, const GhRound& p, hipStream_t s);
void launch_quirk_apply(const GhDev& d, int cur, int dcur, const GhRound& p, hipStream_t s);
// the same in one pass, one wave per row (whole rows on this engine: world 1
// or row shards; tile widths >= 32)
void launch_quirk_rows(const GhDev& d, int cur, int dcur, const GhRound& p, hipStream_t s);
// events.hip
void launch_count(const GhDev& d, int cur, const GhRound& p, hipStream_t s);
void launch_fill(const GhDev& d, int cur, int32_t hb0, int32_t ts0, const GhRound& p,
                 hipStream_t s);
// full host rows (hb, ts: [nrows][n]) -> encoded tiled local columns; p.r is
// the round about to run
void launch_pack(const GhDev& d, int cur, const int32_t* hb_rows, const int32_t* ts_rows, int64_t row0,
                 int64_t nrows, const GhRound& p, hipStream_t s);
// tiled local columns -> [nrows][ncs] (local column order) of the external hb
// (what = 0) or the exported ts (what = 1, gh_export_ts); p.r is the round
// about to run
void launch_unpack(const GhDev& d, int cur, int32_t* dst_rows, int64_t row0, int64_t nrows, int what,
                   const GhRound& p, hipStream_t s);
// rows that stop (crash / leave), their frozen-store slots already in frow:
// exact cells into the store, GH_N_FROZEN in both buffers
void launch_freeze(const GhDev& d, int cur, const int32_t* rows, int32_t nr, const GhRound& p, hipStream_t s);
// segments of buffer buf: wide (arena) -> out[0], frozen -> out[1] (device)
void launch_count_wide(const GhDev& d, int buf, unsigned long long* out, hipStream_t s);
// 1 -> *flag if a row that runs the round (und: alive, not stopping in its
// events) has its own heartbeat at INT32_MAX (the round would
// overflow it, slave/slave.go:446); *flag is zeroed by the caller
void launch_hb_check(const GhDev& d, int cur, int32_t* flag, const GhRound& p, hipStream_t s);
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
// rows.hip (row layout): ghost rows, in two parts (GH_GX_PLANE: the sender
// plane words, GH_GX_CODES: the 16-bit codes). pack: rows[0..ns) (owned)
// -> out back to back (ghost_part_bytes each), codes: wcnt[dest[e]] += the
// row's wide segments; wide: their exact cells -> out records
// (ghost_wide_record_bytes each) at wcur[dest]++; unwide: nrec records ->
// fresh arena slots of buffer cur, the ghost rows' markers rewritten
#define GH_GX_PLANE 1
#define GH_GX_CODES 2
// the slices of one exchange chunk (k_gx_idx): destination r's rows are
// wlist[r][src[r] .. src[r] + out[r + 1] - out[r]), at out[r] in the chunk
constexpr int GH_GX_MAXG = 16;
struct GxSlices {
  int32_t g;
  int64_t total;
  int64_t src[GH_GX_MAXG];
  int64_t out[GH_GX_MAXG + 1];
};
// want lists of every shard from the replicated inboxes (rows.hip): wbits
// [G][ceil(n/32)], wsum [G][blocks], wlist [G][n], mcnt [G][G] + [G] totals
void launch_want_lists(const GhDev& d, const GhRound& p, int64_t nrs, int G, uint32_t* wbits, int32_t* wsum,
                       int32_t* wlist, int32_t* mcnt, hipStream_t s);
void launch_ghost_slots(const GhDev& d, const int32_t* mine, const int32_t* cnt, hipStream_t s);
void launch_gx_idx(const int32_t* wlist, int64_t n, const GxSlices& sl, int32_t* rows, int32_t* dest, hipStream_t s);
int64_t ghost_part_bytes(const GhDev& d, int part);
// Same-device in-process shards (LOCAL transport): the peers' sender planes,
// so a shard gathers its ghosts' plane rows straight from their owners'
// tables (no pack, no staging copy)
constexpr int kGxPeers = 16;
struct GxPeers {
  const uint32_t* pl[kGxPeers];  // the owner's plane of the round's input buffer
  int64_t row0[kGxPeers], tstride[kGxPeers];
};
void launch_ghost_gather_plane(const GhDev& d, const GxPeers& pp, const int32_t* ghosts, int64_t ng, int64_t nrs,
                               hipStream_t s);
int64_t ghost_wide_record_bytes(const GhDev& d);
void launch_ghost_pack(const GhDev& d, int cur, const int32_t* rows, const int32_t* dest, int64_t ns, int part,
                       char* out, int32_t* wcnt, hipStream_t s);
void launch_ghost_wide(const GhDev& d, int cur, const int32_t* rows, const int32_t* dest, int64_t ns, int32_t* wcur,
                       char* out, hipStream_t s);
void launch_ghost_unwide(const GhDev& d, int cur, const char* in, int64_t nrec, hipStream_t s);
// order.hip (GH_ORDER_APPEND): list generation lin -> lin ^ 1 (events: rows
// or all; added members in the order of src_ids, else of src_row's new list);
// ring: flags_known = the table's flagged-segment count is current (every
// snapshot is a whole list when it and |D_{r-1}| are 0)
bool list_lds_ok(const GhDev& d);
void launch_list_round(const GhDev& d, int cur, int dcur, const GhRound& p, int lin, hipStream_t s);
void launch_list_events(const GhDev& d, int cur, int lin, const int32_t* rows, int32_t nr, const int32_t* src_ids,
                        int32_t n_src, int32_t src_row, int32_t skip, hipStream_t s);
void launch_list_import(const GhDev& d, int cur, int lb, int64_t row0, int64_t nr, hipStream_t s);
void launch_ring_list(const GhDev& d, int cur, int dcur, const GhRound& p, int lin, int flags_known, hipStream_t s);
void launch_quirk_list(const GhDev& d, int cur, int dcur, const GhRound& p, int lin, hipStream_t s);
void launch_list_cand(const GhDev& d, int lin, int32_t master, hipStream_t s);
void launch_list_pack(const GhDev& d, int g, int32_t* buf, int64_t lo, int64_t hi, hipStream_t s);
void launch_list_unpack(const GhDev& d, int g, const int32_t* buf, int64_t lo, int64_t hi, hipStream_t s);
void launch_list_first(const GhDev& d, int lin, int32_t* out, hipStream_t s);
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
