// Gossip-round kernels for gfx950 (SPEC.md §2-§3, DESIGN.md "Kernels").
//
//   k_base         next buffer's column bases, |D_{r-1}| for the count allreduce
//   k_active_pre / k_active_exact / k_active_post
//                  per row: the <4 guard after REMOVE delivery
//                  (slave/slave.go:504,511). Rows decided by the global count
//                  need nothing else; the few undecided rows get an exact
//                  post-REMOVE count (summed over ranks when sharded).
//   k_peers_pull   per receiver column: k Philox peers, kept iff the sender is
//                  active, alive and lists the receiver (slave/slave.go:527-542).
//   k_ring_*       reference ring topology (slave/slave.go:512-524): per-(tile,row)
//                  snapshot counts, positions, targets + inbox CSR.
//   k_quirk_*      quirk-mode detection pre-pass (SPEC §4).
//   k_round        THE HOT KERNEL: one pass over the narrow table, packed
//                  16-bit: k-peer max-merge, own heartbeat, aging, next-round
//                  flag (slave/slave.go:414-497) for a 256-row x 64-member
//                  tile per workgroup; lists the segments needing the
//                  per-cell rule.
//   k_round_slow   those segments: REMOVE delivery, guard, detection,
//                  cleanup and merge cell by cell (slave/slave.go:276-286,
//                  414-497) on wide values.
//   k_finish       per column: the failed-set bitmap D_r for the next round.
// Member columns are local to the engine's shard (gh_internal.h); rows,
// alive/active and the inboxes are global.
#include <cstdlib>
#include <limits.h>

#include <algorithm>

#include <hip/hip_ext.h>

#include "gh_internal.h"

namespace {

__device__ __forceinline__ int uni(int x) { return __builtin_amdgcn_readfirstlane(x); }

__device__ __forceinline__ bool dbit(const uint32_t* bits, int64_t c) {
  return (bits[c >> 5] >> (c & 31)) & 1u;
}

// Step 1 applies REMOVE(c) at row j when gh_rm_at(d, dcur, c, j)
// (gh_internal.h: every row but a sole detector, or the reference's
// recipients under GH_REMOVE_LIST).

// Decides row i from its global count c = cntg[i] and the global |D| = ndg;
// an undecided row (|D| could push it under the threshold) gets its exact
// local post-REMOVE count in post (u = 1), or is left to k_active_exact's
// full recount in failure storms (u = 2).
__device__ __forceinline__ void active_row(const GhDev& d, int cur, int dcur, const GhRound& p, int i, int ndg,
                                           bool& a, uint8_t& u, int32_t& post) {
  a = false;
  u = 0;
  post = 0;
  if (!d.alive[i]) return;
  const int c = d.cntg[i];
  if (c < p.min_members) {
    a = false;
  } else if (c - ndg >= p.min_members) {
    a = true;
  } else if (d.nd[dcur] > GH_DLIST_MAX) {
    u = 2;
  } else if (!gh_owned(d, i)) {
    u = 1;  // row layout: the owner counts it, this shard adds 0
  } else {
    u = 1;
    int rem = 0;
    const int nd = d.nd[dcur];
    for (int q = 0; q < nd; ++q) {
      const int col = d.dlist[(int64_t)dcur * p.ld + q];
      rem += (gh_get(d, cur, i, col, p.r).x >= 0) && gh_rm_at(d, dcur, col, i);
    }
    post = d.cntl[i] - rem;
  }
}

// ST_ACTIVE_ROWS += the block's active rows: one atomic per workgroup (per
// wave they serialise on one address: 15 us at N = 65,536)
__device__ __forceinline__ void count_active(const GhDev& d, bool a) {
  __shared__ int s_act;
  if (threadIdx.x == 0) s_act = 0;
  __syncthreads();
  const unsigned long long m = __ballot(a);
  if ((threadIdx.x & 63) == 0 && m) atomicAdd(&s_act, __popcll(m));
  __syncthreads();
  if (d.rank == 0 && threadIdx.x == 0 && s_act) atomicAdd(&d.stats[ST_ACTIVE_ROWS], (unsigned long long)s_act);
}

__global__ __launch_bounds__(256) void k_active_pre(GhDev d, int cur, int dcur, GhRound p) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    d.nd[dcur ^ 1] = 0;
    d.nd[2 + (dcur ^ 1)] = 0;
  }
  if (i >= p.n) return;
  d.det_any[i] = 0;
  bool a;
  uint8_t u;
  int32_t post;
  active_row(d, cur, dcur, p, i, d.cntg[p.n], a, u, post);
  d.active[i] = a;
  d.und[i] = u;
  d.post[i] = post;
}

// Failure storms (local |D| > GH_DLIST_MAX): one wave recounts each
// undecided row over the local columns with REMOVE applied. One engine
// (fin): the recount is global, so the row is decided here (k_active_post's
// work for it).
__global__ __launch_bounds__(256) void k_active_exact(GhDev d, int cur, int dcur, GhRound p, int fin) {
  if (d.nd[dcur] <= GH_DLIST_MAX) return;
  const int lane = threadIdx.x & 63;
  for (int i = blockIdx.x * 4 + (threadIdx.x >> 6); i < p.n; i += gridDim.x * 4) {
    if (d.und[i] != 2) continue;
    if (!gh_owned(d, i)) {  // row layout: the owner counts it, this shard adds 0
      if (lane == 0) d.post[i] = 0;
      continue;
    }
    int cnt = 0;
    for (int64_t c = lane * 8; c < p.ld; c += 512) {
      const uint32_t pf = gh_pf8(d, cur, i, c);
      const uint32_t b8 = (d.dbits[c >> 5] >> (c & 31)) & 0xFFu;
#pragma unroll
      for (int j = 0; j < 8; ++j)
        cnt += ((pf >> j) & 1u) && !(((b8 >> j) & 1u) && gh_rm_at(d, dcur, c + j, i));
    }
    for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o);
    if (lane == 0) {
      d.post[i] = cnt;
      if (fin) {
        const bool a = cnt >= p.min_members;
        d.active[i] = a;
        d.stab[(p.r + 1) & 1][i] = !a;  // an undecided row is alive
        if (a && d.rank == 0) atomicAdd(&d.stats[ST_ACTIVE_ROWS], 1ull);
      }
    }
  }
}

// post[] now holds the global post-REMOVE counts of the undecided rows.
__global__ __launch_bounds__(256) void k_active_post(GhDev d, GhRound p) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  bool a = false;
  if (i < p.n) {
    a = d.active[i];
    if (d.und[i]) {
      a = d.post[i] >= p.min_members;
      d.active[i] = a;
    }
    d.stab[(p.r + 1) & 1][i] = d.alive[i] && !a;  // quiet candidates for the next round
  }
  count_active(d, a);
}

// Receivers are this shard's member columns (their column holds the senders'
// view of them); the inbox rows of the other shards arrive by allgather.
// Eight lanes per receiver, lane q checks draw q (q < k), so the dependent
// loads of the draws overlap; the valid senders are compacted in draw order.
__global__ __launch_bounds__(256) void k_peers_pull(GhDev d, int cur, int dcur, GhRound p) {
  const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int t = (int)(gid >> 3);
  const int q = (int)(gid & 7);
  const bool inr = t < d.ncs;
  const int64_t i = d.col0 + t;  // global receiver (>= n in the tail of the last shard)
  const int64_t beg = i * (p.k + 1) + 1;
  bool ok = false;
  int s = 0;
  if (inr && q < p.k && t < d.ncol && d.alive[i] && p.n >= 2) {
    const uint32_t u = gh_philox_word(p.seed, (uint32_t)i, (uint32_t)p.r, GH_TAG_PEER, (uint32_t)(q >> 2), q & 3);
    const uint32_t w = (uint32_t)(((uint64_t)u * (uint64_t)(p.n - 1)) >> 32);
    s = (int)w + ((int64_t)w >= i);
    // (a tier chunk's two words are loaded beside s's alive / active bytes,
    // not after them: one level of dependent loads instead of two)
    const bool tier = gh_m8(d, cur);
    uint32_t aw = 0, lw = 0;
    if (tier) {
      const int64_t cell = gh_cell(d, s, t & ~(int64_t)7);
      aw = d.a4[cur][cell >> 3];
      lw = d.pl[cur][cell >> 3];
    }
    if (d.alive[s] && d.active[s]) {
      // i must be in s's snapshot list: present, not detected by s this
      // round and not REMOVE'd at s in step 1. A tier chunk answers from its
      // two words (code 15: absent or a tombstone; a tier cell is never
      // flagged)
      if (tier) {
        if (!gh_t4_esc(aw)) {
          ok = ((lw >> gh_nib((int)(t & 7))) & 0xFu) != 15u;
        } else {
          const GhCell v = gh_get(d, cur, s, t, p.r);
          ok = v.x >= 0 && !v.f;
        }
      } else {
        const GhCell v = gh_get(d, cur, s, t, p.r);
        ok = v.x >= 0 && !v.f;
      }
      if (ok && dbit(d.dbits, t) && gh_rm_at(d, dcur, t, s)) ok = false;
    }
  }
  const unsigned long long m = __ballot(ok);
  const int lane = threadIdx.x & 63;
  const uint32_t grp = (uint32_t)(m >> (lane & ~7)) & 0xFFu;  // this receiver's valid draws
  if (ok) d.inbox[beg + __builtin_popcount(grp & ((1u << q) - 1u))] = s;
  if (d.nsnd) {  // the nibble path's row record (one engine: receivers are rows 0..n-1, k <= 4)
    const int b8 = lane & ~7;
    int sq[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) sq[u] = __shfl(s, b8 + u);
    if (inr && q == 0 && t < d.ncol) {
      int rec[4], nv = 0;
#pragma unroll
      for (int u = 0; u < 4; ++u) rec[u] = (int)i;
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if ((grp >> u) & 1u) {
#pragma unroll
          for (int v = 0; v < 4; ++v)
            if (v == nv) rec[v] = sq[u];
          nv++;
        }
      const int al = d.alive[i], act = d.active[i];
      const bool quiet = d.cntg[p.n] == 0 && !p.force_slow && !d.m8[2];
      d.nmeta[i] = al | (act << 1) | (nv << 2) | ((quiet && al && !act && nv == 0 && d.stab[p.r & 1][i]) ? 1 << 30 : 0);
      *reinterpret_cast<int4*>(d.nsnd + 4 * i) = int4{rec[0], rec[1], rec[2], rec[3]};
    }
  }
  if (inr && q == 0) {
    if (t < d.ncol && d.alive[i] && (d.active[i] || grp || !d.stab[p.r & 1][i])) d.aq[0] = 1;  // not quiet
    d.inbox[beg - 1] = __builtin_popcount(grp);
    if (d.pvb) d.pvb[i] = (uint8_t)grp;  // G > 1: the bits travel, not the inbox (k_inbox_bits)
  }
}

// Column layout, G > 1: every receiver's inbox from the allgathered validity
// bits of its draws (the same draws as k_peers_pull, in draw order).
__global__ __launch_bounds__(256) void k_inbox_bits(GhDev d, GhRound p) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= p.n) return;
  const uint32_t b = d.pvb[i];
  const int64_t beg = i * (p.k + 1) + 1;
  int nv = 0;
  for (int q = 0; q < p.k; ++q) {
    if (!((b >> q) & 1u)) continue;
    const uint32_t u = gh_philox_word(p.seed, (uint32_t)i, (uint32_t)p.r, GH_TAG_PEER, (uint32_t)(q >> 2), q & 3);
    const uint32_t w = (uint32_t)(((uint64_t)u * (uint64_t)(p.n - 1)) >> 32);
    d.inbox[beg + nv++] = (int)w + ((int64_t)w >= i);
  }
  d.inbox[beg - 1] = nv;
}

// Row layout: sender s's owner checks receiver i's draws against s's row
// (the cells only it holds); pvf[i*k + q] = 1 there, 0 on every other shard,
// so a SUM over shards is the validity of every draw.
__global__ __launch_bounds__(256) void k_peers_rows(GhDev d, int cur, int dcur, GhRound p) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= p.n) return;
  const bool ib = dbit(d.dbits, i);
  for (int q = 0; q < p.k; ++q) {
    int v = 0;
    if (d.alive[i] && p.n >= 2) {
      const uint32_t u = gh_philox_word(p.seed, (uint32_t)i, (uint32_t)p.r, GH_TAG_PEER, (uint32_t)(q >> 2), q & 3);
      const uint32_t w = (uint32_t)(((uint64_t)u * (uint64_t)(p.n - 1)) >> 32);
      const int s = (int)w + ((int64_t)w >= i);
      if (gh_owned(d, s) && d.alive[s] && d.active[s]) {
        const GhCell c = gh_get(d, cur, s, i, p.r);
        v = c.x >= 0 && !c.f && !(ib && gh_rm_at(d, dcur, i, s));
      }
    }
    d.pvf[i * p.k + q] = v;
  }
}

// Row layout: every receiver's inbox from the summed validity of its draws
// (the same layout as k_peers_pull's, on every shard).
__global__ __launch_bounds__(256) void k_inbox_rows(GhDev d, GhRound p) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= p.n) return;
  const int64_t beg = i * (p.k + 1) + 1;
  int nv = 0;
  for (int q = 0; q < p.k; ++q) {
    if (!d.pvf[i * p.k + q]) continue;
    const uint32_t u = gh_philox_word(p.seed, (uint32_t)i, (uint32_t)p.r, GH_TAG_PEER, (uint32_t)(q >> 2), q & 3);
    const uint32_t w = (uint32_t)(((uint64_t)u * (uint64_t)(p.n - 1)) >> 32);
    d.inbox[beg + nv++] = (int)w + ((int64_t)w >= i);
  }
  d.inbox[beg - 1] = nv;
}

// x -> -x over n int32 (a MIN reduction as a MAX of negations)
__global__ void k_negate(int32_t* x, int64_t n) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t < n) x[t] = -x[t];
}

// ---- segment walks -------------------------------------------------------
// The helper kernels below read the table the way k_round does: a lane owns
// 8 consecutive members (16 B of narrow cells), SEG = TW/8 lanes cover one
// row segment of a tile, and consecutive waves take consecutive (tile, row)
// segments in storage order, so every wave instruction is one contiguous
// 1 KiB access.
// Segments are (tile, owned row) pairs, tile-major: segment sid is tile
// sid / nrows, row row0 + sid % nrows.
template <int TW>
struct SegWalk {
  static constexpr int SEG = TW / 8;
  static constexpr int RPW = 64 / SEG;
  int lane, sub, lc;
  int64_t nseg, first, stride, row0, nrows;
  __device__ SegWalk(const GhDev& d, const GhRound& p) {
    lane = threadIdx.x & 63;
    sub = lane / SEG;
    lc = lane % SEG;
    row0 = d.row0;
    nrows = d.nrows;
    nseg = (p.ld / TW) * nrows;
    first = (((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6) * RPW;
    stride = (((int64_t)gridDim.x * blockDim.x) >> 6) * RPW;
  }
  // A contiguous run of segments per wave (k_quirk_*): [run0, run1), steps
  // of RPW * U segments. Consecutive segments are consecutive rows of one
  // tile, so a wave's one-byte-per-segment stores fill whole lines from one
  // XCD (the strided walk had every line of qsum written by 16 workgroups on
  // all 8 XCDs: 3.7 ms for a 1 ms sweep).
  __device__ void run(int U, int64_t& run0, int64_t& run1) const {
    const int64_t nw = stride / RPW, gw = first / RPW, step = (int64_t)RPW * U;
    const int64_t per = ((nseg + nw - 1) / nw + step - 1) / step * step;
    run0 = gw * per;
    run1 = min(nseg, run0 + per);
  }
  __device__ void at(int64_t sid, int64_t& t, int& i) const {
    // (a 64-bit division per segment had dominated the whole-table sweeps:
    // 32-bit when the segment count fits, as it does up to N = 262,144)
    if (nseg <= (int64_t)UINT32_MAX) {
      const uint32_t q = (uint32_t)sid / (uint32_t)nrows;
      t = q;
      i = (int)(row0 + ((uint32_t)sid - q * (uint32_t)nrows));
    } else {
      t = sid / nrows;
      i = (int)(row0 + (sid - t * nrows));
    }
  }
};

// 8-bit REMOVE mask of local columns l0..l0+7 at row i (l0 % 8 == 0)
// (one detector's column is REMOVE'd at every row but that detector's:
// only those columns, sbits, look at det_min)
__device__ __forceinline__ uint32_t removed8(const GhDev& d, int dcur, int64_t l0, int i) {
  const uint32_t m = (d.dbits[l0 >> 5] >> (l0 & 31)) & 0xFFu;
  if (!m) return 0u;
  if (d.rlist) {
    uint32_t out = 0;
    for (int j = 0; j < 8; ++j)
      if (((m >> j) & 1u) && gh_rm_at(d, dcur, l0 + j, i)) out |= 1u << j;
    return out;
  }
  uint32_t sm = (d.sbits[l0 >> 5] >> (l0 & 31)) & m;
  uint32_t out = m & ~sm;
  while (sm) {
    const int j = __builtin_ctz(sm);
    sm &= sm - 1u;
    if (d.det_min[dcur][l0 + j] != i) out |= 1u << j;
  }
  return out;
}

// Ring mode when every snapshot list is a whole list (a single engine, the
// flag count current, no REMOVE pending and no flagged segment anywhere): the
// list is the row's present members in ID order, so the targets are found by
// scanning outward from the sender (one wave per sender row, 512 members per
// step) instead of counting the row.
__device__ __forceinline__ bool ring_whole(const GhDev& d, const GhRound& p) {
  return p.ring_whole && d.cntg[p.n] == 0 && d.cntg[p.n + 1] == 0;
}

// First present member of row s after x (dir > 0) or before x (dir < 0),
// cyclically; the row holds at least one present member. Wave-uniform.
__device__ int ring_next(const GhDev& d, int cur, int s, int x, int dir) {
  const int lane = threadIdx.x & 63;
  const int nch = (d.n + 7) >> 3;
  for (int pass = 0; pass < 2; ++pass) {
    // pass 0: from x onward; pass 1: the wrap-around, from the far end
    int c0 = pass == 0 ? x + dir : (dir > 0 ? 0 : d.n - 1);
    for (;;) {
      if (c0 < 0 || c0 >= d.n) break;
      const int k0 = c0 >> 3;
      const int k = dir > 0 ? k0 + lane : k0 - lane;
      uint32_t m = 0;
      if (k >= 0 && k < nch) {
        m = gh_pf8(d, cur, s, (int64_t)k * 8) & 0xFFu;
        if (k == k0) m &= dir > 0 ? (0xFFu << (c0 & 7)) & 0xFFu : 0xFFu >> (7 - (c0 & 7));
      }
      const unsigned long long hit = __ballot(m != 0);
      if (hit) {
        const int src = __ffsll((long long)hit) - 1;  // the nearest chunk
        const int c = k * 8 + (dir > 0 ? __builtin_ctz(m ? m : 1u) : 31 - __builtin_clz(m ? m : 1u));
        return __shfl(c, src);
      }
      c0 = dir > 0 ? (k0 + 64) * 8 : (k0 - 64) * 8 + 7;
    }
  }
  return -1;
}

__global__ __launch_bounds__(256) void k_ring_fast(GhDev d, int cur, GhRound p) {
  if (!ring_whole(d, p)) return;
  const int s = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (s >= p.n) return;
  int tg[3] = {-1, -1, -1};
  // (row layout: the sender's owner finds its targets, the other shards'
  // targets arrive by allreduce(max))
  if (gh_owned(d, s) && d.alive[s] && d.active[s]) {
    if (d.cntl[s] == 0) {
      if ((threadIdx.x & 63) == 0) atomicAdd(&d.stats[ST_RING_EMPTY], 1ull);  // slave.go:517 division by zero
    } else if (gh_pf8(d, cur, s, s & ~7) >> (s & 7) & 1u) {
      // list[(idx-1) mod L], list[(idx+1) mod L], list[(idx+2) mod L]
      tg[0] = ring_next(d, cur, s, s, -1);
      tg[1] = ring_next(d, cur, s, s, 1);
      tg[2] = ring_next(d, cur, s, tg[1], 1);
    } else {
      // idx = -1: list[L-2], list[0], list[1] (Go's % truncates, then + L)
      const int last = ring_next(d, cur, s, d.n, -1);
      tg[0] = ring_next(d, cur, s, last, -1);
      tg[1] = ring_next(d, cur, s, -1, 1);
      tg[2] = ring_next(d, cur, s, tg[1], 1);
    }
  }
  if ((threadIdx.x & 63) < 3) d.targets[(int64_t)s * 3 + (threadIdx.x & 63)] = tg[threadIdx.x & 63];
}

// Ring mode, part 1: per (tile, sender row) the number of members in the
// sender's snapshot list (present after REMOVE, not detected by it).
template <int TW>
__global__ __launch_bounds__(256) void k_ring_tiles(GhDev d, int cur, int dcur, GhRound p) {
  if (ring_whole(d, p)) return;
  const SegWalk<TW> w(d, p);
  for (int64_t base = w.first; base < w.nseg; base += w.stride) {
    const int64_t sid = base + w.sub;
    const bool valid = sid < w.nseg;
    int64_t t = 0;
    int i = 0;
    if (valid) w.at(sid, t, i);
    const int64_t l0 = t * TW + w.lc * 8;
    int cnt = 0;
    if (valid && d.alive[i] && d.active[i]) {  // only sending rows' counts are read
      const uint32_t pf = gh_pf8(d, cur, i, l0);
      const uint32_t rm = removed8(d, dcur, l0, i);
      cnt = __builtin_popcount(pf & ~(pf >> 8) & ~rm & 0xFFu);  // present, not flagged, not REMOVE'd
    }
#pragma unroll
    for (int o = SegWalk<TW>::SEG / 2; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o);
    if (valid && w.lc == 0) d.rcnt[t * p.n + i] = (uint16_t)cnt;
  }
}

// The local column of the want-th (0-based) member of sender s's snapshot
// list inside tile t (scans the tile-row).
__device__ __forceinline__ int64_t ring_find(const GhDev& d, int cur, int dcur, int s, int64_t t, int want) {
  for (int j = 0; j < d.tw; ++j) {
    const int64_t c = t * d.tw + j;
    const GhCell v = gh_get(d, cur, s, c, 0);
    if (v.x < 0 || v.f) continue;
    if (dbit(d.dbits, c) && gh_rm_at(d, dcur, c, s)) continue;
    if (want-- == 0) return c;
  }
  return -1;
}

// Ring mode, part 2 (one thread per sender row): this shard's list length
// and, when the sender's own column is local, its position in that list.
__global__ __launch_bounds__(256) void k_ring_count(GhDev d, int cur, int dcur, GhRound p) {
  if (ring_whole(d, p)) return;
  const int sdr = blockIdx.x * blockDim.x + threadIdx.x;
  if (sdr >= p.n) return;
  int32_t* out = d.ring + ((int64_t)d.rank * p.n + sdr) * 2;
  // (row layout, one shard's view of the columns: the owner counts its rows)
  if (!(gh_owned(d, sdr) && d.alive[sdr] && d.active[sdr])) {
    out[0] = 0;
    out[1] = -1;
    return;
  }
  const int64_t ntiles = p.ld / d.tw;
  const int64_t ls = (int64_t)sdr - d.col0;
  const int64_t own_t = (ls >= 0 && ls < d.ncol) ? ls / d.tw : -1;
  int64_t total = 0, pos = -1;
  for (int64_t t = 0; t < ntiles; ++t) {
    if (t == own_t) {
      const GhCell v = gh_get(d, cur, sdr, ls, 0);
      const bool in = v.x >= 0 && !v.f &&
                      !(dbit(d.dbits, ls) && gh_rm_at(d, dcur, ls, sdr));
      if (in) {
        pos = total;
        for (int64_t c = t * d.tw; c < ls; ++c) {
          const GhCell x = gh_get(d, cur, sdr, c, 0);
          pos += x.x >= 0 && !x.f &&
                 !(dbit(d.dbits, c) && gh_rm_at(d, dcur, c, sdr));
        }
      }
    }
    total += d.rcnt[t * p.n + sdr];
  }
  out[0] = (int32_t)total;
  out[1] = (int32_t)pos;
}

// Ring mode, part 3 (one thread per sender row): with every shard's (length,
// position) gathered, the sender's targets list[(idx-1) mod L],
// list[(idx+1) mod L], list[(idx+2) mod L] (slave/slave.go:515-524) that fall
// into this shard's columns; the other shards' targets arrive by
// allreduce(max).
__global__ __launch_bounds__(256) void k_ring_select(GhDev d, int cur, int dcur, GhRound p) {
  if (ring_whole(d, p)) return;  // k_ring_fast wrote the targets
  const int sdr = blockIdx.x * blockDim.x + threadIdx.x;
  if (sdr >= p.n) return;
  int32_t tg[3] = {-1, -1, -1};
  if (gh_owned(d, sdr) && d.alive[sdr] && d.active[sdr]) {
    int64_t L = 0, before_me = 0, before_owner = 0;
    const int owner = (int)(sdr / d.ncs);
    for (int g = 0; g < d.world; ++g) {
      const int64_t c = d.ring[((int64_t)g * p.n + sdr) * 2];
      if (g < d.rank) before_me += c;
      if (g < owner) before_owner += c;
      L += c;
    }
    if (L == 0) {
      if (d.rank == 0) atomicAdd(&d.stats[ST_RING_EMPTY], 1ull);  // slave.go:517 div by 0
    } else {
      const int64_t lp = d.ring[((int64_t)owner * p.n + sdr) * 2 + 1];
      const int64_t idx = lp >= 0 ? before_owner + lp : -1;
      const int64_t mine = d.ring[((int64_t)d.rank * p.n + sdr) * 2];
      int64_t want[3] = {idx - 1, idx + 1, idx + 2};
      for (int q = 0; q < 3; ++q) {
        int64_t v = want[q] % L;  // C and Go both truncate toward zero
        if (v < 0) v += L;
        want[q] = v - before_me;  // position inside this shard's part
      }
      const int64_t ntiles = p.ld / d.tw;
      int64_t acc = 0;
      for (int64_t t = 0; t < ntiles && acc < mine; ++t) {
        const int64_t c = d.rcnt[t * p.n + sdr];
        for (int q = 0; q < 3; ++q)
          if (want[q] >= acc && want[q] < acc + c)
            tg[q] = (int32_t)(d.col0 + ring_find(d, cur, dcur, sdr, t, (int)(want[q] - acc)));
        acc += c;
      }
    }
  }
  for (int q = 0; q < 3; ++q) d.targets[(int64_t)sdr * 3 + q] = tg[q];
}

__global__ __launch_bounds__(256) void k_inbox_count(GhDev d, GhRound p) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= p.n) return;
  for (int q = 0; q < 3; ++q) {
    const int t = d.targets[(int64_t)s * 3 + q];
    if (t >= 0 && d.alive[t]) atomicAdd(&d.inbox_cnt[t], 1);
  }
}

// Exclusive scan of inbox_cnt -> inbox_beg; one 1024-thread workgroup. Each
// thread owns a run of a multiple of 4 counters, read and written as int4
// (the arrays are 16-B aligned), so its loads are independent of each other.
__global__ __launch_bounds__(1024) void k_inbox_scan(GhDev d, GhRound p) {
  __shared__ int s_sum[1024];
  const int tid = threadIdx.x;
  const int per = ((p.n + 1023) / 1024 + 3) & ~3;
  const int b = min(p.n, tid * per), e = min(p.n, b + per);
  const bool vec = e - b == per;
  int acc = 0;
  if (vec) {
#pragma unroll 4
    for (int x = b; x < e; x += 4) {
      const int4 v = *reinterpret_cast<const int4*>(d.inbox_cnt + x);
      acc += v.x + v.y + v.z + v.w;
    }
  } else {
    for (int x = b; x < e; ++x) acc += d.inbox_cnt[x];
  }
  s_sum[tid] = acc;
  __syncthreads();
  for (int off = 1; off < 1024; off <<= 1) {
    const int v = tid >= off ? s_sum[tid - off] : 0;
    __syncthreads();
    s_sum[tid] += v;
    __syncthreads();
  }
  int run = tid ? s_sum[tid - 1] : 0;
  if (vec) {
#pragma unroll 4
    for (int x = b; x < e; x += 4) {
      const int4 v = *reinterpret_cast<const int4*>(d.inbox_cnt + x);
      int4 o;
      o.x = run;
      o.y = o.x + v.x;
      o.z = o.y + v.y;
      o.w = o.z + v.z;
      run = o.w + v.w;
      *reinterpret_cast<int4*>(d.inbox_beg + x) = o;
      *reinterpret_cast<int4*>(d.inbox_fill + x) = int4{0, 0, 0, 0};
    }
  } else {
    for (int x = b; x < e; ++x) {
      d.inbox_beg[x] = run;
      d.inbox_fill[x] = 0;
      run += d.inbox_cnt[x];
    }
  }
}

// Inbox order is whatever the atomics give: the merge is a max, so only the
// set of senders matters.
__global__ __launch_bounds__(256) void k_inbox_fill(GhDev d, GhRound p) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= p.n) return;
  if (d.alive[s] && (d.active[s] || d.inbox_cnt[s] || !d.stab[p.r & 1][s])) d.aq[0] = 1;  // row s is not quiet
  for (int q = 0; q < 3; ++q) {
    const int t = d.targets[(int64_t)s * 3 + q];
    if (t >= 0 && d.alive[t]) {
      const int pos = atomicAdd(&d.inbox_fill[t], 1);
      d.inbox[d.inbox_beg[t] + pos] = s;
    }
  }
}

// bits (2j, 2j+1) of the 8-bit lane mask from the halves of pair j's mask
__device__ __forceinline__ uint32_t pair_bits(uint32_t m, int j) {
  return ((m & 1u) | ((m >> 15) & 2u)) << (2 * j);
}

// ---- sender snapshot plane (gh_internal.h: pl) ---------------------------
// 0xFF in each byte of m that has bit 7 set (m: 0x80 / 0x00 bytes), no multiply
// nonzero iff a nibble of a is zero (exact when no nibble is zero; a
// borrow can only add bits above a zero nibble)
__device__ __forceinline__ uint32_t nib_haszero(uint32_t a) { return (a - 0x11111111u) & ~a & 0x88888888u; }

template <bool NT>
__device__ __forceinline__ v4u ldn(const uint16_t* p) {
  if constexpr (NT)
    return __builtin_nontemporal_load(reinterpret_cast<const v4u*>(p));
  else
    return *reinterpret_cast<const v4u*>(p);
}
template <bool NT>
__device__ __forceinline__ void stn(uint16_t* p, v4u v) {
  if constexpr (NT)
    __builtin_nontemporal_store(v, reinterpret_cast<v4u*>(p));
  else
    *reinterpret_cast<v4u*>(p) = v;
}

// base[cur ^ 1]: member c's own heartbeat in buffer cur - GH_BASE_LAG, so the
// round's output (its views of c lag the counter) is narrow; kept when the
// member is not present in its own row.
__device__ __forceinline__ void base_col(const GhDev& d, int cur, int dcur, const GhRound& p, int64_t c) {
  if (c == 0) {
    // k_round variant of this round: the storm one when more than 1/32 of
    // the segments of the last round went to the slow list or hold cells
    // that need the per-cell rule in the lean variant (flagged, tombstone,
    // guard rows); flags are set one round ahead, so a detection wave is
    // seen the round before it happens
    // (quiet segments count too: a collapsed cluster stays on the storm
    // variant, whose quiet skip holds while the output tier does not change;
    // on the nibble or 4-slot lean variant its guard rows would be listed)
    const int64_t measure = (int64_t)*d.nstorm + *d.slow_n + *d.nquiet;
    // ... or when the last round's lane jobs (k_round_jobs) were more than a
    // quarter of the lanes: beyond that the packed storm rule is cheaper than
    // the per-cell one
    const int64_t jobs = d.njobs ? (int64_t)d.njobs[0] : 0;
    *d.mode = p.force_storm || measure * 32 > d.ntiles * (int64_t)d.n ||
              jobs * 4 * GH_JOB_CPL > (int64_t)d.nrows * p.ld;
    if (d.njobs) {
      d.njobs[0] = 0;
      d.njobs[1] = 0;
      d.njobs[3] = 0;
    }
    if (d.a4[0]) {
      // the lean variant writes the next buffer in the 4-bit tier, the storm
      // one in 16 bits; a buffer that changes tier is written whole (no
      // quiet row keeps its old chunks)
      const int w8 = *d.mode == 0;
      d.m8[2] = w8 != d.m8[cur ^ 1];
      d.m8[cur ^ 1] = w8;
      d.m8[3] = 0;  // escaped chunks the round writes
      d.m8[5] = 0;  // row layout: a lane job needs its ghost senders' codes
    }
    *d.slow_n = 0;
    *d.nstorm = 0;
    *d.nquiet = 0;
    d.wn[cur ^ 1] = 0;  // the round rewrites every running row of the next buffer
    d.nflag[cur ^ 1] = 0;  // counted by this round's writers
    // |D_{r-1}| of this shard next to the local counts, for one allreduce
    // (row layout: every shard holds all of D, rank 0 counts it)
    d.cntl[d.n] = (d.rowlay && d.rank != 0) ? 0 : d.nd[dcur];
    d.cntl[d.n + 1] = d.nflag[cur];  // flagged segments of this shard's table (quirk gate, summed)
    d.cntl[d.n + 2] = *d.mode;       // shards running the storm variant (row layout: the ghosts' codes, summed)
    d.pvalid[cur ^ 1] = p.plane;  // this round writes the next buffer's plane
    *d.pfb = 0;
  }
  if (c >= p.ld) return;
  const int32_t b0 = d.base[cur][c];
  int32_t b = b0;
  const int64_t cg = d.col0 + c;
  if (c < d.ncol && cg < p.n && gh_owned(d, cg)) {
    const GhCell v = gh_get(d, cur, cg, c, p.r);
    if (v.x >= 0) b = v.x - GH_BASE_LAG;
  } else if (d.rowlay) {
    b = INT_MIN;  // the owner of row cg decides; the host takes the max over shards
  }
  d.base[cur ^ 1][c] = b;
  if (b != b0 && d.aq) d.aq[0] = 1;
  if (d.dnw) {  // the chunk's move word for the nibble path (8 consecutive lanes, ld % 8 == 0)
    const int64_t delta = (int64_t)b - b0;
    uint32_t x = (uint32_t)(delta & 0xF) << gh_nib((int)(c & 7));
    uint32_t bad = delta < 0 || delta > 15;
#pragma unroll
    for (int o = 1; o < 8; o <<= 1) {
      x |= __shfl_xor(x, o);
      bad |= __shfl_xor(bad, o);
    }
    if ((c & 7) == 0) {
      d.dnw[c >> 3] = x;
      d.dbad[c >> 3] = (uint8_t)bad;
    }
  }
}
__global__ __launch_bounds__(256) void k_base(GhDev d, int cur, int dcur, GhRound p) {
  base_col(d, cur, dcur, p, (int64_t)blockIdx.x * blockDim.x + threadIdx.x);
}

// One engine (world 1): k_base and the <4 guard of every row in one launch.
// No exchange is needed (cntg is cntl, and |D_{r-1}| is nd[dcur], which
// base_col copies to cntl[n] in this same launch), and every row the guard
// decides here is final (k_active_post's work); rows left to the full
// recount (und 2) are finished by k_active_exact.
__global__ __launch_bounds__(256) void k_prologue(GhDev d, int cur, int dcur, GhRound p) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  base_col(d, cur, dcur, p, t);
  if (t == 0) {
    d.nd[dcur ^ 1] = 0;
    d.nd[2 + (dcur ^ 1)] = 0;
  }
  bool a = false;
  if (t < p.n) {
    const int i = (int)t;
    d.det_any[i] = 0;
    uint8_t u;
    int32_t post;
    active_row(d, cur, dcur, p, i, d.nd[dcur], a, u, post);
    if (u == 1) a = post >= p.min_members;
    d.active[i] = a;
    d.und[i] = u;
    d.post[i] = post;
    if (u != 2) d.stab[(p.r + 1) & 1][i] = d.alive[i] && !a;  // quiet candidates for the next round
  }
  count_active(d, a);
}

// The round, fast part. Workgroup tile = RB rows x TW members of one table
// tile; the block index is tile-major so the concurrently running workgroups
// sweep one tile (a contiguous N*TW*2-byte slice of each narrow table)
// together: own-row streams are sequential and peer gathers stay in that
// slice, which the on-die caches hold. Each lane owns 8 consecutive members
// (one 16-B load of narrow cells); SEG = TW/8 lanes cover one row segment,
// so a wave handles 64/SEG rows per instruction. KB = peer loads issued
// together (4 or 8). NT = non-temporal hint on the once-written stream.
//
// A lane is on the fast path when the row is alive and active, no member of
// the lane is REMOVE'd, the lane's own cells are visible-present (age < 30)
// or absent, and every sender's segment is narrow. Then the round reduces to
// packed 16-bit arithmetic on pairs of cells: merged = a sender's heartbeat
// exceeds the own one (max); age 1 if merged, else +1; rebase onto the next
// buffer's base; flag = hb > 1 and age > T_fail. The two diagonals are
// fix-ups around it: a sender's own member carries hb + 1 in its snapshot,
// the row's own member gets hb + 1 and a fresh stamp and is never flagged.
// A segment whose lanes are all on the fast path and whose results stay
// narrow is written here; every other segment of an alive row goes to the
// slow list (k_round_slow, the reference's rule cell by cell). Stopped rows
// are not written (wide and identical in both buffers).
// Rows per workgroup tile: GH_WG_ROWS_WIDE at TW >= 128 (256 rows), else
// GH_WG_CELLS / TW within [64, 1024] (a tall,
// one-tile block: at TW = 64, 256 rows; measured best per width),
// and at least one wave step of 4 waves.
template <int TW>
constexpr int round_rb() {
  if (TW >= 128) return GH_WG_ROWS_WIDE;
  constexpr int rb = GH_WG_CELLS / TW < 64 ? 64 : GH_WG_CELLS / TW > 1024 ? 1024 : GH_WG_CELLS / TW;
  return rb < 2048 / TW ? 2048 / TW : rb;
}

// THE NIBBLE PATH (k_round with IN = 2): a healthy round of a tiered engine
// whose input buffer is in the 4-bit tier with a valid plane (column layout,
// pull k <= 4). The lean rule runs on the tier's nibbles themselves: a cell
// is q = its plane code (lag + 2; the row's own member: lag + 1; 15 absent)
// and a = its age; u = the senders' minimum plane code, the freshest entry
// (gh_internal.h: pl). A sender's heartbeat beats the own one iff u < q (an
// absent own cell takes any sender; u = 15 = no entry), and the own member's
// rule (step 3: hb + 1, merged only by a larger snapshot) is the same
// comparison on its diagonal code. Merged: code u, age 1; else age + 1; then
// the rebase q += base move. The written code is the row's next plane word
// as it stands: the senders of the next round read exactly it.
//
// A lane owns CPL consecutive cells: W = CPL / 8 dwords of the plane and of
// the age plane, and the same W dwords of each of its k senders' plane rows;
// a row segment of 256 members is 256 / CPL lanes (one 128-B line per plane
// row segment). Per dword (8 cells) the rule runs on whole nibble words:
// L = the min of the own and the senders' codes per nibble (masked fields,
// v_pk_min_u16) is the merged code; merged nibbles are those where L differs
// from the own code; the rebase and the ageing are plain 32-bit adds whose
// nibble carries mark the lane out of the tier (round 3's first form split
// even and odd nibbles into bytes with guard bits: 7% slower). RS row steps
// per iteration: all their loads are issued before any is computed. A lane
// whose every cell stays in the tier (codes 2..13, age <= min(T_fail, 15):
// no flag, no REMOVE, no escape, sender codes exact) is written here; any
// other lane of an active row is a lane job (k_round_jobs), and only rows
// under the <4 guard or with more than KB senders send whole segments to the
// slow list (k_round_slow, the per-cell rule).
template <int W>
struct NibWords {
  uint32_t v[W];
};
// Buffer resource over one tile slice of a plane (gfx9 descriptor word 3):
// the lanes then address it by 32-bit byte offsets (buffer_load ... offen,
// the base in SGPRs), with no 64-bit address arithmetic per load; an offset
// past the slice reads 0 and a store past it is dropped.
// The base is made wave-uniform explicitly: a by-value GhDev's arrays indexed
// by the runtime buffer number read as divergent, and a divergent resource
// costs a waterfall loop per access.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t nib_rsrc(const void* p, int64_t bytes) {
  const uint64_t a = reinterpret_cast<uint64_t>(p);
  const uint64_t u = ((uint64_t)(uint32_t)uni((int)(a >> 32)) << 32) | (uint32_t)uni((int)(uint32_t)a);
  return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(u), (short)0,
                                           uni((int)min(bytes, (int64_t)INT_MAX)), 0x00020000);
}
// cache policy of a buffer access on gfx950: 2 = nt (streamed once)
template <int W, int aux>
__device__ __forceinline__ NibWords<W> nib_load(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  NibWords<W> o;
  if constexpr (W == 1) {
    o.v[0] = __builtin_amdgcn_raw_buffer_load_b32(r, (int)off, 0, aux);
  } else if constexpr (W == 2) {
    const auto x = __builtin_amdgcn_raw_buffer_load_b64(r, (int)off, 0, aux);
    o.v[0] = x[0];
    o.v[1] = x[1];
  } else {
    const auto x = __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, aux);
#pragma unroll
    for (int j = 0; j < 4; ++j) o.v[j] = x[j];
  }
  return o;
}
template <int W, int aux>
__device__ __forceinline__ void nib_store(__amdgpu_buffer_rsrc_t r, uint32_t off, const uint32_t* v) {
  if constexpr (W == 1) {
    __builtin_amdgcn_raw_buffer_store_b32(v[0], r, (int)off, 0, aux);
  } else if constexpr (W == 2) {
    typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
    __builtin_amdgcn_raw_buffer_store_b64(u32x2{v[0], v[1]}, r, (int)off, 0, aux);
  } else {
    __builtin_amdgcn_raw_buffer_store_b128(v4u{v[0], v[1], v[2], v[3]}, r, (int)off, 0, aux);
  }
}

// Tile and row block of nibble workgroup bid (the XCD-aware map: XCD x =
// bid % 8 sweeps tiles x, x + 8, ...); k_round_jobs walks the same regions.
template <int TW>
__device__ __forceinline__ void nib_region(const GhDev& d, const GhRound& p, int bid, int& tile, int& rb) {
  constexpr int RB = round_rb<TW>();
  const int nrb = (int)((d.nrows + RB - 1) / RB);
  const int ngroups = (int)(p.ld / TW);
  if (p.xmap && ngroups % 8 == 0) {
    const int x = bid & 7, j = bid >> 3;
    tile = x + 8 * (j / nrb);
    rb = j - (j / nrb) * nrb;
    // (xmap 2: odd rounds sweep the tiles from the other end, starting on
    // the slices the last round wrote last)
    if (p.xmap == 2 && (p.r & 1)) tile = ngroups - 1 - tile;
  } else {
    tile = bid / nrb;
    rb = bid - tile * nrb;
  }
}

// Per nibble of x: 1 (bit 0) where the nibble is 15.
__device__ __forceinline__ uint32_t nib_is15(uint32_t x) {
  const uint32_t e = ~x;
  uint32_t t = e | (e >> 2);
  t |= t >> 1;
  return ~t & 0x11111111u;
}
// The nibble path's rule on one dword (8 cells) of a lane: own lag word qw,
// age word aw, the senders' lag words p0..p3, a1 = nib_is15(qw), dn = the
// base moves. L = min(own, senders) per nibble is the next code before the
// rebase (merged iff it differs from the own code); a nibble add or compare
// that carries marks the lane out of the tier (a lane job), so no guard bits
// are needed. tt (wave-uniform): the wave holds own code-15 cells, which may be tier
// tombstones (code 15, age nibble 1..14): age nibble 14 is older than
// T_cleanup and released (step 5, :490-492: absent, and merges like one),
// the others keep code 15 and age by one, never merged. Without tt no own
// cell has code 15.
// RMV: the lane holds REMOVE'd members (rm1: bit 0 of their nibbles; step 1,
// slave/slave.go:236-240, 276-286), each with two or more detectors, so every
// sender REMOVEs it before sending (no entry) and the row applies
// removeMember: a present cell becomes a tombstone that keeps its ts, i.e. the
// tier cell (15, s) with s = age + 1 - toff (rmk = (16 - toff) per byte;
// T_cleanup >= 15, so no tier age is past it and none is released here), a
// tombstone stays one, and an absent one (the reference panics; counted
// remove_unknown) or a tombstone too young for the tier leaves the lane to
// the lane-job kernel.
// PRE: p0 is already the senders' per-nibble minimum (p1..p3 unused).
template <bool RMV, bool PRE = false>
__device__ __forceinline__ void nib_word(bool tt, uint32_t qw, uint32_t aw, uint32_t p0, uint32_t p1, uint32_t p2,
                                         uint32_t p3, uint32_t a1, uint32_t dn, uint32_t tfk, uint32_t rm1, uint32_t rs1,
                                         uint32_t rmk, uint32_t& QO, uint32_t& AO, uint32_t& LWo, uint32_t& Bm, uint32_t& Lz,
                                         int& mrg, int& gain, int& rel, int& tmb) {
  constexpr uint32_t N1 = 0x11111111u;
  uint32_t Lw = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const uint32_t M = 0x000F000Fu << (4 * j);
    if constexpr (PRE)
      Lw |= pk_min_u16(qw & M, p0 & M);
    else
      Lw |= pk_min_u16(pk_min_u16(pk_min_u16(qw & M, p0 & M), pk_min_u16(p1 & M, p2 & M)), p3 & M);
  }
  uint32_t bad = 0;
  uint32_t pr1 = 0, PRm = 0;  // RMV: present cells REMOVE'd this round
  if constexpr (RMV) {
    const uint32_t RM = rm1 * 15u;
    Lw = (Lw & ~RM) | (qw & RM);  // no sender entry: never merged
    pr1 = rm1 & ~a1;
    PRm = pr1 * 15u;
  }
  uint32_t kp1 = 0, KM = 0;
  if (tt) {
    // a code-15 cell with age nibble s: absent (15), a tombstone released
    // this round (14: its age is T_cleanup + 1, gh_tier_toff), or a kept
    // tombstone (1..13); an escaped chunk's age word is 0 (the lane is a
    // job, whose merge candidates are the plain minimum)
    const uint32_t h3 = (aw >> 1) & (aw >> 2) & (aw >> 3) & N1;  // s >= 14
    kp1 = gh_t4_esc(aw) ? 0u : a1 & ~h3;
    KM = kp1 * 15u;
    Lw |= KM;  // a kept tombstone takes no entry
    rel += __builtin_popcount(a1 & h3 & ~aw);
    // REMOVE of an absent member (remove_unknown), or a release where the
    // member's sole detector may send it: lane jobs
    if constexpr (RMV) bad |= (rm1 & a1 & h3 & aw) | (rs1 & a1 & h3 & ~aw);
  }
  // a sender code unknown (0) or old (14) that the own code does not beat
  Lz |= nib_haszero(Lw) | nib_haszero(Lw ^ 0xEEEEEEEEu);
  LWo = Lw;
  const uint32_t D = Lw ^ qw;
  uint32_t t = D | (D >> 2);
  t |= t >> 1;
  const uint32_t m1 = t & N1;            // merged (bit 0 of the nibble)
  const uint32_t an1 = a1 & ~m1 & ~kp1;  // absent (or released), not merged: stays (15, 15)
  const uint32_t ANm = an1 * 15u;
  const uint32_t MM = m1 * 15u;
  const uint32_t ST = ANm | KM | PRm;    // cells whose code is 15 after the round
  const uint32_t ddx = dn & ~ST;
  const uint32_t S = Lw + ddx;  // next code, rebased
  bad |= ((Lw ^ ddx ^ S) & (N1 - 1u)) | (S < Lw ? 1u : 0u);  // a code past 15 (carry into the next nibble)
  const uint32_t s1 = S >> 1, s2 = S >> 2, s3 = S >> 3;
  bad |= ((s1 & s2 & s3) | ~(s1 | s2 | s3)) & N1 & ~(an1 | kp1 | pr1);  // a code of 14, 15 or below 2
  const uint32_t ag = aw & ~(MM | ANm | PRm);                           // ages that grow by one (kept tombstones to 14 at most)
  const uint32_t inc = N1 & ~(m1 | an1 | pr1);
  const uint32_t T = ag + inc;
  bad |= ((ag ^ inc ^ T) & (N1 - 1u)) | (T < ag ? 1u : 0u);  // an age past 15
  const uint32_t AN = T | m1 | ANm;  // merged: age 1; absent: 15
  const uint32_t X = AN & ~ST;       // ages above min(T_fail, 15)
  const uint32_t K = tfk & ~ST;
  const uint32_t V = X + K;
  bad |= ((X ^ K ^ V) & (N1 - 1u)) | (V < X ? 1u : 0u);
  QO = S;
  AO = AN;
  if constexpr (RMV) {
    // the new tombstones' age nibbles, per byte without carries between
    // nibbles: a + 15 - (toff - 1) carries iff s = a + 1 - toff >= 1 (s <= 14
    // always: a <= 15, toff >= 2), and its low nibble is s - 1
    const uint32_t Xa = aw & PRm;
    const uint32_t Ve = (Xa & 0x0F0F0F0Fu) + rmk, Vo = ((Xa >> 4) & 0x0F0F0F0Fu) + rmk;
    const uint32_t ok = ((Ve >> 4) & 0x01010101u) | (((Vo >> 4) & 0x01010101u) << 4);
    const uint32_t sn = ((Ve & 0x0F0F0F0Fu) + 0x01010101u) | (((Vo & 0x0F0F0F0Fu) + 0x01010101u) << 4);
    bad |= pr1 & ~ok;
    QO |= PRm;
    AO |= sn & PRm;
    tmb += __builtin_popcount(pr1);
  }
  Bm |= bad;
  mrg += __builtin_popcount(m1);
  gain += __builtin_popcount(m1 & a1);
}

// ROWS (row layout, IN = 4): a sender is an owned row of this shard (its
// plane segment in the tile slice, as with columns) or a ghost row whose
// plane words the round's exchange put in the ghost table (row-major,
// gplane); the gathers then take per-sender 64-bit addresses staged in LDS.
// DMA (one engine or column shards, 16 cells per lane): each wave stages its
// 8 rows of a step into its own LDS region by LDS-DMA (buffer_load_dwordx4
// ... lds, 16 B per lane: the own lag and age lines as two 1-KiB pieces, the
// 32 sender lines as four), then computes them on ds_read_b64 in the 16-cell
// lane shape: half the vector-memory load instructions of 8-B register loads,
// and no VGPRs held by loads in flight.
// SPL (16-cell lanes, 256-member tiles; not with DMA): lanes
// m and m + 8 of a row's 16 share 32 cells; lane m gathers 16 B of those
// cells from senders 0 and 1, lane m + 8 from senders 2 and 3 (2 gathers of
// 16 B per row step instead of 4 of 8 B: each wave instruction then touches 8
// lines instead of 4, which halves the gather instructions the TA issues),
// each takes the per-nibble min of its two, the halves swap by DPP
// (row_ror 8), and each lane finishes its own 16 cells (m * 32 + 16 h for
// half h). In the probe (`tools/r05/gprobe4.hip`, a trivial rule at 38
// VGPRs) 1.73-1.84 ms against 1.96-2.24 ms; in the kernel (70 VGPRs, the
// full rule) 2.10-2.12 ms against 1.98-2.01 ms (`profiles/r05_s16_ab_split.txt`):
// off (GH_NIB_SPLIT=0), kept as an A/B build option.
// RMVK: the instantiation that can take REMOVE deliveries itself (nib_word
// RMV); the other one (the steady state's: 10 VGPRs fewer, 7 waves per SIMD
// instead of 6) hands every lane holding a REMOVE'd member to the lane jobs.
// k_round runs the RMV one only in rounds with a pending REMOVE (IN 6).
template <int TW, bool NT, int CPL, bool ROWS, bool DMA = false, bool RMVK = true>
__device__ __forceinline__ void round_block_nib(const GhDev& d, const int cur, const int dcur, const GhRound& p,
                                                const int bid) {
  constexpr int W = CPL / 8;         // dwords per lane and plane
  constexpr int SEG = TW / CPL;      // lanes per row segment
  constexpr int RPW = 64 / SEG;      // rows per wave instruction
  constexpr int RSTEP = 4 * RPW;     // rows per workgroup step
  constexpr int RB = round_rb<TW>();
  constexpr int KB = 4;
  constexpr int RS = GH_NIB_RS > 0 ? GH_NIB_RS : (CPL <= 16 ? 2 : 1);  // row steps per iteration
  static_assert(SEG >= 2 && SEG <= 64 && RB % (RSTEP * RS) == 0, "nibble path: whole row steps");
  static_assert(W == 2 || W == 4, "nibble path: 16 or 32 cells per lane (one or two lane jobs of 16 cells)");
  static_assert(!DMA || (!ROWS && CPL == 16 && TW == 256 && RB % 32 == 0), "LDS-DMA staging: 16-cell lanes, 256-member tiles");
  constexpr int RSD = DMA ? 2 : RS;  // row steps per iteration (DMA: a wave's 8 consecutive rows)
  constexpr bool SPL = (ROWS ? GH_NIB_SPLIT_ROWS : GH_NIB_SPLIT) && !DMA && CPL == 16 && TW == 256;
  // per wave: own lag 1 KiB, age 1 KiB, the 4 gather pieces (sender slot q
  // of the 8 rows) 1 KiB each
  __shared__ __attribute__((aligned(16))) uint32_t s_dma[DMA ? 4 * 1536 : 1];
  constexpr int H = W / 2;  // lane jobs of GH_JOB_CPL cells per job lane
  __shared__ unsigned long long s_merged, s_rel, s_tmb;
  __shared__ int s_quiet, s_nslow, s_slowbase, s_bmove, s_hasjob;
  __shared__ unsigned long long s_d8bad;  // bit l: lane l's columns hold a base move outside 0..15
  // per chunk the base moves as one nibble word in the plane's nibble order
  // (cell j at gh_nib(j))
  __shared__ __attribute__((aligned(16))) uint32_t s_dn[TW / 8];
  __shared__ int s_slow[RB];
  __shared__ int s_meta[RB];
  __shared__ __attribute__((aligned(16))) int s_inb[ROWS ? 4 : RB * KB];
  __shared__ __attribute__((aligned(16))) unsigned long long s_inb64[ROWS ? RB * KB : 2];
  __shared__ int s_need;  // ROWS: a lane job gathers its senders' 16-bit codes (ghosts' codes must travel)

  const int rowend = (int)(d.row0 + d.nrows);
  int tile, rb;
  nib_region<TW>(d, p, bid, tile, rb);
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = uni(tid >> 6);
  const int sub = lane / SEG, lc = lane % SEG;
  const unsigned long long gmask = (SEG == 64 ? ~0ull : ((1ull << SEG) - 1)) << (sub * SEG);
  // the lane's first cell in the tile and its CPL-cell group (SPL: m * 32 + 16 h)
  const int lcell = SPL ? 32 * (lc & 7) + 16 * (lc >> 3) : lc * CPL;
  const int lgrp = lcell / CPL;
  const int64_t l0 = (int64_t)tile * TW + lcell;  // local column of this lane's first cell
  // the lane's REMOVE'd members (D_{r-1}), loaded beside the staging below
  uint32_t rm = 0;
#pragma unroll
  for (int w = 0; w < (CPL + 31) / 32; ++w) rm |= d.dbits[(l0 >> 5) + w];
  if constexpr (CPL < 32) rm = (rm >> (l0 & 31)) & ((1u << CPL) - 1u);
  if (tid == 0) {
    s_merged = s_rel = s_tmb = 0;
    s_quiet = s_nslow = s_bmove = s_hasjob = s_need = 0;
    s_d8bad = 0ull;
  }
  const bool pull = p.peer_mode == GH_PEER_PULL;
  const bool quiet = d.cntg[p.n] == 0 && !p.force_slow && !d.m8[2];
  const uint8_t* __restrict__ stab_cur = d.stab[p.r & 1];
  __syncthreads();
  if (!ROWS && d.nsnd) {  // k_peers_pull's row records (one engine)
    for (int row = tid; row < RB; row += 256) {
      const int i = (int)d.row0 + rb * RB + row;
      int meta = 0;
      int4 sv = {0, 0, 0, 0};
      if (i < rowend) {
        meta = d.nmeta[i];
        sv = *reinterpret_cast<const int4*>(d.nsnd + 4 * (int64_t)i);
      }
      s_meta[row] = meta;
      *reinterpret_cast<int4*>(&s_inb[row * KB]) = int4{sv.x * (TW / 2), sv.y * (TW / 2), sv.z * (TW / 2), sv.w * (TW / 2)};
    }
  }
  for (int t = tid; t < ((!ROWS && d.nsnd) ? 0 : RB * KB); t += 256) {
    const int row = t / KB, q = t - row * KB;
    const int i = (int)d.row0 + rb * RB + row;
    int meta = 0, sv = 0;
    if (i < rowend) {
      const int al = d.alive[i];
      const int cnt = al ? gh_in_cnt(d, pull, p.k, i) : 0;
      const int act = d.active[i];
      meta = al | (act << 1) | (cnt << 2) | ((quiet && al && !act && cnt == 0 && stab_cur[i]) ? 1 << 30 : 0);
      // the sender's plane row segment as a byte offset in the tile slice;
      // unused slots read the own row's (a no-op under the merge)
      if constexpr (ROWS) {
        const int64_t sslot = q < cnt ? d.rslot[d.inbox[gh_in_beg(d, pull, p.k, i) + q]] : i - d.row0;
        const char* a = sslot < d.nrows
                            ? reinterpret_cast<const char*>(d.pl[cur]) + ((int64_t)tile * d.tstride + sslot * TW) / 2
                            : reinterpret_cast<const char*>(d.gplane) + (sslot - d.nrows) * (d.ld / 2) + tile * (TW / 2);
        s_inb64[t] = reinterpret_cast<unsigned long long>(a);
      } else {
        sv = (q < cnt ? d.inbox[gh_in_beg(d, pull, p.k, i) + q] : (int)(i - d.row0)) * (TW / 2);
      }
    } else if constexpr (ROWS) {
      s_inb64[t] = reinterpret_cast<unsigned long long>(d.pl[cur]);  // (never read: the row is idle)
    }
    if (q == 0) s_meta[row] = meta;
    if constexpr (!ROWS) s_inb[t] = sv;
  }
  const int32_t* __restrict__ bo = d.base[cur];
  const int32_t* __restrict__ bn = d.base[cur ^ 1];
  if (d.dnw) {  // base_col's move words (column layout)
    for (int w = tid; w < TW / 8; w += 256) {
      const int64_t wc = (int64_t)tile * (TW / 8) + w;
      const uint32_t x = d.dnw[wc];
      const uint32_t bd = d.dbad[wc];
      s_dn[w] = x;
      if (bd) atomicOr(&s_d8bad, 1ull << (w * 8 / CPL));
      if (x | bd) s_bmove = 1;
    }
  } else {
    for (int cc = tid; cc < TW; cc += 256) {
      const int64_t c = (int64_t)tile * TW + cc;
      const int64_t delta = (int64_t)bn[c] - bo[c];
      if (delta < 0 || delta > 15) atomicOr(&s_d8bad, 1ull << (cc / CPL));
      if (delta) s_bmove = 1;
    }
    for (int w = tid; w < TW / 8; w += 256) {
      uint32_t x = 0;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int64_t c = (int64_t)tile * TW + 8 * w + j;
        x |= (uint32_t)((bn[c] - bo[c]) & 0xF) << gh_nib(j);
      }
      s_dn[w] = x;
    }
  }
  __syncthreads();

  const int c0 = (int)(d.col0 + l0);
  const int64_t tcell = (int64_t)tile * d.tstride;
  const int64_t tbytes = d.tstride / 2;  // one tile slice of a plane
  const auto plo_t = nib_rsrc(reinterpret_cast<const char*>(d.pl[cur]) + tcell / 2, tbytes);
  const auto pln_t = nib_rsrc(reinterpret_cast<const char*>(d.pl[cur ^ 1]) + tcell / 2, tbytes);
  const auto a4o_t = nib_rsrc(reinterpret_cast<const char*>(d.a4[cur]) + tcell / 2, tbytes);
  const auto a4n_t = nib_rsrc(reinterpret_cast<const char*>(d.a4[cur ^ 1]) + tcell / 2, tbytes);
  const uint32_t lbp = (uint32_t)lcell / 2;  // the lane's byte offset in a plane row segment
  const uint32_t gbp = (uint32_t)(lc & 7) * 16;  // SPL: the lane pair's 16 B of a sender's segment
  const bool tile_still = s_bmove == 0;
  // REMOVE'd members on the nibble path (nib_word RMV): canonical recipients
  // (every running row but a sole detector, SPEC D4) and tier tombstones with
  // T_cleanup >= 15 (toff >= 2; GH_NIB_RMV=0 in the environment restores the
  // lane jobs). A member with one detector: that row keeps its own cell (it
  // is a lane job there, rmrow), and the detector may send the member, so a
  // cell that is absent after step 5 (a tombstone released this round, RS1)
  // is a lane job; a lane with two such members of different detectors is a
  // lane job in every row.
  bool rmv = false;
  int rmrow = -1;
  uint32_t rs = 0;  // the lane's REMOVE'd cells whose member has one detector
  if (RMVK && p.nib_rmv && rm != 0u && !d.rlist && d.toff >= 2) {
    rmv = true;
    for (uint32_t m = rm; m; m &= m - 1u) {
      const int j = __builtin_ctz(m);
      if (d.det_cnt[dcur][l0 + j] == 1) {
        const int dm = d.det_min[dcur][l0 + j];
        rmv &= rmrow < 0 || rmrow == dm;
        rmrow = dm;
        rs |= 1u << j;
      }
    }
  }
  uint32_t RM1[W], RS1[W];  // per dword, bit 0 of each REMOVE'd cell's nibble (all; one detector)
#pragma unroll
  for (int w = 0; w < W; ++w) {
    const uint32_t b8 = rmv ? (rm >> (8 * w)) & 0xFFu : 0u, s8 = rmv ? (rs >> (8 * w)) & 0xFFu : 0u;
    uint32_t x = 0, y = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      x |= ((b8 >> j) & 1u) << gh_nib(j);
      y |= ((s8 >> j) & 1u) << gh_nib(j);
    }
    RM1[w] = x;
    RS1[w] = y;
  }
  const bool wrmv = RMVK && __ballot(rmv) != 0;  // (wave-uniform)
  const uint32_t rmk = (uint32_t)(15 - (d.toff - 1)) * 0x01010101u;
  // the lane needs the per-cell rule (a lane job) in every row when it holds
  // a REMOVE'd member off the RMV path or a base move outside 0..15
  const bool lane_job = (rm != 0u && !rmv) || ((s_d8bad >> lgrp) & 1ull) != 0;
  // this wave's lane-job region (no atomics: the wave owns it)
  uint4* __restrict__ jreg = d.jobs + ((int64_t)bid * 4 + wave) * GH_JOB_CAP * 2;
  int wjobs = 0;
  uint32_t DN[W];  // the base moves of dword w, nibble order
#pragma unroll
  for (int x = 0; x < W; ++x) DN[x] = s_dn[lgrp * W + x];
  const uint32_t tfk = (uint32_t)(15 - min(max(p.t_fail, 0), 15)) * 0x11111111u;  // age + tfk carries iff age > T_fail
  uint32_t n_mrg = 0, n_rel = 0, n_tmb = 0;

#pragma unroll 1
  for (int it = 0; it < RB / RSTEP; it += RSD) {
    int iu[RSD];
    bool alu[RSD], oku[RSD];
    uint32_t owu[RSD];
    NibWords<W> awu[RSD], qwu[RSD], pwu[RSD][4];
    char* wb = reinterpret_cast<char*>(s_dma) + (DMA ? wave * 6144 : 0);
    if constexpr (DMA) {
      // the wave's rows it * RSTEP + wave * 8 .. + 7 of the block: their own
      // lines are one contiguous KiB of each plane's tile slice; DMA lane l
      // moves bytes [16 l, 16 l + 16), and for sender slot q the 16 B at
      // (l % 8) * 16 of row l / 8's sender line (hipcc does not wait for an
      // LDS-DMA: the waits are explicit)
      typedef __attribute__((address_space(3))) void lds_t;
      const int rbase = it * RSTEP + wave * 8;
      const uint32_t own = (uint32_t)(rb * RB + rbase) * (TW / 2) + (uint32_t)lane * 16u;
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the previous step's LDS reads are done
      __builtin_amdgcn_raw_ptr_buffer_load_lds(plo_t, (lds_t*)wb, 16, (int)own, 0, 0, GH_NIB_OWN_AUX);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(a4o_t, (lds_t*)(wb + 1024), 16, (int)own, 0, 0, GH_NIB_AGE_AUX);
      const int4 sv4 = *reinterpret_cast<const int4*>(&s_inb[(rbase + (lane >> 3)) * KB]);
      const uint32_t dcol = (uint32_t)(lane & 7) * 16u;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(plo_t, (lds_t*)(wb + 2048), 16, (int)((uint32_t)sv4.x + dcol), 0, 0,
                                               GH_NIB_GAT_AUX);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(plo_t, (lds_t*)(wb + 3072), 16, (int)((uint32_t)sv4.y + dcol), 0, 0,
                                               GH_NIB_GAT_AUX);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(plo_t, (lds_t*)(wb + 4096), 16, (int)((uint32_t)sv4.z + dcol), 0, 0,
                                               GH_NIB_GAT_AUX);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(plo_t, (lds_t*)(wb + 5120), 16, (int)((uint32_t)sv4.w + dcol), 0, 0,
                                               GH_NIB_GAT_AUX);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
#pragma unroll
    for (int u = 0; u < RSD; ++u) {
      const int rr = DMA ? it * RSTEP + wave * 8 + u * RPW + sub : wave * RPW + (it + u) * RSTEP + sub;
      const int i_raw = (int)d.row0 + rb * RB + rr;
      const bool valid = i_raw < rowend;
      const int i = valid ? i_raw : rowend - 1;  // in-range row for the loads of idle lanes
      const int rs = valid ? rr : 0;
      const int meta = s_meta[rs];
      const bool skip = ((meta >> 30) & 1) && tile_still;  // quiet row, bases still
      if (valid && skip && lc == 0) atomicAdd(&s_quiet, 1);
      const int cntv = (meta >> 2) & 0x0FFFFFFF;  // bits 2..29: a ring receiver can have N - 1 senders
      alu[u] = (meta & 1) && valid && !skip;
      oku[u] = ((meta >> 1) & 1) && cntv <= KB;  // active (not a guard row), at most KB senders
      iu[u] = i;
      const uint32_t islot = (uint32_t)(i - d.row0);
      const uint32_t ow = islot * (TW / 2) + lbp;
      owu[u] = ow;
      if constexpr (DMA) {
        const int o = (u * RPW + sub) * (TW / 2) + (int)lbp;
        typedef uint32_t u2 __attribute__((ext_vector_type(2)));
        const u2 q2 = *reinterpret_cast<const u2*>(wb + o);
        const u2 a2 = *reinterpret_cast<const u2*>(wb + 1024 + o);
        qwu[u].v[0] = q2[0], qwu[u].v[1] = q2[1];
        awu[u].v[0] = a2[0], awu[u].v[1] = a2[1];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const u2 g2 = *reinterpret_cast<const u2*>(wb + 2048 + q * 1024 + o);
          pwu[u][q].v[0] = g2[0], pwu[u][q].v[1] = g2[1];
        }
        continue;
      }
      // the age words are read once (no peer reads them): they stream past
      // the caches the plane lines live in; the own plane words are a line
      // the row's receivers gather too
      awu[u] = nib_load<W, GH_NIB_AGE_AUX>(a4o_t, ow);
      qwu[u] = nib_load<W, GH_NIB_OWN_AUX>(plo_t, ow);
      if constexpr (ROWS && SPL) {
        // (the pair's 16 B of senders 2h, 2h + 1, as below)
        typedef uint32_t gw4 __attribute__((ext_vector_type(4)));
        typedef const __attribute__((address_space(1))) gw4 ggw4;
        const int q0 = (lc >> 3) != 0 ? 2 : 0;
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          const gw4 x = *reinterpret_cast<ggw4*>(s_inb64[rs * KB + q0 + t] + gbp);
          pwu[u][2 * t].v[0] = x[0], pwu[u][2 * t].v[1] = x[1];
          pwu[u][2 * t + 1].v[0] = x[2], pwu[u][2 * t + 1].v[1] = x[3];
        }
      } else if constexpr (ROWS) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          typedef uint32_t gw __attribute__((ext_vector_type(W)));
          typedef const __attribute__((address_space(1))) gw ggw;
          const gw x = *reinterpret_cast<ggw*>(s_inb64[rs * KB + q] + lbp);
#pragma unroll
          for (int w = 0; w < W; ++w) pwu[u][q].v[w] = x[w];
        }
      } else {
        const int4 sv4 = *reinterpret_cast<const int4*>(&s_inb[rs * KB]);
        const int sv[4] = {sv4.x, sv4.y, sv4.z, sv4.w};
        if constexpr (SPL) {
          // senders 2h, 2h + 1 of the row, 16 B each (pwu[u][0..1]: the first,
          // pwu[u][2..3]: the second)
          const bool h1 = (lc >> 3) != 0;
#pragma unroll
          for (int t = 0; t < 2; ++t) {
            const NibWords<4> x = nib_load<4, GH_NIB_GAT_AUX>(plo_t, (uint32_t)(h1 ? sv[2 + t] : sv[t]) + gbp);
            pwu[u][2 * t].v[0] = x.v[0], pwu[u][2 * t].v[1] = x.v[1];
            pwu[u][2 * t + 1].v[0] = x.v[2], pwu[u][2 * t + 1].v[1] = x.v[3];
          }
        } else {
#pragma unroll
          for (int q = 0; q < 4; ++q) pwu[u][q] = nib_load<W, GH_NIB_GAT_AUX>(plo_t, (uint32_t)sv[q] + lbp);
        }
      }
    }
#pragma unroll
    for (int u = 0; u < RSD; ++u) {
      const int i = iu[u];
      const bool al = alu[u];
      uint32_t QO[W], AO[W], LW[W], A1[W], Bm = 0, Lz = 0;
      int mrg = 0, gain = 0, rel = 0, tmb = 0;
      bool esc = false;
      uint32_t a1any = 0;
#pragma unroll
      for (int w = 0; w < W; ++w) {
        esc |= gh_t4_esc(awu[u].v[w]);
        A1[w] = nib_is15(qwu[u].v[w]);
        a1any |= A1[w];
      }
      // (wave-uniform) the wave's own cells include code 15 (absent or a tier
      // tombstone): the rule ages and releases tombstones
      const bool tt = GH_TIER_TOMB && (!GH_TIER_TOMB_GATE || __ballot(a1any != 0) != 0);
      if constexpr (SPL) {
        // the pair's 32 cells: the min of my two senders over them; I keep
        // my half's dword w and send the partner its half's (DPP row_ror 8:
        // lane m <-> m + 8 of the same row), then the min of the two is my
        // senders' minimum
        const bool h1 = (lc >> 3) != 0;
        uint32_t PS[2];
#pragma unroll
        for (int w = 0; w < 2; ++w) {
          uint32_t lo = 0, hi = 0;  // cells of half 0 / half 1, dword w
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const uint32_t M = 0x000F000Fu << (4 * j);
            lo |= pk_min_u16(pwu[u][0].v[w] & M, pwu[u][2].v[w] & M);
            hi |= pk_min_u16(pwu[u][1].v[w] & M, pwu[u][3].v[w] & M);
          }
          const uint32_t keep = h1 ? hi : lo;
          const uint32_t got = (uint32_t)__builtin_amdgcn_mov_dpp((int)(h1 ? lo : hi), 0x128, 0xF, 0xF, false);
          uint32_t mn = 0;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const uint32_t M = 0x000F000Fu << (4 * j);
            mn |= pk_min_u16(keep & M, got & M);
          }
          PS[w] = mn;
        }
        if (wrmv) {
#pragma unroll
          for (int w = 0; w < W; ++w)
            nib_word<true, true>(tt, qwu[u].v[w], awu[u].v[w], PS[w], 0u, 0u, 0u, A1[w], DN[w], tfk, RM1[w], RS1[w], rmk,
                                 QO[w], AO[w], LW[w], Bm, Lz, mrg, gain, rel, tmb);
        } else {
#pragma unroll
          for (int w = 0; w < W; ++w)
            nib_word<false, true>(tt, qwu[u].v[w], awu[u].v[w], PS[w], 0u, 0u, 0u, A1[w], DN[w], tfk, 0u, 0u, 0u, QO[w],
                                  AO[w], LW[w], Bm, Lz, mrg, gain, rel, tmb);
        }
      } else if (wrmv) {
#pragma unroll
        for (int w = 0; w < W; ++w)
          nib_word<true>(tt, qwu[u].v[w], awu[u].v[w], pwu[u][0].v[w], pwu[u][1].v[w], pwu[u][2].v[w], pwu[u][3].v[w],
                         A1[w], DN[w], tfk, RM1[w], RS1[w], rmk, QO[w], AO[w], LW[w], Bm, Lz, mrg, gain, rel, tmb);
      } else {
#pragma unroll
        for (int w = 0; w < W; ++w)
          nib_word<false>(tt, qwu[u].v[w], awu[u].v[w], pwu[u][0].v[w], pwu[u][1].v[w], pwu[u][2].v[w], pwu[u][3].v[w],
                          A1[w], DN[w], tfk, 0u, 0u, 0u, QO[w], AO[w], LW[w], Bm, Lz, mrg, gain, rel, tmb);
      }
      bool ob = false;
      const int jd = i - c0;
      // (a wave-uniform branch: 1 wave in TW / CPL... holds an own member)
      if (__ballot((unsigned)jd < (unsigned)CPL) != 0 && (unsigned)jd < (unsigned)CPL) {
        // the row's own member (step 3, :443-448): hb + 1 with a fresh
        // stamp, never flagged; the rule above merged and rebased it on its
        // diagonal code, whose written code is one lower (the snapshot
        // carries hb + 1) and whose age is 1. Absent, a guard row or at the
        // heartbeat cap: the per-cell rule
        const int wj = jd >> 3, sh = gh_nib(jd & 7);
#pragma unroll
        for (int x = 0; x < W; ++x)
          if (x == wj) {
            const int qd = (int)((qwu[u].v[x] >> sh) & 0xFu);
            ob = qd == 15 || (int64_t)bo[l0 + jd] + (GH_P_REF - qd) >= INT32_MAX || ((rm >> jd) & 1u);
            QO[x] -= 1u << sh;
            AO[x] = (AO[x] & ~(0xFu << sh)) | (1u << sh);
          }
      }
      // a row under the <4 guard, with more than KB senders (or every row,
      // GH_FORCE_SLOW) sends its whole segment to the slow list; in any other
      // row a lane whose cells leave the tier or need the per-cell rule is a
      // lane job (k_round_jobs), and the segment's other lanes are written here
      const bool rowok = oku[u] && !p.force_slow && i != p.shadow_row;  // (D7 shadows: the per-cell rule)
      const bool jb = al && rowok && (lane_job || esc || ob || Bm != 0 || Lz != 0 || i == rmrow);
      const unsigned long long jm = __ballot(jb);
      // a job whose rule gathers its senders' 16-bit codes (a REMOVE'd member,
      // an unknown or old minimum): with ghost senders, their codes travel
      if constexpr (ROWS) {
        // (a REMOVE'd member's only carrier is its sole detector, whose
        // candidate soleval holds: no codes for those)
        const bool rm_codes = rm != 0u && (d.rlist || !d.soleval);
        if (__ballot(jb && (rm_codes || Lz != 0)) != 0 && lane == 0) s_need = 1;
      }
      bool jslow = false;
      if (jm) {
        const int nj = __popcll(jm);
        if (wjobs + H * nj <= GH_JOB_CAP) {
          if (jb) {
            const int pos = wjobs + H * (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(jm >> 32),
                                                                        __builtin_amdgcn_mbcnt_lo((uint32_t)jm, 0u));
            // per 16 cells a job: row, tile and 16-cell lane, the minimum
            // plane words; then the lane's own lag and age words (the job
            // kernel needs not re-read them)
#pragma unroll
            for (int h = 0; h < H; ++h) {
              jreg[2 * (pos + h)] = uint4{(uint32_t)i, ((uint32_t)tile << 8) | (uint32_t)(lgrp * H + h), LW[2 * h],
                                          LW[2 * h + 1]};
              jreg[2 * (pos + h) + 1] = uint4{qwu[u].v[2 * h], qwu[u].v[2 * h + 1], awu[u].v[2 * h], awu[u].v[2 * h + 1]};
            }
          }
          wjobs += H * nj;
        } else {
          jslow = (jm & gmask) != 0;  // the wave's region is full: segments with jobs go slow, whole
        }
      }
      const bool seg_slow = jslow || (__ballot(al && !rowok) & gmask) != 0;
      int dpres = 0;
      if (al && !seg_slow && !jb) {
        nib_store<W, NT ? GH_NIB_ST_AUX : 0>(pln_t, owu[u], QO);
        nib_store<W, NT ? GH_NIB_ST_AUX : 0>(a4n_t, owu[u], AO);
        n_mrg += (uint32_t)mrg;
        n_rel += (uint32_t)rel;
        n_tmb += (uint32_t)tmb;
        dpres = gain - tmb;
      } else if (al && seg_slow && lc == 0) {
        s_slow[atomicAdd(&s_nslow, 1)] = i;
      }
      if (__ballot(dpres != 0) != 0) {  // absent cells merged, present ones REMOVE'd: the row's count moves
#pragma unroll
        for (int o2 = SEG / 2; o2 > 0; o2 >>= 1) dpres += __shfl_xor(dpres, o2);
        if (lc == 0 && dpres) atomicAdd(&d.cntl[i], dpres);
      }
    }
  }

  if (lane == 0) {
    d.jobn[(int64_t)bid * 4 + wave] = wjobs;
    if (wjobs) s_hasjob = 1;
  }
  if (n_mrg) atomicAdd(&s_merged, (unsigned long long)n_mrg);
  if (n_rel) atomicAdd(&s_rel, (unsigned long long)n_rel);
  if (n_tmb) atomicAdd(&s_tmb, (unsigned long long)n_tmb);
  __syncthreads();
  if (tid == 0) {
    if (s_nslow) s_slowbase = atomicAdd(d.slow_n, s_nslow);
    if (s_merged) atomicAdd(&d.stats[ST_MERGED], s_merged);
    if (s_rel) atomicAdd(&d.stats[ST_RELEASED], s_rel);
    if (s_tmb) atomicAdd(&d.stats[ST_TOMBSTONED], s_tmb);
    if (s_quiet) atomicAdd(d.nquiet, s_quiet);
    if (s_hasjob) d.jlist[atomicAdd(&d.njobs[3], 1)] = bid;  // k_round_jobs walks the listed workgroups only
    if (ROWS && s_need) d.m8[5] = 1;
  }
  __syncthreads();
  for (int t = tid; t < s_nslow; t += 256) d.slow[s_slowbase + t] = ((int64_t)tile << 32) | (uint32_t)s_slow[t];
}

// IN: 0 = a 16-bit input (full grid), 1 = a tier input by the 16-bit rule
// (widened), 3 = a 16-bit input in a tiered engine (rarely selected: a
// persistent 1/8 grid); IN = 2 (a tier input by the nibble path) is
// round_block_nib above
template <int KB, int TW, int TPW, bool NT, bool STORM, int IN>
__device__ __forceinline__ void round_block(const GhDev& d, const int cur, const int dcur, const GhRound& p,
                                            const int bid) {
  constexpr int CPL = 8;
  constexpr int SEG = TW / CPL;
  constexpr int RPW = 64 / SEG;
  constexpr int RSTEP = 4 * RPW;
  constexpr int RB = round_rb<TW>();  // rows per workgroup tile
  __shared__ unsigned long long s_merged, s_det, s_rel, s_storm, s_tomb, s_unk;
  __shared__ int s_quiet;  // row segments skipped as quiet
  // this tile's per-pair constants: rebase (base_next - base_cur) << 5
  // (0x8000: jump beyond 1023, no present cell stays narrow) and the code
  // bound of "hb > 1"
  __shared__ uint32_t s_d5[TW / 2];
  __shared__ uint32_t s_t5[TW / 2];
  // REMOVE of D_{r-1} per pair: 0xFFFF halves for columns with >= 2
  // detectors (every row removes them); s_rm1: a column with one detector
  __shared__ uint32_t s_rm[TW / 2];
  __shared__ uint32_t s_rm1[TW / 2];
  // this tile's detections per column (count, first detector)
  __shared__ int s_dcnt[TW];
  __shared__ int s_dmin[TW];
  // this tile's segments for the slow list, appended with one global atomic
  __shared__ int s_nslow, s_slowbase;
  __shared__ int s_bmove;  // a column base of the tile moved this round
  __shared__ int s_slow[RB];
  // per-row metadata of the workgroup's rows, staged once for its TPW tiles:
  // s_meta = alive | active << 1 | inbox count << 2; s_inb = first KB senders
  __shared__ int s_meta[RB];
  __shared__ __attribute__((aligned(16))) int s_inb[RB * KB];
  // row layout: the senders' table slots (owned or ghost rows)
  __shared__ __attribute__((aligned(16))) int s_isl[RB * KB];

  // block -> (tile group of TPW consecutive tiles, row block); group-major so
  // that the running workgroups sweep the same tiles together
  const int nrb = (int)((d.nrows + RB - 1) / RB);
  const int ngroups = (int)(p.ld / TW) / TPW;
  const int rowend = (int)(d.row0 + d.nrows);
  int group, rb;
  if (p.xmap && ngroups % 8 == 0) {
    // XCD-aware: blocks b and b+8 share an XCD (round-robin dispatch, speed
    // only), so XCD x = b % 8 sweeps groups x, x+8, ... and its L2 holds the
    // slice it is on.
    const int x = bid & 7;
    const int j = bid >> 3;
    group = x + 8 * (j / nrb);
    rb = j - (j / nrb) * nrb;
  } else {
    group = bid / nrb;
    rb = bid - group * nrb;
  }
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = uni(tid >> 6);
  const int sub = lane / SEG;
  const int lc = lane % SEG;
  const unsigned long long gmask = (SEG == 64 ? ~0ull : ((1ull << SEG) - 1)) << (sub * SEG);

  if (tid == 0) {
    s_merged = s_det = s_rel = s_storm = s_tomb = s_unk = 0;
    s_quiet = 0;
    s_bmove = 0;  // set by the first tile's setup after the staging barrier
  }
  const bool pull = p.peer_mode == GH_PEER_PULL;
  // quiet rows may be skipped: no REMOVE pending anywhere (|D_{r-1}| = 0)
  const bool quiet = d.cntg[p.n] == 0 && !p.force_slow && !(d.a4[0] && d.m8[2]);
  const uint8_t* __restrict__ stab_cur = d.stab[p.r & 1];
  uint8_t* __restrict__ stab_nxt = d.stab[(p.r + 1) & 1];
  if constexpr (STORM) {
    // row metadata once per row, then only the inbox slots in use (storms
    // and guard rows have few senders)
    for (int row = tid; row < RB; row += 256) {
      const int i = (int)d.row0 + rb * RB + row;
      int meta = 0;
      if (i < rowend) {
        const int al = d.alive[i];
        const int cnt = al ? gh_in_cnt(d, pull, p.k, i) : 0;
        const int act = d.active[i];
        meta = al | (act << 1) | (cnt << 2) | ((quiet && al && !act && cnt == 0 && stab_cur[i]) ? 1 << 30 : 0);
      }
      s_meta[row] = meta;
    }
    __syncthreads();
    for (int t = tid; t < RB * KB; t += 256) {
      const int row = t / KB, q = t - row * KB;
      const int i = (int)d.row0 + rb * RB + row;
      if (q < ((s_meta[row] >> 2) & 0x0FFFFFFF)) {
        const int sv = d.inbox[gh_in_beg(d, pull, p.k, i) + q];
        s_inb[t] = sv;
        if (d.rowlay) s_isl[t] = d.rslot[sv];
      }
    }
  } else {
    // one pass, no barrier in between: healthy rounds use every slot
    for (int t = tid; t < RB * KB; t += 256) {
      const int row = t / KB, q = t - row * KB;
      const int i = (int)d.row0 + rb * RB + row;
      int meta = 0, sv = 0;
      if (i < rowend) {
        const int al = d.alive[i];
        const int cnt = al ? gh_in_cnt(d, pull, p.k, i) : 0;
        const int act = d.active[i];
        meta = al | (act << 1) | (cnt << 2) | ((quiet && al && !act && cnt == 0 && stab_cur[i]) ? 1 << 30 : 0);
        if (q < cnt) sv = d.inbox[gh_in_beg(d, pull, p.k, i) + q];
      }
      if (q == 0) s_meta[row] = meta;
      s_inb[t] = sv;
      if (d.rowlay) s_isl[t] = d.rslot[sv];
    }
  }
  // every row of the workgroup quiet (a collapsed cluster): a tile whose
  // bases stayed is skipped whole, its row segments counted as quiet
  bool myq = true;
  for (int row = tid; row < RB; row += 256)
    if ((int)d.row0 + rb * RB + row < rowend) myq &= ((s_meta[row] >> 30) & 1) != 0;
  const bool allq = __syncthreads_and(myq) != 0;
  const int nvrows = min(RB, rowend - ((int)d.row0 + rb * RB));

  const uint16_t* __restrict__ hno = d.hn[cur];
  uint16_t* __restrict__ hnn = d.hn[cur ^ 1];
  const int32_t* __restrict__ bo = d.base[cur];
  const int32_t* __restrict__ bn = d.base[cur ^ 1];
  // 4-bit tier of the buffer read / written (gh_internal.h: a4): a lane's 8
  // cells are its plane word and its age word (4 B each), widened to packed
  // 16-bit codes in registers; an escaped chunk is read from / written to hn
  // (lean variants: one instantiation per input tier)
  constexpr bool RD8 = IN == 1 || IN == 2;
  // (the tier write path only where a tiered engine runs: pull k <= 4, one
  // tile per workgroup)
  constexpr bool W8 = !STORM && KB == 4 && TPW == 1;
  const bool m8c = STORM ? gh_m8(d, cur) : RD8, m8n = W8 && gh_m8(d, cur ^ 1);
  const uint32_t* __restrict__ a4o = d.a4[cur];
  uint32_t* __restrict__ a4n = d.a4[cur ^ 1];
  int n_esc = 0;  // escaped chunks written
  // sender plane: read by the lean 4-slot variant when valid, written by
  // every variant in plane mode
  constexpr bool PLANE_RD = !STORM && KB == 4;
  const bool use_plane = PLANE_RD && p.plane && d.pvalid[cur];
  const uint32_t* __restrict__ plo = d.pl[cur];
  uint32_t* __restrict__ pln = d.pl[cur ^ 1];
  int n_fb = 0;  // plane fallbacks of this wave
  uint32_t n_mrg16 = 0;  // merges x 16
  int n_det = 0, n_rel = 0;
  int n_tomb = 0, n_unk = 0;  // REMOVE: tombstoned / unknown member

#pragma unroll 1
  for (int tt = 0; tt < TPW; ++tt) {
  const int tile = group * TPW + tt;
  const int64_t l0 = (int64_t)tile * TW + lc * CPL;                   // local column of this lane's first cell
  const int c0 = (int)(d.col0 + l0);                                  // its global member id
  // uniform tile bases; rows are 32-bit byte offsets (table slots) from them
  const int64_t tcell = (int64_t)tile * d.tstride;
  const char* hno_t = reinterpret_cast<const char*>(hno + tcell);
  char* hnn_t = reinterpret_cast<char*>(hnn + tcell);
  const char* plo_t = reinterpret_cast<const char*>(plo) + (plo ? tcell / 2 : 0);
  char* pln_t = reinterpret_cast<char*>(pln) + (pln ? tcell / 2 : 0);
  const char* a4o_t = reinterpret_cast<const char*>(a4o) + (a4o ? tcell / 2 : 0);
  char* a4n_t = reinterpret_cast<char*>(a4n) + (a4n ? tcell / 2 : 0);
  const uint32_t lb = (uint32_t)lc * (CPL * 2);  // lane's byte offset in a row segment (narrow)
  const uint32_t lbp = (uint32_t)lc * 4;         // ... in a plane (or age plane) row segment
  if (tid == 0) s_nslow = 0;
  for (int t = tid; t < TW; t += 256) {
    s_dcnt[t] = 0;
    s_dmin[t] = INT_MAX;
  }

  // REMOVE'd members in the lane: its segments go to the slow list
  const uint32_t my8 = (d.dbits[l0 >> 5] >> (l0 & 31)) & 0xFFu;
  for (int pp = tid; pp < TW / 2; pp += 256) {
    uint32_t dd = 0, th = 0, rmm = 0, rm1 = 0;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int64_t c = (int64_t)tile * TW + 2 * pp + h;
      if (dbit(d.dbits, c)) {
        if (d.det_cnt[dcur][c] == 1 || d.rlist)  // a recipient set the packed path does not hold
          rm1 = 1;
        else
          rmm |= 0xFFFFu << (16 * h);
      }
      const int64_t delta = (int64_t)bn[c] - bo[c];
      const uint32_t d5h = (delta > 1023 || delta < -1023) ? 0x8000u : ((uint32_t)(delta << 5) & 0xFFFFu);
      const int64_t thr = 1 - (int64_t)bn[c];
      const uint32_t tc = thr < 0 ? 0xFFFFu : thr > 1023 ? 0x7FFFu : (uint32_t)((thr << 5) | 31);
      dd |= d5h << (16 * h);
      th |= tc << (16 * h);
    }
    if (dd) s_bmove = 1;
    s_d5[pp] = dd;
    s_t5[pp] = th;
    s_rm[pp] = rmm;
    s_rm1[pp] = rm1;
  }
  const uint32_t tfp = (uint32_t)min(p.t_fail, 31) * 0x10001u;
  // tombstone age + tsk carries into bit 5 iff age >= the saturation age
  const uint32_t tsk = (uint32_t)(32 - (d.tsa ? d.tsa : GH_N_TAGEMAX)) * 0x10001u;
  // ... and into bit 5 iff age > tsa with saturation (never written by the
  // round: such a cell goes to the per-cell rule, which caps it), else as tsk
  const uint32_t tsk1 = d.tsa ? (uint32_t)(31 - d.tsa) * 0x10001u : tsk;
  const uint32_t tsm = d.tsa ? 0xFFFFFFFFu : 0u;  // tombstone ages saturate at tsa (SPEC §1)
  const uint32_t tcp = (uint32_t)min(p.t_cleanup, 31) * 0x10001u;
  __syncthreads();
  const bool tile_still = s_bmove == 0;
  // lean: no REMOVE in the lane; storm: REMOVE applied in the packed path
  // unless a column has a single detector (that row keeps the member)
  bool lane_ok = !p.force_slow;
  if constexpr (STORM) {
#pragma unroll
    for (int j = 0; j < 4; ++j) lane_ok &= s_rm1[lc * 4 + j] == 0;
  } else {
    lane_ok &= my8 == 0;
  }

  constexpr int NIT = RB / RSTEP;
  const bool tile_quiet = allq && tile_still;
  if (tile_quiet && tid == 0) atomicAdd(&s_quiet, nvrows);
#pragma unroll 1
  for (int it = 0; it < (tile_quiet ? 0 : NIT); ++it) {
    const int rr = wave * RPW + it * RSTEP + sub;
    const int i_raw = (int)d.row0 + rb * RB + rr;
    const bool valid = i_raw < rowend;
    const int i = valid ? i_raw : rowend - 1;  // in-range row for the loads of idle lanes
    const uint32_t islot = (uint32_t)(i - d.row0);  // its table slot
    const int rs = valid ? rr : 0;
    int meta = s_meta[rs];
    if constexpr (RPW == 1) meta = uni(meta);
    // a quiet row in a tile whose bases stayed: nothing to read or write
    const bool skip = ((meta >> 30) & 1) && tile_still;
    if (valid && skip && lc == 0) atomicAdd(&s_quiet, 1);
    if (__ballot(valid && !skip) == 0) continue;
    const bool al = (meta & 1) && valid && !skip;
    const int cntv = (meta >> 2) & 0x0FFFFFFF;  // bits 2..29: a ring receiver can have N - 1 senders
    const uint32_t ob = islot * (TW * 2) + lb;  // own segment, bytes from the tile base

    // own segment and the senders' snapshots, issued together: plane words
    // when the plane is valid, else the first KB senders' 16-bit segments
    // (slots q >= cntv hold the own row, a no-op under the max)
    const uint32_t obp = islot * (TW / 2) + lbp;  // ... in the plane and the age plane
    v4u w = {0u, 0u, 0u, 0u};
    uint32_t a4w = 0u, q4w = 0u;
    if (m8c) {
      a4w = *reinterpret_cast<const uint32_t*>(a4o_t + obp);
      q4w = *reinterpret_cast<const uint32_t*>(plo_t + obp);
    } else {
      w = ldn<false>(reinterpret_cast<const uint16_t*>(hno_t + ob));  // re-read by peers: keep it cached
    }
    const int jd = i - c0;
    const bool own_in = (unsigned)jd < 8u;
    int ps[KB];
    const bool act = (meta >> 1) & 1;  // else the row is under the <4 guard (step 2)
    // guard rows in the lean variant: the 8-slot instantiation (ring
    // inboxes, pull k > 4) takes them, so a collapsed cluster runs lean; the
    // 4-slot one lists them (the stamp select cost 4% of the healthy pull
    // round, measured A/B on one box)
    constexpr bool LEAN_GUARD = KB > 4;
    bool bad = (!STORM && !LEAN_GUARD && !act) || cntv > KB || i == p.shadow_row;  // (D7 shadows: per-cell rule)
    // the staged slots, one LDS read per 4 (unused slots hold 0)
    int sv[KB];
#pragma unroll
    for (int q4 = 0; q4 < KB; q4 += 4) {
      const int4 v = *reinterpret_cast<const int4*>(&s_inb[rs * KB + q4]);
      sv[q4] = v.x;
      sv[q4 + 1] = v.y;
      sv[q4 + 2] = v.z;
      sv[q4 + 3] = v.w;
    }
#pragma unroll
    for (int q = 0; q < KB; ++q) {
      int s = q < cntv ? sv[q] : i;
      if constexpr (RPW == 1) s = uni(s);
      ps[q] = s;
    }
    // the senders' table slots (column layout: their row ids)
    uint32_t psl[KB];
    if (d.rowlay) {
#pragma unroll
      for (int q4 = 0; q4 < KB; q4 += 4) {
        const int4 v = *reinterpret_cast<const int4*>(&s_isl[rs * KB + q4]);
        const int v4[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int u = 0; u < 4; ++u) psl[q4 + u] = q4 + u < cntv ? (uint32_t)v4[u] : islot;
      }
    } else {
#pragma unroll
      for (int q = 0; q < KB; ++q) psl[q] = (uint32_t)ps[q];
    }
    // a sender's segment: an owned row's in this tile of the table, a ghost
    // row's (row layout, slot >= nrows) in the row-major ghost table
    auto snd16 = [&](uint32_t sl) -> const uint16_t* {
      if (d.gcodes && (int64_t)sl >= d.nrows) return d.gcodes + ((int64_t)sl - d.nrows) * d.ld + l0;
      return reinterpret_cast<const uint16_t*>(hno_t + (sl * (TW * 2) + lb));
    };
    auto sndp = [&](uint32_t sl) -> const uint32_t* {
      if (d.gplane && (int64_t)sl >= d.nrows) return d.gplane + ((((int64_t)sl - d.nrows) * d.ld + l0) >> 3);
      return reinterpret_cast<const uint32_t*>(plo_t + (sl * (TW / 2) + lbp));
    };
    uint32_t pw[KB];
    if constexpr (PLANE_RD) {
      if (use_plane) {
        // unused slots read the own row's codes: the own offsets, never
        // above the own cell, so a no-op under the merge (an unknown or old
        // code there only costs a fallback)
#pragma unroll
        for (int q = 0; q < KB; ++q) pw[q] = *sndp(psl[q]);
      }
    }
    if (m8c) {  // widen the own chunk (an escaped one is hn's)
      if (gh_t4_esc(a4w))
        w = ldn<false>(reinterpret_cast<const uint16_t*>(hno_t + ob));
      else
        w = c4_dec(q4w, a4w, own_in ? jd : -1, d.toff);
    }
    bad |= (w[0] & 0xFFFFu) == GH_N_WIDE;  // own segment wide
    // The row's own member in the lane (step 3, :443-448): hb + 1 with a
    // fresh stamp (age 0, so age 1 after the round's +1), never flagged.
    // An own cell that is not visible, or at the heartbeat cap, is slow.
    if (own_in && act) {
      const int sh = 16 * (jd & 1);
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (j == (jd >> 1)) {
          const uint32_t hv = (w[j] >> sh) & 0xFFFFu;
          if (hv >= 0x8000u || (int64_t)bo[l0 + jd] + (hv >> 5) >= INT32_MAX ||
              (STORM && ((s_rm[lc * 4 + j] >> sh) & 1u)))
            bad = true;
          else
            w[j] = (w[j] & ~(0x1Fu << sh)) + (0x20u << sh);
        }
    }
    // ms[j]: the senders' snapshot codes of pair j, packed max (negative
    // halves: no visible entry)
    uint32_t ms[4];
    bool need16 = true;
    if constexpr (PLANE_RD) {
      if (use_plane) {
        // per pair, the min over senders of the plane codes is the freshest
        // entry (fields kept at their bit position: the min of masked
        // halves); exact unless it is 0 (a sender unknown) or 14 (only
        // entries older than the window): then the wave gathers 16-bit codes
        uint32_t Lw = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const uint32_t M = 0x000F000Fu << (4 * j);
          uint32_t L = pw[0] & M;
#pragma unroll
          for (int q = 1; q < KB; ++q) L = pk_min_u16(L, pw[q] & M);
          Lw |= L;
          const uint32_t c5 = j == 0 ? pk_shl16(L, 5) : j == 1 ? pk_shl16(L, 1) : j == 2 ? pk_lshr16(L, 3) : pk_lshr16(L, 7);
          // offset = REF + 1 - code; codes 14, 15: no merge (-1)
          ms[j] = pk_sub_u16((uint32_t)((GH_P_REF + 1) << 5) * 0x10001u, c5) |
                  pk_sra15(pk_sub_u16((uint32_t)(13 << 5) * 0x10001u, c5));
        }
        need16 = __ballot((nib_haszero(Lw) | nib_haszero(Lw ^ 0xEEEEEEEEu)) != 0) != 0;
        n_fb += need16;
      }
    }
    if (need16) {
      // four slots at a time (an 8-slot inbox keeps only four segments live);
      // a later group runs only when a lane of the wave uses it
#pragma unroll
      for (int g = 0; g < KB; g += 4) {
        if (g > 0 && __ballot(g < cntv) == 0) break;
        // a sender's chunk into the merge: a wide segment is slow; its own
        // member in the lane carries hb + 1 in its snapshot (the sender's
        // heartbeat of this round); the packed max over senders
        auto fold = [&](v4u pv, const int q) {
          bad |= q < cntv && (pv[0] & 0xFFFFu) == GH_N_WIDE;
          const int js = ps[q] - c0;
          if (q < cntv && (unsigned)js < 8u) {
            const int sh = 16 * (js & 1);
#pragma unroll
            for (int j = 0; j < 4; ++j)
              if (j == (js >> 1) && ((pv[j] >> sh) & 0x8000u) == 0) pv[j] += 0x20u << sh;
          }
#pragma unroll
          for (int j = 0; j < 4; ++j) ms[j] = q == 0 ? pv[j] : pk_max_i16(ms[j], pv[j]);
        };
        if (m8c) {
          // tier sender chunks (plane and age words; unused slots: all
          // absent), all four issued, then widened one at a time (an escaped
          // one is read from hn)
          // (row layout: a ghost sender is a row of the ghost table, 16-bit
          // codes, not a tier chunk; in a round whose ghosts carry only their
          // plane the lane goes to the slow list, as below)
          uint32_t su[4], sa[4];
          bool gs[4];
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const int q = g + u;
            gs[u] = d.gcodes && q < cntv && (int64_t)psl[q] >= d.nrows;
            const uint32_t off = (gs[u] ? islot : psl[q]) * (TW / 2) + lbp;
            const bool ld = (STORM ? q < cntv : KB > 4 ? __ballot(q < cntv) != 0 : true) && !gs[u];
            su[u] = ld ? *reinterpret_cast<const uint32_t*>(plo_t + off) : ~0u;
            sa[u] = ld ? *reinterpret_cast<const uint32_t*>(a4o_t + off) : ~0u;
          }
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            v4u pv;
            const int js = ps[g + u] - c0;
            if (gs[u]) {
              bad |= p.gpo;
              pv = p.gpo ? v4u{~0u, ~0u, ~0u, ~0u} : ldn<false>(snd16(psl[g + u]));
            } else if (gh_t4_esc(sa[u])) {
              pv = ldn<false>(reinterpret_cast<const uint16_t*>(hno_t + (psl[g + u] * (TW * 2) + lb)));
            } else {
              pv = c4_dec(su[u], sa[u], (unsigned)js < 8u ? js : -1, d.toff);
            }
            fold(pv, g + u);
          }
        } else {
          v4u pv[4];
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const int q = g + u;
            // row layout, a round whose ghosts carry only their plane
            // (p.gpo): a ghost sender's 16-bit codes are not here yet, so
            // the lane goes to the slow list (k_round_slow runs after they
            // arrive) and reads the own row instead
            const bool gq = p.gpo && q < cntv && (int64_t)psl[q] >= d.nrows;
            bad |= gq;
            const uint16_t* src = snd16(gq ? islot : psl[q]);
            if constexpr (STORM) {
              // storms hold few senders (guard rows none): load only the used
              // slots, the rest are absent (-1, a no-op under the max)
              pv[u] = q < cntv ? ldn<false>(src) : v4u{~0u, ~0u, ~0u, ~0u};
            } else if constexpr (KB > 4) {
              // 8-slot inboxes (ring, pull k > 4) are mostly part-empty, and
              // empty in a collapsed cluster: slots no lane of the wave uses
              // are not loaded
              pv[u] = __ballot(q < cntv) != 0 ? ldn<false>(src) : v4u{~0u, ~0u, ~0u, ~0u};
            } else {
              pv[u] = ldn<false>(src);  // unused slots hold the own row: a no-op under the max
            }
          }
#pragma unroll
          for (int u = 0; u < 4; ++u) bad |= g + u < cntv && (pv[u][0] & 0xFFFFu) == GH_N_WIDE;
          // A sender's own member in the lane: its snapshot carries hb + 1
          // there (the sender's heartbeat of this round).
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const int js = ps[g + u] - c0;
            if (g + u < cntv && (unsigned)js < 8u) {
              const int sh = 16 * (js & 1);
#pragma unroll
              for (int j = 0; j < 4; ++j)
                if (j == (js >> 1) && ((pv[u][j] >> sh) & 0x8000u) == 0) pv[u][j] += 0x20u << sh;
            }
          }
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            uint32_t m4 = pk_max_i16(pk_max_i16(pv[0][j], pv[1][j]), pk_max_i16(pv[2][j], pv[3][j]));
            ms[j] = g == 0 ? m4 : pk_max_i16(ms[j], m4);
          }
        }
      }
    }

    v4u o;
    // acc: bit 5/21 = a special own cell (age >= 30, wide marker), bit 15/31
    // = a result outside the narrow window; ev: detected or released cells
    uint32_t acc = 0, detb = 0, relb = 0, stb = 0, mcnt = 0, tomb16 = 0, unk16 = 0;
    uint32_t fo = 0;  // flagged results: next round's detections
    const v4u d5 = *reinterpret_cast<const v4u*>(&s_d5[lc * 4]);
    const v4u t5 = *reinterpret_cast<const v4u*>(&s_t5[lc * 4]);
    v4u rmv = {0u, 0u, 0u, 0u};
    if constexpr (STORM) rmv = *reinterpret_cast<const v4u*>(&s_rm[lc * 4]);
    int dp16 = 0;  // (present after - present before) x 16
    // storm: a guard row without senders or REMOVE in the lane takes the
    // folded rule (the collapsed regime)
    const bool gfast = STORM && !act && cntv == 0 && (rmv[0] | rmv[1] | rmv[2] | rmv[3]) == 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t rmj = rmv[j];  // REMOVE'd columns: not in any sender's snapshot
      const uint32_t m = ms[j] | rmj;
      const uint32_t x = w[j];
      uint32_t mm, y0, npre;  // merged mask, value if not merged, absent-before mask
      if constexpr (!STORM) {
        // own cells other than visible (age < 30) or absent go to the slow
        // list: flagged, tombstone, wide marker (x + 1 keeps bit 15), age 30/31
        const uint32_t hx = pk_sra15(x);
        acc |= (pk_add_u16(x, 0x00010001u) & 0x80008000u) | ((((x & 0x001F001Fu) + 0x00020002u) & ~hx) & 0x00200020u);
        mm = pk_sra15(pk_subs_i16(x | 0x001F001Fu, m));     // merged: a sender's heartbeat is larger
        y0 = pk_adds_u16(x, 0x00010001u);                   // not merged: age + 1 (absent stays)
        // a guard row (step 2, :504-509) stamps its present cells: age 1
        if (LEAN_GUARD && !act) y0 = (((x & 0x7FE07FE0u) | 0x00010001u) & ~hx) | (x & hx);
        npre = hx;
      } else if (gfast) {
        // a guard row with no senders and no REMOVE in the lane (a collapsed
        // cluster): present cells stamped, tombstones age, absent stays;
        // nothing merges, is detected or released (the rule below with
        // act = 0, m = -1, rmj = 0 folded)
        const uint32_t z = pk_add_u16(x | 0x001F001Fu, 0x00010001u);
        const uint32_t ta0 = pk_zero_mask(z);                  // tombstone or absent
        const uint32_t ab = pk_zero_mask(pk_add_u16(x, 0x00010001u));  // absent
        // a tombstone at its saturation age keeps it (slave/slave.go:490 only
        // compares it with now - COOLDOWN); beyond it (or at the 16-bit cap
        // without saturation) the per-cell rule takes the segment
        const uint32_t satb = ((((x & 0x001F001Fu) + tsk) & 0x00200020u) >> 5) & ~ab & ta0 & tsm;
        acc |= ((x & 0x001F001Fu) + tsk1) & ~ab & ta0 & 0x00200020u;
        mm = 0u;
        y0 = (((x & 0x7FE07FE0u) | 0x00010001u) & ~ta0) | (pk_adds_u16(x, 0x00010001u & ~satb) & ta0);
        npre = ta0;
        stb = ~0u;  // a guard row: what the lean variant lists
      } else {
        // cell classes: (x | 31) + 1 is 0 for a tombstone or absent cell, has
        // bit 15 for a flagged present one and not for a visible one
        const uint32_t actm = act ? 0xFFFFFFFFu : 0u;
        const uint32_t z = pk_add_u16(x | 0x001F001Fu, 0x00010001u);
        const uint32_t ta0 = pk_zero_mask(z);                  // tombstone or absent
        const uint32_t ab = pk_zero_mask(pk_add_u16(x, 0x00010001u));  // absent
        // step 1 REMOVE: a present cell becomes a tombstone of its age
        tomb16 += __builtin_popcount(rmj & ~ta0);
        unk16 += __builtin_popcount(rmj & ab);
        const uint32_t xr = x | (rmj & 0xFFE0FFE0u);
        const uint32_t fl0 = pk_sra15(z) & ~rmj;               // flagged present
        const uint32_t ta = ta0 | rmj;                         // tombstone or absent
        const uint32_t fl = fl0 & actm;                        // detected now (step 4, active rows)
        const uint32_t ag = x & 0x001F001Fu;
        const uint32_t st = pk_sra15(pk_subs_i16(tcp, ag)) & actm;  // age > T_cleanup (step 5, active rows)
        const uint32_t rel = (ta | fl) & st;                   // absent after step 5 (released, or absent)
        // tombstone next round (absent cells never are: they merge, even
        // when T_cleanup reaches the age field and st says "fresh")
        const uint32_t keep = ((ta & ~ab) | fl) & ~st;
        const uint32_t nowm = ~ta & ~actm;                     // guard rows: present cells stamped now
        // age >= 30 or wide marker; a guard row's tombstone beyond its
        // saturation age (at it, it keeps its age: satb)
        acc |= (((ag + 0x00020002u) & ~ab & ~nowm) | ((ag + tsk1) & ta & ~ab & ~actm)) & 0x00200020u;
        const uint32_t satb = (((ag + tsk) & 0x00200020u) >> 5) & ta & ~ab & tsm;
        const uint32_t key = ((xr & ~(nowm & 0x80008000u)) | 0x001F001Fu) | rel;  // heartbeat key (absent: -1)
        mm = pk_sra15(pk_subs_i16(key, m)) & ~keep;            // merged (step 6)
        // not merged: age + 1 (a detected cell becomes a tombstone of its
        // age), released cells absent, absent stays absent; guard rows'
        // present cells age 1
        const uint32_t yact = pk_adds_u16(xr | (fl & 0xFFE0FFE0u), 0x00010001u & ~satb) | rel;
        y0 = (((xr & 0x7FE07FE0u) | 0x00010001u) & nowm) | (yact & ~nowm);
        npre = ta0;
        stb |= ((fl0 | ta) & ~ab) | (LEAN_GUARD ? 0u : ~actm);  // what the lean variant lists
        detb |= pair_bits(fl, j);
        relb |= pair_bits(rel & ~ab, j);
      }
      const uint32_t mv = (m & 0x7FE07FE0u) | 0x00010001u;   // merged: its heartbeat, age 1
      uint32_t y = (mv & mm) | (y0 & ~mm);
      const uint32_t hy = pk_sra15(y);                       // tombstone or absent halves
      y = pk_sub_u16(y, d5[j] & ~hy);                        // rebase present halves
      acc |= (y | pk_add_u16(y, 0x00200020u)) & ~hy & 0x80008000u;  // offset left [0, 1022]
      const uint32_t c1 = pk_subs_i16(tfp, y & 0x001F001Fu); // age > T_fail
      const uint32_t c2 = pk_subs_i16(t5[j], y);             // hb > 1
      const uint32_t flo = c1 & c2 & ~hy & 0x80008000u;
      y |= flo;
      fo |= flo;
      o[j] = y;
      mcnt += __builtin_popcount(mm);
      dp16 += __builtin_popcount(npre) - __builtin_popcount(hy);
    }
    if (own_in) {  // the own member is never detected: no flag on a present own cell
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (j == (jd >> 1) && ((o[j] >> (16 * (jd & 1))) & 0xFFFFu) < GH_N_TOMB) o[j] &= ~(0x8000u << (16 * (jd & 1)));
    }
    const bool ok = lane_ok && !bad && acc == 0;
    const bool seg_ok = (__ballot(al && !ok) & gmask) == 0;
    if constexpr (STORM || LEAN_GUARD) {
      // an inactive row stays a quiet candidate only while none of its
      // segments changes (segments listed for the per-cell kernel, e.g. the
      // 4-slot lean variant's inactive rows or saturated tombstones, are
      // judged there)
      uint32_t chg = 0;
      if (al && !act && seg_ok) chg = (o[0] ^ w[0]) | (o[1] ^ w[1]) | (o[2] ^ w[2]) | (o[3] ^ w[3]);
      if ((__ballot(chg != 0) & gmask) != 0 && lc == 0) stab_nxt[i] = 0;
    }
    int dpres = 0;  // present after - present before
    bool any_det = false;
    if (al) {
      if (seg_ok) {
        if (m8n) {
          // the tier: the age word, the plane word below is the lag
          uint32_t age = 0;
          const bool t4 = c4_enc(o, own_in ? jd : -1, age, d.toff);
          uint32_t* ap = reinterpret_cast<uint32_t*>(a4n_t + obp);
          if constexpr (NT)
            __builtin_nontemporal_store(t4 ? age : GH_T4_ESC, ap);
          else
            *ap = t4 ? age : GH_T4_ESC;
          if (!t4) {  // escaped: the 16-bit chunk
            stn<NT>(reinterpret_cast<uint16_t*>(hnn_t + ob), o);
            n_esc++;
          }
        } else {
          stn<NT>(reinterpret_cast<uint16_t*>(hnn_t + ob), o);
        }
        if (p.plane) {
          const uint32_t pwd = plane_word(o, own_in ? jd : -1);
          uint32_t* pp = reinterpret_cast<uint32_t*>(pln_t + (islot * (TW / 2) + lbp));
          if constexpr (NT)
            __builtin_nontemporal_store(pwd, pp);
          else
            *pp = pwd;
        }
        dpres = dp16 >> 4;
        n_mrg16 += mcnt;
        if constexpr (STORM) {
          n_tomb += (int)(tomb16 >> 4);
          n_unk += (int)(unk16 >> 4);
        }
        if (STORM && (detb | relb)) {  // storms: detections per column, releases
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            if ((detb >> j) & 1u) {
              atomicAdd(&s_dcnt[lc * CPL + j], 1);
              atomicMin(&s_dmin[lc * CPL + j], i);
            }
          }
          n_det += __builtin_popcount(detb);
          n_rel += __builtin_popcount(relb);
          any_det = detb != 0;
        }
      } else if (lc == 0) {
        s_slow[atomicAdd(&s_nslow, 1)] = i;
      }
    }
    if (__ballot(dpres != 0 || any_det) != 0) {  // rare in healthy rounds: skip the segment sums
#pragma unroll
      for (int o2 = SEG / 2; o2 > 0; o2 >>= 1) {
        dpres += __shfl_xor(dpres, o2);
        any_det |= __shfl_xor((int)any_det, o2) != 0;
      }
      if (lc == 0) {
        if (dpres) atomicAdd(&d.cntl[i], dpres);
        if (any_det) d.det_any[i] = 1;
      }
    }
    // storm measure: committed segments that hold (storm variant) or will
    // hold next round (flagged results) cells the lean variant cannot take
    if (al && seg_ok && (__ballot(stb != 0 || fo != 0) & gmask) != 0 && lc == 0) atomicAdd(&s_storm, 1ull);
  }

  __syncthreads();
  if (tid == 0) s_bmove = 0;  // read before the barrier above; the next tile's setup writes it after two more
  for (int t = tid; t < TW; t += 256) {
    if (s_dcnt[t]) {
      const int64_t c = (int64_t)tile * TW + t;
      atomicAdd(&d.det_cnt[dcur ^ 1][c], s_dcnt[t]);
      atomicMin(&d.det_min[dcur ^ 1][c], s_dmin[t]);
    }
  }
  if (tid == 0 && s_nslow) s_slowbase = atomicAdd(d.slow_n, s_nslow);
  __syncthreads();
  for (int t = tid; t < s_nslow; t += 256) d.slow[s_slowbase + t] = ((int64_t)tile << 32) | (uint32_t)s_slow[t];
  __syncthreads();  // s_nslow / s_slow are reused by the next tile
  }  // tiles

  if (PLANE_RD && n_fb && lane == 0) atomicAdd(d.pfb, n_fb);
  if (n_esc) atomicAdd(&d.m8[3], n_esc);
  if (n_mrg16) atomicAdd(&s_merged, (unsigned long long)(n_mrg16 >> 4));
  if (n_det) atomicAdd(&s_det, (unsigned long long)n_det);
  if (n_rel) atomicAdd(&s_rel, (unsigned long long)n_rel);
  if (n_tomb) atomicAdd(&s_tomb, (unsigned long long)n_tomb);
  if (n_unk) atomicAdd(&s_unk, (unsigned long long)n_unk);
  __syncthreads();
  if (tid == 0) {
    // s_storm counts every written segment with a flagged cell (lean: only
    // those): the quirk pre-pass gate
    if (s_storm) atomicAdd(&d.nflag[cur ^ 1], 1);
    if (s_merged) atomicAdd(&d.stats[ST_MERGED], s_merged);
    if (s_det) atomicAdd(&d.stats[ST_DETECTIONS], s_det);
    if (s_rel) atomicAdd(&d.stats[ST_RELEASED], s_rel);
    if (s_storm) atomicAdd(d.nstorm, (int)s_storm);
    if (s_tomb) atomicAdd(&d.stats[ST_TOMBSTONED], s_tomb);
    if (s_unk) atomicAdd(&d.stats[ST_REMOVE_UNKNOWN], s_unk);
    if (s_quiet) atomicAdd(d.nquiet, s_quiet);
  }
}

// The variants are launched every round (lean on a 16-bit input; in a
// tiered engine also the nibble path on a 4-bit-tier input and the lean one
// on it by the 16-bit rule; storm); the ones k_base, the input's tier and the
// plane did not select return at once. The nibble path runs one block per workgroup; the
// storm variant and the rarely selected lean ones of a tiered engine run 1/8
// of the workgroups, each taking blocks a multiple of 8 apart (same XCD), so
// idle they are a small dispatch (IN 6 too: compiled for 5 waves per SIMD,
// 96 VGPRs, as its block loop left to the compiler took 106 and at 6 waves
// spilled 72 bytes per lane; the host's full-grid REMOVE launch is IN 7).
template <int KB, int TW, int TPW, bool NT, bool STORM, int IN>
__global__ __launch_bounds__(256, (STORM && TW >= 64) ? GH_STORM_WAVES : (STORM && TW >= 32) ? 4 : IN == 6 ? 5 : IN == 7 ? GH_RMV_WAVES : (IN == 2 || IN == 4 || IN == 5) ? GH_NIB_WAVES : 1) void k_round(GhDev d, int cur, int dcur, GhRound p) {
  if (*d.mode != (int)STORM) return;
  if constexpr (!STORM) {
    int want = 0;
    if (d.a4[0])
      want = !gh_m8(d, cur) ? 3 : (KB == 4 && p.plane && d.pvalid[cur] && gh_m8(d, cur ^ 1)) ? (d.rowlay ? 4 : 2) : 1;
    if (want == 2 && p.nib_dma && TW == 256 && GH_NIB_CPL == 16) want = 5;  // LDS-DMA staging (GH_NIB_DMA)
    // a REMOVE pending (|D_{r-1}| > 0): the instantiation that takes it on the
    // nibble path (GH_NIB_RMV=2: in every round, A/B)
    // (p.rmv_full: the host launched IN 6 in place of IN 2, so IN 6 must run
    // whatever the device's count says: the round's nibble path is never skipped)
    if (want == 2 && (p.rmv_full || p.nib_rmv == 2 || (p.nib_rmv && d.cntg[p.n] > 0))) want = 6;
    if (want != (IN == 7 ? 6 : IN)) return;  // (IN 7: IN 6 on a full grid)
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    d.m8[4] = STORM ? 1 : (IN == 2 || IN == 4 || IN == 5 || IN == 6 || IN == 7) ? 3 : IN == 1 ? 2 : 0;
    // launch_round's variant number of this launch (IN 3 is variant 0 of a tiered engine)
    if (d.vlog) d.vlog[p.vslot] = STORM ? 1 : (IN == 6 || IN == 7) ? 4 : (IN == 2 || IN == 4 || IN == 5) ? 3 : IN == 1 ? 2 : 0;
  }
  // every running row a quiet candidate and no base moved (one engine): the
  // round reads and writes nothing (a collapsed cluster)
  if (d.world == 1 && !d.rowlay && d.aq[0] == 0 && d.cntg[p.n] == 0 && !p.force_slow && !(d.a4[0] && d.m8[2])) {
    if (blockIdx.x == 0 && threadIdx.x == 0) *d.nquiet = (int)min<int64_t>(d.ntiles * d.nrows, INT_MAX);
    return;
  }
  if constexpr (STORM || IN == 1 || IN == 3) {
    constexpr int RB = round_rb<TW>();
    const int nblk = (int)((d.nrows + RB - 1) / RB) * ((int)(p.ld / TW) / TPW);
    for (int b = blockIdx.x; b < nblk; b += gridDim.x) {
      round_block<KB, TW, TPW, NT, STORM, IN>(d, cur, dcur, p, b);
      __syncthreads();  // LDS of this block before the next
    }
  } else if constexpr (IN == 2) {
    round_block_nib<TW, NT, GH_NIB_CPL, false, false, false>(d, cur, dcur, p, blockIdx.x);  // one block per workgroup
  } else if constexpr (IN == 4) {
    round_block_nib<TW, NT, GH_NIB_CPL, true>(d, cur, dcur, p, blockIdx.x);
  } else if constexpr (IN == 7) {
    // IN 6 when the host knows a REMOVE is pending (p.rmv_full, the round's
    // stream): one block per workgroup, no block loop (the loop's registers
    // had spilled 72 bytes per lane at 6 waves)
    round_block_nib<TW, NT, GH_NIB_CPL, false>(d, cur, dcur, p, blockIdx.x);
  } else if constexpr (IN == 6) {
    // launched on the side stream every round and idle in most: a grid of
    // 1/8 of the workgroups (an idle full grid cost 30 us of dispatch behind
    // the nibble path), each looping over its blocks when it runs
    constexpr int RB = round_rb<TW>();
    const int nblk = (int)((d.nrows + RB - 1) / RB) * (int)(p.ld / TW);
    for (int b = blockIdx.x; b < nblk; b += gridDim.x) {
      round_block_nib<TW, NT, GH_NIB_CPL, false>(d, cur, dcur, p, b);
      __syncthreads();  // LDS of this block before the next
    }
  } else if constexpr (IN == 5) {
    if constexpr (TW == 256 && GH_NIB_CPL == 16) round_block_nib<TW, NT, 16, false, true>(d, cur, dcur, p, blockIdx.x);
  } else {
    // one block per workgroup (a loop here costs the lean variants 20+ VGPRs)
    round_block<KB, TW, TPW, NT, STORM, IN>(d, cur, dcur, p, blockIdx.x);
  }
}

// The round, slow part: the segments k_round listed, the reference's rule
// cell by cell on exact cells (slave/slave.go:276-286, 414-497; SPEC §2
// steps 1-6), with k_round's lane shape (8 consecutive members per lane, SEG
// lanes per segment, 16-B loads). Reads buffer cur and writes only the
// listed segments of cur ^ 1, narrow where every cell of a segment has a
// narrow code, else into a fresh slot of the next buffer's wide arena. In
// failure storms most segments come here.
template <int TW, int CPL>
__device__ void redo_all(const GhDev& d, int cur, int dcur, const GhRound& p);

// The lane jobs whose segment must go wide (k_round_jobs' redo list): one
// thread, in a kernel of its own (a one-wave grid: its private arrays would
// give every wave of a large grid a scratch allocation, 70 us of dispatch),
// disjoint from the slow list's segments (which never hold lane jobs).
template <int TW>
__global__ __launch_bounds__(64) void k_round_redo(GhDev d, int cur, int dcur, GhRound p) {
  if (threadIdx.x == 0) redo_all<TW, GH_JOB_CPL>(d, cur, dcur, p);
}

template <int TW>
__global__ __launch_bounds__(256) void k_round_slow(GhDev d, int cur, int dcur, GhRound p) {
  constexpr int CPL = 8;
  constexpr int SEG = TW / CPL;
  constexpr int RPW = 64 / SEG;
  const int lane = threadIdx.x & 63;
  const int sub = lane / SEG, lc = lane % SEG;
  const unsigned long long gmask = (SEG == 64 ? ~0ull : ((1ull << SEG) - 1)) << (sub * SEG);
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
  const int64_t nseg = *d.slow_n;
  if (nseg > 0 && blockIdx.x == 0 && threadIdx.x == 0) atomicAdd(&d.nflag[cur ^ 1], 1);  // may write flags
  const bool pull = p.peer_mode == GH_PEER_PULL;
  const int32_t r = p.r;
  const int nxt = cur ^ 1;
  int n_unknown = 0, n_tomb = 0, n_det = 0, n_rel = 0, n_merged = 0;
  for (int64_t s0 = wave * RPW; s0 < nseg; s0 += nw * RPW) {
    const int64_t sid = s0 + sub;
    const bool valid = sid < nseg;
    const int64_t e = d.slow[valid ? sid : s0];
    const int64_t tile = e >> 32;
    const int i = (int)(e & 0xFFFFFFFF);
    const int64_t l0 = tile * TW + lc * CPL;
    const int64_t c0 = d.col0 + l0;
    const bool ac = d.active[i];
    const int cnt = gh_in_cnt(d, pull, p.k, i);
    const int64_t beg = gh_in_beg(d, pull, p.k, i);
    const uint32_t my8 = (d.dbits[l0 >> 5] >> (l0 & 31)) & 0xFFu;
    const bool shr = i == p.shadow_row;  // the introducer's D7 shadow entries (GhDev.shadow)
    bool fit = true, any_det = false;
    int dpres = 0;  // present after - present before
    GhCell o[8];
    uint4 nx = {0u, 0u, 0u, 0u};
    uint4 raw = {0u, 0u, 0u, 0u};  // the chunk as read (narrow codes or a wide marker)
    if (valid) {
      raw = gh_ld16(d, cur, i, l0);
      GhCell A[8], X[8];
      gh_dec8(d, cur, i, l0, r, raw, A);
      int64_t m[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) m[j] = -1;
      for (int q = 0; q < cnt; ++q) {
        const int s = d.inbox[beg + q];
        gh_get8(d, cur, s, l0, r, X);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          // sender snapshot: present and not detected by s, +1 on s's
          // diagonal (its heartbeat of this round), not REMOVE'd at s
          int64_t val = (X[j].x < 0 || X[j].f) ? -1 : (int64_t)X[j].x + ((c0 + j) == s);
          if (((my8 >> j) & 1u) && gh_rm_at(d, dcur, l0 + j, s)) val = -1;
          m[j] = max(m[j], val);
        }
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int64_t c = c0 + j;
        const GhCell v = A[j];
        int64_t x = v.x;
        bool now = false;  // ts := r in this round
        // D7: the introducer's RecentFailList entry beside its present member
        // c: a removal this round keeps that entry (its ts) as the tombstone
        int32_t sh = (shr && x >= 0 && valid) ? d.shadow[l0 + j] : GH_NO_SHADOW;
        const int32_t sh0 = sh;
        int32_t tts = v.ts;  // the ts a tombstone keeps
        // step 1: REMOVE delivery (slave/slave.go:236-240, 276-286)
        if (((my8 >> j) & 1u) && gh_rm_at(d, dcur, l0 + j, i)) {
          if (x >= 0) {
            x = GH_TOMBSTONE;
            if (sh != GH_NO_SHADOW) {  // nothing appended to RecentFailList (:278-281)
              tts = sh;
              sh = GH_NO_SHADOW;
            } else {
              n_tomb++;
            }
          } else if (x == GH_ABSENT) {
            n_unknown++;
          }
        }
        if (!ac) {
          if (x >= 0) now = true;  // step 2 guard (:505-507)
        } else {
          if (c == i) {
            if (x >= 0) {  // step 3 own heartbeat (:443-448); INT32_MAX is refused before the round
              if (x == INT32_MAX) atomicExch(d.err, GH_ERANGE);
              else x += 1;
              now = true;
            }
          } else if (x >= 0 && v.f) {  // step 4 detect (:468-473), decided at the last write
            x = GH_TOMBSTONE;
            if (sh != GH_NO_SHADOW) {
              tts = sh;
              sh = GH_NO_SHADOW;
            }
            n_det++;
            any_det = true;
            atomicAdd(&d.det_cnt[dcur ^ 1][l0 + j], 1);
            atomicMin(&d.det_min[dcur ^ 1][l0 + j], i);
          }
          if (x == GH_TOMBSTONE && (int64_t)tts < (int64_t)r - p.t_cleanup) {  // step 5 clean (:490-492)
            x = GH_ABSENT;
            n_rel++;
          }
          if (sh != GH_NO_SHADOW && (int64_t)sh < (int64_t)r - p.t_cleanup) {  // ... the shadow entry too (D7)
            sh = GH_NO_SHADOW;
            n_rel++;
          }
        }
        if (sh != sh0) {
          d.shadow[l0 + j] = GH_NO_SHADOW;
          atomicSub(d.nshadow, 1);
        }
        if (x >= GH_ABSENT && m[j] > x) {  // step 6 merge (:424-426, :435-437)
          x = m[j];
          now = true;
          n_merged++;
        }
        GhCell out = gh_absent();
        if (x != GH_ABSENT) {
          const int32_t t2 = now ? r : tts;
          out = GhCell{(int32_t)x, t2, x >= 0 && gh_flag_for((int32_t)x, t2, c, i, r + 1, p.t_fail)};
        }
        o[j] = out;
        dpres += (out.x >= 0) - (v.x >= 0);
      }
      nx = gh_enc8(d, nxt, l0, r + 1, o, fit);
    }
    // a segment is narrow iff every lane of it has narrow codes
    const bool narrow = (__ballot(valid && !fit) & gmask) == 0;
    // an inactive row stays a quiet candidate while its segments are
    // rewritten unchanged (narrow, same codes; a wide input never is)
    const bool same = narrow && (raw.x & 0xFFFFu) != GH_N_WIDE && raw.x == nx.x && raw.y == nx.y &&
                      raw.z == nx.z && raw.w == nx.w;
    const bool seg_same = (__ballot(valid && !same) & gmask) == 0;
    if (valid) {
      int64_t slot = 0;
      if (!narrow) {
        const int64_t sl = lc == 0 ? gh_wide_alloc(d, nxt) : 0;
        slot = __shfl(sl, sub * SEG);
      }
      if (slot >= 0) gh_put8(d, nxt, i, l0, narrow, nx, slot, o);  // with its plane word (wide: unknown, 0)
    }
#pragma unroll
    for (int o2 = SEG / 2; o2 > 0; o2 >>= 1) {
      dpres += __shfl_xor(dpres, o2);
      any_det |= __shfl_xor((int)any_det, o2) != 0;
    }
    if (lc == 0 && valid) {
      if (dpres) atomicAdd(&d.cntl[i], dpres);
      if (any_det) d.det_any[i] = 1;
      if (ac || !seg_same) d.stab[(p.r + 1) & 1][i] = 0;
    }
  }
  if (n_unknown) atomicAdd(&d.stats[ST_REMOVE_UNKNOWN], (unsigned long long)n_unknown);
  if (n_tomb) atomicAdd(&d.stats[ST_TOMBSTONED], (unsigned long long)n_tomb);
  if (n_det) atomicAdd(&d.stats[ST_DETECTIONS], (unsigned long long)n_det);
  if (n_rel) atomicAdd(&d.stats[ST_RELEASED], (unsigned long long)n_rel);
  if (n_merged) atomicAdd(&d.stats[ST_MERGED], (unsigned long long)n_merged);
}

// ---- lane jobs of the nibble path (gh_internal.h: jobs) ------------------
// Per-lane tallies of a job's cells.
struct JobAcc {
  int unknown, tomb, det, rel, merged, dpres, esc;
  bool flag, any_det;
};
// The reference's rule cell by cell (SPEC §2 steps 1, 3-6 of an active row;
// slave/slave.go:276-286, 414-497) for the 8 cells (i, l0 .. l0 + 7) of a
// lane job, given as A (exact cells of buffer cur): the same per-cell code
// as k_round_slow, but each cell's merge candidate comes from the senders'
// minimum plane code u (nibble gh_nib(j) of uw) the nibble path already
// gathered: the freshest sender entry is bo[j] + GH_P_REF + 1 - u (exact for
// u in 1..13; 15 = no entry). A cell of a REMOVE'd column (only a sole
// detector keeps it, :344-346) or with an unknown (0) or old (14) code
// gathers its senders' exact cells instead. Detections come back as a cell
// mask (detm) for the caller to count once the chunk is written. Returns the
// cells for buffer cur ^ 1 in o.
__device__ __forceinline__ void job_rule(const GhDev& d, int cur, int dcur, const GhRound& p, int i, int64_t l0,
                                         uint32_t uw, const GhCell A[8], const int32_t bo[8], GhCell o[8], JobAcc& a,
                                         uint32_t& detm) {
  const int32_t r = p.r;
  const int64_t c0 = d.col0 + l0;
  const uint32_t my8 = (d.dbits[l0 >> 5] >> (l0 & 31)) & 0xFFu;
  detm = 0;
  // merge candidates: from the plane codes, then (a rolled loop: the code
  // stays small) the cells that gather their senders' exact cells
  int64_t mm[8];
  uint32_t ex = 0;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const uint32_t u = (uw >> gh_nib(j)) & 0xFu;
    mm[j] = u == GH_P_NONE ? -1 : (int64_t)bo[j] + (GH_P_REF + 1 - (int)u);
    if (((my8 >> j) & 1u) || u == GH_P_UNK || u == GH_P_OLD) ex |= 1u << j;
  }
  if (ex) {
    const bool pull = p.peer_mode == GH_PEER_PULL;
    const int cnt = gh_in_cnt(d, pull, p.k, i);
    const int64_t beg = gh_in_beg(d, pull, p.k, i);
#pragma unroll 1
    for (; ex; ex &= ex - 1) {
      const int j = __builtin_ctz(ex);
      const bool rmj = (my8 >> j) & 1u;
      int64_t m = -1;
#pragma unroll 1
      for (int q = 0; q < cnt; ++q) {
        const int s = d.inbox[beg + q];
        if (rmj && gh_rm_at(d, dcur, l0 + j, s)) continue;  // s REMOVEs it before sending
        if (rmj && d.soleval && !d.rlist) {  // s is its sole detector (row shards: maybe a ghost)
          m = max(m, (int64_t)d.soleval[l0 + j]);
          continue;
        }
        const GhCell X = gh_get(d, cur, s, l0 + j, r);
        if (X.x >= 0 && !X.f) m = max(m, (int64_t)X.x + ((c0 + j) == s));
      }
#pragma unroll
      for (int q = 0; q < 8; ++q)
        if (q == j) mm[q] = m;
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int64_t c = c0 + j;
    const bool rmj = (my8 >> j) & 1u;
    const int64_t m = mm[j];
    const GhCell v = A[j];
    int64_t x = v.x;
    bool now = false;  // ts := r in this round
    if (rmj && gh_rm_at(d, dcur, l0 + j, i)) {  // step 1: REMOVE delivery (:236-240, 276-286)
      if (x >= 0) {
        x = GH_TOMBSTONE;
        a.tomb++;
      } else if (x == GH_ABSENT) {
        a.unknown++;
      }
    }
    if (c == i) {
      if (x >= 0) {  // step 3 own heartbeat (:443-448); INT32_MAX is refused before the round
        if (x == INT32_MAX) atomicExch(d.err, GH_ERANGE);
        else x += 1;
        now = true;
      }
    } else if (x >= 0 && v.f) {  // step 4 detect (:468-473), decided at the last write
      x = GH_TOMBSTONE;
      a.det++;
      a.any_det = true;
      detm |= 1u << j;
    }
    if (x == GH_TOMBSTONE && (int64_t)v.ts < (int64_t)r - p.t_cleanup) {  // step 5 clean (:490-492)
      x = GH_ABSENT;
      a.rel++;
    }
    if (x >= GH_ABSENT && m > x) {  // step 6 merge (:424-426, :435-437)
      x = m;
      now = true;
      a.merged++;
    }
    GhCell out = gh_absent();
    if (x != GH_ABSENT) {
      const int32_t t2 = now ? r : v.ts;
      out = GhCell{(int32_t)x, t2, x >= 0 && gh_flag_for((int32_t)x, t2, c, i, r + 1, p.t_fail)};
      a.flag |= out.f;
    }
    o[j] = out;
    a.dpres += (out.x >= 0) - (v.x >= 0);
  }
}

// One chunk (i, l0 .. l0 + 7) of a lane job, lean: its codes in buffer cur
// (the tier's nibbles or, escaped, the 16-bit chunk: the three words are
// loaded together), the rule of job_rule in 32-bit arithmetic on decoded
// cells (every value an encodable cell can take fits: heartbeats <= INT32_MAX
// with the INT32_MAX refusal before the round), and, when every result has a
// narrow code, the write of buffer cur ^ 1 (tier chunk where it fits, else
// escaped, with its plane word). Returns false, writing nothing, when the
// input is a wide segment or a result needs the wide arena (the redo pass, redo_all).
__device__ __forceinline__ bool job_chunk(const GhDev& d, int cur, int dcur, const GhRound& p, int i, int64_t l0,
                                          uint32_t uw, uint32_t plw, uint32_t a4w, JobAcc& acc, uint32_t& detm) {
  const int nxt = cur ^ 1;
  const int32_t r = p.r;
  const int64_t cell = gh_cell(d, i, l0);
  const int jd = gh_jd(d, i, l0);
  const int4 b0 = *reinterpret_cast<const int4*>(d.base[cur] + l0);
  const int4 b1 = *reinterpret_cast<const int4*>(d.base[cur] + l0 + 4);
  const int4 n0 = *reinterpret_cast<const int4*>(d.base[nxt] + l0);
  const int4 n1 = *reinterpret_cast<const int4*>(d.base[nxt] + l0 + 4);
  const int32_t bo[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
  const int32_t bn[8] = {n0.x, n0.y, n0.z, n0.w, n1.x, n1.y, n1.z, n1.w};
  uint32_t xw[4];
  if (!gh_t4_esc(a4w)) {
    const v4u w = c4_dec(plw, a4w, jd, d.toff);
    xw[0] = w[0], xw[1] = w[1], xw[2] = w[2], xw[3] = w[3];
  } else {  // an escaped chunk: its 16-bit codes
    const uint4 hx = *reinterpret_cast<const uint4*>(d.hn[cur] + cell);
    xw[0] = hx.x, xw[1] = hx.y, xw[2] = hx.z, xw[3] = hx.w;
  }
  const uint32_t h0 = xw[0] & 0xFFFFu;
  if (h0 == GH_N_WIDE || h0 == GH_N_FROZEN) return false;  // a wide input: the redo pass (redo_all)
  const uint32_t my8 = (d.dbits[l0 >> 5] >> (l0 & 31)) & 0xFFu;
  // merge candidates: from the plane codes, then (a rolled loop) the cells
  // that gather their senders' exact cells
  int32_t mm[8];
  uint32_t ex = 0;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const uint32_t u = (uw >> gh_nib(j)) & 0xFu;
    mm[j] = u == GH_P_NONE ? -1 : bo[j] + (GH_P_REF + 1 - (int32_t)u);
    if (((my8 >> j) & 1u) || u == GH_P_UNK || u == GH_P_OLD) ex |= 1u << j;
  }
  const int64_t c0 = d.col0 + l0;
  if (ex) {
    const bool pull = p.peer_mode == GH_PEER_PULL;
    const int cnt = gh_in_cnt(d, pull, p.k, i);
    const int64_t beg = gh_in_beg(d, pull, p.k, i);
#pragma unroll 1
    for (; ex; ex &= ex - 1) {
      const int j = __builtin_ctz(ex);
      const bool rmj = (my8 >> j) & 1u;
      int32_t m = -1;
      bool okg = true;
#pragma unroll 1
      for (int q = 0; q < cnt; ++q) {
        const int s = d.inbox[beg + q];
        if (rmj && gh_rm_at(d, dcur, l0 + j, s)) continue;  // s REMOVEs it before sending
        // the sender's cell from its narrow code (a tier nibble or an escaped
        // code); a wide or stopped sender segment: the redo pass (redo_all)
        const int64_t sl = gh_slot(d, s);
        uint32_t h;
        if (d.gcodes && sl >= d.nrows) {  // row layout: a ghost row, 16-bit codes in the ghost table
          const uint16_t* gr = d.gcodes + (sl - d.nrows) * d.ld;
          h = gr[l0 + j];
          const uint32_t h0 = gr[(l0 + j) & ~(int64_t)7];
          okg &= h0 != GH_N_WIDE && h0 != GH_N_FROZEN;
          const int32_t off = (int32_t)((h >> 5) & 1023u);
          if (h != GH_N_ABSENT && off != 1023 && (h >> 15) == 0)
            m = max(m, d.base[cur][l0 + j] + off + (int32_t)((c0 + j) == s));
          continue;
        }
        const int64_t sc = gh_cell_slot(d, sl, l0 + j);
        const uint32_t sa = d.a4[cur][sc >> 3];
        if (gh_t4_esc(sa)) {
          h = d.hn[cur][sc];
          const uint32_t h0 = d.hn[cur][sc & ~(int64_t)7];
          okg &= h0 != GH_N_WIDE && h0 != GH_N_FROZEN;
        } else {
          const uint32_t u = (d.pl[cur][sc >> 3] >> gh_nib((int)(sc & 7))) & 0xFu;
          // tier: visible with offset GH_P_REF + 1 - u (GH_P_REF - u on s's
          // own member, its plane diagonal code), or absent (15)
          h = u == GH_P_NONE ? GH_N_ABSENT : (uint32_t)(GH_P_REF + 1 - (int)u - (int)((c0 + j) == s)) << 5;
        }
        const int32_t off = (int32_t)((h >> 5) & 1023u);
        if (h != GH_N_ABSENT && off != 1023 && (h >> 15) == 0)  // present and not flagged (detected by s)
          m = max(m, d.base[cur][l0 + j] + off + (int32_t)((c0 + j) == s));
      }
      if (!okg) return false;
#pragma unroll
      for (int q = 0; q < 8; ++q)
        if (q == j) mm[q] = m;
    }
  }
  uint32_t nw[4] = {0u, 0u, 0u, 0u};
  bool fit = true;
  detm = 0;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int64_t c = c0 + j;
    // the cell (x, ts, flag) of buffer cur (SPEC §1)
    const uint32_t h = (xw[j >> 1] >> (16 * (j & 1))) & 0xFFFFu;
    const int32_t age = (int32_t)(h & 31u), off = (int32_t)((h >> 5) & 1023u);
    const int32_t vx = h == GH_N_ABSENT ? GH_ABSENT : off == 1023 ? GH_TOMBSTONE : bo[j] + off;
    const int32_t vts = r - age;
    const bool vf = vx >= 0 && (h >> 15) != 0;
    int32_t x = vx;
    bool now = false;  // ts := r in this round
    if (((my8 >> j) & 1u) && gh_rm_at(d, dcur, l0 + j, i)) {  // step 1 REMOVE (:236-240, 276-286)
      if (x >= 0) {
        x = GH_TOMBSTONE;
        acc.tomb++;
      } else if (x == GH_ABSENT) {
        acc.unknown++;
      }
    }
    if (c == i) {
      if (x >= 0) {  // step 3 own heartbeat (:443-448); INT32_MAX is refused before the round
        if (x == INT32_MAX) atomicExch(d.err, GH_ERANGE);
        else x += 1;
        now = true;
      }
    } else if (x >= 0 && vf) {  // step 4 detect (:468-473), decided at the last write
      x = GH_TOMBSTONE;
      acc.det++;
      acc.any_det = true;
      detm |= 1u << j;
    }
    if (x == GH_TOMBSTONE && vts < r - p.t_cleanup) {  // step 5 clean (:490-492)
      x = GH_ABSENT;
      acc.rel++;
    }
    if (x >= GH_ABSENT && mm[j] > x) {  // step 6 merge (:424-426, :435-437)
      x = mm[j];
      now = true;
      acc.merged++;
    }
    // the cell for round r + 1 in buffer cur ^ 1, narrow (gh_enc16)
    uint32_t code = GH_N_ABSENT;
    if (x != GH_ABSENT) {
      const int32_t t2 = now ? r : vts;
      int32_t a2 = r + 1 - t2;
      if (x < 0) {
        if (d.tsa && a2 > d.tsa) a2 = d.tsa;
        fit &= a2 >= 0 && a2 <= GH_N_TAGEMAX;
        code = GH_N_TOMB | ((uint32_t)a2 & 31u);
      } else {
        const bool fl = x > 1 && c != i && t2 < r + 1 - p.t_fail;  // gh_flag_for, round r + 1
        const uint32_t o2 = (uint32_t)x - (uint32_t)bn[j];          // x - base, wrapped if below
        fit &= o2 <= (uint32_t)GH_N_OFFMAX && a2 >= 0 && a2 <= GH_N_AGEMAX;
        code = (fl ? 0x8000u : 0u) | ((o2 & 1023u) << 5) | ((uint32_t)a2 & 31u);
        acc.flag |= fl;
      }
    }
    nw[j >> 1] |= code << (16 * (j & 1));
    acc.dpres += (x >= 0) - (vx >= 0);
  }
  if (!fit) return false;
  const v4u nv = {nw[0], nw[1], nw[2], nw[3]};
  d.pl[nxt][cell >> 3] = plane_word(nv, jd);
  uint32_t a4n;
  if (c4_enc(nv, jd, a4n, d.toff)) {
    d.a4[nxt][cell >> 3] = a4n;
  } else {
    d.a4[nxt][cell >> 3] = GH_T4_ESC;
    *reinterpret_cast<uint4*>(d.hn[nxt] + cell) = uint4{nw[0], nw[1], nw[2], nw[3]};
    acc.esc++;
  }
  return true;
}

// The lane jobs the nibble path wrote this round (only when it ran: m8[4] =
// 3), one workgroup per nibble workgroup's region at a time (one tile, one
// block of rows): detections aggregate per column and row-count deltas per
// row in LDS. A job whose cells all have narrow codes is written here (tier
// chunks where they fit, else escaped 16-bit chunks, with their plane
// words); one that needs the wide arena goes to the redo list.
template <int TW, int CPL>
__global__ __launch_bounds__(256, GH_JOB_WAVES) void k_round_jobs(GhDev d, int cur, int dcur, GhRound p) {
  if (d.m8[4] != 3) return;
  const int nlist = d.njobs[3];  // the nibble workgroups with jobs (none in a quiet steady-state round)
  if (nlist == 0) return;
  constexpr int W = CPL / 8;
  constexpr int RB = round_rb<TW>();
  __shared__ int s_dcnt[TW], s_dmin[TW], s_drow[RB];
  __shared__ unsigned long long s_st[6];  // unknown, tomb, det, rel, merged, escaped chunks
  __shared__ int s_jobs, s_flag;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int nxt = cur ^ 1;
  if (threadIdx.x < 6) s_st[threadIdx.x] = 0;
  if (threadIdx.x == 0) s_jobs = s_flag = 0;
  JobAcc tot{};
  for (int x = blockIdx.x; x < nlist; x += gridDim.x) {
    const int64_t b = d.jlist[x];
    const int nj = d.jobn[b * 4 + wave];
    int tile, rb;
    nib_region<TW>(d, p, (int)b, tile, rb);
    const int64_t cbase = (int64_t)tile * TW;
    const int64_t rbase = d.row0 + (int64_t)rb * RB;
    for (int t = threadIdx.x; t < TW; t += 256) {
      s_dcnt[t] = 0;
      s_dmin[t] = INT_MAX;
    }
    for (int t = threadIdx.x; t < RB; t += 256) s_drow[t] = 0;
    __syncthreads();
    const uint4* jreg = d.jobs + (b * 4 + wave) * GH_JOB_CAP * 2;
    for (int e = lane; e < nj; e += 64) {
      const uint4 jb = jreg[2 * e];
      const uint4 jo = jreg[2 * e + 1];  // the lane's own lag words, age words
      const int i = (int)jb.x;
      const int64_t l0 = (int64_t)(jb.y >> 8) * TW + (int64_t)(jb.y & 255u) * CPL;
      uint32_t detl = 0;  // detections, bit 8 w + j
      JobAcc a{};
      bool fit = true;
      // chunk by chunk (a rolled loop: the code stays small), each written as
      // soon as it is known to fit; a chunk that needs the wide arena sends
      // the lane to the redo pass (redo_all, k_round_redo), which recomputes and counts it whole
      // (overwriting any chunk written here)
#pragma unroll 1
      for (int w = 0; w < W && fit; ++w) {
        uint32_t dm8 = 0;
        fit = job_chunk(d, cur, dcur, p, i, l0 + 8 * w, w ? jb.w : jb.z, w ? jo.y : jo.x, w ? jo.w : jo.z, a, dm8);
        detl |= dm8 << (8 * w);
      }
      if (!fit) {
        const int pos = atomicAdd(&d.njobs[1], 1);
        if (pos < GH_REDO_CAP) d.redo[pos] = jb;
        else atomicExch(d.err, GH_ENOMEM);
        continue;
      }
      for (uint32_t m = detl; m; m &= m - 1) {
        const int64_t t = l0 + __builtin_ctz(m) - cbase;
        atomicAdd(&s_dcnt[t], 1);
        atomicMin(&s_dmin[t], i);
      }
      if (a.dpres) atomicAdd(&s_drow[i - rbase], a.dpres);
      if (a.any_det) d.det_any[i] = 1;
      tot.unknown += a.unknown;
      tot.tomb += a.tomb;
      tot.det += a.det;
      tot.rel += a.rel;
      tot.merged += a.merged;
      tot.esc += a.esc;
      tot.flag |= a.flag;
    }
    if (lane == 0 && nj) atomicAdd(&s_jobs, nj);
    __syncthreads();
    for (int t = threadIdx.x; t < TW; t += 256)
      if (s_dcnt[t]) {
        atomicAdd(&d.det_cnt[dcur ^ 1][cbase + t], s_dcnt[t]);
        atomicMin(&d.det_min[dcur ^ 1][cbase + t], s_dmin[t]);
      }
    for (int t = threadIdx.x; t < RB; t += 256)
      if (s_drow[t]) atomicAdd(&d.cntl[rbase + t], s_drow[t]);
  }
  if (tot.unknown) atomicAdd(&s_st[0], (unsigned long long)tot.unknown);
  if (tot.tomb) atomicAdd(&s_st[1], (unsigned long long)tot.tomb);
  if (tot.det) atomicAdd(&s_st[2], (unsigned long long)tot.det);
  if (tot.rel) atomicAdd(&s_st[3], (unsigned long long)tot.rel);
  if (tot.merged) atomicAdd(&s_st[4], (unsigned long long)tot.merged);
  if (tot.esc) atomicAdd(&s_st[5], (unsigned long long)tot.esc);
  if (tot.flag) s_flag = 1;
  __syncthreads();
  if (threadIdx.x == 0) {
    if (s_st[0]) atomicAdd(&d.stats[ST_REMOVE_UNKNOWN], s_st[0]);
    if (s_st[1]) atomicAdd(&d.stats[ST_TOMBSTONED], s_st[1]);
    if (s_st[2]) atomicAdd(&d.stats[ST_DETECTIONS], s_st[2]);
    if (s_st[3]) atomicAdd(&d.stats[ST_RELEASED], s_st[3]);
    if (s_st[4]) atomicAdd(&d.stats[ST_MERGED], s_st[4]);
    if (s_st[5]) atomicAdd(&d.m8[3], (int)s_st[5]);
    if (s_jobs) atomicAdd(&d.njobs[0], s_jobs);
    if (s_flag) atomicAdd(&d.nflag[nxt], 1);  // the quirk gate: written segments may hold flags
  }
}

// The same lane jobs with every lane busy: a wave takes 64 (nibble
// workgroup, wave) job regions at once, scans their job counts and deals the
// jobs out one per lane (a region usually holds one or two, so the
// one-region-at-a-time form above ran most of its lanes empty and synced
// its workgroup twice per region). Detections and row counts go straight to
// the global counters (a region's jobs rarely share a column or a row).
template <int TW, int CPL>
__global__ __launch_bounds__(256, GH_JOBF_WAVES) void k_round_jobs_flat(GhDev d, int cur, int dcur, GhRound p) {
  if (d.m8[4] != 3) return;
  const int nlist = d.njobs[3];  // the nibble workgroups with jobs (none in a quiet steady-state round)
  if (nlist == 0) return;
  constexpr int W = CPL / 8;
  __shared__ unsigned long long s_st[6];  // unknown, tomb, det, rel, merged, escaped chunks
  __shared__ int s_jobs, s_flag;
  // per wave: its 64 regions' inclusive job counts and region indices (in LDS,
  // not registers: the job rule needs all 128 the 4-wave bound leaves)
  __shared__ int s_incl[4][64];
  __shared__ int s_reg[4][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int nxt = cur ^ 1;
  if (threadIdx.x < 6) s_st[threadIdx.x] = 0;
  if (threadIdx.x == 0) s_jobs = s_flag = 0;
  __syncthreads();
  JobAcc tot{};
  const int64_t nslot = (int64_t)nlist * 4;
  const int64_t nwv = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t s0 = (((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6) * 64; s0 < nslot; s0 += nwv * 64) {
    const int64_t sl = s0 + lane;
    int reg = 0, nj = 0;
    if (sl < nslot) {
      reg = d.jlist[sl >> 2] * 4 + (int)(sl & 3);
      nj = d.jobn[reg];
    }
    int incl = nj;  // inclusive scan of the regions' job counts
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int y = __shfl_up(incl, o);
      if (lane >= o) incl += y;
    }
    const int total = __builtin_amdgcn_readfirstlane(__shfl(incl, 63));  // (wave-uniform)
    if (lane == 0 && total) atomicAdd(&s_jobs, total);
    __builtin_amdgcn_wave_barrier();  // (the last step's reads of this wave's slots are done)
    s_incl[wave][lane] = incl;
    s_reg[wave][lane] = reg;
    __builtin_amdgcn_wave_barrier();
    for (int base = 0; base < total; base += 64) {
      const int t = base + lane;
      if (t >= total) continue;
      // the region holding job t: the first slot whose inclusive count exceeds t
      int lo = 0;
#pragma unroll
      for (int st = 32; st > 0; st >>= 1)
        if (s_incl[wave][lo + st - 1] <= t) lo += st;
      const int before = lo ? s_incl[wave][lo - 1] : 0;
      const uint4* jreg = d.jobs + (int64_t)s_reg[wave][lo] * GH_JOB_CAP * 2;
      const int e = t - before;
      const uint4 jb = jreg[2 * e];
      const uint4 jo = jreg[2 * e + 1];  // the lane's own lag words, age words
      const int i = (int)jb.x;
      const int64_t l0 = (int64_t)(jb.y >> 8) * TW + (int64_t)(jb.y & 255u) * CPL;
      uint32_t detl = 0;  // detections, bit 8 w + j
      JobAcc a{};
      bool fit = true;
#pragma unroll 1
      for (int w = 0; w < W && fit; ++w) {
        uint32_t dm8 = 0;
        fit = job_chunk(d, cur, dcur, p, i, l0 + 8 * w, w ? jb.w : jb.z, w ? jo.y : jo.x, w ? jo.w : jo.z, a, dm8);
        detl |= dm8 << (8 * w);
      }
      if (!fit) {  // the redo pass recomputes and counts the lane whole
        const int pos = atomicAdd(&d.njobs[1], 1);
        if (pos < GH_REDO_CAP) d.redo[pos] = jb;
        else atomicExch(d.err, GH_ENOMEM);
        continue;
      }
      for (uint32_t m = detl; m; m &= m - 1) {
        const int64_t c = l0 + __builtin_ctz(m);
        atomicAdd(&d.det_cnt[dcur ^ 1][c], 1);
        atomicMin(&d.det_min[dcur ^ 1][c], i);
      }
      if (a.dpres) atomicAdd(&d.cntl[i], a.dpres);
      if (a.any_det) d.det_any[i] = 1;
      tot.unknown += a.unknown;
      tot.tomb += a.tomb;
      tot.det += a.det;
      tot.rel += a.rel;
      tot.merged += a.merged;
      tot.esc += a.esc;
      tot.flag |= a.flag;
    }
  }
  if (tot.unknown) atomicAdd(&s_st[0], (unsigned long long)tot.unknown);
  if (tot.tomb) atomicAdd(&s_st[1], (unsigned long long)tot.tomb);
  if (tot.det) atomicAdd(&s_st[2], (unsigned long long)tot.det);
  if (tot.rel) atomicAdd(&s_st[3], (unsigned long long)tot.rel);
  if (tot.merged) atomicAdd(&s_st[4], (unsigned long long)tot.merged);
  if (tot.esc) atomicAdd(&s_st[5], (unsigned long long)tot.esc);
  if (tot.flag) s_flag = 1;
  __syncthreads();
  if (threadIdx.x == 0) {
    if (s_st[0]) atomicAdd(&d.stats[ST_REMOVE_UNKNOWN], s_st[0]);
    if (s_st[1]) atomicAdd(&d.stats[ST_TOMBSTONED], s_st[1]);
    if (s_st[2]) atomicAdd(&d.stats[ST_DETECTIONS], s_st[2]);
    if (s_st[3]) atomicAdd(&d.stats[ST_RELEASED], s_st[3]);
    if (s_st[4]) atomicAdd(&d.stats[ST_MERGED], s_st[4]);
    if (s_st[5]) atomicAdd(&d.m8[3], (int)s_st[5]);
    if (s_jobs) atomicAdd(&d.njobs[0], s_jobs);
    if (s_flag) atomicAdd(&d.nflag[nxt], 1);  // the quirk gate: written segments may hold flags
  }
}

// Lane jobs whose cells need the wide arena (k_round_jobs' redo list), by
// one thread: each listed segment becomes wide in buffer cur ^ 1 (a fresh
// arena slot holding every chunk as the nibble path and the jobs wrote it),
// then every listed lane of that segment writes its exact cells into the
// slot. Rare (imports far from the counters, views older than the 16-bit
// window), so the search for a segment's other entries is a plain scan.
template <int TW, int CPL>
__device__ __forceinline__ void redo_lane(const GhDev& d, int cur, int dcur, const GhRound& p, const uint4& jb,
                                          int64_t slot, JobAcc& tot) {
  constexpr int W = CPL / 8;
  const int i = (int)jb.x;
  const int64_t l0 = (int64_t)(jb.y >> 8) * TW + (int64_t)(jb.y & 255u) * CPL;
  const uint32_t uw[2] = {jb.z, jb.w};
  JobAcc a{};
#pragma unroll
  for (int w = 0; w < W; ++w) {
    const int64_t c = l0 + 8 * w;
    const int4 b0 = *reinterpret_cast<const int4*>(d.base[cur] + c);
    const int4 b1 = *reinterpret_cast<const int4*>(d.base[cur] + c + 4);
    const int32_t bo[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
    GhCell A[8], o[8];
    gh_get8(d, cur, i, c, p.r, A);
    uint32_t detm;
    job_rule(d, cur, dcur, p, i, c, uw[w], A, bo, o, a, detm);
    bool fit = true;
    const uint4 nx = gh_enc8(d, cur ^ 1, c, p.r + 1, o, fit);
    gh_put8(d, cur ^ 1, i, c, false, nx, slot, o);
    for (uint32_t m = detm; m; m &= m - 1) {
      const int64_t cc = c + __builtin_ctz(m);
      atomicAdd(&d.det_cnt[dcur ^ 1][cc], 1);
      atomicMin(&d.det_min[dcur ^ 1][cc], i);
    }
  }
  if (a.dpres) atomicAdd(&d.cntl[i], a.dpres);
  if (a.any_det) d.det_any[i] = 1;
  tot.unknown += a.unknown;
  tot.tomb += a.tomb;
  tot.det += a.det;
  tot.rel += a.rel;
  tot.merged += a.merged;
}
template <int TW, int CPL>
__device__ void redo_all(const GhDev& d, int cur, int dcur, const GhRound& p) {
  if (d.m8[4] != 3) return;
  const int nr = min(d.njobs[1], GH_REDO_CAP);
  const int nxt = cur ^ 1;
  JobAcc tot{};
  for (int e = 0; e < nr; ++e) {
    const uint4 jb = d.redo[e];
    if (jb.x == 0xFFFFFFFFu) continue;  // done with an earlier entry of its segment
    const int i = (int)jb.x;
    const int64_t t0 = (int64_t)(jb.y >> 8) * TW;
    const int64_t slot = gh_wide_alloc(d, nxt);
    if (slot < 0) return;  // the arena is full: err = GH_ENOMEM, the state is lost
    for (int64_t c = t0; c < t0 + TW; c += 8) {  // the segment as written so far, into the slot
      GhCell v[8];
      gh_get8(d, nxt, i, c, p.r + 1, v);
      gh_put8(d, nxt, i, c, false, uint4{0u, 0u, 0u, 0u}, slot, v);
    }
    redo_lane<TW, CPL>(d, cur, dcur, p, jb, slot, tot);
    for (int e2 = e + 1; e2 < nr; ++e2) {
      const uint4 j2 = d.redo[e2];
      if (j2.x == jb.x && (j2.y >> 8) == (jb.y >> 8)) {
        redo_lane<TW, CPL>(d, cur, dcur, p, j2, slot, tot);
        d.redo[e2].x = 0xFFFFFFFFu;
      }
    }
  }
  if (nr) atomicAdd(&d.nflag[nxt], 1);
  if (tot.unknown) atomicAdd(&d.stats[ST_REMOVE_UNKNOWN], (unsigned long long)tot.unknown);
  if (tot.tomb) atomicAdd(&d.stats[ST_TOMBSTONED], (unsigned long long)tot.tomb);
  if (tot.det) atomicAdd(&d.stats[ST_DETECTIONS], (unsigned long long)tot.det);
  if (tot.rel) atomicAdd(&d.stats[ST_RELEASED], (unsigned long long)tot.rel);
  if (tot.merged) atomicAdd(&d.stats[ST_MERGED], (unsigned long long)tot.merged);
}

// Columns: bitmap + list of D_r, and reset the consumed D_{r-1}
// accumulators for reuse in round r+1 (the rows' counts are kept current by
// the round kernels).
__global__ __launch_bounds__(256) void k_finish(GhDev d, int dcur, GhRound p) {
  const int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int dnew = dcur ^ 1;
  bool has = false, sole = false;
  if (x == 0) d.aq[0] = 0;  // the next round's writers of base_col / the inbox pass set it
  if (x < p.ld) {
    has = d.det_cnt[dnew][x] > 0;
    sole = d.det_cnt[dnew][x] == 1;
    d.det_cnt[dcur][x] = 0;
    d.det_min[dcur][x] = INT_MAX;
  }
  const unsigned long long m = __ballot(has), ms = __ballot(sole);
  const int lane = threadIdx.x & 63;
  if (x - lane < p.ld && lane == 0) {
    const int64_t w = (x - lane) >> 5;
    d.dbits[w] = (uint32_t)m;
    d.dbits[w + 1] = (uint32_t)(m >> 32);
    d.sbits[w] = (uint32_t)ms;
    d.sbits[w + 1] = (uint32_t)(ms >> 32);
    if (m) {
      atomicAdd(&d.nd[dnew], __popcll(m));
      if (!d.rowlay || d.rank == 0)  // row layout: every shard holds all columns
        atomicAdd(&d.stats[ST_FAILED], (unsigned long long)__popcll(m));
    }
  }
  if (has) {
    // list order is irrelevant: only k_active_pre's recount reads it
    const int pos = atomicAdd(&d.nd[2 + dnew], 1);
    d.dlist[(int64_t)dnew * p.ld + pos] = (int32_t)x;
  }
}

// ---- quirk-mode detection (SPEC §4, slave/slave.go:464-477 with :283) ----
// detectfailure ranges over the slice removeMember shifts, so in each run of
// consecutive candidates (in list order = present cells after REMOVE, member
// order) only the candidates at even offsets are removed, plus the last list
// entry if it is a candidate. The pre-pass below rewrites the detection flag
// of the current table to exactly that set, so k_round (detection) and the
// peers (a sender's snapshot keeps its skipped candidates) follow it as is.
//
// Run state s = parity of the trailing run of candidates before a cell (0 at
// the start of a row). A stretch of cells maps s to f(s): with a present
// non-candidate in it f is constant (the parity of the candidates after the
// last one), else f(s) = s ^ (its candidates & 1). Bits: 0 = has a present
// non-candidate, 1 = value, 2 = has a present cell.
__device__ __forceinline__ int q_compose(int a, int b) {  // a, then b
  return ((a | b) & 5) | ((b & 1) ? (b & 2) : ((a ^ b) & 2));
}
__device__ __forceinline__ int q_apply(int f, int s) { return (f & 1) ? ((f >> 1) & 1) : (s ^ ((f >> 1) & 1)); }
// The composed map of 8 consecutive cells with list members P and candidates
// F (F within P), in closed form: with a non-candidate in the stretch, the
// parity of the candidates after the last one; else the parity of all.
__device__ __forceinline__ int q_summary8(uint32_t P, uint32_t F) {
  if (!P) return 0;
  const uint32_t B = P & ~F;
  if (B) return 5 | ((__builtin_popcount(F >> (32 - __builtin_clz(B))) & 1) << 1);
  return 4 | ((__builtin_popcount(F) & 1) << 1);
}

// one segment per (tile, row): the tile's run summary (segmented scan over
// the SEG lanes, last lane holds the whole tile). A wave takes U segment
// steps per iteration, their tier words loaded together (a full-table sweep
// at one step in flight per wave was latency-bound: ~1 TB/s).
template <int TW>
__global__ __launch_bounds__(256) void k_quirk_sum(GhDev d, int cur, int dcur, GhRound p) {
  if (p.qgate && d.cntg[p.n + 1] == 0) return;  // no candidate in any shard's table
  constexpr int SEG = SegWalk<TW>::SEG;
  constexpr int U = 4;
  const SegWalk<TW> w(d, p);
  const bool tier = gh_m8(d, cur);
  const unsigned long long smask = ((SEG == 64) ? ~0ull : ((1ull << SEG) - 1)) << (w.sub * SEG);
  int64_t run0, run1;
  w.run(U, run0, run1);
  for (int64_t base = run0; base < run1; base += U * w.RPW) {
    int64_t tu[U];
    int iu[U];
    bool vu[U];
    uint32_t au[U], qu[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t sid = base + u * w.RPW + w.sub;
      vu[u] = sid < run1;
      tu[u] = 0;
      iu[u] = (int)w.row0;
      if (vu[u]) w.at(sid, tu[u], iu[u]);
      au[u] = 0u;
      qu[u] = 0u;
      if (vu[u] && tier) {  // (issued before the row's state is known: no dependent load chain)
        const int64_t wi = gh_cell(d, iu[u], tu[u] * TW + w.lc * 8) >> 3;
        au[u] = d.a4[cur][wi];
        qu[u] = d.pl[cur][wi];
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u)  // only active rows detect (k_quirk_apply): a stopped row's frozen cells are not decoded
      vu[u] = vu[u] && d.alive[iu[u]] && d.active[iu[u]];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t c = tu[u] * TW + w.lc * 8;
      int f = 0;
      bool esc = false;
      if (vu[u]) {
        uint32_t pf;
        if (tier && !gh_t4_esc(au[u])) {
          pf = gh_t4_present8(qu[u]);  // a tier chunk: no flag
        } else {
          esc = true;
          pf = gh_pf8(d, cur, iu[u], c);
        }
        const uint32_t P = pf & ~removed8(d, dcur, c, iu[u]) & 0xFFu;
        f = q_summary8(P, (pf >> 8) & P);
      }
      // (bit 3 of the stored summary: the segment holds a chunk that can
      // hold flags, i.e. an escaped one; k_quirk_apply skips the others)
      const bool seg_esc = (__ballot(esc) & smask) != 0;
#pragma unroll
      for (int o = 1; o < SEG; o <<= 1) {
        const int other = __shfl_up(f, o, SEG);
        if (w.lc >= o) f = q_compose(other, f);
      }
      if (vu[u] && w.lc == SEG - 1) d.qsum[tu[u] * p.n + iu[u]] = (uint8_t)(f | (seg_esc ? 8 : 0));
    }
  }
}

// k_quirk_sum with 32 cells per lane (tile widths >= 32): a lane loads its 4
// chunks' lag and age words at once (16 B each) and a tier chunk, which holds
// no candidate, contributes only whether a listed member is in it (summary
// 5, else the identity 0); only escaped chunks take the 8-cell rule. The
// 8-cell form ran 3.1 ms over the N = 65,536 table, VALU-heavy per 8 cells.
template <int TW>
__global__ __launch_bounds__(256) void k_quirk_sum32(GhDev d, int cur, int dcur, GhRound p) {
  if (p.qgate && d.cntg[p.n + 1] == 0) return;  // no candidate in any shard's table
  constexpr int SEGL = TW / 32;   // lanes per (tile, row) segment
  constexpr int RPWL = 64 / SEGL;  // segments per wave instruction
  constexpr int U = 2;
  const int lane = threadIdx.x & 63, sub = lane / SEGL, lc = lane % SEGL;
  const int64_t nrows = d.nrows, nseg = (p.ld / TW) * nrows;
  const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
  const int64_t gw = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  constexpr int64_t step = (int64_t)RPWL * U;
  // one contiguous run of segments per wave (SegWalk::run)
  const int64_t per = ((nseg + nw - 1) / nw + step - 1) / step * step;
  const int64_t run0 = gw * per, run1 = min(nseg, run0 + per);
  const bool small = nseg <= (int64_t)UINT32_MAX;
  const bool tier = gh_m8(d, cur);
  const unsigned long long smask = ((SEGL == 64) ? ~0ull : ((1ull << SEGL) - 1)) << (sub * SEGL);
  for (int64_t base = run0; base < run1; base += step) {
    int64_t tu[U];
    int iu[U];
    bool vu[U];
    v4u au[U], qu[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t sid = base + u * RPWL + sub;
      vu[u] = sid < run1;
      tu[u] = 0;
      iu[u] = (int)d.row0;
      if (vu[u]) {
        if (small) {
          const uint32_t q = (uint32_t)sid / (uint32_t)nrows;
          tu[u] = q;
          iu[u] = (int)(d.row0 + ((uint32_t)sid - q * (uint32_t)nrows));
        } else {
          tu[u] = sid / nrows;
          iu[u] = (int)(d.row0 + (sid - tu[u] * nrows));
        }
      }
      au[u] = qu[u] = v4u{0u, 0u, 0u, 0u};
      if (vu[u] && tier) {
        const int64_t wi = gh_cell(d, iu[u], tu[u] * TW + lc * 32) >> 3;  // (4-word aligned)
        au[u] = *reinterpret_cast<const v4u*>(d.a4[cur] + wi);
        qu[u] = *reinterpret_cast<const v4u*>(d.pl[cur] + wi);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) vu[u] = vu[u] && d.alive[iu[u]] && d.active[iu[u]];  // (as k_quirk_sum)
#pragma unroll
    for (int u = 0; u < U; ++u) {
      int f = 0;
      bool esc = false;
      if (vu[u]) {
        const int64_t c0 = tu[u] * TW + lc * 32;
        const uint32_t rmw = d.dbits[c0 >> 5];  // the lane's 32 columns' REMOVE bits
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int64_t c = c0 + 8 * k;
          const uint32_t rm8 = ((rmw >> (8 * k)) & 0xFFu) ? removed8(d, dcur, c, iu[u]) : 0u;
          int fk;
          if (tier && !gh_t4_esc(au[u][k])) {
            fk = (gh_t4_present8(qu[u][k]) & ~rm8) ? 5 : 0;  // listed members, no candidate
          } else {
            esc = true;
            const uint32_t pf = gh_pf8(d, cur, iu[u], c);
            const uint32_t P = pf & ~rm8 & 0xFFu;
            fk = q_summary8(P, (pf >> 8) & P);
          }
          f = q_compose(f, fk);
        }
      }
      const bool seg_esc = (__ballot(esc) & smask) != 0;
#pragma unroll
      for (int o = 1; o < SEGL; o <<= 1) {
        const int other = __shfl_up(f, o, SEGL);
        if (lc >= o) f = q_compose(other, f);
      }
      if (vu[u] && lc == SEGL - 1) d.qsum[tu[u] * p.n + iu[u]] = (uint8_t)(f | (seg_esc ? 8 : 0));
    }
  }
}

// one thread per row: exclusive prefix over the shard's tiles (in place),
// the shard's total and its last tile holding a present cell
__global__ __launch_bounds__(256) void k_quirk_prefix(GhDev d, GhRound p) {
  if (p.qgate && d.cntg[p.n + 1] == 0) return;  // no candidate in any shard's table
  const int i = (int)d.row0 + blockIdx.x * blockDim.x + threadIdx.x;
  if (!gh_owned(d, i)) return;
  const int64_t ntiles = p.ld / d.tw;
  int pre = 0, last = -1;
  for (int64_t t = 0; t < ntiles; ++t) {
    const int f = d.qsum[t * p.n + i];
    d.qsum[t * p.n + i] = (uint8_t)(pre | (f & 8));  // (bit 3 kept: the segment may hold flags)
    if (f & 4) last = (int)t;
    pre = q_compose(pre, f & 7);
  }
  d.qall[(int64_t)d.rank * p.n + i] = (uint8_t)pre;
  d.qlast[i] = last;
}

// one thread per row: the run state entering this shard (the shards before
// it, in member order) and whether the row's last list entry is here
__global__ __launch_bounds__(256) void k_quirk_carry(GhDev d, GhRound p) {
  const int i = (int)d.row0 + blockIdx.x * blockDim.x + threadIdx.x;
  if (!gh_owned(d, i)) return;
  int s = 0;
  bool later = false;
  // row layout: the whole row is here, nothing enters from other shards
  for (int g = 0; g < (d.rowlay ? 0 : d.world); ++g) {
    const int f = d.qall[(int64_t)g * p.n + i];
    if (g < d.rank) s = q_apply(f, s);
    if (g > d.rank && (f & 4)) later = true;
  }
  const bool mine_last = !later && (d.qall[(int64_t)d.rank * p.n + i] & 4);
  d.qcarry[i] = (uint8_t)(s | (mine_last ? 2 : 0));
}

// one segment per (tile, row) of an active row: each lane gets the run state
// before its 4 cells (exclusive segmented scan + the tile's carry-in) and
// clears the flag of every candidate the reference's loop skips
template <int TW>
__global__ __launch_bounds__(256) void k_quirk_apply(GhDev d, int cur, int dcur, GhRound p) {
  if (p.qgate && d.cntg[p.n + 1] == 0) return;  // no candidate in any shard's table
  // (gh_clearflags8 rewrites the plane words of the chunks it changes)
  constexpr int SEG = SegWalk<TW>::SEG;
  constexpr int U = 4;  // segment steps per iteration, loads issued together (as k_quirk_sum)
  const SegWalk<TW> w(d, p);
  const bool tier = gh_m8(d, cur);
  int64_t run0, run1;
  w.run(U, run0, run1);
  for (int64_t base = run0; base < run1; base += U * w.RPW) {
    int64_t tu[U];
    int iu[U], qsu[U];
    bool inu[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t sid = base + u * w.RPW + w.sub;
      inu[u] = sid < run1;
      tu[u] = 0;
      iu[u] = (int)w.row0;
      if (inu[u]) w.at(sid, tu[u], iu[u]);
      qsu[u] = inu[u] ? d.qsum[tu[u] * p.n + iu[u]] : 0;
    }
    // a segment with no escaped chunk holds no flag: nothing to clear (the
    // run state entering later segments is in the prefix already)
    uint32_t au[U], qu[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      au[u] = qu[u] = 0u;
      if ((qsu[u] & 8) && tier) {
        const int64_t wi = gh_cell(d, iu[u], tu[u] * TW + w.lc * 8) >> 3;
        au[u] = d.a4[cur][wi];
        qu[u] = d.pl[cur][wi];
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int qs = qsu[u];
      if (__ballot((qs & 8) != 0) == 0) continue;
      const int64_t t = tu[u];
      const int i = iu[u];
      const int64_t c = t * TW + w.lc * 8;
      const bool valid = inu[u] && (qs & 8) && d.alive[i] && d.active[i];  // only active rows detect (and send)
      uint32_t pf = 0u, rm = 0u;
      if (valid) {
        if (tier && !gh_t4_esc(au[u])) {  // a tier chunk: no flag
          pf = gh_t4_present8(qu[u]);
        } else {
          pf = gh_pf8(d, cur, i, c);
        }
        rm = removed8(d, dcur, c, i);
      }
      const int qc = d.qcarry[i];
      const int ql = d.qlast[i];
      const uint32_t P = pf & ~rm & 0xFFu, F = (pf >> 8) & P;  // list members, candidates
      const int f = q_summary8(P, F);
      int lastj = P ? w.lc * 8 + 31 - __builtin_clz(P) : -1;
      int incl = f;
#pragma unroll
      for (int o = 1; o < SEG; o <<= 1) {
        const int other = __shfl_up(incl, o, SEG);
        if (w.lc >= o) incl = q_compose(other, incl);
      }
      int excl = __shfl_up(incl, 1, SEG);
      if (w.lc == 0) excl = 0;
#pragma unroll
      for (int o = SEG / 2; o > 0; o >>= 1) lastj = max(lastj, __shfl_xor(lastj, o));
      if (!valid) continue;
      int st = q_apply(excl, q_apply(qs, qc & 1));
      const int lastc = ((qc & 2) && ql == t) ? lastj : -1;  // the row's last list entry, if here
      uint32_t clear = 0;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        if (!((P >> j) & 1u)) continue;
        if (!((F >> j) & 1u)) {
          st = 0;
          continue;
        }
        if (!(st == 0 || w.lc * 8 + j == lastc)) clear |= 1u << j;  // skipped this round
        st ^= 1;
      }
      if (clear) gh_clearflags8(d, cur, i, c, clear);
    }
  }
}

// The run state of 32 consecutive cells with list members P and candidates
// F (F within P), in q_summary8's closed form.
__device__ __forceinline__ int q_summary32(uint32_t P, uint32_t F) {
  if (!P) return 0;
  const uint32_t B = P & ~F;
  if (B) return 5 | ((__builtin_popcount((F >> (31 - __builtin_clz(B))) >> 1) & 1) << 1);
  return 4 | ((__builtin_popcount(F) & 1) << 1);
}

// List members and candidates of row i's 32 cells c0..c0+31 (c0 % 32 == 0,
// one tile segment: TW >= 32) after step 1's REMOVE, from the chunks' age
// and lag words au, qu (tier) and the columns' REMOVE and one-detector bits
// rmw, smw. Only an escaped chunk can hold a flag: the escaped chunks' 16-bit
// cells are loaded together before any is decoded (one load latency per
// window, not four).
__device__ __forceinline__ void quirk_lane32(const GhDev& d, int cur, int dcur, int i, int64_t c0, bool tier, bool in,
                                             const v4u& au, const v4u& qu, uint32_t rmw, uint32_t smw, uint32_t& P,
                                             uint32_t& F) {
  P = F = 0u;
  if (!in) return;
  uint4 hx[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    hx[k] = uint4{0u, 0u, 0u, 0u};
    if (!tier || gh_t4_esc(au[k])) hx[k] = gh_ld16(d, cur, i, c0 + 8 * k);
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int64_t c = c0 + 8 * k;
    // removed8 from the preloaded words: a one-detector column spares its detector's row
    const uint32_t m = (rmw >> (8 * k)) & 0xFFu;
    uint32_t sm = (smw >> (8 * k)) & m, rm8 = m & ~sm;
    if (d.rlist) {
      rm8 = m ? removed8(d, dcur, c, i) : 0u;
      sm = 0u;
    }
    while (sm) {
      const int j = __builtin_ctz(sm);
      sm &= sm - 1u;
      if (d.det_min[dcur][c + j] != i) rm8 |= 1u << j;
    }
    uint32_t pk, fk = 0u;
    if (tier && !gh_t4_esc(au[k])) {
      pk = gh_t4_present8(qu[k]) & ~rm8;  // a tier chunk: no candidate
    } else {
      const uint32_t pf = gh_pf8x(d, cur, i, c, hx[k]);
      pk = pf & ~rm8 & 0xFFu;
      fk = (pf >> 8) & pk;
    }
    P |= pk << (8 * k);
    F |= fk << (8 * k);
  }
}
__device__ __forceinline__ void quirk_load32(const GhDev& d, int cur, int i, int64_t c0, bool tier, bool in, v4u& au,
                                             v4u& qu, uint32_t& rmw, uint32_t& smw) {
  au = qu = v4u{0u, 0u, 0u, 0u};
  rmw = smw = 0u;
  if (!in) return;
  if (tier) {
    const int64_t wi = gh_cell(d, i, c0) >> 3;  // (4-word aligned)
    au = *reinterpret_cast<const v4u*>(d.a4[cur] + wi);
    qu = *reinterpret_cast<const v4u*>(d.pl[cur] + wi);
  }
  rmw = d.dbits[c0 >> 5];
  smw = d.sbits[c0 >> 5];
}

// Quirk-mode detection in one pass when every row is whole on this engine
// (one engine, or row shards), tile widths >= 32: one wave per row walks it
// in member order, 2,048 cells (64 lanes x 32) per window and QW windows'
// loads per step, the run state carried from window to window (a wave scan
// of the lanes' summaries), and clears the flag of every candidate at an
// odd run offset that is not the row's last list entry (found first, from
// the row's end). The same flags as k_quirk_sum + k_quirk_prefix +
// k_quirk_apply, which sweep the table twice (slave/slave.go:464-477 with
// :283; SPEC §4).
template <int TW>
__global__ __launch_bounds__(256) void k_quirk_rows(GhDev d, int cur, int dcur, GhRound p) {
  if (p.qgate && d.cntg[p.n + 1] == 0) return;  // no candidate in the table
  constexpr int QW = 4;
  const int lane = threadIdx.x & 63;
  const int64_t nwv = ((int64_t)gridDim.x * blockDim.x) >> 6;
  const bool tier = gh_m8(d, cur);
  const int64_t nwin = (p.ld + 2047) / 2048;
  for (int64_t r = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; r < d.nrows; r += nwv) {
    const int i = (int)(d.row0 + r);
    if (!(d.alive[i] && d.active[i])) continue;  // only active rows detect (and send)
    // the row's last list entry (usually in the last window)
    int64_t lastc = -1;
    for (int64_t w = nwin - 1; w >= 0 && lastc < 0; --w) {
      const int64_t c0 = w * 2048 + lane * 32;
      v4u au, qu;
      uint32_t rmw, smw, P, F;
      quirk_load32(d, cur, i, c0, tier, c0 < p.ld, au, qu, rmw, smw);
      quirk_lane32(d, cur, dcur, i, c0, tier, c0 < p.ld, au, qu, rmw, smw, P, F);
      const unsigned long long b = __ballot(P != 0u);
      if (b) {
        const int hl = 63 - __builtin_clzll(b);
        const int hp = __shfl(P ? 31 - __builtin_clz(P) : 0, hl);
        lastc = w * 2048 + hl * 32 + hp;
      }
    }
    if (lastc < 0) continue;  // an empty list: no candidate
    const int64_t wend = lastc / 2048 + 1;  // windows up to the last entry's
    int carry = 0;                          // run state entering the window
    for (int64_t w0 = 0; w0 < wend; w0 += QW) {
      v4u au[QW], qu[QW];
      uint32_t rmw[QW], smw[QW], P[QW], F[QW];
#pragma unroll
      for (int u = 0; u < QW; ++u) {
        const int64_t c0 = (w0 + u) * 2048 + lane * 32;
        quirk_load32(d, cur, i, c0, tier, w0 + u < wend && c0 < p.ld, au[u], qu[u], rmw[u], smw[u]);
      }
#pragma unroll
      for (int u = 0; u < QW; ++u) {
        const int64_t c0 = (w0 + u) * 2048 + lane * 32;
        quirk_lane32(d, cur, dcur, i, c0, tier, w0 + u < wend && c0 < p.ld, au[u], qu[u], rmw[u], smw[u], P[u], F[u]);
      }
#pragma unroll
      for (int u = 0; u < QW; ++u) {
        int incl = q_summary32(P[u], F[u]);
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
          const int other = __shfl_up(incl, o);
          if (lane >= o) incl = q_compose(other, incl);
        }
        int excl = __shfl_up(incl, 1);
        if (lane == 0) excl = 0;
        int st = q_apply(excl, carry);
        carry = q_apply(__shfl(incl, 63), carry);
        if (!F[u]) continue;
        const int64_t c0 = (w0 + u) * 2048 + lane * 32;
        uint32_t clear = 0u;
        for (int j = 0; j < 32; ++j) {
          if (!((P[u] >> j) & 1u)) continue;
          if (!((F[u] >> j) & 1u)) {
            st = 0;
            continue;
          }
          if (st != 0 && c0 + j != lastc) clear |= 1u << j;  // skipped this round
          st ^= 1;
        }
#pragma unroll
        for (int k = 0; k < 4; ++k)
          if ((clear >> (8 * k)) & 0xFFu) gh_clearflags8(d, cur, i, c0 + 8 * k, (clear >> (8 * k)) & 0xFFu);
      }
    }
  }
}

}  // namespace

// d.tw -> template tile width
#define GH_TW_DISPATCH(F, ...)                  \
  switch (d.tw) {                              \
    case 8: F<8>(__VA_ARGS__); break;          \
    case 16: F<16>(__VA_ARGS__); break;        \
    case 32: F<32>(__VA_ARGS__); break;        \
    case 128: F<128>(__VA_ARGS__); break;      \
    case 256: F<256>(__VA_ARGS__); break;      \
    default: F<64>(__VA_ARGS__); break;        \
  }

static unsigned seg_grid(const GhRound& p, int tw) {
  const int64_t waves = ((p.ld / tw) * p.n + (64 / (tw / 8)) - 1) / (64 / (tw / 8));
  return (unsigned)std::max<int64_t>(1, std::min<int64_t>((waves + 3) / 4, 16384));
}

template <int TW>
static void quirk_sum(const GhDev& d, int cur, int dcur, const GhRound& p, hipStream_t s) {
  if constexpr (TW >= 32)
    hipLaunchKernelGGL(k_quirk_sum32<TW>, dim3(seg_grid(p, TW)), dim3(256), 0, s, d, cur, dcur, p);
  else
    hipLaunchKernelGGL(k_quirk_sum<TW>, dim3(seg_grid(p, TW)), dim3(256), 0, s, d, cur, dcur, p);
}
template <int TW>
static void quirk_rows(const GhDev& d, int cur, int dcur, const GhRound& p, hipStream_t s) {
  if constexpr (TW >= 32) {
    const unsigned g = (unsigned)std::max<int64_t>(1, std::min<int64_t>((d.nrows + 3) / 4, 16384));
    hipLaunchKernelGGL(k_quirk_rows<TW>, dim3(g), dim3(256), 0, s, d, cur, dcur, p);
  }
}
template <int TW>
static void quirk_apply(const GhDev& d, int cur, int dcur, const GhRound& p, hipStream_t s) {
  hipLaunchKernelGGL(k_quirk_apply<TW>, dim3(seg_grid(p, TW)), dim3(256), 0, s, d, cur, dcur, p);
}
template <int TW>
static void ring_tiles(const GhDev& d, int cur, int dcur, const GhRound& p, hipStream_t s) {
  hipLaunchKernelGGL(k_ring_tiles<TW>, dim3(seg_grid(p, TW)), dim3(256), 0, s, d, cur, dcur, p);
}

void launch_quirk_scan(const GhDev& d, int cur, int dcur, const GhRound& p, hipStream_t s) {
  GH_TW_DISPATCH(quirk_sum, d, cur, dcur, p, s)
  hipLaunchKernelGGL(k_quirk_prefix, dim3((p.n + 255) / 256), dim3(256), 0, s, d, p);
}

void launch_quirk_rows(const GhDev& d, int cur, int dcur, const GhRound& p, hipStream_t s) {
  GH_TW_DISPATCH(quirk_rows, d, cur, dcur, p, s)
}

void launch_quirk_apply(const GhDev& d, int cur, int dcur, const GhRound& p, hipStream_t s) {
  hipLaunchKernelGGL(k_quirk_carry, dim3((p.n + 255) / 256), dim3(256), 0, s, d, p);
  GH_TW_DISPATCH(quirk_apply, d, cur, dcur, p, s)
}

// k_active_exact idles in all but failure storms: a grid-stride loop over
// rows on a small grid keeps its idle dispatch short
static unsigned exact_grid(const GhRound& p) { return (unsigned)std::min<int64_t>(1024, ((int64_t)p.n + 3) / 4); }
void launch_active_pre(const GhDev& d, int cur, int dcur, const GhRound& p, hipStream_t s) {
  hipLaunchKernelGGL(k_active_pre, dim3((p.n + 255) / 256), dim3(256), 0, s, d, cur, dcur, p);
  hipLaunchKernelGGL(k_active_exact, dim3(exact_grid(p)), dim3(256), 0, s, d, cur, dcur, p, 0);
}
void launch_prologue(const GhDev& d, int cur, int dcur, const GhRound& p, hipStream_t s) {
  const int64_t nt = std::max<int64_t>(p.ld, p.n);
  hipLaunchKernelGGL(k_prologue, dim3((unsigned)((nt + 255) / 256)), dim3(256), 0, s, d, cur, dcur, p);
  hipLaunchKernelGGL(k_active_exact, dim3(exact_grid(p)), dim3(256), 0, s, d, cur, dcur, p, 1);
}

void launch_active_post(const GhDev& d, const GhRound& p, hipStream_t s) {
  hipLaunchKernelGGL(k_active_post, dim3((p.n + 255) / 256), dim3(256), 0, s, d, p);
}

void launch_peers_pull(const GhDev& d, int cur, int dcur, const GhRound& p, hipStream_t s) {
  hipLaunchKernelGGL(k_peers_pull, dim3((unsigned)(((int64_t)d.ncs * 8 + 255) / 256)), dim3(256), 0, s, d, cur, dcur, p);
}

void launch_peers_rows(const GhDev& d, int cur, int dcur, const GhRound& p, hipStream_t s) {
  hipLaunchKernelGGL(k_peers_rows, dim3((p.n + 255) / 256), dim3(256), 0, s, d, cur, dcur, p);
}

void launch_inbox_bits(const GhDev& d, const GhRound& p, hipStream_t s) {
  hipLaunchKernelGGL(k_inbox_bits, dim3((p.n + 255) / 256), dim3(256), 0, s, d, p);
}

void launch_inbox_rows(const GhDev& d, const GhRound& p, hipStream_t s) {
  hipLaunchKernelGGL(k_inbox_rows, dim3((p.n + 255) / 256), dim3(256), 0, s, d, p);
}

void launch_negate(int32_t* x, int64_t n, hipStream_t s) {
  if (n > 0) hipLaunchKernelGGL(k_negate, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, x, n);
}

void launch_ring_count(const GhDev& d, int cur, int dcur, const GhRound& p, hipStream_t s) {
  if (p.ring_whole) hipLaunchKernelGGL(k_ring_fast, dim3((p.n + 3) / 4), dim3(256), 0, s, d, cur, p);
  GH_TW_DISPATCH(ring_tiles, d, cur, dcur, p, s)
  hipLaunchKernelGGL(k_ring_count, dim3((p.n + 255) / 256), dim3(256), 0, s, d, cur, dcur, p);
}

void launch_ring_select(const GhDev& d, int cur, int dcur, const GhRound& p, hipStream_t s) {
  hipLaunchKernelGGL(k_ring_select, dim3((p.n + 255) / 256), dim3(256), 0, s, d, cur, dcur, p);
}

void launch_inbox(const GhDev& d, const GhRound& p, hipStream_t s) {
  (void)hipMemsetAsync(d.inbox_cnt, 0, sizeof(int32_t) * p.n, s);
  hipLaunchKernelGGL(k_inbox_count, dim3((p.n + 255) / 256), dim3(256), 0, s, d, p);
  hipLaunchKernelGGL(k_inbox_scan, dim3(1), dim3(1024), 0, s, d, p);
  hipLaunchKernelGGL(k_inbox_fill, dim3((p.n + 255) / 256), dim3(256), 0, s, d, p);
}

// the full-grid REMOVE launch as IN 7 (GH_RMV_FULL7=0 at run time: IN 6, A/B)
static bool rmv_full7() {
  static const bool on = [] {
    const char* v = std::getenv("GH_RMV_FULL7");
    return GH_RMV_FULL7 && (!v || std::atoi(v) != 0);
  }();
  return on;
}

// variant: 0 lean on a 16-bit input, 1 storm, 2 lean on a 4-bit-tier input
// by the 16-bit rule, 3 the nibble path (IN 2, or IN 4 on row shards), 4 the
// nibble path that takes REMOVE deliveries (IN 6, column layout)
template <int KB, int TW, int TPW>
static bool launch_round_tpw(const GhDev& d, int cur, int dcur, const GhRound& p, hipStream_t s, bool nt, int variant,
                             hipEvent_t t0, hipEvent_t t1) {
  constexpr int RB = round_rb<TW>();
  const int64_t nrb = (d.nrows + RB - 1) / RB;
  const int64_t nblk = nrb * (p.ld / TW / TPW);
  if (nblk == 0) return false;
  const bool tiered = d.a4[0] != nullptr;
  const bool few = variant == 1 || variant == 2 || (variant == 0 && tiered);
  // (a resident-sized grid for the persistent variants, 1,280 workgroups for
  // the storm one, measured slower: storm 5.3 -> 6.0 ms). The REMOVE-taking
  // nibble path (variant 4): a full grid when the host knows a REMOVE is
  // pending (p.rmv_full), else a 1/8 grid whose workgroups loop over their
  // blocks (idle in most rounds: a full grid cost 31 us of dispatch; active,
  // 1/8 grid 3.4-3.7 ms against 2.7-3.2 ms full, a resident-sized one 3.5-4.1)
  const bool few4 = variant == 4 && tiered && !p.rmv_full;
  const dim3 grid((unsigned)((few || few4) ? std::max<int64_t>(8, (nblk / 8 + 7) / 8 * 8) : nblk)), blk(256);
#define GH_ROUND_LAUNCH(NT, ST, IN) \
  hipExtLaunchKernelGGL((k_round<KB, TW, TPW, NT, ST, IN>), grid, blk, 0, s, t0, t1, 0, d, cur, dcur, p)
#define GH_ROUND_NT(ST, IN)        \
  do {                             \
    if (nt)                        \
      GH_ROUND_LAUNCH(true, ST, IN);  \
    else                           \
      GH_ROUND_LAUNCH(false, ST, IN); \
  } while (0)
  if constexpr (KB == 4 && TPW == 1 && TW >= 64) {  // a tiered engine (host: c8)
    if (tiered) {
      switch (variant) {
        case 0: GH_ROUND_NT(false, 3); return true;
        case 2: GH_ROUND_NT(false, 1); return true;
        case 3:
          if (d.rowlay)
            GH_ROUND_NT(false, 4);  // row layout: ghost senders
          else if (p.nib_dma && TW == 256)
            GH_ROUND_NT(false, 5);  // LDS-DMA staging
          else
            GH_ROUND_NT(false, 2);
          return true;
        case 4:  // the nibble path that takes REMOVE deliveries (column layout; returns at once otherwise)
          if (d.rowlay) return false;
          if (p.rmv_full && rmv_full7())
            GH_ROUND_NT(false, 7);
          else
            GH_ROUND_NT(false, 6);
          return true;
        default: break;
      }
    }
  }
  if (variant == 1)
    GH_ROUND_NT(true, 0);
  else if (variant == 0)
    GH_ROUND_NT(false, 0);
  else
    return false;
  return true;
#undef GH_ROUND_NT
#undef GH_ROUND_LAUNCH
}

template <int TW>
static void round_slow(const GhDev& d, int cur, int dcur, const GhRound& p, hipStream_t s) {
  // one resident generation (150 VGPRs: 3 waves per SIMD, 768 workgroups
  // on 256 CUs); the segments are dealt out by a grid-stride loop, and an
  // idle launch (most rounds) dispatches less (GH_SLOW_GRID: A/B)
  static const unsigned g = [] {
    const char* v = std::getenv("GH_SLOW_GRID");
    return v ? (unsigned)std::max(1, std::atoi(v)) : 768u;
  }();
  hipLaunchKernelGGL((k_round_slow<TW>), dim3(g), dim3(256), 0, s, d, cur, dcur, p);
}


// tiles per workgroup: ld / TW is a multiple of 8 (host padding)
template <int KB, int TW>
static bool launch_round_tw(const GhDev& d, int cur, int dcur, const GhRound& p, hipStream_t s, bool nt, int storm,
                            hipEvent_t t0, hipEvent_t t1) {
  switch (p.tpw) {
    case 1: return launch_round_tpw<KB, TW, 1>(d, cur, dcur, p, s, nt, storm, t0, t1);
    case 2: return launch_round_tpw<KB, TW, 2>(d, cur, dcur, p, s, nt, storm, t0, t1);
    case 8: return launch_round_tpw<KB, TW, 8>(d, cur, dcur, p, s, nt, storm, t0, t1);
    default: return launch_round_tpw<KB, TW, 4>(d, cur, dcur, p, s, nt, storm, t0, t1);
  }
}

template <int KB>
static bool launch_round_kb(const GhDev& d, int cur, int dcur, const GhRound& p, hipStream_t s, bool nt, int storm,
                            hipEvent_t t0, hipEvent_t t1) {
  switch (d.tw) {
    case 8: return launch_round_tw<KB, 8>(d, cur, dcur, p, s, nt, storm, t0, t1);
    case 16: return launch_round_tw<KB, 16>(d, cur, dcur, p, s, nt, storm, t0, t1);
    case 32: return launch_round_tw<KB, 32>(d, cur, dcur, p, s, nt, storm, t0, t1);
    case 128: return launch_round_tw<KB, 128>(d, cur, dcur, p, s, nt, storm, t0, t1);
    case 256: return launch_round_tw<KB, 256>(d, cur, dcur, p, s, nt, storm, t0, t1);
    default: return launch_round_tw<KB, 64>(d, cur, dcur, p, s, nt, storm, t0, t1);
  }
}

bool launch_round(const GhDev& d, int cur, int dcur, const GhRound& p, hipStream_t s, bool nt, int storm, hipEvent_t t0,
                  hipEvent_t t1) {
  if (p.peer_mode == GH_PEER_PULL && p.k <= 4)
    return launch_round_kb<4>(d, cur, dcur, p, s, nt, storm, t0, t1);
  return launch_round_kb<8>(d, cur, dcur, p, s, nt, storm, t0, t1);
}

void launch_base(const GhDev& d, int cur, int dcur, const GhRound& p, hipStream_t s) {
  hipLaunchKernelGGL(k_base, dim3((unsigned)((p.ld + 255) / 256)), dim3(256), 0, s, d, cur, dcur, p);
}

void launch_finish(const GhDev& d, int dcur, const GhRound& p, hipStream_t s) {
  hipLaunchKernelGGL(k_finish, dim3((unsigned)((p.ld + 255) / 256)), dim3(256), 0, s, d, dcur, p);
}

// the lane jobs dealt one per lane (GH_JOBS_FLAT=0 at run time: one region
// at a time, A/B)
static bool jobs_flat() {
  static const bool on = [] {
    const char* v = std::getenv("GH_JOBS_FLAT");
    return !v || std::atoi(v) != 0;
  }();
  return on;
}
template <int TW>
static void round_jobs(const GhDev& d, int cur, int dcur, const GhRound& p, hipStream_t s) {
  if constexpr (TW >= 64) {
    const unsigned g = (unsigned)std::min<int64_t>(2048, std::max<int64_t>(1, d.jobw));
    if (jobs_flat())
      hipLaunchKernelGGL((k_round_jobs_flat<TW, GH_JOB_CPL>), dim3(std::min<unsigned>(g, 1024)), dim3(256), 0, s, d,
                         cur, dcur, p);
    else
      hipLaunchKernelGGL((k_round_jobs<TW, GH_JOB_CPL>), dim3(g), dim3(256), 0, s, d, cur, dcur, p);
    hipLaunchKernelGGL((k_round_redo<TW>), dim3(1), dim3(64), 0, s, d, cur, dcur, p);
  }
}
void launch_round_jobs(const GhDev& d, int cur, int dcur, const GhRound& p, hipStream_t s) {
  if (!d.jobs) return;
  GH_TW_DISPATCH(round_jobs, d, cur, dcur, p, s)
}

void launch_round_slow(const GhDev& d, int cur, int dcur, const GhRound& p, hipStream_t s) {
  GH_TW_DISPATCH(round_slow, d, cur, dcur, p, s)
}
