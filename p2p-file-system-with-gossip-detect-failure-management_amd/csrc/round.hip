// Gossip-round kernels for gfx950 (SPEC.md §2-§3, DESIGN.md "Kernels").
//
//   k_prep / k_active_pre / k_active_exact / k_active_post
//                  per row: the <4 guard after REMOVE delivery
//                  (slave/slave.go:504,511). Rows decided by the global count
//                  need nothing else; the few undecided rows get an exact
//                  post-REMOVE count (summed over ranks when sharded).
//   k_peers_pull   per receiver column: k Philox peers, kept iff the sender is
//                  active, alive and lists the receiver (slave/slave.go:527-542).
//   k_ring_*       reference ring topology (slave/slave.go:512-524): per-(tile,row)
//                  snapshot counts, positions, targets + inbox CSR.
//   k_quirk_*      quirk-mode detection pre-pass (SPEC §4).
//   k_round        THE HOT KERNEL: one pass over the table applying REMOVE
//                  delivery, guard, own heartbeat, detection, cleanup and the
//                  k-peer max-merge (slave/slave.go:276-286,414-497) for a
//                  64-row x TW-member tile per workgroup.
//   k_finish       per row/column: reduce the pass's partial counts, build
//                  the failed-set bitmap D_r for the next round.
// Member columns are local to the engine's shard (gh_internal.h); rows,
// alive/active and the inboxes are global.
#include <limits.h>

#include <algorithm>

#include "gh_internal.h"

namespace {

__device__ __forceinline__ int uni(int x) { return __builtin_amdgcn_readfirstlane(x); }

__device__ __forceinline__ bool dbit(const uint32_t* bits, int64_t c) {
  return (bits[c >> 5] >> (c & 31)) & 1u;
}

// Step 1 applies REMOVE(c) at row j unless j is c's only detector
// (slave/slave.go:344-346: a detector does not message itself).
__device__ __forceinline__ bool removes_at(int dc, int dm, int j) { return !(dc == 1 && dm == j); }

// |D_{r-1}| of this shard next to the local counts, for one allreduce.
__global__ void k_prep(GhDev d, int dcur) { d.cntl[d.n] = d.nd[dcur]; }

// Decides rows from the global count cntg and global |D| = cntg[n]; an
// undecided row (|D| could push it under the threshold) gets its exact local
// post-REMOVE count in post[] (und = 1), or is left to k_active_exact's full
// recount in failure storms (und = 2).
__global__ __launch_bounds__(256) void k_active_pre(GhDev d, int cur, int dcur, GhRound p) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    d.nd[dcur ^ 1] = 0;
    d.nd[2 + (dcur ^ 1)] = 0;
  }
  if (i >= p.n) return;
  d.det_any[i] = 0;
  bool a = false;
  uint8_t u = 0;
  int32_t post = 0;
  if (d.alive[i]) {
    const int c = d.cntg[i];
    const int ndg = d.cntg[p.n];
    if (c < p.min_members) {
      a = false;
    } else if (c - ndg >= p.min_members) {
      a = true;
    } else if (d.nd[dcur] > GH_DLIST_MAX) {
      u = 2;
    } else {
      u = 1;
      const int32_t* hb = d.hb[cur];
      const int32_t* dc = d.det_cnt[dcur];
      const int32_t* dm = d.det_min[dcur];
      int rem = 0;
      const int nd = d.nd[dcur];
      for (int q = 0; q < nd; ++q) {
        const int col = d.dlist[(int64_t)dcur * p.ld + q];
        rem += (hb[gh_cell(d, i, col)] >= 0) && removes_at(dc[col], dm[col], i);
      }
      post = d.cntl[i] - rem;
    }
  }
  d.active[i] = a;
  d.und[i] = u;
  d.post[i] = post;
}

// Failure storms (local |D| > GH_DLIST_MAX): one wave recounts each
// undecided row over the local columns with REMOVE applied.
__global__ __launch_bounds__(256) void k_active_exact(GhDev d, int cur, int dcur, GhRound p) {
  if (d.nd[dcur] <= GH_DLIST_MAX) return;
  const int i = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (i >= p.n || d.und[i] != 2) return;
  const int32_t* hb = d.hb[cur];
  const int32_t* dc = d.det_cnt[dcur];
  const int32_t* dm = d.det_min[dcur];
  int cnt = 0;
  for (int64_t c = lane * 4; c < p.ld; c += 256) {
    const int4 v = *reinterpret_cast<const int4*>(hb + gh_cell(d, i, c));
    const uint32_t b4 = (d.dbits[c >> 5] >> (c & 31)) & 0xFu;
    const int x[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int j = 0; j < 4; ++j)
      cnt += x[j] >= 0 && !(((b4 >> j) & 1u) && removes_at(dc[c + j], dm[c + j], i));
  }
  for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o);
  if (lane == 0) d.post[i] = cnt;
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
  }
  const unsigned long long m = __ballot(a);
  if (d.rank == 0 && (threadIdx.x & 63) == 0 && m)
    atomicAdd(&d.stats[ST_ACTIVE_ROWS], (unsigned long long)__popcll(m));
}

// Receivers are this shard's member columns (their column holds the senders'
// view of them); the inbox rows of the other shards arrive by allgather.
__global__ __launch_bounds__(256) void k_peers_pull(GhDev d, int cur, int dcur, GhRound p) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= d.ncs) return;
  const int64_t i = d.col0 + t;  // global receiver (>= n in the tail of the last shard)
  const int64_t beg = i * p.k;
  int nv = 0;
  if (t < d.ncol && d.alive[i] && p.n >= 2) {
    const bool ib = dbit(d.dbits, t);
    const int dci = ib ? d.det_cnt[dcur][t] : 0;
    const int dmi = ib ? d.det_min[dcur][t] : 0;
    for (int q = 0; q < p.k; ++q) {
      const uint32_t u = gh_philox_word(p.seed, (uint32_t)i, (uint32_t)p.r, GH_TAG_PEER,
                                        (uint32_t)(q >> 2), q & 3);
      const uint32_t w = (uint32_t)(((uint64_t)u * (uint64_t)(p.n - 1)) >> 32);
      const int s = (int)w + ((int64_t)w >= i);
      if (!d.alive[s] || !d.active[s]) continue;
      const int64_t off = gh_cell(d, s, t);
      const int32_t v = d.hb[cur][off];
      // i must be in s's snapshot list: present, not detected by s this
      // round and not REMOVE'd at s in step 1.
      if (v < 0 || (v & GH_FLAG)) continue;
      if (ib && removes_at(dci, dmi, s)) continue;
      d.inbox[beg + nv++] = s;
    }
  }
  d.inbox_cnt[i] = nv;
}

// ---- segment walks -------------------------------------------------------
// The helper kernels below read the table the way k_round does: a lane owns
// 4 consecutive members, SEG = TW/4 lanes cover one row segment of a tile,
// and consecutive waves take consecutive (tile, row) segments in storage
// order, so every wave instruction is one contiguous 1 KiB access.
typedef int v4i __attribute__((ext_vector_type(4)));

template <int TW>
struct SegWalk {
  static constexpr int SEG = TW / 4;
  static constexpr int RPW = 64 / SEG;
  int lane, sub, lc;
  int64_t nseg, first, stride;
  __device__ SegWalk(const GhRound& p) {
    lane = threadIdx.x & 63;
    sub = lane / SEG;
    lc = lane % SEG;
    nseg = (p.ld / TW) * p.n;
    first = (((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6) * RPW;
    stride = (((int64_t)gridDim.x * blockDim.x) >> 6) * RPW;
  }
};

// 4-bit REMOVE mask of local columns l0..l0+3 at row i
__device__ __forceinline__ uint32_t removed4(const GhDev& d, int dcur, int64_t l0, int i) {
  uint32_t m = (d.dbits[l0 >> 5] >> (l0 & 31)) & 0xFu;
  uint32_t out = 0;
  for (int j = 0; j < 4; ++j)
    if (((m >> j) & 1u) && removes_at(d.det_cnt[dcur][l0 + j], d.det_min[dcur][l0 + j], i)) out |= 1u << j;
  return out;
}

// Ring mode, part 1: per (tile, sender row) the number of members in the
// sender's snapshot list (present after REMOVE, not detected by it).
template <int TW>
__global__ __launch_bounds__(256) void k_ring_tiles(GhDev d, int cur, int dcur, GhRound p) {
  const SegWalk<TW> w(p);
  for (int64_t base = w.first; base < w.nseg; base += w.stride) {
    const int64_t sid = base + w.sub;
    const bool valid = sid < w.nseg;
    const int64_t t = valid ? sid / p.n : 0;
    const int i = valid ? (int)(sid - t * p.n) : 0;
    const int64_t l0 = t * TW + w.lc * 4;
    int cnt = 0;
    if (valid) {
      const v4i v = *reinterpret_cast<const v4i*>(d.hb[cur] + t * d.tstride + (int64_t)i * TW + w.lc * 4);
      const uint32_t rm = removed4(d, dcur, l0, i);
#pragma unroll
      for (int j = 0; j < 4; ++j) cnt += v[j] >= 0 && !(v[j] & GH_FLAG) && !((rm >> j) & 1u);
    }
#pragma unroll
    for (int o = SegWalk<TW>::SEG / 2; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o);
    if (valid && w.lc == 0) d.rcnt[sid] = (uint16_t)cnt;
  }
}

// The local column of the want-th (0-based) member of sender s's snapshot
// list inside tile t (scans the tile-row).
__device__ __forceinline__ int64_t ring_find(const GhDev& d, const int32_t* hb, int dcur, int s, int64_t t, int want) {
  for (int j = 0; j < d.tw; ++j) {
    const int64_t c = t * d.tw + j;
    const int32_t v = hb[gh_cell(d, s, c)];
    if (v < 0 || (v & GH_FLAG)) continue;
    if (dbit(d.dbits, c) && removes_at(d.det_cnt[dcur][c], d.det_min[dcur][c], s)) continue;
    if (want-- == 0) return c;
  }
  return -1;
}

// Ring mode, part 2 (one thread per sender row): this shard's list length
// and, when the sender's own column is local, its position in that list.
__global__ __launch_bounds__(256) void k_ring_count(GhDev d, int cur, int dcur, GhRound p) {
  const int sdr = blockIdx.x * blockDim.x + threadIdx.x;
  if (sdr >= p.n) return;
  int32_t* out = d.ring + ((int64_t)d.rank * p.n + sdr) * 2;
  if (!(d.alive[sdr] && d.active[sdr])) {
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
      const int32_t* hb = d.hb[cur];
      const int32_t v = hb[gh_cell(d, sdr, ls)];
      const bool in = v >= 0 && !(v & GH_FLAG) &&
                      !(dbit(d.dbits, ls) && removes_at(d.det_cnt[dcur][ls], d.det_min[dcur][ls], sdr));
      if (in) {
        pos = total;
        for (int64_t c = t * d.tw; c < ls; ++c) {
          const int32_t x = hb[gh_cell(d, sdr, c)];
          pos += x >= 0 && !(x & GH_FLAG) &&
                 !(dbit(d.dbits, c) && removes_at(d.det_cnt[dcur][c], d.det_min[dcur][c], sdr));
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
  const int sdr = blockIdx.x * blockDim.x + threadIdx.x;
  if (sdr >= p.n) return;
  int32_t tg[3] = {-1, -1, -1};
  if (d.alive[sdr] && d.active[sdr]) {
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
            tg[q] = (int32_t)(d.col0 + ring_find(d, d.hb[cur], dcur, sdr, t, (int)(want[q] - acc)));
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

// Exclusive scan of inbox_cnt -> inbox_beg; one 1024-thread workgroup.
__global__ __launch_bounds__(1024) void k_inbox_scan(GhDev d, GhRound p) {
  __shared__ int s_sum[1024];
  const int tid = threadIdx.x;
  const int per = (p.n + 1023) / 1024;
  const int b = min(p.n, tid * per), e = min(p.n, b + per);
  int acc = 0;
  for (int x = b; x < e; ++x) acc += d.inbox_cnt[x];
  s_sum[tid] = acc;
  __syncthreads();
  for (int off = 1; off < 1024; off <<= 1) {
    const int v = tid >= off ? s_sum[tid - off] : 0;
    __syncthreads();
    s_sum[tid] += v;
    __syncthreads();
  }
  int run = tid ? s_sum[tid - 1] : 0;
  for (int x = b; x < e; ++x) {
    d.inbox_beg[x] = run;
    d.inbox_fill[x] = 0;
    run += d.inbox_cnt[x];
  }
}

// Inbox order is whatever the atomics give: the merge is a max, so only the
// set of senders matters.
__global__ __launch_bounds__(256) void k_inbox_fill(GhDev d, GhRound p) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= p.n) return;
  for (int q = 0; q < 3; ++q) {
    const int t = d.targets[(int64_t)s * 3 + q];
    if (t >= 0 && d.alive[t]) {
      const int pos = atomicAdd(&d.inbox_fill[t], 1);
      d.inbox[d.inbox_beg[t] + pos] = s;
    }
  }
}

template <bool NT>
__device__ __forceinline__ v4i ldv(const int32_t* p) {
  if constexpr (NT)
    return __builtin_nontemporal_load(reinterpret_cast<const v4i*>(p));
  else
    return *reinterpret_cast<const v4i*>(p);
}
template <bool NT>
__device__ __forceinline__ void stv(int32_t* p, v4i v) {
  if constexpr (NT)
    __builtin_nontemporal_store(v, reinterpret_cast<v4i*>(p));
  else
    *reinterpret_cast<v4i*>(p) = v;
}

// The fused round. Workgroup tile = GH_RB rows x TW members of one table
// tile; the block index is tile-major so the concurrently running workgroups
// sweep one tile (a contiguous N*TW*4-byte slice of each table) together:
// own-row streams are sequential and peer gathers stay in that slice, which
// the on-die caches hold. Each lane owns 4 consecutive members (16-B
// loads/stores); SEG = TW/4 lanes cover one row segment, so a wave handles
// 64/SEG rows per instruction. KB = peer loads issued together (4 or 8).
// NT = non-temporal hints on the once-touched streams (own ts in/out, new hb
// out), leaving the caches to the re-read old-hb slice.
// Rows per workgroup tile: GH_RB, or more when a wave step covers more rows
// (narrow tiles), so all 4 waves have rows.
template <int TW>
constexpr int round_rb() {
  return 1024 / TW > GH_RB ? 1024 / TW : GH_RB;
}

template <int KB, int TW, int TPW, bool NT, bool EXACT>
__global__ __launch_bounds__(256) void k_round(GhDev d, int cur, int dcur, GhRound p) {
  constexpr int SEG = TW / 4;
  constexpr int RPW = 64 / SEG;
  constexpr int RSTEP = 4 * RPW;
  constexpr int RB = round_rb<TW>();  // rows per workgroup tile
  __shared__ int s_dcnt[TW];
  __shared__ int s_dmin[TW];
  __shared__ uint16_t s_part[RB];
  __shared__ unsigned long long s_st[ST_COUNT];
  // per-row metadata of the workgroup's rows, staged once for its TPW tiles
  // so that every row iteration issues its own and its peers' loads back to
  // back: s_meta = alive | active << 1 | inbox count << 2; s_inb = first KB
  // senders
  __shared__ int s_meta[RB];
  __shared__ int s_beg[RB];
  __shared__ int s_inb[RB * KB];

  // block -> (tile group of TPW consecutive tiles, row block); group-major so
  // that the running workgroups sweep the same tiles together
  const int nrb = (p.n + RB - 1) / RB;
  const int ngroups = (int)(p.ld / TW) / TPW;
  int group, rb;
  if (p.xmap && ngroups % 8 == 0) {
    // XCD-aware: blocks b and b+8 share an XCD (round-robin dispatch, speed
    // only), so XCD x = b % 8 sweeps groups x, x+8, ... and its L2 holds the
    // slice it is on.
    const int x = blockIdx.x & 7;
    const int j = blockIdx.x >> 3;
    group = x + 8 * (j / nrb);
    rb = j - (j / nrb) * nrb;
  } else {
    group = blockIdx.x / nrb;
    rb = blockIdx.x - group * nrb;
  }
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = uni(tid >> 6);
  const int sub = lane / SEG;
  const int lc = lane % SEG;

  if (tid < ST_COUNT) s_st[tid] = 0;
  const bool pull = p.peer_mode == GH_PEER_PULL;
  for (int t = tid; t < RB; t += 256) {
    const int i = rb * RB + t;
    int meta = 0, beg = 0;
    if (i < p.n) {
      const int al = d.alive[i];
      meta = al | (d.active[i] << 1) | ((al ? d.inbox_cnt[i] : 0) << 2);
      beg = pull ? i * p.k : d.inbox_beg[i];
    }
    if (p.ablate == 2) meta &= 3;
    s_meta[t] = meta;
    s_beg[t] = beg;
  }
  __syncthreads();
  for (int t = tid; t < RB * KB; t += 256) {
    const int row = t / KB, q = t - row * KB;
    s_inb[t] = q < (s_meta[row] >> 2) ? d.inbox[s_beg[row] + q] : 0;
  }
  __syncthreads();

  const int32_t* __restrict__ hbo = d.hb[cur];
  int32_t* __restrict__ hbn = d.hb[cur ^ 1];
  int32_t* __restrict__ tsb = d.ts;
  const int32_t r = p.r;
  int n_unknown = 0, n_tomb = 0, n_det = 0, n_rel = 0, n_merged = 0;

#pragma unroll 1
  for (int tt = 0; tt < TPW; ++tt) {
  const int tile = group * TPW + tt;
  const int64_t l0 = (int64_t)tile * TW + lc * 4;                   // local column of this lane's first cell
  const int64_t c0 = d.col0 + l0;                                   // its global member id
  const int64_t tb = (int64_t)tile * ((int64_t)p.n * TW) + lc * 4;  // tile base + lane offset
  for (int t = tid; t < TW; t += 256) {
    s_dcnt[t] = 0;
    s_dmin[t] = INT_MAX;
  }
  for (int t = tid; t < RB; t += 256) s_part[t] = 0;
  __syncthreads();

  // REMOVE bits of this lane's 4 members (rare: slow path only when set)
  const uint32_t my4 = (d.dbits[l0 >> 5] >> (l0 & 31)) & 0xFu;
  int dc[4] = {0, 0, 0, 0}, dm[4] = {0, 0, 0, 0};
  if (my4) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      dc[j] = d.det_cnt[dcur][l0 + j];
      dm[j] = d.det_min[dcur][l0 + j];
    }
  }

  // One row iteration = RPW rows per wave: the own segment and the first KB
  // senders' segments are issued together, then merged.
  struct Rows {
    v4i v;        // own segment
    v4i pv[KB];   // first KB senders' segments
    int ps[KB];   // their row ids
    int meta, i, rr;
    bool valid;
  };
  auto issue = [&](Rows& L, int it) {
    L.rr = wave * RPW + it * RSTEP + sub;
    const int i_raw = rb * RB + L.rr;
    L.valid = i_raw < p.n;
    L.i = L.valid ? i_raw : p.n - 1;  // in-range row for the loads of idle lanes
    const int rs = L.valid ? L.rr : 0;
    int meta = s_meta[rs];
    if constexpr (RPW == 1) meta = uni(meta);
    L.meta = meta;
    const int cntv = meta >> 2;
    L.v = ldv<false>(hbo + tb + (int64_t)L.i * TW);  // re-read by peers: keep it cached
#pragma unroll
    for (int q = 0; q < KB; ++q) {
      int s = L.i;
      if (q < cntv) {
        s = s_inb[rs * KB + q];
        if constexpr (RPW == 1) s = uni(s);
      }
      L.ps[q] = s;
      L.pv[q] = ldv<false>(hbo + tb + (int64_t)(p.ablate == 1 ? L.i : s) * TW);
    }
  };
  auto merge_seg = [&](int m[4], const v4i& x4, int s) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int x = x4[j];
      // sender snapshot: present and not detected by s (sign and flag
      // clear), +1 on s's diagonal
      int val = (x & (int)(0x80000000u | GH_FLAG)) ? -1 : gh_hbv(x) + ((c0 + j) == s);
      if (((my4 >> j) & 1u) && removes_at(dc[j], dm[j], s)) val = -1;
      m[j] = max(m[j], val);
    }
  };

  constexpr int NIT = RB / RSTEP;
#pragma unroll 1
  for (int it = 0; it < NIT; ++it) {
    Rows L;
    issue(L, it);
    const int i = L.i;
    const int64_t off = tb + (int64_t)i * TW;
    const int al = (L.meta & 1) && L.valid;
    const int ac = (L.meta >> 1) & 1;
    const int cntv = L.meta >> 2;

    int m[4] = {-1, -1, -1, -1};
#pragma unroll
    for (int q = 0; q < KB; ++q)
      if (q < cntv) merge_seg(m, L.pv[q], L.ps[q]);
    // rare: more senders than KB (ring mode hubs)
    int cmax = cntv;
    if constexpr (RPW > 1) {
#pragma unroll
      for (int o = SEG; o < 64; o <<= 1) cmax = max(cmax, __shfl_xor(cmax, o));
    }
    for (int q = KB; q < cmax; ++q) {
      if (q < cntv) {
        const int s = d.inbox[s_beg[L.valid ? L.rr : 0] + q];
        merge_seg(m, ldv<false>(hbo + tb + (int64_t)s * TW), s);
      }
    }

    v4i xo = L.v;
    int npres = 0;
    bool any_det = false;
    if (al) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int64_t c = c0 + j;
        const int64_t oj = off + j;
        const int32_t w = xo[j];
        int x = gh_ext(w);
        const int a = gh_age(w);  // meaningful unless absent
        bool now = false;         // ts := r in this round
        // step 1: REMOVE delivery (slave/slave.go:236-240, 276-286)
        if (((my4 >> j) & 1u) && removes_at(dc[j], dm[j], i)) {
          if (x >= 0) {
            x = GH_TOMBSTONE;
            n_tomb++;
          } else if (x == GH_ABSENT) {
            n_unknown++;
          }
        }
        if (!ac) {
          if (x >= 0) now = true;  // step 2 guard (:505-507)
        } else {
          if (c == i) {
            if (x >= 0) {  // step 3 own heartbeat (:443-448)
              x = min(x + 1, GH_HB_MAX);
              now = true;
            }
          } else if (x >= 0 && (w & GH_FLAG)) {  // step 4 detect (:468-473), decided at the last write
            x = GH_TOMBSTONE;
            n_det++;
            any_det = true;
            atomicAdd(&s_dcnt[lc * 4 + j], 1);
            atomicMin(&s_dmin[lc * 4 + j], i);
          }
          if (x == GH_TOMBSTONE && gh_stale<EXACT>(d, w, oj, r, p.t_cleanup)) {  // step 5 clean (:490-492)
            x = GH_ABSENT;
            n_rel++;
            if (a < GH_AGE_CAP) tsb[oj] = r - a;  // an absent cell keeps its ts in ts[]
          }
        }
        if (x >= GH_ABSENT && m[j] > x) {  // step 6 merge (:424-426, :435-437)
          x = m[j];
          now = true;
          n_merged++;
        }
        int32_t out = GH_ABSENT;
        if (x != GH_ABSENT) {
          int an = 1;  // age in round r+1 of a cell stamped now
          if (!now) {
            an = gh_inc(a);
            if (a == GH_AGE_CAP - 1) tsb[oj] = r + 1 - GH_AGE_CAP;  // saturates: keep the exact ts
          }
          out = x >= 0 ? gh_present(x, an, gh_flag_for<EXACT>(d, x, an, c, i, oj, r + 1, p.t_fail)) : gh_tomb(an);
        }
        xo[j] = out;
      }
    }
    // crashed rows are frozen: their cells are carried into the new buffer as is
#pragma unroll
    for (int j = 0; j < 4; ++j) npres += xo[j] >= 0;
    if (L.valid) stv<NT>(hbn + off, xo);
#pragma unroll
    for (int o = SEG / 2; o > 0; o >>= 1) {
      npres += __shfl_xor(npres, o);
      any_det |= __shfl_xor((int)any_det, o) != 0;
    }
    if (lc == 0 && L.valid) {
      s_part[L.rr] = (uint16_t)npres;
      if (any_det) d.det_any[i] = 1;
    }
  }

  __syncthreads();
  const int row0 = rb * RB;
  for (int t = tid; t < RB; t += 256)
    if (row0 + t < p.n) d.part[(int64_t)tile * p.n + row0 + t] = s_part[t];
  for (int t = tid; t < TW; t += 256) {
    if (s_dcnt[t]) {
      const int64_t c = (int64_t)tile * TW + t;
      atomicAdd(&d.det_cnt[dcur ^ 1][c], s_dcnt[t]);
      atomicMin(&d.det_min[dcur ^ 1][c], s_dmin[t]);
    }
  }
  __syncthreads();  // s_dcnt / s_part are reused by the next tile
  }  // tiles

  if (n_unknown) atomicAdd(&s_st[ST_REMOVE_UNKNOWN], (unsigned long long)n_unknown);
  if (n_tomb) atomicAdd(&s_st[ST_TOMBSTONED], (unsigned long long)n_tomb);
  if (n_det) atomicAdd(&s_st[ST_DETECTIONS], (unsigned long long)n_det);
  if (n_rel) atomicAdd(&s_st[ST_RELEASED], (unsigned long long)n_rel);
  if (n_merged) atomicAdd(&s_st[ST_MERGED], (unsigned long long)n_merged);
  __syncthreads();
  if (tid < ST_COUNT && s_st[tid]) atomicAdd(&d.stats[tid], s_st[tid]);
}

// Rows: sum the per-tile partial counts (local present count). Columns:
// bitmap + list of D_r, and reset the consumed D_{r-1} accumulators for reuse
// in round r+1.
__global__ __launch_bounds__(256) void k_finish(GhDev d, int dcur, GhRound p, int nchunks) {
  const int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (x < p.n) {
    int s0 = 0, s1 = 0, s2 = 0, s3 = 0;
    int ch = 0;
    for (; ch + 4 <= nchunks; ch += 4) {
      s0 += d.part[(int64_t)ch * p.n + x];
      s1 += d.part[(int64_t)(ch + 1) * p.n + x];
      s2 += d.part[(int64_t)(ch + 2) * p.n + x];
      s3 += d.part[(int64_t)(ch + 3) * p.n + x];
    }
    for (; ch < nchunks; ++ch) s0 += d.part[(int64_t)ch * p.n + x];
    d.cntl[x] = s0 + s1 + s2 + s3;
  }
  const int dnew = dcur ^ 1;
  bool has = false;
  if (x < p.ld) {
    has = d.det_cnt[dnew][x] > 0;
    d.det_cnt[dcur][x] = 0;
    d.det_min[dcur][x] = INT_MAX;
  }
  const unsigned long long m = __ballot(has);
  const int lane = threadIdx.x & 63;
  if (x - lane < p.ld && lane == 0) {
    const int64_t w = (x - lane) >> 5;
    d.dbits[w] = (uint32_t)m;
    d.dbits[w + 1] = (uint32_t)(m >> 32);
    if (m) {
      atomicAdd(&d.nd[dnew], __popcll(m));
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

// one segment per (tile, row): the tile's run summary (segmented scan over
// the SEG lanes, last lane holds the whole tile)
template <int TW>
__global__ __launch_bounds__(256) void k_quirk_sum(GhDev d, int cur, int dcur, GhRound p) {
  constexpr int SEG = SegWalk<TW>::SEG;
  const SegWalk<TW> w(p);
  for (int64_t base = w.first; base < w.nseg; base += w.stride) {
    const int64_t sid = base + w.sub;
    const bool valid = sid < w.nseg;
    const int64_t t = valid ? sid / p.n : 0;
    const int i = valid ? (int)(sid - t * p.n) : 0;
    int f = 0;
    if (valid) {
      const v4i v = *reinterpret_cast<const v4i*>(d.hb[cur] + t * d.tstride + (int64_t)i * TW + w.lc * 4);
      const uint32_t rm = removed4(d, dcur, t * TW + w.lc * 4, i);
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (v[j] >= 0 && !((rm >> j) & 1u)) f = q_compose(f, (v[j] & GH_FLAG) ? 6 : 5);
    }
#pragma unroll
    for (int o = 1; o < SEG; o <<= 1) {
      const int other = __shfl_up(f, o, SEG);
      if (w.lc >= o) f = q_compose(other, f);
    }
    if (valid && w.lc == SEG - 1) d.qsum[sid] = (uint8_t)f;
  }
}

// one thread per row: exclusive prefix over the shard's tiles (in place),
// the shard's total and its last tile holding a present cell
__global__ __launch_bounds__(256) void k_quirk_prefix(GhDev d, GhRound p) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= p.n) return;
  const int64_t ntiles = p.ld / d.tw;
  int pre = 0, last = -1;
  for (int64_t t = 0; t < ntiles; ++t) {
    const int f = d.qsum[t * p.n + i];
    d.qsum[t * p.n + i] = (uint8_t)pre;
    if (f & 4) last = (int)t;
    pre = q_compose(pre, f);
  }
  d.qall[(int64_t)d.rank * p.n + i] = (uint8_t)pre;
  d.qlast[i] = last;
}

// one thread per row: the run state entering this shard (the shards before
// it, in member order) and whether the row's last list entry is here
__global__ __launch_bounds__(256) void k_quirk_carry(GhDev d, GhRound p) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= p.n) return;
  int s = 0;
  bool later = false;
  for (int g = 0; g < d.world; ++g) {
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
  constexpr int SEG = SegWalk<TW>::SEG;
  const SegWalk<TW> w(p);
  for (int64_t base = w.first; base < w.nseg; base += w.stride) {
    const int64_t sid = base + w.sub;
    const int64_t t = sid < w.nseg ? sid / p.n : 0;
    const int i = sid < w.nseg ? (int)(sid - t * p.n) : 0;
    const bool valid = sid < w.nseg && d.alive[i] && d.active[i];  // only active rows detect (and send)
    int32_t* cell = d.hb[cur] + t * d.tstride + (int64_t)i * TW + w.lc * 4;
    v4i v = {-1, -1, -1, -1};
    uint32_t rm = 0;
    if (valid) {
      v = *reinterpret_cast<const v4i*>(cell);
      rm = removed4(d, dcur, t * TW + w.lc * 4, i);
    }
    int f = 0, lastj = -1;
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (v[j] >= 0 && !((rm >> j) & 1u)) {
        f = q_compose(f, (v[j] & GH_FLAG) ? 6 : 5);
        lastj = w.lc * 4 + j;
      }
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
    const int qc = d.qcarry[i];
    int s = q_apply(excl, q_apply(d.qsum[sid], qc & 1));
    const int lastc = ((qc & 2) && d.qlast[i] == t) ? lastj : -1;  // the row's last list entry, if here
    bool changed = false;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (!(v[j] >= 0 && !((rm >> j) & 1u))) continue;
      if (!(v[j] & GH_FLAG)) {
        s = 0;
        continue;
      }
      if (!(s == 0 || w.lc * 4 + j == lastc)) {
        v[j] &= ~GH_FLAG;  // skipped this round
        changed = true;
      }
      s ^= 1;
    }
    if (changed) *reinterpret_cast<v4i*>(cell) = v;
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
  const int64_t waves = ((p.ld / tw) * p.n + (64 / (tw / 4)) - 1) / (64 / (tw / 4));
  return (unsigned)std::max<int64_t>(1, std::min<int64_t>((waves + 3) / 4, 16384));
}

template <int TW>
static void quirk_sum(const GhDev& d, int cur, int dcur, const GhRound& p, hipStream_t s) {
  hipLaunchKernelGGL(k_quirk_sum<TW>, dim3(seg_grid(p, TW)), dim3(256), 0, s, d, cur, dcur, p);
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

void launch_quirk_apply(const GhDev& d, int cur, int dcur, const GhRound& p, hipStream_t s) {
  hipLaunchKernelGGL(k_quirk_carry, dim3((p.n + 255) / 256), dim3(256), 0, s, d, p);
  GH_TW_DISPATCH(quirk_apply, d, cur, dcur, p, s)
}

void launch_prep(const GhDev& d, int dcur, hipStream_t s) {
  hipLaunchKernelGGL(k_prep, dim3(1), dim3(1), 0, s, d, dcur);
}

void launch_active_pre(const GhDev& d, int cur, int dcur, const GhRound& p, hipStream_t s) {
  hipLaunchKernelGGL(k_active_pre, dim3((p.n + 255) / 256), dim3(256), 0, s, d, cur, dcur, p);
  hipLaunchKernelGGL(k_active_exact, dim3((p.n + 3) / 4), dim3(256), 0, s, d, cur, dcur, p);
}

void launch_active_post(const GhDev& d, const GhRound& p, hipStream_t s) {
  hipLaunchKernelGGL(k_active_post, dim3((p.n + 255) / 256), dim3(256), 0, s, d, p);
}

void launch_peers_pull(const GhDev& d, int cur, int dcur, const GhRound& p, hipStream_t s) {
  hipLaunchKernelGGL(k_peers_pull, dim3((d.ncs + 255) / 256), dim3(256), 0, s, d, cur, dcur, p);
}

void launch_ring_count(const GhDev& d, int cur, int dcur, const GhRound& p, hipStream_t s) {
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

template <int KB, int TW, int TPW>
static void launch_round_tpw(const GhDev& d, int cur, int dcur, const GhRound& p, hipStream_t s, bool nt) {
  constexpr int RB = round_rb<TW>();
  const int nrb = (p.n + RB - 1) / RB;
  const dim3 grid((unsigned)(nrb * (p.ld / TW / TPW))), blk(256);
  // timeouts at or above the age cap need the exact ts of saturated cells
  if (p.t_fail >= GH_AGE_CAP || p.t_cleanup >= GH_AGE_CAP)
    hipLaunchKernelGGL((k_round<KB, TW, TPW, false, true>), grid, blk, 0, s, d, cur, dcur, p);
  else if (nt)
    hipLaunchKernelGGL((k_round<KB, TW, TPW, true, false>), grid, blk, 0, s, d, cur, dcur, p);
  else
    hipLaunchKernelGGL((k_round<KB, TW, TPW, false, false>), grid, blk, 0, s, d, cur, dcur, p);
}

// tiles per workgroup: ld / TW is a multiple of 8 (host padding)
template <int KB, int TW>
static void launch_round_tw(const GhDev& d, int cur, int dcur, const GhRound& p, hipStream_t s, bool nt) {
  switch (p.tpw) {
    case 1: launch_round_tpw<KB, TW, 1>(d, cur, dcur, p, s, nt); break;
    case 2: launch_round_tpw<KB, TW, 2>(d, cur, dcur, p, s, nt); break;
    case 8: launch_round_tpw<KB, TW, 8>(d, cur, dcur, p, s, nt); break;
    default: launch_round_tpw<KB, TW, 4>(d, cur, dcur, p, s, nt); break;
  }
}

template <int KB>
static void launch_round_kb(const GhDev& d, int cur, int dcur, const GhRound& p, hipStream_t s, bool nt) {
  switch (d.tw) {
    case 8: launch_round_tw<KB, 8>(d, cur, dcur, p, s, nt); break;
    case 16: launch_round_tw<KB, 16>(d, cur, dcur, p, s, nt); break;
    case 32: launch_round_tw<KB, 32>(d, cur, dcur, p, s, nt); break;
    case 128: launch_round_tw<KB, 128>(d, cur, dcur, p, s, nt); break;
    case 256: launch_round_tw<KB, 256>(d, cur, dcur, p, s, nt); break;
    default: launch_round_tw<KB, 64>(d, cur, dcur, p, s, nt); break;
  }
}

void launch_round(const GhDev& d, int cur, int dcur, const GhRound& p, hipStream_t s, bool nt) {
  if (p.peer_mode == GH_PEER_PULL && p.k <= 4)
    launch_round_kb<4>(d, cur, dcur, p, s, nt);
  else
    launch_round_kb<8>(d, cur, dcur, p, s, nt);
}

void launch_finish(const GhDev& d, int dcur, const GhRound& p, hipStream_t s) {
  const int64_t span = p.ld > p.n ? p.ld : p.n;
  const int nchunks = (int)(p.ld / d.tw);
  hipLaunchKernelGGL(k_finish, dim3((unsigned)((span + 255) / 256)), dim3(256), 0, s, d, dcur, p,
                     nchunks);
}
