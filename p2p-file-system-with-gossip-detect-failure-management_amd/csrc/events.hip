// Churn and state-maintenance kernels (SPEC.md §5, §3). All tables use the
// tiled layout of gh_internal.h (gh_cell) over the shard's local columns.
//   k_count        local present count per row (after events / import)
//   k_fill         synthetic full-membership start (BASELINE configs 2-4)
//   k_pack/unpack  host (hb, ts) rows <-> encoded tiled local columns
//                  (import/export/lsm; gh_internal.h "cell encoding")
//   k_freeze       exact ts of rows that stop (crash / leave) into ts[]
//   k_rowbits      presence bitmap of some rows over the local columns (the
//                  rows' lists, gathered across shards by the host)
//   k_leave        LEAVE delivery: slave/slave.go:310-336 -> :232-235
//   k_join_*       JOIN at the introducer and its full-list broadcast:
//                  slave/slave.go:224-231, 250-274
#include <algorithm>

#include "gh_internal.h"

namespace {

constexpr unsigned kMaxGrid = 65536;

// One wave per row: each lane reads 4 consecutive members (gh_load4), the
// wave 256 members per step.
__global__ __launch_bounds__(256) void k_count(GhDev d, int cur, GhRound p) {
  const int i = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (i >= p.n) return;
  int cnt = 0;
  for (int64_t c = lane * 4; c < p.ld; c += 256) {
    const v4i v = gh_load4(d, cur, i, c);
    cnt += (v.x >= 0) + (v.y >= 0) + (v.z >= 0) + (v.w >= 0);
  }
  for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o);
  if (lane == 0) d.cntl[i] = cnt;
}

// Encoded cell (member cg of row i) for external (hb, ts) in the round r
// about to run.
__device__ __forceinline__ int32_t encode(int32_t x, int32_t t, int64_t cg, int64_t i, const GhRound& p) {
  if (x == GH_ABSENT) return GH_ABSENT;
  const int a = min(max(p.r - t, 0), GH_AGE_CAP);
  return x >= 0 ? gh_present(x, a, x > 1 && cg != i && t < p.r - p.t_fail) : gh_tomb(a);
}

// A set of (tile, row) segments: rows (a list, or [row0, row0 + nrows)) x
// tiles (a list, or all of them); tile-major so that consecutive segments
// are consecutive in memory.
struct SegSet {
  const int32_t* rows;
  int64_t row0, nrows;
  const int32_t* tiles;
  int64_t ntl;
  __device__ int64_t count() const { return nrows * ntl; }
  __device__ void at(int64_t sid, int64_t& i, int64_t& t) const {
    const int64_t a = sid / nrows, r = sid - a * nrows;
    i = rows ? rows[r] : row0 + r;
    t = tiles ? tiles[a] : a;
  }
};

// Read-modify-write of whole segments: G = min(TW, 64) lanes per segment,
// CPL = TW / G cells per lane. op(i, c, off, v) returns the new wide value
// of cell (i, local c) at table offset off. A segment that changed is
// stored narrow when every cell has a narrow code, else wide. Nothing else
// in the launch reads the segments it writes.
template <int TW, class Op>
__global__ __launch_bounds__(256) void k_seg(GhDev d, int buf, SegSet set, const int32_t* gate, Op op) {
  if (gate && *gate == 0) return;
  constexpr int G = TW < 64 ? TW : 64;
  constexpr int CPL = TW / G;
  constexpr int SPW = 64 / G;
  const int lane = threadIdx.x & 63;
  const int sub = lane / G, lg = lane % G;
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
  const int64_t total = set.count();
  const unsigned long long gmask = (G == 64 ? ~0ull : ((1ull << G) - 1)) << (sub * G);
  uint16_t* hn = d.hn[buf];
  int32_t* hw = d.hw[buf];
  const int32_t* base = d.base[buf];
  for (int64_t s0 = wave * SPW; s0 < total; s0 += nw * SPW) {
    const int64_t sid = s0 + sub;
    const bool valid = sid < total;
    int64_t i = 0, t = 0;
    if (valid) set.at(sid, i, t);
    int32_t v[CPL];
    bool changed = false, fit = true;
#pragma unroll
    for (int k = 0; k < CPL; ++k) {
      const int64_t c = t * TW + lg + k * G;
      const int64_t off = t * d.tstride + i * TW + lg + k * G;
      int32_t x = GH_ABSENT;
      if (valid) {
        const uint32_t nx = hn[off];
        x = nx == GH_N_WIDE ? hw[off] : gh_dec16(nx, base[c]);
        const int32_t y = op(i, c, off, x);
        changed |= y != x;
        x = y;
        gh_enc16(x, base[c], fit);
      }
      v[k] = x;
    }
    const bool any = (__ballot(changed) & gmask) != 0;
    const bool narrow = (__ballot(!fit) & gmask) == 0;
    if (!valid || !any) continue;
#pragma unroll
    for (int k = 0; k < CPL; ++k) {
      const int64_t c = t * TW + lg + k * G;
      const int64_t off = t * d.tstride + i * TW + lg + k * G;
      if (narrow) {
        bool f = true;
        hn[off] = (uint16_t)gh_enc16(v[k], base[c], f);
      } else {
        hw[off] = v[k];
        hn[off] = (uint16_t)GH_N_WIDE;
      }
    }
  }
}

struct OpFill {
  GhDev d;
  int32_t hb0, ts0;
  GhRound p;
  __device__ int32_t operator()(int64_t i, int64_t c, int64_t off, int32_t) const {
    if (c >= d.ncol) {
      d.ts[off] = 0;
      return GH_ABSENT;
    }
    d.ts[off] = ts0;
    return encode(hb0, ts0, d.col0 + c, i, p);
  }
};

struct OpPack {
  GhDev d;
  const int32_t *hb_rows, *ts_rows;
  int64_t row0;
  GhRound p;
  __device__ int32_t operator()(int64_t i, int64_t c, int64_t off, int32_t x) const {
    if (c >= d.ncol) return x;
    const int64_t src = (i - row0) * d.n + d.col0 + c;
    d.ts[off] = ts_rows[src];
    return encode(hb_rows[src], ts_rows[src], d.col0 + c, i, p);
  }
};

// Fresh joiner processes start with an empty MemberList (SPEC D7).
struct OpReset {
  GhDev d;
  __device__ int32_t operator()(int64_t, int64_t, int64_t off, int32_t) const {
    d.ts[off] = 0;
    return GH_ABSENT;
  }
};

// LEAVE from each leaver c to every alive member j of c's list (j != c):
// removeMember(c) at j. colq[c] = the leaver's index q in the gathered
// bitmaps rbits [world][nl][ncsw] (-1: not a leaver).
struct OpLeave {
  GhDev d;
  int32_t nl;
  __device__ int32_t operator()(int64_t j, int64_t c, int64_t, int32_t x) const {
    const int q = d.colq[c];
    if (q < 0 || !d.alive[j] || d.col0 + c == j || !gh_gbit(d, d.rbits, nl, q, j)) return x;
    if (x >= 0) {
      atomicAdd(&d.stats[ST_TOMBSTONED], 1ull);
      return gh_tomb(gh_age(x));  // keeps its ts (slave/slave.go:280)
    }
    if (x == GH_ABSENT) atomicAdd(&d.stats[ST_REMOVE_UNKNOWN], 1ull);
    return x;
  }
};

// addNewMember at the introducer (slave/slave.go:250-255) for the joiners
// whose column is local (colq[c] >= 0). nd[4] counts this shard's adds.
struct OpJoinAdd {
  GhDev d;
  __device__ int32_t operator()(int64_t, int64_t c, int64_t, int32_t x) const {
    if (d.colq[c] < 0 || x >= 0) return x;
    atomicAdd(&d.nd[4], 1);
    return gh_present(0, 0);  // hb 0, ts = now (age 0 in round r)
  }
};

// The introducer's full list to every alive member of it (:256-272), merged
// with MergeMemberList's rule at now = r. nd[4] = adds over all shards;
// rbits row 0 = the introducer's list after the adds.
struct OpJoinBcast {
  GhDev d;
  int cur;
  int32_t I;
  __device__ int32_t operator()(int64_t j, int64_t c, int64_t, int32_t x) const {
    if (c >= d.ncol || j == I || !d.alive[j] || !gh_gbit(d, d.rbits, 1, 0, j)) return x;
    const int32_t mv = gh_get(d, cur, I, c);
    if (mv < 0) return x;
    const int32_t m = gh_hbv(mv);
    const int32_t e = gh_ext(x);
    if (e >= GH_ABSENT && m > e) {
      atomicAdd(&d.stats[ST_MERGED], 1ull);
      return gh_present(m, 0);  // ts = now: not stale next round
    }
    return x;
  }
};

// MergeMemberList of an external list into row obs at tick p.r - 1 (the last
// completed round): the cell's age in the coming round p.r is 1. colq[c] =
// the listed heartbeat of local member c (< -2: not listed).
struct OpMergeList {
  GhDev d;
  GhRound p;
  __device__ int32_t operator()(int64_t obs, int64_t c, int64_t off, int32_t x) const {
    const int32_t m = d.colq[c];
    const int32_t e = gh_ext(x);
    if (m < -2 || !(e >= GH_ABSENT && m > e)) return x;  // :424-426, :435-438; tombstones blocked (:432-434)
    atomicAdd(&d.nd[5], 1);
    return gh_present(m, 1, gh_flag_for<false>(d, m, 1, d.col0 + c, obs, off, p.r, p.t_fail));
  }
};

// q -> colq[local column of ids[q]] for the ids local to this shard
__global__ void k_scatter(GhDev d, const int32_t* ids, const int32_t* vals, int32_t n) {
  const int q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= n) return;
  const int64_t lc = (int64_t)ids[q] - d.col0;
  if (lc >= 0 && lc < d.ncol) d.colq[lc] = vals ? vals[q] : q;
}

// what = 0: external hb; what = 1: exact ts = r - age where the age has it
// (alive rows, unsaturated), else the kept ts[].
__global__ __launch_bounds__(256) void k_unpack(GhDev d, int cur, int32_t* dst, int64_t row0, int64_t nrows,
                                                int what, GhRound p) {
  const int64_t per_tile = nrows * d.tw, total = nrows * d.ld;
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    const int64_t t = idx / per_tile, rem = idx - t * per_tile;
    const int64_t i = row0 + (rem >> d.lgtw);
    const int64_t c = (t << d.lgtw) + (rem & (d.tw - 1));
    if (c >= d.ncs) continue;
    const int32_t v = gh_get(d, cur, i, c);
    int32_t x;
    if (what == 0)
      x = gh_ext(v);
    else if (v != GH_ABSENT && d.alive[i] && gh_age(v) < GH_AGE_CAP)
      x = p.r - gh_age(v);
    else
      x = d.ts[gh_cell(d, i, c)];
    dst[(i - row0) * d.ncs + c] = x;
  }
}

// A stopped row is frozen while the round counter moves on, so its ages stop
// meaning anything: keep the exact ts, and store the row wide in BOTH
// buffers (the round skips it). Flags after values: k_freeze_mark.
__global__ __launch_bounds__(256) void k_freeze(GhDev d, int cur, const int32_t* rows, int32_t nr, GhRound p) {
  const int64_t total = (int64_t)nr * d.ld;
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = rows[idx / d.ld], c = idx % d.ld;
    const int64_t off = gh_cell(d, i, c);
    const int32_t v = gh_get(d, cur, i, c);
    if (c < d.ncol && v != GH_ABSENT && gh_age(v) < GH_AGE_CAP) d.ts[off] = p.r - gh_age(v);
    d.hw[0][off] = v;
    d.hw[1][off] = v;
  }
}
__global__ __launch_bounds__(256) void k_freeze_mark(GhDev d, const int32_t* rows, int32_t nr) {
  const int64_t total = (int64_t)nr * d.ld;
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    const int64_t off = gh_cell(d, rows[idx / d.ld], idx % d.ld);
    d.hn[0][off] = (uint16_t)GH_N_WIDE;
    d.hn[1][off] = (uint16_t)GH_N_WIDE;
  }
}

// bit b of word w of row q = local column 32w+b of rows[q] is present
__global__ __launch_bounds__(256) void k_rowbits(GhDev d, int cur, const int32_t* rows, int32_t nr) {
  uint32_t* out = d.rbits + (int64_t)d.rank * nr * d.ncsw;
  const int64_t total = (int64_t)nr * d.ncsw;
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    const int q = (int)(idx / d.ncsw);
    const int64_t w = idx - (int64_t)q * d.ncsw;
    const int row = rows[q];
    uint32_t bits = 0;
    for (int b = 0; b < 32; b += 4) {
      const int64_t c = w * 32 + b;
      if (c >= d.ncol) break;
      const v4i v = gh_load4(d, cur, row, c);
      for (int j = 0; j < 4; ++j)
        if (c + j < d.ncol && v[j] >= 0) bits |= 1u << (b + j);
    }
    out[idx] = bits;
  }
}

// wide segments of buffer buf (first narrow cell = GH_N_WIDE) -> *out
__global__ __launch_bounds__(256) void k_count_wide(GhDev d, int buf, unsigned long long* out) {
  const int64_t total = d.ntiles * d.n;
  unsigned long long cnt = 0;
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    const int64_t t = idx / d.n, i = idx - t * d.n;
    cnt += d.hn[buf][t * d.tstride + i * d.tw] == GH_N_WIDE;
  }
  for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o);
  if ((threadIdx.x & 63) == 0 && cnt) atomicAdd(out, cnt);
}

// base[buf][c] = v for every local column
__global__ void k_setbase(GhDev d, int buf, int32_t v) {
  const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c < d.ld) d.base[buf][c] = v;
}

unsigned grid_for(int64_t work) {
  return (unsigned)std::max<int64_t>(1, std::min<int64_t>((work + 255) / 256, kMaxGrid));
}

}  // namespace

template <class Op>
static void seg_launch(const GhDev& d, int buf, SegSet set, const int32_t* gate, Op op, hipStream_t s) {
  const int64_t segs = set.nrows * set.ntl;
  if (segs == 0) return;
  const int64_t spw = d.tw < 64 ? 64 / d.tw : 1;
  const unsigned grid = grid_for((segs + spw - 1) / spw * 64);
  switch (d.tw) {
    case 8: hipLaunchKernelGGL((k_seg<8, Op>), dim3(grid), dim3(256), 0, s, d, buf, set, gate, op); break;
    case 16: hipLaunchKernelGGL((k_seg<16, Op>), dim3(grid), dim3(256), 0, s, d, buf, set, gate, op); break;
    case 32: hipLaunchKernelGGL((k_seg<32, Op>), dim3(grid), dim3(256), 0, s, d, buf, set, gate, op); break;
    case 128: hipLaunchKernelGGL((k_seg<128, Op>), dim3(grid), dim3(256), 0, s, d, buf, set, gate, op); break;
    case 256: hipLaunchKernelGGL((k_seg<256, Op>), dim3(grid), dim3(256), 0, s, d, buf, set, gate, op); break;
    default: hipLaunchKernelGGL((k_seg<64, Op>), dim3(grid), dim3(256), 0, s, d, buf, set, gate, op); break;
  }
}

static SegSet rows_set(const GhDev& d, const int32_t* rows, int64_t row0, int64_t nrows) {
  return SegSet{rows, row0, nrows, nullptr, d.ntiles};
}

// colq = -1, then colq[local column of ids[q]] = vals ? vals[q] : q
static void scatter(const GhDev& d, const int32_t* ids, const int32_t* vals, int32_t n, int fill, hipStream_t s) {
  (void)hipMemsetAsync(d.colq, fill, sizeof(int32_t) * d.ld, s);
  if (n > 0) hipLaunchKernelGGL(k_scatter, dim3((n + 255) / 256), dim3(256), 0, s, d, ids, vals, n);
}

void launch_count(const GhDev& d, int cur, const GhRound& p, hipStream_t s) {
  hipLaunchKernelGGL(k_count, dim3((p.n + 3) / 4), dim3(256), 0, s, d, cur, p);
}

void launch_fill(const GhDev& d, int cur, int32_t hb0, int32_t ts0, const GhRound& p, hipStream_t s) {
  hipLaunchKernelGGL(k_setbase, dim3((unsigned)((d.ld + 255) / 256)), dim3(256), 0, s, d, cur, hb0 - GH_BASE_LAG);
  seg_launch(d, cur, rows_set(d, nullptr, 0, p.n), nullptr, OpFill{d, hb0, ts0, p}, s);
}

void launch_pack(const GhDev& d, int cur, const int32_t* hb_rows, const int32_t* ts_rows, int64_t row0,
                 int64_t nrows, const GhRound& p, hipStream_t s) {
  seg_launch(d, cur, rows_set(d, nullptr, row0, nrows), nullptr, OpPack{d, hb_rows, ts_rows, row0, p}, s);
}

void launch_unpack(const GhDev& d, int cur, int32_t* dst_rows, int64_t row0, int64_t nrows, int what,
                   const GhRound& p, hipStream_t s) {
  if (nrows == 0) return;
  hipLaunchKernelGGL(k_unpack, dim3(grid_for(nrows * d.ld)), dim3(256), 0, s, d, cur, dst_rows, row0, nrows, what, p);
}

void launch_freeze(const GhDev& d, int cur, const int32_t* rows, int32_t nr, const GhRound& p, hipStream_t s) {
  if (nr == 0) return;
  hipLaunchKernelGGL(k_freeze, dim3(grid_for((int64_t)nr * d.ld)), dim3(256), 0, s, d, cur, rows, nr, p);
  hipLaunchKernelGGL(k_freeze_mark, dim3(grid_for((int64_t)nr * d.ld)), dim3(256), 0, s, d, rows, nr);
}

void launch_count_wide(const GhDev& d, int buf, unsigned long long* out, hipStream_t s) {
  (void)hipMemsetAsync(out, 0, sizeof(unsigned long long), s);
  hipLaunchKernelGGL(k_count_wide, dim3(grid_for(d.ntiles * d.n)), dim3(256), 0, s, d, buf, out);
}

void launch_rowbits(const GhDev& d, int cur, const int32_t* rows, int32_t nr, hipStream_t s) {
  if (nr == 0) return;
  hipLaunchKernelGGL(k_rowbits, dim3(grid_for((int64_t)nr * d.ncsw)), dim3(256), 0, s, d, cur, rows, nr);
}

void launch_leave(const GhDev& d, int cur, const int32_t* leavers, const int32_t* tiles, int32_t ntl, int32_t nl,
                  const GhRound& p, hipStream_t s) {
  (void)p;
  if (ntl == 0) return;
  scatter(d, leavers, nullptr, nl, 0xFF, s);
  seg_launch(d, cur, SegSet{nullptr, 0, d.n, tiles, ntl}, nullptr, OpLeave{d, nl}, s);
}

void launch_join_add(const GhDev& d, int cur, const int32_t* joiners, int32_t nj, int32_t introducer,
                     const GhRound& p, hipStream_t s) {
  (void)p;
  (void)hipMemsetAsync(d.nd + 4, 0, sizeof(int32_t), s);
  scatter(d, joiners, nullptr, nj, 0xFF, s);
  seg_launch(d, cur, rows_set(d, nullptr, introducer, 1), nullptr, OpJoinAdd{d}, s);
}

void launch_join_bcast(const GhDev& d, int cur, int32_t introducer, const GhRound& p, hipStream_t s) {
  seg_launch(d, cur, rows_set(d, nullptr, 0, p.n), d.nd + 4, OpJoinBcast{d, cur, introducer}, s);
}

void launch_join_reset(const GhDev& d, int cur, const int32_t* rows, int32_t nr, const GhRound& p,
                       hipStream_t s) {
  (void)p;
  seg_launch(d, cur, rows_set(d, rows, 0, nr), nullptr, OpReset{d}, s);
}

void launch_merge_list(const GhDev& d, int cur, int32_t obs, const int32_t* ids, const int32_t* hb, int64_t n,
                       const GhRound& p, hipStream_t s) {
  if (n == 0) return;
  scatter(d, ids, hb, (int32_t)n, 0x80, s);
  seg_launch(d, cur, rows_set(d, nullptr, obs, 1), nullptr, OpMergeList{d, p}, s);
}
