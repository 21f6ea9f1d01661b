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

// One wave per row: each lane reads 4 consecutive members (one tile), the
// wave 256 members per step.
__global__ __launch_bounds__(256) void k_count(GhDev d, int cur, GhRound p) {
  const int i = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (i >= p.n) return;
  const int32_t* hb = d.hb[cur];
  int cnt = 0;
  for (int64_t c = lane * 4; c < p.ld; c += 256) {
    const int4 v = *reinterpret_cast<const int4*>(hb + gh_cell(d, i, c));
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

// Storage-order walk over rows [row0, row0+nrows) of every local tile.
struct RowsWalk {
  int64_t per_tile, total;
  __device__ RowsWalk(const GhDev& d, int64_t nrows) : per_tile(nrows * d.tw), total(nrows * d.ld) {}
  // idx -> (row i, local column c, tiled offset of cell (i, c))
  __device__ void at(const GhDev& d, int64_t idx, int64_t row0, int64_t& i, int64_t& c, int64_t& off) const {
    const int64_t t = idx / per_tile;
    const int64_t rem = idx - t * per_tile;
    i = row0 + (rem >> d.lgtw);
    const int64_t cw = rem & (d.tw - 1);
    c = (t << d.lgtw) + cw;
    off = t * d.tstride + (i << d.lgtw) + cw;
  }
};

__global__ __launch_bounds__(256) void k_fill(GhDev d, int cur, int32_t hb0, int32_t ts0, GhRound p) {
  const RowsWalk w(d, p.n);
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < w.total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    int64_t i, c, off;
    w.at(d, idx, 0, i, c, off);
    if (c < d.ncol) {
      d.hb[cur][off] = encode(hb0, ts0, d.col0 + c, i, p);
      d.ts[off] = ts0;
    } else {
      d.hb[cur][off] = GH_ABSENT;
      d.ts[off] = 0;
    }
  }
}

__global__ __launch_bounds__(256) void k_pack(GhDev d, int cur, const int32_t* hb_rows, const int32_t* ts_rows,
                                              int64_t row0, int64_t nrows, GhRound p) {
  const RowsWalk w(d, nrows);
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < w.total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    int64_t i, c, off;
    w.at(d, idx, row0, i, c, off);
    if (c >= d.ncol) continue;
    const int64_t src = (i - row0) * d.n + d.col0 + c;
    d.hb[cur][off] = encode(hb_rows[src], ts_rows[src], d.col0 + c, i, p);
    d.ts[off] = ts_rows[src];
  }
}

// what = 0: external hb; what = 1: exact ts = r - age where the age has it
// (alive rows, unsaturated), else the kept ts[].
__global__ __launch_bounds__(256) void k_unpack(GhDev d, int cur, int32_t* dst, int64_t row0, int64_t nrows,
                                                int what, GhRound p) {
  const RowsWalk w(d, nrows);
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < w.total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    int64_t i, c, off;
    w.at(d, idx, row0, i, c, off);
    if (c >= d.ncs) continue;
    const int32_t v = d.hb[cur][off];
    int32_t x;
    if (what == 0)
      x = gh_ext(v);
    else if (v != GH_ABSENT && d.alive[i] && gh_age(v) < GH_AGE_CAP)
      x = p.r - gh_age(v);
    else
      x = d.ts[off];
    dst[(i - row0) * d.ncs + c] = x;
  }
}

// A stopped row is frozen (k_round carries it unchanged) while the round
// counter moves on, so its ages stop meaning anything: keep the exact ts.
__global__ __launch_bounds__(256) void k_freeze(GhDev d, int cur, const int32_t* rows, int32_t nr, GhRound p) {
  const int64_t total = (int64_t)nr * d.ncol;
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    const int64_t off = gh_cell(d, rows[idx / d.ncol], idx % d.ncol);
    const int32_t v = d.hb[cur][off];
    if (v != GH_ABSENT && gh_age(v) < GH_AGE_CAP) d.ts[off] = p.r - gh_age(v);
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
    for (int b = 0; b < 32; ++b) {
      const int64_t c = w * 32 + b;
      if (c < d.ncol && d.hb[cur][gh_cell(d, row, c)] >= 0) bits |= 1u << b;
    }
    out[idx] = bits;
  }
}

// LEAVE from each leaver c to every alive member j of c's list (j != c):
// removeMember(c) at j. The leavers' lists are the gathered bitmaps rbits
// [world][nl][ncsw]; cell (j, c) lives on c's shard.
__global__ __launch_bounds__(256) void k_leave(GhDev d, int cur, const int32_t* leavers, int32_t nl,
                                               GhRound p) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  int unknown = 0, tomb = 0;
  if (j < p.n && d.alive[j]) {
    int32_t* hb = d.hb[cur];
    for (int q = 0; q < nl; ++q) {
      const int c = leavers[q];
      const int64_t lc = (int64_t)c - d.col0;
      if (lc < 0 || lc >= d.ncol) continue;
      if (c == j || !gh_gbit(d, d.rbits, nl, q, j)) continue;
      const int64_t off = gh_cell(d, j, lc);
      const int32_t x = hb[off];
      if (x >= 0) {
        hb[off] = gh_tomb(gh_age(x));  // keeps its ts (slave/slave.go:280)
        tomb++;
      } else if (x == GH_ABSENT) {
        unknown++;
      }
    }
  }
  if (tomb) atomicAdd(&d.stats[ST_TOMBSTONED], (unsigned long long)tomb);
  if (unknown) atomicAdd(&d.stats[ST_REMOVE_UNKNOWN], (unsigned long long)unknown);
}

// Fresh joiner processes start with an empty MemberList (SPEC D7).
__global__ __launch_bounds__(256) void k_join_reset(GhDev d, int cur, const int32_t* rows,
                                                    int32_t nr, GhRound p) {
  const int64_t total = (int64_t)nr * p.ld;
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    const int64_t off = gh_cell(d, rows[idx / p.ld], idx % p.ld);
    d.hb[cur][off] = GH_ABSENT;
    d.ts[off] = 0;
  }
}

// addNewMember at the introducer (slave/slave.go:250-255) for the joiners
// whose column is local. nd[4] counts this shard's adds.
__global__ void k_join_add(GhDev d, int cur, const int32_t* joiners, int32_t nj, int32_t I,
                           GhRound p) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  int added = 0;
  for (int q = 0; q < nj; ++q) {
    const int64_t lc = (int64_t)joiners[q] - d.col0;
    if (lc < 0 || lc >= d.ncol) continue;
    const int64_t off = gh_cell(d, I, lc);
    if (d.hb[cur][off] < 0) {
      d.hb[cur][off] = gh_present(0, 0);  // hb 0, ts = now (age 0 in round r)
      added++;
    }
  }
  d.nd[4] = added;
}

// The introducer's full list to every alive member of it (:256-272), merged
// with MergeMemberList's rule at now = r. nd[4] = adds over all shards;
// rbits row 0 = the introducer's list after the adds.
__global__ __launch_bounds__(256) void k_join_bcast(GhDev d, int cur, int32_t I, GhRound p) {
  if (d.nd[4] == 0) return;
  int32_t* hb = d.hb[cur];
  const RowsWalk w(d, p.n);
  int merged = 0;
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < w.total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    int64_t j, c, off;
    w.at(d, idx, 0, j, c, off);
    if (c >= d.ncol || j == I || !d.alive[j] || !gh_gbit(d, d.rbits, 1, 0, j)) continue;
    const int32_t mv = hb[gh_cell(d, I, c)];
    if (mv < 0) continue;
    const int32_t m = gh_hbv(mv);
    const int32_t x = gh_ext(hb[off]);
    if (x >= GH_ABSENT && m > x) {
      hb[off] = gh_present(m, 0);  // ts = now: not stale next round
      merged++;
    }
  }
  if (merged) atomicAdd(&d.stats[ST_MERGED], (unsigned long long)merged);
}

// MergeMemberList of an external list into row `obs` at tick p.r - 1 (the
// last completed round): the cell's age in the coming round p.r is 1.
__global__ __launch_bounds__(256) void k_merge_list(GhDev d, int cur, int32_t obs, const int32_t* ids,
                                                    const int32_t* hb, int64_t n, GhRound p) {
  const int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (x >= n) return;
  const int32_t c = ids[x];
  const int64_t lc = (int64_t)c - d.col0;
  if (lc < 0 || lc >= d.ncol) return;
  const int64_t off = gh_cell(d, obs, lc);
  const int32_t v = d.hb[cur][off];
  const int32_t cur_hb = gh_ext(v);
  const int32_t m = hb[x];
  if (cur_hb >= GH_ABSENT && m > cur_hb) {  // :424-426, :435-438; tombstones blocked (:432-434)
    d.hb[cur][off] = gh_present(m, 1, gh_flag_for<false>(d, m, 1, c, obs, off, p.r, p.t_fail));
    atomicAdd(&d.nd[5], 1);
  }
}

unsigned grid_for(int64_t work) {
  return (unsigned)std::max<int64_t>(1, std::min<int64_t>((work + 255) / 256, kMaxGrid));
}

}  // namespace

void launch_count(const GhDev& d, int cur, const GhRound& p, hipStream_t s) {
  hipLaunchKernelGGL(k_count, dim3((p.n + 3) / 4), dim3(256), 0, s, d, cur, p);
}

void launch_fill(const GhDev& d, int cur, int32_t hb0, int32_t ts0, const GhRound& p, hipStream_t s) {
  hipLaunchKernelGGL(k_fill, dim3(grid_for((int64_t)p.n * p.ld)), dim3(256), 0, s, d, cur, hb0, ts0, p);
}

void launch_pack(const GhDev& d, int cur, const int32_t* hb_rows, const int32_t* ts_rows, int64_t row0,
                 int64_t nrows, const GhRound& p, hipStream_t s) {
  if (nrows == 0) return;
  hipLaunchKernelGGL(k_pack, dim3(grid_for(nrows * d.ld)), dim3(256), 0, s, d, cur, hb_rows, ts_rows, row0, nrows, p);
}

void launch_unpack(const GhDev& d, int cur, int32_t* dst_rows, int64_t row0, int64_t nrows, int what,
                   const GhRound& p, hipStream_t s) {
  if (nrows == 0) return;
  hipLaunchKernelGGL(k_unpack, dim3(grid_for(nrows * d.ld)), dim3(256), 0, s, d, cur, dst_rows, row0, nrows, what, p);
}

void launch_freeze(const GhDev& d, int cur, const int32_t* rows, int32_t nr, const GhRound& p, hipStream_t s) {
  if (nr == 0 || d.ncol == 0) return;
  hipLaunchKernelGGL(k_freeze, dim3(grid_for((int64_t)nr * d.ncol)), dim3(256), 0, s, d, cur, rows, nr, p);
}

void launch_rowbits(const GhDev& d, int cur, const int32_t* rows, int32_t nr, hipStream_t s) {
  if (nr == 0) return;
  hipLaunchKernelGGL(k_rowbits, dim3(grid_for((int64_t)nr * d.ncsw)), dim3(256), 0, s, d, cur, rows, nr);
}

void launch_leave(const GhDev& d, int cur, const int32_t* leavers, int32_t nl, const GhRound& p,
                  hipStream_t s) {
  hipLaunchKernelGGL(k_leave, dim3((p.n + 255) / 256), dim3(256), 0, s, d, cur, leavers, nl, p);
}

void launch_join_add(const GhDev& d, int cur, const int32_t* joiners, int32_t nj, int32_t introducer,
                     const GhRound& p, hipStream_t s) {
  hipLaunchKernelGGL(k_join_add, dim3(1), dim3(64), 0, s, d, cur, joiners, nj, introducer, p);
}

void launch_join_bcast(const GhDev& d, int cur, int32_t introducer, const GhRound& p, hipStream_t s) {
  hipLaunchKernelGGL(k_join_bcast, dim3(grid_for((int64_t)p.n * p.ld)), dim3(256), 0, s, d, cur, introducer, p);
}

void launch_join_reset(const GhDev& d, int cur, const int32_t* rows, int32_t nr, const GhRound& p,
                       hipStream_t s) {
  if (nr == 0) return;
  hipLaunchKernelGGL(k_join_reset, dim3(grid_for((int64_t)nr * p.ld)), dim3(256), 0, s, d, cur, rows, nr, p);
}

void launch_merge_list(const GhDev& d, int cur, int32_t obs, const int32_t* ids, const int32_t* hb, int64_t n,
                       const GhRound& p, hipStream_t s) {
  if (n == 0) return;
  hipLaunchKernelGGL(k_merge_list, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, d, cur, obs, ids, hb, n, p);
}
