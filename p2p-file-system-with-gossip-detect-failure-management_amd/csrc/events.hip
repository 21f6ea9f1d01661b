// Churn and state-maintenance kernels (SPEC.md §5, §3).
//   k_count        present count per row (after events / import)
//   k_flags        recompute the eligibility bit of imported rows
//   k_fill         synthetic full-membership start (BASELINE configs 2-4)
//   k_leave        LEAVE delivery: slave/slave.go:310-336 -> :232-235
//   k_join_*       JOIN at the introducer and its full-list broadcast:
//                  slave/slave.go:224-231, 250-274
#include <algorithm>

#include "gh_internal.h"

namespace {

// One wave per row: lanes sweep the row 256 columns per step.
__global__ __launch_bounds__(256) void k_count(GhDev d, int cur, GhRound p) {
  const int i = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (i >= p.n) return;
  const int32_t* row = d.hb[cur] + (int64_t)i * p.ld;
  int cnt = 0;
  for (int64_t c = lane * 4; c < p.ld; c += 256) {
    const int4 v = *reinterpret_cast<const int4*>(row + c);
    cnt += (v.x >= 0) + (v.y >= 0) + (v.z >= 0) + (v.w >= 0);
  }
  for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o);
  if (lane == 0) d.cnt[i] = cnt;
}

__device__ __forceinline__ int32_t with_flag(int32_t x, int32_t t, int64_t c, int64_t i,
                                             int32_t lim_next) {
  if (x >= 0) {
    x &= GH_HBMASK;
    if (x > 1 && c != i && t < lim_next) x |= GH_FLAG;
  }
  return x;
}

__global__ __launch_bounds__(256) void k_flags(GhDev d, int cur, int64_t row0, int64_t nrows,
                                               GhRound p) {
  const int64_t total = nrows * p.ld;
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = row0 + idx / p.ld;
    const int64_t c = idx % p.ld;
    const int64_t off = i * p.ld + c;
    // p.r is the round about to run: eligible <=> ts < r - T_fail
    d.hb[cur][off] = with_flag(d.hb[cur][off], d.ts[off], c, i, p.r - p.t_fail);
  }
}

__global__ __launch_bounds__(256) void k_fill(GhDev d, int cur, int32_t hb0, int32_t ts0,
                                              GhRound p) {
  const int64_t total = (int64_t)p.n * p.ld;
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = idx / p.ld;
    const int64_t c = idx % p.ld;
    if (c < p.n) {
      d.hb[cur][idx] = with_flag(hb0, ts0, c, i, p.r - p.t_fail);
      d.ts[idx] = ts0;
    } else {
      d.hb[cur][idx] = GH_ABSENT;
      d.ts[idx] = 0;
    }
  }
}

// LEAVE from each leaver c to every alive member j of c's list (j != c):
// removeMember(c) at j.
__global__ __launch_bounds__(256) void k_leave(GhDev d, int cur, const int32_t* leavers, int32_t nl,
                                               GhRound p) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  int unknown = 0, tomb = 0;
  if (j < p.n && d.alive[j]) {
    int32_t* hb = d.hb[cur];
    for (int q = 0; q < nl; ++q) {
      const int c = leavers[q];
      if (c == j || hb[(int64_t)c * p.ld + j] < 0) continue;
      const int64_t off = (int64_t)j * p.ld + c;
      const int32_t x = hb[off];
      if (x >= 0) {
        hb[off] = GH_TOMBSTONE;
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
    const int64_t off = (int64_t)rows[idx / p.ld] * p.ld + idx % p.ld;
    d.hb[cur][off] = GH_ABSENT;
    d.ts[off] = 0;
  }
}

// addNewMember at the introducer (slave/slave.go:250-255). nd[4] counts adds.
__global__ void k_join_add(GhDev d, int cur, const int32_t* joiners, int32_t nj, int32_t I,
                           GhRound p) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  int added = 0;
  for (int q = 0; q < nj; ++q) {
    const int64_t off = (int64_t)I * p.ld + joiners[q];
    if (d.hb[cur][off] < 0) {
      d.hb[cur][off] = 0;
      d.ts[off] = p.r;
      added++;
    }
  }
  d.nd[4] = added;
}

// The introducer's full list to every alive member of it (:256-272), merged
// with MergeMemberList's rule at now = r. Grid: rows x 256-column chunks.
__global__ __launch_bounds__(256) void k_join_bcast(GhDev d, int cur, int32_t I, GhRound p) {
  if (d.nd[4] == 0) return;
  const int64_t nchunks = p.ld / GH_CHUNK;
  int32_t* hb = d.hb[cur];
  const int32_t* rowI = hb + (int64_t)I * p.ld;
  int merged = 0;
  for (int64_t tile = blockIdx.x; tile < (int64_t)p.n * nchunks; tile += gridDim.x) {
    const int64_t j = tile / nchunks;
    const int64_t c = (tile % nchunks) * GH_CHUNK + threadIdx.x;
    if (!(d.alive[j] && rowI[j] >= 0 && j != I)) continue;
    const int32_t mv = rowI[c];
    if (mv < 0) continue;
    const int32_t m = mv & GH_HBMASK;
    const int64_t off = j * p.ld + c;
    const int32_t xr = hb[off];
    const int32_t x = xr >= 0 ? (xr & GH_HBMASK) : xr;
    if (x >= GH_ABSENT && m > x) {
      hb[off] = m;  // ts = now: never eligible next round, so no flag
      d.ts[off] = p.r;
      merged++;
    }
  }
  if (merged) atomicAdd(&d.stats[ST_MERGED], (unsigned long long)merged);
}

}  // namespace

void launch_count(const GhDev& d, int cur, const GhRound& p, hipStream_t s) {
  hipLaunchKernelGGL(k_count, dim3((p.n + 3) / 4), dim3(256), 0, s, d, cur, p);
}

void launch_flags(const GhDev& d, int cur, int64_t row0, int64_t nrows, const GhRound& p,
                  hipStream_t s) {
  const int64_t cells = nrows * p.ld;
  if (cells == 0) return;
  hipLaunchKernelGGL(k_flags, dim3((unsigned)std::min<int64_t>((cells + 255) / 256, 65536)), dim3(256), 0, s, d, cur, row0,
                     nrows, p);
}

void launch_fill(const GhDev& d, int cur, int32_t hb0, int32_t ts0, const GhRound& p,
                 hipStream_t s) {
  const int64_t cells = (int64_t)p.n * p.ld;
  hipLaunchKernelGGL(k_fill, dim3((unsigned)std::min<int64_t>((cells + 255) / 256, 65536)), dim3(256), 0, s, d, cur, hb0,
                     ts0, p);
}

void launch_leave(const GhDev& d, int cur, const int32_t* leavers, int32_t nl, const GhRound& p,
                  hipStream_t s) {
  hipLaunchKernelGGL(k_leave, dim3((p.n + 255) / 256), dim3(256), 0, s, d, cur, leavers, nl, p);
}

void launch_join(const GhDev& d, int cur, const int32_t* joiners, int32_t nj, int32_t introducer,
                 const GhRound& p, hipStream_t s) {
  hipLaunchKernelGGL(k_join_add, dim3(1), dim3(64), 0, s, d, cur, joiners, nj, introducer, p);
  const int64_t nchunks = p.ld / GH_CHUNK;
  hipLaunchKernelGGL(k_join_bcast, dim3((unsigned)std::min<int64_t>(p.n * nchunks, 65536)), dim3(256), 0, s, d, cur,
                     introducer, p);
}

void launch_join_reset(const GhDev& d, int cur, const int32_t* rows, int32_t nr, const GhRound& p,
                       hipStream_t s) {
  const int64_t cells = (int64_t)nr * p.ld;
  if (cells == 0) return;
  hipLaunchKernelGGL(k_join_reset, dim3((unsigned)std::min<int64_t>((cells + 255) / 256, 65536)), dim3(256), 0, s, d, cur,
                     rows, nr, p);
}
