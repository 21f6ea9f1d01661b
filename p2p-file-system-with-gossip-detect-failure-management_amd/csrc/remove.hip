// The reference's REMOVE recipients (GH_REMOVE_LIST; one engine, member-ID
// list order).
//
// detectfailure (slave/slave.go:460-482) calls removeMember(c) and then
// Remove(c) (:472-473) for each member it detects, in list order, and Remove
// messages every member of the detector's list as it stands at that moment,
// itself excluded (:338-363, :344-346). So row j receives REMOVE(c) in round
// r + 1 iff some row i that detected c in round r listed j when it did:
//
//   R(j, c) = exists i in det(c): listed_i(j) and not (det_i(j) and j <= c)
//
// (listed_i = the row's list before the sweep: present after step 1's
// REMOVEs, self excluded; det_i = the members the sweep removed; in ID order
// the ones removed before c are those below it, and c itself). Split by j:
//
//   j <  c: det(c) meets surv(j) = {i : listed_i(j), not det_i(j)}
//   j >  c: det(c) meets lst(j)  = {i : listed_i(j)}
//   j == c: never (c is gone from every detector's list)
//
// k_rm_cols builds, over the rows that ran the sweep, the column bitmaps
// det(x), surv(x), lst(x) and the counts |surv(x)|, |lst(x)| in one pass over
// the round's input table; k_rm_recv decides every (j, c) of D_r from the
// counts (an empty set: no; |det(c)| + |set| > rows: yes, by pigeonhole) and
// intersects the two bitmaps only where neither settles it (detection storms).
// A healthy cluster's crash wave needs no intersection at all: every row
// detects a crashed member, and a live receiver survives in every list.
#include <limits.h>

#include "gh_internal.h"

namespace {

// Any detection in this round (D_r non-empty): ccnt[2 ld + 1]
__global__ __launch_bounds__(256) void k_rm_any(GhDev d, int dnew, GhRound p) {
  int any = 0;
  for (int64_t x = threadIdx.x; x < p.ld; x += 256) any |= d.det_cnt[dnew][x] > 0;
  if (__syncthreads_or(any) && threadIdx.x == 0) d.ccnt[2 * p.ld + 1] = 1;
}

// One workgroup per 256 local columns x 256 rows: thread (chunk k, group g)
// reads 8 columns of 32 rows and writes their 24 bitmap words.
__global__ __launch_bounds__(256) void k_rm_cols(GhDev d, int cur, int dcur, GhRound p) {
  if (d.ccnt[2 * p.ld + 1] == 0) return;
  __shared__ int s_surv[256], s_lst[256], s_rows;
  const int nrb = (int)((p.n + 255) / 256);
  const int cb = blockIdx.x / nrb, rb = blockIdx.x - cb * nrb;
  const int k = threadIdx.x & 31, g = threadIdx.x >> 5;
  const int64_t c = (int64_t)cb * 256 + 8 * k;
  s_surv[threadIdx.x] = 0;
  s_lst[threadIdx.x] = 0;
  if (threadIdx.x == 0) s_rows = 0;
  __syncthreads();
  uint32_t wd[8] = {}, ws[8] = {}, wl[8] = {};
  const int64_t i0 = (int64_t)rb * 256 + 32 * g;
  int rows = 0;
  if (c < p.ld) {
    const uint32_t b8 = (d.dbits[c >> 5] >> (c & 31)) & 0xFFu;  // D_{r-1} in these columns
    const bool tier = gh_m8(d, cur);
    // 8 rows at a time, their plane and age words loaded together: a tier
    // chunk's present cells are its codes other than 15 (it holds no flag),
    // only escaped chunks decode their 16-bit codes
    for (int q0 = 0; q0 < 32; q0 += 8) {
      uint32_t pw[8], aw[8];
      uint8_t act[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int64_t i = i0 + q0 + u;
        act[u] = i < p.n ? d.active[i] : 0;
        pw[u] = aw[u] = 0;
        if (tier && i < p.n) {
          const int64_t cell = gh_cell(d, i, c);
          aw[u] = d.a4[cur][cell >> 3];
          pw[u] = d.pl[cur][cell >> 3];
        }
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int q = q0 + u;
        const int64_t i = i0 + q;
        if (!act[u]) continue;
        rows++;
        uint32_t pf;
        if (tier && !gh_t4_esc(aw[u])) {
          const uint32_t n15 = ~pw[u];  // a nibble of 15 is absent or a tombstone
          uint32_t t = n15 | (n15 >> 2);
          t |= t >> 1;
          pf = 0;
#pragma unroll
          for (int j = 0; j < 8; ++j) pf |= ((t >> gh_nib(j)) & 1u) << j;
        } else {
          pf = gh_pf8(d, cur, i, c);
        }
        uint32_t lst = pf & 0xFFu;
        for (uint32_t m = lst & b8; m; m &= m - 1) {  // step 1: REMOVE'd at row i
          const int j = __builtin_ctz(m);
          if (gh_rm_at(d, dcur, c + j, i)) lst &= ~(1u << j);
        }
        if (i >= c && i < c + 8) lst &= ~(1u << (i - c));  // Remove skips self (:344-346)
        const uint32_t det = (pf >> 8) & lst;              // the sweep's removals
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          wd[j] |= ((det >> j) & 1u) << q;
          ws[j] |= ((lst & ~det) >> j & 1u) << q;
          wl[j] |= ((lst >> j) & 1u) << q;
        }
      }
    }
    const int64_t w = i0 >> 5;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if (c + j >= p.ld) break;
      const int64_t o = (c + j) * d.nw + w;
      if (w < d.nw) {
        d.cdet[o] = wd[j];
        d.csurv[o] = ws[j];
        d.clst[o] = wl[j];
      }
      atomicAdd(&s_surv[8 * k + j], __popc(ws[j]));
      atomicAdd(&s_lst[8 * k + j], __popc(wl[j]));
    }
  }
  if (k == 0 && cb == 0) atomicAdd(&s_rows, rows);
  __syncthreads();
  const int64_t cc = (int64_t)cb * 256 + threadIdx.x;
  if (cc < p.ld) {
    if (s_surv[threadIdx.x]) atomicAdd(&d.ccnt[cc], s_surv[threadIdx.x]);
    if (s_lst[threadIdx.x]) atomicAdd(&d.ccnt[p.ld + cc], s_lst[threadIdx.x]);
  }
  if (threadIdx.x == 0 && cb == 0 && s_rows) atomicAdd(&d.ccnt[2 * p.ld], s_rows);
}

__device__ __forceinline__ bool meets(const uint32_t* a, const uint32_t* b, int64_t nw) {
  for (int64_t w = 0; w < nw; ++w)
    if (a[w] & b[w]) return true;
  return false;
}

// One workgroup per member c of D_r (grid-stride), a thread per 32 receivers.
// The nonzero words of det(c) are listed in LDS first, so an intersection
// costs one word per listed word (at most |det(c)|), not N / 32: a member
// with few detectors (the common case outside storms, where counts and the
// pigeonhole rule settle most pairs) is decided in O(|det(c)|) per receiver.
constexpr int RM_NZ_CAP = 2048;  // listed words (nw <= 2048 up to N = 65,536; beyond: the full scan)
__global__ __launch_bounds__(256) void k_rm_recv(GhDev d, int dnew, GhRound p) {
  __shared__ uint32_t s_w[RM_NZ_CAP], s_v[RM_NZ_CAP];
  __shared__ int s_nz;
  const int nd = d.nd[2 + dnew];
  const int nact = d.ccnt[2 * p.ld];
  for (int q = blockIdx.x; q < nd; q += gridDim.x) {
    const int64_t c = d.dlist[(int64_t)dnew * p.ld + q];
    const int detc = d.det_cnt[dnew][c];
    const uint32_t* dcol = d.cdet + c * d.nw;
    if (threadIdx.x == 0) s_nz = 0;
    __syncthreads();
    for (int64_t w = threadIdx.x; w < d.nw; w += 256) {
      const uint32_t v = dcol[w];
      if (v) {
        const int at = atomicAdd(&s_nz, 1);
        if (at < RM_NZ_CAP) {
          s_w[at] = (uint32_t)w;
          s_v[at] = v;
        }
      }
    }
    __syncthreads();
    const int nz = s_nz;
    for (int64_t w = threadIdx.x; w < d.nw; w += 256) {
      uint32_t out = 0;
      for (int b = 0; b < 32; ++b) {
        const int64_t j = 32 * w + b;
        if (j >= p.n || j == c) continue;
        const bool low = j < c;
        const int cnt = low ? d.ccnt[j] : d.ccnt[p.ld + j];
        bool r = false;
        if (cnt == 0) {
          r = false;
        } else if (detc + cnt > nact) {
          r = true;  // pigeonhole: both sets live in the rows that ran the sweep
        } else {
          const uint32_t* other = (low ? d.csurv : d.clst) + j * d.nw;
          if (nz <= RM_NZ_CAP) {
            for (int e = 0; e < nz && !r; ++e) r = (s_v[e] & other[s_w[e]]) != 0u;
          } else {
            r = meets(dcol, other, d.nw);
          }
        }
        out |= (uint32_t)r << b;
      }
      d.rcv[dnew][c * d.nw + w] = out;
    }
    __syncthreads();  // s_nz / the list before the next member
  }
}

}  // namespace

void launch_rm_cols(const GhDev& d, int cur, int dcur, const GhRound& p, hipStream_t s) {
  (void)hipMemsetAsync(d.ccnt, 0, sizeof(int32_t) * (2 * p.ld + 2), s);
  hipLaunchKernelGGL(k_rm_any, dim3(1), dim3(256), 0, s, d, dcur ^ 1, p);
  const int64_t nrb = (p.n + 255) / 256;
  hipLaunchKernelGGL(k_rm_cols, dim3((unsigned)(((p.ld + 255) / 256) * nrb)), dim3(256), 0, s, d, cur, dcur, p);
}

void launch_rm_recv(const GhDev& d, int dnew, const GhRound& p, hipStream_t s) {
  hipLaunchKernelGGL(k_rm_recv, dim3((unsigned)std::min<int64_t>(4096, std::max<int64_t>(1, p.n))), dim3(256), 0, s, d,
                     dnew, p);
}
