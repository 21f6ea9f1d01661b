// Master re-election (SPEC §9): the per-row master check and
// vote target, and rebuild_file_meta's metadata rewrite.
//
//   k_vote_scan    updateMemberList's tail (slave/slave.go:451-457) and
//                  revote_master's target (:930-948) for every row at once:
//                  is the row's master in its list, and which member is
//                  MemberList[0] (the lowest present id, SPEC D1). One wave
//                  per row; the wave stops at the row's first present cell,
//                  so a healthy row costs one 128 B segment, not N cells.
//   k_rebuild      rebuild_file_meta (:986-1043) over the file table, one
//                  thread per file (the files are replicated on every shard).
#include "gh_internal.h"

namespace {

// out[i] = n - (first present global member of row i in this shard's
// columns), 0 if none; out[n + i] = 1 if mview[i] is a present local member.
// Both reduce across shards with MAX.
__global__ __launch_bounds__(256) void k_vote_scan(GhDev d, int cur, const int32_t* mview, int32_t* out) {
  const int lane = threadIdx.x & 63;
  const int64_t i = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (i >= d.n) return;
  if (!gh_owned(d, i)) {  // row layout: the row's owner answers (MAX over shards)
    if (lane == 0) out[i] = out[d.n + i] = 0;
    return;
  }
  int32_t first = 0;
  for (int64_t c0 = 0; c0 < d.ncol; c0 += 64) {
    const int64_t c = c0 + lane;
    const bool pres = c < d.ncol && gh_get(d, cur, i, c, 0).x >= 0;
    const unsigned long long m = __ballot(pres);
    if (m) {
      first = d.n - (int32_t)(d.col0 + c0 + __ffsll((long long)m) - 1);
      break;
    }
  }
  if (lane == 0) {
    const int64_t mc = (int64_t)mview[i] - d.col0;
    out[i] = first;
    out[d.n + i] = (mc >= 0 && mc < d.ncol && gh_get(d, cur, i, mc, 0).x >= 0) ? 1 : 0;
  }
}

// rebuild_file_meta at the new master M, whose list starts L[0..nl) (nl <= 5;
// f0 = L[0] is the member every remote store query goes to, :994). For each
// file: entries (m, version) for every m of M's list whose store was read
// with the file in it (M's own store for m = M, f0's for every other m),
// sorted ascending by version (:1028, sortByValue reverses a descending
// order), ties in list order (SPEC D10); Node_list = the first 4 (:1030-1033),
// Version = the first entry's (:1035), Timestamp = now. A member's store holds
// exactly the files whose metadata lists it (SPEC §9), so every entry carries
// the file's version and the sorted order is list order. M's metadata map
// starts empty, so a file in neither store is gone.
__global__ __launch_bounds__(256) void k_rebuild(GhDev d, int32_t R, int32_t M, int4 L03, int32_t L4, int32_t nl,
                                                 int32_t m_listed, int32_t now) {
  const int64_t f = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (f >= d.fcap || d.ver[f] < 0) return;
  int32_t* rp = d.rep + f * R;
  const int32_t f0 = L03.x;
  bool in_m = false, in_0 = false;
  for (int q = 0; q < R; ++q) {
    in_m |= rp[q] == M;
    in_0 |= rp[q] == f0;
  }
  const int32_t L[5] = {L03.x, L03.y, L03.z, L03.w, L4};
  const int cap = R < 4 ? R : 4;
  int k = 0;
  if (in_0) {
    // every m != M of the list holds it; among L's first 5 at most one is M
    for (int q = 0; q < nl && k < cap; ++q)
      if (L[q] != M || in_m) rp[k++] = L[q];
  } else if (in_m && m_listed) {
    rp[k++] = M;  // only M's own store has it (M may sit anywhere in L; a
                  // list without M never reads M's store)
  }
  for (int q = k; q < R; ++q) rp[q] = -1;
  if (k == 0) {
    d.ver[f] = -1;
  } else {
    d.fts[f] = now;
  }
}

}  // namespace

void launch_vote_scan(const GhDev& d, int cur, const int32_t* mview, int32_t* out, hipStream_t s) {
  hipLaunchKernelGGL(k_vote_scan, dim3((unsigned)((d.n + 3) / 4)), dim3(256), 0, s, d, cur, mview, out);
}

void launch_rebuild(const GhDev& d, int32_t R, int32_t M, const int32_t* L, int32_t nl, int32_t m_listed,
                    int32_t now, hipStream_t s) {
  const int4 l03 = make_int4(L[0], L[1], L[2], L[3]);
  hipLaunchKernelGGL(k_rebuild, dim3((unsigned)((d.fcap + 255) / 256)), dim3(256), 0, s, d, R, M, l03, L[4], nl,
                     m_listed, now);
}
