// Replica placement kernels (SPEC.md §6): the master's Init_replica /
// Handle_put_request / Update_metadata (master/master.go:74-175) for a batch of
// files at once, one lane per file, Philox draws keyed by (seed; file, draw).
// The master's list (and, for repair, the observer's) arrives as gathered
// presence bitmaps in rbits (q = 0 master, q = 1 observer), the same on every
// shard. The file table is sharded by file ID (gh_fslot: file f on shard
// f % G): each shard places, repairs and looks up only its own files, and the
// lanes of other shards' files write INT32_MIN, so one allreduce(max) of the
// outputs gives every shard the batch's results.
#include "gh_internal.h"

namespace {

// Member_list = present members of the master row, ID order
// (master/master.go:46, slave/slave.go:478). One 1024-thread workgroup.
__global__ __launch_bounds__(1024) void k_candidates(GhDev d, int32_t nr) {
  __shared__ int s_sum[1024];
  const int tid = threadIdx.x;
  const int per = (d.n + 1023) / 1024;
  const int b = min(d.n, tid * per), e = min(d.n, b + per);
  int cnt = 0;
  for (int c = b; c < e; ++c) cnt += gh_gbit(d, d.rbits, nr, 0, c);
  s_sum[tid] = cnt;
  __syncthreads();
  for (int off = 1; off < 1024; off <<= 1) {
    const int v = tid >= off ? s_sum[tid - off] : 0;
    __syncthreads();
    s_sum[tid] += v;
    __syncthreads();
  }
  int pos = tid ? s_sum[tid - 1] : 0;
  for (int c = b; c < e; ++c)
    if (gh_gbit(d, d.rbits, nr, 0, c)) d.cand[pos++] = c;
  if (tid == 1023) d.ncand[0] = s_sum[1023];
}

// Init_replica (master/master.go:129-150). nodes[0..len) are kept first; the
// reference's time-seeded Intn(M-1) becomes Philox word 0 of block
// (f, draw, PLACE, 0) mapped by multiply-shift, so cand[M-1] is never drawn.
__device__ int init_replica(const GhDev& d, int32_t nr, int32_t f, int64_t fl, int32_t* nodes, int& len, int R,
                            uint64_t seed) {
  if (len >= R) return GH_OK;
  const int M = d.ncand[0];
  if (M <= 1) return GH_EPLACEMENT_STARVED;  // Intn(<=0) panics
  const int32_t last = d.cand[M - 1];
  int in_pool = 0;
  for (int x = 0; x < len; ++x) {
    const int32_t a = nodes[x];
    in_pool += (a >= 0 && a < d.n && a < last && gh_gbit(d, d.rbits, nr, 0, a));
  }
  if ((M - 1) - in_pool < R - len) return GH_EPLACEMENT_STARVED;  // infinite loop
  uint32_t dr = d.draws[fl];
  uint32_t budget = GH_MAX_DRAWS;
  int l = len;
  int32_t tmp[8];
  for (int x = 0; x < 8; ++x) tmp[x] = x < l ? nodes[x] : -1;
  while (l < R) {
    if (budget-- == 0) return GH_EPLACEMENT_STARVED;
    const uint32_t u = gh_philox_word(seed, (uint32_t)f, dr, GH_TAG_PLACE, 0, 0);
    dr++;
    const uint32_t num = (uint32_t)(((uint64_t)u * (uint64_t)(M - 1)) >> 32);
    const int32_t a = d.cand[num];
    bool dup = false;
    for (int x = 0; x < l; ++x) dup |= tmp[x] == a;  // isAddressExist (:137)
    if (!dup) tmp[l++] = a;
  }
  d.draws[fl] = dr;
  for (int x = 0; x < l; ++x) nodes[x] = tmp[x];
  len = l;
  return GH_OK;
}

// put (Handle_put_request, :152-175) for io_a[0..n): out io_b replicas,
// io_c versions, io_d status.
__global__ __launch_bounds__(256) void k_put(GhDev d, int32_t nr, int64_t n, int32_t R, int32_t now,
                                             uint64_t seed) {
  const int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (x >= n) return;
  const int32_t f = d.io_a[x];
  const int64_t fl = gh_fslot(d, f);
  if (fl < 0) {  // another shard's file
    for (int q = 0; q < R; ++q) d.io_b[x * R + q] = INT_MIN;
    d.io_c[x] = d.io_d[x] = INT_MIN;
    return;
  }
  int32_t* rp = d.rep + fl * R;
  int32_t nodes[8];
  if (d.ver[fl] < 0) {  // Update_timestamp: new File_info (:239-245)
    d.ver[fl] = 0;
    for (int q = 0; q < R; ++q) rp[q] = -1;
  }
  d.fts[fl] = now;
  int len = 0;
  for (int q = 0; q < R; ++q) {
    nodes[q] = rp[q];
    len += rp[q] >= 0;
  }
  const int st = init_replica(d, nr, f, fl, nodes, len, R, seed);
  if (st == GH_OK) {
    for (int q = 0; q < R; ++q) rp[q] = q < len ? nodes[q] : -1;
    d.ver[fl] += 1;  // :159
  }
  for (int q = 0; q < R; ++q) d.io_b[x * R + q] = rp[q];
  d.io_c[x] = d.ver[fl];
  d.io_d[x] = st;
}

// Update_metadata (:74-127) with available = the observer row's present set
// (rbits q = 1).
// One lane per local slot (file fl * G + rank).
__global__ __launch_bounds__(256) void k_repair(GhDev d, int32_t nr, int32_t R, uint64_t seed) {
  const int64_t fl = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (fl >= d.fcap || d.ver[fl] < 0) return;
  const int64_t f = fl * d.fsh + d.frank;
  int32_t* rp = d.rep + fl * R;
  int32_t working[8];
  int wl = 0;
  for (int q = 0; q < R; ++q) {
    const int32_t a = rp[q];
    if (a >= 0 && a < d.n && gh_gbit(d, d.rbits, nr, 1, a)) working[wl++] = a;  // :93-99
  }
  if (wl >= R) return;  // :104
  int32_t nodes[8];
  for (int q = 0; q < 8; ++q) nodes[q] = q < wl ? working[q] : -1;
  int len = wl;
  const int st = init_replica(d, nr, (int32_t)f, fl, nodes, len, R, seed);  // :106-107
  for (int q = 0; q < R; ++q) rp[q] = q < len ? nodes[q] : -1;
  const int slot = atomicAdd(d.nplan, 1);
  gh_plan_entry e;
  e.file = (int32_t)f;
  e.node1 = wl > 0 ? working[0] : -1;  // :120 (SPEC D5)
  e.version = d.ver[fl];
  e.status = st;
  int nn = 0;
  for (int q = wl; q < len; ++q) e.new_nodes[nn++] = nodes[q];  // :110-115
  for (int q = nn; q < 8; ++q) e.new_nodes[q] = -1;
  e.n_new = nn;
  d.plan[slot] = e;
}

// get/ls (:177-212) and delete (:249-259) for io_a[0..n) -> io_b, io_c.
__global__ __launch_bounds__(256) void k_get(GhDev d, int64_t n, int32_t R, int del) {
  const int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (x >= n) return;
  const int64_t fl = gh_fslot(d, d.io_a[x]);
  if (fl < 0) {  // another shard's file
    for (int q = 0; q < R; ++q) d.io_b[x * R + q] = INT_MIN;
    d.io_c[x] = INT_MIN;
    return;
  }
  const bool has = d.ver[fl] >= 0;
  int32_t* rp = d.rep + fl * R;
  for (int q = 0; q < R; ++q) {
    d.io_b[x * R + q] = has ? rp[q] : -1;
    if (del) rp[q] = -1;
  }
  d.io_c[x] = d.ver[fl];
  if (del) d.ver[fl] = -1;
}

// If_file_updated_recent (:214-229) for io_a[0..n) -> io_d (0/1).
__global__ __launch_bounds__(256) void k_conflicts(GhDev d, int64_t n, int32_t now, int32_t window) {
  const int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (x >= n) return;
  const int64_t fl = gh_fslot(d, d.io_a[x]);
  d.io_d[x] = fl < 0 ? INT_MIN : (d.ver[fl] >= 0 && (int64_t)now - d.fts[fl] < window);
}

}  // namespace

void launch_conflicts(const GhDev& d, int64_t n, int32_t now, int32_t window, hipStream_t s) {
  hipLaunchKernelGGL(k_conflicts, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, d, n, now, window);
}

void launch_candidates(const GhDev& d, int32_t nr, hipStream_t s) {
  hipLaunchKernelGGL(k_candidates, dim3(1), dim3(1024), 0, s, d, nr);
}

void launch_put(const GhDev& d, int32_t nr, int64_t n, int32_t R, int32_t now, uint64_t seed, hipStream_t s) {
  hipLaunchKernelGGL(k_put, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, d, nr, n, R, now, seed);
}

void launch_repair(const GhDev& d, int32_t nr, int32_t R, uint64_t seed, hipStream_t s) {
  hipLaunchKernelGGL(k_repair, dim3((unsigned)((d.fcap + 255) / 256)), dim3(256), 0, s, d, nr, R, seed);
}

void launch_get(const GhDev& d, int64_t n, int32_t R, int del, hipStream_t s) {
  hipLaunchKernelGGL(k_get, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, d, n, R, del);
}
