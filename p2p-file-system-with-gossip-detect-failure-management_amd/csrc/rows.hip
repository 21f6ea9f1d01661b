// Row layout (GH_LAYOUT_ROWS, north_star; DESIGN.md "Multi-GPU"): the ghost
// rows a shard's receivers pull. Before a round, each owner packs the rows
// other shards asked for (their senders this round) into per-destination
// blocks and alltoallv moves them (comm.h: ncclAllToAllv) straight into the
// receivers' ghost tables (gh_internal.h gcodes / gplane, row-major, ghost j
// = slot nrows + j), so k_round / k_round_slow read a sender by its slot.
// Two parts travel separately: a ghost's sender plane (0.5 B per cell, all
// a healthy round's k_round reads) and its 16-bit codes (2 B per cell, for
// storm rounds and for the segments k_round leaves to k_round_slow). The
// replaced reference step is the UDP list push between hosts,
// slave/slave.go:527-542.
//   k_ghost_pack    rows to send -> back-to-back plane words or codes;
//                   the codes part counts the wide segments per destination
//   k_ghost_wide    the exact cells of those wide segments (rare)
//   k_ghost_unwide  received wide segments -> fresh arena slots of the
//                   current buffer, the ghost rows' marker chunks rewritten
#include "gh_internal.h"

namespace {

// one thread per 8-cell chunk of a sent row; part GH_GX_PLANE: the row's
// plane words (ld / 2 bytes per row), GH_GX_CODES: its narrow codes (ld * 2
// bytes per row), counting its wide segments in wcnt[dest[e]]
__global__ __launch_bounds__(256) void k_ghost_pack(GhDev d, int cur, const int32_t* rows, const int32_t* dest,
                                                    int64_t ns, int part, char* out, int32_t* wcnt) {
  const int64_t cpr = d.ld >> 3;
  const int64_t total = ns * cpr;
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    const int64_t e = idx / cpr, k = idx - e * cpr, c = k * 8;
    const int64_t cell = gh_cell(d, rows[e], c);
    if (part == GH_GX_PLANE) {
      reinterpret_cast<uint32_t*>(out)[e * cpr + k] = d.pl[cur][cell >> 3];
    } else {
      const uint4 x = gh_ld16(d, cur, rows[e], c);  // (a tier chunk's codes decoded)
      *reinterpret_cast<uint4*>(out + (e * d.ld + c) * 2) = x;
      if ((c & (d.tw - 1)) == 0 && (x.x & 0xFFFFu) == GH_N_WIDE) atomicAdd(&wcnt[dest[e]], 1);
    }
  }
}

// part GH_GX_PLANE with tiles of >= 32 members: one thread per 32 cells
// (16 B of plane words, 8 lanes per 128-B tile segment); the 4-B-per-thread
// form of k_ghost_pack moved a shard's 737 MB at ~1.1 TB/s
__global__ __launch_bounds__(256) void k_ghost_pack_plane(GhDev d, int cur, const int32_t* rows, int64_t ns,
                                                          char* out) {
  const int64_t qpr = d.ld >> 5;  // 16-B groups per row
  const int64_t total = ns * qpr;
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    const int64_t e = idx / qpr, k = idx - e * qpr;
    const int64_t cell = gh_cell(d, rows[e], k * 32);
    reinterpret_cast<uint4*>(out)[idx] = *reinterpret_cast<const uint4*>(d.pl[cur] + (cell >> 3));
  }
}

// same-device in-process shards: ghost j's plane row straight from its
// owner's table (tiles of >= 32 members, 16 B per thread as above)
__global__ __launch_bounds__(256) void k_ghost_gather_plane(GhDev d, GxPeers pp, const int32_t* ghosts, int64_t ng,
                                                            int64_t nrs) {
  const int64_t qpr = d.ld >> 5;
  const int64_t total = ng * qpr;
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    const int64_t j = idx / qpr, c = (idx - j * qpr) * 32;
    const int64_t s = ghosts[j];
    const int h = (int)(s / nrs);
    const int64_t cell = (c >> d.lgtw) * pp.tstride[h] + ((s - pp.row0[h]) << d.lgtw) + (c & (d.tw - 1));
    reinterpret_cast<uint4*>(d.gplane)[idx] = *reinterpret_cast<const uint4*>(pp.pl[h] + (cell >> 3));
  }
}

// a wide record: (row, tile), the segment's TW exact heartbeats, its flag
// bytes (a sender's ts is never read)
__host__ __device__ inline int64_t ghost_wide_bytes(int tw) { return ((8 + 4 * (int64_t)tw + tw / 8) + 15) / 16 * 16; }

// one thread per (sent row, tile); wcur[r] = the next record slot for
// destination r (starts at the destination's first record)
__global__ __launch_bounds__(256) void k_ghost_wide(GhDev d, int cur, const int32_t* rows, const int32_t* dest,
                                                    int64_t ns, int32_t* wcur, char* out) {
  const int64_t total = ns * d.ntiles;
  const int64_t rec = ghost_wide_bytes(d.tw);
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    const int64_t e = idx / d.ntiles, t = idx - e * d.ntiles;
    const int32_t s = rows[e];
    const uint4 h = gh_ld16(d, cur, s, t * d.tw);  // (a tier chunk is never wide)
    if ((h.x & 0xFFFFu) != GH_N_WIDE) continue;
    const int64_t slot = gh_wide_slot(h.x, h.y);
    char* o = out + (int64_t)atomicAdd(&wcur[dest[e]], 1) * rec;
    reinterpret_cast<int32_t*>(o)[0] = s;
    reinterpret_cast<int32_t*>(o)[1] = (int32_t)t;
    int32_t* xs = reinterpret_cast<int32_t*>(o + 8);
    uint8_t* fs = reinterpret_cast<uint8_t*>(o + 8 + 4 * (int64_t)d.tw);
    const bool ok = slot < d.wcap;  // a corrupt marker reads as absent cells
    for (int j = 0; j < d.tw; ++j) xs[j] = ok ? d.wh[cur][slot * d.tw + j] : GH_ABSENT;
    for (int j = 0; j < d.tw / 8; ++j) fs[j] = ok ? d.wf[cur][(slot * d.tw >> 3) + j] : 0;
  }
}

// one thread per received wide record: the ghost row's segment gets a fresh
// arena slot of buffer cur (the round reads ghosts with cur's arena)
__global__ __launch_bounds__(256) void k_ghost_unwide(GhDev d, int cur, const char* in, int64_t nrec) {
  const int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (x >= nrec) return;
  const char* o = in + x * ghost_wide_bytes(d.tw);
  const int32_t s = reinterpret_cast<const int32_t*>(o)[0];
  const int64_t t = reinterpret_cast<const int32_t*>(o)[1];
  const int32_t* xs = reinterpret_cast<const int32_t*>(o + 8);
  const uint8_t* fs = reinterpret_cast<const uint8_t*>(o + 8 + 4 * (int64_t)d.tw);
  const int64_t g = (int64_t)d.rslot[s] - d.nrows;  // its ghost row
  if (g < 0 || g >= d.gcap) return;
  const int64_t a = gh_wide_alloc(d, cur);
  if (a < 0) return;  // arena full: the state is lost (d.err)
  for (int j = 0; j < d.tw; ++j) {
    d.wh[cur][a * d.tw + j] = xs[j];
    d.wt[cur][a * d.tw + j] = 0;
  }
  for (int j = 0; j < d.tw / 8; ++j) d.wf[cur][(a * d.tw >> 3) + j] = fs[j];
  const uint4 m = gh_wide_chunk(a);
  for (int j = 0; j < d.tw; j += 8) *reinterpret_cast<uint4*>(d.gcodes + g * d.ld + t * d.tw + j) = m;
}

// ---- the round's want lists on the device --------------------------------
// Every shard holds every receiver's inbox (replicated), so every shard
// computes every shard's wants alike: want[r] = the senders, owned by
// another shard, of the receivers shard r owns, ascending. wbits: [G][nw]
// bitmaps; wlist: [G][n] the compacted lists; mcnt: [G][G] counts, M[r][o] =
// the rows of owner o in want[r] (the exchange's send and receive sizes).
__global__ __launch_bounds__(256) void k_want_mark(GhDev d, GhRound p, int64_t nrs, uint32_t* wbits, int64_t nw) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= p.n) return;
  const bool pull = p.peer_mode == GH_PEER_PULL;
  const int64_t r = i / nrs;
  const int cnt = gh_in_cnt(d, pull, p.k, i);
  const int64_t beg = gh_in_beg(d, pull, p.k, i);
  for (int q = 0; q < cnt; ++q) {
    const int64_t s = d.inbox[beg + q];
    if (s / nrs != r) atomicOr(&wbits[r * nw + (s >> 5)], 1u << (s & 31));
  }
}

// per (rank, 256-word block): the block's set bits (wsum[r][b])
__global__ __launch_bounds__(256) void k_want_sum(const uint32_t* wbits, int64_t nw, int32_t* wsum, int64_t nb) {
  const int64_t r = blockIdx.y, b = blockIdx.x;
  const int64_t w = b * 256 + threadIdx.x;
  int tot = w < nw ? __popc(wbits[r * nw + w]) : 0;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) tot += __shfl_xor(tot, o);
  __shared__ int s_w[4];
  if ((threadIdx.x & 63) == 0) s_w[threadIdx.x >> 6] = tot;
  __syncthreads();
  if (threadIdx.x == 0) wsum[r * nb + b] = s_w[0] + s_w[1] + s_w[2] + s_w[3];
}

// per rank: exclusive prefix of its block sums (one thread per rank; nb is small)
__global__ void k_want_scan(int32_t* wsum, int64_t nb, int G, int32_t* wtot) {
  const int r = threadIdx.x;
  if (r >= G) return;
  int acc = 0;
  for (int64_t b = 0; b < nb; ++b) {
    const int v = wsum[r * nb + b];
    wsum[r * nb + b] = acc;
    acc += v;
  }
  wtot[r] = acc;
}

// compaction: the set bits of each block in ascending order at the block's
// offset; M[r][owner] counted per block in LDS
__global__ __launch_bounds__(256) void k_want_fill(const uint32_t* wbits, int64_t nw, const int32_t* wsum, int64_t nb,
                                                   int64_t n, int64_t nrs, int G, int32_t* wlist, int32_t* mcnt) {
  const int64_t r = blockIdx.y, b = blockIdx.x;
  const int64_t w = b * 256 + threadIdx.x;
  const uint32_t x = w < nw ? wbits[r * nw + w] : 0u;
  __shared__ int s_w[4], s_m[64];
  const int c = __popc(x);
  // exclusive prefix of c over the block
  int incl = c;
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(incl, o);
    if (lane >= o) incl += y;
  }
  if (lane == 63) s_w[threadIdx.x >> 6] = incl;
  if (threadIdx.x < 64) s_m[threadIdx.x] = 0;
  __syncthreads();
  int base = wsum[r * nb + b] + incl - c;
  for (int q = 0; q < (int)(threadIdx.x >> 6); ++q) base += s_w[q];
  for (uint32_t m = x; m; m &= m - 1) {
    const int64_t s = w * 32 + __builtin_ctz(m);
    wlist[r * n + base++] = (int32_t)s;
    atomicAdd(&s_m[s / nrs], 1);
  }
  __syncthreads();
  if (threadIdx.x < G && s_m[threadIdx.x]) atomicAdd(&mcnt[r * G + threadIdx.x], s_m[threadIdx.x]);
}

// this shard's ghost slots: every row it does not own unmapped, ghost j
// (want[me][j]) at slot nrows + j
__global__ __launch_bounds__(256) void k_ghost_slots(GhDev d) {
  const int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (x < d.n && !gh_owned(d, x)) d.rslot[x] = -1;
}
__global__ __launch_bounds__(256) void k_ghost_slots_set(GhDev d, const int32_t* mine, const int32_t* cnt) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j < *cnt) d.rslot[mine[j]] = (int32_t)(d.nrows + j);
}

// rows (and destinations) of one exchange chunk: for each destination r the
// slice [lo_r, hi_r) of this shard's send list to r, back to back
__global__ __launch_bounds__(256) void k_gx_idx(const int32_t* wlist, int64_t n, GxSlices sl, int32_t* rows,
                                                int32_t* dest) {
  const int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (x >= sl.total) return;
  int r = 0;
  while (r + 1 < sl.g && sl.out[r + 1] <= x) ++r;
  rows[x] = wlist[(int64_t)r * n + sl.src[r] + (x - sl.out[r])];
  dest[x] = r;
}

unsigned ghost_grid(int64_t work) {
  return (unsigned)std::max<int64_t>(1, std::min<int64_t>((work + 255) / 256, 65536));
}

}  // namespace

namespace {
__global__ __launch_bounds__(256) void k_sole_vals(GhDev d, int cur, int dcur, GhRound p) {
  const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= d.ld) return;
  int32_t v = -1;
  if (d.det_cnt[dcur][c] == 1) {
    const int64_t j = d.det_min[dcur][c];
    if (gh_owned(d, j) && d.alive[j]) {
      const GhCell X = gh_get(d, cur, j, c, p.r);
      if (X.x >= 0 && !X.f) v = X.x + ((d.col0 + c) == j);
    }
  }
  d.soleval[c] = v;
}
}  // namespace

void launch_sole_vals(const GhDev& d, int cur, int dcur, const GhRound& p, hipStream_t s) {
  hipLaunchKernelGGL(k_sole_vals, dim3((unsigned)((d.ld + 255) / 256)), dim3(256), 0, s, d, cur, dcur, p);
}

void launch_ghost_gather_plane(const GhDev& d, const GxPeers& pp, const int32_t* ghosts, int64_t ng, int64_t nrs,
                               hipStream_t s) {
  if (ng > 0)
    hipLaunchKernelGGL(k_ghost_gather_plane, dim3(ghost_grid(ng * (d.ld >> 5))), dim3(256), 0, s, d, pp, ghosts, ng,
                       nrs);
}

int64_t ghost_part_bytes(const GhDev& d, int part) { return part == GH_GX_PLANE ? d.ld / 2 : d.ld * 2; }
int64_t ghost_wide_record_bytes(const GhDev& d) { return ghost_wide_bytes(d.tw); }

void launch_ghost_pack(const GhDev& d, int cur, const int32_t* rows, const int32_t* dest, int64_t ns, int part,
                       char* out, int32_t* wcnt, hipStream_t s) {
  if (ns == 0) return;
  if (part == GH_GX_PLANE && d.tw >= 32 && d.ld % 32 == 0) {
    hipLaunchKernelGGL(k_ghost_pack_plane, dim3(ghost_grid(ns * (d.ld >> 5))), dim3(256), 0, s, d, cur, rows, ns, out);
    return;
  }
  hipLaunchKernelGGL(k_ghost_pack, dim3(ghost_grid(ns * (d.ld >> 3))), dim3(256), 0, s, d, cur, rows, dest, ns, part,
                     out, wcnt);
}

void launch_ghost_wide(const GhDev& d, int cur, const int32_t* rows, const int32_t* dest, int64_t ns, int32_t* wcur,
                       char* out, hipStream_t s) {
  if (ns == 0) return;
  hipLaunchKernelGGL(k_ghost_wide, dim3(ghost_grid(ns * d.ntiles)), dim3(256), 0, s, d, cur, rows, dest, ns, wcur,
                     out);
}

void launch_want_lists(const GhDev& d, const GhRound& p, int64_t nrs, int G, uint32_t* wbits, int32_t* wsum,
                       int32_t* wlist, int32_t* mcnt, hipStream_t s) {
  const int64_t nw = ((int64_t)p.n + 31) / 32, nb = (nw + 255) / 256;
  (void)hipMemsetAsync(wbits, 0, sizeof(uint32_t) * G * nw, s);
  (void)hipMemsetAsync(mcnt, 0, sizeof(int32_t) * (G * G + G), s);
  hipLaunchKernelGGL(k_want_mark, dim3((unsigned)((p.n + 255) / 256)), dim3(256), 0, s, d, p, nrs, wbits, nw);
  hipLaunchKernelGGL(k_want_sum, dim3((unsigned)nb, (unsigned)G), dim3(256), 0, s, wbits, nw, wsum, nb);
  hipLaunchKernelGGL(k_want_scan, dim3(1), dim3(64), 0, s, wsum, nb, G, mcnt + G * G);
  hipLaunchKernelGGL(k_want_fill, dim3((unsigned)nb, (unsigned)G), dim3(256), 0, s, wbits, nw, wsum, nb, (int64_t)p.n,
                     nrs, G, wlist, mcnt);
}

void launch_ghost_slots(const GhDev& d, const int32_t* mine, const int32_t* cnt, hipStream_t s) {
  hipLaunchKernelGGL(k_ghost_slots, dim3((unsigned)((d.n + 255) / 256)), dim3(256), 0, s, d);
  hipLaunchKernelGGL(k_ghost_slots_set, dim3((unsigned)((d.n + 255) / 256)), dim3(256), 0, s, d, mine, cnt);
}

void launch_gx_idx(const int32_t* wlist, int64_t n, const GxSlices& sl, int32_t* rows, int32_t* dest, hipStream_t s) {
  if (sl.total == 0) return;
  hipLaunchKernelGGL(k_gx_idx, dim3((unsigned)((sl.total + 255) / 256)), dim3(256), 0, s, wlist, n, sl, rows, dest);
}

void launch_ghost_unwide(const GhDev& d, int cur, const char* in, int64_t nrec, hipStream_t s) {
  if (nrec == 0) return;
  hipLaunchKernelGGL(k_ghost_unwide, dim3((unsigned)((nrec + 255) / 256)), dim3(256), 0, s, d, cur, in, nrec);
}
