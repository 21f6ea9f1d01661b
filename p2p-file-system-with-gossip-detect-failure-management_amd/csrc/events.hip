// Churn and state-maintenance kernels (SPEC.md §5, §3). All tables use the
// tiled layout of gh_internal.h (gh_cell) over the shard's local columns.
//   k_count        local present count per row (after events / import)
//   k_fill         synthetic full-membership start (BASELINE configs 2-4)
//   k_pack/unpack  host (hb, ts) rows <-> encoded tiled local columns
//                  (import/export/lsm; gh_internal.h "cell encoding")
//   k_freeze       exact cells of rows that stop (crash / leave) into the
//                  frozen store
//   k_hb_check     the int32 heartbeat bound (slave/slave.go:446, Go int)
//   k_rowbits      presence bitmap of some rows over the local columns (the
//                  rows' lists, gathered across shards by the host)
//   k_leave        LEAVE delivery: slave/slave.go:310-336 -> :232-235
//   k_join_*       JOIN at the introducer and its full-list broadcast:
//                  slave/slave.go:224-231, 250-274
#include <algorithm>

#include "gh_internal.h"

namespace {

constexpr unsigned kMaxGrid = 65536;

// One wave per row: each lane reads 8 consecutive members (gh_pf8), the wave
// 512 members per step.
__global__ __launch_bounds__(256) void k_count(GhDev d, int cur, GhRound p) {
  const int i = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (i >= p.n) return;
  int cnt = 0;
  if (gh_owned(d, i))  // row layout: other shards count their rows, this one adds 0
    for (int64_t c = lane * 8; c < p.ld; c += 512) cnt += __builtin_popcount(gh_pf8(d, cur, i, c) & 0xFFu);
  for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o);
  if (lane == 0) d.cntl[i] = cnt;
}

// Cell of an external (hb, ts) for member cg of row i, in a buffer for round r.
__device__ __forceinline__ GhCell external(int32_t x, int32_t t, int64_t cg, int64_t i, const GhRound& p) {
  if (x == GH_ABSENT) return gh_absent();
  if (x < 0) return GhCell{GH_TOMBSTONE, t, false};
  return GhCell{x, t, gh_flag_for(x, t, cg, i, p.r, p.t_fail)};
}

__device__ __forceinline__ bool same(const GhCell& a, const GhCell& b) {
  return a.x == b.x && (a.x == GH_ABSENT || a.ts == b.ts) && (a.x < 0 || a.f == b.f);
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

// Read-modify-write of whole segments of buffer buf (for round p.r), in
// k_round's lane shape: a lane owns one 8-cell chunk, SEG = TW/8 lanes a
// segment. op(i, c, v) returns the new cell (i, local c). A segment that
// changed (every segment when `force`: rows that start running again must
// lose their GH_N_FROZEN marks) is stored narrow when every cell has a
// narrow code, else wide (its old arena slot when it was wide, a fresh one
// otherwise). Nothing else in the launch reads the segments it writes.
template <int TW, class Op>
__global__ __launch_bounds__(256) void k_seg(GhDev d, int buf, SegSet set, const int32_t* gate, GhRound p, bool force,
                                             Op op) {
  if (gate && *gate == 0) return;
  constexpr int SEG = TW / 8;
  constexpr int RPW = 64 / SEG;
  const int lane = threadIdx.x & 63;
  const int sub = lane / SEG, lc = lane % SEG;
  const unsigned long long gmask = (SEG == 64 ? ~0ull : ((1ull << SEG) - 1)) << (sub * SEG);
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
  const int64_t total = set.count();
  // the ops' counters, summed per wave and added once (one global atomic
  // per cell serialised a 1% LEAVE wave's 43 M tombstones: 0.5 s)
  uint32_t tal[2] = {0u, 0u};
  for (int64_t s0 = wave * RPW; s0 < total; s0 += nw * RPW) {
    const int64_t sid = s0 + sub;
    const bool valid = sid < total;
    int64_t i = 0, t = 0;
    if (valid) set.at(sid, i, t);
    const int64_t c = t * TW + lc * 8;
    bool changed = force, fit = true;
    int dpres = 0;  // present after - present before, this lane's cells
    GhCell v[8];
    uint4 x = {0u, 0u, 0u, 0u}, nx = {0u, 0u, 0u, 0u};
    if (valid) {
      x = gh_ld16(d, buf, i, c);
      gh_dec8(d, buf, i, c, p.r, x, v);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const GhCell y = op(i, c + j, v[j], tal);
        changed |= !same(y, v[j]);
        dpres += (y.x >= 0) - (v[j].x >= 0);
        v[j] = y;
      }
      nx = gh_enc8(d, buf, c, p.r, v, fit);
    }
    const bool any = (__ballot(changed) & gmask) != 0;
    const bool narrow = (__ballot(valid && !fit) & gmask) == 0;
    // the row's present count follows the segment (no full recount after
    // events: k_count reads the whole table, 2.3 ms at N=65,536)
    if (__ballot(dpres != 0) != 0) {
#pragma unroll
      for (int o = SEG / 2; o > 0; o >>= 1) dpres += __shfl_xor(dpres, o);
      if (valid && lc == 0 && dpres != 0) atomicAdd(&d.cntl[i], dpres);
    }
    if (!valid || !any) continue;
    int64_t slot = 0;
    if (!narrow) {
      // a wide segment keeps its slot (every chunk holds it); else a new one
      if ((x.x & 0xFFFFu) == GH_N_WIDE) {
        slot = gh_wide_slot(x.x, x.y);
      } else {
        int64_t s = lc == 0 ? gh_wide_alloc(d, buf) : 0;
        slot = __shfl(s, sub * SEG);
      }
    }
    if (slot < 0) continue;  // arena full: the state is lost (d.err)
    gh_put8(d, buf, i, c, narrow, nx, slot, v);
  }
  if constexpr (Op::kTally) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      tal[0] += __shfl_xor(tal[0], o);
      tal[1] += __shfl_xor(tal[1], o);
    }
    if (lane == 0 && (tal[0] | tal[1])) op.flush(tal);
  }
}

struct OpFill {
  static constexpr bool kTally = false;
  GhDev d;
  int32_t hb0, ts0;
  GhRound p;
  __device__ GhCell operator()(int64_t i, int64_t c, const GhCell&, uint32_t*) const {
    if (c >= d.ncol) return gh_absent();
    return external(hb0, ts0, d.col0 + c, i, p);
  }
};

struct OpPack {
  static constexpr bool kTally = false;
  GhDev d;
  const int32_t *hb_rows, *ts_rows;
  int64_t row0;
  GhRound p;
  __device__ GhCell operator()(int64_t i, int64_t c, const GhCell& v, uint32_t*) const {
    if (c >= d.ncol) return v;
    const int64_t src = (i - row0) * d.n + d.col0 + c;
    return external(hb_rows[src], ts_rows[src], d.col0 + c, i, p);
  }
};

// Fresh joiner processes start with an empty MemberList (SPEC D7).
struct OpReset {
  static constexpr bool kTally = false;
  __device__ GhCell operator()(int64_t, int64_t, const GhCell&, uint32_t*) const { return gh_absent(); }
};

// LEAVE from each leaver c to every alive member j of c's list (j != c):
// removeMember(c) at j. colq[c] = the leaver's index q in the gathered
// bitmaps rbits [world][nl][ncsw] (-1: not a leaver).
struct OpLeave {
  static constexpr bool kTally = true;  // tombstoned, unknown
  GhDev d;
  int32_t nl;
  int32_t shadow_row;  // GhRound.shadow_row
  __device__ GhCell operator()(int64_t j, int64_t c, const GhCell& v, uint32_t* t) const {
    const int q = d.colq[c];
    if (q < 0 || !d.alive[j] || d.col0 + c == j || !gh_gbit(d, d.rbits, nl, q, j)) return v;
    if (v.x >= 0 && j == shadow_row && d.shadow[c] != GH_NO_SHADOW) {
      // the introducer holds c in RecentFailList too (D7): that entry, its
      // ts, is the tombstone; nothing is appended (:278-281)
      const int32_t ts = d.shadow[c];
      d.shadow[c] = GH_NO_SHADOW;
      atomicSub(d.nshadow, 1);
      return GhCell{GH_TOMBSTONE, ts, false};
    }
    if (v.x >= 0) {
      t[0]++;
      return GhCell{GH_TOMBSTONE, v.ts, false};  // keeps its ts (slave/slave.go:280)
    }
    if (v.x == GH_ABSENT) t[1]++;
    return v;
  }
  __device__ void flush(const uint32_t* t) const {
    if (t[0]) atomicAdd(&d.stats[ST_TOMBSTONED], (unsigned long long)t[0]);
    if (t[1]) atomicAdd(&d.stats[ST_REMOVE_UNKNOWN], (unsigned long long)t[1]);
  }
};

// addNewMember at the introducer (slave/slave.go:250-255) for the joiners
// whose column is local (colq[c] >= 0). nd[4] counts this shard's adds.
struct OpJoinAdd {
  static constexpr bool kTally = true;  // adds
  GhDev d;
  GhRound p;
  __device__ GhCell operator()(int64_t, int64_t c, const GhCell& v, uint32_t* t) const {
    if (d.colq[c] < 0 || v.x >= 0) return v;
    t[0]++;
    if (v.x == GH_TOMBSTONE) {  // MemberInList reads MemberList only: the tombstone stays beside it (D7)
      d.shadow[c] = v.ts;
      atomicAdd(d.nshadow, 1);
    }
    return GhCell{0, p.r, false};  // hb 0, ts = now
  }
  __device__ void flush(const uint32_t* t) const { atomicAdd(&d.nd[4], (int)t[0]); }
};

// The introducer's full list to every alive member of it (:256-272), merged
// with MergeMemberList's rule at now = r. nd[4] = adds over all shards;
// rbits row 0 = the introducer's list after the adds.
struct OpJoinBcast {
  GhDev d;
  int cur;
  int32_t I;
  GhRound p;
  static constexpr bool kTally = true;  // merges
  __device__ void flush(const uint32_t* t) const { atomicAdd(&d.stats[ST_MERGED], (unsigned long long)t[0]); }
  __device__ GhCell operator()(int64_t j, int64_t c, const GhCell& v, uint32_t* t) const {
    if (c >= d.ncol || j == I || !d.alive[j] || !gh_gbit(d, d.rbits, 1, 0, j)) return v;
    const GhCell m = gh_get(d, cur, I, c, p.r);
    if (m.x < 0) return v;
    if (v.x >= GH_ABSENT && m.x > v.x) {
      t[0]++;
      return GhCell{m.x, p.r, gh_flag_for(m.x, p.r, d.col0 + c, j, p.r, p.t_fail)};  // ts = now
    }
    return v;
  }
};

// MergeMemberList of an external list into row obs at tick p.r - 1 (the last
// completed round). colq[c] = the listed heartbeat of local member c (< -2:
// not listed).
struct OpMergeList {
  GhDev d;
  GhRound p;
  static constexpr bool kTally = true;  // merges
  __device__ void flush(const uint32_t* t) const { atomicAdd(&d.nd[5], (int)t[0]); }
  __device__ GhCell operator()(int64_t obs, int64_t c, const GhCell& v, uint32_t* t) const {
    const int32_t m = d.colq[c];
    if (m < -2 || !(v.x >= GH_ABSENT && m > v.x)) return v;  // :424-426, :435-438; tombstones blocked (:432-434)
    t[0]++;
    return GhCell{m, p.r - 1, gh_flag_for(m, p.r - 1, d.col0 + c, obs, p.r, p.t_fail)};
  }
};

// q -> colq[local column of ids[q]] for the ids local to this shard
__global__ void k_scatter(GhDev d, const int32_t* ids, const int32_t* vals, int32_t n) {
  const int q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= n) return;
  const int64_t lc = (int64_t)ids[q] - d.col0;
  if (lc >= 0 && lc < d.ncol) d.colq[lc] = vals ? vals[q] : q;
}

// One chunk per thread: what = 0: external hb; what = 1: exported ts
// (gh_export_ts).
__global__ __launch_bounds__(256) void k_unpack(GhDev d, int cur, int32_t* dst, int64_t row0, int64_t nrows,
                                                int what, GhRound p) {
  const int64_t cpt = d.tw >> 3;  // chunks per segment
  const int64_t per_tile = nrows * cpt, total = per_tile * d.ntiles;
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    const int64_t t = idx / per_tile, rem = idx - t * per_tile;
    const int64_t i = row0 + rem / cpt;
    const int64_t c = t * d.tw + (rem % cpt) * 8;
    if (c >= d.ncs || !gh_owned(d, i)) continue;  // row layout: the owner writes the row
    GhCell v[8];
    gh_get8(d, cur, i, c, p.r, v);
    int32_t* o = dst + (i - row0) * d.ncs + c;
    const int lim = (int)min<int64_t>(8, d.ncs - c);
    for (int j = 0; j < lim; ++j) o[j] = what == 0 ? v[j].x : gh_export_ts(v[j], p.r, d.tsa);
  }
}

// A stopped row is frozen while the round counter moves on: its exact cells
// go to the frozen store (slot frow[i], set by the host), then both buffers
// mark the row GH_N_FROZEN (k_freeze_mark; the round never touches it).
__global__ __launch_bounds__(256) void k_freeze(GhDev d, int cur, const int32_t* rows, int32_t nr, GhRound p) {
  const int64_t cpr = d.ld >> 3;  // chunks per row
  const int64_t total = (int64_t)nr * cpr;
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = rows[idx / cpr], c = (idx % cpr) * 8;
    GhCell v[8];
    gh_get8(d, cur, i, c, p.r, v);
    const int64_t w = (int64_t)d.frow[i] * d.ld + c;
    *reinterpret_cast<int4*>(d.fzh + w) = int4{v[0].x, v[1].x, v[2].x, v[3].x};
    *reinterpret_cast<int4*>(d.fzh + w + 4) = int4{v[4].x, v[5].x, v[6].x, v[7].x};
    *reinterpret_cast<int4*>(d.fzt + w) = int4{v[0].ts, v[1].ts, v[2].ts, v[3].ts};
    *reinterpret_cast<int4*>(d.fzt + w + 4) = int4{v[4].ts, v[5].ts, v[6].ts, v[7].ts};
  }
}
__global__ __launch_bounds__(256) void k_freeze_mark(GhDev d, const int32_t* rows, int32_t nr) {
  const int64_t cpr = d.ld >> 3;
  const int64_t total = (int64_t)nr * cpr;
  const uint32_t m = GH_N_FROZEN | (GH_N_FROZEN << 16);
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    const int64_t off = gh_cell(d, rows[idx / cpr], (idx % cpr) * 8);
    *reinterpret_cast<uint4*>(d.hn[0] + off) = uint4{m, m, m, m};
    *reinterpret_cast<uint4*>(d.hn[1] + off) = uint4{m, m, m, m};
    if (d.a4[0]) {  // a stopped row's chunks are escaped in both tiers' buffers at all times
      d.a4[0][off >> 3] = GH_T4_ESC;
      d.a4[1][off >> 3] = GH_T4_ESC;
    }
    if (d.pl[0]) {  // never a sender: its plane words say unknown
      d.pl[0][off >> 3] = 0u;
      d.pl[1][off >> 3] = 0u;
    }
  }
}

// bit b of word w of row q = local column 32w+b of rows[q] is present
__global__ __launch_bounds__(256) void k_rowbits(GhDev d, int cur, const int32_t* rows, int32_t nr) {
  // row layout: slice 0 holds every member; the row's owner writes it, the
  // other shards write zeros (the host sums the slices)
  uint32_t* out = d.rbits + (d.rowlay ? 0 : (int64_t)d.rank * nr * d.ncsw);
  const int64_t total = (int64_t)nr * d.ncsw;
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    const int q = (int)(idx / d.ncsw);
    const int64_t w = idx - (int64_t)q * d.ncsw;
    const int row = rows[q];
    uint32_t bits = 0;
    for (int b = 0; b < 32 && gh_owned(d, row); b += 8) {
      const int64_t c = w * 32 + b;
      if (c >= d.ncol) break;
      bits |= (gh_pf8(d, cur, row, c) & 0xFFu) << b;  // padding cells are absent
    }
    out[idx] = bits;
  }
}

// segments of buffer buf: wide -> out[0], frozen -> out[1]
__global__ __launch_bounds__(256) void k_count_wide(GhDev d, int buf, unsigned long long* out) {
  const int64_t total = d.ntiles * d.nrows;  // owned rows: slots 0..nrows
  unsigned long long cw = 0, cf = 0;
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    const int64_t t = idx / d.nrows, i = idx - t * d.nrows;
    const uint32_t h = gh_ld16s(d, buf, i, t * d.tw, -1).x & 0xFFFFu;  // (a marker is never a tier chunk)
    cw += h == GH_N_WIDE;
    cf += h == GH_N_FROZEN;
  }
  for (int o = 32; o > 0; o >>= 1) {
    cw += __shfl_xor(cw, o);
    cf += __shfl_xor(cf, o);
  }
  if ((threadIdx.x & 63) == 0) {
    if (cw) atomicAdd(out, cw);
    if (cf) atomicAdd(out + 1, cf);
  }
}

// an alive row whose own heartbeat is INT32_MAX (its column is local)
__global__ __launch_bounds__(256) void k_hb_check(GhDev d, int cur, int32_t* flag, GhRound p) {
  const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= d.ncol) return;
  const int64_t i = d.col0 + c;
  // und: the rows that run the round (the host's scratch copy of alive
  // without this round's crashes and leaves)
  if (i < d.n && gh_owned(d, i) && d.und[i] && gh_get(d, cur, i, c, p.r).x == INT32_MAX) *flag = 1;
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
static void seg_launch(const GhDev& d, int buf, SegSet set, const int32_t* gate, const GhRound& p, Op op,
                       hipStream_t s, bool force = false) {
  const int64_t segs = set.nrows * set.ntl;
  if (segs == 0) return;
  const int64_t spw = 64 / (d.tw / 8);  // segments per wave
  const unsigned grid = grid_for((segs + spw - 1) / spw * 64);
#define GH_SEG_CASE(TW) \
  hipLaunchKernelGGL((k_seg<TW, Op>), dim3(grid), dim3(256), 0, s, d, buf, set, gate, p, force, op)
  switch (d.tw) {
    case 8: GH_SEG_CASE(8); break;
    case 16: GH_SEG_CASE(16); break;
    case 32: GH_SEG_CASE(32); break;
    case 128: GH_SEG_CASE(128); break;
    case 256: GH_SEG_CASE(256); break;
    default: GH_SEG_CASE(64); break;
  }
#undef GH_SEG_CASE
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
  seg_launch(d, cur, rows_set(d, nullptr, d.row0, d.nrows), nullptr, p, OpFill{d, hb0, ts0, p}, s, true);
}

void launch_pack(const GhDev& d, int cur, const int32_t* hb_rows, const int32_t* ts_rows, int64_t row0,
                 int64_t nrows, const GhRound& p, hipStream_t s) {
  // the owned rows of [row0, row0 + nrows)
  const int64_t a = std::max<int64_t>(row0, d.row0), b = std::min<int64_t>(row0 + nrows, d.row0 + d.nrows);
  if (b > a)
    seg_launch(d, cur, rows_set(d, nullptr, a, b - a), nullptr, p, OpPack{d, hb_rows, ts_rows, row0, p}, s, true);
}

void launch_unpack(const GhDev& d, int cur, int32_t* dst_rows, int64_t row0, int64_t nrows, int what,
                   const GhRound& p, hipStream_t s) {
  if (nrows == 0) return;
  hipLaunchKernelGGL(k_unpack, dim3(grid_for(nrows * d.ld / 8)), dim3(256), 0, s, d, cur, dst_rows, row0, nrows, what,
                     p);
}

void launch_freeze(const GhDev& d, int cur, const int32_t* rows, int32_t nr, const GhRound& p, hipStream_t s) {
  if (nr == 0) return;
  hipLaunchKernelGGL(k_freeze, dim3(grid_for((int64_t)nr * d.ld / 8)), dim3(256), 0, s, d, cur, rows, nr, p);
  hipLaunchKernelGGL(k_freeze_mark, dim3(grid_for((int64_t)nr * d.ld / 8)), dim3(256), 0, s, d, rows, nr);
}

void launch_count_wide(const GhDev& d, int buf, unsigned long long* out, hipStream_t s) {
  (void)hipMemsetAsync(out, 0, 2 * sizeof(unsigned long long), s);
  if (d.nrows > 0) hipLaunchKernelGGL(k_count_wide, dim3(grid_for(d.ntiles * d.nrows)), dim3(256), 0, s, d, buf, out);
}

void launch_rowbits(const GhDev& d, int cur, const int32_t* rows, int32_t nr, hipStream_t s) {
  if (nr == 0) return;
  hipLaunchKernelGGL(k_rowbits, dim3(grid_for((int64_t)nr * d.ncsw)), dim3(256), 0, s, d, cur, rows, nr);
}

void launch_leave(const GhDev& d, int cur, const int32_t* leavers, const int32_t* tiles, int32_t ntl, int32_t nl,
                  const GhRound& p, hipStream_t s) {
  if (ntl == 0) return;
  scatter(d, leavers, nullptr, nl, 0xFF, s);
  seg_launch(d, cur, SegSet{nullptr, d.row0, d.nrows, tiles, ntl}, nullptr, p, OpLeave{d, nl, p.shadow_row}, s);
}

void launch_join_add(const GhDev& d, int cur, const int32_t* joiners, int32_t nj, int32_t introducer,
                     const GhRound& p, hipStream_t s) {
  (void)hipMemsetAsync(d.nd + 4, 0, sizeof(int32_t), s);
  scatter(d, joiners, nullptr, nj, 0xFF, s);
  if (gh_owned(d, introducer)) seg_launch(d, cur, rows_set(d, nullptr, introducer, 1), nullptr, p, OpJoinAdd{d, p}, s);
}

void launch_join_bcast(const GhDev& d, int cur, int32_t introducer, const GhRound& p, hipStream_t s) {
  seg_launch(d, cur, rows_set(d, nullptr, d.row0, d.nrows), d.nd + 4, p, OpJoinBcast{d, cur, introducer, p}, s);
}

void launch_join_reset(const GhDev& d, int cur, const int32_t* rows, int32_t nr, const GhRound& p,
                       hipStream_t s) {
  seg_launch(d, cur, rows_set(d, rows, 0, nr), nullptr, p, OpReset{}, s, true);
}

void launch_merge_list(const GhDev& d, int cur, int32_t obs, const int32_t* ids, const int32_t* hb, int64_t n,
                       const GhRound& p, hipStream_t s) {
  if (n == 0) return;
  scatter(d, ids, hb, (int32_t)n, 0x80, s);
  if (gh_owned(d, obs)) seg_launch(d, cur, rows_set(d, nullptr, obs, 1), nullptr, p, OpMergeList{d, p}, s);
}

void launch_hb_check(const GhDev& d, int cur, int32_t* flag, const GhRound& p, hipStream_t s) {
  if (d.ncol > 0)
    hipLaunchKernelGGL(k_hb_check, dim3((unsigned)((d.ncol + 255) / 256)), dim3(256), 0, s, d, cur, flag, p);
}
