// MemberList order (GH_ORDER_APPEND; SPEC.md §7 D1, DESIGN.md "List order").
//
// The reference keeps each member's list as a Go slice: members are appended
// when they are added (slave/slave.go:255 addNewMember, :437 MergeMemberList
// in the received list's order), removal closes the gap (:283), and four
// things read the order: ring targets (:515-524), quirk-mode detection runs
// (:464-477), MemberList[0] (:936, :994) and the master's placement
// candidates (master/master.go:46, :135). The table holds the SET of each
// list; this file keeps the ORDER beside it:
//   lord[b][i * ld + p]  the member at position p of row i's list,
//   llen[b][i]           its length,
// double-buffered (b = the host's lcur for the current state), rebuilt by one
// workgroup per row whenever the table's membership changes:
//   k_list_round   after a round: the members that stayed keep their order;
//                  the ones added are appended sender by sender in ID order
//                  (the delivery order, SPEC §2), each sender's in the order
//                  of its snapshot list (its list after REMOVE and detection)
//   k_list_events  after events / an external datagram: stayed members keep
//                  their order, added ones follow a given source list (the
//                  joiners in event order, the introducer's new list, the
//                  datagram)
//   k_list_import  rows written whole (import, full membership): ID order
//   k_ring_list    ring targets list[(idx-1) mod L], [(idx+1)], [(idx+2)] of
//                  every sender's snapshot list in list order
//   k_quirk_list   quirk-mode runs over the list order: the flags of skipped
//                  candidates are cleared (the ID-order pre-pass, round.hip,
//                  in list order)
//   k_list_cand / k_list_first   master's candidates, MemberList[0]
// One engine, or row shards (GH_LAYOUT_ROWS): every shard keeps every row's
// list (a replica) and rebuilds only the rows it owns; the owners' changed
// lists (lchg) are then copied to every shard (k_list_pack / k_list_unpack,
// gossiphip.cpp list_sync), so the senders' snapshot lists, the master's
// candidates and MemberList[0] of any row are local reads everywhere. Column
// shards are refused (a row's order spans every column).
#include <limits.h>

#include "gh_internal.h"

namespace {

constexpr int kMaxSenders = 128;  // distinct senders of one receiver per batch (k_list_round)

// REMOVE of member c delivered to row j at step 1 (D_{r-1}; the sole
// detector does not message itself, slave/slave.go:344-346)
__device__ __forceinline__ bool removed_at(const GhDev& d, int dcur, int64_t c, int64_t j) {
  if (!((d.dbits[c >> 5] >> (c & 31)) & 1u)) return false;
  return gh_rm_at(d, dcur, c, j);
}

__device__ __forceinline__ bool bit(const uint32_t* b, int64_t c) { return (b[c >> 5] >> (c & 31)) & 1u; }

// Exclusive prefix of pred over the 256 threads of the block (4 waves) and
// the block's total. Uniform call (two barriers).
__device__ __forceinline__ int block_prefix(bool pred, int& total, int* s_w) {
  const unsigned long long m = __ballot(pred);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int before = __popcll(m & ((1ull << lane) - 1ull));
  if (lane == 0) s_w[w] = __popcll(m);
  __syncthreads();
  int off = 0;
  total = 0;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    off += q < w ? s_w[q] : 0;
    total += s_w[q];
  }
  __syncthreads();
  return off + before;
}

// Row i's list in generation g: lord[lsel[g][i]] + i * ld, llen[g][i]
// entries, own member at lself[g][i] (-1: not listed).
__device__ __forceinline__ const int32_t* list_of(const GhDev& d, int g, int64_t i) {
  return d.lord[d.lsel[g][i]] + i * d.ld;
}

// Generation g ^ 1 of row i = generation g (thread 0).
__device__ __forceinline__ void keep_row(const GhDev& d, int g, int64_t i) {
  if (threadIdx.x == 0) {
    d.lsel[g ^ 1][i] = d.lsel[g][i];
    d.llen[g ^ 1][i] = d.llen[g][i];
    d.lself[g ^ 1][i] = d.lself[g][i];
  }
}

// The members of row i present in buffer buf and not in the LDS set `stay`
// (stay null: not present in buffer old) -> LDS set `app`; returns their
// count (uniform).
__device__ int mark_added(const GhDev& d, int buf, int old, int64_t i, const uint32_t* stay, uint32_t* app, int* s_w) {
  int a = 0;
  for (int64_t c8 = (int64_t)threadIdx.x * 8; c8 < d.n; c8 += (int64_t)blockDim.x * 8) {
    const uint32_t pf = gh_pf8(d, buf, i, c8) & 0xFFu;
    const uint32_t was = stay ? (stay[c8 >> 5] >> (c8 & 31)) & 0xFFu : gh_pf8(d, old, i, c8) & 0xFFu;
    const uint32_t m = pf & ~was;
    if (m) {
      atomicOr(&app[c8 >> 5], m << (c8 & 31));
      a += __builtin_popcount(m);
    }
  }
  for (int o = 32; o > 0; o >>= 1) a += __shfl_xor(a, o);
  if ((threadIdx.x & 63) == 0) s_w[threadIdx.x >> 6] = a;
  __syncthreads();
  const int tot = s_w[0] + s_w[1] + s_w[2] + s_w[3];
  __syncthreads();
  return tot;
}

// Appends, in the order of list src[0..ns), the members of `app` that
// `visible` admits; clears their bits; a row's own member i sets *s_self.
// pos / need are uniform.
template <class Visible>
__device__ void append_from(const int32_t* src, int ns, uint32_t* app, int32_t* dst, int& pos, int& need, int* s_w,
                            int64_t i, int* s_self, Visible visible) {
  for (int b = 0; b < ns && need > 0; b += blockDim.x) {
    const int q = b + threadIdx.x;
    int c = -1;
    bool take = false;
    if (q < ns) {
      c = src[q];
      take = c >= 0 && bit(app, c) && visible(c);
    }
    int tot;
    const int o = block_prefix(take, tot, s_w);
    if (take) {
      dst[pos + o] = c;
      if (c == i) *s_self = pos + o;
      atomicAnd(&app[c >> 5], ~(1u << (c & 31)));
    }
    pos += tot;
    need -= tot;
    __syncthreads();
  }
}

// Old list of row i (generation g) -> dst, keeping the members `keep` admits
// in order; their bits -> LDS set `stay`; the own member's new position ->
// *s_self. Returns the count (uniform).
template <class Keep>
__device__ int compact(const GhDev& d, int g, int64_t i, int32_t* dst, uint32_t* stay, int* s_w, int* s_self,
                       Keep keep_fn) {
  const int L = d.llen[g][i];
  const int32_t* src = list_of(d, g, i);
  int pos = 0;
  for (int b = 0; b < L; b += blockDim.x) {
    const int q = b + threadIdx.x;
    int c = -1;
    bool keep = false;
    if (q < L) {
      c = src[q];
      keep = keep_fn(c);
    }
    int tot;
    const int o = block_prefix(keep, tot, s_w);
    if (keep) {
      dst[pos + o] = c;
      if (c == i) *s_self = pos + o;
      atomicOr(&stay[c >> 5], 1u << (c & 31));
    }
    pos += tot;
  }
  __syncthreads();
  return pos;
}

// After a round (before k_finish: D_{r-1} and the inboxes are intact). One
// workgroup per row; dynamic LDS: two member bitmaps. A row without removals
// keeps its list and buffer (members added are appended in place, past the
// end the senders read); a row with removals is rewritten into its other
// buffer.
__global__ __launch_bounds__(256) void k_list_round(GhDev d, int cur, int dcur, GhRound p, int g) {
  extern __shared__ uint32_t s_bits[];
  __shared__ int s_w[4];
  __shared__ int s_snd[kMaxSenders];
  __shared__ int s_ns, s_rem, s_self;
  const int64_t i = blockIdx.x;
  if (i >= d.n) return;
  if (!d.alive[i] || !gh_owned(d, i)) {  // a stopped row is not touched by the round; another shard's row: its owner's copy follows
    keep_row(d, g, i);
    return;
  }
  const int nxt = cur ^ 1;
  const bool act = d.active[i];
  const int L = d.llen[g][i];
  const int target = d.cntl[i];  // present after the round (kept current by the round kernels)
  // removals in this row: a detection (step 4), or a REMOVE of D_{r-1} (step
  // 1) of a member it lists
  if (threadIdx.x == 0) {
    s_rem = d.det_any[i];
    s_self = d.lself[g][i];
  }
  __syncthreads();
  const int nd = d.cntg[p.n];
  if (!s_rem && nd > 0) {
    if (d.nd[dcur] > GH_DLIST_MAX) {
      s_rem = 1;  // storms: assume so
    } else {
      for (int q = threadIdx.x; q < d.nd[dcur]; q += blockDim.x) {
        const int c = d.dlist[(int64_t)dcur * p.ld + q];
        if (removed_at(d, dcur, c, i) && gh_get(d, cur, i, c, 0).x >= 0) s_rem = 1;
      }
    }
  }
  __syncthreads();
  const bool rem = s_rem != 0;
  if (!rem && target == L) {
    keep_row(d, g, i);
    return;
  }
  const int nw = (d.n + 31) >> 5;
  uint32_t* stay = s_bits;
  uint32_t* app = s_bits + nw;
  for (int w = threadIdx.x; w < 2 * nw; w += blockDim.x) s_bits[w] = 0;
  __syncthreads();
  const int b0 = d.lsel[g][i];
  const int bo = rem ? b0 ^ 1 : b0;  // output buffer: in place when nothing left the list
  int32_t* dst = d.lord[bo] + i * d.ld;
  int pos = L;
  if (rem) {
    if (threadIdx.x == 0) s_self = -1;
    __syncthreads();
    // members that stayed: not REMOVE'd (step 1), not detected (step 4: a
    // flag of an active row), still present (a removed member the merge
    // brings back is appended again)
    pos = compact(d, g, i, dst, stay, s_w, &s_self, [&](int c) {
      return gh_get(d, nxt, i, c, 0).x >= 0 && !removed_at(d, dcur, c, i) && !(act && gh_get(d, cur, i, c, 0).f);
    });
  }
  int need = target - pos;
  if (need > 0) {
    need = mark_added(d, nxt, cur, i, rem ? stay : nullptr, app, s_w);
    // the receiver's senders, ascending and distinct (SPEC §2 delivery order),
    // taken kMaxSenders at a time: each batch holds the smallest distinct
    // senders above the last batch's largest (a ring inbox has no bound)
    const bool pull = p.peer_mode == GH_PEER_PULL;
    const int cnt = gh_in_cnt(d, pull, p.k, i);
    const int64_t beg = gh_in_beg(d, pull, p.k, i);
    int last = -1;
    for (;;) {
      if (threadIdx.x == 0) {
        int ns = 0;
        for (int q = 0; q < cnt; ++q) {
          const int s = d.inbox[beg + q];
          if (s <= last) continue;
          int at = ns;
          bool dup = false;
          for (int x = 0; x < ns; ++x) {
            if (s_snd[x] == s) dup = true;
            if (s_snd[x] > s && at == ns) at = x;
          }
          if (dup || at == kMaxSenders) continue;  // a duplicate, or above a full batch
          for (int x = (ns < kMaxSenders ? ns : kMaxSenders - 1); x > at; --x) s_snd[x] = s_snd[x - 1];
          s_snd[at] = s;
          if (ns < kMaxSenders) ns++;
        }
        s_ns = ns;
      }
      __syncthreads();
      const int ns = s_ns;
      for (int q = 0; q < ns && need > 0; ++q) {
        const int s = s_snd[q];
        // s's snapshot: its list (generation g) after REMOVE delivery and detection
        append_from(list_of(d, g, s), d.llen[g][s], app, dst, pos, need, s_w, i, &s_self,
                    [&](int c) { return !gh_get(d, cur, s, c, 0).f && !removed_at(d, dcur, c, s); });
      }
      if (ns < kMaxSenders || need <= 0) break;  // (uniform: ns and need are the same in every thread)
      last = s_snd[kMaxSenders - 1];
      __syncthreads();  // s_snd is refilled
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    if (pos != target) atomicExch(d.err, GH_EINVAL);  // the order lost track of the set
    d.lsel[g ^ 1][i] = (uint8_t)bo;
    d.llen[g ^ 1][i] = pos;
    d.lself[g ^ 1][i] = s_self;
    if (d.lchg) d.lchg[i] = 1;  // row shards: copied to every shard
  }
}

// After events or an external datagram (table buffer cur, counts current):
// generation g -> g ^ 1, each row rewritten into its other buffer. rows: the
// rows to rebuild (null: blockIdx.x); skip: a row left alone (-1 none).
// Added members follow src_ids[0..n_src) if given, else the new list
// (generation g ^ 1) of row src_row, else none may be added.
__global__ __launch_bounds__(256) void k_list_events(GhDev d, int cur, int g, const int32_t* rows,
                                                     const int32_t* src_ids, int n_src, int src_row, int skip) {
  extern __shared__ uint32_t s_bits[];
  __shared__ int s_w[4];
  __shared__ int s_self;
  const int64_t i = rows ? rows[blockIdx.x] : blockIdx.x;
  if (i >= d.n || i == skip) return;
  if (!d.alive[i] || !gh_owned(d, i)) {  // (row shards: the owner's copy follows)
    keep_row(d, g, i);
    return;
  }
  const int nw = (d.n + 31) >> 5;
  uint32_t* stay = s_bits;
  uint32_t* app = s_bits + nw;
  for (int w = threadIdx.x; w < 2 * nw; w += blockDim.x) s_bits[w] = 0;
  if (threadIdx.x == 0) s_self = -1;
  __syncthreads();
  const int bo = d.lsel[g][i] ^ 1;
  int32_t* dst = d.lord[bo] + i * d.ld;
  int pos = compact(d, g, i, dst, stay, s_w, &s_self, [&](int c) { return gh_get(d, cur, i, c, 0).x >= 0; });
  const int target = d.cntl[i];
  int need = target - pos;
  if (need > 0) {
    need = mark_added(d, cur, cur, i, stay, app, s_w);
    auto any = [](int) { return true; };
    if (src_ids)
      append_from(src_ids, n_src, app, dst, pos, need, s_w, i, &s_self, any);
    else if (src_row >= 0)
      append_from(list_of(d, g ^ 1, src_row), d.llen[g ^ 1][src_row], app, dst, pos, need, s_w, i, &s_self, any);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    if (pos != target) atomicExch(d.err, GH_EINVAL);
    d.lsel[g ^ 1][i] = (uint8_t)bo;
    d.llen[g ^ 1][i] = pos;
    d.lself[g ^ 1][i] = s_self;
    if (d.lchg) d.lchg[i] = 1;
  }
}

// Rows [row0, row0 + nr) written whole: their lists in member-ID order (the
// order a dense import implies), in place in generation g.
__global__ __launch_bounds__(256) void k_list_import(GhDev d, int cur, int g, int64_t row0) {
  __shared__ int s_w[4];
  __shared__ int s_self;
  const int64_t i = row0 + blockIdx.x;
  if (i >= d.n || !gh_owned(d, i)) return;  // (row shards: the owner's copy follows)
  if (threadIdx.x == 0) s_self = -1;
  __syncthreads();
  int32_t* dst = d.lord[d.lsel[g][i]] + i * d.ld;
  int pos = 0;
  for (int64_t b = 0; b < d.n; b += blockDim.x) {
    const int64_t c = b + threadIdx.x;
    const bool pres = c < d.n && gh_get(d, cur, i, c, 0).x >= 0;
    int tot;
    const int o = block_prefix(pres, tot, s_w);
    if (pres) {
      dst[pos + o] = (int32_t)c;
      if (c == i) s_self = pos + o;
    }
    pos += tot;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    d.llen[g][i] = pos;
    d.lself[g][i] = s_self;
    if (d.lchg) d.lchg[i] = 1;
  }
}

// Ring mode in list order (slave/slave.go:512-524): per sender row, its
// snapshot list = its list without the members REMOVE'd at it or detected by
// it; idx = its own position there (-1 if absent), L = the length; targets
// list[(idx-1) mod L], list[(idx+1) mod L], list[(idx+2) mod L], Go's
// truncated % plus L for negatives. whole (flag counts current, no REMOVE
// pending, no flagged segment anywhere): every snapshot is the whole list,
// indexed directly.
__global__ __launch_bounds__(256) void k_ring_list(GhDev d, int cur, int dcur, GhRound p, int g, int whole) {
  __shared__ int s_w[4];
  __shared__ int s_idx;
  __shared__ int s_tg[3];
  const int64_t s = blockIdx.x;
  if (s >= p.n) return;
  if (threadIdx.x < 3) s_tg[threadIdx.x] = -1;
  whole = whole && d.cntg[p.n] == 0 && d.cntg[p.n + 1] == 0;
  if (threadIdx.x == 0) s_idx = whole ? d.lself[g][s] : -1;
  __syncthreads();
  if (d.alive[s] && d.active[s] && gh_owned(d, s)) {  // (row shards: each sender's owner; the targets are max-reduced)
    const int L = d.llen[g][s];
    const int32_t* sl = list_of(d, g, s);
    auto in_snap = [&](int c) { return !gh_get(d, cur, s, c, 0).f && !removed_at(d, dcur, c, s); };
    int len = L;
    if (!whole) {
      len = 0;
      for (int b = 0; b < L; b += blockDim.x) {
        const int q = b + threadIdx.x;
        const int c = q < L ? sl[q] : -1;
        const bool in = c >= 0 && in_snap(c);
        int tot;
        const int o = block_prefix(in, tot, s_w);
        if (in && c == s) s_idx = len + o;
        len += tot;
      }
    }
    __syncthreads();
    if (len == 0) {
      if (threadIdx.x == 0) atomicAdd(&d.stats[ST_RING_EMPTY], 1ull);  // slave.go:517 division by zero
    } else {
      const int64_t idx = s_idx;
      int64_t want[3] = {idx - 1, idx + 1, idx + 2};
      for (int q = 0; q < 3; ++q) {
        int64_t v = want[q] % len;  // C and Go both truncate toward zero
        if (v < 0) v += len;
        want[q] = v;
      }
      if (whole) {
        if (threadIdx.x < 3) s_tg[threadIdx.x] = sl[want[threadIdx.x]];
      } else {
        int at = 0;
        for (int b = 0; b < L; b += blockDim.x) {
          const int q = b + threadIdx.x;
          const int c = q < L ? sl[q] : -1;
          const bool in = c >= 0 && in_snap(c);
          int tot;
          const int o = block_prefix(in, tot, s_w);
          if (in)
            for (int x = 0; x < 3; ++x)
              if (want[x] == at + o) s_tg[x] = c;
          at += tot;
        }
      }
    }
  }
  __syncthreads();
  if (threadIdx.x < 3) d.targets[s * 3 + threadIdx.x] = s_tg[threadIdx.x];
}

// Quirk-mode run state (round.hip's pre-pass, here over single list
// entries): a stretch maps the parity s of the trailing candidate run before
// it to f(s). Bits: 0 = holds a non-candidate list member, 1 = value, 2 = holds
// a list member; 0 is the identity.
__device__ __forceinline__ int run_compose(int a, int b) {  // a, then b
  return ((a | b) & 5) | ((b & 1) ? (b & 2) : ((a ^ b) & 2));
}
__device__ __forceinline__ int run_apply(int f, int s) { return (f & 1) ? ((f >> 1) & 1) : (s ^ ((f >> 1) & 1)); }

// Clears the detection flag of present cell (i, c) of buffer buf (atomic:
// cells of one row share words).
__device__ void clear_flag(const GhDev& d, int buf, int64_t i, int64_t c) {
  const int64_t c8 = c & ~(int64_t)7;
  const int64_t cell0 = gh_cell(d, i, c8);
  // a tier chunk holds no flag; an escaped one is hn's
  if (gh_m8(d, buf) && !gh_t4_esc(d.a4[buf][cell0 >> 3])) return;
  const uint2 hd = *reinterpret_cast<const uint2*>(d.hn[buf] + cell0);
  const uint32_t h0 = hd.x & 0xFFFFu;
  if (h0 == GH_N_FROZEN) return;
  if (h0 == GH_N_WIDE) {
    const int64_t slot = gh_wide_slot(hd.x, hd.y);
    if (slot >= d.wcap) return;
    const int64_t fb = gh_wcell(d, slot, c) >> 3;  // flag byte of the chunk
    uint8_t* bp = d.wf[buf] + fb;
    uint32_t* wp = reinterpret_cast<uint32_t*>(reinterpret_cast<uintptr_t>(bp) & ~(uintptr_t)3);
    const int sh = 8 * (int)(reinterpret_cast<uintptr_t>(bp) & 3) + (int)(c & 7);
    atomicAnd(wp, ~(1u << sh));
    return;
  }
  const int64_t cell = cell0 + (c & 7);
  uint32_t* wp = reinterpret_cast<uint32_t*>(d.hn[buf] + (cell & ~(int64_t)1));
  atomicAnd(wp, ~(0x8000u << (16 * (int)(cell & 1))));
}

// Quirk-mode detection in list order (slave/slave.go:464-477 with :283): in
// each run of consecutive candidates of the list after REMOVE delivery, the
// candidates at even offsets are detected, plus the list's last entry;
// the others' flags are cleared.
__global__ __launch_bounds__(256) void k_quirk_list(GhDev d, int cur, int dcur, GhRound p, int g) {
  __shared__ int s_w[4];
  __shared__ int s_f[256];
  __shared__ int s_last;
  const int64_t i = blockIdx.x;
  if (p.qgate && d.cntg[p.n + 1] == 0) return;  // no flag anywhere
  if (i == 0 && threadIdx.x == 0) d.pvalid[cur] = 0;  // cleared flags: the sender plane is stale
  if (i >= p.n || !(d.alive[i] && d.active[i]) || !gh_owned(d, i)) return;
  const int L = d.llen[g][i];
  const int32_t* sl = list_of(d, g, i);
  if (threadIdx.x == 0) s_last = -1;
  __syncthreads();
  // the last list entry after REMOVE delivery
  for (int b = 0; b < L; b += blockDim.x) {
    const int q = b + threadIdx.x;
    if (q < L && !removed_at(d, dcur, sl[q], i)) atomicMax(&s_last, q);
  }
  __syncthreads();
  const int last = s_last;
  int s = 0;  // run parity entering the chunk
  for (int b = 0; b < L; b += blockDim.x) {
    const int q = b + threadIdx.x;
    int c = -1, f = 0;
    bool cand = false;
    if (q < L) {
      c = sl[q];
      if (!removed_at(d, dcur, c, i)) {
        cand = gh_get(d, cur, i, c, 0).f;
        f = cand ? 6 : 5;
      }
    }
    // inclusive scan of the run maps over the chunk (Hillis-Steele)
    s_f[threadIdx.x] = f;
    __syncthreads();
    for (int off = 1; off < (int)blockDim.x; off <<= 1) {
      const int other = threadIdx.x >= off ? s_f[threadIdx.x - off] : 0;
      __syncthreads();
      s_f[threadIdx.x] = run_compose(other, s_f[threadIdx.x]);
      __syncthreads();
    }
    const int excl = threadIdx.x ? s_f[threadIdx.x - 1] : 0;
    const int st = run_apply(excl, s);
    if (cand && !(st == 0 || q == last)) clear_flag(d, cur, i, c);  // skipped this round
    s = run_apply(s_f[blockDim.x - 1], s);
    __syncthreads();
  }
  (void)s_w;
}

// Member_list (master/master.go:46): the master row's list in list order.
__global__ __launch_bounds__(256) void k_list_cand(GhDev d, int g, int32_t master) {
  const int L = d.llen[g][master];
  const int32_t* sl = list_of(d, g, master);
  for (int q = blockIdx.x * blockDim.x + threadIdx.x; q < L; q += gridDim.x * blockDim.x) d.cand[q] = sl[q];
  if (blockIdx.x == 0 && threadIdx.x == 0) d.ncand[0] = L;
}

// MemberList_i[0] in k_vote_scan's encoding: n - member, 0 for an empty list.
__global__ __launch_bounds__(256) void k_list_first(GhDev d, int g, int32_t* out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= d.n) return;
  out[i] = d.llen[g][i] > 0 ? d.n - list_of(d, g, i)[0] : 0;
}

// Row shards: the lists of the rows in [lo, hi) this shard changed (lchg),
// packed for the other shards: [count | rows | lens | selfs | offsets |
// entries] (R = hi - lo int32 each for the per-row parts), entries of the rows
// back to back in row order. k_list_pack_index: one workgroup scans the
// range's rows in ascending order and writes the header; k_list_pack_copy:
// one workgroup per packed row copies its entries and clears its lchg.
__global__ __launch_bounds__(1024) void k_list_pack_index(GhDev d, int g, int32_t* buf, int64_t lo, int64_t hi) {
  __shared__ int s_w[16], s_c[16];
  __shared__ int64_t s_base, s_rows;
  if (threadIdx.x == 0) s_base = s_rows = 0;
  __syncthreads();
  const int64_t R = hi - lo;
  for (int64_t b = lo; b < hi; b += blockDim.x) {
    const int64_t i = b + threadIdx.x;
    const bool chg = i < hi && d.lchg[i];
    const int len = chg ? d.llen[g][i] : 0;
    // block-wide exclusive prefix of chg (rows) and len (entries)
    const unsigned long long m = __ballot(chg);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    int lx = len;
    for (int o = 1; o < 64; o <<= 1) {
      const int y = __shfl_up(lx, o);
      if (lane >= o) lx += y;
    }
    if (lane == 63) s_w[w] = lx;
    if (lane == 0) s_c[w] = __popcll(m);
    __syncthreads();
    int64_t woff = 0;
    int wrow = 0;
    for (int q = 0; q < w; ++q) woff += s_w[q], wrow += s_c[q];
    const int64_t row_at = s_rows + wrow + __popcll(m & ((1ull << lane) - 1ull));
    const int64_t ent_at = s_base + woff + lx - len;
    if (chg) {
      buf[1 + row_at] = (int32_t)i;
      buf[1 + R + row_at] = len;
      buf[1 + 2 * R + row_at] = d.lself[g][i];
      buf[1 + 3 * R + row_at] = (int32_t)ent_at;  // (a range holds at most R * ld < 2^31 entries: list_sync)
    }
    __syncthreads();
    if (threadIdx.x == blockDim.x - 1) {
      int64_t tot = 0;
      int tr = 0;
      for (int q = 0; q < (int)(blockDim.x >> 6); ++q) tot += s_w[q], tr += s_c[q];
      s_base += tot;
      s_rows += tr;
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) buf[0] = (int32_t)s_rows;
}

__global__ __launch_bounds__(256) void k_list_pack_copy(GhDev d, int g, int32_t* buf, int64_t R) {
  const int nr = buf[0];
  const int32_t* ent_hdr = buf + 1 + 3 * R;
  int32_t* ent = buf + 1 + 4 * R;
  for (int r = blockIdx.x; r < nr; r += gridDim.x) {
    const int64_t i = buf[1 + r];
    const int len = buf[1 + R + r];
    const int32_t* src = d.lord[d.lsel[g][i]] + i * d.ld;
    int32_t* dst = ent + ent_hdr[r];
    for (int q = threadIdx.x; q < len; q += blockDim.x) dst[q] = src[q];
    if (threadIdx.x == 0) d.lchg[i] = 0;
  }
}

// Another shard's packed lists into this shard's replicas of generation g, in
// place (nothing reads the rows' earlier lists any more).
__global__ __launch_bounds__(256) void k_list_unpack(GhDev d, int g, const int32_t* buf, int64_t R) {
  const int nr = buf[0];
  const int32_t* ent = buf + 1 + 4 * R;
  for (int r = blockIdx.x; r < nr; r += gridDim.x) {
    const int64_t i = buf[1 + r];
    const int len = buf[1 + R + r];
    const int64_t off = buf[1 + 3 * R + r];
    int32_t* dst = d.lord[d.lsel[g][i]] + i * d.ld;
    for (int q = threadIdx.x; q < len; q += blockDim.x) dst[q] = ent[off + q];
    if (threadIdx.x == 0) {
      d.llen[g][i] = len;
      d.lself[g][i] = buf[1 + 2 * R + r];
    }
  }
}

size_t list_lds(const GhDev& d) { return sizeof(uint32_t) * 2 * (size_t)((d.n + 31) / 32); }

}  // namespace

bool list_lds_ok(const GhDev& d) { return list_lds(d) <= 64 * 1024; }

void launch_list_round(const GhDev& d, int cur, int dcur, const GhRound& p, int lin, hipStream_t s) {
  hipLaunchKernelGGL(k_list_round, dim3(d.n), dim3(256), list_lds(d), s, d, cur, dcur, p, lin);
}

void launch_list_events(const GhDev& d, int cur, int lin, const int32_t* rows, int32_t nr, const int32_t* src_ids,
                        int32_t n_src, int32_t src_row, int32_t skip, hipStream_t s) {
  const int32_t grid = rows ? nr : d.n;
  if (grid <= 0) return;
  hipLaunchKernelGGL(k_list_events, dim3(grid), dim3(256), list_lds(d), s, d, cur, lin, rows, src_ids, n_src, src_row,
                     skip);
}

void launch_list_import(const GhDev& d, int cur, int lb, int64_t row0, int64_t nr, hipStream_t s) {
  if (nr <= 0) return;
  hipLaunchKernelGGL(k_list_import, dim3((unsigned)nr), dim3(256), 0, s, d, cur, lb, row0);
}

void launch_ring_list(const GhDev& d, int cur, int dcur, const GhRound& p, int lin, int whole, hipStream_t s) {
  hipLaunchKernelGGL(k_ring_list, dim3(p.n), dim3(256), 0, s, d, cur, dcur, p, lin, whole);
}

void launch_quirk_list(const GhDev& d, int cur, int dcur, const GhRound& p, int lin, hipStream_t s) {
  hipLaunchKernelGGL(k_quirk_list, dim3(p.n), dim3(256), 0, s, d, cur, dcur, p, lin);
}

void launch_list_cand(const GhDev& d, int lin, int32_t master, hipStream_t s) {
  hipLaunchKernelGGL(k_list_cand, dim3(std::max<int32_t>(1, std::min<int32_t>((d.n + 255) / 256, 1024))), dim3(256),
                     0, s, d, lin, master);
}

// Row shards: this shard's changed lists of rows [lo, hi) (lchg, cleared)
// packed into buf (1 + 4 (hi - lo) + entries int32), and another shard's pack
// of the same range into the replicas.
void launch_list_pack(const GhDev& d, int g, int32_t* buf, int64_t lo, int64_t hi, hipStream_t s) {
  hipLaunchKernelGGL(k_list_pack_index, dim3(1), dim3(1024), 0, s, d, g, buf, lo, hi);
  hipLaunchKernelGGL(k_list_pack_copy, dim3((unsigned)std::min<int64_t>(hi - lo, 4096)), dim3(256), 0, s, d, g, buf,
                     hi - lo);
}
void launch_list_unpack(const GhDev& d, int g, const int32_t* buf, int64_t lo, int64_t hi, hipStream_t s) {
  hipLaunchKernelGGL(k_list_unpack, dim3((unsigned)std::min<int64_t>(hi - lo, 4096)), dim3(256), 0, s, d, g, buf,
                     hi - lo);
}

void launch_list_first(const GhDev& d, int lin, int32_t* out, hipStream_t s) {
  hipLaunchKernelGGL(k_list_first, dim3((d.n + 255) / 256), dim3(256), 0, s, d, lin, out);
}
