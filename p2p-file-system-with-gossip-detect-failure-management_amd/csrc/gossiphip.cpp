// libgossiphip host side: the C-ABI of include/gossiphip.h over the HIP
// kernels in round.hip / events.hip / place.hip / elect.hip. One handle = one engine =
// one gfx950 device, one HIP stream, its tables resident in HBM. A sharded
// engine (gh_create_sharded) is rank g of G column shards of one cluster;
// its O(N) per-round exchanges go through comm.h (RCCL, or threads of one
// process).
//
// Reference interfaces replaced (paths under the reference tree):
//   InitSlave / InitMaster            slave/slave.go:95, master/master.go:38
//   HeartBeat round loop              main.go:27-33, slave/slave.go:499-544
//   GetMsg JOIN/LEAVE/REMOVE          slave/slave.go:207-248
//   UDP list exchange between hosts   slave/slave.go:527-542 (-> comm.h)
//   Handle_put_request / Update_metadata / Get_* / Delete_file_info
//                                     master/master.go:74-259
//   revote_master / rebuild_file_meta slave/slave.go:930-1043
// There is no CPU fallback: without a gfx950 device gh_create fails.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <climits>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "comm.h"
#include "gh_internal.h"

namespace {

struct Engine {
  gh_config cfg{};
  int32_t n = 0;
  int64_t ld = 0;
  int rank = 0, world = 1;
  std::unique_ptr<GhComm> comm;
  hipStream_t stream = nullptr;
  // a tiered engine launches the round variants the nibble path does not need
  // on a side stream (forked after the round's inputs, joined before the lane
  // jobs): one of the four runs, the three idle ones return at once while the
  // nibble path runs, off the round's critical path
  hipStream_t vstream = nullptr, vstream2 = nullptr;
  hipEvent_t vfork = nullptr, vjoin = nullptr, vjoin2 = nullptr;
  hipEvent_t vstart = nullptr;  // the nibble launch's start stamp when not timing (the side stream's fork)
  hipEvent_t vstop = nullptr;   // the last idle launch's end stamp when not timing (the join)
  GhDev d{};
  int cur = 0, dcur = 0;
  int32_t round = 0;
  std::vector<uint8_t> alive;   // host mirror (source of truth for events)
  std::vector<gh_event> pending;
  int32_t* ev_buf = nullptr;    // device scratch for event member lists
  int32_t* rows_buf = nullptr;  // device scratch for a few row ids
  int64_t rbits_rows = 0;       // rows rbits can hold
  bool nt = true;        // k_round non-temporal streams (gh_set_round_variant)
  int xmap = 1;          // k_round XCD-aware tile map (gh_set_round_variant)
  int tpw = 1;           // k_round tiles per workgroup (GH_ROUND_TPW)
  int force_storm = 0;   // storm variant every round (GH_FORCE_STORM, diagnostics)
  int force_slow = 0;    // every segment by the per-cell rule (GH_FORCE_SLOW, diagnostics)
  int nib_rmv = 1;       // REMOVE'd members with >= 2 detectors on the nibble path (GH_NIB_RMV=0: lane jobs,
                         // 2: the REMOVE-taking instantiation every round; A/B)
  int nib_dma = 0;       // the nibble path stages its lines by LDS-DMA (GH_NIB_DMA=1, A/B)
  bool shadow_any = false;  // the introducer's row may hold D7 shadow entries (GhDev.shadow; re-read after each gh_step)
  bool timing = false;
  int side = 1;          // idle round variants on the side stream (GH_SIDE=0: in line; 2: two side streams)
  // the current table may hold flags no round kernel counted (import, fill,
  // events, list merges): the next quirk pre-pass runs ungated
  bool qforce = true;
  // the current table was rewritten whole outside a round (import, fill):
  // its sender plane is stale (pvalid[cur] = 0 before the next round). Events
  // and list merges keep the plane (gh_put8 writes each chunk's plane word)
  bool pforce = true;
  // the table was written outside a round: no row is a quiet candidate
  bool sforce = true;
  // row layout (GH_LAYOUT_ROWS): rows per shard, host mirror of rslot, the
  // current ghost rows, exchange buffers (grown on demand)
  bool rowlay = false;
  int64_t nrs = 0;
  int64_t segs_g = 0;    // wide-arena sizing: segments of owned rows + the ghost table, the largest over the shards
  int64_t segs_all = 0;  // segments the arena may ever have to hold (row layout: every row as a ghost)
  bool dry = false;       // gh_footprint: create() only counts its allocations
  int64_t dry_bytes = 0;
  std::vector<int32_t> rslot_h;
  std::vector<int32_t> ghosts;
  std::vector<std::vector<int32_t>> gx_send;  // rows this shard sends each rank this round
  std::vector<int64_t> gx_rcnt, gx_rbeg;      // ghosts from each owner: count, first ghost index
  int64_t gx_maxsend = 0;                     // the most rows any shard sends (the chunk count)
  // device want lists (round_ghosts): the set-up ghosts are want[me] in
  // wlist, this shard's send list to r is wlist[r][gx_soff[r], + gx_sn[r])
  bool gx_dev = false;
  uint32_t* wbits = nullptr;
  int32_t *wsum = nullptr, *wlist = nullptr, *mcnt = nullptr;
  std::vector<int32_t> gx_m;            // host copy of mcnt: [G][G] counts, [G] totals
  std::vector<int64_t> gx_sn, gx_soff;  // rows this shard sends each rank, their offset in want[r]
  bool gpo = false;                           // this round's ghosts carry only their plane (GhRound.gpo)
  bool plane_valid = false;                   // the current buffer's plane was written by a round
  int32_t* gwcnt = nullptr;  // [2 * world] wide counts / cursors per destination
  void* gbuf[4] = {nullptr, nullptr, nullptr, nullptr};  // send, recv, wide send, wide recv
  size_t gcap_bytes[4] = {0, 0, 0, 0};
  int32_t* gidx = nullptr;   // [2 * cap] rows to send, their destinations
  int64_t gidx_cap = 0;
  int64_t gx_rows = 0, gx_out = 0, gx_in = 0;  // the last exchange: ghost rows, bytes sent / received
  int plane = 0;         // sender snapshot plane (pull mode, 3 <= k <= 4, N >= GH_PLANE_MIN_N; GH_PLANE=0/1)
  int c8 = 0;            // 4-bit tier (plane mode, column layout; GH_C8=0 drops it)
  // GH_ORDER_APPEND: per-row list order kept beside the table (order.hip);
  // lcur = the list buffer of the current state
  bool lorder = false;
  int lcur = 0;
  // nflag of the current buffer counts its flagged segments (a round wrote
  // it; host writes do not count theirs)
  bool flags_known = false;
  // upper bound of every heartbeat in the table (int32 overflow check,
  // slave/slave.go:446): +1 per round, max of imported / merged values
  int64_t hb_bound = 0;
  // frozen store (stopped rows): slot per row (-1 running), free slots
  std::vector<int32_t> frow;
  std::vector<int32_t> fz_free;
  int64_t fzcap = 0;
  std::string lost;  // non-empty: the device state was lost (arena overflow)
  double timed_ms = 0.0;
  int64_t timed_launches = 0;
  std::vector<hipEvent_t> evs;
  // tmode 1 (GH_TMODE, default): only the nibble launch carries its own
  // start / stop events; the other variants are timed together by two
  // events around them, and the device logs which variant ran (vlog).
  // tmode 0: every variant launch carries its own events.
  int tmode = 1;
  int join_stamp = 1;  // GH_JOIN_STAMP=0: the join as an event recorded after the side stream's last launch (A/B)
  int quirk_rows = 1;  // GH_QUIRK_ROWS=0: the two-sweep quirk pre-pass where the one-pass row walk applies (A/B)
  int gx_direct = 1;  // GH_GX_DIRECT=0: same-device in-process row shards pack and copy their ghosts' planes (A/B)
  GxPeers gx_pub{};   // what this shard publishes for the direct gather (entry 0)
  int side_order = 0;  // GH_SIDE_ORDER=1: the side stream's idle variants as IN 1, IN 3, storm, IN 6 (A/B)
  int32_t* vlog = nullptr;
  int64_t vlog_cap = 0;
  // |D| of the last round as read at the end of gh_step (one engine; -1
  // unknown): a first round with a REMOVE pending launches IN 6 on a full grid
  int32_t last_nd = -1;
  std::string err;
  std::vector<void*> allocs;
};

int set_err(Engine* e, int code, const std::string& msg) {
  if (e) e->err = msg;
  return code;
}

#define HIPCHK(e, call)                                                          \
  do {                                                                           \
    hipError_t _st = (call);                                                     \
    if (_st != hipSuccess)                                                       \
      return set_err((e), GH_EHIP, std::string(#call) + ": " + hipGetErrorString(_st)); \
  } while (0)

#define COMMCHK(e, call)                                                          \
  do {                                                                            \
    if ((call) != 0) return set_err((e), GH_EHIP, "collective failed: " + (e)->comm->err); \
  } while (0)

template <class T>
int dalloc(Engine* e, T** p, size_t count, int fill_byte) {
  void* q = nullptr;
  const size_t bytes = std::max<size_t>(count * sizeof(T), 16);
  if (e->dry) {  // gh_footprint: count the bytes, allocate nothing
    e->dry_bytes += (int64_t)bytes;
    *p = nullptr;
    return GH_OK;
  }
  if (hipMalloc(&q, bytes) != hipSuccess) {
    (void)hipGetLastError();
    return set_err(e, GH_ENOMEM, "hipMalloc of " + std::to_string(bytes) + " bytes failed");
  }
  e->allocs.push_back(q);
  // on the engine's (non-blocking) stream: a null-stream memset is not
  // ordered with it and could land after the first kernel writing q
  if (hipMemsetAsync(q, fill_byte, bytes, e->stream) != hipSuccess)
    return set_err(e, GH_EHIP, "hipMemsetAsync failed");
  *p = static_cast<T*>(q);
  return GH_OK;
}

// Device staging buffer for import/export/read-outs.
struct Staging {
  void* p = nullptr;
  int alloc(Engine* e, size_t bytes) {
    if (hipMalloc(&p, std::max<size_t>(bytes, 16)) != hipSuccess) {
      (void)hipGetLastError();
      p = nullptr;
      return set_err(e, GH_ENOMEM, "staging allocation failed");
    }
    return GH_OK;
  }
  template <class T>
  T* as() const {
    return static_cast<T*>(p);
  }
  ~Staging() {
    if (p) (void)hipFree(p);
  }
};

GhRound round_params(const Engine* e, int32_t r) {
  GhRound p{};
  p.r = r;
  p.n = e->n;
  p.ld = e->ld;
  p.t_fail = e->cfg.t_fail;
  p.t_cleanup = e->cfg.t_cleanup;
  p.min_members = e->cfg.min_members;
  p.k = e->cfg.fanout;
  p.seed = e->cfg.seed;
  p.peer_mode = e->cfg.peer_mode;
  p.xmap = e->xmap;
  p.tpw = e->tpw;
  p.force_storm = e->force_storm;
  p.force_slow = e->force_slow;
  p.nib_rmv = e->nib_rmv;
  p.nib_dma = e->nib_dma;
  p.shadow_row = e->shadow_any ? e->cfg.introducer : -1;
  p.plane = e->plane;
  // (a row shard holds its senders' whole rows: their lists)
  p.ring_whole = (e->world == 1 || e->rowlay) && e->flags_known;
  return p;
}

// Releases one allocation made by dalloc.
void dfree(Engine* e, void* p) {
  if (!p) return;
  auto it = std::find(e->allocs.begin(), e->allocs.end(), p);
  if (it != e->allocs.end()) e->allocs.erase(it);
  (void)hipFree(p);
}

int upload_frow(Engine* e) {
  HIPCHK(e, hipMemcpyAsync(e->d.frow, e->frow.data(), sizeof(int32_t) * e->n, hipMemcpyHostToDevice, e->stream));
  HIPCHK(e, hipStreamSynchronize(e->stream));
  return GH_OK;
}

// Frozen-store slots for rows that stop (growing the store), then their
// exact cells into it and GH_N_FROZEN into both buffers. rows_dev holds the
// same ids on the device.
int freeze_rows(Engine* e, const std::vector<int32_t>& rows, const int32_t* rows_dev, const GhRound& p) {
  if (rows.empty()) return GH_OK;
  GhDev& d = e->d;
  int64_t need = 0;
  for (int32_t i : rows)
    if (e->frow[i] < 0) need++;
  if (need > (int64_t)e->fz_free.size()) {
    const int64_t cap = std::max<int64_t>(e->fzcap + need - (int64_t)e->fz_free.size(),
                                          std::min<int64_t>(2 * e->fzcap + 16, e->n));
    int32_t *h = nullptr, *t = nullptr;
    int rc;
    if ((rc = dalloc(e, &h, (size_t)cap * e->ld, 0xFF)) || (rc = dalloc(e, &t, (size_t)cap * e->ld, 0))) return rc;
    if (e->fzcap > 0) {
      HIPCHK(e, hipMemcpyAsync(h, d.fzh, sizeof(int32_t) * e->fzcap * e->ld, hipMemcpyDeviceToDevice, e->stream));
      HIPCHK(e, hipMemcpyAsync(t, d.fzt, sizeof(int32_t) * e->fzcap * e->ld, hipMemcpyDeviceToDevice, e->stream));
    }
    HIPCHK(e, hipStreamSynchronize(e->stream));
    dfree(e, d.fzh);
    dfree(e, d.fzt);
    d.fzh = h;
    d.fzt = t;
    for (int64_t q = cap - 1; q >= e->fzcap; --q) e->fz_free.push_back((int32_t)q);
    e->fzcap = cap;
  }
  for (int32_t i : rows)
    if (e->frow[i] < 0) {
      e->frow[i] = e->fz_free.back();
      e->fz_free.pop_back();
    }
  int rc;
  if ((rc = upload_frow(e))) return rc;
  launch_freeze(d, e->cur, rows_dev, (int32_t)rows.size(), p, e->stream);
  HIPCHK(e, hipGetLastError());
  HIPCHK(e, hipStreamSynchronize(e->stream));
  return GH_OK;
}

// Rows that run again (join of a stopped member, import, init_full) after
// their segments were rewritten: their frozen-store slots are free.
int release_rows(Engine* e, const std::vector<int32_t>& rows) {
  bool any = false;
  for (int32_t i : rows)
    if (e->frow[i] >= 0) {
      e->fz_free.push_back(e->frow[i]);
      e->frow[i] = -1;
      any = true;
    }
  return any ? upload_frow(e) : GH_OK;
}

// Device error flag: GH_ENOMEM (wide arena overflow in a round) loses the
// state; the caller decides what else may be recovered.
int read_err(Engine* e, int32_t* err) {
  HIPCHK(e, hipMemcpyAsync(err, e->d.err, sizeof(int32_t), hipMemcpyDeviceToHost, e->stream));
  HIPCHK(e, hipStreamSynchronize(e->stream));
  return GH_OK;
}

// The device state is gone after an arena overflow inside a round.
int check_lost(Engine* e) {
  if (!e->lost.empty()) return set_err(e, GH_ENOMEM, e->lost);
  return GH_OK;
}
int lose(Engine* e, const char* where) {
  e->lost = std::string(where) + ": the wide-segment arena overflowed (" + std::to_string(e->d.wcap) +
            " slots per buffer); the engine state is lost. Raise gh_config.wide_segments.";
  return set_err(e, GH_ENOMEM, e->lost);
}

// Slots of the wide arena per buffer (DESIGN.md "Data layout"): the
// configured count, else every segment when that is small, else 1/32 of
// them, at least 2^26 cells' worth (grown between calls when half full).
int64_t arena_slots(const gh_config* cfg, int64_t segs, int tw) {
  if (cfg->wide_segments > 0) return std::min<int64_t>(cfg->wide_segments, segs);
  const int64_t slot_bytes = (int64_t)tw * 8 + tw / 8;
  if (2 * segs * slot_bytes <= (int64_t)2 << 30) return segs;
  return std::max<int64_t>(std::min<int64_t>(segs, ((int64_t)1 << 26) / tw), segs / 32);
}

// Grows both wide arenas to `cap` slots, keeping the current buffer's slots
// (same indices, so its chunks' slot numbers stay valid).
int grow_arena(Engine* e, int64_t cap) {
  GhDev& d = e->d;
  int32_t used = 0;
  HIPCHK(e, hipMemcpyAsync(&used, d.wn + e->cur, sizeof used, hipMemcpyDeviceToHost, e->stream));
  HIPCHK(e, hipStreamSynchronize(e->stream));
  used = (int32_t)std::min<int64_t>(used, d.wcap);
  const int64_t tw = d.tw;
  for (int b = 0; b < 2; ++b) {
    int32_t *h = nullptr, *t = nullptr;
    uint8_t* f = nullptr;
    int rc;
    if ((rc = dalloc(e, &h, (size_t)cap * tw, 0xFF)) || (rc = dalloc(e, &t, (size_t)cap * tw, 0)) ||
        (rc = dalloc(e, &f, (size_t)cap * tw / 8, 0)))
      return rc;
    if (b == e->cur && used > 0) {
      HIPCHK(e, hipMemcpyAsync(h, d.wh[b], sizeof(int32_t) * used * tw, hipMemcpyDeviceToDevice, e->stream));
      HIPCHK(e, hipMemcpyAsync(t, d.wt[b], sizeof(int32_t) * used * tw, hipMemcpyDeviceToDevice, e->stream));
      HIPCHK(e, hipMemcpyAsync(f, d.wf[b], (size_t)used * tw / 8, hipMemcpyDeviceToDevice, e->stream));
    }
    HIPCHK(e, hipStreamSynchronize(e->stream));
    dfree(e, d.wh[b]);
    dfree(e, d.wt[b]);
    dfree(e, d.wf[b]);
    d.wh[b] = h;
    d.wt[b] = t;
    d.wf[b] = f;
  }
  d.wcap = cap;
  // allocations past the old capacity were refused (never written)
  HIPCHK(e, hipMemcpyAsync(d.wn + e->cur, &used, sizeof used, hipMemcpyHostToDevice, e->stream));
  HIPCHK(e, hipStreamSynchronize(e->stream));
  return GH_OK;
}

// Before and between rounds: grow the arena when the current buffer of any
// shard uses more than half of it. Every decision is collective (one
// allreduce(max) of the shards' flags), so all shards run the same
// collectives after it: *busy = some shard uses more than a quarter (gh_step
// then checks after every round); check_err: an arena overflow of the last
// round on any shard loses the state on every shard. The arena caps and
// segs_all are the same on every shard, so the early return is too.
int maybe_grow(Engine* e, bool* busy = nullptr, bool check_err = false) {
  GhDev& d = e->d;
  const int64_t segs = e->segs_all;
  if (busy) *busy = false;
  if (d.wcap >= segs) return GH_OK;  // every segment fits: no overflow, nothing to grow
  int32_t used = 0, err = 0;
  HIPCHK(e, hipMemcpyAsync(&used, d.wn + e->cur, sizeof used, hipMemcpyDeviceToHost, e->stream));
  if (check_err) HIPCHK(e, hipMemcpyAsync(&err, d.err, sizeof err, hipMemcpyDeviceToHost, e->stream));
  HIPCHK(e, hipStreamSynchronize(e->stream));
  int32_t v[3] = {2 * (int64_t)used > d.wcap ? 1 : 0, 4 * (int64_t)used > d.wcap ? 1 : 0, err == GH_ENOMEM ? 1 : 0};
  int32_t* flag = d.wn + 4;
  HIPCHK(e, hipMemcpyAsync(flag, v, sizeof v, hipMemcpyHostToDevice, e->stream));
  COMMCHK(e, e->comm->allreduce(flag, flag, 3, GH_DT_I32, GH_OP_MAX, e->stream));
  HIPCHK(e, hipMemcpyAsync(v, flag, sizeof v, hipMemcpyDeviceToHost, e->stream));
  HIPCHK(e, hipStreamSynchronize(e->stream));
  if (v[2]) return lose(e, "gh_step");
  if (busy) *busy = v[1] != 0;
  if (!v[0]) return GH_OK;
  return grow_arena(e, std::min<int64_t>(segs, 2 * d.wcap));
}

int reset_pending_removes(Engine* e) {
  GhDev& d = e->d;
  for (int b = 0; b < 2; ++b) {
    HIPCHK(e, hipMemsetAsync(d.det_cnt[b], 0, sizeof(int32_t) * e->ld, e->stream));
    HIPCHK(e, hipMemsetAsync(d.det_min[b], 0x7F, sizeof(int32_t) * e->ld, e->stream));
  }
  HIPCHK(e, hipMemsetAsync(d.dbits, 0, sizeof(uint32_t) * (e->ld / 32 + 2), e->stream));
  HIPCHK(e, hipMemsetAsync(d.sbits, 0, sizeof(uint32_t) * (e->ld / 32 + 2), e->stream));
  HIPCHK(e, hipMemsetAsync(d.nd, 0, sizeof(int32_t) * 8, e->stream));
  HIPCHK(e, hipMemsetAsync(d.det_any, 0, e->n, e->stream));
  e->last_nd = 0;  // (only the rounds and this reset write nd[0..1])
  return GH_OK;
}

int upload_alive(Engine* e) {
  HIPCHK(e, hipMemcpyAsync(e->d.alive, e->alive.data(), e->n, hipMemcpyHostToDevice, e->stream));
  HIPCHK(e, hipStreamSynchronize(e->stream));
  return GH_OK;
}

int upload(Engine* e, int32_t* dst, const std::vector<int32_t>& v) {
  if (v.empty()) return GH_OK;
  HIPCHK(e, hipMemcpyAsync(dst, v.data(), v.size() * sizeof(int32_t), hipMemcpyHostToDevice, e->stream));
  HIPCHK(e, hipStreamSynchronize(e->stream));
  return GH_OK;
}

// Presence bitmaps of rows[0..nr) (device ids) over ALL members, gathered
// from every shard into d.rbits [world][nr][ncsw].
int gather_rows(Engine* e, const int32_t* rows_dev, int32_t nr) {
  GhDev& d = e->d;
  if (nr > e->rbits_rows) {
    uint32_t* nb = nullptr;
    int rc;
    if ((rc = dalloc(e, &nb, (size_t)e->world * nr * d.ncsw, 0))) return rc;
    d.rbits = nb;  // the old buffer stays in allocs until gh_destroy
    e->rbits_rows = nr;
  }
  launch_rowbits(d, e->cur, rows_dev, nr, e->stream);
  HIPCHK(e, hipGetLastError());
  if (e->rowlay) {  // slice 0: the owner's bits, zeros elsewhere -> their sum
    COMMCHK(e, e->comm->allreduce(d.rbits, d.rbits, (size_t)nr * d.ncsw, GH_DT_I32, GH_OP_SUM, e->stream));
    return GH_OK;
  }
  const size_t bytes = sizeof(uint32_t) * (size_t)nr * d.ncsw;
  COMMCHK(e, e->comm->allgather(d.rbits + (size_t)e->rank * nr * d.ncsw, d.rbits, bytes, e->stream));
  return GH_OK;
}

// ---- row layout: ghost rows ------------------------------------------------
int row_owner(const Engine* e, int64_t i) { return (int)(i / e->nrs); }

// Device scratch b of at least `bytes` (grown, never shrunk).
int gbuf_reserve(Engine* e, int b, size_t bytes) {
  if (bytes <= e->gcap_bytes[b]) return GH_OK;
  dfree(e, e->gbuf[b]);
  e->gbuf[b] = nullptr;
  e->gcap_bytes[b] = 0;
  char* q = nullptr;
  int rc;
  if ((rc = dalloc(e, &q, bytes, 0))) return rc;
  e->gbuf[b] = q;
  e->gcap_bytes[b] = bytes;
  return GH_OK;
}

// Send staging of one ghost_move chunk (the parts travel in chunks of at
// most this many bytes per shard).
constexpr int64_t kGhostChunk = (int64_t)1 << 30;

// Every shard calls this with the same `want` (want[r]: the rows rank r needs
// and does not own, ascending). Its own wants become ghost j = slot nrows + j
// (ascending, so grouped by owner); the rows it owns that other ranks want
// are its send lists. The previous ghosts are dropped; nothing moves yet
// (ghost_move).
// The ghost table holds at least nr rows (its rows are rewritten every round).
int ghost_reserve(Engine* e, int64_t nr) {
  GhDev& d = e->d;
  if (nr > d.gcap) {
    const int64_t cap = std::max<int64_t>(nr, d.gcap + d.gcap / 4);
    dfree(e, d.gcodes);
    dfree(e, d.gplane);
    d.gcodes = nullptr;
    d.gplane = nullptr;
    d.gcap = 0;
    int rc;
    if ((rc = dalloc(e, &d.gcodes, (size_t)cap * e->ld, 0xFF))) return rc;
    if (e->plane && (rc = dalloc(e, &d.gplane, (size_t)cap * e->ld / 8, 0xFF))) return rc;
    d.gcap = cap;
  }
  return GH_OK;
}

int ghost_setup(Engine* e, const std::vector<std::vector<int32_t>>& want) {
  GhDev& d = e->d;
  const int G = e->world, me = e->rank;
  for (int32_t s : e->ghosts) e->rslot_h[s] = -1;
  e->ghosts = want[me];
  e->gx_dev = false;
  const int64_t nr = (int64_t)e->ghosts.size();
  int rc;
  if ((rc = ghost_reserve(e, nr))) return rc;
  e->gx_rcnt.assign(G, 0);
  e->gx_rbeg.assign(G, 0);
  for (int64_t j = 0; j < nr; ++j) {
    e->rslot_h[e->ghosts[j]] = (int32_t)(d.nrows + j);
    e->gx_rcnt[row_owner(e, e->ghosts[j])]++;
  }
  for (int r = 1; r < G; ++r) e->gx_rbeg[r] = e->gx_rbeg[r - 1] + e->gx_rcnt[r - 1];
  e->gx_send.assign(G, {});
  e->gx_sn.assign(G, 0);
  e->gx_soff.assign(G, 0);
  std::vector<int64_t> sends(G, 0);  // every shard's send rows (replicated wants: the same everywhere)
  for (int r = 0; r < G; ++r)
    for (int32_t s : want[r]) {
      const int o = row_owner(e, s);
      sends[o]++;
      if (o == me) e->gx_send[r].push_back(s);
    }
  for (int r = 0; r < G; ++r) e->gx_sn[r] = (int64_t)e->gx_send[r].size();
  e->gx_maxsend = *std::max_element(sends.begin(), sends.end());
  e->gx_rows = nr;
  e->gx_out = e->gx_in = 0;
  HIPCHK(e, hipMemcpyAsync(d.rslot, e->rslot_h.data(), sizeof(int32_t) * e->n, hipMemcpyHostToDevice, e->stream));
  return GH_OK;
}

// device list of rows (and their destinations) in gidx
int upload_rows(Engine* e, const std::vector<int32_t>& rows, const std::vector<int32_t>& dst) {
  const int64_t ns = (int64_t)rows.size();
  if (ns > e->gidx_cap) {
    dfree(e, e->gidx);
    e->gidx = nullptr;
    e->gidx_cap = 0;
    int rc;
    if ((rc = dalloc(e, &e->gidx, 2 * std::max<int64_t>(ns, 1024), 0))) return rc;
    e->gidx_cap = std::max<int64_t>(ns, 1024);
  }
  if (ns) {
    HIPCHK(e, hipMemcpyAsync(e->gidx, rows.data(), sizeof(int32_t) * ns, hipMemcpyHostToDevice, e->stream));
    HIPCHK(e, hipMemcpyAsync(e->gidx + e->gidx_cap, dst.data(), sizeof(int32_t) * ns, hipMemcpyHostToDevice,
                             e->stream));
  }
  return GH_OK;
}

// Moves one part of the set-up ghost rows (GH_GX_PLANE: sender plane words,
// GH_GX_CODES: 16-bit codes and then the wide segments' exact cells) from
// their owners straight into the ghost table, by alltoallv with receive
// displacements, in C chunks (the same C on every shard): chunk c carries
// rows [c*n/C, (c+1)*n/C) of every (source, destination) list.
// The rows (and destinations) of slice [lo_r, hi_r) of every send list into
// gidx: uploaded from the host lists, or gathered on the device from the
// want lists (gx_dev). Returns the row count.
int send_rows(Engine* e, const std::vector<int64_t>& lo, const std::vector<int64_t>& hi, int64_t* ns) {
  const int G = e->world;
  if (!e->gx_dev) {
    std::vector<int32_t> rows, dst;
    for (int r = 0; r < G; ++r)
      for (int64_t x = lo[r]; x < hi[r]; ++x) {
        rows.push_back(e->gx_send[r][x]);
        dst.push_back(r);
      }
    *ns = (int64_t)rows.size();
    return upload_rows(e, rows, dst);
  }
  GxSlices sl{};
  sl.g = G;
  sl.out[0] = 0;
  for (int r = 0; r < G; ++r) {
    sl.src[r] = e->gx_soff[r] + lo[r];
    sl.out[r + 1] = sl.out[r] + (hi[r] - lo[r]);
  }
  sl.total = sl.out[G];
  *ns = sl.total;
  if (sl.total > e->gidx_cap) {
    dfree(e, e->gidx);
    e->gidx = nullptr;
    e->gidx_cap = 0;
    int rc;
    if ((rc = dalloc(e, &e->gidx, 2 * std::max<int64_t>(sl.total, 1024), 0))) return rc;
    e->gidx_cap = std::max<int64_t>(sl.total, 1024);
  }
  launch_gx_idx(e->wlist, e->n, sl, e->gidx, e->gidx + e->gidx_cap, e->stream);
  HIPCHK(e, hipGetLastError());
  return GH_OK;
}

int ghost_move(Engine* e, int part) {
  GhDev& d = e->d;
  const int G = e->world;
  if (part == GH_GX_PLANE && e->gx_dev && e->gx_direct && d.tw >= 32 && G <= kGxPeers) {
    // same-device in-process shards: every shard gathers its ghosts' plane
    // rows from their owners' tables (the owners publish their planes)
    e->gx_pub.pl[0] = d.pl[e->cur];
    e->gx_pub.row0[0] = d.row0;
    e->gx_pub.tstride[0] = d.tstride;
    const void* all[kGxPeers] = {};
    const int rc = e->comm->share(&e->gx_pub, e->stream, all);
    if (rc < 0) return set_err(e, GH_EHIP, "collective failed: " + e->comm->err);
    if (rc == 0) {
      GxPeers pp{};
      for (int h = 0; h < G; ++h) {
        const GxPeers* o = static_cast<const GxPeers*>(all[h]);
        pp.pl[h] = o->pl[0];
        pp.row0[h] = o->row0[0];
        pp.tstride[h] = o->tstride[0];
      }
      launch_ghost_gather_plane(d, pp, e->wlist + (size_t)e->rank * e->n, e->gx_rows, e->nrs, e->stream);
      HIPCHK(e, hipGetLastError());
      COMMCHK(e, e->comm->share_done(e->stream));
      const int64_t B = ghost_part_bytes(d, part);
      for (int r = 0; r < G; ++r) {
        e->gx_out += e->gx_sn[r] * B;
        e->gx_in += e->gx_rcnt[r] * B;
      }
      return GH_OK;
    }
  }
  const int64_t B = ghost_part_bytes(d, part);
  const int64_t C = std::max<int64_t>(1, (e->gx_maxsend * B + kGhostChunk - 1) / kGhostChunk);
  char* region = part == GH_GX_PLANE ? reinterpret_cast<char*>(d.gplane) : reinterpret_cast<char*>(d.gcodes);
  int rc;
  if (part == GH_GX_CODES) HIPCHK(e, hipMemsetAsync(e->gwcnt, 0, sizeof(int32_t) * G, e->stream));
  std::vector<size_t> sb(G), rb(G), rd(G);
  std::vector<int64_t> lo(G), hi(G);
  for (int64_t c = 0; c < C; ++c) {
    for (int r = 0; r < G; ++r) {
      const int64_t m = e->gx_sn[r];
      lo[r] = c * m / C;
      hi[r] = (c + 1) * m / C;
      sb[r] = (size_t)(hi[r] - lo[r]) * B;
      const int64_t q = e->gx_rcnt[r], qlo = c * q / C, qhi = (c + 1) * q / C;
      rb[r] = (size_t)(qhi - qlo) * B;
      rd[r] = (size_t)(e->gx_rbeg[r] + qlo) * B;
    }
    int64_t ns = 0;
    if ((rc = send_rows(e, lo, hi, &ns)) || (rc = gbuf_reserve(e, 0, (size_t)std::max<int64_t>(ns, 1) * B)))
      return rc;
    launch_ghost_pack(d, e->cur, e->gidx, e->gidx + e->gidx_cap, ns, part,
                      static_cast<char*>(e->gbuf[0]), e->gwcnt, e->stream);
    HIPCHK(e, hipGetLastError());
    COMMCHK(e, e->comm->alltoallv(e->gbuf[0], sb.data(), region, rb.data(), e->stream, rd.data()));
    for (int r = 0; r < G; ++r) {
      e->gx_out += (int64_t)sb[r];
      e->gx_in += (int64_t)rb[r];
    }
  }
  if (part != GH_GX_CODES) return GH_OK;
  // wide segments of the sent rows: every shard's per-destination counts
  const int me = e->rank;
  int32_t* mat = e->gwcnt + 2 * G;
  COMMCHK(e, e->comm->allgather(e->gwcnt, mat, sizeof(int32_t) * G, e->stream));
  std::vector<int32_t> m((size_t)G * G);
  HIPCHK(e, hipMemcpyAsync(m.data(), mat, sizeof(int32_t) * G * G, hipMemcpyDeviceToHost, e->stream));
  HIPCHK(e, hipStreamSynchronize(e->stream));
  int64_t any = 0;
  for (int32_t v : m) any += v;
  if (any == 0) return GH_OK;
  const int64_t REC = ghost_wide_record_bytes(d);
  std::vector<int32_t> cur0(G);
  int64_t ws = 0, wr = 0;
  for (int r = 0; r < G; ++r) {
    cur0[r] = (int32_t)ws;
    ws += m[(size_t)me * G + r];  // my records to r
    wr += m[(size_t)r * G + me];  // r's records to me
    sb[r] = (size_t)m[(size_t)me * G + r] * REC;
    rb[r] = (size_t)m[(size_t)r * G + me] * REC;
    lo[r] = 0;
    hi[r] = e->gx_sn[r];
  }
  int64_t ns = 0;
  if ((rc = send_rows(e, lo, hi, &ns)) || (rc = gbuf_reserve(e, 2, (size_t)std::max<int64_t>(ws, 1) * REC)) ||
      (rc = gbuf_reserve(e, 3, (size_t)std::max<int64_t>(wr, 1) * REC)))
    return rc;
  HIPCHK(e, hipMemcpyAsync(e->gwcnt + G, cur0.data(), sizeof(int32_t) * G, hipMemcpyHostToDevice, e->stream));
  launch_ghost_wide(d, e->cur, e->gidx, e->gidx + e->gidx_cap, ns, e->gwcnt + G,
                    static_cast<char*>(e->gbuf[2]), e->stream);
  HIPCHK(e, hipGetLastError());
  COMMCHK(e, e->comm->alltoallv(e->gbuf[2], sb.data(), e->gbuf[3], rb.data(), e->stream));
  e->gx_out += ws * REC;
  e->gx_in += wr * REC;
  launch_ghost_unwide(d, e->cur, static_cast<const char*>(e->gbuf[3]), wr, e->stream);
  HIPCHK(e, hipGetLastError());
  return GH_OK;
}

// The whole ghost rows (plane and codes).
int ghost_exchange(Engine* e, const std::vector<std::vector<int32_t>>& want) {
  int rc;
  if ((rc = ghost_setup(e, want))) return rc;
  if (e->plane && (rc = ghost_move(e, GH_GX_PLANE))) return rc;
  return ghost_move(e, GH_GX_CODES);
}

// Row layout: the exchange staging ghost_move grows during the rounds, at
// the expected size of a healthy Philox-pull round: each of the shard's
// nrows receivers draws k senders uniformly from the N - 1 others, so the
// distinct remote senders (the ghost rows received, and by symmetry the rows
// sent) are (N - nrows) * (1 - (1 - 1/(N-1))^(k * nrows)); the send side is
// staged one chunk at a time. Column layout: 0 (its exchanges are O(N)
// vectors allocated by create).
int64_t exchange_footprint(const Engine* e) {
  if (!e->rowlay || e->world < 2) return 0;
  const double n = (double)e->n, nr = (double)e->d.nrows, k = (double)e->cfg.fanout;
  const int64_t distinct = (int64_t)std::ceil((n - nr) * (1.0 - std::pow(1.0 - 1.0 / (n - 1.0), k * nr)));
  // one chunk of send staging (the ghost table is allocated by create)
  return std::min<int64_t>(kGhostChunk, distinct * e->ld * 2);
}

// The round's ghosts: the senders of each shard's receivers that other
// shards own, from the (replicated) pull inboxes. A healthy round (no shard
// in the storm variant, the plane valid) moves only their sender planes
// (e->gpo; the codes follow after k_round if a segment needs the per-cell
// rule), any other round the whole rows.
int round_ghosts(Engine* e, const GhRound& p) {
  const int G = e->world, me = e->rank;
  if (G <= GH_GX_MAXG) {
    // the want lists on the device: the host reads back G x G counts only
    GhDev& d = e->d;
    launch_want_lists(d, p, e->nrs, G, e->wbits, e->wsum, e->wlist, e->mcnt, e->stream);
    HIPCHK(e, hipGetLastError());
    int32_t storm = 0;  // shards in the storm variant (summed by decide_active)
    e->gx_m.resize((size_t)G * G + G);
    HIPCHK(e, hipMemcpyAsync(e->gx_m.data(), e->mcnt, sizeof(int32_t) * e->gx_m.size(), hipMemcpyDeviceToHost,
                             e->stream));
    HIPCHK(e, hipMemcpyAsync(&storm, d.cntg + e->n + 2, sizeof storm, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(e, hipStreamSynchronize(e->stream));
    const int32_t* M = e->gx_m.data();
    int rc;
    if ((rc = ghost_reserve(e, M[G * G + me]))) return rc;
    for (int32_t s : e->ghosts) e->rslot_h[s] = -1;  // host-set ghosts (a join broadcast) are gone
    e->ghosts.clear();
    e->gx_dev = true;
    e->gx_rcnt.assign(G, 0);
    e->gx_rbeg.assign(G, 0);
    e->gx_sn.assign(G, 0);
    e->gx_soff.assign(G, 0);
    std::vector<int64_t> sends(G, 0);
    for (int r = 0; r < G; ++r)
      for (int o = 0; o < G; ++o) {
        const int64_t c = M[r * G + o];
        sends[o] += c;
        if (o < me) e->gx_soff[r] += c;
      }
    for (int r = 0; r < G; ++r) {
      e->gx_rcnt[r] = M[me * G + r];
      e->gx_sn[r] = M[r * G + me];
      if (r) e->gx_rbeg[r] = e->gx_rbeg[r - 1] + e->gx_rcnt[r - 1];
    }
    e->gx_maxsend = *std::max_element(sends.begin(), sends.end());
    e->gx_rows = M[G * G + me];
    e->gx_out = e->gx_in = 0;
    launch_ghost_slots(d, e->wlist + (size_t)me * e->n, e->mcnt + G * G + me, e->stream);
    HIPCHK(e, hipGetLastError());
    // (list order: the list kernels read the ghost senders' flags, so their
    // 16-bit codes travel every round)
    e->gpo = e->plane && e->plane_valid && storm == 0 && !e->lorder;
    if (e->plane && (rc = ghost_move(e, GH_GX_PLANE))) return rc;
    return e->gpo ? GH_OK : ghost_move(e, GH_GX_CODES);
  }
  const int k = e->cfg.fanout;
  const bool pull = e->cfg.peer_mode == GH_PEER_PULL;
  // pull: [n][k + 1] (count, senders); ring: CSR (beg, cnt) into <= 3N senders
  std::vector<int32_t> inbox(pull ? (size_t)e->n * (k + 1) : 3 * (size_t)e->n), beg, cnt;
  int32_t storm = 0;  // shards in the storm variant (summed by decide_active)
  HIPCHK(e, hipMemcpyAsync(inbox.data(), e->d.inbox, sizeof(int32_t) * inbox.size(), hipMemcpyDeviceToHost,
                           e->stream));
  if (!pull) {
    beg.resize(e->n);
    cnt.resize(e->n);
    HIPCHK(e, hipMemcpyAsync(beg.data(), e->d.inbox_beg, sizeof(int32_t) * e->n, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(e, hipMemcpyAsync(cnt.data(), e->d.inbox_cnt, sizeof(int32_t) * e->n, hipMemcpyDeviceToHost, e->stream));
  }
  HIPCHK(e, hipMemcpyAsync(&storm, e->d.cntg + e->n + 2, sizeof storm, hipMemcpyDeviceToHost, e->stream));
  HIPCHK(e, hipStreamSynchronize(e->stream));
  std::vector<std::vector<uint8_t>> mark(G, std::vector<uint8_t>(e->n, 0));
  for (int64_t i = 0; i < e->n; ++i) {
    const int r = row_owner(e, i);
    const int32_t* b = pull ? inbox.data() + i * (k + 1) + 1 : inbox.data() + beg[i];
    const int nb = pull ? b[-1] : cnt[i];
    for (int q = 0; q < nb; ++q)
      if (row_owner(e, b[q]) != r) mark[r][b[q]] = 1;
  }
  std::vector<std::vector<int32_t>> want(G);
  for (int r = 0; r < G; ++r)
    for (int32_t s = 0; s < e->n; ++s)
      if (mark[r][s]) want[r].push_back(s);
  e->gpo = e->plane && e->plane_valid && storm == 0 && !e->lorder;
  if (!e->gpo) return ghost_exchange(e, want);
  int rc;
  if ((rc = ghost_setup(e, want))) return rc;
  return ghost_move(e, GH_GX_PLANE);
}

// After k_round in a plane-only round: the ghosts' 16-bit codes, when any
// shard's k_round listed segments for k_round_slow (one collective decision).
int ghost_codes_if_slow(Engine* e) {
  if (!e->rowlay || e->world < 2 || !e->gpo) return GH_OK;
  // segments for k_round_slow, or (4-bit tier) lane jobs that gather their
  // senders' codes (a REMOVE'd member, an unknown or old minimum)
  int32_t* flag = e->d.wn + 4;
  HIPCHK(e, hipMemcpyAsync(flag, e->d.slow_n, sizeof(int32_t), hipMemcpyDeviceToDevice, e->stream));
  if (e->c8)
    HIPCHK(e, hipMemcpyAsync(flag + 1, e->d.m8 + 5, sizeof(int32_t), hipMemcpyDeviceToDevice, e->stream));
  else
    HIPCHK(e, hipMemsetAsync(flag + 1, 0, sizeof(int32_t), e->stream));
  COMMCHK(e, e->comm->allreduce(flag, flag, 2, GH_DT_I32, GH_OP_MAX, e->stream));
  int32_t any[2] = {0, 0};
  HIPCHK(e, hipMemcpyAsync(any, flag, sizeof any, hipMemcpyDeviceToHost, e->stream));
  HIPCHK(e, hipStreamSynchronize(e->stream));
  return any[0] > 0 || any[1] > 0 ? ghost_move(e, GH_GX_CODES) : GH_OK;
}

int allreduce_i32(Engine* e, int32_t* send, int32_t* recv, size_t count) {
  COMMCHK(e, e->comm->allreduce(send, recv, count, GH_DT_I32, GH_OP_SUM, e->stream));
  return GH_OK;
}

// SPEC.md §5: crashes, then leaves (all leavers stop first), then joins.
int reset_shadows(Engine* e);

// Row shards with list order: every shard keeps every row's list; the lists
// of generation g this shard's owned rows changed (lchg) go to every other
// shard. The host reads the changed rows' lengths (one sync) and counts the
// entries per range of R rows (R * ld <= 2^26 entries: the pack's int32
// offsets cannot wrap and its scratch stays bounded, G x 256 MiB at most);
// the shards allgather those counts, then for each range any shard changed:
// pack, allgather the packs (sized by the largest), unpack the others' into
// the replicas. An import or a join broadcast changes every row (~N^2 / G
// entries per shard) and takes N / R ranges; a round changes a few rows.
int list_sync(Engine* e, int g) {
  if (!e->d.lchg) return GH_OK;
  GhDev& d = e->d;
  const int G = e->world;
  std::vector<int32_t> chg(e->n), len(e->n);
  HIPCHK(e, hipMemcpyAsync(chg.data(), d.lchg, sizeof(int32_t) * e->n, hipMemcpyDeviceToHost, e->stream));
  HIPCHK(e, hipMemcpyAsync(len.data(), d.llen[g], sizeof(int32_t) * e->n, hipMemcpyDeviceToHost, e->stream));
  HIPCHK(e, hipStreamSynchronize(e->stream));
  const int64_t R = std::max<int64_t>(1, ((int64_t)1 << 26) / std::max<int64_t>(e->ld, 1));
  const int64_t nch = (e->n + R - 1) / R;
  std::vector<int32_t> cnt(nch, 0);
  for (int64_t i = 0; i < e->n; ++i)
    if (chg[i]) cnt[i / R] += len[i] + 1;  // entries + 1: a changed row with an empty list travels too (<= R (ld + 1))
  int rc;
  if ((rc = gbuf_reserve(e, 2, sizeof(int32_t) * nch)) || (rc = gbuf_reserve(e, 3, sizeof(int32_t) * nch * G)))
    return rc;
  HIPCHK(e, hipMemcpyAsync(e->gbuf[2], cnt.data(), sizeof(int32_t) * nch, hipMemcpyHostToDevice, e->stream));
  COMMCHK(e, e->comm->allgather(e->gbuf[2], e->gbuf[3], sizeof(int32_t) * nch, e->stream));
  std::vector<int32_t> all((size_t)nch * G);
  HIPCHK(e, hipMemcpyAsync(all.data(), e->gbuf[3], sizeof(int32_t) * nch * G, hipMemcpyDeviceToHost, e->stream));
  HIPCHK(e, hipStreamSynchronize(e->stream));
  for (int64_t c = 0; c < nch; ++c) {
    int64_t maxent = -1;
    for (int r = 0; r < G; ++r) maxent = std::max<int64_t>(maxent, all[(size_t)r * nch + c]);
    const int64_t lo = c * R, hi = std::min<int64_t>(lo + R, e->n);
    if (maxent <= 0) continue;  // no shard changed a row of the range
    const size_t words = 1 + 4 * (size_t)(hi - lo) + (size_t)maxent;  // (maxent bounds the entries)
    if ((rc = gbuf_reserve(e, 2, words * sizeof(int32_t))) || (rc = gbuf_reserve(e, 3, words * sizeof(int32_t) * G)))
      return rc;
    int32_t* sendb = static_cast<int32_t*>(e->gbuf[2]);
    int32_t* recvb = static_cast<int32_t*>(e->gbuf[3]);
    launch_list_pack(d, g, sendb, lo, hi, e->stream);
    HIPCHK(e, hipGetLastError());
    COMMCHK(e, e->comm->allgather(sendb, recvb, words * sizeof(int32_t), e->stream));
    for (int r = 0; r < G; ++r)
      if (r != e->rank) launch_list_unpack(d, g, recvb + (size_t)r * words, lo, hi, e->stream);
    HIPCHK(e, hipGetLastError());
  }
  return GH_OK;
}

int process_events(Engine* e, int32_t r) {
  if (e->pending.empty()) return GH_OK;
  e->qforce = true;
  e->flags_known = false;
  e->sforce = true;
  const GhRound p = round_params(e, r);
  std::vector<gh_event> ev;
  ev.swap(e->pending);
  std::vector<int32_t> stopped;  // rows that stop running this round
  for (const auto& x : ev)
    if (x.kind == GH_EV_CRASH && e->alive[x.member]) {
      e->alive[x.member] = 0;
      stopped.push_back(x.member);
    }
  std::vector<int32_t> leavers;
  for (const auto& x : ev)
    if (x.kind == GH_EV_LEAVE && e->alive[x.member]) {
      e->alive[x.member] = 0;
      leavers.push_back(x.member);
      stopped.push_back(x.member);
    }
  int rc;
  if (e->rowlay) {  // a shard freezes and resets only the rows it owns
    std::vector<int32_t> own;
    for (int32_t i : stopped)
      if (gh_owned(e->d, i)) own.push_back(i);
    stopped.swap(own);
  }
  if (!stopped.empty()) {
    if ((rc = upload(e, e->ev_buf, stopped))) return rc;
    if ((rc = freeze_rows(e, stopped, e->ev_buf, p))) return rc;
  }
  if ((rc = upload_alive(e))) return rc;
  if (!leavers.empty()) {
    // the distinct local tiles holding a leaver's column
    std::vector<int32_t> tiles;
    for (int32_t c : leavers) {
      const int64_t lc = (int64_t)c - e->d.col0;
      if (lc >= 0 && lc < e->d.ncol) tiles.push_back((int32_t)(lc / e->d.tw));
    }
    std::sort(tiles.begin(), tiles.end());
    tiles.erase(std::unique(tiles.begin(), tiles.end()), tiles.end());
    std::vector<int32_t> buf(leavers);
    buf.insert(buf.end(), tiles.begin(), tiles.end());
    if ((rc = upload(e, e->ev_buf, buf))) return rc;
    if ((rc = gather_rows(e, e->ev_buf, (int32_t)leavers.size()))) return rc;
    launch_leave(e->d, e->cur, e->ev_buf, e->ev_buf + leavers.size(), (int32_t)tiles.size(),
                 (int32_t)leavers.size(), p, e->stream);
    HIPCHK(e, hipStreamSynchronize(e->stream));
  }
  std::vector<int32_t> joiners, fresh;
  for (const auto& x : ev)
    if (x.kind == GH_EV_JOIN) {
      joiners.push_back(x.member);
      if (!e->alive[x.member]) {
        fresh.push_back(x.member);
        e->alive[x.member] = 1;
      }
    }
  if (e->rowlay) {
    std::vector<int32_t> own;
    for (int32_t i : fresh)
      if (gh_owned(e->d, i)) own.push_back(i);
    fresh.swap(own);
  }
  if (!fresh.empty()) {
    if ((rc = upload(e, e->ev_buf, fresh))) return rc;
    // a restarted introducer starts with empty lists: no shadow entry
    if (std::find(fresh.begin(), fresh.end(), e->cfg.introducer) != fresh.end() && (rc = reset_shadows(e))) return rc;
    launch_join_reset(e->d, e->cur, e->ev_buf, (int32_t)fresh.size(), p, e->stream);
    HIPCHK(e, hipStreamSynchronize(e->stream));
    if ((rc = release_rows(e, fresh))) return rc;
  }
  if ((rc = upload_alive(e))) return rc;
  const int32_t I = e->cfg.introducer;
  if (!joiners.empty() && I >= 0 && I < e->n && e->alive[I]) {
    if ((rc = upload(e, e->ev_buf, joiners))) return rc;
    launch_join_add(e->d, e->cur, e->ev_buf, (int32_t)joiners.size(), I, p, e->stream);
    HIPCHK(e, hipGetLastError());
    e->shadow_any = true;  // a joiner the introducer held tombstoned gets a shadow entry (D7)
    if ((rc = allreduce_i32(e, e->d.nd + 4, e->d.nd + 4, 1))) return rc;
    if ((rc = upload(e, e->rows_buf, {I}))) return rc;
    if ((rc = gather_rows(e, e->rows_buf, 1))) return rc;
    if (e->rowlay && e->world > 1) {  // every shard merges the introducer's row: a ghost of it
      std::vector<std::vector<int32_t>> want(e->world);
      for (int r = 0; r < e->world; ++r)
        if (r != row_owner(e, I)) want[r].push_back(I);
      if ((rc = ghost_exchange(e, want))) return rc;
    }
    launch_join_bcast(e->d, e->cur, I, p, e->stream);
  }
  // (the row counts followed every segment the events rewrote: k_seg)
  HIPCHK(e, hipGetLastError());
  if (e->lorder) {
    // list order (order.hip): a fresh process starts from an empty list;
    // the introducer appends its joiners in event order, every receiver of
    // its broadcast appends what it lacks in the introducer's list order
    for (int32_t j : fresh) HIPCHK(e, hipMemsetAsync(e->d.llen[e->lcur] + j, 0, sizeof(int32_t), e->stream));
    if (!joiners.empty() && I >= 0 && I < e->n && e->alive[I]) {
      if ((rc = upload(e, e->ev_buf, joiners))) return rc;
      if ((rc = upload(e, e->rows_buf, {I}))) return rc;
      launch_list_events(e->d, e->cur, e->lcur, e->rows_buf, 1, e->ev_buf, (int32_t)joiners.size(), -1, -1,
                         e->stream);
      if ((rc = list_sync(e, e->lcur ^ 1))) return rc;  // (row shards: the introducer's new list everywhere)
      launch_list_events(e->d, e->cur, e->lcur, nullptr, 0, nullptr, 0, I, I, e->stream);
    } else {
      launch_list_events(e->d, e->cur, e->lcur, nullptr, 0, nullptr, 0, -1, -1, e->stream);
    }
    HIPCHK(e, hipGetLastError());
    e->lcur ^= 1;
    if ((rc = list_sync(e, e->lcur))) return rc;
  }
  return GH_OK;
}

int ensure_io(Engine* e, int64_t n) {
  if (n <= e->d.io_cap) return GH_OK;
  GhDev& d = e->d;
  const int64_t cap = std::max<int64_t>(n, 1024);
  const int R = e->cfg.replicas;
  int rc;
  if ((rc = dalloc(e, &d.io_a, cap, 0)) || (rc = dalloc(e, &d.io_b, cap * R, 0)) ||
      (rc = dalloc(e, &d.io_c, cap, 0)) || (rc = dalloc(e, &d.io_d, cap, 0)))
    return rc;
  d.io_cap = cap;
  return GH_OK;
}

int check_files(Engine* e, const int32_t* files, int64_t n, bool distinct) {
  if (e->cfg.max_files <= 0) return set_err(e, GH_EINVAL, "engine created with max_files = 0");
  if (n < 0 || (n > 0 && !files)) return set_err(e, GH_EINVAL, "bad file list");
  for (int64_t x = 0; x < n; ++x)
    if (files[x] < 0 || files[x] >= e->cfg.max_files) return set_err(e, GH_EINVAL, "file id out of range");
  if (distinct) {
    std::vector<int32_t> s(files, files + n);
    std::sort(s.begin(), s.end());
    if (std::adjacent_find(s.begin(), s.end()) != s.end())
      return set_err(e, GH_EINVAL, "file ids in one call must be distinct");
  }
  return GH_OK;
}

// Rows [row0, row0+n_rows) of the external hb (what = 0) or ts (what = 1),
// decoded from the tiled local columns of every shard -> host [n_rows][n].
int export_table(Engine* e, int32_t* out, int what, int64_t row0, int64_t n_rows) {
  const GhDev& d = e->d;
  if (e->rowlay) {  // each row from its owner: zeros elsewhere, summed
    const size_t cnt = (size_t)n_rows * d.ncs;
    Staging st;
    int rc;
    if ((rc = st.alloc(e, sizeof(int32_t) * cnt))) return rc;
    HIPCHK(e, hipMemsetAsync(st.p, 0, sizeof(int32_t) * cnt, e->stream));
    launch_unpack(d, e->cur, st.as<int32_t>(), row0, n_rows, what, round_params(e, e->round + 1), e->stream);
    HIPCHK(e, hipGetLastError());
    COMMCHK(e, e->comm->allreduce(st.p, st.p, cnt, GH_DT_I32, GH_OP_SUM, e->stream));
    std::vector<int32_t> host(cnt);
    HIPCHK(e, hipMemcpyAsync(host.data(), st.p, sizeof(int32_t) * cnt, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(e, hipStreamSynchronize(e->stream));
    for (int64_t r = 0; r < n_rows; ++r) std::memcpy(out + r * e->n, host.data() + r * d.ncs, sizeof(int32_t) * e->n);
    return GH_OK;
  }
  const size_t chunk = (size_t)n_rows * d.ncs;  // one shard's [n_rows][ncs]
  Staging st;
  int rc;
  if ((rc = st.alloc(e, sizeof(int32_t) * chunk * e->world))) return rc;
  launch_unpack(d, e->cur, st.as<int32_t>() + chunk * e->rank, row0, n_rows, what, round_params(e, e->round + 1),
                e->stream);
  HIPCHK(e, hipGetLastError());
  COMMCHK(e, e->comm->allgather(st.as<int32_t>() + chunk * e->rank, st.p, sizeof(int32_t) * chunk, e->stream));
  std::vector<int32_t> host(chunk * e->world);
  HIPCHK(e, hipMemcpyAsync(host.data(), st.p, sizeof(int32_t) * host.size(), hipMemcpyDeviceToHost, e->stream));
  HIPCHK(e, hipStreamSynchronize(e->stream));
  for (int g = 0; g < e->world; ++g) {
    const int64_t c0 = (int64_t)g * d.ncs;
    const int64_t nc = std::max<int64_t>(0, std::min<int64_t>(d.ncs, e->n - c0));
    for (int64_t r = 0; r < n_rows && nc > 0; ++r)
      std::memcpy(out + r * e->n + c0, host.data() + chunk * g + r * d.ncs, sizeof(int32_t) * nc);
  }
  return GH_OK;
}

// Ghost table rows of a row shard of nrows receivers: the distinct remote
// senders of a healthy pull round, (N - nrows)(1 - (1 - 1/(N-1))^(k nrows))
// expected, with 5% to spare (ghost_setup grows the table when a round needs
// more).
int64_t ghost_cap(int64_t n, int64_t nrows, int k) {
  const double nn = (double)n, nr = (double)nrows;
  const double dist = (nn - nr) * (1.0 - std::pow(1.0 - 1.0 / std::max(nn - 1.0, 1.0), (double)k * nr));
  return std::min<int64_t>(n - nrows, (int64_t)std::ceil(dist * 1.05) + 64);
}

// dry: gh_footprint's walk of the same allocations with no device, no
// communicator and no memory (*handle = the Engine holding dry_bytes; the
// caller deletes it)
int create(const gh_config* cfg, int32_t rank, int32_t world, int32_t transport, const uint8_t* comm_id,
           void** handle, bool dry = false) {
  if (!cfg || !handle) return GH_EINVAL;
  *handle = nullptr;
  if (cfg->n_members < 1 || cfg->fanout < 1 || cfg->fanout > GH_MAXK || cfg->replicas < 1 ||
      cfg->replicas > 8 || cfg->min_members < 0 || cfg->max_files < 0 || cfg->max_files > INT32_MAX ||
      (cfg->peer_mode != GH_PEER_PULL && cfg->peer_mode != GH_PEER_RING) ||
      (cfg->detect_mode != GH_DETECT_CANONICAL && cfg->detect_mode != GH_DETECT_QUIRK) ||
      cfg->introducer < 0 || cfg->introducer >= cfg->n_members || cfg->master < 0 ||
      cfg->master >= cfg->n_members || cfg->t_fail < 0 || cfg->t_cleanup < 0 || cfg->wide_segments < 0 ||
      (cfg->list_order != GH_ORDER_ID && cfg->list_order != GH_ORDER_APPEND))
    return GH_EINVAL;
  if (world < 1 || rank < 0 || rank >= world) return GH_EINVAL;
  // the list order of a row spans every member column: one engine holds it
  // list order on shards: row shards only (a row's order spans every column)
  if (cfg->list_order == GH_ORDER_APPEND && world > 1 && cfg->shard_layout != GH_LAYOUT_ROWS) return GH_EINVAL;
  // the reference's REMOVE recipients: one engine (a recipient set spans
  // every row and column), member-ID list order (remove.hip)
  if (cfg->remove_mode != GH_REMOVE_ALL && cfg->remove_mode != GH_REMOVE_LIST) return GH_EINVAL;
  if (cfg->remove_mode == GH_REMOVE_LIST && (world > 1 || cfg->list_order != GH_ORDER_ID)) return GH_EINVAL;
  if (world > 1 && !comm_id && !dry) return GH_EINVAL;
  if (transport != GH_COMM_RCCL && transport != GH_COMM_LOCAL) return GH_EINVAL;
  if (!dry) {
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= cfg->device || cfg->device < 0) {
      (void)hipGetLastError();
      return GH_ENODEV;
    }
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, cfg->device) != hipSuccess) return GH_ENODEV;
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) return GH_ENODEV;
    if (hipSetDevice(cfg->device) != hipSuccess) return GH_ENODEV;
  }

  Engine* e = new Engine();
  e->dry = dry;
  e->cfg = *cfg;
  e->n = cfg->n_members;
  e->rank = rank;
  e->world = world;
  e->alive.assign(e->n, 0);
  e->frow.assign(e->n, -1);
  // slower dissemination (k < 3) leaves views outside the plane's window;
  // below GH_PLANE_MIN_N the tables sit in the on-die caches and the round is
  // launch-bound, where 256-member tiles leave too few workgroups
  // (GH_PLANE=1 keeps it at any N, GH_PLANE=0 drops it)
  const bool plane_ok = cfg->peer_mode == GH_PEER_PULL && cfg->fanout >= 3 && cfg->fanout <= 4;
  e->plane = plane_ok && cfg->n_members >= GH_PLANE_MIN_N;
  if (const char* v = std::getenv("GH_PLANE")) e->plane = plane_ok && std::atoi(v) != 0;
  // plane mode gathers one 128-B plane line per 256 members
  int tw = cfg->tile_width ? cfg->tile_width : e->plane ? GH_TW_PLANE : GH_TW_DEFAULT;
  if (const char* v = std::getenv("GH_TILE_W")) tw = std::atoi(v);
  if (const char* v = std::getenv("GH_ROUND_NT")) e->nt = std::atoi(v) != 0;
  if (const char* v = std::getenv("GH_ROUND_XMAP")) e->xmap = std::min(2, std::max(0, std::atoi(v)));
  if (const char* v = std::getenv("GH_ROUND_TPW")) e->tpw = std::atoi(v);
  if (const char* v = std::getenv("GH_FORCE_STORM")) e->force_storm = std::atoi(v) != 0;
  if (const char* v = std::getenv("GH_FORCE_SLOW")) e->force_slow = std::atoi(v) != 0;
  if (const char* v = std::getenv("GH_NIB_RMV")) e->nib_rmv = std::min(2, std::max(0, std::atoi(v)));
  if (const char* v = std::getenv("GH_NIB_DMA")) e->nib_dma = std::atoi(v) != 0;
  if (tw != 8 && tw != 16 && tw != 32 && tw != 64 && tw != 128 && tw != 256) {
    delete e;
    return GH_EINVAL;
  }
  if (e->tpw != 1 && e->tpw != 2 && e->tpw != 4 && e->tpw != 8) e->tpw = 1;
  // the 4-bit tier streams the steady state the plane serves at 1 B per cell,
  // half of it the plane itself (its window is the plane's: lags of healthy
  // pull dissemination); the row layout ships 16-bit ghost rows
  e->c8 = e->plane && e->tpw == 1 && tw >= 64;
  if (const char* v = std::getenv("GH_SIDE")) e->side = std::min(2, std::max(0, std::atoi(v)));
  if (const char* v = std::getenv("GH_TMODE")) e->tmode = std::atoi(v) != 0;
  if (const char* v = std::getenv("GH_SIDE_ORDER")) e->side_order = std::atoi(v) != 0;
  if (const char* v = std::getenv("GH_JOIN_STAMP")) e->join_stamp = std::atoi(v) != 0;
  if (const char* v = std::getenv("GH_QUIRK_ROWS")) e->quirk_rows = std::atoi(v) != 0;
  if (const char* v = std::getenv("GH_GX_DIRECT")) e->gx_direct = std::atoi(v) != 0;
  if (const char* v = std::getenv("GH_C8")) e->c8 = e->c8 && std::atoi(v) != 0;
  if (cfg->shard_layout != GH_LAYOUT_COLUMNS && cfg->shard_layout != GH_LAYOUT_ROWS) {
    delete e;
    return GH_EINVAL;
  }
  // communicator
  std::string cerr;
  GhComm* c = nullptr;
  if (dry)
    c = gh_comm_single();
  else if (world == 1 && transport != GH_COMM_RCCL)
    c = gh_comm_single();
  else if (world == 1 && !comm_id)
    c = gh_comm_single();
  else if (transport == GH_COMM_RCCL)
    c = gh_comm_rccl(rank, world, comm_id, &cerr);
  else
    c = gh_comm_local(rank, world, comm_id, cfg->device, &cerr);
  if (!c) {
    std::fprintf(stderr, "gh_create_sharded: %s\n", cerr.c_str());
    delete e;
    return GH_EHIP;
  }
  c->rank = rank;
  c->world = world;
  e->comm.reset(c);
  // column shard: [rank*ncs, rank*ncs + ncol), padded so that 8 | (ld / tw)
  // (the XCD-aware map gives each of the 8 XCDs the same number of tiles).
  // Row shard: all columns; rows [rank*nrs, rank*nrs + nrows) plus ghosts.
  const bool rowlay = cfg->shard_layout == GH_LAYOUT_ROWS;
  const int64_t ncs = rowlay ? (e->n + 31) / 32 * 32 : ((e->n + world - 1) / world + 31) / 32 * 32;
  const int64_t col0 = rowlay ? 0 : (int64_t)rank * ncs;
  const int64_t ncol = std::max<int64_t>(0, std::min<int64_t>(ncs, e->n - col0));
  const int64_t nrs = rowlay ? ((int64_t)e->n + world - 1) / world : e->n;
  const int64_t row0 = rowlay ? std::min<int64_t>((int64_t)rank * nrs, e->n) : 0;
  const int64_t nrows = rowlay ? std::min<int64_t>(nrs, e->n - row0) : e->n;
  // ghost rows (row layout)
  const int64_t gcap = rowlay && world > 1 ? ghost_cap(e->n, nrows, cfg->fanout) : 0;
  e->rowlay = rowlay;
  e->nrs = nrs;
  e->lorder = cfg->list_order == GH_ORDER_APPEND;
  const int64_t pad = std::max<int64_t>(GH_PAD, 8 * (int64_t)tw);
  e->ld = (ncs + pad - 1) / pad * pad;
  // the idle round variants' side stream at the highest priority: their
  // workgroups (which return at once) dispatch ahead of the nibble path's
  // instead of queueing behind all of them
  int prio_lo = 0, prio_hi = 0;
  if (!dry) (void)hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi);
  if (!dry && (hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking) != hipSuccess ||
               hipStreamCreateWithPriority(&e->vstream, hipStreamNonBlocking, prio_hi) != hipSuccess ||
               hipStreamCreateWithPriority(&e->vstream2, hipStreamNonBlocking, prio_hi) != hipSuccess ||
               hipEventCreateWithFlags(&e->vfork, hipEventDisableTiming) != hipSuccess ||
               hipEventCreateWithFlags(&e->vjoin, hipEventDisableTiming) != hipSuccess ||
               hipEventCreateWithFlags(&e->vjoin2, hipEventDisableTiming) != hipSuccess ||
               hipEventCreate(&e->vstart) != hipSuccess || hipEventCreate(&e->vstop) != hipSuccess)) {
    gh_destroy(e);  // the streams and events created before the failing one, and the communicator
    return GH_EHIP;
  }
  GhDev& d = e->d;
  d.n = e->n;
  d.ld = e->ld;
  d.tw = tw;
  d.lgtw = __builtin_ctz((unsigned)tw);
  d.rowlay = rowlay;
  d.row0 = row0;
  d.nrows = nrows;
  d.nslots = nrows;  // ghosts live in the ghost table (gcodes / gplane)
  d.tstride = d.nslots * tw;
  d.ntiles = e->ld / tw;
  d.col0 = col0;
  d.ncol = (int32_t)ncol;
  d.ncs = (int32_t)ncs;
  d.ncsw = (int32_t)(ncs / 32);
  d.rank = rank;
  d.world = world;
  d.tsa = cfg->t_cleanup < GH_TSAT_T ? cfg->t_cleanup + 1 : 0;
  d.toff = gh_tier_toff(cfg->t_cleanup);
  d.rlist = cfg->remove_mode == GH_REMOVE_LIST;
  // every shard sizes (and grows) its arena from the same segment count, the
  // largest over the shards, so the grow and lose decisions are collective
  // (ghost rows' wide segments take arena slots of the current buffer too)
  int64_t slots_max = d.nslots + gcap;
  if (rowlay)
    for (int32_t g = 0; g < world; ++g) {
      const int64_t r0 = std::min<int64_t>((int64_t)g * nrs, e->n), nr = std::min<int64_t>(nrs, e->n - r0);
      slots_max = std::max<int64_t>(slots_max, nr + (world > 1 ? ghost_cap(e->n, nr, cfg->fanout) : 0));
    }
  e->segs_g = d.ntiles * slots_max;
  e->segs_all = rowlay ? d.ntiles * (int64_t)e->n : e->segs_g;
  d.wcap = arena_slots(cfg, e->segs_g, tw);
  e->cfg.tile_width = tw;
  const int64_t cells = d.nslots * e->ld;
  const int64_t nch = e->ld / tw;  // tiles: per-(tile, row) ring / quirk summaries
  const int64_t slots = (int64_t)world * ncs;  // global rows incl. the last shard's tail
  const int64_t inbox = std::max<int64_t>(slots * (cfg->fanout + 1), 3 * (int64_t)e->n);
  int rc = GH_OK;
  do {
    if ((rc = dalloc(e, &d.hn[0], cells, 0xFF)) || (rc = dalloc(e, &d.hn[1], cells, 0xFF)) ||
        (rc = dalloc(e, &d.base[0], e->ld, 0)) || (rc = dalloc(e, &d.base[1], e->ld, 0)) ||
        (rc = dalloc(e, &d.colq, e->ld, 0)) || (rc = dalloc(e, &d.wn, 8, 0)) || (rc = dalloc(e, &d.err, 1, 0)) ||
        (rc = dalloc(e, &d.frow, e->n, 0xFF)) ||
        (rc = dalloc(e, &d.slow, (size_t)(e->ld / tw) * nrows, 0)) || (rc = dalloc(e, &d.slow_n, 4, 0)) ||
        (rc = dalloc(e, &d.mode, 4, 0)) || (rc = dalloc(e, &d.nstorm, 4, 0)) ||
        (rc = dalloc(e, &d.nflag, 2, 0)) || (rc = dalloc(e, &d.pvalid, 2, 0)) ||
        (rc = dalloc(e, &d.pfb, 1, 0)) ||
        (rc = dalloc(e, &d.stab[0], e->n, 0)) || (rc = dalloc(e, &d.stab[1], e->n, 0)) ||
        (rc = dalloc(e, &d.nquiet, 1, 0)) || (rc = dalloc(e, &d.aq, 1, 0x01)))
      break;
    const char* dnw_env = std::getenv("GH_DNW");  // 0: the nibble path derives the moves from the bases (A/B)
    if (e->c8 && !rowlay && !(dnw_env && std::atoi(dnw_env) == 0) &&
        ((rc = dalloc(e, &d.dnw, e->ld / 8, 0)) || (rc = dalloc(e, &d.dbad, e->ld / 8, 0))))
      break;
    const char* nrec_env = std::getenv("GH_NREC");  // 0: stage the rows from the inboxes (A/B)
    if (e->c8 && world == 1 && !rowlay && cfg->peer_mode == GH_PEER_PULL && !(nrec_env && std::atoi(nrec_env) == 0) &&
        ((rc = dalloc(e, &d.nmeta, e->n, 0)) || (rc = dalloc(e, &d.nsnd, 4 * (size_t)e->n, 0))))
      break;
    if (e->plane && ((rc = dalloc(e, &d.pl[0], cells / 8, 0xFF)) || (rc = dalloc(e, &d.pl[1], cells / 8, 0xFF))))
      break;
    // 4-bit tier: every chunk escaped (age word 0), both buffers 16-bit
    // until a round writes one
    if ((rc = dalloc(e, &d.m8, 8, 0))) break;
    if (e->c8 && ((rc = dalloc(e, &d.a4[0], cells / 8, 0)) || (rc = dalloc(e, &d.a4[1], cells / 8, 0))))
      break;
    // the nibble path's lane jobs: one region of GH_JOB_CAP per wave of its
    // grid (GH_WG_ROWS_WIDE rows x one tile per workgroup, 4 waves)
    if (e->c8) {
      d.jobw = ((d.nrows + GH_WG_ROWS_WIDE - 1) / GH_WG_ROWS_WIDE) * d.ntiles;
      if ((rc = dalloc(e, &d.jobs, (size_t)d.jobw * 4 * GH_JOB_CAP * 2, 0)) ||
          (rc = dalloc(e, &d.jobn, (size_t)d.jobw * 4, 0)) || (rc = dalloc(e, &d.njobs, 8, 0)) ||
          (rc = dalloc(e, &d.jlist, (size_t)d.jobw, 0)) ||
          (rc = dalloc(e, &d.redo, GH_REDO_CAP, 0)))
        break;
    }
    if ((rc = dalloc(e, &d.alive, e->n, 0)) || (rc = dalloc(e, &d.active, e->n, 0)) ||
        (rc = dalloc(e, &d.det_any, e->n, 0)) || (rc = dalloc(e, &d.und, e->n, 0)) ||
        (rc = dalloc(e, &d.cntl, e->n + 8, 0)) ||
        // one engine: the global counts ARE the local ones (no copy per round)
        (e->world == 1 ? (d.cntg = d.cntl, 0) : (rc = dalloc(e, &d.cntg, e->n + 8, 0))) ||
        (rc = dalloc(e, &d.post, e->n, 0)))
      break;
    if ((rc = dalloc(e, &d.det_cnt[0], e->ld, 0)) || (rc = dalloc(e, &d.det_cnt[1], e->ld, 0)) ||
        (rc = dalloc(e, &d.det_min[0], e->ld, 0x7F)) || (rc = dalloc(e, &d.det_min[1], e->ld, 0x7F)) ||
        (rc = dalloc(e, &d.dbits, e->ld / 32 + 2, 0)) || (rc = dalloc(e, &d.sbits, e->ld / 32 + 2, 0)) ||
        (rc = dalloc(e, &d.dlist, 2 * e->ld, 0)) ||
        (rc = dalloc(e, &d.nd, 8, 0)) || (rc = dalloc(e, &d.shadow, e->ld, 0x80)) ||
        (rc = dalloc(e, &d.nshadow, 1, 0)))
      break;
    // GH_REMOVE_LIST: the recipients of two REMOVE sets and the column
    // bitmaps of a sweep, [ld][ceil(n / 32)] words each (remove.hip)
    if (d.rlist) {
      d.nw = ((int64_t)e->n + 31) / 32;
      const size_t words = (size_t)e->ld * d.nw;
      if ((rc = dalloc(e, &d.rcv[0], words, 0)) || (rc = dalloc(e, &d.rcv[1], words, 0)) ||
          (rc = dalloc(e, &d.cdet, words, 0)) || (rc = dalloc(e, &d.csurv, words, 0)) ||
          (rc = dalloc(e, &d.clst, words, 0)) || (rc = dalloc(e, &d.ccnt, 2 * e->ld + 2, 0)))
        break;
    }
    if ((rc = dalloc(e, &d.inbox_beg, e->n, 0)) ||
        (rc = dalloc(e, &d.inbox_cnt, slots, 0)) || (rc = dalloc(e, &d.inbox_fill, e->n, 0)) ||
        (rc = dalloc(e, &d.inbox, inbox, 0)) || (rc = dalloc(e, &d.targets, 3 * (int64_t)e->n, 0xFF)) ||
        (rc = dalloc(e, &d.stats, ST_COUNT, 0)) || (rc = dalloc(e, &e->ev_buf, 2 * (int64_t)e->n + 16, 0)) ||
        (rc = dalloc(e, &e->rows_buf, 16, 0)))
      break;
    if (cfg->peer_mode == GH_PEER_RING &&
        ((rc = dalloc(e, &d.ring, 2 * (int64_t)world * e->n, 0)) || (rc = dalloc(e, &d.rcnt, nch * e->n, 0))))
      break;
    if (cfg->detect_mode == GH_DETECT_QUIRK &&
        ((rc = dalloc(e, &d.qsum, nch * e->n, 0)) || (rc = dalloc(e, &d.qall, (int64_t)world * e->n, 0)) ||
         (rc = dalloc(e, &d.qcarry, e->n, 0)) || (rc = dalloc(e, &d.qlast, e->n, 0))))
      break;
    if ((rc = dalloc(e, &d.rbits, (size_t)world * 2 * d.ncsw, 0))) break;
    if (e->lorder) {
      if (!list_lds_ok(d)) {
        rc = set_err(e, GH_EINVAL, "GH_ORDER_APPEND: N too large for the per-row list kernels");
        break;
      }
      if ((rc = dalloc(e, &d.lord[0], (size_t)e->n * e->ld, 0)) || (rc = dalloc(e, &d.lord[1], (size_t)e->n * e->ld, 0)) ||
          (rc = dalloc(e, &d.llen[0], e->n, 0)) || (rc = dalloc(e, &d.llen[1], e->n, 0)) ||
          (rc = dalloc(e, &d.lself[0], e->n, 0xFF)) || (rc = dalloc(e, &d.lself[1], e->n, 0xFF)) ||
          (rc = dalloc(e, &d.lsel[0], e->n, 0)) || (rc = dalloc(e, &d.lsel[1], e->n, 0)))
        break;
      if (rowlay && world > 1 && (rc = dalloc(e, &d.lchg, e->n, 0))) break;
    }
    if (!rowlay && world > 1 && cfg->peer_mode == GH_PEER_PULL &&
        (rc = dalloc(e, &d.pvb, (size_t)world * ncs + 64, 0)))
      break;
    if (rowlay) {
      e->rslot_h.assign(e->n, -1);
      for (int64_t i = row0; i < row0 + nrows; ++i) e->rslot_h[i] = (int32_t)(i - row0);
      if ((world > 1 && (rc = dalloc(e, &d.soleval, e->ld, 0xFF))) ||
          (rc = dalloc(e, &d.rslot, e->n, 0xFF)) || (rc = dalloc(e, &d.pvf, (int64_t)e->n * cfg->fanout, 0)) ||
          (rc = dalloc(e, &e->gwcnt, 2 * (int64_t)world + (int64_t)world * world, 0)))
        break;
      if (gcap > 0 && ((rc = dalloc(e, &d.gcodes, (size_t)gcap * e->ld, 0xFF)) ||
                       (e->plane && (rc = dalloc(e, &d.gplane, (size_t)gcap * e->ld / 8, 0xFF)))))
        break;
      d.gcap = gcap;
      // the device want lists of every shard (round_ghosts)
      if (world > 1 && world <= GH_GX_MAXG) {
        const int64_t nw = ((int64_t)e->n + 31) / 32, nb = (nw + 255) / 256;
        if ((rc = dalloc(e, &e->wbits, (size_t)world * nw, 0)) || (rc = dalloc(e, &e->wsum, (size_t)world * nb, 0)) ||
            (rc = dalloc(e, &e->wlist, (size_t)world * e->n, 0)) ||
            (rc = dalloc(e, &e->mcnt, (size_t)world * world + world, 0)))
          break;
      }
      if (!dry && hipMemcpyAsync(d.rslot, e->rslot_h.data(), sizeof(int32_t) * e->n, hipMemcpyHostToDevice,
                                 e->stream) != hipSuccess) {
        rc = GH_EHIP;
        break;
      }
    }
    for (int b = 0; b < 2 && rc == GH_OK; ++b)
      if ((rc = dalloc(e, &d.wh[b], (size_t)d.wcap * tw, 0xFF)) || (rc = dalloc(e, &d.wt[b], (size_t)d.wcap * tw, 0)) ||
          (rc = dalloc(e, &d.wf[b], (size_t)d.wcap * tw / 8, 0)))
        break;
    if (rc) break;
    e->rbits_rows = 2;
    if ((rc = dalloc(e, &d.cand, e->n, 0)) || (rc = dalloc(e, &d.ncand, 4, 0))) break;
    // the file table sharded by file ID: shard g holds files g, g + G, ...
    d.fsh = std::max(e->world, 1);
    d.frank = e->rank;
    d.fcap = cfg->max_files > 0 ? (cfg->max_files + d.fsh - 1) / d.fsh : 0;
    if (d.fcap > 0) {
      if ((rc = dalloc(e, &d.rep, d.fcap * cfg->replicas, 0xFF)) || (rc = dalloc(e, &d.ver, d.fcap, 0xFF)) ||
          (rc = dalloc(e, &d.fts, d.fcap, 0)) || (rc = dalloc(e, &d.draws, d.fcap, 0)) ||
          (rc = dalloc(e, &d.plan, d.fcap, 0)) || (rc = dalloc(e, &d.nplan, 4, 0)))
        break;
    }
  } while (0);
  if (rc != GH_OK) {
    std::fprintf(stderr, "gh_create: %s\n", e->err.c_str());
    gh_destroy(e);
    return rc;
  }
  if (dry) {
    *handle = e;
    return GH_OK;
  }
  if (hipDeviceSynchronize() != hipSuccess) {
    gh_destroy(e);
    return GH_EHIP;
  }
  *handle = e;
  return GH_OK;
}

// Per-round exchange of the global present counts and |D_{r-1}|, then the
// <4 guard (SPEC §2 step 2) for every row.
int decide_active(Engine* e, const GhRound& p) {
  GhDev& d = e->d;
  int rc;
  if (e->world == 1) {  // with k_base in one launch (gh_step skips launch_base)
    launch_prologue(d, e->cur, e->dcur, p, e->stream);
    HIPCHK(e, hipGetLastError());
    return GH_OK;
  }
  if ((rc = allreduce_i32(e, d.cntl, d.cntg, (size_t)e->n + 3))) return rc;
  launch_active_pre(d, e->cur, e->dcur, p, e->stream);
  HIPCHK(e, hipGetLastError());
  if (e->world > 1 && (rc = allreduce_i32(e, d.post, d.post, (size_t)e->n))) return rc;
  launch_active_post(d, p, e->stream);
  HIPCHK(e, hipGetLastError());
  return GH_OK;
}

// Quirk-mode detection (SPEC §4): rewrite this round's detection flags to
// the reference's range-over-mutated-slice set before anything reads them.
int quirk_flags(Engine* e, const GhRound& p) {
  GhDev& d = e->d;
  if (e->lorder) {  // runs over the list order
    launch_quirk_list(d, e->cur, e->dcur, p, e->lcur, e->stream);
    HIPCHK(e, hipGetLastError());
    return GH_OK;
  }
  if (e->quirk_rows && (e->world == 1 || e->rowlay) && d.tw >= 32) {  // whole rows here: one pass
    launch_quirk_rows(d, e->cur, e->dcur, p, e->stream);
    HIPCHK(e, hipGetLastError());
    return GH_OK;
  }
  launch_quirk_scan(d, e->cur, e->dcur, p, e->stream);
  HIPCHK(e, hipGetLastError());
  if (e->world > 1 && !e->rowlay)  // row layout: a row's runs never cross shards
    COMMCHK(e, e->comm->allgather(d.qall + (size_t)e->rank * e->n, d.qall, e->n, e->stream));
  launch_quirk_apply(d, e->cur, e->dcur, p, e->stream);
  HIPCHK(e, hipGetLastError());
  return GH_OK;
}

// Who merges whose snapshot this round: pull inboxes (owner of the
// receiver's column draws and validates, allgather) or ring targets.
int build_inboxes(Engine* e, const GhRound& p) {
  GhDev& d = e->d;
  if (e->rowlay) {
    if (e->cfg.peer_mode == GH_PEER_PULL) {
      // validity at the senders' owners, summed; every shard builds all inboxes
      launch_peers_rows(d, e->cur, e->dcur, p, e->stream);
      HIPCHK(e, hipGetLastError());
      int rc;
      if (e->world > 1 && (rc = allreduce_i32(e, d.pvf, d.pvf, (size_t)e->n * e->cfg.fanout))) return rc;
      launch_inbox_rows(d, p, e->stream);
    } else {
      // ring (slave/slave.go:515-524): each sender's owner holds its whole
      // row, its list, so it finds the 3 targets alone (the ring kernels on
      // a one-shard view of the columns, skipping rows it does not own);
      // allreduce(max) of the targets, then every shard builds every CSR
      // inbox. In a healthy cluster the targets are the adjacent members,
      // so the want lists below are a halo of a few rows per shard boundary.
      if (e->lorder) {  // the owned senders' neighbours in list order (the others' targets stay -1)
        launch_ring_list(d, e->cur, e->dcur, p, e->lcur, e->flags_known, e->stream);
      } else {
        GhDev v = d;
        v.rank = 0;
        v.world = 1;
        launch_ring_count(v, e->cur, e->dcur, p, e->stream);
        launch_ring_select(v, e->cur, e->dcur, p, e->stream);
      }
      HIPCHK(e, hipGetLastError());
      if (e->world > 1)
        COMMCHK(e, e->comm->allreduce(d.targets, d.targets, 3 * (size_t)e->n, GH_DT_I32, GH_OP_MAX, e->stream));
      launch_inbox(d, p, e->stream);
    }
    HIPCHK(e, hipGetLastError());
    return e->world > 1 ? round_ghosts(e, p) : GH_OK;
  }
  if (e->cfg.peer_mode == GH_PEER_PULL) {
    launch_peers_pull(d, e->cur, e->dcur, p, e->stream);
    HIPCHK(e, hipGetLastError());
    if (e->world > 1) {
      // one validity byte per receiver (k <= 8 draws) instead of its
      // (k + 1)-int inbox row: every shard redraws the peers and rebuilds
      COMMCHK(e, e->comm->allgather(d.pvb + (size_t)e->rank * d.ncs, d.pvb, (size_t)d.ncs, e->stream));
      launch_inbox_bits(d, p, e->stream);
      HIPCHK(e, hipGetLastError());
    }
    return GH_OK;
  }
  if (e->lorder) {  // neighbours in list order (single GPU)
    launch_ring_list(d, e->cur, e->dcur, p, e->lcur, e->flags_known, e->stream);
    launch_inbox(d, p, e->stream);
    HIPCHK(e, hipGetLastError());
    return GH_OK;
  }
  launch_ring_count(d, e->cur, e->dcur, p, e->stream);
  HIPCHK(e, hipGetLastError());
  if (e->world > 1)
    COMMCHK(e, e->comm->allgather(d.ring + (size_t)e->rank * e->n * 2, d.ring, sizeof(int32_t) * e->n * 2,
                                  e->stream));
  launch_ring_select(d, e->cur, e->dcur, p, e->stream);
  HIPCHK(e, hipGetLastError());
  if (e->world > 1)
    COMMCHK(e, e->comm->allreduce(d.targets, d.targets, 3 * (size_t)e->n, GH_DT_I32, GH_OP_MAX, e->stream));
  launch_inbox(d, p, e->stream);
  HIPCHK(e, hipGetLastError());
  return GH_OK;
}

// Runs an encoding launch (pack / fill) of buffer cur until it fits the wide
// arena: on overflow the arena grows and the launch repeats (both are
// idempotent rewrites of whole rows).
template <class F>
int encode_rows(Engine* e, const char* what, F launch) {
  const int64_t segs = e->segs_all;
  for (;;) {
    launch();
    HIPCHK(e, hipGetLastError());
    int32_t err = 0;
    int rc;
    if ((rc = read_err(e, &err))) return rc;
    if (e->world > 1) {  // every shard grows together
      int32_t* flag = e->d.wn + 2;
      HIPCHK(e, hipMemcpyAsync(flag, &err, sizeof err, hipMemcpyHostToDevice, e->stream));
      COMMCHK(e, e->comm->allreduce(flag, flag, 1, GH_DT_I32, GH_OP_MAX, e->stream));
      HIPCHK(e, hipMemcpyAsync(&err, flag, sizeof err, hipMemcpyDeviceToHost, e->stream));
      HIPCHK(e, hipStreamSynchronize(e->stream));
      err = err ? GH_ENOMEM : 0;
    }
    if (err == 0) return GH_OK;
    if (err != GH_ENOMEM || e->d.wcap >= segs) return lose(e, what);
    HIPCHK(e, hipMemsetAsync(e->d.err, 0, sizeof(int32_t), e->stream));
    if ((rc = grow_arena(e, std::min<int64_t>(segs, 2 * e->d.wcap)))) return rc;
  }
}

// Buffer cur emptied (all absent narrow, arena reset) before a whole-table
// rewrite.
// No D7 shadow entry (rows written whole hold no member twice).
int reset_shadows(Engine* e) {
  HIPCHK(e, hipMemsetAsync(e->d.shadow, 0x80, sizeof(int32_t) * (size_t)e->ld, e->stream));
  HIPCHK(e, hipMemsetAsync(e->d.nshadow, 0, sizeof(int32_t), e->stream));
  e->shadow_any = false;
  return GH_OK;
}

int clear_table(Engine* e) {
  GhDev& d = e->d;
  HIPCHK(e, hipMemsetAsync(d.hn[e->cur], 0xFF, sizeof(uint16_t) * (size_t)d.nslots * e->ld, e->stream));
  HIPCHK(e, hipMemsetAsync(d.m8 + e->cur, 0, sizeof(int32_t), e->stream));  // hn alone holds it
  HIPCHK(e, hipMemsetAsync(d.wn + e->cur, 0, sizeof(int32_t), e->stream));
  HIPCHK(e, hipMemsetAsync(d.err, 0, sizeof(int32_t), e->stream));
  e->lost.clear();
  return GH_OK;
}

// Stopped rows of [row0, row0 + n) go to the frozen store, running ones
// leave it (after their segments were rewritten).
int settle_rows(Engine* e, int64_t row0, int64_t n, const GhRound& p) {
  std::vector<int32_t> stopped, running;
  for (int64_t i = row0; i < row0 + n; ++i)
    if (gh_owned(e->d, i)) (e->alive[i] ? running : stopped).push_back((int32_t)i);
  int rc;
  if ((rc = release_rows(e, running))) return rc;
  for (size_t b = 0; b < stopped.size(); b += (size_t)e->n) {
    const std::vector<int32_t> part(stopped.begin() + b, stopped.begin() + std::min(stopped.size(), b + e->n));
    if ((rc = upload(e, e->ev_buf, part))) return rc;
    if ((rc = freeze_rows(e, part, e->ev_buf, p))) return rc;
  }
  return GH_OK;
}

}  // namespace

extern "C" {

int gh_abi_version(void) { return GH_ABI_VERSION; }

void gh_config_default(gh_config* cfg) {
  if (!cfg) return;
  std::memset(cfg, 0, sizeof(*cfg));
  cfg->n_members = 10;
  cfg->fanout = 3;
  cfg->peer_mode = GH_PEER_PULL;
  cfg->detect_mode = GH_DETECT_CANONICAL;
  cfg->t_fail = 5;      // PERIOD 5e9 ns / 1 s (slave/slave.go:24, main.go:11)
  cfg->t_cleanup = 5;   // COOLDOWN (slave/slave.go:25)
  cfg->min_members = 4; // slave/slave.go:504
  cfg->replicas = 4;    // master/master.go:131
  cfg->introducer = 0;
  cfg->master = 0;
  cfg->device = 0;
  cfg->seed = 0x5EED0001ull;
  cfg->max_files = 0;
}

const char* gh_last_error(void* h) {
  return h ? static_cast<Engine*>(h)->err.c_str() : "null handle";
}

void gh_destroy(void* h) {
  Engine* e = static_cast<Engine*>(h);
  if (!e) return;
  if (e->dry) {  // (gh_footprint: nothing on a device)
    delete e;
    return;
  }
  (void)hipSetDevice(e->cfg.device);
  if (e->stream) (void)hipStreamSynchronize(e->stream);
  e->comm.reset();
  for (auto ev : e->evs) (void)hipEventDestroy(ev);
  if (e->vlog) (void)hipFree(e->vlog);
  for (void* p : e->allocs) (void)hipFree(p);
  if (e->stream) (void)hipStreamDestroy(e->stream);
  if (e->vstream) (void)hipStreamDestroy(e->vstream);
  if (e->vstream2) (void)hipStreamDestroy(e->vstream2);
  if (e->vfork) (void)hipEventDestroy(e->vfork);
  if (e->vjoin) (void)hipEventDestroy(e->vjoin);
  if (e->vjoin2) (void)hipEventDestroy(e->vjoin2);
  if (e->vstart) (void)hipEventDestroy(e->vstart);
  if (e->vstop) (void)hipEventDestroy(e->vstop);
  delete e;
}

int gh_create(const gh_config* cfg, void** handle) {
  return create(cfg, 0, 1, GH_COMM_LOCAL, nullptr, handle);
}

int gh_create_sharded(const gh_config* cfg, int32_t rank, int32_t world, int32_t transport,
                      const uint8_t* comm_id, void** handle) {
  return create(cfg, rank, world, transport, comm_id, handle);
}

int gh_footprint(const gh_config* cfg, int32_t rank, int32_t world, int32_t transport, int64_t* create_bytes,
                 int64_t* exchange_bytes) {
  void* h = nullptr;
  const int rc = create(cfg, rank, world, transport, nullptr, &h, true);
  if (rc != GH_OK) return rc;
  Engine* e = static_cast<Engine*>(h);
  if (create_bytes) *create_bytes = e->dry_bytes;
  if (exchange_bytes) *exchange_bytes = exchange_footprint(e);
  delete e;
  return GH_OK;
}

int gh_comm_unique_id(uint8_t* id) {
  if (!id) return GH_EINVAL;
  std::string err;
  if (gh_comm_rccl_unique_id(id, &err) != 0) {
    std::fprintf(stderr, "gh_comm_unique_id: %s\n", err.c_str());
    return GH_EHIP;
  }
  return GH_OK;
}

int gh_shard_info(void* h, int32_t* rank, int32_t* world, int64_t* col0, int64_t* ncols) {
  Engine* e = static_cast<Engine*>(h);
  if (!e) return GH_EINVAL;
  if (rank) *rank = e->rank;
  if (world) *world = e->world;
  if (col0) *col0 = e->d.col0;
  if (ncols) *ncols = e->d.ncol;
  return GH_OK;
}

int gh_encoding_info(void* h, int64_t* wide_segments, int64_t* slow_segments, int32_t* storm_mode,
                     int64_t* storm_segments, int64_t* quiet_segments) {
  Engine* e = static_cast<Engine*>(h);
  if (!e) return GH_EINVAL;
  HIPCHK(e, hipSetDevice(e->cfg.device));
  Staging st;
  int rc;
  if ((rc = st.alloc(e, 2 * sizeof(unsigned long long)))) return rc;
  launch_count_wide(e->d, e->cur, st.as<unsigned long long>(), e->stream);
  HIPCHK(e, hipGetLastError());
  unsigned long long w[2] = {0, 0};
  int32_t sl = 0, mode = 0, ns = 0, nq = 0;
  HIPCHK(e, hipMemcpyAsync(w, st.p, sizeof w, hipMemcpyDeviceToHost, e->stream));
  HIPCHK(e, hipMemcpyAsync(&sl, e->d.slow_n, sizeof sl, hipMemcpyDeviceToHost, e->stream));
  HIPCHK(e, hipMemcpyAsync(&mode, e->d.mode, sizeof mode, hipMemcpyDeviceToHost, e->stream));
  HIPCHK(e, hipMemcpyAsync(&ns, e->d.nstorm, sizeof ns, hipMemcpyDeviceToHost, e->stream));
  HIPCHK(e, hipMemcpyAsync(&nq, e->d.nquiet, sizeof nq, hipMemcpyDeviceToHost, e->stream));
  HIPCHK(e, hipStreamSynchronize(e->stream));
  if (wide_segments) *wide_segments = (int64_t)(w[0] + w[1]);
  if (slow_segments) *slow_segments = sl;
  if (storm_mode) *storm_mode = mode;
  if (storm_segments) *storm_segments = ns;
  if (quiet_segments) *quiet_segments = nq;
  return GH_OK;
}

int gh_plane_info(void* h, int32_t* enabled, int32_t* valid, int64_t* fallback_waves) {
  Engine* e = static_cast<Engine*>(h);
  if (!e) return GH_EINVAL;
  HIPCHK(e, hipSetDevice(e->cfg.device));
  int32_t v[2] = {0, 0};
  HIPCHK(e, hipMemcpyAsync(&v[0], e->d.pvalid + e->cur, sizeof(int32_t), hipMemcpyDeviceToHost, e->stream));
  HIPCHK(e, hipMemcpyAsync(&v[1], e->d.pfb, sizeof(int32_t), hipMemcpyDeviceToHost, e->stream));
  HIPCHK(e, hipStreamSynchronize(e->stream));
  if (enabled) *enabled = e->plane;
  if (valid) *valid = e->pforce ? 0 : v[0];
  if (fallback_waves) *fallback_waves = v[1];
  return GH_OK;
}

int gh_tier_info(void* h, int32_t* enabled, int32_t* current_8bit, int64_t* escaped_chunks, int32_t* last_variant) {
  Engine* e = static_cast<Engine*>(h);
  if (!e) return GH_EINVAL;
  HIPCHK(e, hipSetDevice(e->cfg.device));
  int32_t v[5] = {0, 0, 0, 0, 0};
  HIPCHK(e, hipMemcpyAsync(v, e->d.m8, sizeof v, hipMemcpyDeviceToHost, e->stream));
  HIPCHK(e, hipStreamSynchronize(e->stream));
  if (enabled) *enabled = e->c8;
  if (current_8bit) *current_8bit = e->c8 ? v[e->cur] : 0;
  if (escaped_chunks) *escaped_chunks = e->c8 ? v[3] : 0;
  if (last_variant) *last_variant = v[4];
  return GH_OK;
}

int gh_job_info(void* h, int64_t* lane_jobs, int64_t* redo_lanes) {
  Engine* e = static_cast<Engine*>(h);
  if (!e) return GH_EINVAL;
  HIPCHK(e, hipSetDevice(e->cfg.device));
  int32_t nj[2] = {0, 0};
  if (e->d.njobs) {
    HIPCHK(e, hipMemcpyAsync(nj, e->d.njobs, sizeof nj, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(e, hipStreamSynchronize(e->stream));
  }
  if (lane_jobs) *lane_jobs = nj[0];
  if (redo_lanes) *redo_lanes = std::min<int64_t>(nj[1], GH_REDO_CAP);
  return GH_OK;
}

int gh_exchange_info(void* h, int64_t* ghost_rows, int64_t* bytes_out, int64_t* bytes_in) {
  Engine* e = static_cast<Engine*>(h);
  if (!e) return GH_EINVAL;
  if (ghost_rows) *ghost_rows = e->gx_rows;
  if (bytes_out) *bytes_out = e->gx_out;
  if (bytes_in) *bytes_in = e->gx_in;
  return GH_OK;
}

int gh_file_info(void* h, int64_t* slots, int32_t* shards, int64_t* held) {
  Engine* e = static_cast<Engine*>(h);
  if (!e) return GH_EINVAL;
  if (slots) *slots = e->d.fcap;
  if (shards) *shards = e->d.fsh;
  if (held) {
    *held = 0;
    if (e->d.fcap > 0) {
      HIPCHK(e, hipSetDevice(e->cfg.device));
      std::vector<int32_t> ver(e->d.fcap);
      HIPCHK(e, hipMemcpyAsync(ver.data(), e->d.ver, sizeof(int32_t) * e->d.fcap, hipMemcpyDeviceToHost, e->stream));
      HIPCHK(e, hipStreamSynchronize(e->stream));
      *held = std::count_if(ver.begin(), ver.end(), [](int32_t v) { return v >= 0; });
    }
  }
  return GH_OK;
}

int gh_memory_info(void* h, int64_t* device_bytes, int64_t* wide_used, int64_t* wide_cap, int64_t* frozen_rows) {
  Engine* e = static_cast<Engine*>(h);
  if (!e) return GH_EINVAL;
  HIPCHK(e, hipSetDevice(e->cfg.device));
  const GhDev& d = e->d;
  int32_t used = 0;
  HIPCHK(e, hipMemcpyAsync(&used, d.wn + e->cur, sizeof used, hipMemcpyDeviceToHost, e->stream));
  HIPCHK(e, hipStreamSynchronize(e->stream));
  if (device_bytes) {
    // the tables (narrow x2, wide arenas x2, frozen store); per-row and
    // per-column vectors and the file table are counted by hipMemGetInfo
    // callers, not here
    const int64_t cells = d.nslots * e->ld;
    *device_bytes = 2 * cells * 2 + (e->plane ? cells : 0) + (e->c8 ? cells : 0) + 2 * d.wcap * ((int64_t)d.tw * 8 + d.tw / 8) +
                    e->fzcap * e->ld * 8 + (e->lorder ? 2 * (int64_t)e->n * e->ld * 4 : 0) +
                    d.gcap * (e->ld * 2 + (e->plane ? e->ld / 2 : 0));  // row layout: the ghost table
  }
  if (wide_used) *wide_used = std::min<int64_t>(used, d.wcap);
  if (wide_cap) *wide_cap = d.wcap;
  if (frozen_rows) *frozen_rows = (int64_t)std::count_if(e->frow.begin(), e->frow.end(), [](int32_t x) { return x >= 0; });
  return GH_OK;
}

int gh_get_round(void* h, int32_t* round) {
  Engine* e = static_cast<Engine*>(h);
  if (!e || !round) return GH_EINVAL;
  *round = e->round;
  return GH_OK;
}

int gh_import_state(void* h, const int32_t* hb, const int32_t* ts, const uint8_t* alive, int64_t row0,
                    int64_t n_rows, int32_t round) {
  Engine* e = static_cast<Engine*>(h);
  if (!e) return GH_EINVAL;
  if (row0 < 0 || n_rows < 0 || row0 + n_rows > e->n || (n_rows > 0 && (!hb || !ts || !alive)))
    return set_err(e, GH_EINVAL, "row range / null buffer");
  int64_t hmax = 0;
  for (int64_t x = 0; x < n_rows * e->n; ++x) {
    if (hb[x] < GH_TOMBSTONE) return set_err(e, GH_ERANGE, "hb value below -2");
    hmax = std::max<int64_t>(hmax, hb[x]);
  }
  HIPCHK(e, hipSetDevice(e->cfg.device));
  const bool full = row0 == 0 && n_rows == e->n;
  int rc;
  if (!full && (rc = check_lost(e))) return rc;
  e->qforce = true;
  e->flags_known = false;
  e->pforce = true;
  const GhRound p = round_params(e, round + 1);
  if (n_rows > 0) {
    // host rows -> device staging -> encoded tiled local columns
    Staging sh, st;
    const size_t bytes = sizeof(int32_t) * e->n * n_rows;
    if ((rc = sh.alloc(e, bytes)) || (rc = st.alloc(e, bytes))) return rc;
    HIPCHK(e, hipMemcpyAsync(sh.p, hb, bytes, hipMemcpyHostToDevice, e->stream));
    HIPCHK(e, hipMemcpyAsync(st.p, ts, bytes, hipMemcpyHostToDevice, e->stream));
    if (full && (rc = clear_table(e))) return rc;
    rc = encode_rows(e, "gh_import_state", [&] {
      launch_pack(e->d, e->cur, sh.as<int32_t>(), st.as<int32_t>(), row0, n_rows, p, e->stream);
    });
    if (rc) return rc;
    std::copy(alive, alive + n_rows, e->alive.begin() + row0);
    if ((rc = settle_rows(e, row0, n_rows, p))) return rc;
  }
  if ((rc = upload_alive(e))) return rc;
  e->round = round;
  e->hb_bound = full ? hmax : std::max(e->hb_bound, hmax);
  e->pending.clear();
  if ((rc = reset_pending_removes(e))) return rc;
  if (e->cfg.introducer >= row0 && e->cfg.introducer < row0 + n_rows && (rc = reset_shadows(e))) return rc;
  launch_count(e->d, e->cur, p, e->stream);
  if (e->lorder) {
    launch_list_import(e->d, e->cur, e->lcur, row0, n_rows, e->stream);  // dense rows: ID order
    if ((rc = list_sync(e, e->lcur))) return rc;
  }
  HIPCHK(e, hipGetLastError());
  HIPCHK(e, hipStreamSynchronize(e->stream));
  return GH_OK;
}

int gh_export_state(void* h, int32_t* hb, int32_t* ts, uint8_t* alive, int64_t row0, int64_t n_rows) {
  Engine* e = static_cast<Engine*>(h);
  if (!e) return GH_EINVAL;
  if (row0 < 0 || n_rows < 0 || row0 + n_rows > e->n) return set_err(e, GH_EINVAL, "row range");
  HIPCHK(e, hipSetDevice(e->cfg.device));
  int rc;
  if ((rc = check_lost(e))) return rc;
  if (n_rows > 0 && hb && (rc = export_table(e, hb, 0, row0, n_rows))) return rc;
  if (n_rows > 0 && ts && (rc = export_table(e, ts, 1, row0, n_rows))) return rc;
  if (alive) std::copy(e->alive.begin() + row0, e->alive.begin() + row0 + n_rows, alive);
  return GH_OK;
}

int gh_init_full(void* h, int32_t hb0, int32_t ts0, int32_t round) {
  Engine* e = static_cast<Engine*>(h);
  if (!e) return GH_EINVAL;
  if (hb0 < 0) return set_err(e, GH_ERANGE, "hb0 below 0");
  HIPCHK(e, hipSetDevice(e->cfg.device));
  e->qforce = true;
  e->flags_known = false;
  e->pforce = true;
  std::fill(e->alive.begin(), e->alive.end(), 1);
  int rc;
  if ((rc = upload_alive(e))) return rc;
  e->round = round;
  e->pending.clear();
  const GhRound p = round_params(e, round + 1);
  if ((rc = clear_table(e))) return rc;
  rc = encode_rows(e, "gh_init_full", [&] { launch_fill(e->d, e->cur, hb0, ts0, p, e->stream); });
  if (rc) return rc;
  if ((rc = settle_rows(e, 0, e->n, p))) return rc;
  e->hb_bound = hb0;
  if ((rc = reset_pending_removes(e))) return rc;
  if ((rc = reset_shadows(e))) return rc;
  launch_count(e->d, e->cur, p, e->stream);
  if (e->lorder) {
    launch_list_import(e->d, e->cur, e->lcur, 0, e->n, e->stream);
    if ((rc = list_sync(e, e->lcur))) return rc;
  }
  HIPCHK(e, hipGetLastError());
  HIPCHK(e, hipStreamSynchronize(e->stream));
  return GH_OK;
}

int gh_apply_events(void* h, const gh_event* ev, int64_t n) {
  Engine* e = static_cast<Engine*>(h);
  if (!e || n < 0 || (n > 0 && !ev)) return GH_EINVAL;
  for (int64_t x = 0; x < n; ++x) {
    if (ev[x].kind < GH_EV_JOIN || ev[x].kind > GH_EV_CRASH) return set_err(e, GH_EINVAL, "event kind");
    if (ev[x].member < 0 || ev[x].member >= e->n) return set_err(e, GH_EINVAL, "event member");
  }
  e->pending.insert(e->pending.end(), ev, ev + n);
  return GH_OK;
}

int gh_step(void* h, int32_t rounds, gh_round_stats* stats) {
  Engine* e = static_cast<Engine*>(h);
  if (!e || rounds < 0) return GH_EINVAL;
  HIPCHK(e, hipSetDevice(e->cfg.device));
  int rc0;
  bool busy = false;
  if ((rc0 = check_lost(e)) || (rc0 = maybe_grow(e, &busy))) return rc0;
  // |D| of the last call's final round, read at its end: taken here and
  // cleared, so a call that returns early leaves no stale value behind
  const int32_t last_nd = e->last_nd;
  e->last_nd = -1;
  HIPCHK(e, hipMemsetAsync(e->d.stats, 0, sizeof(unsigned long long) * ST_COUNT, e->stream));
  if (e->timing && (int64_t)e->evs.size() < 12 * (int64_t)rounds) {
    while ((int64_t)e->evs.size() < 12 * (int64_t)rounds) {
      hipEvent_t ev;
      HIPCHK(e, hipEventCreate(&ev));
      e->evs.push_back(ev);
    }
  }
  // timing the nibble launch alone (the others bracketed, the variant that ran logged)
  const bool tsel = e->timing && e->tmode == 1 && e->c8 && e->side != 2;
  if (tsel && e->vlog_cap < rounds) {  // (gh_set_timing allocates 4,096 rounds' worth)
    HIPCHK(e, hipStreamSynchronize(e->stream));
    if (e->vlog) HIPCHK(e, hipFree(e->vlog));
    e->vlog = nullptr;
    e->vlog_cap = 0;
    HIPCHK(e, hipMalloc(&e->vlog, sizeof(int32_t) * rounds));
    e->vlog_cap = rounds;
  }
  e->d.vlog = tsel ? e->vlog : nullptr;
  const int32_t first = e->round + 1;
  int32_t done = 0;
  int status = GH_OK;
  std::vector<int8_t> mvlog(tsel ? rounds : 0, 3);  // the variant each round's nibble launch was (tsel)
  for (int32_t q = 0; q < rounds; ++q) {
    const int32_t r = e->round + 1;
    int rc;
    if (e->hb_bound >= INT32_MAX) {
      // a heartbeat may sit at INT32_MAX: the round would overflow Go's
      // HeartbeatCount (slave/slave.go:446) in our int32; refused (SPEC §2)
      // before its events are applied, so they stay pending. The rows that
      // run it: alive and not crashing or leaving in its events (und is the
      // round's scratch, rewritten by decide_active)
      std::vector<uint8_t> runs(e->alive.begin(), e->alive.end());
      for (const auto& x : e->pending)
        if (x.kind == GH_EV_CRASH || x.kind == GH_EV_LEAVE) runs[x.member] = 0;
      HIPCHK(e, hipMemcpyAsync(e->d.und, runs.data(), e->n, hipMemcpyHostToDevice, e->stream));
      int32_t* flag = e->d.wn + 2;
      int32_t hit = 0;
      HIPCHK(e, hipMemsetAsync(flag, 0, sizeof(int32_t), e->stream));
      launch_hb_check(e->d, e->cur, flag, round_params(e, r), e->stream);
      HIPCHK(e, hipGetLastError());
      COMMCHK(e, e->comm->allreduce(flag, flag, 1, GH_DT_I32, GH_OP_MAX, e->stream));
      HIPCHK(e, hipMemcpyAsync(&hit, flag, sizeof hit, hipMemcpyDeviceToHost, e->stream));
      HIPCHK(e, hipStreamSynchronize(e->stream));
      if (hit) {
        status = set_err(e, GH_ERANGE, "a running member's heartbeat is INT32_MAX: the round would overflow it");
        break;
      }
    }
    if ((rc = process_events(e, r))) return rc;
    if (e->pforce) {  // the table was rewritten outside a round: no valid plane
      HIPCHK(e, hipMemsetAsync(e->d.pvalid + e->cur, 0, sizeof(int32_t), e->stream));
      e->pforce = false;
      e->sforce = true;
      e->plane_valid = false;
    }
    if (e->sforce) {  // written outside a round: no quiet rows
      for (int b = 0; b < 2; ++b) HIPCHK(e, hipMemsetAsync(e->d.stab[b], 0, e->n, e->stream));
      e->sforce = false;
    }
    const GhRound p = round_params(e, r);
    if (e->world > 1) launch_base(e->d, e->cur, e->dcur, p, e->stream);  // world 1: in decide_active
    if (e->rowlay && e->world > 1)  // each column's base from its owner row's shard
      COMMCHK(e, e->comm->allreduce(e->d.base[e->cur ^ 1], e->d.base[e->cur ^ 1], e->ld, GH_DT_I32, GH_OP_MAX,
                                    e->stream));
    if ((rc = decide_active(e, p))) return rc;
    if (e->cfg.detect_mode == GH_DETECT_QUIRK) {
      // skip the pre-pass when no shard's table holds a flag (the round
      // kernels count flagged segments as they write; the counts are summed
      // by decide_active's allreduce, so every shard takes the same branch)
      GhRound pq = p;
      pq.qgate = !e->qforce;
      if ((rc = quirk_flags(e, pq))) return rc;
      e->qforce = false;
    }
    e->gpo = false;
    if ((rc = build_inboxes(e, p))) return rc;
    if (e->d.soleval) {  // row shards: the single detectors' candidates of the REMOVE'd columns
      launch_sole_vals(e->d, e->cur, e->dcur, p, e->stream);
      HIPCHK(e, hipGetLastError());
      COMMCHK(e, e->comm->allreduce(e->d.soleval, e->d.soleval, e->ld, GH_DT_I32, GH_OP_MAX, e->stream));
    }
    GhRound pr = p;
    pr.gpo = e->gpo;  // row layout: the ghosts carry only their plane so far
    pr.vslot = q;
    pr.rmv_full = q == 0 && e->world == 1 && last_nd > 0;
    // the variants of k_round; the ones not selected return at once. With
    // timing on, a launch stamps its own start and end (events 12q + 2v,
    // 12q + 2v + 1 of variant v; hipExtLaunchKernel, no event packets between
    // the kernels): every launch, or (tsel) the nibble path's, and the other
    // variants together, from the start of the first (v0) to the end of the
    // last (v4) (events 12q + 10, 12q + 11), as a stamped launch costs its
    // stream ~5 us
    // The nibble launch: IN 2 (variant 3), or IN 6 (variant 4, on a full
    // grid) when the host knows a REMOVE is pending (the first round of a
    // call after a detection, one engine, the tier's default modes): IN 2
    // cannot be the one selected then, so it is not launched, and the
    // REMOVE round's nibble path runs on the round's stream
    const bool rmv_main = e->c8 && pr.rmv_full && !e->rowlay && e->nib_rmv >= 1 && !e->nib_dma &&
                          (!e->timing || tsel);
    const int mv = rmv_main ? 4 : 3;
    if (e->timing && tsel) mvlog[q] = (int8_t)mv;
    const int nside = rmv_main ? 3 : 4;
    // the idle variants, the first nside of them (side stream: the first one
    // is dispatched between the nibble path's workgroups, the rest after it)
    int sides[4] = {0, 1, 2, 4};
    if (e->side_order) {
      sides[0] = 2, sides[1] = 0, sides[2] = 1;
    }
    auto ev = [&](int v, int end) -> hipEvent_t {
      if (!e->timing) return nullptr;
      if (!tsel) return e->evs[12 * q + 2 * v + end];
      if (v == mv) return e->evs[12 * q + 6 + end];
      if (v == sides[0] && end == 0) return e->evs[12 * q + 10];
      if (v == sides[nside - 1] && end == 1) return e->evs[12 * q + 11];
      return nullptr;
    };
    if (e->c8 && !e->side) {
      // lean 16-bit input, storm, lean tier input by the 16-bit rule, the
      // nibble path that takes REMOVE deliveries, then the steady nibble
      // path, all on the round's stream
      for (int x = 0; x < nside; ++x)
        launch_round(e->d, e->cur, e->dcur, pr, e->stream, e->nt, sides[x], ev(sides[x], 0), ev(sides[x], 1));
      launch_round(e->d, e->cur, e->dcur, pr, e->stream, e->nt, mv, ev(mv, 0), ev(mv, 1));
    } else if (e->c8 && e->side == 2) {
      // the same on two side streams, so that after the nibble path only one
      // idle launch per stream is left to run (the first on each spans it)
      HIPCHK(e, hipEventRecord(e->vfork, e->stream));
      HIPCHK(e, hipStreamWaitEvent(e->vstream, e->vfork, 0));
      HIPCHK(e, hipStreamWaitEvent(e->vstream2, e->vfork, 0));
      for (int v : {0, 1}) launch_round(e->d, e->cur, e->dcur, pr, e->vstream, e->nt, v, ev(v, 0), ev(v, 1));
      for (int v : {4, 2}) launch_round(e->d, e->cur, e->dcur, pr, e->vstream2, e->nt, v, ev(v, 0), ev(v, 1));
      HIPCHK(e, hipEventRecord(e->vjoin, e->vstream));
      HIPCHK(e, hipEventRecord(e->vjoin2, e->vstream2));
      launch_round(e->d, e->cur, e->dcur, pr, e->stream, e->nt, 3, ev(3, 0), ev(3, 1));
      HIPCHK(e, hipStreamWaitEvent(e->stream, e->vjoin, 0));
      HIPCHK(e, hipStreamWaitEvent(e->stream, e->vjoin2, 0));
    } else if (e->c8) {
      // lean 16-bit input, storm, lean tier input by the 16-bit rule and the
      // REMOVE-taking nibble path on the side stream, beside the nibble
      // launch
      // (forked at the nibble launch's own start stamp: its stream's earlier
      // work, the inboxes, is done then; an event packet of its own before
      // it had cost the round ~10 us)
      hipEvent_t st = e->timing ? ev(mv, 0) : e->vstart;
      launch_round(e->d, e->cur, e->dcur, pr, e->stream, e->nt, mv, st, ev(mv, 1));
      HIPCHK(e, hipStreamWaitEvent(e->vstream, st, 0));
      // joined at the last idle launch's own end stamp (as the fork uses the
      // nibble launch's start stamp), not at an event packet after it
      // (a last launch that did not happen, e.g. IN 6 on row shards: an event
      // packet after the others)
      hipEvent_t jn = nullptr;
      for (int x = 0; x < nside; ++x) {
        hipEvent_t t1 = ev(sides[x], 1);
        const bool last = x == nside - 1 && e->join_stamp;
        if (last && !t1) t1 = e->vstop;
        if (launch_round(e->d, e->cur, e->dcur, pr, e->vstream, e->nt, sides[x], ev(sides[x], 0), t1) && last) jn = t1;
      }
      if (!jn) {
        HIPCHK(e, hipEventRecord(e->vjoin, e->vstream));
        jn = e->vjoin;
      }
      HIPCHK(e, hipStreamWaitEvent(e->stream, jn, 0));
    } else {  // lean 16-bit input, storm
      for (int v = 0; v < 2; ++v) launch_round(e->d, e->cur, e->dcur, pr, e->stream, e->nt, v, ev(v, 0), ev(v, 1));
    }
    // (row layout: the ghosts' codes before the kernels that may read them)
    if ((rc = ghost_codes_if_slow(e))) return rc;
    launch_round_jobs(e->d, e->cur, e->dcur, pr, e->stream);
    launch_round_slow(e->d, e->cur, e->dcur, pr, e->stream);
    if (e->rowlay && e->world > 1) {
      // every shard detected in its own rows: D_r's counts and first
      // detectors over all of them (MIN as the MAX of negations)
      int32_t* dc = e->d.det_cnt[e->dcur ^ 1];
      int32_t* dm = e->d.det_min[e->dcur ^ 1];
      if ((rc = allreduce_i32(e, dc, dc, e->ld))) return rc;
      launch_negate(dm, e->ld, e->stream);
      COMMCHK(e, e->comm->allreduce(dm, dm, e->ld, GH_DT_I32, GH_OP_MAX, e->stream));
      launch_negate(dm, e->ld, e->stream);
      HIPCHK(e, hipGetLastError());
    }
    if (e->lorder) {  // the lists of the next state (needs D_{r-1} and the inboxes)
      launch_list_round(e->d, e->cur, e->dcur, p, e->lcur, e->stream);
      e->lcur ^= 1;
      if ((rc = list_sync(e, e->lcur))) return rc;
    }
    // the reference's REMOVE recipients of D_r: the sweep's column bitmaps
    // (needs D_{r-1}, before k_finish replaces it), then per member of D_r
    if (e->d.rlist) launch_rm_cols(e->d, e->cur, e->dcur, p, e->stream);
    launch_finish(e->d, e->dcur, p, e->stream);
    if (e->d.rlist) launch_rm_recv(e->d, e->dcur ^ 1, p, e->stream);
    HIPCHK(e, hipGetLastError());
    e->cur ^= 1;
    e->dcur ^= 1;
    e->round = r;
    e->plane_valid = e->plane;  // the round wrote the next buffer's plane
    e->flags_known = true;
    e->hb_bound = std::min<int64_t>(INT32_MAX, e->hb_bound + 1);
    done++;
    if (busy && q + 1 < rounds) {
      // a quarter of the arena in use on some shard: check and grow after
      // every round (collectively), so only a jump from under 1/4 to over
      // 1/1 in one round can overflow it
      if ((rc = maybe_grow(e, &busy, true))) return rc;
    }
  }
  unsigned long long st[ST_COUNT];
  int32_t nshadow = 0;
  COMMCHK(e, e->comm->allreduce(e->d.stats, e->d.stats, ST_COUNT, GH_DT_U64, GH_OP_SUM, e->stream));
  HIPCHK(e, hipMemcpyAsync(st, e->d.stats, sizeof st, hipMemcpyDeviceToHost, e->stream));
  if (e->shadow_any) HIPCHK(e, hipMemcpyAsync(&nshadow, e->d.nshadow, sizeof nshadow, hipMemcpyDeviceToHost, e->stream));
  int32_t nd_last = -1;
  if (e->world == 1 && done > 0)
    HIPCHK(e, hipMemcpyAsync(&nd_last, e->d.nd + e->dcur, sizeof nd_last, hipMemcpyDeviceToHost, e->stream));
  HIPCHK(e, hipStreamSynchronize(e->stream));
  e->last_nd = nd_last;
  e->shadow_any = nshadow > 0;  // (each shard for its own columns)
  {
    int32_t err = 0;
    int rc;
    if ((rc = read_err(e, &err))) return rc;
    if (err == GH_ENOMEM) return lose(e, "gh_step");
    if (err) {
      // reported once: the flag is cleared, so the next call starts clean
      HIPCHK(e, hipMemsetAsync(e->d.err, 0, sizeof(int32_t), e->stream));
      HIPCHK(e, hipStreamSynchronize(e->stream));
      return set_err(e, err, "device error in a round");
    }
  }
  if (e->timing) {
    std::vector<int32_t> vl;
    if (tsel && done > 0) {
      vl.resize(done);
      // (on the engine's stream: a first use of the null stream costs ms)
      HIPCHK(e, hipMemcpyAsync(vl.data(), e->vlog, sizeof(int32_t) * done, hipMemcpyDeviceToHost, e->stream));
      HIPCHK(e, hipStreamSynchronize(e->stream));
    }
    for (int32_t q = 0; q < done; ++q) {
      float ms = 0.f;  // the variant that ran
      if (tsel) {
        const int b = vl[q] == mvlog[q] ? 12 * q + 6 : 12 * q + 10;
        HIPCHK(e, hipEventElapsedTime(&ms, e->evs[b], e->evs[b + 1]));
      }
      for (int v = 0; !tsel && v < (e->c8 ? 5 : 2); ++v) {
        float mv = 0.f;
        const int b = 12 * q + 2 * v;
        HIPCHK(e, hipEventElapsedTime(&mv, e->evs[b], e->evs[b + 1]));
        ms = std::max(ms, mv);
      }
      e->timed_ms += ms;
      e->timed_launches++;
    }
  }
  if (stats) {
    std::memset(stats, 0, sizeof(*stats));
    stats->rounds = done;
    stats->last_round = done ? e->round : first - 1;
    stats->detections = (int64_t)st[ST_DETECTIONS];
    stats->failed_members = (int64_t)st[ST_FAILED];
    stats->remove_unknown = (int64_t)st[ST_REMOVE_UNKNOWN];
    stats->ring_empty = (int64_t)st[ST_RING_EMPTY];
    stats->active_rows = (int64_t)st[ST_ACTIVE_ROWS];
    stats->merged_cells = (int64_t)st[ST_MERGED];
    stats->released = (int64_t)st[ST_RELEASED];
    stats->tombstoned = (int64_t)st[ST_TOMBSTONED];
  }
  return status;
}

int gh_read_failed(void* h, uint32_t* bitmap, int64_t n_words) {
  Engine* e = static_cast<Engine*>(h);
  if (!e || !bitmap) return GH_EINVAL;
  const int64_t words = (e->n + 31) / 32;
  if (n_words < words) return set_err(e, GH_EINVAL, "bitmap too small");
  HIPCHK(e, hipSetDevice(e->cfg.device));
  const GhDev& d = e->d;
  Staging st;
  int rc;
  if ((rc = st.alloc(e, sizeof(uint32_t) * (size_t)d.ncsw * e->world))) return rc;
  // shard g's pending D bits cover members [g*ncs, (g+1)*ncs): word-aligned
  // (row layout: every shard holds all of them)
  if (e->rowlay)
    HIPCHK(e, hipMemcpyAsync(st.p, d.dbits, sizeof(uint32_t) * d.ncsw, hipMemcpyDeviceToDevice, e->stream));
  else
    COMMCHK(e, e->comm->allgather(d.dbits, st.p, sizeof(uint32_t) * d.ncsw, e->stream));
  std::memset(bitmap, 0, n_words * sizeof(uint32_t));
  HIPCHK(e, hipMemcpyAsync(bitmap, st.p, words * sizeof(uint32_t), hipMemcpyDeviceToHost, e->stream));
  HIPCHK(e, hipStreamSynchronize(e->stream));
  return GH_OK;
}

int gh_read_detectors(void* h, int32_t* rows, int64_t cap, int64_t* n_out) {
  Engine* e = static_cast<Engine*>(h);
  if (!e || !n_out || (cap > 0 && !rows)) return GH_EINVAL;
  HIPCHK(e, hipSetDevice(e->cfg.device));
  Staging st;
  int rc;
  if ((rc = st.alloc(e, e->n))) return rc;
  COMMCHK(e, e->comm->allreduce(e->d.det_any, st.p, e->n, GH_DT_U8, GH_OP_MAX, e->stream));
  std::vector<uint8_t> any(e->n);
  HIPCHK(e, hipMemcpyAsync(any.data(), st.p, e->n, hipMemcpyDeviceToHost, e->stream));
  HIPCHK(e, hipStreamSynchronize(e->stream));
  int64_t k = 0;
  for (int32_t i = 0; i < e->n; ++i)
    if (any[i]) {
      if (k < cap) rows[k] = i;
      k++;
    }
  *n_out = k;
  return GH_OK;
}

int gh_lsm(void* h, int32_t observer, int32_t* ids, int32_t* hb, int32_t* ts, int64_t cap, int64_t* n_out) {
  Engine* e = static_cast<Engine*>(h);
  if (!e || !n_out) return GH_EINVAL;
  if (observer < 0 || observer >= e->n) return set_err(e, GH_EINVAL, "observer");
  HIPCHK(e, hipSetDevice(e->cfg.device));
  std::vector<int32_t> rh(e->n), rt(e->n);
  int rc = gh_export_state(h, rh.data(), rt.data(), nullptr, observer, 1);
  if (rc != GH_OK) return rc;
  std::vector<int32_t> order;  // list order (GH_ORDER_APPEND), else member-ID order
  if (e->lorder) {
    int32_t len = 0;
    uint8_t b = 0;
    HIPCHK(e, hipMemcpyAsync(&len, e->d.llen[e->lcur] + observer, sizeof len, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(e, hipMemcpyAsync(&b, e->d.lsel[e->lcur] + observer, 1, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(e, hipStreamSynchronize(e->stream));
    order.resize(std::max<int32_t>(len, 0));
    if (len > 0)
      HIPCHK(e, hipMemcpyAsync(order.data(), e->d.lord[b & 1] + (int64_t)observer * e->ld, sizeof(int32_t) * len,
                               hipMemcpyDeviceToHost, e->stream));
    HIPCHK(e, hipStreamSynchronize(e->stream));
  } else {
    for (int32_t c = 0; c < e->n; ++c)
      if (rh[c] >= 0) order.push_back(c);
  }
  int64_t k = 0;
  for (int32_t c : order)
    if (rh[c] >= 0) {
      if (k < cap) {
        if (ids) ids[k] = c;
        if (hb) hb[k] = rh[c];
        if (ts) ts[k] = rt[c];
      }
      k++;
    }
  *n_out = k;
  return GH_OK;
}

int gh_merge_list(void* h, int32_t observer, const int32_t* ids, const int32_t* hb, int64_t n, int64_t* merged) {
  Engine* e = static_cast<Engine*>(h);
  if (!e || n < 0 || (n > 0 && (!ids || !hb))) return GH_EINVAL;
  if (observer < 0 || observer >= e->n) return set_err(e, GH_EINVAL, "observer");
  {
    std::vector<int32_t> s(ids, ids + n);
    for (int64_t x = 0; x < n; ++x) {
      if (ids[x] < 0 || ids[x] >= e->n) return set_err(e, GH_EINVAL, "member id out of range");
      if (hb[x] < 0) return set_err(e, GH_ERANGE, "heartbeat below 0");
    }
    std::sort(s.begin(), s.end());
    if (std::adjacent_find(s.begin(), s.end()) != s.end()) return set_err(e, GH_EINVAL, "member ids must be distinct");
  }
  HIPCHK(e, hipSetDevice(e->cfg.device));
  int rc0;
  if ((rc0 = check_lost(e)) || (rc0 = maybe_grow(e))) return rc0;
  e->qforce = true;
  e->flags_known = false;
  e->sforce = true;
  int32_t cnt = 0;
  if (n > 0 && e->alive[observer]) {  // GetMsg runs only while Alive (slave/slave.go:208)
    Staging st;
    int rc;
    if ((rc = st.alloc(e, sizeof(int32_t) * 2 * n))) return rc;
    HIPCHK(e, hipMemcpyAsync(st.p, ids, sizeof(int32_t) * n, hipMemcpyHostToDevice, e->stream));
    HIPCHK(e, hipMemcpyAsync(st.as<int32_t>() + n, hb, sizeof(int32_t) * n, hipMemcpyHostToDevice, e->stream));
    HIPCHK(e, hipMemsetAsync(e->d.nd + 5, 0, sizeof(int32_t), e->stream));
    const GhRound p = round_params(e, e->round + 1);
    launch_merge_list(e->d, e->cur, observer, st.as<int32_t>(), st.as<int32_t>() + n, n, p, e->stream);
    HIPCHK(e, hipGetLastError());
    if ((rc = allreduce_i32(e, e->d.nd + 5, e->d.nd + 5, 1))) return rc;
    if (e->lorder) {  // added members in datagram order (:433-437), then the row back in place
      if ((rc = upload(e, e->rows_buf, {observer}))) return rc;
      launch_list_events(e->d, e->cur, e->lcur, e->rows_buf, 1, st.as<int32_t>(), (int32_t)n, -1, -1, e->stream);
      const int g = e->lcur, g2 = g ^ 1;  // the row's new generation becomes its current one
      HIPCHK(e, hipMemcpyAsync(e->d.lsel[g] + observer, e->d.lsel[g2] + observer, 1, hipMemcpyDeviceToDevice, e->stream));
      HIPCHK(e, hipMemcpyAsync(e->d.llen[g] + observer, e->d.llen[g2] + observer, sizeof(int32_t),
                               hipMemcpyDeviceToDevice, e->stream));
      HIPCHK(e, hipMemcpyAsync(e->d.lself[g] + observer, e->d.lself[g2] + observer, sizeof(int32_t),
                               hipMemcpyDeviceToDevice, e->stream));
      if ((rc = list_sync(e, g))) return rc;
    }
    HIPCHK(e, hipMemcpyAsync(&cnt, e->d.nd + 5, sizeof cnt, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(e, hipStreamSynchronize(e->stream));
    int32_t err = 0;
    if ((rc = read_err(e, &err))) return rc;
    if (err) return lose(e, "gh_merge_list");
    for (int64_t x = 0; x < n; ++x) e->hb_bound = std::max<int64_t>(e->hb_bound, hb[x]);
  }
  if (merged) *merged = cnt;
  return GH_OK;
}

// File-sharded tables: each shard wrote its own files' outputs and INT32_MIN
// for the others' (place.hip), so a max over the shards is every file's.
static int merge_file_outputs(Engine* e, int64_t n, int32_t R, bool with_status) {
  if (e->world <= 1) return GH_OK;
  COMMCHK(e, e->comm->allreduce(e->d.io_b, e->d.io_b, (size_t)n * R, GH_DT_I32, GH_OP_MAX, e->stream));
  COMMCHK(e, e->comm->allreduce(e->d.io_c, e->d.io_c, (size_t)n, GH_DT_I32, GH_OP_MAX, e->stream));
  if (with_status) COMMCHK(e, e->comm->allreduce(e->d.io_d, e->d.io_d, (size_t)n, GH_DT_I32, GH_OP_MAX, e->stream));
  return GH_OK;
}

int gh_put(void* h, const int32_t* files, int64_t n, int32_t* replicas, int32_t* versions, int32_t* status) {
  Engine* e = static_cast<Engine*>(h);
  if (!e) return GH_EINVAL;
  int rc;
  if ((rc = check_files(e, files, n, true))) return rc;
  if (n == 0) return GH_OK;
  HIPCHK(e, hipSetDevice(e->cfg.device));
  if ((rc = ensure_io(e, n))) return rc;
  const int R = e->cfg.replicas;
  HIPCHK(e, hipMemcpyAsync(e->d.io_a, files, sizeof(int32_t) * n, hipMemcpyHostToDevice, e->stream));
  if ((rc = upload(e, e->rows_buf, {e->cfg.master}))) return rc;
  if ((rc = gather_rows(e, e->rows_buf, 1))) return rc;
  if (e->lorder)  // Member_list in list order
    launch_list_cand(e->d, e->lcur, e->cfg.master, e->stream);
  else
    launch_candidates(e->d, 1, e->stream);
  launch_put(e->d, 1, n, R, e->round, e->cfg.seed, e->stream);
  HIPCHK(e, hipGetLastError());
  if ((rc = merge_file_outputs(e, n, R, true))) return rc;
  std::vector<int32_t> rep(n * R), ver(n), st(n);
  HIPCHK(e, hipMemcpyAsync(rep.data(), e->d.io_b, sizeof(int32_t) * n * R, hipMemcpyDeviceToHost, e->stream));
  HIPCHK(e, hipMemcpyAsync(ver.data(), e->d.io_c, sizeof(int32_t) * n, hipMemcpyDeviceToHost, e->stream));
  HIPCHK(e, hipMemcpyAsync(st.data(), e->d.io_d, sizeof(int32_t) * n, hipMemcpyDeviceToHost, e->stream));
  HIPCHK(e, hipStreamSynchronize(e->stream));
  if (replicas) std::copy(rep.begin(), rep.end(), replicas);
  if (versions) std::copy(ver.begin(), ver.end(), versions);
  if (status) std::copy(st.begin(), st.end(), status);
  for (int64_t x = 0; x < n; ++x)
    if (st[x] != GH_OK) return set_err(e, GH_EPLACEMENT_STARVED, "placement starved for some file");
  return GH_OK;
}

int gh_put_conflicts(void* h, const int32_t* files, int64_t n, int32_t window, uint8_t* conflict) {
  Engine* e = static_cast<Engine*>(h);
  if (!e || (n > 0 && !conflict)) return GH_EINVAL;
  int rc;
  if ((rc = check_files(e, files, n, false))) return rc;
  if (n == 0) return GH_OK;
  HIPCHK(e, hipSetDevice(e->cfg.device));
  if ((rc = ensure_io(e, n))) return rc;
  HIPCHK(e, hipMemcpyAsync(e->d.io_a, files, sizeof(int32_t) * n, hipMemcpyHostToDevice, e->stream));
  launch_conflicts(e->d, n, e->round, window, e->stream);
  HIPCHK(e, hipGetLastError());
  if (e->world > 1) COMMCHK(e, e->comm->allreduce(e->d.io_d, e->d.io_d, n, GH_DT_I32, GH_OP_MAX, e->stream));
  std::vector<int32_t> out(n);
  HIPCHK(e, hipMemcpyAsync(out.data(), e->d.io_d, sizeof(int32_t) * n, hipMemcpyDeviceToHost, e->stream));
  HIPCHK(e, hipStreamSynchronize(e->stream));
  for (int64_t x = 0; x < n; ++x) conflict[x] = (uint8_t)out[x];
  return GH_OK;
}

int gh_repair(void* h, int32_t observer, gh_plan_entry* plan, int64_t cap, int64_t* n_plan) {
  Engine* e = static_cast<Engine*>(h);
  if (!e || !n_plan || (cap > 0 && !plan)) return GH_EINVAL;
  if (e->cfg.max_files <= 0) return set_err(e, GH_EINVAL, "engine created with max_files = 0");
  if (observer < 0 || observer >= e->n) return set_err(e, GH_EINVAL, "observer");
  HIPCHK(e, hipSetDevice(e->cfg.device));
  HIPCHK(e, hipMemsetAsync(e->d.nplan, 0, sizeof(int32_t), e->stream));
  int rc;
  if ((rc = upload(e, e->rows_buf, {e->cfg.master, observer}))) return rc;
  if ((rc = gather_rows(e, e->rows_buf, 2))) return rc;
  if (e->lorder)
    launch_list_cand(e->d, e->lcur, e->cfg.master, e->stream);
  else
    launch_candidates(e->d, 2, e->stream);
  launch_repair(e->d, 2, e->cfg.replicas, e->cfg.seed, e->stream);
  HIPCHK(e, hipGetLastError());
  int32_t np = 0;
  std::vector<gh_plan_entry> all;
  if (e->world > 1) {
    // each shard planned its own files: allgather the counts, then the
    // entries (padded to the largest count)
    const int G = e->world;
    Staging sc;
    if ((rc = sc.alloc(e, sizeof(int32_t) * (G + 1)))) return rc;
    int32_t* cnt = sc.as<int32_t>();
    HIPCHK(e, hipMemcpyAsync(cnt + G, e->d.nplan, sizeof(int32_t), hipMemcpyDeviceToDevice, e->stream));
    COMMCHK(e, e->comm->allgather(cnt + G, cnt, sizeof(int32_t), e->stream));
    std::vector<int32_t> counts(G);
    HIPCHK(e, hipMemcpyAsync(counts.data(), cnt, sizeof(int32_t) * G, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(e, hipStreamSynchronize(e->stream));
    const int64_t mx = *std::max_element(counts.begin(), counts.end());
    if (mx > 0) {
      Staging sp;
      const size_t B = sizeof(gh_plan_entry) * (size_t)mx;
      if ((rc = sp.alloc(e, B * (G + 1)))) return rc;
      char* base = sp.as<char>();
      if (counts[e->rank] > 0)
        HIPCHK(e, hipMemcpyAsync(base + B * G, e->d.plan, sizeof(gh_plan_entry) * counts[e->rank],
                                 hipMemcpyDeviceToDevice, e->stream));
      COMMCHK(e, e->comm->allgather(base + B * G, base, B, e->stream));
      std::vector<gh_plan_entry> got((size_t)mx * G);
      HIPCHK(e, hipMemcpyAsync(got.data(), base, B * G, hipMemcpyDeviceToHost, e->stream));
      HIPCHK(e, hipStreamSynchronize(e->stream));
      for (int g = 0; g < G; ++g) all.insert(all.end(), got.begin() + (size_t)g * mx, got.begin() + (size_t)g * mx + counts[g]);
    }
    np = (int32_t)all.size();
  } else {
    HIPCHK(e, hipMemcpyAsync(&np, e->d.nplan, sizeof np, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(e, hipStreamSynchronize(e->stream));
    all.resize(np);
    if (np > 0) {
      HIPCHK(e, hipMemcpyAsync(all.data(), e->d.plan, sizeof(gh_plan_entry) * np, hipMemcpyDeviceToHost,
                               e->stream));
      HIPCHK(e, hipStreamSynchronize(e->stream));
    }
  }
  std::sort(all.begin(), all.end(), [](const gh_plan_entry& a, const gh_plan_entry& b) { return a.file < b.file; });
  rc = GH_OK;
  for (int64_t x = 0; x < np; ++x)
    if (all[x].status != GH_OK) rc = GH_EPLACEMENT_STARVED;
  // quirk mode: Update_metadata re-makes its plan map for every repaired
  // file (master/master.go:118), so it returns the last one only (SPEC D5;
  // files in ID order stand for Go's map order); the metadata of every file
  // was repaired all the same
  if (e->cfg.detect_mode == GH_DETECT_QUIRK && np > 1) {
    all.erase(all.begin(), all.end() - 1);
    np = 1;
  }
  for (int64_t x = 0; x < np; ++x)
    if (x < cap) plan[x] = all[x];
  *n_plan = np;
  if (rc != GH_OK) set_err(e, rc, "placement starved for some file");
  return rc;
}

static int get_or_delete(Engine* e, const int32_t* files, int64_t n, int32_t* replicas, int32_t* versions,
                         int del) {
  int rc;
  if ((rc = check_files(e, files, n, del != 0))) return rc;
  if (n == 0) return GH_OK;
  HIPCHK(e, hipSetDevice(e->cfg.device));
  if ((rc = ensure_io(e, n))) return rc;
  const int R = e->cfg.replicas;
  HIPCHK(e, hipMemcpyAsync(e->d.io_a, files, sizeof(int32_t) * n, hipMemcpyHostToDevice, e->stream));
  launch_get(e->d, n, R, del, e->stream);
  HIPCHK(e, hipGetLastError());
  if ((rc = merge_file_outputs(e, n, R, false))) return rc;
  std::vector<int32_t> rep(n * R), ver(n);
  HIPCHK(e, hipMemcpyAsync(rep.data(), e->d.io_b, sizeof(int32_t) * n * R, hipMemcpyDeviceToHost, e->stream));
  HIPCHK(e, hipMemcpyAsync(ver.data(), e->d.io_c, sizeof(int32_t) * n, hipMemcpyDeviceToHost, e->stream));
  HIPCHK(e, hipStreamSynchronize(e->stream));
  if (replicas) std::copy(rep.begin(), rep.end(), replicas);
  if (versions) std::copy(ver.begin(), ver.end(), versions);
  return GH_OK;
}

int gh_get_files(void* h, const int32_t* files, int64_t n, int32_t* replicas, int32_t* versions) {
  Engine* e = static_cast<Engine*>(h);
  if (!e) return GH_EINVAL;
  return get_or_delete(e, files, n, replicas, versions, 0);
}

int gh_delete_files(void* h, const int32_t* files, int64_t n, int32_t* old_replicas) {
  Engine* e = static_cast<Engine*>(h);
  if (!e) return GH_EINVAL;
  return get_or_delete(e, files, n, old_replicas, nullptr, 1);
}

// SPEC §9: the per-row half of the election on the device; the tally is the
// host's (gossipsim.Cluster), as Receive_vote is per-candidate control flow.
int gh_vote_scan(void* h, const int32_t* mview, int32_t* first, int32_t* list_len, uint8_t* has_master) {
  Engine* e = static_cast<Engine*>(h);
  if (!e || !mview) return GH_EINVAL;
  const int32_t n = e->n;
  for (int32_t i = 0; i < n; ++i)
    if (mview[i] < 0 || mview[i] >= n) return set_err(e, GH_EINVAL, "mview: member id out of range");
  HIPCHK(e, hipSetDevice(e->cfg.device));
  Staging st;
  int rc;
  if ((rc = st.alloc(e, sizeof(int32_t) * 4 * (size_t)n))) return rc;
  int32_t* mv = st.as<int32_t>();
  int32_t* out = mv + n;       // [2n]: MAX-reduced first / has_master
  int32_t* len = out + 2 * n;  // [n]: SUM-reduced list lengths
  HIPCHK(e, hipMemcpyAsync(mv, mview, sizeof(int32_t) * n, hipMemcpyHostToDevice, e->stream));
  launch_vote_scan(e->d, e->cur, mv, out, e->stream);
  if (e->lorder) launch_list_first(e->d, e->lcur, out, e->stream);  // MemberList[0] in list order
  HIPCHK(e, hipGetLastError());
  COMMCHK(e, e->comm->allreduce(out, out, 2 * (size_t)n, GH_DT_I32, GH_OP_MAX, e->stream));
  if ((rc = allreduce_i32(e, e->d.cntl, len, (size_t)n))) return rc;
  std::vector<int32_t> host(3 * (size_t)n);
  HIPCHK(e, hipMemcpyAsync(host.data(), out, sizeof(int32_t) * 3 * n, hipMemcpyDeviceToHost, e->stream));
  HIPCHK(e, hipStreamSynchronize(e->stream));
  for (int32_t i = 0; i < n; ++i) {
    if (first) first[i] = host[i] > 0 ? n - host[i] : -1;
    if (has_master) has_master[i] = (uint8_t)host[n + i];
    if (list_len) list_len[i] = host[2 * (size_t)n + i];
  }
  return GH_OK;
}

// The whole file table <-> this shard's slots (file f at slot f / G of shard
// f % G): export allgathers every shard's slots; import keeps this shard's.
int gh_export_files(void* h, int32_t* replicas, int32_t* versions, int32_t* timestamps, uint32_t* draws) {
  Engine* e = static_cast<Engine*>(h);
  if (!e) return GH_EINVAL;
  if (e->cfg.max_files <= 0) return set_err(e, GH_EINVAL, "engine created with max_files = 0");
  HIPCHK(e, hipSetDevice(e->cfg.device));
  const GhDev& d = e->d;
  const int R = e->cfg.replicas, G = e->world;
  const int64_t slots = d.fcap, W = slots * (R + 3);  // int32 words of one shard's slots
  Staging st;
  int rc;
  if ((rc = st.alloc(e, sizeof(int32_t) * W * (G + 1)))) return rc;
  int32_t* mine = st.as<int32_t>() + W * G;
  HIPCHK(e, hipMemcpyAsync(mine, d.rep, sizeof(int32_t) * slots * R, hipMemcpyDeviceToDevice, e->stream));
  HIPCHK(e, hipMemcpyAsync(mine + slots * R, d.ver, sizeof(int32_t) * slots, hipMemcpyDeviceToDevice, e->stream));
  HIPCHK(e, hipMemcpyAsync(mine + slots * (R + 1), d.fts, sizeof(int32_t) * slots, hipMemcpyDeviceToDevice, e->stream));
  HIPCHK(e, hipMemcpyAsync(mine + slots * (R + 2), d.draws, sizeof(int32_t) * slots, hipMemcpyDeviceToDevice, e->stream));
  COMMCHK(e, e->comm->allgather(mine, st.p, sizeof(int32_t) * W, e->stream));
  std::vector<int32_t> all((size_t)W * G);
  HIPCHK(e, hipMemcpyAsync(all.data(), st.p, sizeof(int32_t) * W * G, hipMemcpyDeviceToHost, e->stream));
  HIPCHK(e, hipStreamSynchronize(e->stream));
  for (int g = 0; g < G; ++g) {
    const int32_t* b = all.data() + (size_t)W * g;
    for (int64_t fl = 0; fl < slots; ++fl) {
      const int64_t f = fl * G + g;
      if (f >= e->cfg.max_files) break;
      if (replicas)
        for (int q = 0; q < R; ++q) replicas[f * R + q] = b[fl * R + q];
      if (versions) versions[f] = b[slots * R + fl];
      if (timestamps) timestamps[f] = b[slots * (R + 1) + fl];
      if (draws) draws[f] = (uint32_t)b[slots * (R + 2) + fl];
    }
  }
  return GH_OK;
}

int gh_import_files(void* h, const int32_t* replicas, const int32_t* versions, const int32_t* timestamps,
                    const uint32_t* draws) {
  Engine* e = static_cast<Engine*>(h);
  if (!e || !replicas || !versions || !timestamps || !draws) return GH_EINVAL;
  if (e->cfg.max_files <= 0) return set_err(e, GH_EINVAL, "engine created with max_files = 0");
  const GhDev& d = e->d;
  const int R = e->cfg.replicas, G = e->world;
  const int64_t slots = d.fcap;
  std::vector<int32_t> rep((size_t)slots * R, -1), ver(slots, -1), fts(slots, 0);
  std::vector<uint32_t> dr(slots, 0);
  for (int64_t fl = 0; fl < slots; ++fl) {
    const int64_t f = fl * G + e->rank;
    if (f >= e->cfg.max_files) break;
    for (int q = 0; q < R; ++q) {
      const int32_t a = replicas[f * R + q];
      if (a < -1 || a >= e->n) return set_err(e, GH_EINVAL, "replica id out of range");
      rep[fl * R + q] = a;
    }
    ver[fl] = versions[f];
    fts[fl] = timestamps[f];
    dr[fl] = draws[f];
  }
  HIPCHK(e, hipSetDevice(e->cfg.device));
  HIPCHK(e, hipMemcpyAsync(d.rep, rep.data(), sizeof(int32_t) * rep.size(), hipMemcpyHostToDevice, e->stream));
  HIPCHK(e, hipMemcpyAsync(d.ver, ver.data(), sizeof(int32_t) * slots, hipMemcpyHostToDevice, e->stream));
  HIPCHK(e, hipMemcpyAsync(d.fts, fts.data(), sizeof(int32_t) * slots, hipMemcpyHostToDevice, e->stream));
  HIPCHK(e, hipMemcpyAsync(d.draws, dr.data(), sizeof(uint32_t) * slots, hipMemcpyHostToDevice, e->stream));
  HIPCHK(e, hipStreamSynchronize(e->stream));
  return GH_OK;
}

int gh_set_master(void* h, int32_t master) {
  Engine* e = static_cast<Engine*>(h);
  if (!e) return GH_EINVAL;
  if (master < 0 || master >= e->n) return set_err(e, GH_EINVAL, "master");
  e->cfg.master = master;
  return GH_OK;
}

int gh_rebuild_meta(void* h, int32_t new_master, int32_t* f0, int64_t* n_files) {
  Engine* e = static_cast<Engine*>(h);
  if (!e) return GH_EINVAL;
  if (new_master < 0 || new_master >= e->n) return set_err(e, GH_EINVAL, "new_master");
  if (e->cfg.max_files <= 0) return set_err(e, GH_EINVAL, "engine created with max_files = 0");
  // the first 5 members of M's list (list order); 5 covers "first 4 other than M"
  std::vector<int32_t> ids(e->n);
  int64_t nl = 0;
  int rc = gh_lsm(h, new_master, ids.data(), nullptr, nullptr, e->n, &nl);
  if (rc != GH_OK) return rc;
  if (nl == 0) return set_err(e, GH_EINVAL, "new master's list is empty");
  int32_t L[5] = {-1, -1, -1, -1, -1};
  const int32_t k = (int32_t)std::min<int64_t>(nl, 5);
  for (int32_t q = 0; q < k; ++q) L[q] = ids[q];
  const int32_t m_listed = std::find(ids.begin(), ids.begin() + nl, new_master) != ids.begin() + nl;
  launch_rebuild(e->d, e->cfg.replicas, new_master, L, k, m_listed, e->round, e->stream);
  HIPCHK(e, hipGetLastError());
  std::vector<int32_t> ver(e->d.fcap);
  HIPCHK(e, hipMemcpyAsync(ver.data(), e->d.ver, sizeof(int32_t) * e->d.fcap, hipMemcpyDeviceToHost, e->stream));
  HIPCHK(e, hipStreamSynchronize(e->stream));
  int32_t kept = (int32_t)std::count_if(ver.begin(), ver.end(), [](int32_t v) { return v >= 0; });
  if (e->world > 1) {  // each shard counted its own files
    Staging sk;
    if ((rc = sk.alloc(e, sizeof(int32_t)))) return rc;
    HIPCHK(e, hipMemcpyAsync(sk.p, &kept, sizeof kept, hipMemcpyHostToDevice, e->stream));
    if ((rc = allreduce_i32(e, sk.as<int32_t>(), sk.as<int32_t>(), 1))) return rc;
    HIPCHK(e, hipMemcpyAsync(&kept, sk.p, sizeof kept, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(e, hipStreamSynchronize(e->stream));
  }
  e->cfg.master = new_master;
  if (f0) *f0 = L[0];
  if (n_files) *n_files = kept;
  return GH_OK;
}

int gh_set_round_variant(void* h, int32_t nontemporal, int32_t xcd_map) {
  Engine* e = static_cast<Engine*>(h);
  if (!e) return GH_EINVAL;
  e->nt = nontemporal != 0;
  e->xmap = xcd_map != 0;
  return GH_OK;
}

int gh_set_timing(void* h, int32_t enable) {
  Engine* e = static_cast<Engine*>(h);
  if (!e) return GH_EINVAL;
  e->timing = enable != 0;
  e->timed_ms = 0.0;
  e->timed_launches = 0;
  if (e->timing && !e->vlog) {  // the variant log, outside the timed steps
    HIPCHK(e, hipSetDevice(e->cfg.device));
    HIPCHK(e, hipMalloc(&e->vlog, sizeof(int32_t) * 4096));
    e->vlog_cap = 4096;
  }
  return GH_OK;
}

int gh_read_timing(void* h, double* total_ms, int64_t* launches) {
  Engine* e = static_cast<Engine*>(h);
  if (!e) return GH_EINVAL;
  if (total_ms) *total_ms = e->timed_ms;
  if (launches) *launches = e->timed_launches;
  return GH_OK;
}

// Debug hook (not part of the ABI header): raw narrow codes of row `row`,
// local columns [c0, c0 + n) of the current buffer, and their bases.
int gh_debug_raw(void* h, int32_t row, int64_t c0, int64_t n, uint16_t* codes, int32_t* bases) {
  Engine* e = static_cast<Engine*>(h);
  if (!e || row < 0 || row >= e->n || c0 < 0 || c0 + n > e->ld) return GH_EINVAL;
  HIPCHK(e, hipSetDevice(e->cfg.device));
  for (int64_t c = c0; c < c0 + n; ++c) {
    const int64_t slot = e->rowlay ? e->rslot_h[row] : row;
    if (slot < 0 || slot >= e->d.nrows) return set_err(e, GH_EINVAL, "row not owned by this shard");
    const int64_t cell = gh_cell_slot(e->d, slot, c);
    int32_t m8 = 0;
    uint32_t a4 = 0, u4 = 0;
    if (e->c8) {
      HIPCHK(e, hipMemcpy(&m8, e->d.m8 + e->cur, 4, hipMemcpyDeviceToHost));
      HIPCHK(e, hipMemcpy(&a4, e->d.a4[e->cur] + (cell >> 3), 4, hipMemcpyDeviceToHost));
      HIPCHK(e, hipMemcpy(&u4, e->d.pl[e->cur] + (cell >> 3), 4, hipMemcpyDeviceToHost));
    }
    if (m8 && !gh_t4_esc(a4)) {  // the 16-bit code of a tier cell
      const int sh = gh_nib((int)(c & 7));
      const uint32_t u = (u4 >> sh) & 15u, a = (a4 >> sh) & 15u;
      const int diag = e->d.col0 + c == row;  // the plane's diagonal code
      // u = 15: absent (age nibble 15) or a tombstone of age toff + a (a
      // tier tombstone exists only with an offset, and its age lies in
      // 0..30: anything else is a corrupt cell, reported as an error)
      if (u == 15u && a != 15u && (e->d.toff == GH_TOFF_NONE || e->d.toff + (int)a < 0 || e->d.toff + (int)a > 30))
        return set_err(e, GH_EINVAL, "a tier tombstone outside the tombstone window");
      codes[c - c0] = u == 15u ? (uint16_t)(a == 15u ? GH_N_ABSENT : (GH_N_TOMB | (uint32_t)(e->d.toff + (int)a)))
                               : (uint16_t)(((GH_P_REF + 1 - diag - (int)u) << 5) | a);
    } else {
      HIPCHK(e, hipMemcpy(codes + (c - c0), e->d.hn[e->cur] + cell, 2, hipMemcpyDeviceToHost));
    }
    HIPCHK(e, hipMemcpy(bases + (c - c0), e->d.base[e->cur] + c, 4, hipMemcpyDeviceToHost));
  }
  return GH_OK;
}

// Debug hook (not part of the ABI header): the 4-bit tier nibbles of row
// `row`, local columns [c0, c0 + n) of the current buffer: (lag code << 4) |
// age nibble per cell, or 0xFF where the chunk is escaped or the buffer is
// not in the tier.
// Debug (tests only, not in the header, like gh_debug_tier): recounts the
// present cells of every running row this engine holds in the current
// buffer (k_count) and compares them with the maintained counts cntl, which
// the rounds, events and list merges keep by per-segment deltas and which
// the <4 guard and active[] read. *mismatched = rows whose maintained count
// differs, *first_row = the first of them (-1: none). The maintained counts
// are restored, so the check changes nothing.
// Debug (tests only, not in the header): the D7 shadow entries of this
// engine's local columns [col0, col0 + ncols): out[c] = the ts of the
// introducer's RecentFailList entry beside its present member, or
// GH_NO_SHADOW; *count = entries the engine counts (nshadow).
int gh_debug_shadow(void* h, int32_t* out, int64_t n_out, int32_t* count) {
  Engine* e = static_cast<Engine*>(h);
  if (!e || !out || !count || n_out < e->d.ncol) return GH_EINVAL;
  HIPCHK(e, hipSetDevice(e->cfg.device));
  HIPCHK(e, hipMemcpyAsync(out, e->d.shadow, sizeof(int32_t) * (size_t)e->d.ncol, hipMemcpyDeviceToHost, e->stream));
  HIPCHK(e, hipMemcpyAsync(count, e->d.nshadow, sizeof(int32_t), hipMemcpyDeviceToHost, e->stream));
  HIPCHK(e, hipStreamSynchronize(e->stream));
  return GH_OK;
}

int gh_debug_counts(void* h, int64_t* mismatched, int32_t* first_row) {
  Engine* e = static_cast<Engine*>(h);
  if (!e || !mismatched || !first_row) return GH_EINVAL;
  HIPCHK(e, hipSetDevice(e->cfg.device));
  const size_t bytes = sizeof(int32_t) * (size_t)e->n;
  std::vector<int32_t> kept(e->n), exact(e->n);
  HIPCHK(e, hipMemcpyAsync(kept.data(), e->d.cntl, bytes, hipMemcpyDeviceToHost, e->stream));
  launch_count(e->d, e->cur, round_params(e, e->round + 1), e->stream);
  HIPCHK(e, hipGetLastError());
  HIPCHK(e, hipMemcpyAsync(exact.data(), e->d.cntl, bytes, hipMemcpyDeviceToHost, e->stream));
  HIPCHK(e, hipMemcpyAsync(e->d.cntl, kept.data(), bytes, hipMemcpyHostToDevice, e->stream));
  HIPCHK(e, hipStreamSynchronize(e->stream));
  *mismatched = 0;
  *first_row = -1;
  for (int64_t i = 0; i < e->n; ++i) {
    const bool held = !e->rowlay || (i >= e->d.row0 && i < e->d.row0 + e->d.nrows);
    if (!held || !e->alive[i] || kept[i] == exact[i]) continue;
    if (*first_row < 0) *first_row = (int32_t)i;
    ++*mismatched;
  }
  return GH_OK;
}

int gh_debug_tier(void* h, int32_t row, int64_t c0, int64_t n, uint8_t* out) {
  Engine* e = static_cast<Engine*>(h);
  if (!e || !out || row < 0 || row >= e->n || c0 < 0 || c0 + n > e->ld) return GH_EINVAL;
  HIPCHK(e, hipSetDevice(e->cfg.device));
  HIPCHK(e, hipStreamSynchronize(e->stream));
  int32_t m8 = 0;
  if (e->c8) HIPCHK(e, hipMemcpy(&m8, e->d.m8 + e->cur, 4, hipMemcpyDeviceToHost));
  const int64_t slot = e->rowlay ? e->rslot_h[row] : row;
  if (slot < 0 || slot >= e->d.nrows) return set_err(e, GH_EINVAL, "row not owned by this shard");
  for (int64_t c = c0; c < c0 + n; ++c) {
    out[c - c0] = 0xFF;
    if (!m8) continue;
    const int64_t cell = gh_cell_slot(e->d, slot, c);
    uint32_t a4 = 0, u4 = 0, a40 = 0;
    HIPCHK(e, hipMemcpy(&a4, e->d.a4[e->cur] + (cell >> 3), 4, hipMemcpyDeviceToHost));
    HIPCHK(e, hipMemcpy(&u4, e->d.pl[e->cur] + (cell >> 3), 4, hipMemcpyDeviceToHost));
    a40 = a4;
    if (gh_t4_esc(a40)) continue;
    const int sh = gh_nib((int)(c & 7));
    out[c - c0] = (uint8_t)((((u4 >> sh) & 15u) << 4) | ((a4 >> sh) & 15u));
  }
  return GH_OK;
}

int gh_sync(void* h) {
  Engine* e = static_cast<Engine*>(h);
  if (!e) return GH_EINVAL;
  HIPCHK(e, hipSetDevice(e->cfg.device));
  HIPCHK(e, hipStreamSynchronize(e->stream));
  return GH_OK;
}

}  // extern "C"
