/*
 * ORACLE / TEST INFRASTRUCTURE ONLY.
 *
 * tablesim — a plain-C CPU restatement of the reference's gossip membership,
 * failure detection and replica placement, in the synchronous-round form of
 * SPEC.md. It is the checker for libgossiphip's HIP path: only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg load it. Nothing in
 * the product path links or calls it.
 *
 * It is written as the straightforward multi-phase algorithm (phase A: steps
 * 1-5 per row; snapshot copy; phase B: ring targets; phase C: merge), not the
 * GPU's single-pass form, so that the two are independent implementations.
 *
 * Reference functions restated (paths under /root/reference):
 *   removeMember        slave/slave.go:276-286   -> or_remove_member
 *   MergeMemberList     slave/slave.go:414-440   -> or_merge_row
 *   updateMemberList    slave/slave.go:442-458   -> phase_a (own hb++)
 *   detectfailure       slave/slave.go:460-482   -> phase_a (detect)
 *   cleanFailList       slave/slave.go:484-497   -> phase_a (clean)
 *   HeartBeat           slave/slave.go:499-544   -> guard + ring targets
 *   addNewMember/Join   slave/slave.go:250-308   -> apply_events (join)
 *   Leave               slave/slave.go:310-336   -> apply_events (leave)
 *   Init_replica        master/master.go:129-150 -> or_init_replica
 *   Handle_put_request  master/master.go:152-175 -> or_put
 *   Update_metadata     master/master.go:74-127  -> or_repair
 *   Get_file_* / Delete master/master.go:177-259 -> or_get_files/or_delete_files
 *
 * Parity status: the reference has no tests, fixtures or runnable toolchain
 * here (no Go), so this oracle is pinned by hand-derived known-answer tests
 * (tests/golden/) and by cross-checking against the literal
 * list-semantics replay oracle/listsim.py — not by reference outputs
 * ("parity unpinned" against the reference binary itself).
 */
#include <limits.h>
#include <omp.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../include/gossiphip.h"
#include "philox.h"

#define OR_MAX_DRAWS_PER_CALL (1u << 20)

typedef struct ors {
  gh_config cfg;
  int32_t n;     /* members (columns)                                      */
  int64_t rows;  /* observer rows (== n except in the bench sample)        */
  int32_t round; /* last completed round                                   */
  int32_t *hb, *ts, *snap;
  uint8_t *alive, *active, *det_any;
  int32_t *det_cnt, *det_min;   /* pending REMOVE set D_{r-1} (per column) */
  int32_t *ndet_cnt, *ndet_min; /* detections of the current round         */
  int32_t *targets;             /* ring mode: rows x 3                     */
  /* GH_REMOVE_LIST (the reference's REMOVE recipients, slave/slave.go:344):
   * per row the members listed before the detection sweep (self excluded)
   * and the members the sweep detected, W = ceil(n / 64) words each; per
   * column the rows REMOVE(c) reaches: recv (D_{r-1}, delivered in step 1)
   * and nrecv (D_r, built after phase A) */
  int64_t W;
  uint64_t *lbase, *ldet, *recv, *nrecv;
  /* SPEC D7: a JOIN of a member the introducer holds tombstoned appends it to
   * MemberList while its RecentFailList entry stays (slave/slave.go:228-230,
   * 250-255: MemberInList reads MemberList only). shadow[c] = the ts of that
   * entry beside the present cell (I, c), OR_NO_SHADOW when none. */
  int32_t *shadow;
  gh_event *ev;
  int64_t nev, evcap;
  int64_t fcap;
  int32_t *rep, *ver, *fts;
  uint32_t *draws;
  int threads;
  char err[256];
} ors;

#define OR_NO_SHADOW INT32_MIN
#define HB(s, i, c) ((s)->hb[(int64_t)(i) * (s)->n + (c)])
#define TS(s, i, c) ((s)->ts[(int64_t)(i) * (s)->n + (c)])
#define SNAP(s, i, c) ((s)->snap[(int64_t)(i) * (s)->n + (c)])

static int fail(ors *s, int code, const char *msg) {
  if (s) snprintf(s->err, sizeof s->err, "%s", msg);
  return code;
}

int or_create(const gh_config *cfg, int64_t rows, void **out) {
  if (!cfg || !out || cfg->n_members < 1 || rows < 1 || rows > cfg->n_members) return GH_EINVAL;
  if (cfg->fanout < 1 || cfg->fanout > 8 || cfg->replicas < 1 || cfg->replicas > 8) return GH_EINVAL;
  ors *s = (ors *)calloc(1, sizeof(ors));
  s->cfg = *cfg;
  s->n = cfg->n_members;
  s->rows = rows;
  int64_t cells = (int64_t)rows * s->n;
  s->hb = (int32_t *)malloc(cells * 4);
  s->ts = (int32_t *)malloc(cells * 4);
  s->snap = (int32_t *)malloc(cells * 4);
  s->alive = (uint8_t *)calloc(rows, 1);
  s->active = (uint8_t *)calloc(rows, 1);
  s->det_any = (uint8_t *)calloc(rows, 1);
  s->det_cnt = (int32_t *)calloc(s->n, 4);
  s->det_min = (int32_t *)malloc((size_t)s->n * 4);
  s->ndet_cnt = (int32_t *)calloc(s->n, 4);
  s->ndet_min = (int32_t *)malloc((size_t)s->n * 4);
  s->targets = (int32_t *)malloc((size_t)rows * 3 * 4);
  s->shadow = (int32_t *)malloc((size_t)s->n * 4);
  for (int32_t c = 0; c < s->n; ++c) s->shadow[c] = OR_NO_SHADOW;
  s->W = (s->n + 63) / 64;
  if (cfg->remove_mode == GH_REMOVE_LIST) {
    s->lbase = (uint64_t *)calloc((size_t)rows * s->W, 8);
    s->ldet = (uint64_t *)calloc((size_t)rows * s->W, 8);
    s->recv = (uint64_t *)calloc((size_t)s->n * s->W, 8);
    s->nrecv = (uint64_t *)calloc((size_t)s->n * s->W, 8);
  } else if (cfg->remove_mode != GH_REMOVE_ALL) {
    free(s->hb);
    free(s->ts);
    free(s->snap);
    free(s);
    return GH_EINVAL;
  }
  if (!s->hb || !s->ts || !s->snap) {
    free(s->hb);
    free(s->ts);
    free(s->snap);
    free(s);
    return GH_ENOMEM;
  }
  for (int64_t x = 0; x < cells; ++x) {
    s->hb[x] = GH_ABSENT;
    s->ts[x] = 0;
  }
  for (int32_t c = 0; c < s->n; ++c) s->det_min[c] = s->ndet_min[c] = INT_MAX;
  s->fcap = cfg->max_files;
  if (s->fcap > 0) {
    int R = cfg->replicas;
    s->rep = (int32_t *)malloc(s->fcap * R * 4);
    s->ver = (int32_t *)malloc(s->fcap * 4);
    s->fts = (int32_t *)calloc(s->fcap, 4);
    s->draws = (uint32_t *)calloc(s->fcap, 4);
    for (int64_t x = 0; x < s->fcap * R; ++x) s->rep[x] = -1;
    for (int64_t f = 0; f < s->fcap; ++f) s->ver[f] = -1;
  }
  s->threads = 1;
  *out = s;
  return GH_OK;
}

void or_destroy(void *h) {
  ors *s = (ors *)h;
  if (!s) return;
  free(s->hb);
  free(s->ts);
  free(s->snap);
  free(s->alive);
  free(s->active);
  free(s->det_any);
  free(s->det_cnt);
  free(s->det_min);
  free(s->lbase);
  free(s->ldet);
  free(s->recv);
  free(s->nrecv);
  free(s->ndet_cnt);
  free(s->ndet_min);
  free(s->targets);
  free(s->shadow);
  free(s->ev);
  free(s->rep);
  free(s->ver);
  free(s->fts);
  free(s->draws);
  free(s);
}

const char *or_last_error(void *h) { return h ? ((ors *)h)->err : "null handle"; }

int or_set_threads(void *h, int threads) {
  ors *s = (ors *)h;
  s->threads = threads < 1 ? 1 : threads;
  return GH_OK;
}

int or_import_state(void *h, const int32_t *hb, const int32_t *ts, const uint8_t *alive,
                    int64_t row0, int64_t n_rows, int32_t round) {
  ors *s = (ors *)h;
  if (row0 < 0 || n_rows < 0 || row0 + n_rows > s->rows) return fail(s, GH_EINVAL, "row range");
  for (int64_t x = 0; x < n_rows * s->n; ++x) {
    if (hb[x] < GH_TOMBSTONE) return fail(s, GH_ERANGE, "hb below -2"); /* Go int: any value >= 0 */
  }
  memcpy(s->hb + row0 * s->n, hb, n_rows * s->n * 4);
  memcpy(s->ts + row0 * s->n, ts, n_rows * s->n * 4);
  memcpy(s->alive + row0, alive, n_rows);
  s->round = round;
  for (int32_t c = 0; c < s->n; ++c) {
    s->det_cnt[c] = 0;
    s->det_min[c] = INT_MAX;
    s->shadow[c] = OR_NO_SHADOW; /* an imported list holds no member twice */
  }
  memset(s->det_any, 0, s->rows);
  return GH_OK;
}

/* Exported ts (SPEC.md §1): 0 for an absent member (the reference keeps no
 * entry for it); with COOLDOWN < 30 rounds, a tombstone older than
 * COOLDOWN + 1 rounds as exactly COOLDOWN + 1 rounds old -- its UpdateTime is
 * only ever compared with now - COOLDOWN (cleanFailList,
 * slave/slave.go:490), so every older value decides the same. */
static int32_t export_ts(const ors *s, int32_t hb, int32_t ts) {
  if (hb == GH_ABSENT) return 0;
  int32_t now = s->round + 1;
  const int32_t tsa = s->cfg.t_cleanup + 1;
  if (hb == GH_TOMBSTONE && s->cfg.t_cleanup < 30 && (int64_t)now - ts > tsa) return now - tsa;
  return ts;
}

int or_export_state(void *h, int32_t *hb, int32_t *ts, uint8_t *alive, int64_t row0,
                    int64_t n_rows) {
  ors *s = (ors *)h;
  if (row0 < 0 || n_rows < 0 || row0 + n_rows > s->rows) return fail(s, GH_EINVAL, "row range");
  if (hb) memcpy(hb, s->hb + row0 * s->n, n_rows * s->n * 4);
  if (ts) {
    const int32_t *H = s->hb + row0 * s->n, *T = s->ts + row0 * s->n;
    for (int64_t x = 0; x < n_rows * s->n; ++x) ts[x] = export_ts(s, H[x], T[x]);
  }
  if (alive) memcpy(alive, s->alive + row0, n_rows);
  return GH_OK;
}

int or_init_full(void *h, int32_t hb0, int32_t ts0, int32_t round) {
  ors *s = (ors *)h;
  if (hb0 < 0) return fail(s, GH_ERANGE, "hb0");
  int64_t cells = s->rows * s->n;
  for (int64_t x = 0; x < cells; ++x) {
    s->hb[x] = hb0;
    s->ts[x] = ts0;
  }
  memset(s->alive, 1, s->rows);
  s->round = round;
  for (int32_t c = 0; c < s->n; ++c) {
    s->det_cnt[c] = 0;
    s->det_min[c] = INT_MAX;
    s->shadow[c] = OR_NO_SHADOW;
  }
  return GH_OK;
}

/* Test access to the D7 shadow entries (SPEC D7): out[c] = the ts of the
 * introducer's RecentFailList entry beside its present member c, or
 * INT32_MIN. */
int or_debug_shadow(void *h, int32_t *out) {
  ors *s = (ors *)h;
  memcpy(out, s->shadow, (size_t)s->n * 4);
  return GH_OK;
}

int or_get_round(void *h, int32_t *round) {
  *round = ((ors *)h)->round;
  return GH_OK;
}

int or_apply_events(void *h, const gh_event *ev, int64_t n) {
  ors *s = (ors *)h;
  for (int64_t x = 0; x < n; ++x) {
    if (ev[x].kind < GH_EV_JOIN || ev[x].kind > GH_EV_CRASH) return fail(s, GH_EINVAL, "event kind");
    if (ev[x].member < 0 || ev[x].member >= s->rows) return fail(s, GH_EINVAL, "event member");
  }
  if (s->nev + n > s->evcap) {
    s->evcap = (s->nev + n) * 2 + 16;
    s->ev = (gh_event *)realloc(s->ev, s->evcap * sizeof(gh_event));
  }
  memcpy(s->ev + s->nev, ev, n * sizeof(gh_event));
  s->nev += n;
  return GH_OK;
}

/* removeMember(c) at row j (slave/slave.go:276-286). At the introducer a
 * member that is also in RecentFailList (D7 shadow) leaves MemberList and
 * keeps that entry, with its own ts, and nothing is appended (:278-281). */
static inline void or_remove_member(ors *s, int64_t j, int32_t c, gh_round_stats *st) {
  int32_t v = HB(s, j, c);
  if (v >= 0 && j == s->cfg.introducer && s->shadow[c] != OR_NO_SHADOW) {
    HB(s, j, c) = GH_TOMBSTONE;
    TS(s, j, c) = s->shadow[c];
    s->shadow[c] = OR_NO_SHADOW;
  } else if (v >= 0) {
    HB(s, j, c) = GH_TOMBSTONE; /* appended to RecentFailList with its ts (:280) */
    st->tombstoned++;
  } else if (v == GH_ABSENT) {
    st->remove_unknown++; /* reference: MemberList[-1] panic (:280) */
  }
}

/* MergeMemberList (slave/slave.go:414-440) of one message `msg` (n cells,
 * >=0 present) into row j at time r. */
static inline int64_t or_merge_row(ors *s, int64_t j, const int32_t *msg, int32_t r) {
  int64_t merged = 0;
  int32_t *row = s->hb + j * s->n;
  int32_t *trow = s->ts + j * s->n;
  for (int32_t c = 0; c < s->n; ++c) {
    int32_t m = msg[c];
    if (m < 0) continue;
    int32_t v = row[c];
    /* present and lower (:424-426) or absent and not tombstoned (:430-438) */
    if (v >= GH_ABSENT && m > v) {
      row[c] = m;
      trow[c] = r;
      merged++;
    }
  }
  return merged;
}

static void apply_events(ors *s, int32_t r, gh_round_stats *st) {
  if (s->nev == 0) return;
  /* crashes */
  for (int64_t x = 0; x < s->nev; ++x)
    if (s->ev[x].kind == GH_EV_CRASH) s->alive[s->ev[x].member] = 0;
  /* leaves: every leaver stops first (Alive=false, slave/slave.go:551,334) */
  uint8_t *leaving = (uint8_t *)calloc(s->rows, 1);
  for (int64_t x = 0; x < s->nev; ++x) {
    int32_t c = s->ev[x].member;
    if (s->ev[x].kind == GH_EV_LEAVE && s->alive[c]) {
      leaving[c] = 1;
      s->alive[c] = 0;
    }
  }
  for (int64_t x = 0; x < s->nev; ++x) {
    int32_t c = s->ev[x].member;
    if (s->ev[x].kind != GH_EV_LEAVE || !leaving[c]) continue;
    leaving[c] = 0; /* once per leaver */
    /* LEAVE goes to every member of c's list except c (:316-319) */
    for (int64_t j = 0; j < s->rows; ++j) {
      if (j == c || !s->alive[j] || c >= s->n || HB(s, c, j) < 0) continue;
      or_remove_member(s, j, c, st); /* :232-235 */
    }
  }
  free(leaving);
  /* joins */
  int any_join = 0;
  for (int64_t x = 0; x < s->nev; ++x) {
    int32_t c = s->ev[x].member;
    if (s->ev[x].kind != GH_EV_JOIN) continue;
    any_join = 1;
    if (!s->alive[c]) { /* fresh process: empty MemberList and RecentFailList (SPEC D7) */
      for (int32_t m = 0; m < s->n; ++m) {
        HB(s, c, m) = GH_ABSENT;
        TS(s, c, m) = 0;
      }
      if (c == s->cfg.introducer)
        for (int32_t m = 0; m < s->n; ++m) s->shadow[m] = OR_NO_SHADOW;
      s->alive[c] = 1;
    }
  }
  int32_t I = s->cfg.introducer;
  if (any_join && I >= 0 && I < s->rows && s->alive[I]) {
    int added = 0;
    for (int64_t x = 0; x < s->nev; ++x) {
      int32_t c = s->ev[x].member;
      if (s->ev[x].kind != GH_EV_JOIN) continue;
      if (HB(s, I, c) < 0) { /* !MemberInList (:228-230) -> addNewMember (:250-255) */
        /* a tombstone stays in RecentFailList beside the new entry (D7) */
        if (HB(s, I, c) == GH_TOMBSTONE) s->shadow[c] = TS(s, I, c);
        HB(s, I, c) = 0;
        TS(s, I, c) = r;
        added++;
      }
    }
    if (added) {
      /* full list to every member of I's list, I and the joiner included (:256-272) */
      int32_t *msg = (int32_t *)malloc((size_t)s->n * 4);
      memcpy(msg, s->hb + (int64_t)I * s->n, (size_t)s->n * 4);
      for (int64_t j = 0; j < s->rows; ++j) {
        if (!s->alive[j] || msg[j] < 0) continue;
        st->merged_cells += or_merge_row(s, j, msg, r);
      }
      free(msg);
    }
  }
  s->nev = 0;
}

/* Phase A for one alive row i: steps 1-5 of SPEC §2. Returns 1 if active. */
static int phase_a(ors *s, int64_t i, int32_t r, gh_round_stats *st, int32_t *ldc, int32_t *ldm) {
  int32_t n = s->n;
  int32_t *row = s->hb + i * n;
  int32_t *trow = s->ts + i * n;
  /* step 1: REMOVE delivery */
  const int literal = s->cfg.remove_mode == GH_REMOVE_LIST;
  for (int32_t c = 0; c < n; ++c) {
    int32_t dc = s->det_cnt[c];
    if (dc == 0) continue;
    if (literal) {
      /* no detector of c had row i in its list when it sent REMOVE(c) */
      if (!((s->recv[(int64_t)c * s->W + (i >> 6)] >> (i & 63)) & 1u)) continue;
    } else if (dc == 1 && s->det_min[c] == i) {
      continue; /* the sole detector does not message itself (:344-346) */
    }
    or_remove_member(s, i, c, st);
  }
  /* step 2: guard */
  int64_t L = 0;
  for (int32_t c = 0; c < n; ++c) L += row[c] >= 0;
  if (L < s->cfg.min_members) {
    for (int32_t c = 0; c < n; ++c)
      if (row[c] >= 0) trow[c] = r; /* :505-507 */
    return 0;
  }
  st->active_rows++;
  /* step 3: own heartbeat (:443-448) */
  if (i < n && row[i] >= 0) {
    row[i] += 1;
    trow[i] = r;
  }
  /* step 4: detect (:460-477) */
  int32_t limit = r - s->cfg.t_fail;
  int quirk = s->cfg.detect_mode == GH_DETECT_QUIRK;
  int32_t last_present = -1;
  if (quirk)
    for (int32_t c = n - 1; c >= 0; --c)
      if (row[c] >= 0) {
        last_present = c;
        break;
      }
  int prev_cand = 0;
  int64_t off = 0;
  int found = 0;
  uint64_t *lb = literal ? s->lbase + i * s->W : NULL;
  uint64_t *ld = literal ? s->ldet + i * s->W : NULL;
  if (literal) { /* the list the sweep starts from, self excluded (:344-346) */
    memset(lb, 0, (size_t)s->W * 8);
    memset(ld, 0, (size_t)s->W * 8);
    for (int32_t c = 0; c < n; ++c)
      if (row[c] >= 0 && c != i) lb[c >> 6] |= 1ull << (c & 63);
  }
  for (int32_t c = 0; c < n; ++c) {
    int32_t v = row[c];
    if (v < 0) continue; /* not in the list */
    int cand = (c != i) && v > 1 && trow[c] < limit;
    if (!cand) {
      prev_cand = 0;
      continue;
    }
    int det = 1;
    if (quirk) {
      off = prev_cand ? off + 1 : 0;
      det = ((off & 1) == 0) || c == last_present;
    }
    prev_cand = 1;
    if (!det) continue;
    row[c] = GH_TOMBSTONE; /* removeMember keeps the stale ts (:280) */
    if (i == s->cfg.introducer && s->shadow[c] != OR_NO_SHADOW) { /* ... or the RecentFailList entry's (D7) */
      trow[c] = s->shadow[c];
      s->shadow[c] = OR_NO_SHADOW;
    }
    if (literal) ld[c >> 6] |= 1ull << (c & 63);
    st->detections++;
    found = 1;
    ldc[c] += 1; /* this thread's D_r counts; rows ascend within a thread */
    if ((int32_t)i < ldm[c]) ldm[c] = (int32_t)i;
  }
  if (found) s->det_any[i] = 1;
  /* step 5: clean (:484-497) */
  int32_t climit = r - s->cfg.t_cleanup;
  for (int32_t c = 0; c < n; ++c) {
    if (row[c] == GH_TOMBSTONE && trow[c] < climit) {
      row[c] = GH_ABSENT;
      st->released++;
    }
  }
  if (i == s->cfg.introducer) /* RecentFailList entries beside present members (D7) */
    for (int32_t c = 0; c < n; ++c)
      if (s->shadow[c] != OR_NO_SHADOW && s->shadow[c] < climit) {
        s->shadow[c] = OR_NO_SHADOW;
        st->released++;
      }
  return 1;
}

static void stats_add(gh_round_stats *a, const gh_round_stats *b) {
  a->detections += b->detections;
  a->failed_members += b->failed_members;
  a->remove_unknown += b->remove_unknown;
  a->ring_empty += b->ring_empty;
  a->active_rows += b->active_rows;
  a->merged_cells += b->merged_cells;
  a->released += b->released;
  a->tombstoned += b->tombstoned;
}

/* One round; GH_ERANGE (nothing done, the round's events stay pending) when
 * a member that runs this round (alive, not crashing or leaving in its
 * events) has its own heartbeat at INT32_MAX: Go's int would go on counting
 * (slave/slave.go:446), our int32 cannot (SPEC.md §2). */
static int one_round(ors *s, gh_round_stats *acc) {
  int32_t r = s->round + 1;
  int32_t n = s->n;
  int64_t rows = s->rows;
  gh_round_stats st;
  memset(&st, 0, sizeof st);
  for (int64_t i = 0; i < rows && i < n; ++i) {
    if (!s->alive[i] || HB(s, i, i) != INT32_MAX) continue;
    int stops = 0; /* a crash or leave of i in this round's events stops it first */
    for (int64_t x = 0; x < s->nev; ++x)
      stops |= s->ev[x].member == i && (s->ev[x].kind == GH_EV_CRASH || s->ev[x].kind == GH_EV_LEAVE);
    if (!stops) return fail(s, GH_ERANGE, "a heartbeat would pass INT32_MAX");
  }
  apply_events(s, r, &st);
  memset(s->det_any, 0, rows);
  for (int32_t c = 0; c < n; ++c) {
    s->ndet_cnt[c] = 0;
    s->ndet_min[c] = INT_MAX;
  }
  /* phase A (per-thread D_r accumulators, merged once per thread) */
#pragma omp parallel num_threads(s->threads)
  {
    gh_round_stats ls;
    memset(&ls, 0, sizeof ls);
    int32_t *ldc = (int32_t *)calloc(n, 4);
    int32_t *ldm = (int32_t *)malloc((size_t)n * 4);
    for (int32_t c = 0; c < n; ++c) ldm[c] = INT_MAX;
#pragma omp for schedule(static)
    for (int64_t i = 0; i < rows; ++i) {
      s->active[i] = 0;
      if (!s->alive[i]) continue;
      s->active[i] = (uint8_t)phase_a(s, i, r, &ls, ldc, ldm);
    }
#pragma omp critical(or_stats)
    {
      stats_add(&st, &ls);
      for (int32_t c = 0; c < n; ++c) {
        s->ndet_cnt[c] += ldc[c];
        if (ldm[c] < s->ndet_min[c]) s->ndet_min[c] = ldm[c];
      }
    }
    free(ldc);
    free(ldm);
  }
  if (s->cfg.remove_mode == GH_REMOVE_LIST) {
    /* REMOVE(c) from detector i reaches i's list as it stands right after
     * removeMember(c) in the sweep (:472-473): the listed members but the
     * ones the sweep removed up to c (ID order), c itself included */
    const int64_t W = s->W;
#pragma omp parallel for num_threads(s->threads) schedule(dynamic, 16)
    for (int32_t c = 0; c < n; ++c) {
      uint64_t *rc = s->nrecv + (int64_t)c * W;
      memset(rc, 0, (size_t)W * 8);
      if (s->ndet_cnt[c] == 0) continue;
      const int64_t cw = c >> 6;
      const uint64_t upto = (c & 63) == 63 ? ~0ull : ((1ull << ((c & 63) + 1)) - 1);
      for (int64_t i = 0; i < rows; ++i) {
        const uint64_t *ld = s->ldet + i * W;
        if (!s->active[i] || !((ld[cw] >> (c & 63)) & 1u)) continue;
        const uint64_t *lb = s->lbase + i * W;
        for (int64_t w = 0; w < W; ++w) {
          const uint64_t gone = w < cw ? ld[w] : w == cw ? (ld[w] & upto) : 0;
          rc[w] |= lb[w] & ~gone;
        }
      }
    }
    uint64_t *t = s->recv;
    s->recv = s->nrecv;
    s->nrecv = t;
  }
  /* snapshot of every active alive row after steps 1-5 (what it sends) */
#pragma omp parallel for num_threads(s->threads) schedule(static)
  for (int64_t i = 0; i < rows; ++i)
    if (s->active[i]) memcpy(s->snap + i * n, s->hb + i * n, (size_t)n * 4);

  /* phase B/C: targets and merge */
  if (s->cfg.peer_mode == GH_PEER_RING) {
    /* neighbours in list order (slave/slave.go:515-524) */
    for (int64_t sdr = 0; sdr < rows; ++sdr) {
      int32_t *t = s->targets + sdr * 3;
      t[0] = t[1] = t[2] = -1;
      if (!s->active[sdr]) continue;
      const int32_t *sn = s->snap + sdr * n;
      int64_t L = 0, idx = -1;
      for (int32_t c = 0; c < n; ++c)
        if (sn[c] >= 0) {
          if (c == sdr) idx = L;
          L++;
        }
      if (L == 0) {
        st.ring_empty++;
        continue;
      }
      int64_t want[3] = {idx - 1, idx + 1, idx + 2};
      for (int q = 0; q < 3; ++q) {
        int64_t v = want[q] % L; /* Go and C both truncate toward zero */
        if (v < 0) v += L;
        want[q] = v;
      }
      int64_t rank = 0;
      for (int32_t c = 0; c < n; ++c)
        if (sn[c] >= 0) {
          for (int q = 0; q < 3; ++q)
            if (want[q] == rank) t[q] = c;
          rank++;
        }
    }
    /* deliver: receiver i takes the max over every datagram addressed to it
     * (sequential MergeMemberList calls in any order give the same row) */
    int32_t *m = (int32_t *)malloc((size_t)n * 4);
    uint8_t *hit = (uint8_t *)calloc(rows, 1);
    for (int64_t sdr = 0; sdr < rows; ++sdr)
      for (int q = 0; q < 3; ++q) {
        int32_t tg = s->targets[sdr * 3 + q];
        if (tg >= 0 && tg < rows) hit[tg] = 1;
      }
    for (int64_t i = 0; i < rows; ++i) {
      if (!hit[i] || !s->alive[i]) continue;
      for (int32_t c = 0; c < n; ++c) m[c] = -1;
      for (int64_t sdr = 0; sdr < rows; ++sdr) {
        if (!s->active[sdr]) continue;
        const int32_t *t = s->targets + sdr * 3;
        if (t[0] != i && t[1] != i && t[2] != i) continue;
        const int32_t *sn = s->snap + sdr * n;
        for (int32_t c = 0; c < n; ++c)
          if (sn[c] > m[c]) m[c] = sn[c];
      }
      st.merged_cells += or_merge_row(s, i, m, r);
    }
    free(m);
    free(hit);
  } else {
    int k = s->cfg.fanout;
    uint64_t P = (uint64_t)rows;
#pragma omp parallel num_threads(s->threads)
    {
      int64_t merged = 0;
      int32_t *m = (int32_t *)malloc((size_t)n * 4);
#pragma omp for schedule(static)
      for (int64_t i = 0; i < rows; ++i) {
        if (!s->alive[i] || P < 2) continue;
        int have = 0;
        for (int t = 0; t < k; ++t) {
          uint32_t u = or_philox_word(s->cfg.seed, (uint32_t)i, (uint32_t)r, OR_TAG_PEER,
                                      (uint32_t)(t >> 2), t & 3);
          uint64_t q = ((uint64_t)u * (P - 1)) >> 32;
          int64_t p = (int64_t)q + ((int64_t)q >= i);
          if (!s->alive[p] || !s->active[p] || SNAP(s, p, i) < 0) continue;
          const int32_t *sn = s->snap + p * n;
          if (!have) {
            for (int32_t c = 0; c < n; ++c) m[c] = sn[c];
            have = 1;
          } else {
            for (int32_t c = 0; c < n; ++c)
              if (sn[c] > m[c]) m[c] = sn[c];
          }
        }
        if (have) merged += or_merge_row(s, i, m, r);
      }
      free(m);
#pragma omp atomic
      st.merged_cells += merged;
    }
  }
  /* D_r becomes the pending REMOVE set of round r+1 */
  int64_t nd = 0;
  for (int32_t c = 0; c < n; ++c) {
    s->det_cnt[c] = s->ndet_cnt[c];
    s->det_min[c] = s->ndet_min[c];
    nd += s->ndet_cnt[c] > 0;
  }
  st.failed_members = nd;
  s->round = r;
  acc->rounds++;
  acc->last_round = r;
  stats_add(acc, &st);
  return GH_OK;
}

int or_step(void *h, int32_t rounds, gh_round_stats *stats) {
  ors *s = (ors *)h;
  gh_round_stats acc;
  memset(&acc, 0, sizeof acc);
  acc.last_round = s->round;
  int rc = GH_OK;
  for (int32_t x = 0; x < rounds && rc == GH_OK; ++x) rc = one_round(s, &acc);
  if (stats) *stats = acc;
  return rc;
}

int or_read_failed(void *h, uint32_t *bitmap, int64_t n_words) {
  ors *s = (ors *)h;
  if (n_words < (s->n + 31) / 32) return fail(s, GH_EINVAL, "bitmap too small");
  memset(bitmap, 0, n_words * 4);
  for (int32_t c = 0; c < s->n; ++c)
    if (s->det_cnt[c] > 0) bitmap[c >> 5] |= 1u << (c & 31);
  return GH_OK;
}

int or_read_detectors(void *h, int32_t *rows_out, int64_t cap, int64_t *n_out) {
  ors *s = (ors *)h;
  int64_t k = 0;
  for (int64_t i = 0; i < s->rows; ++i)
    if (s->det_any[i]) {
      if (k < cap) rows_out[k] = (int32_t)i;
      k++;
    }
  *n_out = k;
  return GH_OK;
}

int or_lsm(void *h, int32_t obs, int32_t *ids, int32_t *hb, int32_t *ts, int64_t cap,
           int64_t *n_out) {
  ors *s = (ors *)h;
  if (obs < 0 || obs >= s->rows) return fail(s, GH_EINVAL, "observer");
  int64_t k = 0;
  for (int32_t c = 0; c < s->n; ++c)
    if (HB(s, obs, c) >= 0) {
      if (k < cap) {
        if (ids) ids[k] = c;
        if (hb) hb[k] = HB(s, obs, c);
        if (ts) ts[k] = TS(s, obs, c);
      }
      k++;
    }
  *n_out = k;
  return GH_OK;
}

/* MergeMemberList (slave/slave.go:414-440) of an external list into row obs
 * at the current tick (the last completed round); ids distinct. */
int or_merge_list(void *h, int32_t obs, const int32_t *ids, const int32_t *hb, int64_t n, int64_t *merged) {
  ors *s = (ors *)h;
  if (obs < 0 || obs >= s->rows) return fail(s, GH_EINVAL, "observer");
  uint8_t *seen = (uint8_t *)calloc(s->n, 1);
  for (int64_t x = 0; x < n; ++x) {
    int bad = ids[x] < 0 || ids[x] >= s->n ? GH_EINVAL : hb[x] < 0 ? GH_ERANGE : seen[ids[x]] ? GH_EINVAL : 0;
    if (bad) {
      free(seen);
      return fail(s, bad, bad == GH_ERANGE ? "heartbeat below 0" : "member ids out of range or repeated");
    }
    seen[ids[x]] = 1;
  }
  free(seen);
  int64_t m = 0;
  if (s->alive[obs]) {
    for (int64_t x = 0; x < n; ++x) {
      int32_t c = ids[x];
      int32_t v = HB(s, obs, c);
      if (v >= GH_ABSENT && hb[x] > v) { /* present and lower, or absent and not tombstoned */
        HB(s, obs, c) = hb[x];
        TS(s, obs, c) = s->round;
        m++;
      }
    }
  }
  *merged = m;
  return GH_OK;
}

/* ---------------------------------------------------------------- files */

/* Member_list of the master: present members of the master row, ID order
 * (master/master.go:46 aliasing slave/slave.go:478). */
static int32_t *candidates(ors *s, int64_t *M) {
  int32_t *cand = (int32_t *)malloc((size_t)s->n * 4);
  int64_t m = 0;
  int32_t ms = s->cfg.master;
  if (ms >= 0 && ms < s->rows)
    for (int32_t c = 0; c < s->n; ++c)
      if (HB(s, ms, c) >= 0) cand[m++] = c;
  *M = m;
  return cand;
}

/* Init_replica (master/master.go:129-150) with Philox draws. nodes[] holds
 * `*len` valid entries; returns GH_OK or GH_EPLACEMENT_STARVED. */
static int or_init_replica(ors *s, int32_t f, int32_t *nodes, int *len, const int32_t *cand,
                           int64_t M, const uint8_t *is_cand_choosable) {
  int R = s->cfg.replicas;
  if (*len >= R) return GH_OK;
  if (M <= 1) return GH_EPLACEMENT_STARVED; /* Intn(<=0) panics (:135) */
  int64_t in_pool = 0;
  for (int x = 0; x < *len; ++x)
    if (nodes[x] >= 0 && nodes[x] < s->n && is_cand_choosable[nodes[x]]) in_pool++;
  if ((M - 1) - in_pool < R - *len) return GH_EPLACEMENT_STARVED; /* infinite loop (:130) */
  int32_t tmp[8];
  int tl = *len;
  for (int x = 0; x < tl; ++x) tmp[x] = nodes[x];
  uint32_t d = s->draws[f];
  uint32_t budget = OR_MAX_DRAWS_PER_CALL;
  while (tl < R) {
    if (budget-- == 0) return GH_EPLACEMENT_STARVED;
    uint32_t u = or_philox_word(s->cfg.seed, (uint32_t)f, d, OR_TAG_PLACE, 0, 0);
    d++;
    uint64_t num = ((uint64_t)u * (uint64_t)(M - 1)) >> 32; /* r.Intn(len-1) (:135) */
    int32_t a = cand[num];
    int dup = 0;
    for (int x = 0; x < tl; ++x) dup |= tmp[x] == a; /* isAddressExist (:137) */
    if (!dup) tmp[tl++] = a;
  }
  s->draws[f] = d;
  for (int x = 0; x < tl; ++x) nodes[x] = tmp[x];
  *len = tl;
  return GH_OK;
}

static uint8_t *choosable_map(ors *s, const int32_t *cand, int64_t M) {
  uint8_t *map = (uint8_t *)calloc(s->n, 1);
  for (int64_t x = 0; x + 1 < M; ++x) map[cand[x]] = 1; /* the last is never drawn */
  return map;
}

int or_put(void *h, const int32_t *files, int64_t n, int32_t *replicas, int32_t *versions,
           int32_t *status) {
  ors *s = (ors *)h;
  int R = s->cfg.replicas;
  for (int64_t x = 0; x < n; ++x)
    if (files[x] < 0 || files[x] >= s->fcap) return fail(s, GH_EINVAL, "file id");
  int64_t M;
  int32_t *cand = candidates(s, &M);
  uint8_t *map = choosable_map(s, cand, M);
  int rc = GH_OK;
  for (int64_t x = 0; x < n; ++x) {
    int32_t f = files[x];
    int32_t *rp = s->rep + (int64_t)f * R;
    if (s->ver[f] < 0) { /* Update_timestamp: new File_info (:239-245) */
      s->ver[f] = 0;
      for (int q = 0; q < R; ++q) rp[q] = -1;
    }
    s->fts[f] = s->round;
    int len = 0;
    while (len < R && rp[len] >= 0) len++;
    int st = or_init_replica(s, f, rp, &len, cand, M, map);
    if (st == GH_OK) s->ver[f] += 1; /* :159 */
    else rc = GH_EPLACEMENT_STARVED;
    if (status) status[x] = st;
    if (versions) versions[x] = s->ver[f];
    if (replicas)
      for (int q = 0; q < R; ++q) replicas[x * R + q] = rp[q];
  }
  free(cand);
  free(map);
  return rc;
}

/* If_file_updated_recent (master/master.go:214-229): now - ts < 60 s. */
int or_put_conflicts(void *h, const int32_t *files, int64_t n, int32_t window, uint8_t *conflict) {
  ors *s = (ors *)h;
  for (int64_t x = 0; x < n; ++x) {
    int32_t f = files[x];
    if (f < 0 || f >= s->fcap) return fail(s, GH_EINVAL, "file id");
    conflict[x] = s->ver[f] >= 0 && (int64_t)s->round - s->fts[f] < window;
  }
  return GH_OK;
}

int or_repair(void *h, int32_t observer, gh_plan_entry *plan, int64_t cap, int64_t *n_plan) {
  ors *s = (ors *)h;
  if (observer < 0 || observer >= s->rows) return fail(s, GH_EINVAL, "observer");
  int R = s->cfg.replicas;
  int64_t M;
  int32_t *cand = candidates(s, &M);
  uint8_t *map = choosable_map(s, cand, M);
  int64_t np = 0;
  int rc = GH_OK;
  gh_plan_entry last;
  memset(&last, 0, sizeof last);
  for (int64_t f = 0; f < s->fcap; ++f) {
    if (s->ver[f] < 0) continue;
    int32_t *rp = s->rep + f * R;
    int32_t working[8];
    int wl = 0;
    for (int q = 0; q < R; ++q) {
      int32_t a = rp[q];
      if (a < 0) continue;
      if (a < s->n && HB(s, observer, a) >= 0) working[wl++] = a; /* :93-99 */
    }
    if (wl >= R) continue; /* :104 */
    for (int q = 0; q < R; ++q) rp[q] = q < wl ? working[q] : -1; /* :106 */
    int len = wl;
    int st = or_init_replica(s, (int32_t)f, rp, &len, cand, M, map); /* :107 */
    if (st != GH_OK) rc = GH_EPLACEMENT_STARVED;
    {
      gh_plan_entry *e = np < cap ? plan + np : &last;
      memset(e, 0, sizeof *e);
      e->file = (int32_t)f;
      e->node1 = wl > 0 ? working[0] : -1; /* :120 */
      e->version = s->ver[f];              /* :105 */
      e->status = st;
      int nn = 0;
      for (int q = wl; q < len; ++q) e->new_nodes[nn++] = rp[q]; /* :110-115 */
      for (int q = nn; q < 8; ++q) e->new_nodes[q] = -1;
      e->n_new = nn;
      if (e != &last) last = *e;
    }
    np++;
  }
  free(cand);
  free(map);
  /* quirk mode: the plan map is re-made per file (master/master.go:118), so
   * only the last repaired file's entry is returned */
  if (s->cfg.detect_mode == GH_DETECT_QUIRK && np > 1) {
    if (cap > 0) plan[0] = last;
    np = 1;
  }
  *n_plan = np;
  return rc;
}

int or_get_files(void *h, const int32_t *files, int64_t n, int32_t *replicas,
                 int32_t *versions) {
  ors *s = (ors *)h;
  int R = s->cfg.replicas;
  for (int64_t x = 0; x < n; ++x) {
    int32_t f = files[x];
    if (f < 0 || f >= s->fcap) return fail(s, GH_EINVAL, "file id");
    if (versions) versions[x] = s->ver[f];
    if (replicas)
      for (int q = 0; q < R; ++q) replicas[x * R + q] = s->ver[f] >= 0 ? s->rep[(int64_t)f * R + q] : -1;
  }
  return GH_OK;
}

/* The master's file metadata as flat arrays (gh_export_files /
 * gh_import_files), and the master row (gh_set_master). */
int or_export_files(void *h, int32_t *rep, int32_t *ver, int32_t *fts, uint32_t *draws) {
  ors *s = (ors *)h;
  if (!s || s->fcap <= 0) return GH_EINVAL;
  const int R = s->cfg.replicas;
  memcpy(rep, s->rep, sizeof(int32_t) * s->fcap * R);
  memcpy(ver, s->ver, sizeof(int32_t) * s->fcap);
  memcpy(fts, s->fts, sizeof(int32_t) * s->fcap);
  memcpy(draws, s->draws, sizeof(uint32_t) * s->fcap);
  return GH_OK;
}

int or_import_files(void *h, const int32_t *rep, const int32_t *ver, const int32_t *fts, const uint32_t *draws) {
  ors *s = (ors *)h;
  if (!s || s->fcap <= 0) return GH_EINVAL;
  const int R = s->cfg.replicas;
  memcpy(s->rep, rep, sizeof(int32_t) * s->fcap * R);
  memcpy(s->ver, ver, sizeof(int32_t) * s->fcap);
  memcpy(s->fts, fts, sizeof(int32_t) * s->fcap);
  memcpy(s->draws, draws, sizeof(uint32_t) * s->fcap);
  return GH_OK;
}

int or_set_master(void *h, int32_t master) {
  ors *s = (ors *)h;
  if (!s || master < 0 || master >= s->n) return GH_EINVAL;
  s->cfg.master = master;
  return GH_OK;
}

int or_delete_files(void *h, const int32_t *files, int64_t n, int32_t *old_replicas) {
  ors *s = (ors *)h;
  int R = s->cfg.replicas;
  for (int64_t x = 0; x < n; ++x) {
    int32_t f = files[x];
    if (f < 0 || f >= s->fcap) return fail(s, GH_EINVAL, "file id");
    for (int q = 0; q < R; ++q) {
      if (old_replicas) old_replicas[x * R + q] = s->ver[f] >= 0 ? s->rep[(int64_t)f * R + q] : -1;
      s->rep[(int64_t)f * R + q] = -1;
    }
    s->ver[f] = -1;
  }
  return GH_OK;
}

void or_philox(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]) {
  or_philox4x32_10_raw(ctr, key, out);
}
