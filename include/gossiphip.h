/*
 * gossiphip.h — C-ABI of libgossiphip, the MI355X-native batched
 * gossip-membership / failure-detection / replica-placement engine.
 *
 * This is the drop-in boundary for the hot path of
 * xiaoxin0515/P2P-File-system-with-Gossip-Detect-Failure-Management
 * (SURVEY.md §8b). The reference has no FFI; its hot path sits behind Go
 * methods and a net/rpc service. Each entry point below names the reference
 * interface it replaces (file:line under the reference tree). Semantics:
 * SPEC.md. Host bindings: INTEGRATION.md (cgo stub) and
 * p2p-file-system-with-gossip-detect-failure-management_amd/gossipsim (ctypes).
 *
 * Conventions
 *   - Every function returns 0 (GH_OK) or a negative GH_E* code; the reason is
 *     in gh_last_error(h). The reference instead log.Fatal/log.Panic's
 *     (slave/slave.go:214,262-270; master/master.go:130-135).
 *   - Buffers are caller-owned host memory, read or written only during the
 *     call. The handle owns all device memory (HBM) and the HIP stream.
 *   - A handle is not thread-safe (call it from one thread; cgo callers use
 *     runtime.LockOSThread).
 *   - Member IDs are dense int32 in [0, n_members); file IDs dense int32 in
 *     [0, max_files).
 *   - There is no CPU fallback: gh_create fails with GH_ENODEV when no gfx950
 *     device is usable.
 */
#ifndef GOSSIPHIP_H_
#define GOSSIPHIP_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GH_ABI_VERSION 7

/* ---- error codes ---------------------------------------------------- */
#define GH_OK 0
#define GH_EINVAL (-1)               /* bad argument / shape                    */
#define GH_ENODEV (-2)               /* no usable HIP device                    */
#define GH_ENOMEM (-3)               /* device allocation failed / wide arena full */
#define GH_EHIP (-4)                 /* HIP runtime error                       */
#define GH_EPLACEMENT_STARVED (-5)   /* master/master.go:130-135 hang / panic   */
#define GH_ERANGE (-6)               /* heartbeat would pass INT32_MAX / < range */

/* ---- cell encoding (SPEC.md §1) -------------------------------------- */
#define GH_ABSENT (-1)     /* not in MemberList                              */
#define GH_TOMBSTONE (-2)  /* in RecentFailList (slave/slave.go:65)          */

/* ---- modes ------------------------------------------------------------ */
#define GH_PEER_PULL 0     /* receiver pulls k Philox-selected peers          */
#define GH_PEER_RING 1     /* reference ring push, slave/slave.go:512-524     */
#define GH_DETECT_CANONICAL 0
#define GH_DETECT_QUIRK 1  /* Go range-over-mutated-slice skip, slave.go:464   */
/* MemberList order (SPEC.md §7 D1). GH_ORDER_ID keeps every list in member-ID
 * order: pull mode with canonical detection is order-free (the benched
 * configurations), and it needs no per-row order state. GH_ORDER_APPEND keeps
 * the reference's slice order: members are appended when added
 * (slave/slave.go:255 addNewMember, :437 MergeMemberList, in received-list
 * order, senders in ID order) and keep their relative order when others are
 * removed (:283); ring targets (:515-524), quirk runs (:464-477),
 * MemberList[0] (:936, :994), placement candidates (master/master.go:46,
 * :135) and lsm follow it. One engine or row shards (GH_LAYOUT_ROWS: every
 * shard keeps every row's list, the owners' changes are copied each round);
 * column shards refuse it (gh_create_sharded: GH_EINVAL). HBM +8*N*N bytes
 * per engine / shard (double-buffered [N][N] int32 lists); row shards also
 * keep the list copy's scratch, grown to (G + 1) x 256 MiB at most (the
 * changed lists travel in ranges of 2^26 / N rows). */
#define GH_ORDER_ID 0
#define GH_ORDER_APPEND 1
/* Who receives a detector's REMOVE (SPEC D4). GH_REMOVE_LIST is the
 * reference: Remove (slave/slave.go:338-363) runs right after removeMember
 * inside the detection sweep (:472-473) and messages every member of the
 * detector's list as it stands then (the member itself and the members the
 * sweep removed before it are gone, the later ones still listed), itself
 * excluded (:344-346). GH_REMOVE_ALL delivers it to every alive row but a sole
 * detector (equal whenever the detectors' lists agree, as in a healthy
 * cluster; the victim of a false positive then removes itself too). */
#define GH_REMOVE_ALL 0
#define GH_REMOVE_LIST 1

/* ---- events (SPEC.md §5) ---------------------------------------------- */
#define GH_EV_JOIN 1       /* slave/slave.go:288 Join + :250 addNewMember     */
#define GH_EV_LEAVE 2      /* slave/slave.go:310 Leave                        */
#define GH_EV_CRASH 3      /* README.md:30 "CTRL+C to crash node"            */

typedef struct gh_config {
  int32_t n_members;     /* N; member IDs 0..N-1                             */
  int32_t fanout;        /* k (pull mode), 1..8                              */
  int32_t peer_mode;     /* GH_PEER_PULL | GH_PEER_RING                      */
  int32_t detect_mode;   /* GH_DETECT_CANONICAL | GH_DETECT_QUIRK            */
  int32_t t_fail;        /* PERIOD in rounds, slave/slave.go:24 (5)          */
  int32_t t_cleanup;     /* COOLDOWN in rounds, slave/slave.go:25 (5)        */
  int32_t min_members;   /* literal 4, slave/slave.go:504,511                */
  int32_t replicas;      /* 4, master/master.go:131 (1..8)                   */
  int32_t introducer;    /* INTRODUCER_ADDR, slave/slave.go:22 (0)           */
  int32_t master;        /* master row whose list is Member_list (0)        */
  int32_t device;        /* HIP device ordinal                               */
  int32_t tile_width;    /* HBM layout: members per table tile (32, 64, 128,
                            256; 0 = default 64), see DESIGN.md             */
  uint64_t seed;         /* Philox key for peers and placement draws         */
  int64_t max_files;     /* file-metadata capacity (0 = no files)            */
  int64_t wide_segments; /* slots of each wide-segment arena (HBM layout,
                            DESIGN.md); 0 = auto (all segments when small,
                            else 1/32 of them, grown between calls)        */
  int32_t shard_layout;  /* sharded engines (gh_create_sharded):
                            GH_LAYOUT_COLUMNS (0, default) or GH_LAYOUT_ROWS */
  int32_t list_order;    /* GH_ORDER_ID (0, default) or GH_ORDER_APPEND      */
  int32_t remove_mode;   /* REMOVE recipients: GH_REMOVE_ALL (0, default) or
                            GH_REMOVE_LIST (the reference's, slave.go:344)  */
  int32_t reserved[3];
} gh_config;

typedef struct gh_event {
  int32_t kind;          /* GH_EV_*                                          */
  int32_t member;
} gh_event;

/* Counters accumulated over the rounds of one gh_step call. */
typedef struct gh_round_stats {
  int64_t rounds;         /* rounds executed by this call                    */
  int64_t last_round;     /* `now` of the last round executed                */
  int64_t detections;     /* cells removed by detectfailure (slave.go:472)   */
  int64_t failed_members; /* Σ_rounds distinct members detected that round   */
  int64_t remove_unknown; /* REMOVE/LEAVE of an unknown member (slave.go:280 panic) */
  int64_t ring_empty;     /* ring sender with empty list (slave.go:517 div-by-0)   */
  int64_t active_rows;    /* Σ_rounds rows passing the <4 guard              */
  int64_t merged_cells;   /* cells advanced or added by MergeMemberList      */
  int64_t released;       /* tombstones dropped by cleanFailList             */
  int64_t tombstoned;     /* tombstones created by REMOVE/LEAVE delivery     */
} gh_round_stats;

/* One re-replication plan entry (master/master.go:27-31 Replicate_info). */
typedef struct gh_plan_entry {
  int32_t file;
  int32_t node1;          /* first working replica, -1 if none (SPEC D5)     */
  int32_t version;
  int32_t n_new;
  int32_t status;         /* GH_OK or GH_EPLACEMENT_STARVED                  */
  int32_t new_nodes[8];   /* first n_new valid                               */
} gh_plan_entry;

/* Fills *cfg with the reference defaults (SURVEY.md §5 Config). */
void gh_config_default(gh_config* cfg);

/* Replaces InitSlave/InitMaster (slave/slave.go:95, master/master.go:38) for
 * N members at once. HBM: the 16-bit narrow table (x2), 4*N*N bytes; in pull
 * mode with 3 <= k <= 4 from N = 16,384 the sender plane (x2, N*N bytes) and
 * the 4-bit tier's age plane (x2, N*N bytes); plus the wide-segment arenas
 * (gh_config.wide_segments) and a frozen store for stopped rows that grows
 * with them (gh_memory_info). */
int gh_create(const gh_config* cfg, void** handle);
void gh_destroy(void* h);
const char* gh_last_error(void* h);
int gh_abi_version(void);

/* Whole-state transfer (host <-> HBM). Rows [row0, row0+n_rows) of the N x N
 * tables. `round` is the tick of the last completed round. hb: any int32
 * >= -2 (GH_ABSENT, GH_TOMBSTONE, heartbeats up to INT32_MAX; below -2 is
 * GH_ERANGE); ts: any int32. Pending REMOVEs are cleared on import. Export:
 * the ts of an absent cell is 0 (the reference keeps no entry for it), and
 * with T_cleanup < 30 a tombstone older than T_cleanup + 1 rounds exports
 * ts = round + 1 - (T_cleanup + 1) (its age is only ever compared with
 * COOLDOWN, slave/slave.go:490; SPEC.md §1). */
int gh_import_state(void* h, const int32_t* hb, const int32_t* ts,
                    const uint8_t* alive, int64_t row0, int64_t n_rows,
                    int32_t round);
int gh_export_state(void* h, int32_t* hb, int32_t* ts, uint8_t* alive,
                    int64_t row0, int64_t n_rows);
/* Every row alive and holding every member at (hb0, ts0): the synthetic
 * full-membership start of BASELINE configs 2-4, filled on the device. */
int gh_init_full(void* h, int32_t hb0, int32_t ts0, int32_t round);
int gh_get_round(void* h, int32_t* round);

/* Queue churn for the next round (GetMsg JOIN/LEAVE dispatch,
 * slave/slave.go:224-240; crash = process death). */
int gh_apply_events(void* h, const gh_event* ev, int64_t n);

/* Run `rounds` synchronous gossip rounds (HeartBeat, slave/slave.go:499,
 * driven by the 1 s loop of main.go:27-33, with MergeMemberList :414,
 * detectfailure :460, cleanFailList :484). Blocks until done; stats may be
 * NULL. Heartbeats are Go ints in the reference (master/master.go:18) and
 * int32 here: a round in which a running member's own heartbeat is
 * INT32_MAX is refused with GH_ERANGE (the rounds before it completed;
 * stats->rounds says how many). GH_ENOMEM: the wide arena overflowed inside
 * a round and the state is lost (re-import or destroy). */
int gh_step(void* h, int32_t rounds, gh_round_stats* stats);

/* Members detected in the last round as an N-bit bitmap (REMOVE broadcast
 * set, slave/slave.go:338). */
int gh_read_failed(void* h, uint32_t* bitmap, int64_t n_words);
/* Rows that detected a failure in the last round (they call Fail_recover,
 * slave/slave.go:479-481). Returns the count via *n_out (<= cap written). */
int gh_read_detectors(void* h, int32_t* rows, int64_t cap, int64_t* n_out);
/* "lsm" (slave/slave.go:558-561): observer's present members, in list order
 * (member-ID order under GH_ORDER_ID). */
int gh_lsm(void* h, int32_t observer, int32_t* ids, int32_t* hb, int32_t* ts,
           int64_t cap, int64_t* n_out);

/* MergeMemberList (slave/slave.go:414-440) of one received list into the
 * observer's row at the engine's current tick (the last completed round):
 * ids[x] (distinct members) with heartbeats hb[x] >= 0; the remote ts is
 * ignored (:426, :437). Present members advance when hb is larger, absent
 * ones are added, tombstoned ones are left alone. A stopped observer does
 * not receive (GetMsg runs while Alive). *merged = cells changed. Decoding
 * a reference datagram into (ids, hb) is the host's codec. */
int gh_merge_list(void* h, int32_t observer, const int32_t* ids, const int32_t* hb, int64_t n,
                  int64_t* merged);

/* "put" placement: Handle_put_request (master/master.go:152) for n distinct
 * files. replicas: [n][replicas] (-1 padded), versions [n], status [n]
 * (GH_OK / GH_EPLACEMENT_STARVED). Returns GH_EPLACEMENT_STARVED if any file
 * starved. */
int gh_put(void* h, const int32_t* files, int64_t n, int32_t* replicas,
           int32_t* versions, int32_t* status);
/* If_file_updated_recent (master/master.go:214-229) for n files: conflict[x]
 * = 1 if the file exists and was put less than `window` rounds ago (the
 * reference's 60 s write-write window at 1 s rounds: window = 60). The put
 * path asks for confirmation on a conflict (server/server.go:79-114). */
int gh_put_conflicts(void* h, const int32_t* files, int64_t n, int32_t window, uint8_t* conflict);
/* Update_metadata (master/master.go:74) with available = observer's list;
 * plan entries in file order. *n_plan = number of entries (<= cap written).
 * Every file's metadata is repaired. GH_DETECT_QUIRK engines also keep the
 * reference's plan-map remake (:118, SPEC D5): the plan holds only the entry
 * of the highest repaired file id (Go's map order is random, so which file
 * the reference returns is unpinned). */
int gh_repair(void* h, int32_t observer, gh_plan_entry* plan, int64_t cap,
              int64_t* n_plan);
/* get / ls (master/master.go:177-212): versions -1 if absent. */
int gh_get_files(void* h, const int32_t* files, int64_t n, int32_t* replicas,
                 int32_t* versions);
/* delete (master/master.go:249-259): old replicas returned. */
int gh_delete_files(void* h, const int32_t* files, int64_t n,
                    int32_t* old_replicas);

/* ---- master re-election (SPEC §9; slave/slave.go:930-1051) ------------- */
/* The master check at the end of updateMemberList (slave/slave.go:451-457)
 * and revote_master's target (:930-948), for every row of the current table:
 * list_len[i] = len(MemberList_i); has_master[i] = 1 if member mview[i] (row
 * i's own idea of the master, self.master) is in row i's list; first[i] =
 * MemberList_i[0] (under GH_ORDER_ID the lowest present member id, SPEC D1),
 * -1 for an empty list. mview: [N] member ids. Outputs: [N] each; any output may be NULL.
 * The vote tally (Receive_vote :968-984, RPC TCPServer.Vote
 * server/server.go:231) is per-candidate control flow and stays on the host
 * (gossipsim.Cluster). */
int gh_vote_scan(void* h, const int32_t* mview, int32_t* first, int32_t* list_len,
                 uint8_t* has_master);
/* rebuild_file_meta (slave/slave.go:986-1043) run by the newly elected
 * master M: the file table is rebuilt from the members' local stores as the
 * reference reads them (M's own, and MemberList_M[0]'s for every other member,
 * :994), Node_list = the first 4 entries in ascending-version order, Version
 * = the first entry's, Timestamp = the current tick; files in no store read
 * are dropped. M becomes the engine's master row (placement candidates,
 * gh_put/gh_repair). *f0 = MemberList_M[0] (the member that receives
 * Assign_new_master, :1000 / server/server.go:236), may be NULL;
 * *n_files = files left in the table, may be NULL. GH_EINVAL if M's list is
 * empty. */
int gh_rebuild_meta(void* h, int32_t new_master, int32_t* f0, int64_t* n_files);
/* A master's file metadata (its SDFSMaster maps, master/master.go:38-44) as
 * flat arrays over files 0..max_files-1: replica lists [F][R] (-1 = none),
 * versions [F] (-1 = no such file), put timestamps [F], placement draw
 * counters [F]. gh_export_files copies the engine's table out (every rank gets
 * the whole table); gh_import_files replaces it (every rank takes its own
 * files). A master demoted by an election while its process kept running
 * (slave/slave.go:1122-1175: members whose self.master still names it send
 * their Update_metadata calls there) answers from its own maps: a host keeps
 * them beside the engine's and swaps them in, with gh_set_master, to run
 * those calls (gossipsim.Cluster). */
int gh_export_files(void* h, int32_t* replicas, int32_t* versions, int32_t* timestamps, uint32_t* draws);
int gh_import_files(void* h, const int32_t* replicas, const int32_t* versions, const int32_t* timestamps,
                    const uint32_t* draws);
/* The member whose list is the master's Member_list (placement candidates of
 * gh_put / gh_repair, master/master.go:46); gh_create takes gh_config.master,
 * gh_rebuild_meta sets the new master. */
int gh_set_master(void* h, int32_t master);

/* ---- multi-GPU: one cluster column-sharded over G ranks ----------------
 * Rank g holds all N observer rows for member columns [g*ncs, g*ncs+ncol)
 * (ncs = roundup(ceil(N/G), 32)): 4*N*ncs bytes of narrow table plus arenas.
 * Merge, detection, cleanup and REMOVE delivery of a member happen on its
 * column's rank; per round the ranks exchange only O(N) vectors (present
 * counts, pull inboxes or ring positions/targets) by RCCL over xGMI. This
 * replaces the reference's per-host processes exchanging UDP lists
 * (slave/slave.go:499-544) for a simulated cluster spread over GPUs.
 * SPMD contract: every rank calls every gh_* function of a sharded handle
 * with the same arguments in the same order (most calls are collective);
 * every rank returns the same (global) results. */
#define GH_COMM_RCCL 0    /* one process per GPU, RCCL over xGMI              */
#define GH_COMM_LOCAL 1   /* ranks are threads of one process (any devices)  */
#define GH_COMM_ID_BYTES 128
/* Shard layouts (DESIGN.md "Multi-GPU"):
 *   GH_LAYOUT_COLUMNS  rank g holds member columns [g*ncs, g*ncs + ncs) of
 *                      ALL rows; every per-round exchange is O(N) (default)
 *   GH_LAYOUT_ROWS     rank g holds observer rows [g*nrs, g*nrs + nrs) with
 *                      ALL columns (north_star): each round the senders'
 *                      rows that a shard's receivers pull cross shards by
 *                      one alltoallv (ncclAllToAllv), O(N^2 k/G) bytes.
 *                      Pull mode only (ring mode: GH_EINVAL). */
#define GH_LAYOUT_COLUMNS 0
#define GH_LAYOUT_ROWS 1

/* RCCL unique id for gh_create_sharded (call on rank 0, send to all). */
int gh_comm_unique_id(uint8_t* id);
/* comm_id: GH_COMM_RCCL -> the unique id; GH_COMM_LOCAL -> a NUL-terminated
 * group key shared by the ranks (<= GH_COMM_ID_BYTES). world == 1 needs no
 * transport (comm_id may be NULL). cfg->device selects the rank's GPU. */
int gh_create_sharded(const gh_config* cfg, int32_t rank, int32_t world, int32_t transport,
                      const uint8_t* comm_id, void** handle);
int gh_shard_info(void* h, int32_t* rank, int32_t* world, int64_t* col0, int64_t* ncols);

/* Table encoding of this engine's shard (diagnostic; DESIGN.md "Data layout"):
 * (tile, row) segments of the current table held wide (arena or frozen
 * store, stopped rows included); segments the last round ran through the per-cell
 * rule (k_round_slow); the round kernel variant of the last round (0 lean,
 * 1 storm) and its storm measure; the row segments the last round skipped as
 * quiet (inactive rows that stopped changing). Any output may be NULL. No
 * reference counterpart. */
int gh_encoding_info(void* h, int64_t* wide_segments, int64_t* slow_segments, int32_t* storm_mode,
                     int64_t* storm_segments, int64_t* quiet_segments);
/* Sender snapshot plane (diagnostic; DESIGN.md "Sender plane"): whether the
 * engine keeps one (pull mode, 3 <= k <= 4, N >= 16,384), whether the current table's plane is
 * valid for the next round, and how many waves of the last round gathered
 * 16-bit sender codes although the plane was valid (a sender code outside
 * the plane's window). Any output may be NULL. No reference counterpart. */
int gh_plane_info(void* h, int32_t* enabled, int32_t* valid, int64_t* fallback_waves);
/* 4-bit tier (diagnostic; DESIGN.md "4-bit tier"): whether the engine keeps
 * one (plane mode, column layout; GH_C8=0 drops it), whether the current
 * table is held in it (lag and age nibbles, escaped chunks in 16 bits), how
 * many chunks the last round's packed 16-bit path wrote escaped, and the
 * round kernel variant of the last round (0 lean on a 16-bit input, 1 storm,
 * 2 lean on a tier input widened to 16 bits, 3 the nibble path). Any output
 * may be NULL. No reference counterpart. */
int gh_tier_info(void* h, int32_t* enabled, int32_t* current_8bit, int64_t* escaped_chunks, int32_t* last_variant);
/* Lane jobs of the nibble path (diagnostic; DESIGN.md "Lane jobs"): in the
 * last round, the lanes (16 cells of a row) whose cells left the 4-bit tier
 * or needed the per-cell rule -- crashed members' aging, flagged and
 * tombstoned cells, REMOVE -- and were done by k_round_jobs instead of
 * sending their whole 256-cell segments to the slow list, and how many of
 * them needed a wide segment (k_round_redo). Any output may be NULL. No
 * reference counterpart. (ABI 6) */
int gh_job_info(void* h, int64_t* lane_jobs, int64_t* redo_lanes);
/* Row layout (GH_LAYOUT_ROWS): the last ghost-row exchange of this shard --
 * the sender rows it received, and the bytes it sent and received by
 * alltoallv (narrow codes, plane words, wide segments). Zero in the column
 * layout, whose exchanges are O(N) collectives. Any output may be NULL. No
 * reference counterpart (it replaces the UDP list pushes, slave/slave.go:527-542). */
int gh_exchange_info(void* h, int64_t* ghost_rows, int64_t* bytes_out, int64_t* bytes_in);
/* HBM held by the tables (narrow x2 + wide arenas + frozen store), wide-arena
 * slots in use / per buffer, and stopped rows in the frozen store. Any
 * output may be NULL. Diagnostic; no reference counterpart. */
int gh_memory_info(void* h, int64_t* device_bytes, int64_t* wide_used, int64_t* wide_cap, int64_t* frozen_rows);
/* The file table of this engine / shard (placement is per file,
 * master/master.go:74-150): sharded by file ID, file f on shard f % G at slot
 * f / G, so *slots = ceil(max_files / G) files' replica lists, versions and
 * timestamps; *shards = G (1 for one engine); *held = the files put and not
 * deleted in this shard's slots. Any output may be NULL. Diagnostic. */
int gh_file_info(void* h, int64_t* slots, int32_t* shards, int64_t* held);
/* The HBM one shard (rank of world, layout and sizes from cfg) would hold,
 * without a device or a communicator (a dry walk of gh_create's
 * allocations): *create_bytes = everything gh_create allocates;
 * *exchange_bytes = the row layout's ghost-row exchange buffers at a
 * healthy pull round's expected distinct remote senders (0 in the column
 * layout). The frozen store (grows with stopped rows) and per-call staging
 * are not included. Plans config 4 (N = 262,144 over 8 GPUs) before any
 * allocation. Any output may be NULL. No reference counterpart. */
int gh_footprint(const gh_config* cfg, int32_t rank, int32_t world, int32_t transport, int64_t* create_bytes,
                 int64_t* exchange_bytes);

/* Tuning knobs of the round kernel (k_round): non-temporal stores of the new
 * table and the XCD-aware block->tile map. Results do not depend on them;
 * the defaults (both on) are the measured fastest. */
int gh_set_round_variant(void* h, int32_t nontemporal, int32_t xcd_map);

/* Device timing of the fused round kernel (HIP events on the engine's
 * stream), for bench.py's roofline: enable, then read the sum of kernel
 * durations (ms) and launch count since enabling. */
int gh_set_timing(void* h, int32_t enable);
int gh_read_timing(void* h, double* total_ms, int64_t* launches);
/* Block until all queued device work has finished. */
int gh_sync(void* h);

#ifdef __cplusplus
}
#endif

#endif /* GOSSIPHIP_H_ */
