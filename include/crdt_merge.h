/* crdt_merge.h — C-ABI of the MI355X-native MapCrdt merge hot path.
 *
 * The reference (Dart package `crdt` v4.0.2, /root/reference) has no FFI: its
 * boundary is the abstract class Crdt<K,V> (lib/src/crdt.dart:7) and its
 * storage SPI (lib/src/crdt.dart:140-169), implemented by MapCrdt
 * (lib/src/map_crdt.dart:9-53).  This header is the C surface a dart:ffi shim
 * subclassing Crdt would bind (INTEGRATION.md shows that binding); every entry
 * point names the reference member it replaces.
 *
 * Data model.  The host (Dart, or the Python mirror in crdt_amd/) owns keys,
 * values and node-id strings and interns them:
 *   key_id  : dense uint32 id, assigned in first-committed order, so id order is
 *             the LinkedHashMap insertion order (map_crdt.dart:10);
 *   lt      : int64 Hlc.logicalTime = (millis << 16) + counter (hlc.dart:16);
 *   rank    : uint32 order-preserving rank of the nodeId under Dart
 *             String.compareTo (hlc.dart:160), so nodeId equality == rank equality;
 *   val     : uint32 value handle; CRDT_NULL_VALUE marks a tombstone
 *             (record.dart:17, isDeleted <=> value == null).
 * The device keeps one row per key id: {i64 lt; u32 rank; i32 mod_hi; u32 mod_lo; u32 val},
 * 24 B apart by default (32 B with crdt_set_row_bytes: 8 zero bytes of padding), where
 * mod is Record.modified.logicalTime.  A row whose mod < 0 is invisible to
 * merge and to recordMap() (map_crdt.dart:42-45); never-written rows hold a
 * negative mod.
 *
 * Domain: |millis| < 2^47 for every clock and wall value (Dart int wraps past it).
 * Threading: a ctx is one replica shard (one GPU); calls on one ctx are synchronous and
 * must not run concurrently, exactly like the single-isolate reference.  A ctx joined
 * to a communicator (crdt_comm_init_*) is one of n_ranks key shards of ONE replica: its
 * crdt_merge calls are collective (every rank calls with the same n_changesets and
 * wall_millis) and the library runs the exchanges itself (SURVEY §8(b) "Threading").
 */
#ifndef CRDT_MERGE_H
#define CRDT_MERGE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CRDT_ABI_VERSION 5          /* 3: crdt_timing gained part1_records (round 3); 4: crdt_route_tune_info
                                       reports five ways, crdt_timing gained sent_bytes (round 5); 5: the
                                       collective deadline, crdt_set_comm_timeout / crdt_comm_state (round 6) */
#define CRDT_NULL_VALUE 0xFFFFFFFFu

/* Status codes.  1..3 mirror the reference exceptions (hlc.dart:164-189); the
 * host rethrows them with the exact messages of hlc.dart:170,179,188. */
enum crdt_status {
    CRDT_OK = 0,
    CRDT_CLOCK_DRIFT = 1,      /* ClockDriftException(drift_ms)         hlc.dart:164-171 */
    CRDT_DUPLICATE_NODE = 2,   /* DuplicateNodeException(local nodeId)  hlc.dart:182-189 */
    CRDT_OVERFLOW = 3,         /* OverflowException(counter)            hlc.dart:173-180 */
    CRDT_E_INVALID = -1,       /* bad argument (offsets, sizes, null pointers) */
    CRDT_E_HIP = -2,           /* HIP runtime error */
    CRDT_E_NOMEM = -3,         /* device allocation failed */
    CRDT_E_KEY_RANGE = -4,     /* a key_id >= capacity.  crdt_merge on one context: nothing stored and
                                  the canonical unchanged for device batches and on the sorted path;
                                  a host batch on the gather path (its keys stream in under the
                                  apply) may have stored the changesets before the bad id's launch;
                                  on a sharded context the other ranks' rows are stored */
    CRDT_E_NO_DEVICE = -5,     /* no usable gfx950 device */
    CRDT_E_COMM = -6           /* the communicator failed (RCCL error, missing librccl, a callback's error) */
};

/* Where the column pointers of a call live. */
enum crdt_mem { CRDT_MEM_HOST = 0, CRDT_MEM_DEVICE = 1 };

typedef struct crdt_ctx crdt_ctx;

/* R remote changesets, concatenated column-wise.  Changeset j is rows
 * [offsets[j], offsets[j+1]); it is one Map<K, Record<V>> handed to merge()
 * (crdt.dart:77), in its iteration order, so its key ids must be distinct. */
typedef struct crdt_batch {
    const uint32_t* key_id;    /* [n] */
    const int64_t* lt;         /* [n] */
    const uint32_t* rank;      /* [n] */
    const uint32_t* val;       /* [n] */
    const int64_t* millis;     /* optional [n]: Hlc.millis where it differs from lt >> 16 (a parsed
                                  counter > 0xFFFF, hlc.dart:43); NULL means millis = lt >> 16 */
    const uint64_t* offsets;   /* HOST memory, [n_changesets + 1], offsets[0] == 0 */
    uint32_t n_changesets;
    int32_t mem;               /* enum crdt_mem of the five column pointers (and win_flags) */
} crdt_batch;

/* Outcome of a merge / put call. */
typedef struct crdt_result {
    int32_t status;            /* enum crdt_status */
    uint32_t n_stored;         /* changesets whose winners were stored (putRecords ran) */
    uint32_t exc_changeset;    /* changeset that raised, when status in 1..3 */
    uint32_t reserved;
    uint64_t exc_index;        /* record (in that changeset) whose recv() raised; UINT64_MAX when
                                  send() raised after storing (crdt.dart:93) */
    int64_t canonical_lt;      /* Crdt._canonicalTime.logicalTime after the call (crdt.dart:9) */
    int64_t drift_ms;          /* ClockDriftException.drift (hlc.dart:167) */
    int64_t counter;           /* OverflowException.counter (hlc.dart:176) */
    uint64_t n_present;        /* records whose key was present in the local snapshot */
    uint64_t n_won;            /* records stored (winners) */
} crdt_result;

/* Device-side kernel timing of the last call, measured with HIP events on the
 * ctx stream (bench / roofline support; zeros unless enabled). */
typedef struct crdt_timing {
    double scan_ms;            /* K3a: per-changeset max + candidate tiles */
    double clock_ms;           /* K3b/K3c: canonical prefix-max scan, exception resolution (+ the
                                  clock collectives on a sharded ctx) */
    double apply_ms;           /* K2: summed durations of SAMPLED windows of back-to-back apply launches
                                  (8 launches every 32; the sorted path: its whole apply region) */
    uint32_t apply_launches;   /* apply launches inside the sampled windows */
    uint32_t apply_total;      /* apply launches in the call */
    double total_ms;           /* first to last event of the call */
    double route_ms;           /* sharded ctx: route count, count exchange, scatter, record exchange */
    /* sorted path (first window of changesets): the level-1 partition scatter, the level-2 partition
       (its histogram and scatter), the resolve (fold, carry and resolve launches); 0 otherwise */
    double part1_ms;
    double part2_ms;
    double resolve_ms;
    uint64_t part1_records;    /* records the level-1 partition scatter read in that window */
    uint64_t sent_bytes;       /* sharded ctx: bytes this rank handed its peers in the call's all-to-all
                                  exchanges (records, counts; its own part excluded); 0 on one GPU.
                                  Filled whether or not timing is on. */
} crdt_timing;

/* ---- lifecycle ------------------------------------------------------------ */
int crdt_abi_version(void);
const char* crdt_status_string(int status);
int crdt_device_count(int* out);

/* MapCrdt(nodeId) (map_crdt.dart:16) + Crdt() -> refreshCanonicalTime() on the
 * empty map (crdt.dart:31-33): canonical lt = 0.  local_rank is the rank of the
 * local nodeId.  capacity rows are allocated and marked absent. */
int crdt_create(int device, uint32_t local_rank, uint64_t capacity, crdt_ctx** out);
void crdt_destroy(crdt_ctx* ctx);
int crdt_reserve(crdt_ctx* ctx, uint64_t capacity);          /* grow; new rows absent */
/* Pre-size the sorted path's partition scratch for merges of up to n_records applied records
 * (two partitioned copies in the packed form, 27 B per record; a wider form grows them in its first
 * merge), so the first large merge allocates nothing and the buffers are placed while device memory is
 * still unfragmented.  On a single-GPU ctx it also asks for the placement tuner's trials
 * (crdt_place_info): the next sorted merge takes the candidate level-1 buffers, sized for its form
 * (14 B per record at the fan-in) and together at most 1/8 of the device's HBM; they are freed once
 * timed, or after two merges that do not take the sorted path.  Optional. */
int crdt_reserve_scratch(crdt_ctx* ctx, uint64_t n_records);
/* Row size of the device table: 24 (default) or 32 bytes; the rows are copied over.  24-B rows move
 * 25 % fewer bytes in the sorted path's coalesced passes (many-changeset fan-ins); 32-B rows make
 * the gather path's random winner writes one aligned 32-B store (streaming calls where most
 * records win).  Results are identical. */
int crdt_set_row_bytes(crdt_ctx* ctx, uint32_t row_bytes);
int crdt_capacity(const crdt_ctx* ctx, uint64_t* out);
int crdt_set_local_rank(crdt_ctx* ctx, uint32_t rank);        /* after a rank remap */

/* Crdt._canonicalTime (crdt.dart:9-11). */
int crdt_get_canonical(const crdt_ctx* ctx, int64_t* lt);
int crdt_set_canonical(crdt_ctx* ctx, int64_t lt);

/* ---- storage SPI (crdt.dart:140-169) --------------------------------------- */
/* putRecord / putRecords (map_crdt.dart:27-39) and the seed addAll
 * (map_crdt.dart:17): store rows verbatim, no clock update. */
int crdt_put_rows(crdt_ctx* ctx, const uint32_t* key_id, const int64_t* lt, const uint32_t* rank,
                  const uint32_t* val, const int64_t* mod, uint64_t n, int32_t mem);
/* getRecord (map_crdt.dart:24): gather rows; any output pointer may be NULL. */
int crdt_read_rows(crdt_ctx* ctx, const uint32_t* key_id, uint64_t n, int64_t* lt, uint32_t* rank,
                   uint32_t* val, int64_t* mod, int32_t mem);
/* recordMap(modifiedSince) filter (map_crdt.dart:42-45): ids in [0, n_rows) with
 * mod >= since_lt, ascending (= insertion order).  out_ids (HOST) holds n_rows. */
int crdt_modified_since(crdt_ctx* ctx, uint64_t n_rows, int64_t since_lt, uint32_t* out_ids,
                        uint64_t* n_out);
/* purge() (map_crdt.dart:51-52) and rollback of interned-but-uncommitted ids. */
int crdt_clear_rows(crdt_ctx* ctx, uint64_t first, uint64_t count);
/* Re-rank stored node ids after the host inserts a new nodeId between existing
 * ranks: rank := old_to_new[rank] for rows [0, n_rows). */
int crdt_remap_ranks(crdt_ctx* ctx, uint64_t n_rows, const uint32_t* old_to_new, uint32_t n_ranks);

/* ---- Crdt API ------------------------------------------------------------ */
/* put / putAll / delete (crdt.dart:39-58): ONE Hlc.send (hlc.dart:51-74) for the
 * whole call, then rows {C, local_rank, val, C}; n == 0 is a no-op (crdt.dart:48). */
int crdt_put_stamped(crdt_ctx* ctx, const uint32_t* key_id, const uint32_t* val, uint64_t n,
                     int64_t wall_millis, int32_t mem, crdt_result* out);

/* refreshCanonicalTime (crdt.dart:114-121) over rows [0, n_rows). */
int crdt_refresh_canonical(crdt_ctx* ctx, uint64_t n_rows, int64_t* out_lt);

/* R sequential Crdt.merge(changeset_j) calls (crdt.dart:77-94), wall clock
 * fixed at wall_millis for every clock read (hlc.dart:53,82).  Stops at the
 * first exception exactly as the reference: a recv() failure in changeset j
 * stores nothing of j and leaves canonical = the running max before the failing
 * record; a send() failure after j leaves j stored and canonical = R_j.
 * win_flags (optional, [n], same memory kind as the batch): 1 where the record
 * was stored — the Map the reference's removeWhere leaves behind (crdt.dart:80-85)
 * and the watch() events (map_crdt.dart:36-38). */
int crdt_merge(crdt_ctx* ctx, const crdt_batch* batch, int64_t wall_millis, uint8_t* win_flags,
               crdt_result* out);

/* ---- key-sharded multi-GPU (north star config 4) -------------
 * n_ranks ctxs — one per GPU, normally one process per GPU — form ONE replica whose
 * keys are sharded: rank d owns key k iff k % n_ranks == d and stores it at slot
 * k / n_ranks (so each ctx's capacity counts slots).  crdt_merge on such a ctx is
 * collective: every rank passes the same n_changesets and wall_millis and its own
 * PART of each changeset; changeset j is the concatenation, in rank order, of the
 * ranks' parts (a Map's iteration order is whatever its sender produced, so this is a
 * legal order; a replica that arrives whole on one rank is the case where the other
 * parts are empty).  Inside the call the library:
 *   1. scans its parts (per-part max, tiles that may raise);
 *   2. all-gathers the R part maxima and counts -> M_j, and each part's preceding
 *      max / record offset inside changeset j;
 *   3. runs the canonical recurrence and exception scan, MIN all-reduce of the first
 *      event, MAX all-reduce of its details -> the same stop point everywhere;
 *   4. counts its records per (owner, changeset), exchanges the counts, scatters the
 *      records into owner-major send columns {slot, lt, rank, val} and moves them with
 *      ONE grouped all-to-all (every column of every peer in one group);
 *   5. applies the records it received (gather or sorted path) with mod = R_j;
 *   6. SUM all-reduce of the per-record counts and of the key-range error.
 * Every rank returns the same status, stop point, canonical and counts; win_flags
 * (optional, [n] of the local batch) come back to the rank that passed the record.
 * A failure local to one rank (CRDT_E_NOMEM, CRDT_E_INVALID of its own batch, CRDT_E_HIP
 * of a launch or copy) is carried through the call's collectives and returned by EVERY
 * rank — no rank is left waiting in a collective its peers will not post.  Before the
 * record exchange nothing is stored and the canonical clock does not move; a failure in the
 * owners' apply (after the exchange) leaves the other ranks' rows of the stopped call stored
 * and the canonical unchanged (re-merging the same batch is exact).  Rank-local still: a
 * failing transport, a rank that cannot allocate the call's O(R) gather words, and a HIP
 * failure of a read-back of agreed words (without them the rank cannot post what its peers
 * post next).  Those — and a peer that died, hung or faulted — end at the call's DEADLINE:
 * every host wait of a sharded call polls against it (crdt_set_comm_timeout); past it the
 * communicator is aborted (ncclCommAbort for RCCL) and the call returns CRDT_E_COMM.  After
 * CRDT_E_COMM the ctx refuses sharded merges (CRDT_E_COMM) until it joins a communicator
 * again (crdt_comm_free + crdt_comm_init_*), and the rows of its shard the failed call may
 * have touched are undefined (re-sync the shard).
 * Keys in the batch are GLOBAL key ids, unless crdt_set_presharded(ctx, 1): then every
 * record is already on its owner and key_id holds its slot (no record exchange).
 *
 * Backends: RCCL over xGMI (crdt_comm_unique_id on one rank, the host broadcasts the
 * 128 bytes, crdt_comm_init_rccl on every rank; librccl is opened on first use), or a
 * caller's crdt_comm_ops table (a host transport: MPI, TCP, gloo).  No reference
 * counterpart: the reference is single-process (example/crdt_example.dart:21-25). */
enum crdt_reduce_op { CRDT_REDUCE_SUM = 0, CRDT_REDUCE_MAX = 1, CRDT_REDUCE_MIN = 2 };

typedef struct crdt_comm_ops {
    void* user;                /* passed back to every callback */
    int32_t mem;               /* CRDT_MEM_DEVICE: pointers are device memory and an operation is
                                  ordered on `stream` (a hipStream_t) like RCCL's;
                                  CRDT_MEM_HOST: the library synchronises, stages the words through
                                  host memory and the call completes before it returns */
    int32_t reserved;
    /* in-place all-reduce of n signed 64-bit words */
    int (*all_reduce_i64)(void* user, int64_t* words, uint64_t n, int32_t op, void* stream);
    /* recv[r * n + i] = send[i] of rank r */
    int (*all_gather_i64)(void* user, const int64_t* send, int64_t* recv, uint64_t n, void* stream);
    /* one grouped exchange of n_cols columns (column c has elem_bytes[c]-byte elements): to each
       peer d this rank sends elements [send_displs[d], + send_counts[d]) of every column and
       receives [recv_displs[d], + recv_counts[d]) from it; the entries for this rank are 0 (the
       library moves its own chunk itself) */
    int (*all_to_all_v)(void* user, uint32_t n_cols, const void* const* send_cols, void* const* recv_cols,
                        const uint32_t* elem_bytes, const uint64_t* send_counts, const uint64_t* send_displs,
                        const uint64_t* recv_counts, const uint64_t* recv_displs, void* stream);
} crdt_comm_ops;

#define CRDT_COMM_ID_BYTES 128
int crdt_comm_unique_id(uint8_t* id /* [CRDT_COMM_ID_BYTES] */);
int crdt_comm_init_rccl(crdt_ctx* ctx, uint32_t n_ranks, uint32_t rank, const uint8_t* id);
int crdt_comm_init_ops(crdt_ctx* ctx, uint32_t n_ranks, uint32_t rank, const crdt_comm_ops* ops);
int crdt_comm_info(const crdt_ctx* ctx, uint32_t* n_ranks, uint32_t* rank);
int crdt_comm_free(crdt_ctx* ctx);
/* The deadline of one collective crdt_merge, in ms from the call's entry (default 300000, or the
 * CRDT_COMM_TIMEOUT_MS environment variable at crdt_create; 0 = wait forever).  With RCCL every
 * host wait of the call polls the device against it and against ncclCommGetAsyncError; past it
 * the communicator is aborted and the call returns CRDT_E_COMM.  A CRDT_MEM_HOST transport blocks
 * inside its callbacks and must bound each operation itself (e.g. its own timeout); a callback
 * that fails, or returns after the deadline, fails the call the same way. */
int crdt_set_comm_timeout(crdt_ctx* ctx, uint32_t ms);
/* *state: 0 = the communicator is usable, 1 = aborted at a deadline, 2 = aborted on a transport
 * error; *phase: where the current or last collective merge is or was (static text, e.g.
 * "route_l1: record exchange").  Safe to call from another thread while crdt_merge runs (a
 * watchdog's report); the pointer stays valid for the process's life. */
int crdt_comm_state(const crdt_ctx* ctx, int32_t* state, const char** phase);
/* presharded = 1: batches hold only records this rank owns, key_id = slot (no exchange) */
int crdt_set_presharded(crdt_ctx* ctx, int presharded);

/* ---- merge strategy --------------------------------------------------------
 * crdt_merge resolves a batch either by the gather path (one launch per changeset,
 * every record reads its row: K2) or by the sorted path (the applied records are
 * partitioned by key into 4096-key buckets, each bucket's rows are read and written
 * once and its records resolved in LDS; sorted_path.inc).  Both give identical
 * rows, canonical, status and counts.  The sorted path needs: canonical >= 0,
 * capacity <= 2^28; with win_flags, also a batch frame that fits its 64-bit packed key (its
 * flagged form; on a sharded ctx the receivers take it on the all-gathered global frame, with
 * the records crossing the exchange unpacked), else the gather path runs.  path: CRDT_PATH_AUTO (default, also set by the
 * CRDT_MERGE_PATH environment variable = gather | sorted), CRDT_PATH_GATHER,
 * CRDT_PATH_SORTED (whenever allowed).  crdt_last_path reports the path the last
 * crdt_merge took (CRDT_PATH_GATHER or CRDT_PATH_SORTED). */
enum crdt_path { CRDT_PATH_AUTO = 0, CRDT_PATH_GATHER = 1, CRDT_PATH_SORTED = 2 };
int crdt_set_merge_path(crdt_ctx* ctx, int path);

/* Per-record counts (crdt_result.n_present / n_won): library extras, not part of the
 * reference's merge (crdt.dart:77-94 exposes none).  exact = 1 (default): both paths count
 * them.  exact = 0: when the sorted path runs it folds each bucket's records in any order
 * (ties on (lt, rank) decided by changeset, the local row first — the same rows, canonical and
 * status) and reports both counts as UINT64_MAX; the gather path still counts. */
int crdt_set_counts(crdt_ctx* ctx, int exact);
/* A promise that every node-id rank in later batches is < bound (the host interns node ids
 * densely; 0 = no promise, the default).  The sorted path then takes the rank part of its packed
 * key's frame from the bound instead of reading every rank in the scan.  A batch that breaks the
 * promise is never merged wrongly: where the bound is used (a single ctx's packed sorted form) the
 * call returns CRDT_E_INVALID having stored nothing and left the canonical clock as it was (the
 * check runs before any row is written); elsewhere the bound is ignored and the merge is exact. */
int crdt_set_rank_bound(crdt_ctx* ctx, uint32_t bound);
int crdt_last_path(const crdt_ctx* ctx, int* path);
/* How the last crdt_merge ran (diagnostics for tests and profiles): bit flags. */
enum crdt_plan_flags {
    CRDT_PLAN_SORTED = 1,        /* the sorted path ran */
    CRDT_PLAN_PACKED = 2,        /* ... in its packed order-free form (64-bit keys, sorted_path.inc) */
    CRDT_PLAN_TWO_LEVEL = 4,     /* ... with two partition levels (capacity > 2^20) */
    CRDT_PLAN_HIST_IN_SCAN = 8,  /* ... with its level-1 histogram counted by the scan */
    CRDT_PLAN_KEY8 = 16,         /* ... with 13-B final records (1-B key column, 4 key bits in the packed key) */
    CRDT_PLAN_KEY16 = 32,        /* ... and 14-B level-1 records (2-B key column) */
    CRDT_PLAN_HIGH_WATER = 64,   /* ... and its resolve did not read the rows at or above the table's
                                    high-water mark of written rows (never-written fill) */
    CRDT_PLAN_ANCHORED = 128,    /* retired in round 5 (the anchored sorted form, measured 0.25 ms slower
                                    per fan-in step, was removed): never set */
    CRDT_PLAN_WIRE_PACKED = 256, /* sharded ctx: records crossed the all-to-all as 16-B packed
                                    {slot, (lt, rank, changeset) key, val} instead of 20 B */
    CRDT_PLAN_OWN_IN_PLACE = 512, /* sharded ctx: the records this rank owns of its own batch were
                                    scattered straight into the receive columns (no device copy) */
    CRDT_PLAN_FLAGGED = 1024,    /* the sorted path's flagged form: per-record win flags (changeset-ordered
                                    level 2, ordered resolve, flags carried back to input order; sorted_path.inc) */
    CRDT_PLAN_ORDERED = 2048,    /* ... its ordered packed resolve (flags and / or exact n_present / n_won) */
    CRDT_PLAN_COMBINED = 4096,   /* sharded ctx: home records folded to one packed maximum per key before
                                    the all-to-all (the order-free form's map-side combine) */
    CRDT_PLAN_ROUTE_L1 = 8192,   /* sharded ctx: home records partitioned once, straight into their owners'
                                    level-1 buckets; 14-B level-1 records crossed the exchange and the
                                    owners started at level 2 (comm_path.inc, route_l1) */
    CRDT_PLAN_ROUTE_TUNED = 16384, /* sharded ctx: the way (route_l1 or the combine) came from the routing
                                    tuner, a trial or its measured choice (crdt_route_tune_info) */
    CRDT_PLAN_RL1_PIECES_SHIFT = 15, /* bits 15-17: route_l1's pipelined pieces (1-4; 0: not route_l1) */
    CRDT_PLAN_RL1_HEAD = 262144, /* route_l1 folded each owner's first level-1 digit (its 2^20 lowest slots,
                                    the Zipf head) at the sender: one packed maximum per key crossed the
                                    exchange for those keys (comm_path.inc) */
    CRDT_PLAN_COMPACT = 524288   /* the sorted path's compact form: the records' lt field packed as
                                    (lt >> 16 - min, lt & 0xFFFF) in as many bits as the batch needs, so a record's
                                    whole 20-bit level-1 slot rides in its 64-bit key: 12-B partition records
                                    (sorted_path.inc, PackFrame::cb) */
};
int crdt_last_plan(const crdt_ctx* ctx, uint32_t* flags);

/* Sharded ctx: the measured routing of order-free many-changeset fan-ins (comm_path.inc, RouteTune;
 * CRDT_ROUTE_TUNE=0 turns it off).  While every way is open (the auto settings), the first calls take each
 * way twice, the second call of each timed on the host and MAX-reduced over the ranks; later calls with the
 * same (changesets, ranks, capacity) take the fastest.  *best: -1 while the trials run (or before any such
 * call), 0 = route_l1 in 2 pipelined pieces, 1 = the map-side combine, 2 = route_l1 in 4 pieces,
 * 3 = route_l1 in one, 4 = route_l1 in 2 pieces with the head fold (CRDT_PLAN_RL1_HEAD); us[0 .. 4]: their
 * timed calls in microseconds (-1: not yet).  Every way leaves the same rows. */
int crdt_route_tune_info(const crdt_ctx* ctx, int32_t* best, int64_t* us /* [5] */);

/* The level-1 scatter's placement tuner (crdt_merge.hip, PlaceTune; CRDT_PLACE_TRIES, default 3, 1 = off):
 * crdt_reserve_scratch on a single-GPU ctx asks for that many candidate level-1 partition buffers (the
 * warm-up merge takes those that fit in 1/8 of HBM); the next sorted-path merges time the level-1 scatter
 * on each in turn, two
 * rounds, and keep the fastest (the scatter's time follows where its destination lies in physical memory;
 * DESIGN.md §6).  *n: candidates (0 / 1: no trials); *kept: the kept one (-1 while the trials run); *done:
 * merges the tuner has used (the warm-up, then two per candidate); ms[0 .. 3]: each candidate's level-1
 * scatter (the faster of its two trials). */
int crdt_place_info(const crdt_ctx* ctx, int32_t* n, int32_t* kept, int32_t* done, float* ms /* [4] */);

/* ---- measurement ---------------------------------------------------------- */
int crdt_set_timing(crdt_ctx* ctx, int enable);
int crdt_get_timing(const crdt_ctx* ctx, crdt_timing* out);

#ifdef __cplusplus
}
#endif
#endif /* CRDT_MERGE_H */
