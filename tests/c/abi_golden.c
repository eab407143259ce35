/* abi_golden.c — the C-ABI (include/crdt_merge.h) driven from a plain C host, the way a
 * dart:ffi caller drives it: no Python, no torch, host-memory columns.
 *
 * Reads tests/golden/abi_cases.bin (golden cases of the object-level oracle, pinned by the
 * reference's known-answer tests; tests/golden/export_abi_cases.py) and, per case, runs
 *   1. crdt_merge with win flags (the gather path),
 *   2. crdt_merge without flags on the sorted path (CRDT_PATH_SORTED, order-free form),
 *   3. crdt_merge on a 1-rank sharded ctx joined to an in-process loopback crdt_comm_ops table
 *      (CRDT_MEM_HOST) — the library's collective path with its exchanges done by this file,
 *   4. the sorted path again on 32-B rows (crdt_set_row_bytes) with the batch's rank bound declared
 *      (crdt_set_rank_bound: max rank + 1),
 *   5. a 1-rank pre-sharded ctx (crdt_set_presharded) over the loopback table — what
 *      GpuMapCrdt.sharded (dart/lib/src/gpu_map_crdt.dart) sets up,
 *   6. the same over a 1-rank RCCL communicator (crdt_comm_unique_id + crdt_comm_init_rccl),
 * and compares status, stop point, exception fields, canonical, win flags and every row with
 * the expected values, bit for bit.  It also decodes a CrdtJson document with libcrdt_host.so's
 * crdt_json_decode (what GpuMapCrdt.mergeJson calls) and checks its columns.  Exit status 0 = all equal.
 *
 *   gcc -O2 -std=c11 -I include tests/c/abi_golden.c -o tests/c/abi_golden \
 *       -L crdt_amd -l:libcrdt_mi355x.so -l:libcrdt_host.so -Wl,-rpath,'$ORIGIN/../../crdt_amd'
 *   tests/c/abi_golden tests/golden/abi_cases.bin
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "crdt_host.h"
#include "crdt_merge.h"

typedef struct {
    char name[33];
    uint32_t n_ids, n_local, local_rank, R;
    uint64_t n;
    int64_t c0, wall;
    uint32_t has_millis;
    int64_t *l_lt, *l_mod, *lt, *millis, *e_lt, *e_mod;
    uint32_t *l_rank, *l_val, *key, *rank, *val, *e_rank, *e_val;
    uint64_t* offsets;
    uint8_t *e_exists, *e_flags;
    int32_t status;
    uint32_t n_stored, exc_changeset;
    uint64_t exc_index, n_present, n_won;
    int64_t canonical, drift, counter;
} Case;

static const uint8_t* g_p;
static const uint8_t* g_end;

static void* take(size_t bytes) {
    if (g_p + bytes > g_end) { fprintf(stderr, "abi_cases.bin truncated\n"); exit(2); }
    void* out = malloc(bytes ? bytes : 1);
    memcpy(out, g_p, bytes);
    g_p += bytes;
    return out;
}

#define TAKE(dst, type, count) dst = (type*)take(sizeof(type) * (size_t)(count))
#define SCALAR(dst) memcpy(&(dst), g_p, sizeof(dst)), g_p += sizeof(dst)

static void read_case(Case* c) {
    memset(c, 0, sizeof(*c));
    memcpy(c->name, g_p, 32);
    g_p += 32;
    uint32_t pad;
    SCALAR(c->n_ids); SCALAR(c->n_local); SCALAR(c->local_rank); SCALAR(c->R);
    SCALAR(c->n); SCALAR(c->c0); SCALAR(c->wall); SCALAR(c->has_millis); SCALAR(pad);
    TAKE(c->l_lt, int64_t, c->n_local); TAKE(c->l_rank, uint32_t, c->n_local);
    TAKE(c->l_val, uint32_t, c->n_local); TAKE(c->l_mod, int64_t, c->n_local);
    TAKE(c->key, uint32_t, c->n); TAKE(c->lt, int64_t, c->n); TAKE(c->rank, uint32_t, c->n);
    TAKE(c->val, uint32_t, c->n); TAKE(c->offsets, uint64_t, c->R + 1);
    if (c->has_millis) TAKE(c->millis, int64_t, c->n);
    SCALAR(c->status); SCALAR(c->n_stored); SCALAR(c->exc_changeset); SCALAR(pad);
    SCALAR(c->exc_index); SCALAR(c->canonical); SCALAR(c->drift); SCALAR(c->counter);
    SCALAR(c->n_present); SCALAR(c->n_won);
    TAKE(c->e_exists, uint8_t, c->n_ids); TAKE(c->e_lt, int64_t, c->n_ids); TAKE(c->e_rank, uint32_t, c->n_ids);
    TAKE(c->e_val, uint32_t, c->n_ids); TAKE(c->e_mod, int64_t, c->n_ids); TAKE(c->e_flags, uint8_t, c->n);
}

/* ---- a 1-rank loopback communicator (CRDT_MEM_HOST: host words, synchronous) ---------------- */
static int lb_calls;
static int lb_all_reduce(void* user, int64_t* w, uint64_t n, int32_t op, void* stream) {
    (void)user; (void)w; (void)n; (void)op; (void)stream;
    ++lb_calls;
    return 0;                                            /* one rank: the words are the result */
}
static int lb_all_gather(void* user, const int64_t* send, int64_t* recv, uint64_t n, void* stream) {
    (void)user; (void)stream;
    ++lb_calls;
    memcpy(recv, send, n * sizeof(int64_t));
    return 0;
}
static int lb_all_to_all(void* user, uint32_t n_cols, const void* const* s, void* const* r, const uint32_t* eb,
                         const uint64_t* sc, const uint64_t* sd, const uint64_t* rc, const uint64_t* rd, void* stream) {
    (void)user; (void)n_cols; (void)s; (void)r; (void)eb; (void)sd; (void)rd; (void)stream;
    ++lb_calls;
    return (sc[0] || rc[0]) ? 1 : 0;                     /* no peers: the library moves its own chunk */
}

static int check(const Case* c, crdt_ctx* ctx, int rc, const crdt_result* res, const uint8_t* flags,
                 const char* what, int counted) {
    int bad = 0;
#define EXPECT(cond, ...) do { if (!(cond)) { fprintf(stderr, "[%s/%s] ", c->name, what); \
                                 fprintf(stderr, __VA_ARGS__); fputc('\n', stderr); bad = 1; } } while (0)
    EXPECT(rc == c->status, "return %d, want %d", rc, c->status);
    EXPECT(res->status == c->status, "status %d, want %d", res->status, c->status);
    EXPECT(res->n_stored == c->n_stored, "n_stored %u, want %u", res->n_stored, c->n_stored);
    EXPECT(res->canonical_lt == c->canonical, "canonical %lld, want %lld", (long long)res->canonical_lt,
           (long long)c->canonical);
    if (c->status) {
        EXPECT(res->exc_changeset == c->exc_changeset, "exc_changeset %u, want %u", res->exc_changeset,
               c->exc_changeset);
        EXPECT(res->exc_index == c->exc_index, "exc_index %llu, want %llu", (unsigned long long)res->exc_index,
               (unsigned long long)c->exc_index);
        EXPECT(res->drift_ms == c->drift, "drift %lld, want %lld", (long long)res->drift_ms, (long long)c->drift);
        EXPECT(res->counter == c->counter, "counter %lld, want %lld", (long long)res->counter, (long long)c->counter);
    }
    if (counted) {
        EXPECT(res->n_present == c->n_present, "n_present %llu, want %llu", (unsigned long long)res->n_present,
               (unsigned long long)c->n_present);
        EXPECT(res->n_won == c->n_won, "n_won %llu, want %llu", (unsigned long long)res->n_won,
               (unsigned long long)c->n_won);
    }
    if (flags)
        for (uint64_t i = 0; i < c->n; ++i)
            if (flags[i] != c->e_flags[i]) { EXPECT(0, "win flag %llu: %u, want %u", (unsigned long long)i, flags[i], c->e_flags[i]); break; }
    int64_t canon = 0;
    crdt_get_canonical(ctx, &canon);
    EXPECT(canon == c->canonical, "ctx canonical %lld", (long long)canon);
    uint32_t* ids = malloc(sizeof(uint32_t) * c->n_ids);
    int64_t* lt = malloc(sizeof(int64_t) * c->n_ids);
    int64_t* mod = malloc(sizeof(int64_t) * c->n_ids);
    uint32_t* rank = malloc(sizeof(uint32_t) * c->n_ids);
    uint32_t* val = malloc(sizeof(uint32_t) * c->n_ids);
    for (uint32_t i = 0; i < c->n_ids; ++i) ids[i] = i;
    int st = crdt_read_rows(ctx, ids, c->n_ids, lt, rank, val, mod, CRDT_MEM_HOST);
    EXPECT(st == CRDT_OK, "crdt_read_rows %d", st);
    for (uint32_t i = 0; i < c->n_ids && !bad; ++i) {
        if (c->e_exists[i]) {
            EXPECT(lt[i] == c->e_lt[i] && rank[i] == c->e_rank[i] && val[i] == c->e_val[i] && mod[i] == c->e_mod[i],
                   "row %u (%lld, %u, %u, %lld), want (%lld, %u, %u, %lld)", i, (long long)lt[i], rank[i], val[i],
                   (long long)mod[i], (long long)c->e_lt[i], c->e_rank[i], c->e_val[i], (long long)c->e_mod[i]);
        } else {
            EXPECT(mod[i] < 0, "row %u should be absent (mod %lld)", i, (long long)mod[i]);
        }
    }
    free(ids); free(lt); free(mod); free(rank); free(val);
    return bad;
#undef EXPECT
}

/* mode 0: gather + flags; 1: sorted, no flags; 2: 1-rank sharded ctx over the loopback table;
 * 3: sorted on 32-B rows with a declared rank bound; 4: 1-rank pre-sharded ctx, loopback table;
 * 5: 1-rank pre-sharded ctx over RCCL */
static int run(const Case* c, int mode) {
    crdt_ctx* ctx = NULL;
    int st = crdt_create(0, c->local_rank, c->n_ids, &ctx);
    if (st != CRDT_OK) { fprintf(stderr, "crdt_create: %s\n", crdt_status_string(st)); return 1; }
    if (mode == 3) {
        uint32_t bound = 0;
        for (uint64_t i = 0; i < c->n; ++i) if (c->rank[i] + 1 > bound) bound = c->rank[i] + 1;
        if ((st = crdt_set_row_bytes(ctx, 32)) != CRDT_OK || (st = crdt_set_rank_bound(ctx, bound)) != CRDT_OK) {
            fprintf(stderr, "mode 3 setup: %s\n", crdt_status_string(st));
            crdt_destroy(ctx);
            return 1;
        }
    }
    uint32_t* ids = malloc(sizeof(uint32_t) * (c->n_local ? c->n_local : 1));
    int64_t *lt = malloc(8 * (c->n_local + 1)), *mod = malloc(8 * (c->n_local + 1));
    uint32_t *rk = malloc(4 * (c->n_local + 1)), *vl = malloc(4 * (c->n_local + 1));
    uint64_t m = 0;
    for (uint32_t i = 0; i < c->n_local; ++i) {
        if ((uint64_t)c->l_mod[i] == 0x8080808080808080ull) continue;     /* absent: never put */
        ids[m] = i; lt[m] = c->l_lt[i]; rk[m] = c->l_rank[i]; vl[m] = c->l_val[i]; mod[m] = c->l_mod[i];
        ++m;
    }
    st = crdt_put_rows(ctx, ids, lt, rk, vl, mod, m, CRDT_MEM_HOST);
    free(ids); free(lt); free(mod); free(rk); free(vl);
    if (st != CRDT_OK) { fprintf(stderr, "crdt_put_rows: %s\n", crdt_status_string(st)); crdt_destroy(ctx); return 1; }
    crdt_set_canonical(ctx, c->c0);
    crdt_batch b;
    b.key_id = c->key; b.lt = c->lt; b.rank = c->rank; b.val = c->val; b.millis = c->millis;
    b.offsets = c->offsets; b.n_changesets = c->R; b.mem = CRDT_MEM_HOST;
    uint8_t* flags = NULL;
    const char* what = mode == 0 ? "gather" : mode == 1 ? "sorted" : mode == 2 ? "sharded-1" : mode == 3 ? "sorted-32B-bound"
                     : mode == 4 ? "presharded-1" : "presharded-1-rccl";
    if (mode == 0) {
        crdt_set_merge_path(ctx, CRDT_PATH_GATHER);
        flags = calloc(c->n ? c->n : 1, 1);
    } else if (mode == 1 || mode == 3) {
        crdt_set_merge_path(ctx, CRDT_PATH_SORTED);
        crdt_set_counts(ctx, 0);
    } else if (mode == 5) {
        uint8_t id[CRDT_COMM_ID_BYTES];
        uint32_t nr = 0, rk = 9;
        int32_t cst = -1;
        const char* phase = NULL;
        if ((st = crdt_comm_unique_id(id)) != CRDT_OK || (st = crdt_comm_init_rccl(ctx, 1, 0, id)) != CRDT_OK ||
            (st = crdt_set_comm_timeout(ctx, 300000)) != CRDT_OK ||     /* what GpuMapCrdt.sharded calls */
            (st = crdt_set_presharded(ctx, 1)) != CRDT_OK || (st = crdt_comm_info(ctx, &nr, &rk)) != CRDT_OK ||
            (st = crdt_comm_state(ctx, &cst, &phase)) != CRDT_OK || cst != 0 || !phase ||
            nr != 1 || rk != 0) {
            fprintf(stderr, "mode 5 setup: %s\n", crdt_status_string(st));
            crdt_destroy(ctx);
            return 1;
        }
        flags = calloc(c->n ? c->n : 1, 1);
    } else {
        crdt_comm_ops ops;
        memset(&ops, 0, sizeof(ops));
        ops.mem = CRDT_MEM_HOST;
        ops.all_reduce_i64 = lb_all_reduce;
        ops.all_gather_i64 = lb_all_gather;
        ops.all_to_all_v = lb_all_to_all;
        st = crdt_comm_init_ops(ctx, 1, 0, &ops);
        if (st == CRDT_OK && mode == 4) st = crdt_set_presharded(ctx, 1);
        if (st != CRDT_OK) { fprintf(stderr, "crdt_comm_init_ops: %s\n", crdt_status_string(st)); crdt_destroy(ctx); return 1; }
        flags = calloc(c->n ? c->n : 1, 1);
    }
    crdt_result res;
    memset(&res, 0, sizeof(res));
    const int calls0 = lb_calls;
    const int rc = crdt_merge(ctx, &b, c->wall, flags, &res);
    int counted = 1;
    if (mode == 1 || mode == 3) {                        /* the order-free sorted form does not count */
        int path = 0;
        crdt_last_path(ctx, &path);
        counted = path != CRDT_PATH_SORTED;
    }
    int bad = check(c, ctx, rc, &res, flags, what, counted);
    if ((mode == 2 || mode == 4) && c->R && lb_calls == calls0) { fprintf(stderr, "[%s/%s] the communicator was never called\n", c->name, what); bad = 1; }
    if (mode == 5) crdt_comm_free(ctx);
    free(flags);
    crdt_destroy(ctx);
    return bad;
}

/* CrdtJson.decode of a small document through libcrdt_host.so (crdt_json.dart:19-37, hlc.dart:39-46):
 * keys in document order, lt = (millis << 16) + counter, node ids in first-seen order, value spans
 * (length 0 = null). */
/* mergeJson's second half (crdt.dart:100-109 -> merge, crdt.dart:77-94) as the Dart / Python shims
 * run it: the decoded columns (node ids remapped to ranks in String.compareTo order beside the local
 * node "node_a": node_b -> 1, node_c -> 2; value handles = record index, null = 0xFFFFFFFF) merged
 * as one changeset into an empty map on the device.  Every record wins (no local row), every stored
 * row carries modified = R_1 = max(C_0, max lt) and the canonical ends at send(R_1). */
static int json_merge_check(const uint32_t* kid, const int64_t* lt, const uint32_t* node, const uint32_t* vlen,
                            const int64_t* want_lt) {
    crdt_ctx* ctx = NULL;
    int st = crdt_create(0, 0, 16, &ctx);
    if (st != CRDT_OK) { fprintf(stderr, "json merge: crdt_create: %s\n", crdt_status_string(st)); return 1; }
    uint32_t rank[3], val[3];
    for (int i = 0; i < 3; ++i) {
        rank[i] = node[i] + 1;
        val[i] = vlen[i] == 0 ? 0xFFFFFFFFu : (uint32_t)i;
    }
    const uint64_t offs[2] = {0, 3};
    crdt_batch b;
    memset(&b, 0, sizeof(b));
    b.key_id = kid; b.lt = lt; b.rank = rank; b.val = val; b.millis = NULL;
    b.offsets = offs; b.n_changesets = 1; b.mem = CRDT_MEM_HOST;
    const int64_t wall = (want_lt[2] >> 16) + 5000;               /* 5 s after the newest record */
    crdt_result res;
    memset(&res, 0, sizeof(res));
    uint8_t flags[3] = {0, 0, 0};
    int bad = 0;
    st = crdt_merge(ctx, &b, wall, flags, &res);
    const int64_t r1 = want_lt[2];                               /* C_0 = 0 < every lt */
    const int64_t c1 = (r1 + 1) > (wall << 16) ? r1 + 1 : wall << 16;
    if (st != CRDT_OK || res.status != 0 || res.canonical_lt != c1 || !flags[0] || !flags[1] || !flags[2]) {
        fprintf(stderr, "json merge: st %d status %d canonical %lld (want %lld)\n", st, (int)res.status,
                (long long)res.canonical_lt, (long long)c1);
        bad = 1;
    } else {
        int64_t glt[3], gmod[3];
        uint32_t grank[3], gval[3];
        st = crdt_read_rows(ctx, kid, 3, glt, grank, gval, gmod, CRDT_MEM_HOST);
        for (int i = 0; i < 3 && st == CRDT_OK; ++i)
            if (glt[i] != want_lt[i] || grank[i] != rank[i] || gval[i] != val[i] || gmod[i] != r1) {
                fprintf(stderr, "json merge row %d: lt %lld rank %u val %u mod %lld\n", i, (long long)glt[i],
                        grank[i], gval[i], (long long)gmod[i]);
                bad = 1;
            }
        if (st != CRDT_OK) { fprintf(stderr, "json merge: crdt_read_rows: %s\n", crdt_status_string(st)); bad = 1; }
    }
    crdt_destroy(ctx);
    return bad;
}

static int json_decode_check(void) {
    static const char doc[] =
        "{\"k0\":{\"hlc\":\"2024-01-01T00:00:00.000Z-0000-node_b\",\"value\":1},"
        "\"k1\":{\"hlc\":\"2024-01-01T00:00:00.001Z-000A-node_c\",\"value\":null},"
        "\"k2\":{\"hlc\":\"2024-01-01T00:00:01.000Z-FFFF-node_b\",\"value\":\"x\"}}";
    crdt_keys* keys = crdt_keys_create();
    crdt_decoded* d = NULL;
    int bad = 0;
    int st = crdt_json_decode(doc, sizeof(doc) - 1, keys, &d);
    if (st != CRDT_HOST_OK || !d || crdt_decoded_count(d) != 3 || crdt_decoded_node_count(d) != 2) {
        fprintf(stderr, "crdt_json_decode: status %d\n", st);
        bad = 1;
    } else {
        uint32_t kid[3], node[3], vlen[3];
        int64_t lt[3];
        uint64_t voff[3], noff[3];
        char nodes[64];
        crdt_decoded_columns(d, kid, lt, node, voff, vlen);
        crdt_decoded_nodes(d, nodes, sizeof(nodes), noff);
        const int64_t ms = 1704067200000ll;
        const int64_t want_lt[3] = {ms << 16, ((ms + 1) << 16) + 0xA, ((ms + 1000) << 16) + 0xFFFF};
        const uint32_t want_node[3] = {0, 1, 0}, want_len[3] = {1, 0, 3};
        for (int i = 0; i < 3; ++i)
            if (kid[i] != (uint32_t)i || lt[i] != want_lt[i] || node[i] != want_node[i] || vlen[i] != want_len[i]) {
                fprintf(stderr, "crdt_json_decode record %d: key %u lt %lld node %u len %u\n", i, kid[i],
                        (long long)lt[i], node[i], vlen[i]);
                bad = 1;
            }
        if (memcmp(nodes + noff[0], "node_b", 6) != 0 || memcmp(nodes + noff[1], "node_c", 6) != 0 ||
            memcmp(doc + voff[2], "\"x\"", 3) != 0) {
            fprintf(stderr, "crdt_json_decode: node ids / value spans differ\n");
            bad = 1;
        }
        if (!bad) bad = json_merge_check(kid, lt, node, vlen, want_lt);
    }
    if (d) crdt_decoded_free(d);
    crdt_keys_destroy(keys);
    return bad;
}

int main(int argc, char** argv) {
    const char* path = argc > 1 ? argv[1] : "tests/golden/abi_cases.bin";
    FILE* f = fopen(path, "rb");
    if (!f) { perror(path); return 2; }
    fseek(f, 0, SEEK_END);
    const long sz = ftell(f);
    fseek(f, 0, SEEK_SET);
    uint8_t* buf = malloc((size_t)sz);
    if (fread(buf, 1, (size_t)sz, f) != (size_t)sz) { fprintf(stderr, "short read\n"); return 2; }
    fclose(f);
    g_p = buf;
    g_end = buf + sz;
    if (sz < 12 || memcmp(g_p, "CRDTABI1", 8) != 0) { fprintf(stderr, "bad magic\n"); return 2; }
    g_p += 8;
    uint32_t nc;
    SCALAR(nc);
    if (crdt_abi_version() != CRDT_ABI_VERSION) { fprintf(stderr, "ABI version mismatch\n"); return 2; }
    int ndev = 0;
    crdt_device_count(&ndev);
    if (ndev < 1) { fprintf(stderr, "no device\n"); return 3; }
    int bad = 0, runs = 0;
    for (uint32_t k = 0; k < nc; ++k) {
        Case c;
        read_case(&c);
        for (int mode = 0; mode < 6; ++mode, ++runs) bad |= run(&c, mode);
    }
    bad |= json_decode_check();
    printf("abi_golden: %u cases x 6 modes (gather + flags, sorted, 1-rank sharded over a C loopback "
           "communicator, sorted on 32-B rows with a rank bound, 1-rank pre-sharded over the loopback and "
           "over RCCL) + crdt_json_decode: %s\n", nc, bad ? "MISMATCH" : "all equal");
    (void)runs;
    return bad ? 1 : 0;
}
