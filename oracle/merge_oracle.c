/* TEST INFRASTRUCTURE ONLY — columnar CPU restatement of the reference merge.
 *
 * This file is the checker (tests/, __graft_entry__.smoke(), bench.py's
 * cpu_baseline leg), never the product.  It restates, on the columnar row
 * layout the device uses, the sequential semantics of R back-to-back calls of
 * the Dart reference's Crdt.merge (/root/reference, crdt v4.0.2):
 *
 *   merge                 lib/src/crdt.dart:77-94
 *   Hlc.recv              lib/src/hlc.dart:80-97
 *   Hlc.send              lib/src/hlc.dart:51-74
 *   Hlc compare / >=      lib/src/hlc.dart:143-161
 *   logicalTime           lib/src/hlc.dart:16  ((millis<<16)+counter, wrapping)
 *   recordMap filter      lib/src/map_crdt.dart:42-45  (modified.lt < since dropped)
 *   putRecords            lib/src/map_crdt.dart:33-39
 *   refreshCanonicalTime  lib/src/crdt.dart:114-121
 *   put / putAll          lib/src/crdt.dart:39-54
 *
 * A row is "present" for merge iff it exists and its modified lt >= 0 (the
 * recordMap() filter with modifiedSince == null); a never-written row carries
 * mod = INT64_MIN.  Node ids are order-preserving ranks (Dart String.compareTo
 * order), so nodeId equality is rank equality.
 *
 * faithful != 0 additionally mirrors the reference's cost structure: one full
 * snapshot copy of the local map per merge (map_crdt.dart:43) and one wall
 * clock read per remote record (hlc.dart:82).  Results do not depend on it.
 * faithful = T > 1 runs the snapshot copy on T threads (the bulk map copy is the
 * only part of the reference algorithm with no order; the recv loop and the
 * winner loop stay sequential, as in the reference).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#define OR_SHIFT 16
#define OR_MAX_COUNTER 0xFFFF
#define OR_MAX_DRIFT 60000

enum { OR_OK = 0, OR_CLOCK_DRIFT = 1, OR_DUPLICATE_NODE = 2, OR_OVERFLOW = 3, OR_E_INVALID = -1,
       OR_E_KEY_RANGE = -4 };

typedef struct { int64_t lt; uint32_t rank; uint32_t val; int64_t mod; int64_t aux; } or_row;

typedef struct {
    int32_t status;
    uint32_t n_stored;       /* changesets whose winners were stored */
    uint32_t exc_changeset;
    uint32_t pad;
    uint64_t exc_index;      /* record index inside exc_changeset, UINT64_MAX for a send() failure */
    int64_t canonical_lt;
    int64_t drift_ms;
    int64_t counter;
    uint64_t n_present;
    uint64_t n_won;
} or_result;

static inline int64_t wsub(int64_t a, int64_t b) { return (int64_t)((uint64_t)a - (uint64_t)b); }

/* Hlc.send on a canonical held as a logical time (always in canonical form). */
static int or_send(int64_t c, int64_t wall, int64_t* out, int64_t* drift, int64_t* counter)
{
    int64_t millis_old = c >> OR_SHIFT, counter_old = c & OR_MAX_COUNTER;
    int64_t millis_new = millis_old > wall ? millis_old : wall;
    int64_t counter_new = millis_old == millis_new ? counter_old + 1 : 0;
    if (wsub(millis_new, wall) > OR_MAX_DRIFT) { *drift = wsub(millis_new, wall); return OR_CLOCK_DRIFT; }
    if (counter_new > OR_MAX_COUNTER) { *counter = counter_new; return OR_OVERFLOW; }
    *out = (int64_t)(((uint64_t)millis_new << OR_SHIFT) + (uint64_t)counter_new);
    return OR_OK;
}

int or_send_scalar(int64_t c, int64_t wall, int64_t* out, int64_t* drift, int64_t* counter)
{
    return or_send(c, wall, out, drift, counter);
}

static volatile int64_t or_clock_sink;
static inline void or_read_clock(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_REALTIME, &ts);
    or_clock_sink = ts.tv_nsec;
}

int or_merge(or_row* table, uint64_t cap, int64_t* canonical, uint32_t local_rank,
             const uint32_t* key, const int64_t* lt, const uint32_t* rank, const uint32_t* val,
             const int64_t* millis, const uint64_t* offsets, uint32_t n_changesets, int64_t wall,
             uint8_t* win_flags, int faithful, or_result* res)
{
    memset(res, 0, sizeof(*res));
    res->exc_index = UINT64_MAX;
    int64_t c = *canonical;
    uint64_t n_total = offsets[n_changesets];
    if (win_flags) memset(win_flags, 0, n_total);
    for (uint64_t i = 0; i < n_total; ++i)
        if (key[i] >= cap) return OR_E_KEY_RANGE;
    or_row* snap = NULL;
    if (faithful) snap = (or_row*)malloc(cap * sizeof(or_row));

    for (uint32_t j = 0; j < n_changesets; ++j) {
        uint64_t b = offsets[j], e = offsets[j + 1];
        const or_row* local = table;
        if (faithful) {                                  /* recordMap(): copy + filter */
            const int64_t ncap = (int64_t)cap;
#pragma omp parallel for schedule(static) num_threads(faithful) if (faithful > 1)
            for (int64_t k = 0; k < ncap; ++k) {
                snap[k] = table[k];
                if (snap[k].mod < 0) snap[k].mod = INT64_MIN;
            }
            local = snap;
        }
        /* removeWhere: recv loop over every record (may throw, map untouched) */
        for (uint64_t i = b; i < e; ++i) {
            if (faithful) or_read_clock();
            if (c >= lt[i]) continue;                     /* hlc.dart:85 */
            if (rank[i] == local_rank) {                  /* hlc.dart:88-90 */
                res->status = OR_DUPLICATE_NODE; res->exc_changeset = j; res->exc_index = i - b;
                res->canonical_lt = c; res->n_stored = j; *canonical = c; free(snap); return res->status;
            }
            int64_t rm = millis ? millis[i] : (lt[i] >> OR_SHIFT);
            if (wsub(rm, wall) > OR_MAX_DRIFT) {          /* hlc.dart:92-94 */
                res->status = OR_CLOCK_DRIFT; res->exc_changeset = j; res->exc_index = i - b;
                res->drift_ms = wsub(rm, wall);
                res->canonical_lt = c; res->n_stored = j; *canonical = c; free(snap); return res->status;
            }
            c = lt[i];                                    /* hlc.dart:96 */
        }
        /* winners (crdt.dart:83-84): local absent, or local.hlc < remote.hlc */
        int64_t stamp = c;                                /* crdt.dart:86-87 */
        for (uint64_t i = b; i < e; ++i) {
            const or_row* lr = &local[key[i]];
            int present = lr->mod >= 0;
            int win = !present || lt[i] > lr->lt || (lt[i] == lr->lt && rank[i] > lr->rank);
            res->n_present += present;
            if (win) {
                or_row* w = &table[key[i]];
                w->lt = lt[i]; w->rank = rank[i]; w->val = val[i]; w->mod = stamp; w->aux = 0;
                res->n_won++;
                if (win_flags) win_flags[i] = 1;
            }
        }
        res->n_stored = j + 1;
        int64_t drift = 0, counter = 0, nc = 0;           /* crdt.dart:93 */
        int st = or_send(c, wall, &nc, &drift, &counter);
        if (st != OR_OK) {
            res->status = st; res->exc_changeset = j; res->exc_index = UINT64_MAX;
            res->drift_ms = drift; res->counter = counter;
            res->canonical_lt = c; *canonical = c; free(snap); return st;
        }
        c = nc;
    }
    res->canonical_lt = c;
    *canonical = c;
    free(snap);
    return OR_OK;
}

/* put/putAll (crdt.dart:39-54): one send, every record stamped hlc = modified = C. */
int or_put_stamped(or_row* table, uint64_t cap, int64_t* canonical, uint32_t local_rank,
                   const uint32_t* key, const uint32_t* val, uint64_t n, int64_t wall, or_result* res)
{
    memset(res, 0, sizeof(*res));
    res->exc_index = UINT64_MAX;
    if (n == 0) { res->canonical_lt = *canonical; return OR_OK; }
    for (uint64_t i = 0; i < n; ++i) if (key[i] >= cap) return OR_E_KEY_RANGE;
    int64_t nc = 0, drift = 0, counter = 0;
    int st = or_send(*canonical, wall, &nc, &drift, &counter);
    if (st != OR_OK) {
        res->status = st; res->drift_ms = drift; res->counter = counter; res->canonical_lt = *canonical;
        return st;
    }
    for (uint64_t i = 0; i < n; ++i) {
        or_row* w = &table[key[i]];
        w->lt = nc; w->rank = local_rank; w->val = val[i]; w->mod = nc; w->aux = 0;
    }
    *canonical = nc;
    res->canonical_lt = nc;
    res->n_won = n;
    return OR_OK;
}

/* refreshCanonicalTime (crdt.dart:114-121): max lt over recordMap(), 0 if empty. */
int64_t or_refresh(const or_row* table, uint64_t n_rows)
{
    int any = 0;
    int64_t m = 0;
    for (uint64_t k = 0; k < n_rows; ++k) {
        if (table[k].mod < 0) continue;
        if (!any || table[k].lt > m) m = table[k].lt;
        any = 1;
    }
    return any ? m : 0;
}

/* recordMap(modifiedSince) (map_crdt.dart:42-45): ids with mod >= since, in id order. */
uint64_t or_modified_since(const or_row* table, uint64_t n_rows, int64_t since, uint32_t* out)
{
    uint64_t n = 0;
    for (uint64_t k = 0; k < n_rows; ++k)
        if (!(table[k].mod < since)) out[n++] = (uint32_t)k;
    return n;
}

void or_clear_rows(or_row* table, uint64_t first, uint64_t count)
{
    memset(table + first, 0x80, count * sizeof(or_row));
}
