/* TEST INFRASTRUCTURE ONLY — the optimised multi-core CPU baseline (SURVEY §8(d) "CPU baseline (2)").
 *
 * Same results as or_merge() in merge_oracle.c (R back-to-back Crdt.merge calls,
 * lib/src/crdt.dart:77-94, on the columnar row layout), restructured for host
 * cores instead of restating the reference's cost: per changeset j
 *   1. one parallel pass: M_j = max lt, and whether any record is flagged
 *      (rank == local: hlc.dart:88-90; millis - wall > 60000: hlc.dart:92-94) with
 *      lt above the canonical C_{j-1}; only then the exact sequential recv loop
 *      (hlc.dart:80-97) runs over that changeset to find the first raising record;
 *   2. canonical after the recv loop R_j = max(C_{j-1}, M_j) (recv only advances to a larger lt);
 *   3. parallel apply (keys are unique within a changeset, so rows never race):
 *      winner iff absent / invisible or (lt, rank) strictly larger (crdt.dart:83-84),
 *      stored with mod = R_j (crdt.dart:86-87);
 *   4. C_j = Hlc.send(R_j) (crdt.dart:93, hlc.dart:51-74).
 * Used by bench.py's cpu_baseline leg and checked against or_merge() in tests/.
 */
#include <omp.h>
#include <stdint.h>
#include <string.h>

#define OM_SHIFT 16
#define OM_MAX_COUNTER 0xFFFF
#define OM_MAX_DRIFT 60000

typedef struct { int64_t lt; uint32_t rank; uint32_t val; int64_t mod; int64_t aux; } om_row;

typedef struct {
    int32_t status;
    uint32_t n_stored;
    uint32_t exc_changeset;
    uint32_t pad;
    uint64_t exc_index;
    int64_t canonical_lt;
    int64_t drift_ms;
    int64_t counter;
    uint64_t n_present;
    uint64_t n_won;
} om_result;

static inline int64_t om_wsub(int64_t a, int64_t b) { return (int64_t)((uint64_t)a - (uint64_t)b); }

static int om_send(int64_t c, int64_t wall, int64_t* out, int64_t* drift, int64_t* counter)
{
    int64_t m = c >> OM_SHIFT, k = c & OM_MAX_COUNTER;
    int64_t mn = m > wall ? m : wall;
    int64_t kn = m == mn ? k + 1 : 0;
    if (om_wsub(mn, wall) > OM_MAX_DRIFT) { *drift = om_wsub(mn, wall); return 1; }
    if (kn > OM_MAX_COUNTER) { *counter = kn; return 3; }
    *out = (int64_t)(((uint64_t)mn << OM_SHIFT) + (uint64_t)kn);
    return 0;
}

int or_merge_omp(om_row* table, uint64_t cap, int64_t* canonical, uint32_t local_rank,
                 const uint32_t* key, const int64_t* lt, const uint32_t* rank, const uint32_t* val,
                 const int64_t* millis, const uint64_t* offsets, uint32_t n_changesets, int64_t wall,
                 uint8_t* win_flags, int n_threads, om_result* res)
{
    memset(res, 0, sizeof(*res));
    res->exc_index = UINT64_MAX;
    if (n_threads > 0) omp_set_num_threads(n_threads);
    const uint64_t n_total = offsets[n_changesets];
    int bad = 0;
#pragma omp parallel for reduction(| : bad) schedule(static)
    for (uint64_t i = 0; i < n_total; ++i) bad |= key[i] >= cap;
    if (bad) return -4;
    if (win_flags) memset(win_flags, 0, n_total);
    int64_t c = *canonical;
    for (uint32_t j = 0; j < n_changesets; ++j) {
        const uint64_t b = offsets[j], e = offsets[j + 1];
        int64_t mj = INT64_MIN;
        int cand = 0;
        const int64_t cprev = c;
#pragma omp parallel for reduction(max : mj) reduction(| : cand) schedule(static)
        for (uint64_t i = b; i < e; ++i) {
            const int64_t v = lt[i];
            mj = v > mj ? v : mj;
            const int64_t ms = millis ? millis[i] : (v >> OM_SHIFT);
            cand |= (v > cprev) & ((rank[i] == local_rank) | (om_wsub(ms, wall) > OM_MAX_DRIFT));
        }
        if (cand) {                                   /* exact recv loop over this changeset */
            int64_t r = c;
            for (uint64_t i = b; i < e; ++i) {
                if (r >= lt[i]) continue;
                const int64_t ms = millis ? millis[i] : (lt[i] >> OM_SHIFT);
                const int dup = rank[i] == local_rank;
                if (dup || om_wsub(ms, wall) > OM_MAX_DRIFT) {
                    res->status = dup ? 2 : 1;
                    res->exc_changeset = j;
                    res->exc_index = i - b;
                    if (!dup) res->drift_ms = om_wsub(ms, wall);
                    res->canonical_lt = r;
                    res->n_stored = j;
                    *canonical = r;
                    return res->status;
                }
                r = lt[i];
            }
        }
        if (e > b && mj > c) c = mj;                  /* R_j */
        const int64_t stamp = c;
        uint64_t np = 0, nw = 0;
#pragma omp parallel for reduction(+ : np, nw) schedule(static)
        for (uint64_t i = b; i < e; ++i) {
            om_row* w = &table[key[i]];
            const int present = w->mod >= 0;
            const int win = !present || lt[i] > w->lt || (lt[i] == w->lt && rank[i] > w->rank);
            np += present;
            if (win) {
                w->lt = lt[i]; w->rank = rank[i]; w->val = val[i]; w->mod = stamp; w->aux = 0;
                nw++;
                if (win_flags) win_flags[i] = 1;
            }
        }
        res->n_present += np;
        res->n_won += nw;
        res->n_stored = j + 1;
        int64_t drift = 0, counter = 0, nc = 0;
        const int st = om_send(c, wall, &nc, &drift, &counter);
        if (st) {
            res->status = st; res->exc_changeset = j; res->exc_index = UINT64_MAX;
            res->drift_ms = drift; res->counter = counter;
            res->canonical_lt = c; *canonical = c;
            return st;
        }
        c = nc;
    }
    res->canonical_lt = c;
    *canonical = c;
    return 0;
}
