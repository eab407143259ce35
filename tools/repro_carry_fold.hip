// repro_carry_fold.hip — does the carry fold of k_part_carry<true> (sorted_path.inc) compute
// the same rows when written the way it first was?
//
// Round 1 recorded ("carry kernel") that the fold written as one short-circuit
// expression, with the batch registers bl / br / bv left uninitialised for parts that do not
// exist, stored a row's val from a different record than its lt / rank, and that explicit
// `take` flags with every register defined were exact.  That first form was never committed.
// This program restates it (variant A: uninitialised registers read only behind && / ||)
// beside the shipped form (variant B: every register defined) and the same fold on the host,
// on random part states with absent parts, ties on (lt, rank) and both changeset orders, and
// reports every key whose (lt, rank, val, j) differ.  Build and run:
//   hipcc -O3 --offload-arch=gfx950 -o tools/repro_carry_fold tools/repro_carry_fold.hip
//   tools/repro_carry_fold            (prints one summary line per variant)
#include <hip/hip_runtime.h>

#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <vector>

constexpr uint32_t kJLocal = 0xFFFFFFFFu, kJAbsent = 0xFFFFFFFEu;
constexpr uint32_t kB = 8;

__host__ __device__ inline uint32_t jkey(uint32_t j) { return j == 0xFFFFu || j == kJLocal ? 0u : j + 1u; }
__host__ __device__ inline bool beats_j(int64_t l, uint32_t r, uint32_t j, int64_t ol, uint32_t orr, uint32_t oj) {
    return l > ol || (l == ol && (r > orr || (r == orr && jkey(j) < jkey(oj))));
}

struct Out { int64_t l; uint32_t r, v, j; };

// Variant A: the first form.  bl / br / bv are written only for existing parts; the fold reads
// them only behind the short-circuit (bj != kJAbsent && ...), so no indeterminate value is used
// by the C++ semantics — the question is whether the compiled code agrees.
template <bool kDefined>
__global__ void k_fold(const int64_t* __restrict__ pl, const uint32_t* __restrict__ pr, const uint32_t* __restrict__ pv,
                       const uint32_t* __restrict__ pj, const int64_t* __restrict__ tl, const uint32_t* __restrict__ tr,
                       const uint32_t* __restrict__ tpresent, uint32_t nkeys, uint32_t np, Out* __restrict__ out)
{
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= nkeys) return;
    int64_t l = tl[k];
    uint32_t r = tr[k], v = 0, j = tpresent[k] ? kJLocal : kJAbsent;
    for (uint32_t p0 = 0; p0 < np; p0 += kB) {
        int64_t bl[kB];
        uint32_t br[kB], bv[kB], bj[kB];
#pragma unroll
        for (uint32_t q = 0; q < kB; ++q) {
            const uint32_t p = p0 + q;
            bj[q] = kJAbsent;
            if (kDefined) { bl[q] = 0; br[q] = bv[q] = 0; }
            if (p > 0 && p < np) {
                const uint64_t src = (uint64_t)(p - 1) * nkeys + k;
                bj[q] = pj[src];
                bl[q] = pl[src];
                br[q] = pr[src];
                bv[q] = pv[src];
            }
        }
#pragma unroll
        for (uint32_t q = 0; q < kB; ++q) {
            const uint32_t p = p0 + q;
            if (p >= np) break;
            bool take;
            if (kDefined) {
                take = bj[q] != kJAbsent;
                if (take && j != kJAbsent) take = beats_j(bl[q], br[q], bj[q], l, r, j);
            } else {
                take = bj[q] != kJAbsent && (j == kJAbsent || beats_j(bl[q], br[q], bj[q], l, r, j));
            }
            if (take) { l = bl[q]; r = br[q]; v = bv[q]; j = bj[q]; }
        }
    }
    out[k] = Out{l, r, v, j};
}

int main() {
    const uint32_t nkeys = 1u << 20, np = 19;                 // parts 1..18 carry states, part 0 none
    const size_t ns = (size_t)(np - 1) * nkeys;
    std::vector<int64_t> pl(ns), tl(nkeys);
    std::vector<uint32_t> pr(ns), pv(ns), pj(ns), tr(nkeys), tp(nkeys);
    srand(12345);
    for (size_t i = 0; i < ns; ++i) {
        pl[i] = 1000 + rand() % 4;                            // heavy (lt, rank) ties
        pr[i] = rand() % 3;
        pv[i] = (uint32_t)i;                                  // val identifies the record
        pj[i] = rand() % 5 == 0 ? kJAbsent : (uint32_t)(rand() % 4096);
    }
    for (uint32_t k = 0; k < nkeys; ++k) { tl[k] = 1000 + rand() % 4; tr[k] = rand() % 3; tp[k] = rand() % 3 != 0; }
    // host fold (the same rule, sequentially)
    std::vector<Out> ref(nkeys);
    for (uint32_t k = 0; k < nkeys; ++k) {
        int64_t l = tl[k];
        uint32_t r = tr[k], v = 0, j = tp[k] ? kJLocal : kJAbsent;
        for (uint32_t p = 1; p < np; ++p) {
            const size_t src = (size_t)(p - 1) * nkeys + k;
            if (pj[src] == kJAbsent) continue;
            if (j == kJAbsent || beats_j(pl[src], pr[src], pj[src], l, r, j)) { l = pl[src]; r = pr[src]; v = pv[src]; j = pj[src]; }
        }
        ref[k] = Out{l, r, v, j};
    }
    int64_t *d_pl, *d_tl; uint32_t *d_pr, *d_pv, *d_pj, *d_tr, *d_tp; Out* d_out;
    if (hipMalloc(&d_pl, ns * 8) || hipMalloc(&d_pr, ns * 4) || hipMalloc(&d_pv, ns * 4) || hipMalloc(&d_pj, ns * 4) ||
        hipMalloc(&d_tl, nkeys * 8) || hipMalloc(&d_tr, nkeys * 4) || hipMalloc(&d_tp, nkeys * 4) ||
        hipMalloc(&d_out, nkeys * sizeof(Out))) { fprintf(stderr, "hipMalloc failed\n"); return 1; }
    hipMemcpy(d_pl, pl.data(), ns * 8, hipMemcpyHostToDevice);
    hipMemcpy(d_pr, pr.data(), ns * 4, hipMemcpyHostToDevice);
    hipMemcpy(d_pv, pv.data(), ns * 4, hipMemcpyHostToDevice);
    hipMemcpy(d_pj, pj.data(), ns * 4, hipMemcpyHostToDevice);
    hipMemcpy(d_tl, tl.data(), nkeys * 8, hipMemcpyHostToDevice);
    hipMemcpy(d_tr, tr.data(), nkeys * 4, hipMemcpyHostToDevice);
    hipMemcpy(d_tp, tp.data(), nkeys * 4, hipMemcpyHostToDevice);
    int bad_any = 0;
    for (int variant = 0; variant < 2; ++variant) {
        hipMemset(d_out, 0xAB, nkeys * sizeof(Out));
        if (variant == 0) k_fold<false><<<nkeys / 256, 256>>>(d_pl, d_pr, d_pv, d_pj, d_tl, d_tr, d_tp, nkeys, np, d_out);
        else k_fold<true><<<nkeys / 256, 256>>>(d_pl, d_pr, d_pv, d_pj, d_tl, d_tr, d_tp, nkeys, np, d_out);
        if (hipDeviceSynchronize() != hipSuccess) { fprintf(stderr, "kernel failed\n"); return 1; }
        std::vector<Out> got(nkeys);
        hipMemcpy(got.data(), d_out, nkeys * sizeof(Out), hipMemcpyDeviceToHost);
        uint32_t bad = 0, bad_val_only = 0, first = UINT32_MAX;
        for (uint32_t k = 0; k < nkeys; ++k) {
            const Out& a = got[k];
            const Out& b = ref[k];
            const bool same_lrj = a.l == b.l && a.r == b.r && a.j == b.j;
            if (!same_lrj || a.v != b.v) {
                ++bad;
                if (same_lrj) ++bad_val_only;
                if (first == UINT32_MAX) first = k;
            }
        }
        printf("variant %s: %u of %u keys differ from the host fold (%u with equal lt / rank / j but another val)%s\n",
               variant == 0 ? "A (first form, short-circuit over uninitialised registers)"
                            : "B (shipped form, every register defined)",
               bad, nkeys, bad_val_only, bad ? "" : " -- exact");
        if (bad) {
            const Out& a = got[first];
            const Out& b = ref[first];
            printf("  first: key %u got (%lld, %u, %u, %u) want (%lld, %u, %u, %u)\n", first, (long long)a.l, a.r, a.v,
                   a.j, (long long)b.l, b.r, b.v, b.j);
            bad_any = 1;
        }
    }
    return bad_any ? 2 : 0;
}
