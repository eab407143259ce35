// crdt_merge.hip — MI355X (gfx950) implementation of the MapCrdt merge hot path.
//
// Implements include/crdt_merge.h.  The reference is the Dart package `crdt`
// v4.0.2 (/root/reference); every kernel names the reference lines it replaces.
// DESIGN.md has the data layout, the roofline of each kernel and the proof that
// the batched clock algebra below equals R sequential Crdt.merge() calls.
//
// Kernels (one HIP stream per ctx; every call is synchronous at the API edge):
//   K3a k_scan     per-changeset max lt (M_j) + tiles holding a record that can
//                  raise (Hlc.recv, hlc.dart:80-97)            [HBM stream, 8 B/record
//                  + rank/millis only for records above C0]
//   K3b k_clock    one workgroup: canonical recurrence C_j = send(max(C_{j-1}, M_j))
//                  as a prefix max; R_j stamps; first send() failure (hlc.dart:51-74)
//   K3c k_verify   exact first recv() failure inside candidate tiles (ordered
//                  wave scan), only when a candidate exists (rare)
//   K3d k_resolve  stop point, status and final canonical (single thread)
//   K2  k_apply    per changeset: gather the local row, (lt, rank) compare, store
//                  winner {lt, rank, val, mod = R_j} (crdt.dart:83-90)
//                  [HBM: 20 B/record stream + 32 B row gather/scatter]
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>      // comm_path.inc: types / prototypes only (librccl is dlopen-ed)

#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <thread>
#include <new>
#include <vector>

#include "crdt_merge.h"

namespace {

constexpr int kShift = 16;                       // hlc.dart:3
constexpr int64_t kMaxCounter = 0xFFFF;          // hlc.dart:4
constexpr int64_t kMaxDrift = 60000;             // hlc.dart:5

constexpr int kScanThreads = 256;
constexpr int kScanItems = 16;
constexpr int kTile = kScanThreads * kScanItems; // 4096 records per scan tile
constexpr int kApplyThreads = 256;
// K2 records per thread (striped) are chosen per launch: 1, 2, 4 or 8
constexpr int kCounterSlots = 64;                // striped n_present / n_won counters
constexpr int kVerifyBlocks = 64;
constexpr uint32_t kTimingStride = 32;          // every 32 apply launches, time a window of
constexpr uint32_t kTimingWindow = 8;           // 8 back-to-back launches (one event pair)

// Collective words are plain signed int64 so an RCCL MAX / MIN all-reduce combines them:
//   maxima[j]  = M_j, INT64_MIN when changeset j is empty (or not homed here)
//   event[0]   = (j << 40) | i  for a recv() failure at record i of changeset j,
//                (j << 40) | kLowMask for a send() failure after j;  INT64_MAX: none
//   event[1..3]= canonical at the failure / kind / Hlc.millis; INT64_MIN, 0, INT64_MIN: none
constexpr int64_t kLowBits = 40;
constexpr int64_t kLowMask = (1ll << kLowBits) - 1;
constexpr int64_t kEvNone = INT64_MAX;

// One device row per key id; rows are 24 or 32 B apart (crdt_set_row_bytes), fields in order:
//   [0:8)  lt      Record.hlc.logicalTime
//   [8:12) rank    Record.hlc.nodeId rank
//   [12:16) mod_hi high word of Record.modified.logicalTime; its sign bit is the visibility test
//                  (mod < 0: invisible to merge / recordMap, map_crdt.dart:42-45)
//   [16:20) mod_lo low word of modified
//   [20:24) val    Record.value handle
//   [24:32) zero   (32-B rows only)
// The first 16 B are everything the merge decision reads, so a gather of a row is ONE dwordx4
// (gfx950 loads / stores vectors at any dword alignment).  24-B rows (the default) make every
// coalesced pass over the table — the sorted path's bucket loads and whole-line writes — move 25 %
// fewer bytes than 32-B ones; 32-B rows make a random winner write one aligned 32-B store, which the
// gather path's streaming workloads (most records win) run faster.
struct Table {
    char* base;
    uint32_t stride;                 // 24 or 32
};

typedef uint32_t u32x4u __attribute__((ext_vector_type(4), aligned(4)));
typedef uint32_t u32x2u __attribute__((ext_vector_type(2), aligned(4)));
typedef uint32_t u32x8a __attribute__((ext_vector_type(8), aligned(32)));

__host__ __device__ inline char* row_ptr(const Table& t, uint64_t k) { return t.base + k * (uint64_t)t.stride; }
// the decision half {lt lo, lt hi, rank, mod_hi} of row k / the rest {mod_lo, val}
__device__ inline uint4 load_hot(const Table& t, uint64_t k) {
    const u32x4u v = *reinterpret_cast<const u32x4u*>(row_ptr(t, k));
    return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ inline uint2 load_cold(const Table& t, uint64_t k) {
    const u32x2u v = *reinterpret_cast<const u32x2u*>(row_ptr(t, k) + 16);
    return make_uint2(v.x, v.y);
}
__device__ inline void store_hc(const Table& t, uint64_t k, uint4 h, uint2 x) {
    char* p = row_ptr(t, k);
    if (t.stride == 32) {                         // one aligned 32-B store
        u32x8a a;
        a.s0 = h.x; a.s1 = h.y; a.s2 = h.z; a.s3 = h.w; a.s4 = x.x; a.s5 = x.y; a.s6 = 0u; a.s7 = 0u;
        *reinterpret_cast<u32x8a*>(p) = a;
        return;
    }
    u32x4u a;
    a.x = h.x; a.y = h.y; a.z = h.z; a.w = h.w;
    *reinterpret_cast<u32x4u*>(p) = a;
    u32x2u b;
    b.x = x.x; b.y = x.y;
    *reinterpret_cast<u32x2u*>(p + 16) = b;
}
__device__ inline int64_t row_mod(const Table& t, uint64_t k) {
    const uint4 h = load_hot(t, k);
    return (int64_t)(((uint64_t)h.w << 32) | load_cold(t, k).x);
}
__device__ inline void store_row(const Table& t, uint64_t k, int64_t lt, uint32_t rank, uint32_t val, int64_t mod) {
    store_hc(t, k, make_uint4((uint32_t)lt, (uint32_t)((uint64_t)lt >> 32), rank, (uint32_t)((uint64_t)mod >> 32)),
             make_uint2((uint32_t)mod, val));
}

// Device-side per-call words.
struct Misc {
    uint32_t cand_count;   // candidate tiles appended by k_scan
    uint32_t stop;         // changesets to apply (set by k_resolve)
    uint32_t err;          // key range violation
    uint32_t vdone;        // k_verify<true> workgroups finished (the last one resolves)
    uint32_t tiles_hot;    // scan tiles holding a record above C_0, every kHotSample-th (next scan's form)
    crdt_result result;    // filled by k_resolve
    // frame of the batch's records (k_scan<*, *, true>) for the sorted path's packed key
    // (sorted_path.inc), as max-accumulators whose identity is the memset's 0:
    //   fr_lo = max(~ord(lt)), fr_hi = max(ord(lt)), ord(x) = x ^ 2^63 (int64 order as uint64);
    //   fr_rlo = max(~rank), fr_rhi = max(rank)
    unsigned long long fr_lo, fr_hi;
    uint32_t fr_rlo, fr_rhi;
    // a bound of the rows the call wrote (k_put_*: one past the largest in-range key id;
    // k_bucket_items: the end of the last non-empty 4096-key bucket of the sorted path): the
    // table's high-water mark of written rows moves to it (crdt_ctx::hw)
    unsigned long long key_end;
    unsigned long long route_own;   // k_route_plan: bit 0 = the own chunk is scattered into the receive columns;
                                    // bit 1 = the send counts do not add up to the batch (the scatters exit);
                                    // bit 2 (k_shard_combine) = the ranks' collective-shape words differ
    unsigned long long shard_status; // k_shard_combine: the largest local failure code (-CRDT_E_*) any rank put in
                                     // its gather row (0: none) — every rank fails the call with it
    unsigned long long fr_cmax;      // k_scan<.., kFrame>: max of the records' lt & 0xFFFF (the compact frame,
                                     // sorted_path.inc PackFrame::cb)
    unsigned long long present[kCounterSlots];
    unsigned long long won[kCounterSlots];
};                             // size a multiple of 16 B: hipMemsetAsync zeroes it with one fill
                               // kernel (1112 B took an aligned fill plus a tail fill, ~5 us each)
static_assert(sizeof(Misc) % 16 == 0, "Misc is memset as whole 16-B words");

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef long long i64x2 __attribute__((ext_vector_type(2)));

__host__ __device__ inline int64_t wsub(int64_t a, int64_t b) { return (int64_t)((uint64_t)a - (uint64_t)b); }
__host__ __device__ inline int64_t imax(int64_t a, int64_t b) { return a > b ? a : b; }

// ------------------------------------------------------------------ wave helpers
__device__ inline int64_t wave_max(int64_t v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v = imax(v, __shfl_xor(v, off, 64));
    return v;
}

// *dst = max(*dst, max of v over a 256-thread workgroup): one atomic per workgroup, and only
// where it moves the value.  Every thread of the workgroup calls it (it has barriers).
__device__ inline void block_raise_u64(unsigned long long v, unsigned long long* dst) {
    __shared__ unsigned long long s_v[4];
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        const unsigned long long o = __shfl_xor(v, off, 64);
        v = o > v ? o : v;
    }
    if ((threadIdx.x & 63) == 0) s_v[threadIdx.x >> 6] = v;
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < 4; ++w) v = s_v[w] > v ? s_v[w] : v;
        if (v > *(volatile unsigned long long*)dst) atomicMax(dst, v);
    }
    __syncthreads();
}

__device__ inline int64_t wave_scan_max_incl(int64_t v, int lane) {
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        int64_t u = __shfl_up(v, off, 64);
        if (lane >= off) v = imax(v, u);
    }
    return v;
}

// Add this lane's record to bin d (if act) and return its slot among the records of bin d
// counted so far (arbitrary order inside one call).  The lanes sharing the first active lane's
// digit take one atomic together (all of a single-digit wave; most of a skewed one, where one
// hot digit would otherwise serialise on its LDS address), every other lane one of its own.
__device__ inline uint32_t digit_count(uint32_t* bins, uint32_t d, bool act, int lane) {
    const unsigned long long a = __ballot(act);
    if (!a) return 0;
    const int L = __ffsll((long long)a) - 1;
    const uint32_t d0 = __shfl(d, L, 64);
    const bool same = act && d == d0;
    const unsigned long long m = __ballot(same);
    const unsigned long long below = (1ull << lane) - 1;
    uint32_t base = 0;
    if (lane == L) base = atomicAdd(&bins[d0], (uint32_t)__popcll(m));
    base = __shfl(base, L, 64);
    if (same) return base + (uint32_t)__popcll(m & below);
    return act ? atomicAdd(&bins[d], 1u) : 0u;
}

// =============================================================================
// K3a — k_scan: M_j = max lt of changeset j; tiles that may raise in recv().
// A record can raise only if it is flagged (rank == local: DuplicateNode,
// hlc.dart:88-90; millis - wall > 60000: ClockDrift, hlc.dart:92-94) AND its lt
// exceeds the canonical; canonicals never decrease, so lt <= C_0 can never raise.
// =============================================================================
constexpr uint32_t kHotSample = 16;              // tiles_hot counts every 16th tile (one address)

// kEager: rank / millis are loaded with lt instead of after it (one memory round trip per
// tile instead of two) — chosen when the previous call found most tiles above C_0 (streaming
// deltas); otherwise only waves holding such a record load them (the fan-in: ~none do).
// kMillis: the batch carries an explicit millis column (an Hlc whose counter exceeds 0xFFFF);
// without it millis = lt >> 16 and the eager form keeps no millis registers.
__host__ __device__ inline uint64_t ord64(int64_t x) { return (uint64_t)x ^ (1ull << 63); }

// kFrame (the sorted path will run): with rank loaded eagerly, also the frame of the records
// (lt and rank bounds) into misc->fr_*, one set of atomics per workgroup and tile, only where
// it moves a bound (a stale read of a bound never makes a needed atomic look useless)
// kHist (the sorted path's level-1 histogram fused into the scan, single ctx, one window): the
// keys are read with lt and counted per level-1 partition tile (never straddling a changeset) into
// hist[ptb[j] + u][256] — what k_part_hist<true> would write with every changeset applied (tiles of
// changesets >= stop are zeroed once stop is known).  A workgroup takes kHistSub scan tiles per step:
// one level-1 tile of 28672 records, or two of 14336 (ScanHist::htile) — then the boundary falls in the
// middle of the step's fourth scan tile, where a thread's record groups split cleanly (whole 1024- /
// 256-record groups, so every record of one load instruction counts into the same histogram).
constexpr uint32_t kHistSub = 7;                 // scan tiles per workgroup step of the fused histogram

// The level-1 digit of a key id.  One ctx: (k >> shift) & 255 over the ids k < cap.  The routed
// partition of a sharded order-free merge (comm_path.inc, route_l1) partitions GLOBAL key ids of G = 2^gsh
// ranks straight into their owners' level-1 buckets: owner o = k & (G - 1), slot k >> gsh (< cap, the
// shard capacity), digit (o << dsh) | (slot >> shift) — every owner's 2^dsh digits, owner-major.  The
// identity map {0, 8} is the one-ctx digit.
struct KeyMap {
    uint32_t gsh;
    uint32_t dsh;
};
__host__ __device__ inline uint32_t km_digit(KeyMap m, uint32_t k, uint32_t shift) {
    return ((((k & ((1u << m.gsh) - 1u)) << m.dsh) | ((k >> m.gsh) >> shift)) & 255u);
}

struct ScanHist {
    const uint32_t* key;
    const uint32_t* ptb;        // [R + 1] first partition tile of changeset j
    uint64_t cap;
    uint32_t shift;
    uint32_t* hist;
    KeyMap km{0u, 8u};
    uint32_t htile = kHistSub * kTile;      // level-1 tile (records): the step's 28672, or 14336 (two per step)
};

// kVec: a thread's records are 4 groups of 4 consecutive ones (lt read with two 16-B loads per
// group, keys with one) instead of 16 strided ones; every per-tile result is order-free.
template <bool kEager, bool kMillis, bool kFrame, bool kHist, bool kVec>
__device__ __forceinline__ void scan_body(
    const int64_t* __restrict__ lt, const uint32_t* __restrict__ rank,
    const int64_t* __restrict__ millis, const uint64_t* __restrict__ offs,
    const uint32_t* __restrict__ tstart, uint32_t jbase, int64_t c0,
    int64_t wall, uint32_t local_rank,
    int64_t* __restrict__ T, Misc* __restrict__ misc, uint32_t* __restrict__ cand_tile, ScanHist sh, bool jx)
{
    // (kFrame without kEager: the lt frame only — the host declared a rank bound, crdt_set_rank_bound)
    __shared__ int64_t s_max[kScanThreads / 64];
    __shared__ int s_flag[kScanThreads / 64];
    __shared__ unsigned long long s_fr[kFrame ? 5 * (kScanThreads / 64) : 1];
    __shared__ uint32_t s_h[kHist ? 512 : 1];
    static_assert(!kHist || kScanThreads == 256, "one histogram bin per thread");
    // jx (the step-major grid): blockIdx.x is the changeset and blockIdx.y the step, so the workgroups run every
    // changeset's first steps before any changeset's last (shorter) one — fewer, shorter tails when a batch is only
    // a few workgroup rounds deep (cfg3: 4 steps of up to 7 tiles per changeset on ~1024 resident workgroups)
    const uint32_t j = jbase + (jx ? blockIdx.x : blockIdx.y);
    const uint64_t beg = offs[j], end = offs[j + 1];
    const uint32_t t0 = tstart[j], nt = tstart[j + 1] - t0;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    constexpr uint32_t kStep = kHist ? kHistSub : 1u;
    const uint32_t ustride = jx ? gridDim.y : gridDim.x;
    for (uint32_t u = jx ? blockIdx.y : blockIdx.x; u * kStep < nt; u += ustride) {
      if (kHist) {
        s_h[threadIdx.x] = 0;
        s_h[256 + threadIdx.x] = 0;
        __syncthreads();
      }
      const uint32_t te = std::min<uint32_t>(u * kStep + kStep, nt);
      for (uint32_t t = u * kStep; t < te; ++t) {
        const uint64_t base = beg + (uint64_t)t * kTile;
        int64_t m = INT64_MIN;
        int f = 0;
        int64_t v[kScanItems];
        uint32_t rk[kEager ? kScanItems : 1];
        int64_t mv[kEager && kMillis ? kScanItems : 1];
        uint32_t kk[kHist ? kScanItems : 1];
        auto idx = [&](int q) -> uint64_t {
            return kVec ? base + (uint64_t)(q >> 2) * (4 * kScanThreads) + threadIdx.x * 4u + (q & 3)
                        : base + (uint64_t)q * kScanThreads + threadIdx.x;
        };
        bool vec_done[kVec ? kScanItems / 4 : 1];
#pragma unroll
        for (int g = 0; g < (kVec ? kScanItems / 4 : 0); ++g) {
            const uint64_t i0 = idx(4 * g);
            vec_done[kVec ? g : 0] = i0 + 4 <= end;
            if (i0 + 4 <= end) {
                const u32x4u a = *reinterpret_cast<const u32x4u*>(lt + i0);
                const u32x4u b = *reinterpret_cast<const u32x4u*>(lt + i0 + 2);
                v[4 * g] = (int64_t)(((uint64_t)a.y << 32) | a.x); v[4 * g + 1] = (int64_t)(((uint64_t)a.w << 32) | a.z);
                v[4 * g + 2] = (int64_t)(((uint64_t)b.y << 32) | b.x); v[4 * g + 3] = (int64_t)(((uint64_t)b.w << 32) | b.z);
                if (kHist) {
                    const u32x4u kv = *reinterpret_cast<const u32x4u*>(sh.key + i0);
                    kk[kHist ? 4 * g : 0] = kv.x; kk[kHist ? 4 * g + 1 : 0] = kv.y;
                    kk[kHist ? 4 * g + 2 : 0] = kv.z; kk[kHist ? 4 * g + 3 : 0] = kv.w;
                }
                if (kEager) {     // (round 6: the ranks in 16-B loads too — the sharded scan's 4-B loads cost it)
                    const u32x4u rv = *reinterpret_cast<const u32x4u*>(rank + i0);
                    rk[kEager ? 4 * g : 0] = rv.x; rk[kEager ? 4 * g + 1 : 0] = rv.y;
                    rk[kEager ? 4 * g + 2 : 0] = rv.z; rk[kEager ? 4 * g + 3 : 0] = rv.w;
                }
            }
        }
#pragma unroll
        for (int q = 0; q < kScanItems; ++q) {
            const uint64_t i = idx(q);
            const bool vd = kVec && vec_done[kVec ? q >> 2 : 0];
            if (!vd) {
                v[q] = i < end ? lt[i] : INT64_MIN;
                if (kHist) kk[kHist ? q : 0] = i < end ? __builtin_nontemporal_load(sh.key + i) : UINT32_MAX;
            }
            if (kEager) {
                if (!vd) rk[kEager ? q : 0] = i < end ? rank[i] : 0u;
                if (kMillis) mv[kMillis ? q : 0] = (millis && i < end) ? millis[i] : 0;
            }
            m = imax(m, v[q]);
        }
        if (kHist) {
            const uint32_t tb = (t - u * kStep) * (uint32_t)kTile;      // this scan tile inside the step
#pragma unroll
            for (int q = 0; q < kScanItems; ++q) {
                const uint32_t k = kk[kHist ? q : 0];
                // the record's level-1 tile of the step: the same for the whole workgroup at a given q
                // (its group / stride base decides; the thread offset stays below the 1024 / 256 grain)
                const uint32_t gb = kVec ? (uint32_t)(q >> 2) * (4u * kScanThreads) : (uint32_t)q * kScanThreads;
                digit_count(s_h + (tb + gb >= sh.htile ? 256u : 0u), km_digit(sh.km, k, sh.shift),
                            (k >> sh.km.gsh) < sh.cap, lane);
            }
        }
        // rank / millis matter only for records above C0 (the only ones recv() can raise on)
#pragma unroll
        for (int q = 0; q < kScanItems; ++q) {
            if (v[q] > c0) {
                const uint64_t i = idx(q);
                const int64_t ms = (kMillis && millis) ? (kEager ? mv[kEager && kMillis ? q : 0] : millis[i])
                                                       : (v[q] >> kShift);
                const uint32_t r = kEager ? rk[kEager ? q : 0] : rank[i];
                f |= (r == local_rank) | (wsub(ms, wall) > kMaxDrift);
            }
        }
        unsigned long long flo = 0, fhi = 0, frl = 0, frh = 0;   // max-accumulators (0: none)
        uint32_t fcm = 0;                                          // max lt & 0xFFFF (the compact frame)
        if (kFrame) {
#pragma unroll
            for (int q = 0; q < kScanItems; ++q) {
                const uint64_t i = idx(q);
                if (i < end) {
                    const uint64_t o = ord64(v[q]);
                    flo = ~o > flo ? ~o : flo;
                    fhi = o > fhi ? o : fhi;
                    fcm = std::max<uint32_t>(fcm, (uint32_t)v[q] & 0xFFFFu);
                    if (kEager) {
                        const uint32_t r = rk[kEager ? q : 0];
                        frl = (uint32_t)~r > frl ? (uint32_t)~r : frl;
                        frh = r > frh ? r : frh;
                    }
                }
            }
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) {
                const unsigned long long a = __shfl_xor(flo, off, 64), b = __shfl_xor(fhi, off, 64);
                const unsigned long long c = __shfl_xor(frl, off, 64), d = __shfl_xor(frh, off, 64);
                flo = a > flo ? a : flo; fhi = b > fhi ? b : fhi; frl = c > frl ? c : frl; frh = d > frh ? d : frh;
                fcm = std::max<uint32_t>(fcm, (uint32_t)__shfl_xor(fcm, off, 64));
            }
            if (lane == 0) {
                s_fr[5 * w] = flo; s_fr[5 * w + 1] = fhi; s_fr[5 * w + 2] = frl; s_fr[5 * w + 3] = frh; s_fr[5 * w + 4] = fcm;
            }
        }
        m = wave_max(m);
        const int fw = __any(f) | (m > c0 ? 2 : 0);
        if (lane == 0) { s_max[w] = m; s_flag[w] = fw; }
        __syncthreads();
        if (threadIdx.x == 0) {
            if (kFrame) {
                unsigned long long fc = fcm;
                for (int k = 1; k < kScanThreads / 64; ++k) {
                    flo = s_fr[5 * k] > flo ? s_fr[5 * k] : flo;
                    fhi = s_fr[5 * k + 1] > fhi ? s_fr[5 * k + 1] : fhi;
                    frl = s_fr[5 * k + 2] > frl ? s_fr[5 * k + 2] : frl;
                    frh = s_fr[5 * k + 3] > frh ? s_fr[5 * k + 3] : frh;
                    fc = s_fr[5 * k + 4] > fc ? s_fr[5 * k + 4] : fc;
                }
                if (fc > *(volatile unsigned long long*)&misc->fr_cmax) atomicMax(&misc->fr_cmax, fc);
                if (flo > *(volatile unsigned long long*)&misc->fr_lo) atomicMax(&misc->fr_lo, flo);
                if (fhi > *(volatile unsigned long long*)&misc->fr_hi) atomicMax(&misc->fr_hi, fhi);
                if ((uint32_t)frl > *(volatile uint32_t*)&misc->fr_rlo) atomicMax(&misc->fr_rlo, (uint32_t)frl);
                if ((uint32_t)frh > *(volatile uint32_t*)&misc->fr_rhi) atomicMax(&misc->fr_rhi, (uint32_t)frh);
            }
            int64_t tm = s_max[0];
            int tf = s_flag[0];
            for (int k = 1; k < kScanThreads / 64; ++k) { tm = imax(tm, s_max[k]); tf |= s_flag[k]; }
            T[t0 + t] = tm;
            if (tf & 1) {
                const uint32_t c = atomicAdd(&misc->cand_count, 1u);
                cand_tile[c] = t0 + t;
            }
            if ((tf & 2) && ((t0 + t) & (kHotSample - 1)) == 0) atomicAdd(&misc->tiles_hot, 1u);   // sampled
        }
        __syncthreads();
      }
      if (kHist) {
        const uint32_t np = sh.ptb[j + 1] - sh.ptb[j];                  // the changeset's level-1 tiles
        const uint32_t per = sh.htile < kHistSub * kTile ? 2u : 1u;
        for (uint32_t h = 0; h < per; ++h)
            if (u * per + h < np)
                sh.hist[(uint64_t)(sh.ptb[j] + u * per + h) * 256 + threadIdx.x] = s_h[h * 256 + threadIdx.x];
      }
    }
}

template <bool kEager, bool kMillis = true, bool kFrame = false, bool kHist = false, bool kVec = false>
__global__ __launch_bounds__(kScanThreads) void k_scan(
    const int64_t* __restrict__ lt, const uint32_t* __restrict__ rank,
    const int64_t* __restrict__ millis, const uint64_t* __restrict__ offs,
    const uint32_t* __restrict__ tstart, uint32_t jbase, int64_t c0,
    int64_t wall, uint32_t local_rank,
    int64_t* __restrict__ T, Misc* __restrict__ misc, uint32_t* __restrict__ cand_tile, ScanHist sh, bool jx = false)
{
    scan_body<kEager, kMillis, kFrame, kHist, kVec>(lt, rank, millis, offs, tstart, jbase, c0, wall, local_rank, T, misc,
                                                    cand_tile, sh, jx);
}

// M_j = max of changeset j's tile maxima (INT64_MIN when empty).  One block per changeset
// (grid-stride): no same-address atomics, so a single 10M-record changeset costs what
// 1024 small ones do.
__global__ __launch_bounds__(256) void k_tmax(const int64_t* __restrict__ T, const uint32_t* __restrict__ tstart,
                                              uint32_t R, long long* __restrict__ M)
{
    __shared__ int64_t s_max[4];
    for (uint32_t j = blockIdx.x; j < R; j += gridDim.x) {
        const uint32_t a = tstart[j], b = tstart[j + 1];
        int64_t m = INT64_MIN;
        for (uint32_t t = a + threadIdx.x; t < b; t += 256) m = imax(m, T[t]);
        m = wave_max(m);
        if ((threadIdx.x & 63) == 0) s_max[threadIdx.x >> 6] = m;
        __syncthreads();
        if (threadIdx.x == 0) M[j] = (long long)imax(imax(s_max[0], s_max[1]), imax(s_max[2], s_max[3]));
        __syncthreads();
    }
}

// =============================================================================
// K3b — k_clock (one workgroup).  Sequential merges give (crdt.dart:82, 93)
//   R_j = max(C_{j-1}, M_j)               canonical after the recv loop
//   C_j = send(R_j) = max(R_j + 1, W)     W = wall << 16   (hlc.dart:51-74)
// so D_j = C_j - j = max(C_0, max_{k<=j}(max(M_k + 1, W) - k)) — a prefix max.
// Also finds the first changeset whose send() raises (drift, then overflow).
// =============================================================================
__device__ inline bool send_fails(int64_t r, int64_t wall) {
    const int64_t m = r >> kShift, c = r & kMaxCounter;
    const int64_t mn = imax(m, wall);
    const int64_t cn = (m == mn) ? c + 1 : 0;
    return wsub(mn, wall) > kMaxDrift || cn > kMaxCounter;
}

// kTiles (small batches: <= kClockTilesMax tiles, R <= kClockRMax): M_j is reduced here from the
// scan's tile maxima T (LDS max per changeset) instead of by a separate k_tmax launch.
constexpr uint32_t kClockTilesMax = 8192;         // <= 8 tiles per thread (cfg3's 24K tiles: k_tmax is faster)
constexpr uint32_t kClockRMax = 2048;

template <bool kTiles>
__global__ __launch_bounds__(1024) void k_clock(
    const long long* __restrict__ M, const int64_t* __restrict__ T, const uint32_t* __restrict__ tstart,
    uint32_t R, int64_t wall, int64_t c0,
    int64_t* __restrict__ Cprev, int64_t* __restrict__ Rj, int64_t* __restrict__ Cj,
    long long* __restrict__ event)
{
    __shared__ int64_t s_wave[16];
    __shared__ uint32_t s_first;
    __shared__ long long s_M[kTiles ? kClockRMax : 1];
    __shared__ uint32_t s_ts[kTiles ? kClockRMax + 1 : 1];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int64_t W = (int64_t)((uint64_t)wall << kShift);
    int64_t carry = c0;                       // D_0 = C_0
    uint32_t first = UINT32_MAX;
    if (tid == 0) {
        s_first = UINT32_MAX;
        event[0] = kEvNone; event[1] = INT64_MIN; event[2] = 0; event[3] = INT64_MIN;   // = k_event_init
    }
    if (kTiles) {
        for (uint32_t j = tid; j <= R; j += 1024) {
            s_ts[j] = tstart[j];
            if (j < R) s_M[j] = INT64_MIN;
        }
        __syncthreads();
        const uint32_t nt = s_ts[R];
        for (uint32_t u = tid; u < nt; u += 1024) {
            const int64_t tu = T[u];
            uint32_t lo = 0, hi = R;                 // changeset of tile u: largest j with tstart[j] <= u
            while (hi - lo > 1) {
                const uint32_t mid = (lo + hi) >> 1;
                if (s_ts[mid] <= u) lo = mid; else hi = mid;
            }
            atomicMax(&s_M[lo], (long long)tu);
        }
    }
    __syncthreads();
    for (uint32_t base = 0; base < R; base += 1024) {
        const uint32_t j = base + tid;
        const bool valid = j < R;
        const int64_t jj = (int64_t)j + 1;
        const int64_t mj = valid ? (int64_t)(kTiles ? s_M[j] : M[j]) : INT64_MIN;
        const bool has = mj != INT64_MIN;
        const int64_t b = has ? imax(mj + 1, W) : W;
        const int64_t key = valid ? b - jj : INT64_MIN;
        int64_t incl = wave_scan_max_incl(key, lane);
        if (lane == 63) s_wave[w] = incl;
        __syncthreads();
        if (w == 0) {
            int64_t x = lane < 16 ? s_wave[lane] : INT64_MIN;
#pragma unroll
            for (int off = 1; off < 16; off <<= 1) {
                int64_t u = __shfl_up(x, off, 64);
                if (lane >= off) x = imax(x, u);
            }
            if (lane < 16) s_wave[lane] = x;
        }
        __syncthreads();
        const int64_t wprev = w > 0 ? s_wave[w - 1] : INT64_MIN;
        int64_t excl = __shfl_up(incl, 1, 64);
        if (lane == 0) excl = INT64_MIN;
        excl = imax(excl, wprev);
        incl = imax(incl, wprev);
        const int64_t total = s_wave[15];
        const int64_t cprev = imax(carry, excl) + (jj - 1);
        const int64_t ccur = imax(carry, incl) + jj;
        if (valid) {
            const int64_t r = has ? imax(cprev, mj) : cprev;
            Cprev[j] = cprev;
            Rj[j] = r;
            Cj[j] = ccur;
            if (send_fails(r, wall)) first = first < j ? first : j;
        }
        carry = imax(carry, total);
        __syncthreads();
    }
    if (first != UINT32_MAX) atomicMin(&s_first, first);
    __syncthreads();
    if (tid == 0 && s_first != UINT32_MAX)
        atomicMin(event, (long long)(((int64_t)s_first << kLowBits) | kLowMask));
}

// Publish the recv-failure details of the global first event if this ctx holds
// it: event[1] = canonical at the failure, event[2] = kind, event[3] = Hlc.millis.
// (Every thread of the workgroup calls it.)
__device__ void resolve_local_body(const Misc* __restrict__ misc, const long long* __restrict__ cand_key,
                                   const int64_t* __restrict__ cand_P, const uint32_t* __restrict__ cand_kind,
                                   const int64_t* __restrict__ cand_ms, long long* __restrict__ event)
{
    const long long ev = event[0];
    __syncthreads();                           // every thread read event[0] before it is rewritten
    if (threadIdx.x == 0) { event[1] = INT64_MIN; event[2] = 0; event[3] = INT64_MIN; }
    __syncthreads();
    if (ev == kEvNone || (ev & kLowMask) == kLowMask) return;
    const uint32_t n = misc->cand_count;
    for (uint32_t c = threadIdx.x; c < n; c += blockDim.x) {
        if (cand_key[c] == ev) {
            event[1] = cand_P[c];
            event[2] = cand_kind[c];
            event[3] = cand_ms[c];
        }
    }
}

__global__ __launch_bounds__(256) void k_resolve_local(
    const Misc* __restrict__ misc, const long long* __restrict__ cand_key,
    const int64_t* __restrict__ cand_P, const uint32_t* __restrict__ cand_kind,
    const int64_t* __restrict__ cand_ms, long long* __restrict__ event)
{
    resolve_local_body(misc, cand_key, cand_P, cand_kind, cand_ms, event);
}

// =============================================================================
// K3d — k_resolve: stop point, status, final canonical (crdt.dart:80-93 order:
// every recv of changeset j, then its store, then its send).  Thread 0 only.
// =============================================================================
__device__ void resolve_body(const long long* __restrict__ event, uint32_t R, int64_t wall,
                             int64_t c0, const int64_t* __restrict__ Rj, const int64_t* __restrict__ Cj,
                             Misc* __restrict__ misc)
{
    crdt_result res = {};
    res.exc_index = UINT64_MAX;
    const int64_t ev = event[0];
    uint32_t stop;
    if (ev == kEvNone) {
        stop = R;
        res.status = CRDT_OK;
        res.canonical_lt = R ? Cj[R - 1] : c0;
    } else {
        const uint32_t j = (uint32_t)(ev >> kLowBits);
        const int64_t low = ev & kLowMask;
        res.exc_changeset = j;
        if (low == kLowMask) {                       // send() after storing changeset j
            stop = j + 1;
            const int64_t r = Rj[j];
            const int64_t m = r >> kShift, c = r & kMaxCounter;
            const int64_t mn = imax(m, wall);
            res.canonical_lt = r;
            if (wsub(mn, wall) > kMaxDrift) {
                res.status = CRDT_CLOCK_DRIFT;
                res.drift_ms = wsub(mn, wall);
            } else {
                res.status = CRDT_OVERFLOW;
                res.counter = c + 1;
            }
        } else {                                     // recv() inside changeset j
            stop = j;
            res.exc_index = (uint64_t)low;
            res.canonical_lt = event[1];
            res.status = (int32_t)event[2];
            if (res.status == CRDT_CLOCK_DRIFT) res.drift_ms = wsub(event[3], wall);
        }
    }
    res.n_stored = stop;
    misc->stop = stop;
    misc->result = res;
}

__global__ void k_resolve(const long long* __restrict__ event, uint32_t R, int64_t wall,
                          int64_t c0, const int64_t* __restrict__ Rj, const int64_t* __restrict__ Cj,
                          Misc* __restrict__ misc)
{
    if (threadIdx.x == 0) resolve_body(event, R, wall, c0, Rj, Cj, misc);
}

// =============================================================================
// K3c — k_verify: for each candidate tile, the first record i (in iteration
// order) with flag(i) && lt_i > max(C_{j-1}, lt of every earlier record of j),
// i.e. the first Hlc.recv that throws (hlc.dart:85-94).  One wave per tile,
// ordered 64-record rounds with a shuffle prefix max.  Rare path.
// =============================================================================
// kFuse (single-ctx crdt_merge): the last workgroup to finish also runs k_resolve_local and
// k_resolve (Rj / Cj / c0 only read then), saving two launches per merge call.
template <bool kFuse>
__global__ __launch_bounds__(64) void k_verify(
    const int64_t* __restrict__ lt, const uint32_t* __restrict__ rank,
    const int64_t* __restrict__ millis, const uint64_t* __restrict__ offs,
    const uint32_t* __restrict__ tstart, uint32_t R, const int64_t* __restrict__ T,
    const int64_t* __restrict__ Cprev, int64_t wall, uint32_t local_rank,
    Misc* __restrict__ misc, const uint32_t* __restrict__ cand_tile,
    long long* __restrict__ cand_key, int64_t* __restrict__ cand_P,
    uint32_t* __restrict__ cand_kind, int64_t* __restrict__ cand_ms,
    const long long* __restrict__ pbase, const unsigned long long* __restrict__ ibase,
    long long* __restrict__ event, int64_t c0, const int64_t* __restrict__ Rj, const int64_t* __restrict__ Cj,
    uint32_t tile_recs)
{
    // tile_recs: records per tile of T / tstart / cand_tile (kTile, the scan's tiles).
    // pbase / ibase (optional): this ctx holds only a PART of changeset j, preceded in
    // its iteration order by records of other ranks whose max lt is pbase[j] and whose
    // count is ibase[j] (key-sharded "parts" protocol, crdt_amd/dist.py).
    const int lane = threadIdx.x;
    const uint32_t n = misc->cand_count;
    for (uint32_t c = blockIdx.x; c < n; c += gridDim.x) {
        const uint32_t gt = cand_tile[c];
        uint32_t lo = 0, hi = R;                     // largest j with tstart[j] <= gt
        while (hi - lo > 1) {
            const uint32_t mid = (lo + hi) >> 1;
            if (tstart[mid] <= gt) lo = mid; else hi = mid;
        }
        const uint32_t j = lo;
        const uint32_t t = gt - tstart[j];
        int64_t P = Cprev[j];
        if (pbase) P = imax(P, (int64_t)pbase[j]);
        for (uint32_t u = tstart[j] + lane; u < gt; u += 64) P = imax(P, T[u]);
        P = wave_max(P);
        const uint64_t base = offs[j] + (uint64_t)t * tile_recs;
        const uint64_t end = std::min<uint64_t>(base + tile_recs, offs[j + 1]);
        bool found = false;
        uint64_t fi = 0;
        int64_t fp = 0, fms = 0;
        uint32_t fkind = 0;
        for (uint64_t i0 = base; i0 < end; i0 += 64) {
            const uint64_t i = i0 + lane;
            const bool in = i < end;
            const int64_t v = in ? lt[i] : INT64_MIN;
            const uint32_t r = in ? rank[i] : 0;
            const int64_t ms = in ? (millis ? millis[i] : (v >> kShift)) : 0;
            const bool dup = in && r == local_rank;
            const bool drift = in && wsub(ms, wall) > kMaxDrift;
            const int64_t incl = wave_scan_max_incl(v, lane);
            int64_t excl = __shfl_up(incl, 1, 64);
            if (lane == 0) excl = INT64_MIN;
            excl = imax(excl, P);
            const bool viol = (dup || drift) && v > excl;
            const unsigned long long b = __ballot(viol);
            if (b) {
                const int L = __ffsll((long long)b) - 1;
                fi = __shfl(i, L, 64);
                fp = __shfl(excl, L, 64);
                fms = __shfl(ms, L, 64);
                fkind = __shfl(dup ? (uint32_t)CRDT_DUPLICATE_NODE : (uint32_t)CRDT_CLOCK_DRIFT, L, 64);
                found = true;
                break;
            }
            P = imax(P, __shfl(incl, 63, 64));
        }
        if (lane == 0) {
            if (found) {
                const int64_t idx = (int64_t)(fi - offs[j]) + (ibase ? (int64_t)ibase[j] : 0);
                const long long key = (long long)(((int64_t)j << kLowBits) | idx);
                cand_key[c] = key;
                cand_P[c] = fp;
                cand_kind[c] = fkind;
                cand_ms[c] = fms;
                atomicMin(event, key);
            } else {
                cand_key[c] = kEvNone;
            }
        }
    }
    if (kFuse) {
        __shared__ uint32_t s_last;
        __threadfence();                       // this workgroup's candidate words and event min
        if (lane == 0) s_last = atomicAdd(&misc->vdone, 1u) == gridDim.x - 1;
        __syncthreads();
        if (!s_last) return;
        __threadfence();                       // acquire: every other workgroup's writes
        resolve_local_body(misc, cand_key, cand_P, cand_kind, cand_ms, event);
        __syncthreads();
        __threadfence_block();
        if (lane == 0) resolve_body(event, R, wall, c0, Rj, Cj, misc);
    }
}

// =============================================================================
// K2 — k_apply: one changeset (crdt.dart:83-90).  Winner <=> local row invisible
// (mod < 0, incl. never written) or local.hlc < remote.hlc in (lt, rank) order;
// equal keeps local.  Each thread owns 4 consecutive records of a 4-aligned
// group: 16-B stream loads, then all four row gathers (one dwordx4 each) are in
// flight before any is used — no per-record branch around a load.
// (A blocked 4-consecutive-records layout with dwordx4 stream loads measured the
// same on the fan-in and 20 % slower on cfg2, whose new ids are consecutive.)
// =============================================================================
template <int kApplyItems>
__global__ __launch_bounds__(kApplyThreads) void k_apply(
    const uint32_t* __restrict__ key, const int64_t* __restrict__ lt,
    const uint32_t* __restrict__ rank, const uint32_t* __restrict__ val, uint64_t beg,
    uint64_t end, uint32_t j, Table table, uint64_t cap,
    const int64_t* __restrict__ Rj, Misc* __restrict__ misc, uint8_t* __restrict__ flags)
{
    if (j >= misc->stop || (misc->err & 1u)) return;      // uniform: past the stop point / a bad key id
    const int64_t stamp = Rj[j];
    // striped: record q of this thread = base + q * 256 + tid, so a wave's q-th
    // access covers 64 consecutive records (coalesced streams; consecutive new ids
    // give coalesced rows)
    const uint64_t base = beg + (uint64_t)blockIdx.x * (kApplyThreads * kApplyItems) + threadIdx.x;
    uint32_t k[kApplyItems], r[kApplyItems], v[kApplyItems];
    int64_t l[kApplyItems];
    bool in[kApplyItems];
#pragma unroll
    for (int q = 0; q < kApplyItems; ++q) {
        const uint64_t i = base + (uint64_t)q * kApplyThreads;
        in[q] = i < end;
        const uint64_t ii = in[q] ? i : beg;             // always a valid address, no branch
        k[q] = __builtin_nontemporal_load(key + ii);
        l[q] = __builtin_nontemporal_load(lt + ii);
        r[q] = __builtin_nontemporal_load(rank + ii);
        v[q] = __builtin_nontemporal_load(val + ii);
    }
    uint4 h[kApplyItems];
    bool ok[kApplyItems];
#pragma unroll
    for (int q = 0; q < kApplyItems; ++q) {              // all gathers in flight, one dwordx4 each
        ok[q] = in[q] && k[q] < cap;
        const uint64_t row = ok[q] ? k[q] : 0;
        h[q] = load_hot(table, row);
    }
    int npres = 0, nwon = 0;
    bool bad = false;
#pragma unroll
    for (int q = 0; q < kApplyItems; ++q) {
        const int64_t llt = (int64_t)(((uint64_t)h[q].y << 32) | h[q].x);
        const bool present = (int32_t)h[q].w >= 0;
        const bool win = ok[q] && (!present || l[q] > llt || (l[q] == llt && r[q] > h[q].z));
        npres += ok[q] && present;
        nwon += win;
        bad |= in[q] && !ok[q];
        if (win) store_row(table, k[q], l[q], r[q], v[q], stamp);
        if (flags && in[q]) flags[base + (uint64_t)q * kApplyThreads] = win ? 1 : 0;
    }
    if (__any(bad) && (threadIdx.x & 63) == 0) atomicOr(&misc->err, 1u);
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        npres += __shfl_xor(npres, off, 64);
        nwon += __shfl_xor(nwon, off, 64);
    }
    if ((threadIdx.x & 63) == 0) {
        const int slot = (blockIdx.x * (kApplyThreads / 64) + (threadIdx.x >> 6)) & (kCounterSlots - 1);
        if (npres) atomicAdd(&misc->present[slot], (unsigned long long)npres);
        if (nwon) atomicAdd(&misc->won[slot], (unsigned long long)nwon);
    }
}

#include "sorted_path.inc"

// =============================================================================
// Routing (key-sharded ctx, comm_path.inc): partition this rank's part of every
// changeset by owner rank key % G into per-(owner, changeset) chunks of the send
// columns, owner-major then changeset order; slot = key / G.  Order inside a chunk is
// free (keys are distinct within a changeset, so K2 / the resolve do not depend on
// it); the optional perm column gives each sent record's index in the batch (win
// flags come back through it).  counts / cursors: [G][R] words.
// =============================================================================
constexpr int kRouteMaxRanks = 1024;

__global__ __launch_bounds__(kScanThreads) void k_route_count(
    const uint32_t* __restrict__ key, const uint64_t* __restrict__ offs, const uint32_t* __restrict__ tstart,
    uint32_t jbase, uint32_t R, uint32_t G, unsigned long long* __restrict__ counts)
{
    __shared__ uint32_t s_cnt[kRouteMaxRanks];
    const uint32_t j = jbase + blockIdx.y;
    const uint64_t beg = offs[j], end = offs[j + 1];
    const uint32_t nt = tstart[j + 1] - tstart[j];
    for (uint32_t t = blockIdx.x; t < nt; t += gridDim.x) {
        for (uint32_t d = threadIdx.x; d < G; d += kScanThreads) s_cnt[d] = 0;
        __syncthreads();
        const uint64_t base = beg + (uint64_t)t * kTile;
        uint32_t k[kScanItems];
#pragma unroll
        for (int q = 0; q < kScanItems; ++q) {          // every load in flight before the first atomic
            const uint64_t i = base + (uint64_t)q * kScanThreads + threadIdx.x;
            k[q] = i < end ? __builtin_nontemporal_load(key + i) : 0u;
        }
#pragma unroll
        for (int q = 0; q < kScanItems; ++q) {
            const uint64_t i = base + (uint64_t)q * kScanThreads + threadIdx.x;
            if (i < end) atomicAdd(&s_cnt[k[q] % G], 1u);
        }
        __syncthreads();
        for (uint32_t d = threadIdx.x; d < G; d += kScanThreads)
            if (s_cnt[d]) atomicAdd(&counts[(uint64_t)d * R + j], (unsigned long long)s_cnt[d]);
        __syncthreads();
    }
}

// Destination columns of routed records: {slot, lt (or the packed key), rank (unpacked only), val}.
struct RouteCols {
    uint32_t* slot;
    int64_t* lt;
    uint32_t* rank;
    uint32_t* val;
};

// The wire format, decided on the device from the all-gathered frame (Misc::fr_*, k_shard_combine):
// when the global record frame fits the sorted path's packed key (and frame_on), a routed record is
// 16 B {slot, packed (lt, rank, window changeset) in lt, val} instead of 20 B (rank unused).  The host
// reaches the same decision from the same words (frame_of) once it has read them back.
__device__ inline bool route_frame(const Misc* fm, uint32_t frame_on, uint32_t R, PackFrame* pf) {
    *pf = make_frame(fm->fr_lo, fm->fr_hi, fm->fr_rlo, fm->fr_rhi, R);
    return frame_on && pf->ok;
}

// Records for owner `me` (this rank's own chunk) go straight into the receive columns `own` at
// their receive positions (the cursors of row me are receive positions: k_route_plan), so the apply
// reads them in place; own.slot == nullptr: every owner's records go to `send`.
__global__ __launch_bounds__(kScanThreads) void k_route_scatter(
    const uint32_t* __restrict__ key, const int64_t* __restrict__ lt, const uint32_t* __restrict__ rank,
    const uint32_t* __restrict__ val, const uint64_t* __restrict__ offs, const uint32_t* __restrict__ tstart,
    uint32_t jbase, uint32_t R, uint32_t G, unsigned long long* __restrict__ cursor, RouteCols send,
    RouteCols own, uint32_t me, uint64_t* __restrict__ o_perm, const Misc* __restrict__ fm, uint32_t frame_on)
{
    PackFrame pf;
    const bool pk = route_frame(fm, frame_on, R, &pf);
    if (fm->route_own & 2) return;                   // a bad plan (k_route_plan): write nothing
    if (!(fm->route_own & 1)) own.slot = nullptr;
    __shared__ uint32_t s_cnt[kRouteMaxRanks];
    __shared__ unsigned long long s_base[kRouteMaxRanks];
    const uint32_t j = jbase + blockIdx.y;
    const uint64_t beg = offs[j], end = offs[j + 1];
    const uint32_t nt = tstart[j + 1] - tstart[j];
    for (uint32_t t = blockIdx.x; t < nt; t += gridDim.x) {
        for (uint32_t d = threadIdx.x; d < G; d += kScanThreads) s_cnt[d] = 0;
        __syncthreads();
        const uint64_t base = beg + (uint64_t)t * kTile;
        uint32_t k[kScanItems], dst[kScanItems], pos[kScanItems];
#pragma unroll
        for (int q = 0; q < kScanItems; ++q) {
            const uint64_t i = base + (uint64_t)q * kScanThreads + threadIdx.x;
            k[q] = i < end ? __builtin_nontemporal_load(key + i) : 0u;
        }
#pragma unroll
        for (int q = 0; q < kScanItems; ++q) {
            const uint64_t i = base + (uint64_t)q * kScanThreads + threadIdx.x;
            dst[q] = k[q] % G;
            pos[q] = i < end ? atomicAdd(&s_cnt[dst[q]], 1u) : 0u;
        }
        __syncthreads();
        for (uint32_t d = threadIdx.x; d < G; d += kScanThreads)
            s_base[d] = s_cnt[d] ? atomicAdd(&cursor[(uint64_t)d * R + j], (unsigned long long)s_cnt[d]) : 0;
        __syncthreads();
#pragma unroll
        for (int q = 0; q < kScanItems; ++q) {
            const uint64_t i = base + (uint64_t)q * kScanThreads + threadIdx.x;
            if (i < end) {
                const uint64_t o = s_base[dst[q]] + pos[q];
                const RouteCols& oc = own.slot && dst[q] == me ? own : send;
                oc.slot[o] = k[q] / G;
                const int64_t l = __builtin_nontemporal_load(lt + i);
                const uint32_t r = __builtin_nontemporal_load(rank + i);
                if (pk) {
                    oc.lt[o] = (int64_t)pack_record(pf, l, r, j % pf.jwin);
                } else {
                    oc.lt[o] = l;
                    oc.rank[o] = r;
                }
                oc.val[o] = __builtin_nontemporal_load(val + i);
                if (o_perm) o_perm[o] = i;
            }
        }
        __syncthreads();
    }
}

// Wave-aggregated slot in a small LDS counter array: the lanes of a wave holding the same
// destination d (< 2^nbits) find each other by ballots over d's bits; the lowest one adds the group's
// size with one LDS atomic, every lane gets base + its rank in the group (k_route_*<.., kAgg>: with
// G <= 8 owners a wave's 64 lanes otherwise hit at most 8 addresses with 64 atomics).
__device__ inline uint32_t agg_slot(uint32_t* cnt, uint32_t d, bool act, uint32_t nbits, bool want_pos) {
    const int lane = threadIdx.x & 63;
    unsigned long long m = __ballot(act);
    for (uint32_t b = 0; b < nbits; ++b) {
        const bool bit = (d >> b) & 1u;
        const unsigned long long bb = __ballot(act && bit);
        m &= bit ? bb : ~bb;
    }
    if (!act) return 0u;
    const int leader = __ffsll((long long)m) - 1;
    uint32_t base = 0;
    if (lane == leader) base = atomicAdd(&cnt[d], (uint32_t)__popcll(m));
    if (!want_pos) return 0u;
    base = __shfl(base, leader, 64);
    return base + (uint32_t)__popcll(m & ((1ull << lane) - 1));
}

// Vector-load variants of the two routing kernels: a thread's 16 records of a scan tile are 4 groups
// of 4 consecutive ones (16-B key loads; in the scatter also 16-B val / rank and 2 x 16-B lt loads),
// counted with agg_slot.  Same counts; the scatter's output order inside an (owner, changeset)
// run differs, which nothing depends on (keys are distinct inside a changeset; win flags travel
// back through o_perm).
inline uint32_t route_bits(uint32_t G) {              // bits of the largest owner index
    uint32_t b = 0;
    while ((1u << b) < G) ++b;
    return b;
}

__device__ inline uint64_t route_idx(uint64_t base, int q) {
    return base + (uint64_t)(q >> 2) * (4 * kScanThreads) + threadIdx.x * 4u + (q & 3);
}

__global__ __launch_bounds__(kScanThreads) void k_route_count_v(
    const uint32_t* __restrict__ key, const uint64_t* __restrict__ offs, const uint32_t* __restrict__ tstart,
    uint32_t jbase, uint32_t R, uint32_t G, uint32_t nbits, unsigned long long* __restrict__ counts)
{
    __shared__ uint32_t s_cnt[kRouteMaxRanks];
    const uint32_t j = jbase + blockIdx.y;
    const uint64_t beg = offs[j], end = offs[j + 1];
    const uint32_t nt = tstart[j + 1] - tstart[j];
    for (uint32_t t = blockIdx.x; t < nt; t += gridDim.x) {
        for (uint32_t d = threadIdx.x; d < G; d += kScanThreads) s_cnt[d] = 0;
        __syncthreads();
        const uint64_t base = beg + (uint64_t)t * kTile;
        uint32_t k[kScanItems];
#pragma unroll
        for (int g = 0; g < kScanItems / 4; ++g) {
            const uint64_t i0 = route_idx(base, 4 * g);
            if (i0 + 4 <= end) {
                const u32x4u v = *reinterpret_cast<const u32x4u*>(key + i0);
                k[4 * g] = v.x; k[4 * g + 1] = v.y; k[4 * g + 2] = v.z; k[4 * g + 3] = v.w;
            } else {
#pragma unroll
                for (int x = 0; x < 4; ++x) k[4 * g + x] = i0 + x < end ? key[i0 + x] : 0u;
            }
        }
#pragma unroll
        for (int q = 0; q < kScanItems; ++q)
            agg_slot(s_cnt, k[q] % G, route_idx(base, q) < end, nbits, false);
        __syncthreads();
        for (uint32_t d = threadIdx.x; d < G; d += kScanThreads)
            if (s_cnt[d]) atomicAdd(&counts[(uint64_t)d * R + j], (unsigned long long)s_cnt[d]);
        __syncthreads();
    }
}

__global__ __launch_bounds__(kScanThreads) void k_route_scatter_v(
    const uint32_t* __restrict__ key, const int64_t* __restrict__ lt, const uint32_t* __restrict__ rank,
    const uint32_t* __restrict__ val, const uint64_t* __restrict__ offs, const uint32_t* __restrict__ tstart,
    uint32_t jbase, uint32_t R, uint32_t G, uint32_t nbits, unsigned long long* __restrict__ cursor,
    RouteCols send, RouteCols own, uint32_t me, uint64_t* __restrict__ o_perm, const Misc* __restrict__ fm,
    uint32_t frame_on)
{
    PackFrame pf;
    const bool pk = route_frame(fm, frame_on, R, &pf);
    if (fm->route_own & 2) return;                   // a bad plan (k_route_plan): write nothing
    if (!(fm->route_own & 1)) own.slot = nullptr;
    __shared__ uint32_t s_cnt[kRouteMaxRanks];
    __shared__ unsigned long long s_base[kRouteMaxRanks];
    const uint32_t j = jbase + blockIdx.y;
    const uint64_t beg = offs[j], end = offs[j + 1];
    const uint32_t nt = tstart[j + 1] - tstart[j];
    for (uint32_t t = blockIdx.x; t < nt; t += gridDim.x) {
        for (uint32_t d = threadIdx.x; d < G; d += kScanThreads) s_cnt[d] = 0;
        __syncthreads();
        const uint64_t base = beg + (uint64_t)t * kTile;
        uint32_t k[kScanItems], pos[kScanItems];
#pragma unroll
        for (int g = 0; g < kScanItems / 4; ++g) {
            const uint64_t i0 = route_idx(base, 4 * g);
            if (i0 + 4 <= end) {
                const u32x4u v = *reinterpret_cast<const u32x4u*>(key + i0);
                k[4 * g] = v.x; k[4 * g + 1] = v.y; k[4 * g + 2] = v.z; k[4 * g + 3] = v.w;
            } else {
#pragma unroll
                for (int x = 0; x < 4; ++x) k[4 * g + x] = i0 + x < end ? key[i0 + x] : 0u;
            }
        }
#pragma unroll
        for (int q = 0; q < kScanItems; ++q)
            pos[q] = agg_slot(s_cnt, k[q] % G, route_idx(base, q) < end, nbits, true);
        __syncthreads();
        for (uint32_t d = threadIdx.x; d < G; d += kScanThreads)
            s_base[d] = s_cnt[d] ? atomicAdd(&cursor[(uint64_t)d * R + j], (unsigned long long)s_cnt[d]) : 0;
        __syncthreads();
#pragma unroll
        for (int g = 0; g < kScanItems / 4; ++g) {
            const uint64_t i0 = route_idx(base, 4 * g);
            int64_t l[4];
            uint32_t r[4], v[4];
            if (i0 + 4 <= end) {
                const u32x4u a = *reinterpret_cast<const u32x4u*>(lt + i0);
                const u32x4u b = *reinterpret_cast<const u32x4u*>(lt + i0 + 2);
                l[0] = (int64_t)(((uint64_t)a.y << 32) | a.x); l[1] = (int64_t)(((uint64_t)a.w << 32) | a.z);
                l[2] = (int64_t)(((uint64_t)b.y << 32) | b.x); l[3] = (int64_t)(((uint64_t)b.w << 32) | b.z);
                const u32x4u rv = *reinterpret_cast<const u32x4u*>(rank + i0);
                const u32x4u vv = *reinterpret_cast<const u32x4u*>(val + i0);
                r[0] = rv.x; r[1] = rv.y; r[2] = rv.z; r[3] = rv.w;
                v[0] = vv.x; v[1] = vv.y; v[2] = vv.z; v[3] = vv.w;
            } else {
#pragma unroll
                for (int x = 0; x < 4; ++x) {
                    const uint64_t i = i0 + x < end ? i0 + x : beg;
                    l[x] = lt[i]; r[x] = rank[i]; v[x] = val[i];
                }
            }
#pragma unroll
            for (int x = 0; x < 4; ++x) {
                const int q = 4 * g + x;
                const uint64_t i = i0 + x;
                if (i >= end) continue;
                const uint32_t d = k[q] % G;
                const uint64_t o = s_base[d] + pos[q];
                const RouteCols& oc = own.slot && d == me ? own : send;
                oc.slot[o] = k[q] / G;
                if (pk) {
                    oc.lt[o] = (int64_t)pack_record(pf, l[x], r[x], j % pf.jwin);
                } else {
                    oc.lt[o] = l[x];
                    oc.rank[o] = r[x];
                }
                oc.val[o] = v[x];
                if (o_perm) o_perm[o] = i;
            }
        }
        __syncthreads();
    }
}

// Packed routed records back to (lt, rank) columns, for an apply that takes the gather path.
__global__ __launch_bounds__(256) void k_unpack_routed(int64_t* __restrict__ lt, uint32_t* __restrict__ rank,
                                                       uint64_t n, PackFrame pf)
{
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint64_t x = (uint64_t)lt[i];
    lt[i] = pack_lt(pf, x);
    rank[i] = pack_rank(pf, x);
}

// The route plan on the device, from the [G][R] send counts (cnt[d][j]: records of this rank's part
// of changeset j owned by rank d) and the exchanged receive counts (rcv[s][j]: records rank s sends
// here): cursor[d][j] = the first send position of (d, j), send columns owner-major then changeset
// order; with own_in_recv, row `me` instead holds RECEIVE positions — rd[me] (every record received
// from lower ranks) plus the records of this rank's own chunk in earlier changesets — so the
// scatter writes the own chunk where the apply reads it.  One workgroup, chunks of 1024 cells.
// own_in_recv is honoured only when every record this rank receives fits the receive columns'
// capacity recv_cap (Misc::route_own says whether it was); the scatter reads that word.
__global__ __launch_bounds__(1024) void k_route_plan(const unsigned long long* __restrict__ cnt,
                                                     const unsigned long long* __restrict__ rcv, uint32_t G,
                                                     uint32_t R, uint32_t me, uint32_t own_in_recv,
                                                     uint64_t recv_cap, uint64_t n_send,
                                                     unsigned long long* __restrict__ cursor, Misc* __restrict__ misc)
{
    __shared__ unsigned long long s_wave[16];
    __shared__ unsigned long long s_carry, s_rd;
    const uint32_t tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const uint64_t cells = (uint64_t)G * R;
    // (starts with a barrier: every thread has read the previous scan's s_carry before it is reset)
    auto block_scan = [&](const unsigned long long* src, uint64_t n, unsigned long long* dst) {
        __syncthreads();
        if (tid == 0) s_carry = 0;
        __syncthreads();
        for (uint64_t b0 = 0; b0 < n; b0 += 1024) {
            const uint64_t i = b0 + tid;
            const unsigned long long v = i < n ? src[i] : 0ull;
            unsigned long long x = v;
#pragma unroll
            for (int off = 1; off < 64; off <<= 1) {
                const unsigned long long u = __shfl_up(x, off, 64);
                if (lane >= (uint32_t)off) x += u;
            }
            if (lane == 63) s_wave[w] = x;
            __syncthreads();
            unsigned long long pre = s_carry;
            for (uint32_t k = 0; k < w; ++k) pre += s_wave[k];
            if (dst && i < n) dst[i] = pre + x - v;
            __syncthreads();
            if (tid == 0) for (int k = 0; k < 16; ++k) s_carry += s_wave[k];
            __syncthreads();
        }
    };
    block_scan(rcv, cells, nullptr);                     // nr: every record received
    const unsigned long long nr = s_carry;
    block_scan(rcv, (uint64_t)me * R, nullptr);          // rd[me]: records from ranks below me
    if (tid == 0) s_rd = s_carry;
    __syncthreads();
    block_scan(cnt, cells, cursor);                      // send positions, owner-major
    __threadfence_block();
    __syncthreads();
    // the send columns hold n_send records: counts that do not add up to it (offsets and keys out of
    // step) would send the scatter past them, so it writes nothing and the host fails the call
    const bool bad = s_carry != n_send;
    const bool own = own_in_recv && nr <= recv_cap && !bad;
    if (tid == 0) misc->route_own = (own ? 1ull : 0ull) | (bad ? 2ull : 0ull);
    if (!own) return;
    const unsigned long long sd_me = cursor[(uint64_t)me * R];
    __syncthreads();
    for (uint32_t j = tid; j < R; j += 1024) cursor[(uint64_t)me * R + j] += s_rd - sd_me;
}

// Win flags of the sent records (send order, returned by the owners) -> batch order.
__global__ __launch_bounds__(256) void k_flags_back(const uint8_t* __restrict__ sflags,
                                                    const uint64_t* __restrict__ perm, uint64_t n,
                                                    uint8_t* __restrict__ flags)
{
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) flags[perm[i]] = sflags[i];
}

// Part bookkeeping of a sharded merge: gsend[R + j] = records of this rank's part of j, and
// gsend[2R .. 2R + 4) = this rank's record frame (Misc::fr_*, max-accumulators).
constexpr uint32_t kGatherExtra = 7;     // the frame's 4 words, the rank's collective-shape word, its local status,
                                         // the records' largest lt & 0xFFFF (the compact frame, route_l1)
// gsend[2R + 4] = cfg: the per-process settings that shape the collectives after the clock phase
// (comm_path.inc, shard_cfg_word); k_shard_combine checks that every rank sent the same one.
__global__ __launch_bounds__(256) void k_part_counts(const uint64_t* __restrict__ offs, uint32_t R,
                                                     const Misc* __restrict__ misc, long long* __restrict__ gsend,
                                                     long long cfg, long long status)
{
    const uint32_t j = blockIdx.x * 256 + threadIdx.x;
    if (j < R) gsend[R + j] = (long long)(offs[j + 1] - offs[j]);
    if (j == 0) {
        gsend[2 * R] = (long long)misc->fr_lo;
        gsend[2 * R + 1] = (long long)misc->fr_hi;
        gsend[2 * R + 2] = (long long)misc->fr_rlo;
        gsend[2 * R + 3] = (long long)misc->fr_rhi;
        gsend[2 * R + 4] = cfg;
        gsend[2 * R + 5] = status;
        gsend[2 * R + 6] = (long long)misc->fr_cmax;
    }
}

// The gather row of a rank whose local work failed before the gather (its status: -CRDT_E_*, > 0): no
// maxima, no records, no frame — the row only carries the status to the other ranks (k_shard_combine).
__global__ __launch_bounds__(256) void k_fail_row(long long* __restrict__ gsend, uint32_t R, long long cfg,
                                                  long long status)
{
    for (uint32_t j = blockIdx.x * 256 + threadIdx.x; j < R; j += gridDim.x * 256) {
        gsend[j] = INT64_MIN;
        gsend[R + j] = 0;
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        for (int x = 0; x < 4; ++x) gsend[2 * R + x] = 0;
        gsend[2 * R + 4] = cfg;
        gsend[2 * R + 5] = status;
        gsend[2 * R + 6] = 0;
    }
}

// From the all-gathered [G][2R + 4] words (part maxima, part counts, frame): M_j over all parts,
// for this rank's part the max / record count of the parts before it (lower ranks), and the
// frame of every rank's records (the records this rank will receive lie inside it).
__global__ __launch_bounds__(256) void k_shard_combine(const long long* __restrict__ g, uint32_t G, uint32_t me,
                                                       uint32_t R, long long* __restrict__ M,
                                                       long long* __restrict__ pbase,
                                                       unsigned long long* __restrict__ ibase,
                                                       Misc* __restrict__ misc)
{
    const uint32_t j = blockIdx.x * 256 + threadIdx.x;
    const uint64_t row = 2ull * R + kGatherExtra;
    if (j == 0) {
        unsigned long long a = 0, b = 0, c = 0, d = 0;
        for (uint32_t r = 0; r < G; ++r) {
            const unsigned long long* w = reinterpret_cast<const unsigned long long*>(g + r * row + 2ull * R);
            a = w[0] > a ? w[0] : a; b = w[1] > b ? w[1] : b; c = w[2] > c ? w[2] : c; d = w[3] > d ? w[3] : d;
        }
        misc->fr_lo = a; misc->fr_hi = b; misc->fr_rlo = (uint32_t)c; misc->fr_rhi = (uint32_t)d;
        unsigned long long cm = 0;                          // the records' largest lt & 0xFFFF over the ranks
        for (uint32_t r = 0; r < G; ++r) {
            const unsigned long long x = (unsigned long long)g[r * row + 2ull * R + 6];
            cm = x > cm ? x : cm;
        }
        misc->fr_cmax = cm;
        bool same = true;                                   // every rank's collective-shape word alike
        for (uint32_t r = 1; r < G; ++r) same = same && g[r * row + 2ull * R + 4] == g[2ull * R + 4];
        if (!same) misc->route_own = 4ull;                  // (k_route_plan has not run yet)
        unsigned long long fs = 0;                          // a rank's local failure fails every rank
        for (uint32_t r = 0; r < G; ++r) {
            const unsigned long long x = (unsigned long long)g[r * row + 2ull * R + 5];
            fs = x > fs ? x : fs;
        }
        misc->shard_status = fs;
    }
    if (j >= R) return;
    int64_t m = INT64_MIN, pm = INT64_MIN;
    uint64_t ib = 0;
    for (uint32_t r = 0; r < G; ++r) {
        const int64_t v = g[(uint64_t)r * row + j];
        m = imax(m, v);
        if (r < me) {
            pm = imax(pm, v);
            ib += (uint64_t)g[(uint64_t)r * row + R + j];
        }
    }
    M[j] = m;
    pbase[j] = pm;
    ibase[j] = ib;
}

// Per-record counts and the key-range error of this rank, as SUM-reducible words; then one word per
// local failure code (out[kSumWords + code] = 1 for this rank's -CRDT_E_* status, code 1..7), so the
// reduced words tell every rank which failures occurred anywhere.
constexpr int kSumWords = 4, kSumCodes = 8;
__global__ void k_sum_counts(const Misc* __restrict__ misc, bool counted, long long* __restrict__ out, int status)
{
    if (threadIdx.x != 0) return;
    unsigned long long np = 0, nw = 0;
    if (!status)
        for (int s = 0; s < kCounterSlots; ++s) { np += misc->present[s]; nw += misc->won[s]; }
    out[0] = (long long)np;
    out[1] = (long long)nw;
    out[2] = !status && misc->err ? 1 : 0;
    out[3] = counted ? 0 : 1;
    for (int k = 0; k < kSumCodes; ++k) out[kSumWords + k] = 0;
    if (status < 0 && -status < kSumCodes) out[kSumWords - status] = 1;
    else if (status < 0) out[kSumWords + kSumCodes - 1] = 1;
}

// Key ids against the capacity before any row is stored (resident batches of the gather path;
// the sorted path checks them in its level-1 scatter, before its resolve stores anything).
__global__ __launch_bounds__(256) void k_key_check(const uint32_t* __restrict__ key, uint64_t n, uint64_t cap,
                                                   Misc* __restrict__ misc)
{
    // 16-B loads over the 16-B-aligned body (a wave instruction moves 1 KB, not 256 B), scalars around it
    bool bad = false;
    const uint64_t t = (uint64_t)blockIdx.x * 256 + threadIdx.x, stride = (uint64_t)gridDim.x * 256;
    const uint64_t head = std::min<uint64_t>(n, ((16u - ((uintptr_t)key & 15u)) & 15u) / 4u);
    const uint64_t nv = (n - head) / 4;
    const u32x4* __restrict__ kv = reinterpret_cast<const u32x4*>(key + head);
    for (uint64_t i = t; i < nv; i += stride) {
        const u32x4 q = __builtin_nontemporal_load(kv + i);
        bad |= (q.x >= cap) | (q.y >= cap) | (q.z >= cap) | (q.w >= cap);
    }
    if (t < head) bad |= key[t] >= cap;
    if (head + nv * 4 + t < n) bad |= key[head + nv * 4 + t] >= cap;
    if (__any(bad) && (threadIdx.x & 63) == 0) atomicOr(&misc->err, 1u);
}

// Copy every row into a table of another row size (crdt_set_row_bytes).
__global__ __launch_bounds__(256) void k_relayout(Table src, Table dst, uint64_t n)
{
    for (uint64_t k = (uint64_t)blockIdx.x * 256 + threadIdx.x; k < n; k += (uint64_t)gridDim.x * 256)
        store_hc(dst, k, load_hot(src, k), load_cold(src, k));
}

// ----------------------------------------------------------------- SPI kernels
__global__ __launch_bounds__(256) void k_put_rows(
    const uint32_t* __restrict__ key, const int64_t* __restrict__ lt, const uint32_t* __restrict__ rank,
    const uint32_t* __restrict__ val, const int64_t* __restrict__ mod, uint64_t n, Table table,
    uint64_t cap, Misc* __restrict__ misc)
{
    unsigned long long kend = 0;                  // grid-stride (capped grid): few key_end atomics
    bool bad = false;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t k = key[i];
        if (k >= cap) { bad = true; continue; }
        store_row(table, k, lt[i], rank[i], val[i], mod[i]);
        kend = k + 1ull > kend ? k + 1ull : kend;
    }
    if (bad) atomicOr(&misc->err, 1u);
    block_raise_u64(kend, &misc->key_end);
}

// put/putAll rows (crdt.dart:41-42, 51-53): hlc = modified = the one send() result.
__global__ __launch_bounds__(256) void k_put_stamped(
    const uint32_t* __restrict__ key, const uint32_t* __restrict__ val, uint64_t n, int64_t stamp,
    uint32_t local_rank, Table table, uint64_t cap, Misc* __restrict__ misc)
{
    unsigned long long kend = 0;
    bool bad = false;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t k = key[i];
        if (k >= cap) { bad = true; continue; }
        store_row(table, k, stamp, local_rank, val[i], stamp);
        kend = k + 1ull > kend ? k + 1ull : kend;
    }
    if (bad) atomicOr(&misc->err, 1u);
    block_raise_u64(kend, &misc->key_end);
}

__global__ __launch_bounds__(256) void k_read_rows(
    const uint32_t* __restrict__ key, uint64_t n, Table table, uint64_t cap,
    int64_t* __restrict__ lt, uint32_t* __restrict__ rank, uint32_t* __restrict__ val,
    int64_t* __restrict__ mod, Misc* __restrict__ misc)
{
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t k = key[i];
    if (k >= cap) { atomicOr(&misc->err, 1u); return; }
    const uint4 h = load_hot(table, k);
    const uint2 x = load_cold(table, k);
    if (lt) lt[i] = (int64_t)(((uint64_t)h.y << 32) | h.x);
    if (rank) rank[i] = h.z;
    if (val) val[i] = x.y;
    if (mod) mod[i] = (int64_t)(((uint64_t)h.w << 32) | x.x);
}

// refreshCanonicalTime (crdt.dart:114-121): max lt over rows visible to recordMap().
__global__ __launch_bounds__(256) void k_refresh(Table table, uint64_t n,
                                                 long long* __restrict__ out)
{
    __shared__ int64_t s[4];
    int64_t m = INT64_MIN;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const uint4 h = load_hot(table, i);
        if ((int32_t)h.w >= 0) m = imax(m, (int64_t)(((uint64_t)h.y << 32) | h.x));
    }
    m = wave_max(m);
    if ((threadIdx.x & 63) == 0) s[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        m = imax(imax(s[0], s[1]), imax(s[2], s[3]));
        if (m != INT64_MIN) atomicMax(out, (long long)m);
    }
}

// recordMap(modifiedSince) (map_crdt.dart:42-45): order-preserving compaction.
constexpr int kMsPerBlock = 1024;
__global__ __launch_bounds__(256) void k_ms_count(Table table, uint64_t n, int64_t since,
                                                  uint32_t* __restrict__ counts)
{
    __shared__ int s[4];
    const uint64_t base = (uint64_t)blockIdx.x * kMsPerBlock;
    int c = 0;
    for (int q = 0; q < kMsPerBlock / 256; ++q) {
        const uint64_t i = base + q * 256 + threadIdx.x;
        if (i < n) c += !(row_mod(table, i) < since);
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) c += __shfl_xor(c, off, 64);
    if ((threadIdx.x & 63) == 0) s[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) counts[blockIdx.x] = s[0] + s[1] + s[2] + s[3];
}

__global__ __launch_bounds__(1024) void k_ms_scan(uint32_t* __restrict__ counts, uint32_t nb,
                                                  long long* __restrict__ total)
{
    __shared__ unsigned long long s_wave[16];
    __shared__ unsigned long long s_carry;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    if (tid == 0) s_carry = 0;
    __syncthreads();
    for (uint32_t base = 0; base < nb; base += 1024) {
        const uint32_t i = base + tid;
        unsigned long long v = i < nb ? counts[i] : 0;
        unsigned long long x = v;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            unsigned long long u = __shfl_up(x, off, 64);
            if (lane >= off) x += u;
        }
        if (lane == 63) s_wave[w] = x;
        __syncthreads();
        if (w == 0) {
            unsigned long long y = lane < 16 ? s_wave[lane] : 0;
#pragma unroll
            for (int off = 1; off < 16; off <<= 1) {
                unsigned long long u = __shfl_up(y, off, 64);
                if (lane >= off) y += u;
            }
            if (lane < 16) s_wave[lane] = y;
        }
        __syncthreads();
        const unsigned long long pre = (w > 0 ? s_wave[w - 1] : 0) + s_carry;
        if (i < nb) counts[i] = (uint32_t)(pre + x - v);
        __syncthreads();
        if (tid == 0) s_carry += s_wave[15];
        __syncthreads();
    }
    if (tid == 0) *total = (long long)s_carry;
}

__global__ __launch_bounds__(256) void k_ms_write(Table table, uint64_t n, int64_t since,
                                                  const uint32_t* __restrict__ offsets,
                                                  uint32_t* __restrict__ out)
{
    __shared__ int s_wave[4];
    const uint64_t base = (uint64_t)blockIdx.x * kMsPerBlock;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint32_t run = offsets[blockIdx.x];
    for (int q = 0; q < kMsPerBlock / 256; ++q) {
        const uint64_t i = base + q * 256 + threadIdx.x;
        const bool keep = i < n && !(row_mod(table, i) < since);
        const unsigned long long b = __ballot(keep);
        const int before = __popcll(b & ((1ull << lane) - 1));
        if (lane == 0) s_wave[w] = __popcll(b);
        __syncthreads();
        int wpre = 0;
        for (int k = 0; k < w; ++k) wpre += s_wave[k];
        const int tot = s_wave[0] + s_wave[1] + s_wave[2] + s_wave[3];
        if (keep) out[run + wpre + before] = (uint32_t)i;
        run += tot;
        __syncthreads();
    }
}

__global__ __launch_bounds__(256) void k_fill_i64(long long* __restrict__ p, uint64_t n, long long v)
{
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) p[i] = v;
}

__global__ void k_event_init(long long* __restrict__ event)
{
    if (threadIdx.x == 0) { event[0] = kEvNone; event[1] = INT64_MIN; event[2] = 0; event[3] = INT64_MIN; }
}

__global__ __launch_bounds__(256) void k_remap(Table table, uint64_t n,
                                               const uint32_t* __restrict__ lut, uint32_t nl)
{
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint32_t* rk = reinterpret_cast<uint32_t*>(row_ptr(table, i) + 8);
    const uint32_t r = *rk;
    if (r < nl) *rk = lut[r];
}

// ============================================================ host-side context
// CRDT_POISON_ALLOC=1 (debug): every scratch allocation is filled with 0x5A bytes, so a kernel that
// reads scratch it never wrote gives the same wrong answer on every run instead of stale data's
static bool poison_alloc() {
    static const int v = [] { const char* e = getenv("CRDT_POISON_ALLOC"); return e && atoi(e) ? 1 : 0; }();
    return v != 0;
}
template <typename T>
struct DBuf {
    T* p = nullptr;
    size_t n = 0;
    hipError_t ensure(size_t want) {
        if (want <= n && p) return hipSuccess;
        if (p) release();
        size_t m = std::max<size_t>(want, 16);
        hipError_t e = hipMalloc(&p, m * sizeof(T));
        if (e == hipSuccess) n = m;
        if (e == hipSuccess && poison_alloc()) {      // (finished before any stream's next use)
            e = hipMemset(p, 0x5A, m * sizeof(T));
            if (e == hipSuccess) e = hipDeviceSynchronize();
        }
        return e;
    }
    void release() {
        if (p) hipFree(p);
        p = nullptr;
        n = 0;
    }
};

template <typename T>
struct HBuf {
    T* p = nullptr;
    size_t n = 0;
    hipError_t ensure(size_t want) {
        if (want <= n && p) return hipSuccess;
        if (p) { hipHostFree(p); p = nullptr; n = 0; }
        size_t m = std::max<size_t>(want, 16);
        hipError_t e = hipHostMalloc(&p, m * sizeof(T), hipHostMallocDefault);
        if (e == hipSuccess) n = m;
        return e;
    }
    void release() { if (p) hipHostFree(p); p = nullptr; n = 0; }
};

// Changeset segments of the columns an apply phase reads, in changeset order: segment s is
// records [beg[s], end[s]) of changeset j[s].  One per changeset for a local batch; one per
// (changeset, source rank) for records routed in by a sharded merge.
// route_l1 (comm_path.inc): one piece's level-2 + resolve buffers at the owner (one set per piece: the
// host writes a piece's plan while earlier pieces' copies may still be queued)
constexpr uint32_t kRl1MaxPieces = 4;
struct Rl1Scratch {
    DBuf<uint32_t> hist, toff, part, choff, dstart2, tseg, ibase, ibucket, ksu32, kj2;
    DBuf<int64_t> kslt;
    DBuf<u32x4> rec2;
    DBuf<uint64_t> plan;
    HBuf<uint64_t> hplan;
    size_t pw = 0, u32w = 0;        // the plan's words (rl1_owner_prep)
    uint32_t nt2 = 0, nc2 = 0;      // level-2 tiles and scan chunks
    uint32_t ngrp = 0;              // level-1 buckets (groups of segments) level 2 partitions
    size_t nsg = 0;                 // ... and their segments
    uint64_t nw = 0;                // records of the piece at this owner
    void release() {
        hist.release(); toff.release(); part.release(); choff.release(); dstart2.release(); tseg.release();
        ibase.release(); ibucket.release(); ksu32.release(); kj2.release(); kslt.release(); rec2.release();
        plan.release(); hplan.release();
    }
};

struct Segs {
    std::vector<uint64_t> beg, end;
    std::vector<uint32_t> j;
    void from_offsets(const uint64_t* offs, uint32_t R) {
        beg.resize(R); end.resize(R); j.resize(R);
        for (uint32_t x = 0; x < R; ++x) { beg[x] = offs[x]; end[x] = offs[x + 1]; j[x] = x; }
    }
};

}  // namespace

// CRDT_SORTED_FORM bits: switch off a refinement of the packed sorted form (same results; the
// in-process A/B runs of DESIGN.md §5.2 measure each one against the form without it)
constexpr uint32_t kFormNoWholeLines = 64;   // resolve writes changed rows only (partial lines)
constexpr uint32_t kFormNoKey8 = 128;        // 16-B final records (4-B key column)
constexpr uint32_t kFormNoKey16 = 256;       // 16-B level-1 records (4-B key column)
constexpr uint32_t kFormNoReverse = 512;     // partition tiles all fill their ranges forwards
constexpr uint32_t kFormNoHistW = 1024;      // level-2 histogram: 2-B loads, shared bins (k_part_hist)
constexpr uint32_t kFormNoHw = 2048;         // packed resolve reads every row (ignores the high-water mark)
constexpr uint32_t kFormNoVecLoads = 8192;   // level-1 scatter: one 4/8-B load per record and column
constexpr uint32_t kFormNoVecScan = 32768;   // the scan (with the level-1 histogram): strided 8 / 4-B loads
constexpr uint32_t kFormNoVecRoute = 131072; // routing kernels: strided loads, one LDS atomic per record
constexpr uint32_t kFormBigTile2 = 65536;    // level-2 tiles of 32K records (not 8K)
constexpr uint32_t kFormNoOwnInPlace = 524288; // sharded merge: the own chunk copied to the receive columns
// round 6, measured slower and kept as opt-in forms: the flag passes in the scatters' XCD tile order,
// and with four-byte staging + eight-record gathers (CRDT_FBACK_CHK applies to the default byte staging only)
constexpr uint32_t kFormNoCompact = 1u << 20;   // no compact form (PackFrame::cb): 14-B / 13-B partition records
constexpr uint32_t kFormFbackXcd = 1u << 21;
constexpr uint32_t kFormFbackWide = 1u << 22;
constexpr uint32_t kFormScanJx = 1u << 24;      // the clock scan's step-major grid (k_scan's jx) on every batch
constexpr uint32_t kFormNoScanJx = 1u << 25;    // ... on none (default: batches of at most kScanJxMax workgroups)
constexpr uint32_t kFormNoPosT = 1u << 31;      // flagged level 1: positions at the input index (LDS-staged), not
                                                // tile-strided from registers (k_part_scatter1<.., kPT>)
constexpr uint32_t kFormNoItemLists = 1u << 28; // the order-free packed resolve's kernels over every item slot
constexpr uint32_t kFormNoFbackPre = 1u << 27;  // the flag passes of round 5 (k_flags_back), not k_flags_back_pre
constexpr uint32_t kFormFbackPre512 = 1u << 29; // k_flags_back_pre's level-2 pass in 512-thread workgroups (not 256)
constexpr uint32_t kFormNoSparseK = 1u << 26;   // sparse buckets inside k_resolve_packed (not k_resolve_sparse)
constexpr uint32_t kScanJxMax = 8192;           // ~8 rounds of the ~1024 resident scan workgroups (cfg3: 4096)
constexpr uint32_t kFormOverlap = 1u << 23;      // sorted path: split buckets' fold / carry beside the unsplit
                                                 // buckets' resolve (measured slower: opt-in)
constexpr uint32_t kPartPad = 1024;          // records of slack behind every partition buffer (tile-end vector loads)
constexpr uint32_t kPutGrid = 2048;          // k_put_rows / k_put_stamped workgroups (grid-stride)

struct crdt_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    uint32_t local_rank = 0;
    Table table{nullptr, 24};       // capacity rows (crdt_set_row_bytes)
    uint64_t cap = 0;
    int64_t canonical = 0;

    Misc* d_misc = nullptr;
    Misc* h_misc = nullptr;            // pinned
    DBuf<long long> d_M;               // [R]   (single-ctx merge)
    DBuf<long long> d_event;           // [4]
    DBuf<uint64_t> d_plan;             // offsets[R+1] (u64) then tile starts[R+1] (u32): one H2D copy
    HBuf<uint64_t> h_plan;
    const uint64_t* d_offs = nullptr;  // views into d_plan
    const uint32_t* d_tstart = nullptr;
    DBuf<int64_t> d_T, d_Cprev, d_Rj, d_Cj, d_candP, d_candms;
    DBuf<uint32_t> d_candtile, d_candkind;
    DBuf<long long> d_candkey;
    // staging of host-memory batches
    DBuf<uint32_t> s_key, s_rank, s_val;
    // crdt_merge of a host batch: key / val windows are copied on cstream while K2 runs on
    // stream (apply_ranges); kv_key / kv_val = the caller's host columns still to copy
    hipStream_t cstream = nullptr;
    std::vector<hipEvent_t> cevents;
    const uint32_t* kv_key = nullptr;
    const uint32_t* kv_val = nullptr;
    uint64_t kv_n = 0, kv_done = 0, kv_window = 4ull << 20;
    uint32_t kv_win = 0;
    DBuf<int64_t> s_lt, s_millis, s_mod;
    DBuf<uint8_t> s_flags;
    DBuf<uint32_t> s_out;
    DBuf<long long> d_word;
    DBuf<unsigned long long> d_ibase;
    // per-call plan (set by scan, used by later phases)
    uint32_t plan_R = 0;
    uint64_t plan_tiles = 0;
    uint32_t plan_mt = 0;           // most scan tiles of one changeset
    int apply_items = 0;            // K2 records per thread; 0 = by changeset size (CRDT_APPLY_ITEMS: tuning)
    // timing
    bool timing = false;
    std::vector<hipEvent_t> events;
    std::vector<uint32_t> windows;  // launches of each timed apply window (events ev_window(k, *))
    bool sorted_phases = false;     // events ev_window(1..3, *) bracket the sorted path's phases
    uint64_t p1_records = 0;        // records of the first window's level-1 scatter (crdt_timing)
    uint32_t apply_total = 0;
    // sorted path (sorted_path.inc): 0 = auto, 1 = always gather (K2), 2 = sorted when allowed
    int merge_path = 0;
    // High-water mark of written rows: every row >= hw holds the never-written fill (0x80 bytes),
    // so the packed resolve synthesises those rows instead of reading them.  Raised by every row
    // store (put: the keys' bound; merge: the batch's key bound when the scan read the keys, else
    // the whole table), lowered by crdt_clear_rows of a range reaching it.
    uint64_t hw = 0;
    uint64_t hw_read = 0;           // the mark the current merge's kernels rely on (hw at its start)
    uint64_t hw_next = 0;           // hw after the current merge (the capacity unless tightened)
    bool key_end_valid = false;     // this merge's sorted path reduced its bucket bound (Misc::key_end)
    DBuf<u32x4> p1_rec, p2_rec;        // 16-B partitioned records {lt, rank, val}
    DBuf<uint32_t> p1_kj, p2_kj;       // and their kj words
    // PlaceTune (crdt_reserve_scratch, CRDT_PLACE_TRIES): the level-1 scatter's time follows where its
    // destination lands in physical memory (7.6-8.4 ms for the same job on successive
    // allocations in one process), so an explicit reservation takes several candidate level-1 buffers,
    // times the scatter on each in the first merges (candidate 0 = p1_*, k >= 1 = pc_*[k]) and keeps the fastest
    static constexpr int kPlaceMax = 4;
    DBuf<u32x4> pc_rec[kPlaceMax];
    DBuf<uint32_t> pc_kj[kPlaceMax];
    int place_k = 0;                   // candidates under trial (0 / 1: none)
    int place_trial = 0;               // trials done (-1: the warm-up merge comes first); candidate = trial % k,
                                       // two rounds (the clocks still settle over the first merges)
    int place_best = -1;               // the kept candidate (-1: trials not done)
    int place_idle = 0;                // merges since the trials were asked for that did not take the sorted path
    float place_ms[kPlaceMax] = {};    // each candidate's level-1 scatter (ms; the faster of its two trials)
    bool place_timed = false;          // this call times candidate place_trial
    bool place_warm = false;           // this call is the untimed warm-up (the kernels' first launch loads them)
    hipEvent_t place_ev[2] = {};
    DBuf<uint32_t> p_hist, p_toff, p_part, p_choff, p_dstart1, p_dstart2, p_l2map;
    DBuf<uint64_t> p_plan, p_l1beg;
    DBuf<uint32_t> p_ibase, p_ksu32, p_tseg, p_ibucket;   // resolve items per bucket; part-state / carry u32 columns
    DBuf<uint32_t> p_ilist;                  // k_item_lists: per-kernel item lists of the order-free packed resolve
    HBuf<uint32_t> h_ilist;                  // (pinned) their counts
    DBuf<int64_t> p_kslt;
    HBuf<uint64_t> h_pplan;
    bool last_sorted = false;       // the last crdt_merge ran the sorted path
    bool counts = true;             // crdt_set_counts: per-record n_present / n_won (the sorted path
                                    // keeps changeset order for them; off -> its order-free form)
    bool fused = false;             // this plan: tile max in k_clock<true>, resolve in k_verify<true>
    bool scan_eager = false;        // next k_scan loads rank / millis with lt (last call: mostly hot tiles)
    bool no_fuse = false;           // CRDT_NO_FUSE: small merges keep k_tmax / k_resolve_local / k_resolve
    bool xcd_map = true;            // XCD-contiguous tile order in the partition scatters (CRDT_XCD_MAP=0: off)
    bool packed_resolve = true;     // order-free sorted path: packed-key resolve when the frame fits (CRDT_PACKED=0: off)
    bool frame_on = false;          // this plan's scan reduced the record frame into misc->fr_*
    uint32_t rank_bound = 0;        // crdt_set_rank_bound: every rank < bound (0: unknown)
    uint32_t form_off = 0;
    bool env_dynamic = false;
    bool hist_fuse = true;          // CRDT_HIST_FUSE=0: the level-1 histogram as its own pass
    uint32_t l1_tile = 0;           // CRDT_L1_TILE: the level-1 tile in records (0 = chosen per plan: l1_choose)
    uint32_t plan_l1_tile = 28672;  // the level-1 tile of the current plan (ptb, the scan's fused histogram)
    bool last_hist1_fused = false;
    bool frame_lt_only = false;     // this plan's frame: lt from the scan, ranks from rank_bound
    // level-1 histogram counted by the scan (k_scan<.., kHist>) for the sorted path of this plan
    const uint32_t* d_ptb = nullptr;
    uint64_t plan_ptiles = 0;
    DBuf<uint32_t> p_hist1;
    bool hist1_fused = false;
    bool hist1_routed = false;      // ... counted with route_l1's key map (owner-major digits), for route_l1 only
    const uint32_t* hist1_key = nullptr;
    uint32_t hist1_shift = 0;
    bool last_packed = false;       // the last sorted apply used the packed form
    bool last_wire_pk = false;      // the last sharded merge routed 16-B packed records
    bool last_own_in_place = false; // ... and scattered its own chunk into the receive columns
    bool last_key8 = false;         // ... with 1-B final key columns
    bool last_key16 = false;        // ... and 2-B level-1 key columns
    bool last_compact = false;      // ... in the compact form (12-B records; PackFrame::cb)
    bool last_hw = false;           // ... whose packed resolve skipped the rows >= hw_read
    // per-record win flags on the sorted path (the flagged form, sorted_path.inc): CRDT_FLAGS_SORTED=0
    // keeps every flagged merge on the gather path
    bool flags_sorted = true;
    int fback_chk = 6;              // CRDT_FBACK_CHK = 0 / 4 / 6: the flag passes' run-search checkpoints (A/B)
    bool last_flagged = false;      // the last sorted apply was the flagged form
    int combine = 1;                // sharded order-free fan-ins fold home records before routing (CRDT_COMBINE:
                                    // 0 off, 1 auto = from 64 changesets, 2 always)
    bool last_combined = false;
    uint32_t sparse_t = 2048;       // CRDT_SPARSE_T: packed resolve buckets of fewer records read only touched rows
    int route_l1 = 1;               // CRDT_ROUTE_L1=0: sharded order-free merges route records, owners partition;
                                    // 2: route_l1 always with the sender-side head fold; 3: folding every digit
    bool rl1_call_head = false;     // this call's route_l1 folds the owners' leading level-1 digits (the Zipf head)
    bool rl1_call_all = false;      // ... all of them (CRDT_ROUTE_L1=3: tests, A/B)
    bool rl1_cmp = false;           // ... in the compact form (12-B level-1 records + 1-B digits; PackFrame::cb)
    bool last_rl1_head = false;     // ... the last routed merge's did
    uint64_t last_rl1_head_in = 0, last_rl1_head_out = 0;   // ... its head records before / after the fold
    uint32_t last_rl1_head_digits = 0;   // ... the leading level-1 digits it folded (Dh)
    uint64_t sent_bytes = 0;        // this call's bytes to the peers (comm_all_to_all; crdt_timing.sent_bytes)
    uint32_t rl1_pieces = 2;        // CRDT_RL1_SPLIT: route_l1's pipelined pieces (0 / 1: one; up to kRl1MaxPieces)
    uint32_t rl1_call_pieces = 2;   // ... this call's (the tuner's way 2 takes kRl1MaxPieces)
    uint32_t last_rl1_pieces = 0;   // ... the last routed merge's
    bool last_route_l1 = false;     // the last sharded merge partitioned its home records into the owners' buckets
    // the routing of a sharded order-free fan-in, measured (comm_path.inc, RouteTune): route_l1 sends 14-B
    // partition records, the combine folds first and sends ~3.4x fewer bytes at more local work; which is
    // faster depends on the links, so the ctx times each (two calls each, max over ranks) and keeps the faster
    bool route_tune = true;         // CRDT_ROUTE_TUNE=0: the fixed rule (combine at G = 2, route_l1 from G = 4)
    struct RouteTune {
        uint64_t shape = 0;         // (R, G, cap) the trials were taken for
        uint32_t trial = 0;         // trial calls taken (kTrials per way)
        int best = -1;              // 0 route_l1 in 2 pieces, 1 combine, 2 route_l1 in 4, 3 route_l1 in 1,
                                    // 4 route_l1 in 2 pieces with the head fold; -1 while the trials run
        long long us[5] = {-1, -1, -1, -1, -1};   // each way's second call, max over ranks (microseconds)
    } rt;
    int tune_mode = -1;             // this call's way from the tuner (-1: the fixed rule)
    bool tune_trial = false;        // ... and the call took it with both ways open (a trial / a tuned call)
    DBuf<long long> d_tune;         // the trial time's MAX all-reduce word
    HBuf<long long> h_tune;         // ... its pinned staging
    DBuf<uint32_t> rl_rec;          // route_l1: 12-B level-1 payloads, send area [0, n) then the receive area
    DBuf<uint16_t> rl_k16;          // ... and their 2-B key columns
    uint64_t rl_cap = 0;            // records both hold
    Rl1Scratch rl_os[kRl1MaxPieces + 1];   // the owner's level 2 + resolve of each piece (+ the folded head)
    Rl1Scratch rl_hf;               // route_l1's head fold at the sender: level 2 + the emitting resolve
    DBuf<uint32_t> rl_hrec;         // ... the folded head records bound for the peers: 12-B payloads
    DBuf<uint16_t> rl_hk16;         // ... and 2-B key columns
    DBuf<unsigned long long> rl_hcnt;   // ... [G] sent, [G] received, [1] own, [G] bases
    HBuf<unsigned long long> h_hcnt;
    hipEvent_t rl_evh = nullptr;    // ... the fold is done (side stream)
    hipEvent_t ov_ev[2] = {};       // sorted path: the split buckets' fold forks to sstream / joins back
    DBuf<uint32_t> e_key, e_val;    // the combine's emitted (key, packed key, value) list
    DBuf<uint64_t> e_pk;
    DBuf<unsigned long long> e_cnt, e_cur;
    HBuf<unsigned long long> h_ebase;   // the combine's owner bases (pinned staging of e_cur)
    DBuf<uint32_t> e_icnt;           // per emit item: entries, first slots, then [item][owner] entries
    DBuf<uint32_t> e_bbase;          // per bucket: its first emit slot (k_bucket_items)
    DBuf<uint64_t> e_off;            // [item][owner] offsets inside the owner's run
    DBuf<unsigned long long> e_csum; // [chunk of 1024 items][owner] sums, then their offsets
    bool last_ordered = false;      // ... or its ordered packed resolve (exact counts) without flags
    DBuf<uint16_t> f_pos1, f_pos2;  // run offsets: level 1 per input record, level 2 per level-1 record
    DBuf<uint8_t> f_flag1, f_flag2; // flags in level-1 / level-2 order
    DBuf<uint32_t> f_hist2, f_toff2; // level 2's tile histogram / offsets (level 1's stay for the flag pass)
    DBuf<unsigned long long> f_cin_key;   // split buckets: every part's carry-in
    DBuf<uint32_t> f_cin_val;
    DBuf<uint8_t> f_cin_pres;
    bool keys_checked = false;      // the gather apply checked every key id before storing
    bool resolved = false;          // misc->stop / result already computed for this plan
    crdt_timing last_timing{};
    Segs segs;                      // changeset segments of the columns the apply phase reads
    // key-sharded replica (comm_path.inc): this ctx is shard `rank` of `n_ranks`
    uint32_t n_ranks = 1, rank = 0;
    bool has_comm = false;
    bool presharded = false;        // batches hold owned records only, key_id = slot
    crdt_comm_ops ops{};            // the collective backend (RCCL: ops over rccl_comm)
    void* rccl_comm = nullptr;
    DBuf<long long> d_gsend, d_grecv, d_pbase, d_sum;
    DBuf<unsigned long long> d_rcnt, d_rrecv;             // [G][R] route counts sent / received
    DBuf<unsigned long long> d_rcur;                      // [G][R] scatter cursors (k_route_plan)
    hipEvent_t route_ev = nullptr;                        // the route counts have reached the host
    hipStream_t sstream = nullptr;                        // route_l1: the partition of pieces 1 .. P-1
    hipStream_t ostream = nullptr;                        // route_l1: the owner work of pieces 0 .. P-2
    hipEvent_t rl_evs[kRl1MaxPieces] = {};                // route_l1: piece q partitioned
    hipEvent_t rl_evx[kRl1MaxPieces] = {};                // ... piece q exchanged
    hipEvent_t rl_evo = nullptr;                          // ... pieces 0 .. P-2 resolved at the owner
    uint64_t recv_cap = 0;                                // receive columns' capacity (records)
    HBuf<uint64_t> h_rcnt;                                // both, read back once per call
    DBuf<uint32_t> r_skey, r_srank, r_sval, r_key, r_rank, r_val;   // send / receive columns
    DBuf<int64_t> r_slt, r_lt;
    DBuf<uint64_t> r_perm;
    DBuf<uint8_t> r_flags, r_sflags;
    HBuf<uint8_t> h_stage;                                // CRDT_MEM_HOST backends
    HBuf<long long> h_sum;                                // reduced counts / error / uncounted / failure codes
    // failures agreed over the ranks (comm_path.inc): comm_agree's word, route_l1's count exchange
    DBuf<long long> d_agree;
    HBuf<long long> h_agree;
    DBuf<unsigned long long> d_rl1cnt;                    // route_l1: [2][G][P][D] counts, then the status word
    HBuf<uint64_t> h_rl1cnt;
    bool finish_posted = false;                           // this call's finish_apply posted its reduction
    // CRDT_TEST_FAIL="rank:point" (tests): this rank fails with CRDT_E_NOMEM at that point of a sharded merge
    int fail_rank = -1, fail_at = 0;
    // the call's deadline (crdt_set_comm_timeout; comm_path.inc, "the call's deadline"): every host wait of a
    // sharded call polls against it; past it the communicator is aborted and the call returns CRDT_E_COMM
    uint32_t comm_timeout_ms = 300000;
    int64_t comm_deadline_ns = 0;                         // this call's (steady clock; 0: none)
    std::atomic<int> comm_state{0};                       // 0 usable, 1 aborted (deadline), 2 aborted (transport)
    std::atomic<const char*> comm_phase{"idle"};          // where the current / last sharded call is (static text)
    // CRDT_TEST_STALL="rank:point:ms[:d]" (tests): that rank stalls ms at that point (host sleep, or with :d a
    // bounded device spin on the ctx stream); ms < 0: the process exits there (a peer lost mid-call)
    int stall_rank = -1, stall_at = 0, stall_ms = 0;
    bool stall_dev = false;
};

// The level-1 partition tile (records).  The default and 14336 / 28672 are tiles the scan's fused histogram
// counts (one or two per seven scan tiles) and the plan's ptb is laid out in; any other CRDT_L1_TILE (a
// multiple of 1024, an A/B) partitions in its own tiles with the separate histogram pass.
// Per plan (upload_plan): 28672 for changesets of >= 4 such tiles on average (the fan-in: a tie with 14336,
// profiles/r04_l1tile_fused_ab.txt), 14336 for smaller ones, whose last, partial tile is then a smaller
// share (cfg3, ~98K records per changeset: 3.020 vs 3.051 ms, r04_cfg3_l1tile_ab.txt).
constexpr uint32_t kL1TileDefault = 28672;
inline uint32_t l1_choose(const crdt_ctx* c, uint32_t R, uint64_t n) {
    if (c->l1_tile == 14336u || c->l1_tile == 28672u) return c->l1_tile;
    return R && n / R < 4ull * kL1TileDefault ? 14336u : kL1TileDefault;
}
inline uint32_t l1_plan_tile(const crdt_ctx* c) { return c->plan_l1_tile; }


namespace {

#define HIPCHK(expr)                                   \
    do {                                               \
        hipError_t _e = (expr);                        \
        if (_e != hipSuccess) return CRDT_E_HIP;       \
    } while (0)

#define HIPALLOC(expr)                                                     \
    do {                                                                   \
        hipError_t _e = (expr);                                            \
        if (_e == hipErrorOutOfMemory) return CRDT_E_NOMEM;                \
        if (_e != hipSuccess) return CRDT_E_HIP;                           \
    } while (0)

// A HIP failure between two collectives of a sharded call: kept in the call's local status `lst` (the rank
// still posts the collectives, carrying it) instead of returning at once (comm_path.inc, "failures agreed").
#define HIPLST(expr)                                                       \
    do {                                                                   \
        hipError_t _e = (expr);                                            \
        if (_e != hipSuccess && !lst) lst = CRDT_E_HIP;                    \
    } while (0)

// A host wait for the ctx's stream (or an event).  On a sharded ctx joined to a device transport it polls
// against the call's deadline and the transport's asynchronous error (comm_path.inc, comm_wait).
int comm_wait(crdt_ctx* c, hipStream_t s, hipEvent_t e = nullptr);
#define SYNCHK(c, s)                                                       \
    do {                                                                   \
        int _w = comm_wait((c), (s));                                      \
        if (_w) return _w;                                                 \
    } while (0)

inline unsigned grid_for(uint64_t n, unsigned per) { return (unsigned)((n + per - 1) / per); }

hipError_t ensure_events(crdt_ctx* c, size_t n) {
    while (c->events.size() < n) {
        hipEvent_t e;
        hipError_t r = hipEventCreate(&e);
        if (r != hipSuccess) return r;
        c->events.push_back(e);
    }
    return hipSuccess;
}

// The sorted path's two-stream resolve: sstream starts behind everything queued on the ctx stream (fork); the
// ctx stream continues behind everything queued on sstream (join).
int overlap_fork(crdt_ctx* c) {
    if (!c->sstream) HIPCHK(hipStreamCreateWithFlags(&c->sstream, hipStreamNonBlocking));
    for (hipEvent_t& e : c->ov_ev)
        if (!e) HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    HIPCHK(hipEventRecord(c->ov_ev[0], c->stream));
    HIPCHK(hipStreamWaitEvent(c->sstream, c->ov_ev[0], 0));
    return CRDT_OK;
}
int overlap_join(crdt_ctx* c) {
    HIPCHK(hipEventRecord(c->ov_ev[1], c->sstream));
    HIPCHK(hipStreamWaitEvent(c->stream, c->ov_ev[1], 0));
    return CRDT_OK;
}

// Stage a host-memory column into ctx device memory; device-memory columns pass through.
template <typename T>
int stage(crdt_ctx* c, DBuf<T>& buf, const T* src, uint64_t n, int32_t mem, const T** out) {
    if (!src) { *out = nullptr; return CRDT_OK; }
    if (mem == CRDT_MEM_DEVICE) { *out = src; return CRDT_OK; }
    HIPALLOC(buf.ensure(n ? n : 1));
    if (n) HIPCHK(hipMemcpyAsync(buf.p, src, n * sizeof(T), hipMemcpyHostToDevice, c->stream));
    *out = buf.p;
    return CRDT_OK;
}

struct Cols {
    const uint32_t* key = nullptr;
    const int64_t* lt = nullptr;       // packed_in: the packed (lt, rank, window changeset) keys
    const uint32_t* rank = nullptr;
    const uint32_t* val = nullptr;
    const int64_t* millis = nullptr;
    bool packed_in = false;            // records routed in packed (comm_path.inc), for the sorted path
};

int validate_batch(const crdt_batch* b) {
    if (!b || !b->offsets) return CRDT_E_INVALID;
    if (b->mem != CRDT_MEM_HOST && b->mem != CRDT_MEM_DEVICE) return CRDT_E_INVALID;
    if (b->offsets[0] != 0) return CRDT_E_INVALID;
    for (uint32_t j = 0; j < b->n_changesets; ++j)
        if (b->offsets[j + 1] < b->offsets[j]) return CRDT_E_INVALID;
    const uint64_t n = b->offsets[b->n_changesets];
    if (n > 0 && (!b->lt || !b->rank)) return CRDT_E_INVALID;
    if ((uint64_t)b->n_changesets >= (1ull << 24)) return CRDT_E_INVALID;
    for (uint32_t j = 0; j < b->n_changesets; ++j)
        if (b->offsets[j + 1] - b->offsets[j] >= kLowMask) return CRDT_E_INVALID;
    return CRDT_OK;
}

int stage_check_cols(crdt_ctx* c, const crdt_batch* b, Cols* cols) {
    const uint64_t n = b->offsets[b->n_changesets];
    int st;
    if ((st = stage(c, c->s_lt, b->lt, n, b->mem, &cols->lt))) return st;
    if ((st = stage(c, c->s_rank, b->rank, n, b->mem, &cols->rank))) return st;
    if ((st = stage(c, c->s_millis, b->millis, n, b->mem, &cols->millis))) return st;
    return CRDT_OK;
}

int stage_apply_cols(crdt_ctx* c, const crdt_batch* b, Cols* cols) {
    const uint64_t n = b->offsets[b->n_changesets];
    if (n > 0 && (!b->key_id || !b->val)) return CRDT_E_INVALID;
    int st;
    if ((st = stage(c, c->s_key, b->key_id, n, b->mem, &cols->key))) return st;
    if ((st = stage(c, c->s_lt, b->lt, n, b->mem, &cols->lt))) return st;
    if ((st = stage(c, c->s_rank, b->rank, n, b->mem, &cols->rank))) return st;
    if ((st = stage(c, c->s_val, b->val, n, b->mem, &cols->val))) return st;
    return CRDT_OK;
}

// Upload offsets + per-changeset tile starts; returns total tiles and max tiles.
int upload_plan(crdt_ctx* c, const crdt_batch* b, uint64_t* tiles_out, uint32_t* max_tiles) {
    const uint32_t R = b->n_changesets;
    // u64 words: offsets, then packed u32 scan-tile starts and level-1 partition-tile starts
    const size_t half = (R + 2) / 2;
    const size_t words = (R + 1) + 2 * half;
    HIPALLOC(c->h_plan.ensure(words));
    HIPALLOC(c->d_plan.ensure(words));
    uint64_t* h_offs = c->h_plan.p;
    uint32_t* h_tstart = reinterpret_cast<uint32_t*>(c->h_plan.p + (R + 1));
    uint32_t* h_ptb = reinterpret_cast<uint32_t*>(c->h_plan.p + (R + 1) + half);
    uint64_t tiles = 0, ptiles = 0;
    uint32_t mt = 0;
    c->plan_l1_tile = l1_choose(c, R, b->offsets[R] - b->offsets[0]);
    for (uint32_t j = 0; j <= R; ++j) {
        h_offs[j] = b->offsets[j];
        h_tstart[j] = (uint32_t)tiles;
        h_ptb[j] = (uint32_t)ptiles;
        if (j < R) {
            const uint64_t nj = b->offsets[j + 1] - b->offsets[j];
            const uint64_t tj = (nj + kTile - 1) / kTile;
            tiles += tj;
            ptiles += (nj + l1_plan_tile(c) - 1) / l1_plan_tile(c);
            mt = std::max<uint32_t>(mt, (uint32_t)tj);
        }
    }
    if (tiles >= (1ull << 32)) return CRDT_E_INVALID;
    HIPCHK(hipMemcpyAsync(c->d_plan.p, c->h_plan.p, words * sizeof(uint64_t), hipMemcpyHostToDevice, c->stream));
    c->d_offs = c->d_plan.p;
    c->d_tstart = reinterpret_cast<const uint32_t*>(c->d_plan.p + (R + 1));
    c->d_ptb = reinterpret_cast<const uint32_t*>(c->d_plan.p + (R + 1) + half);
    c->plan_ptiles = ptiles;
    *tiles_out = tiles;
    *max_tiles = mt;
    return CRDT_OK;
}

int reset_misc(crdt_ctx* c) {
    HIPCHK(hipMemsetAsync(c->d_misc, 0, sizeof(Misc), c->stream));
    return CRDT_OK;
}

// HIP events of a timed call: start, after the scan, after the clock phase (and its collectives),
// apply start (route_ms = the gap before it), end; then one pair per sampled apply window.
constexpr size_t kEvStart = 0, kEvScan = 1, kEvClock = 2, kEvApply = 3, kEvEnd = 4;
inline size_t ev_window(size_t k, bool end) { return 5 + 2 * k + (end ? 1 : 0); }
inline size_t events_for(size_t nsegs) {     // (windows 1..3 also bracket the sorted path's phases)
    return std::max(ev_window(nsegs / kTimingStride + 2, true), ev_window(3, true)) + 1;
}

inline void raise_hw(crdt_ctx* c, uint64_t key_end) {
    c->hw = std::max<uint64_t>(c->hw, std::min<uint64_t>(key_end, c->cap));
}

inline void ev_record(crdt_ctx* c, size_t idx) {
    if (c->timing && idx < c->events.size()) hipEventRecord(c->events[idx], c->stream);
}

// ---- phases ---------------------------------------------------------------
// allow_fuse (single-ctx crdt_merge): for small batches the tile-max reduction moves into
// k_clock<true> and the resolve kernels into the last k_verify<true> workgroup (c->fused).
// frame: also reduce the records' lt / rank frame into misc->fr_* (the sorted path's packed key;
// the scan then reads every rank with its lt).
// bound_ok: the frame's rank part may come from crdt_set_rank_bound (single ctx; a sharded merge
// reduces the ranks' own frame, which the packed wire records are encoded against).
// route_km (a sharded merge that will likely partition its home records into the owners' level-1 buckets,
// comm_path.inc route_l1): the scan also counts the routed level-1 histogram (keys read with lt and rank).
int phase_scan(crdt_ctx* c, const crdt_batch* home, int64_t wall, long long* d_maxima, bool allow_fuse = false,
               bool frame = false, bool bound_ok = true, bool keys_ready = false, const KeyMap* route_km = nullptr) {
    c->fused = false;
    c->resolved = false;
    c->hist1_fused = false;
    int st = validate_batch(home);
    if (st) return st;
    const uint32_t R = home->n_changesets;
    Cols cols;
    if ((st = stage_check_cols(c, home, &cols))) return st;
    uint64_t tiles = 0;
    uint32_t mt = 0;
    if ((st = upload_plan(c, home, &tiles, &mt))) return st;
    HIPALLOC(c->d_T.ensure(tiles + 1));
    HIPALLOC(c->d_candtile.ensure(tiles + 1));
    HIPALLOC(c->d_candkey.ensure(tiles + 1));
    HIPALLOC(c->d_candP.ensure(tiles + 1));
    HIPALLOC(c->d_candkind.ensure(tiles + 1));
    HIPALLOC(c->d_candms.ensure(tiles + 1));
    if ((st = reset_misc(c))) return st;
    if (!tiles)
        k_fill_i64<<<grid_for(std::max<uint32_t>(R, 1), 256), 256, 0, c->stream>>>(d_maxima, std::max<uint32_t>(R, 1),
                                                                                     INT64_MIN);
    c->plan_R = R;
    c->plan_tiles = tiles;
    c->plan_mt = mt;
    c->frame_on = frame;
    c->frame_lt_only = frame && bound_ok && c->rank_bound && !c->scan_eager;
    c->fused = allow_fuse && !c->no_fuse && tiles > 0 && tiles <= kClockTilesMax && R <= kClockRMax;
    // the sorted path's level-1 histogram rides on the scan when the keys are device-resident
    // (no staging copy of them here) and the call is one window of changesets (sorted_path.inc)
    // (a host batch arrives here as device columns whose keys are still being copied: keys_ready)
    const bool hist = c->frame_lt_only && c->hist_fuse && keys_ready && home->mem == CRDT_MEM_DEVICE &&
                      R <= kWindow && tiles > 0 && home->key_id;
    const bool rhist = !hist && route_km && frame && c->hist_fuse && R <= kWindow && tiles > 0 && home->key_id &&
                       !home->millis;
    if (hist || rhist) {
        HIPALLOC(c->p_hist1.ensure(c->plan_ptiles * kDigits));
        c->hist1_fused = true;
        c->hist1_routed = rhist;
        c->hist1_key = home->key_id;
        c->hist1_shift = rhist || c->cap > (1ull << 20) ? 20u : (uint32_t)kSBits;
    }
    ScanHist shr{home->key_id, c->d_ptb, c->cap, 20u, c->p_hist1.p};
    shr.htile = l1_plan_tile(c);
    ScanHist shist{home->key_id, c->d_ptb, c->cap, c->hist1_shift, c->p_hist1.p};
    shist.htile = l1_plan_tile(c);
    if (rhist) shr.km = *route_km;
    if (tiles) {
        // grid.x: tiles of one changeset strided over at most ~64K blocks in total
        const uint32_t cap_x = std::max<uint32_t>(1, 65536u / std::max<uint32_t>(R, 1));
        const uint32_t gx = std::max<uint32_t>(1, std::min<uint32_t>(mt, cap_x));
        const uint32_t gxh = std::max<uint32_t>(1, std::min<uint32_t>((mt + kHistSub - 1) / kHistSub, cap_x));
        // step-major grid where the batch is only a few workgroup rounds deep (the rounds' tail is what it
        // shortens: cfg3 0.337 -> 0.303 ms); changeset-major otherwise (the 1B fan-in's 35 rounds: a tie)
        const bool hgrid = hist || rhist;
        const uint64_t nwg = (uint64_t)(hgrid ? gxh : gx) * R;
        const bool jx = !(c->form_off & kFormNoScanJx) && ((c->form_off & kFormScanJx) || nwg <= kScanJxMax);
        for (uint32_t jb = 0; jb < R; jb += 65535) {
            const uint32_t gy = std::min<uint32_t>(65535, R - jb);
            const dim3 gdh = jx ? dim3(gy, std::min<uint32_t>(gxh, 65535)) : dim3(gxh, gy);
            const dim3 gd = jx ? dim3(gy, std::min<uint32_t>(gx, 65535)) : dim3(gx, gy);
            if (rhist)                                    // routed histogram: rank read with lt (the frame)
                k_scan<true, false, true, true, true><<<gdh, kScanThreads, 0, c->stream>>>(
                    cols.lt, cols.rank, nullptr, c->d_offs, c->d_tstart, jb, c->canonical, wall,
                    c->local_rank, c->d_T.p, c->d_misc, c->d_candtile.p, shr, jx);
            else if (hist && !(c->form_off & kFormNoVecScan))
                k_scan<false, true, true, true, true><<<gdh, kScanThreads, 0, c->stream>>>(
                    cols.lt, cols.rank, cols.millis, c->d_offs, c->d_tstart, jb, c->canonical, wall,
                    c->local_rank, c->d_T.p, c->d_misc, c->d_candtile.p,
                    shist, jx);
            else if (hist)
                k_scan<false, true, true, true><<<gdh, kScanThreads, 0, c->stream>>>(
                    cols.lt, cols.rank, cols.millis, c->d_offs, c->d_tstart, jb, c->canonical, wall,
                    c->local_rank, c->d_T.p, c->d_misc, c->d_candtile.p, shist, jx);
            else if (c->frame_lt_only)                    // lt frame only: ranks loaded lazily as usual
                k_scan<false, true, true><<<gd, kScanThreads, 0, c->stream>>>(
                    cols.lt, cols.rank, cols.millis, c->d_offs, c->d_tstart, jb, c->canonical, wall,
                    c->local_rank, c->d_T.p, c->d_misc, c->d_candtile.p, ScanHist{}, jx);
            else if (frame && !cols.millis)
                k_scan<true, false, true><<<gd, kScanThreads, 0, c->stream>>>(
                    cols.lt, cols.rank, nullptr, c->d_offs, c->d_tstart, jb, c->canonical, wall,
                    c->local_rank, c->d_T.p, c->d_misc, c->d_candtile.p, ScanHist{}, jx);
            else if (frame)
                k_scan<true, true, true><<<gd, kScanThreads, 0, c->stream>>>(
                    cols.lt, cols.rank, cols.millis, c->d_offs, c->d_tstart, jb, c->canonical, wall,
                    c->local_rank, c->d_T.p, c->d_misc, c->d_candtile.p, ScanHist{}, jx);
            else if (c->scan_eager && !cols.millis)
                k_scan<true, false><<<gd, kScanThreads, 0, c->stream>>>(
                    cols.lt, cols.rank, nullptr, c->d_offs, c->d_tstart, jb, c->canonical, wall,
                    c->local_rank, c->d_T.p, c->d_misc, c->d_candtile.p, ScanHist{}, jx);
            else if (c->scan_eager)
                k_scan<true><<<gd, kScanThreads, 0, c->stream>>>(
                    cols.lt, cols.rank, cols.millis, c->d_offs, c->d_tstart, jb, c->canonical, wall,
                    c->local_rank, c->d_T.p, c->d_misc, c->d_candtile.p, ScanHist{}, jx);
            else
                k_scan<false><<<gd, kScanThreads, 0, c->stream>>>(
                    cols.lt, cols.rank, cols.millis, c->d_offs, c->d_tstart, jb, c->canonical, wall,
                    c->local_rank, c->d_T.p, c->d_misc, c->d_candtile.p, ScanHist{}, jx);
        }
        if (!c->fused)
            k_tmax<<<std::min<uint32_t>(R, 4096), 256, 0, c->stream>>>(c->d_T.p, c->d_tstart, R, d_maxima);
        HIPCHK(hipGetLastError());
    }
    return CRDT_OK;
}

// d_pbase / d_ibase_in (device, [R], optional): this ctx holds only a PART of each changeset,
// preceded in its iteration order by parts whose max lt / record count these give (sharded merge).
int phase_clock(crdt_ctx* c, const crdt_batch* home, int64_t wall, const long long* d_maxima,
                long long* d_event, const long long* d_pbase = nullptr,
                const unsigned long long* d_ibase_in = nullptr) {
    const uint32_t R = c->plan_R;
    if (!home || home->n_changesets != R) return CRDT_E_INVALID;
    int st;
    Cols cols;
    if ((st = stage_check_cols(c, home, &cols))) return st;   // no-op for device batches
    HIPALLOC(c->d_Cprev.ensure(R + 1));
    HIPALLOC(c->d_Rj.ensure(R + 1));
    HIPALLOC(c->d_Cj.ensure(R + 1));
    const unsigned long long* d_ibase = d_ibase_in;
    if (!R) k_event_init<<<1, 64, 0, c->stream>>>(d_event);   // else k_clock initialises the words
    if (c->fused) {                                           // (plan_tiles > 0, R <= kClockRMax)
        k_clock<true><<<1, 1024, 0, c->stream>>>(nullptr, c->d_T.p, c->d_tstart, R, wall, c->canonical,
                                                 c->d_Cprev.p, c->d_Rj.p, c->d_Cj.p, d_event);
        k_verify<true><<<kVerifyBlocks, 64, 0, c->stream>>>(
            cols.lt, cols.rank, cols.millis, c->d_offs, c->d_tstart, R, c->d_T.p, c->d_Cprev.p, wall,
            c->local_rank, c->d_misc, c->d_candtile.p, c->d_candkey.p, c->d_candP.p, c->d_candkind.p,
            c->d_candms.p, d_pbase, d_ibase, d_event, c->canonical, c->d_Rj.p, c->d_Cj.p, (uint32_t)kTile);
        c->resolved = true;                                   // misc->stop / result are set
        HIPCHK(hipGetLastError());
        return CRDT_OK;
    }
    if (R) k_clock<false><<<1, 1024, 0, c->stream>>>(d_maxima, nullptr, nullptr, R, wall, c->canonical,
                                                     c->d_Cprev.p, c->d_Rj.p, c->d_Cj.p, d_event);
    if (c->plan_tiles)
        k_verify<false><<<kVerifyBlocks, 64, 0, c->stream>>>(
            cols.lt, cols.rank, cols.millis, c->d_offs, c->d_tstart, R, c->d_T.p, c->d_Cprev.p, wall,
            c->local_rank, c->d_misc, c->d_candtile.p, c->d_candkey.p, c->d_candP.p, c->d_candkind.p,
            c->d_candms.p, d_pbase, d_ibase, d_event, 0, nullptr, nullptr, (uint32_t)kTile);
    HIPCHK(hipGetLastError());
    return CRDT_OK;
}

int phase_resolve(crdt_ctx* c, long long* d_event) {
    k_resolve_local<<<1, 256, 0, c->stream>>>(c->d_misc, c->d_candkey.p, c->d_candP.p, c->d_candkind.p,
                                              c->d_candms.p, d_event);
    HIPCHK(hipGetLastError());
    return CRDT_OK;
}

// Windowed staging of a host batch's key / val columns (crdt_merge): window w = records
// [w * kKvWindow, ...) is copied on cstream and stream waits for its event before the first K2
// piece that reads it, so the copy of window w + 1 runs under K2 of window w.  (lt / rank are
// staged in full before the scan, which needs every record.)
// (c->kv_window records, default 4M = 32 MB of key + val, ~0.6 ms of PCIe; CRDT_KV_WINDOW: tests)

int kv_copy_next(crdt_ctx* c) {
    const uint64_t b = c->kv_done, e = std::min<uint64_t>(c->kv_n, b + c->kv_window);
    if (c->kv_win >= c->cevents.size()) {
        hipEvent_t ev;
        HIPCHK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
        c->cevents.push_back(ev);
    }
    HIPCHK(hipMemcpyAsync(c->s_key.p + b, c->kv_key + b, (e - b) * sizeof(uint32_t), hipMemcpyHostToDevice,
                          c->cstream));
    HIPCHK(hipMemcpyAsync(c->s_val.p + b, c->kv_val + b, (e - b) * sizeof(uint32_t), hipMemcpyHostToDevice,
                          c->cstream));
    HIPCHK(hipEventRecord(c->cevents[c->kv_win], c->cstream));
    HIPCHK(hipStreamWaitEvent(c->stream, c->cevents[c->kv_win], 0));
    c->kv_win++;
    c->kv_done = e;
    return CRDT_OK;
}

// every remaining window (the sorted path reads the whole columns)
int kv_copy_all(crdt_ctx* c) {
    while (c->kv_key && c->kv_done < c->kv_n) {
        int st = kv_copy_next(c);
        if (st) return st;
    }
    return CRDT_OK;
}

int comm_all_reduce(crdt_ctx* c, long long* d, uint64_t n, int32_t op);   // comm_path.inc
void test_stall(crdt_ctx* c, int point);                                   // ... (CRDT_TEST_STALL)

// The sorted path's frame from the scan's accumulators (read back into h_misc); with a declared
// rank bound its rank part is [0, bound) — the level-1 scatter checks every rank against it.
PackFrame frame_of(const crdt_ctx* c) {
    const Misc* m = c->h_misc;
    const bool any = m->fr_lo != 0 || m->fr_hi != 0;
    const bool bound = c->frame_lt_only;
    const uint32_t rlo = bound ? (any ? ~0u : 0u) : m->fr_rlo;               // ~min: min 0
    const uint32_t rhi = bound ? (any ? c->rank_bound - 1 : 0u) : m->fr_rhi;
    PackFrame f = make_frame(m->fr_lo, m->fr_hi, rlo, rhi, c->plan_R);
    f.rk_limit = bound ? c->rank_bound : UINT32_MAX;
    return f;
}

// Read the call's outcome back (one D2H of Misc, the only sync of the apply phase).  On a
// sharded ctx the per-record counts, the key-range error and "not counted" are SUM-reduced
// over the ranks first, so every rank returns the same result.
// local_st (a sharded ctx): this rank's apply failed before its end (-CRDT_E_*); the SUM reduction is posted
// all the same, carrying the failure, so every rank returns the same status (comm_path.inc).
int finish_apply(crdt_ctx* c, uint8_t* host_flags, const uint8_t* dflags, uint64_t n, bool sorted,
                 crdt_result* out, int local_st = 0) {
    // the order-free sorted form does not count them (the flagged form does)
    const bool counted = !sorted || c->counts || c->last_flagged;
    if (c->has_comm) {                      // (d_sum / h_sum: allocated by comm_attach)
        c->finish_posted = true;
        k_sum_counts<<<1, 64, 0, c->stream>>>(c->d_misc, counted, c->d_sum.p, local_st);
        int st = comm_all_reduce(c, c->d_sum.p, kSumWords + kSumCodes, CRDT_REDUCE_SUM);
        if (st) return st;
        test_stall(c, 5);                   // (kStallReadback: a device spin behind the reduction, tests)
        HIPCHK(hipMemcpyAsync(c->h_sum.p, c->d_sum.p, (kSumWords + kSumCodes) * sizeof(long long),
                              hipMemcpyDeviceToHost, c->stream));
    } else if (local_st) {
        return local_st;
    }
    HIPCHK(hipMemcpyAsync(c->h_misc, c->d_misc, sizeof(Misc), hipMemcpyDeviceToHost, c->stream));
    if (host_flags && n && !local_st) HIPCHK(hipMemcpyAsync(host_flags, dflags, n, hipMemcpyDeviceToHost, c->stream));
    SYNCHK(c, c->stream);
    if (c->has_comm)                        // a rank's failure (the largest code) is every rank's
        for (int k = kSumCodes - 1; k > 0; --k)
            if (c->h_sum.p[kSumWords + k]) return -k;
    crdt_result res = c->h_misc->result;
    c->scan_eager = 2ull * kHotSample * c->h_misc->tiles_hot > c->plan_tiles;
    if (c->key_end_valid && !c->has_comm)        // rows stored lie in the sorted path's buckets
        c->hw_next = std::max<uint64_t>(c->hw, std::min<uint64_t>(c->h_misc->key_end, c->cap));
    uint64_t np = 0, nw = 0;
    for (int s = 0; s < kCounterSlots; ++s) { np += c->h_misc->present[s]; nw += c->h_misc->won[s]; }
    bool all_counted = counted, err = c->h_misc->err != 0;
    if (c->has_comm) {
        np = (uint64_t)c->h_sum.p[0];
        nw = (uint64_t)c->h_sum.p[1];
        err = c->h_sum.p[2] != 0;
        all_counted = c->h_sum.p[3] == 0;
    }
    res.n_present = all_counted ? np : UINT64_MAX;
    res.n_won = all_counted ? nw : UINT64_MAX;
    if (c->h_misc->err & 2u) {                 // a rank at or over crdt_set_rank_bound's bound: the
        res.status = CRDT_E_INVALID;           // resolve stored nothing, the clock does not move
        res.canonical_lt = c->canonical;
        if (out) *out = res;
        return res.status;
    }
    if (err) {
        res.status = CRDT_E_KEY_RANGE;
        if ((sorted || c->keys_checked) && (c->h_misc->err & 1u)) {   // this ctx stored nothing
            res.canonical_lt = c->canonical;
            if (out) *out = res;
            return res.status;
        }
    }
    c->canonical = res.canonical_lt;
    if (out) *out = res;
    return res.status;
}

// K2 over the batch's changeset segments (host lists, changeset order; a changeset may be
// several segments).  n = length of the columns (win flags are indexed like them).
int apply_ranges(crdt_ctx* c, const Cols& cols, const Segs& sg, uint64_t n, int32_t mem,
                 int64_t wall, const long long* d_event, uint8_t* win_flags, crdt_result* out) {
    const uint32_t R = c->plan_R;
    uint8_t* dflags = nullptr;
    if (win_flags) {
        if (mem == CRDT_MEM_DEVICE) {
            dflags = win_flags;
        } else {
            HIPALLOC(c->s_flags.ensure(n ? n : 1));
            dflags = c->s_flags.p;
        }
        if (n) HIPCHK(hipMemsetAsync(dflags, 0, n, c->stream));
    }
    if (!c->resolved)
        k_resolve<<<1, 64, 0, c->stream>>>(d_event, R, wall, c->canonical, c->d_Rj.p, c->d_Cj.p, c->d_misc);
    c->resolved = false;
    // resident keys are checked up front, so a bad id stores nothing (host batches stream their
    // keys in under K2: there the K2 launches after the first bad id store nothing)
    c->keys_checked = !c->kv_key;
    if (c->keys_checked && n)
        k_key_check<<<std::min<uint32_t>(grid_for(n, 256 * 16), 8192), 256, 0, c->stream>>>(cols.key, n, c->cap,
                                                                                           c->d_misc);
    ev_record(c, kEvApply);
    c->windows.clear();
    uint32_t nl = 0;
    c->apply_total = 0;
    bool win_open = false;
    uint32_t win_n = 0;
    for (size_t s = 0; s < sg.j.size(); ++s) {
      const uint32_t j = sg.j[s];
      // one K2 launch per piece of the segment inside one staged key / val window (the whole
      // segment when the columns are resident); a changeset's keys are distinct, so its
      // pieces are independent and all use R_j
      for (uint64_t pb = sg.beg[s], pe; pb < sg.end[s]; pb = pe) {
        pe = sg.end[s];
        if (c->kv_key) {
            while (c->kv_done <= pb) {
                int st = kv_copy_next(c);
                if (st) return st;
            }
            pe = std::min<uint64_t>(pe, c->kv_done);
        }
        const uint64_t b = pb, e = pe;
        // HIP-event timing of sampled windows of kTimingWindow back-to-back launches (one event
        // pair per window, so the events do not split the stream the rest of the time)
        if (c->timing && b == sg.beg[s] && (nl++ % kTimingStride) == 0 && !win_open) {
            win_open = true;
            win_n = 0;
            ev_record(c, ev_window(c->windows.size(), false));
        }
        c->apply_total++;
        // records per thread (measured: more gathers in flight per thread beats more
        // workgroups, down to ~100K records per changeset)
        const int items = c->apply_items ? c->apply_items : ((e - b) >= (512ull << 10) ? 4 : 2);
        const unsigned grid = grid_for(e - b, (uint64_t)kApplyThreads * items);
        if (items == 8)
            k_apply<8><<<grid, kApplyThreads, 0, c->stream>>>(cols.key, cols.lt, cols.rank, cols.val, b, e, j,
                                                              c->table, c->cap, c->d_Rj.p, c->d_misc, dflags);
        else if (items == 4)
            k_apply<4><<<grid, kApplyThreads, 0, c->stream>>>(cols.key, cols.lt, cols.rank, cols.val, b, e, j,
                                                              c->table, c->cap, c->d_Rj.p, c->d_misc, dflags);
        else if (items == 2)
            k_apply<2><<<grid, kApplyThreads, 0, c->stream>>>(cols.key, cols.lt, cols.rank, cols.val, b, e, j,
                                                              c->table, c->cap, c->d_Rj.p, c->d_misc, dflags);
        else
            k_apply<1><<<grid, kApplyThreads, 0, c->stream>>>(cols.key, cols.lt, cols.rank, cols.val, b, e, j,
                                                              c->table, c->cap, c->d_Rj.p, c->d_misc, dflags);
        if (win_open && ++win_n == kTimingWindow) {
            ev_record(c, ev_window(c->windows.size(), true));
            c->windows.push_back(win_n);
            win_open = false;
        }
      }
    }
    if (win_open) {
        ev_record(c, ev_window(c->windows.size(), true));
        c->windows.push_back(win_n);
    }
    HIPCHK(hipGetLastError());
    return finish_apply(c, win_flags && mem == CRDT_MEM_HOST ? win_flags : nullptr, dflags, n, false, out);
}

#ifdef CRDT_PROF_RESOLVE
// resolve phase clocks (CRDT_PROF_RESOLVE builds only)
void prof_resolve_report() {
        unsigned long long pr[8];
        hipMemcpyFromSymbol(pr, HIP_SYMBOL(g_rprof), sizeof(pr));
        fprintf(stderr, "[rprof] items %llu chunks %llu | per item: init %.2f us final %.2f us | per chunk: "
                "A %.2f us B %.2f us | max chunk B %.2f us, max item %.2f us\n", pr[4], pr[5],
                pr[0] / 100.0 / (pr[4] ? pr[4] : 1), pr[3] / 100.0 / (pr[4] ? pr[4] : 1),
                pr[1] / 100.0 / (pr[5] ? pr[5] : 1), pr[2] / 100.0 / (pr[5] ? pr[5] : 1), pr[6] / 100.0,
                pr[7] / 100.0);
        memset(pr, 0, sizeof(pr));
        hipMemcpyToSymbol(HIP_SYMBOL(g_rprof), pr, sizeof(pr));
        static std::vector<unsigned long long> it(1 << 18);
        hipMemcpyFromSymbol(it.data(), HIP_SYMBOL(g_item_dur), it.size() * 8);
        uint64_t hist[8] = {0}, hsum[8] = {0};           // by duration: <25, <50, <100, <200, <400, <800, <1600, more us
        unsigned long long top = 0;
        size_t top_i = 0;
        for (size_t i = 0; i < it.size(); ++i) {
            const double us = (it[i] >> 24) / 100.0;
            if (!it[i]) continue;
            int b = us < 25 ? 0 : us < 50 ? 1 : us < 100 ? 2 : us < 200 ? 3 : us < 400 ? 4 : us < 800 ? 5 : us < 1600 ? 6 : 7;
            hist[b]++;
            hsum[b] += (it[i] >> 8) & 0xFFFF;
            if (it[i] > top) { top = it[i]; top_i = i; }
        }
        fprintf(stderr, "[rprof] items by duration <25/50/100/200/400/800/1600/more us: ");
        for (int b = 0; b < 8; ++b) fprintf(stderr, "%llu(%.1f ch) ", (unsigned long long)hist[b], hist[b] ? (double)hsum[b] / hist[b] : 0.0);
        fprintf(stderr, "| slowest item %zu: %.1f us, %llu chunks, flags %llu\n", top_i, (top >> 24) / 100.0,
                (top >> 8) & 0xFFFF, top & 3);
        std::fill(it.begin(), it.end(), 0ull);
        hipMemcpyToSymbol(HIP_SYMBOL(g_item_dur), it.data(), it.size() * 8);
}
#endif

// PlaceTune's candidate level-1 buffers (crdt_reserve_scratch asked for c->place_k of them), taken by the
// warm-up merge with that call's form and size: extra candidates only while they stay within 1/8 of the
// device's HBM together and leave a quarter of it free (at the 1B fan-in: two of 14 GB); the candidates
// that fit are timed, the rest dropped.
void place_take(crdt_ctx* c, size_t rec_units, size_t kj_units) {
    size_t free_b = 0, total_b = 0;
    if (hipMemGetInfo(&free_b, &total_b) != hipSuccess) free_b = total_b = 0;
    const size_t cb = rec_units * sizeof(u32x4) + kj_units * sizeof(uint32_t);
    size_t used = 0;
    int k = 1;
    for (; k < c->place_k; ++k) {
        if (used + cb > total_b / 8 || free_b < used + cb + total_b / 4) break;
        if (c->pc_rec[k].ensure(rec_units) != hipSuccess || c->pc_kj[k].ensure(kj_units) != hipSuccess) {
            c->pc_rec[k].release();
            c->pc_kj[k].release();
            break;
        }
        used += cb;
    }
    c->place_k = k;
    if (k == 1) {                                      // nothing to try: p1 stays
        c->place_trial = 0;
        c->place_best = 0;
    }
}

// A ctx that asked for placement trials but whose merges do not take the sorted path: the candidates go.
void place_drop(crdt_ctx* c) {
    for (int i = 1; i < crdt_ctx::kPlaceMax; ++i) { c->pc_rec[i].release(); c->pc_kj[i].release(); }
    c->place_k = 1;
    c->place_trial = 0;
    c->place_best = 0;
}

// Sorted path (sorted_path.inc) for the whole batch: k_resolve (stop point), then per
// window of kWindow changesets a level-1 (+ level-2) partition of the applied records and
// the per-bucket LDS resolve.  sg = the batch's changeset segments (host), in changeset
// order; one changeset may be several segments (records routed in from several ranks).
int apply_sorted(crdt_ctx* c, const Cols& cols, const Segs& sg, int64_t wall, const long long* d_event,
                 crdt_result* out, uint8_t* dflags = nullptr,
                 EmitOut* emit = nullptr) {
    const uint32_t R = c->plan_R;
    // dflags (device, zeroed by the caller): the flagged form — packed records, stable level 2, the
    // ordered resolve with per-record flags, and the flags carried back to input order
    const bool fl = dflags != nullptr;
    // emit (comm_path.inc, map-side combine): fold the records against an absent table (the caller sets
    // the key range and hw_read = 0) and emit one packed maximum per key; no row, result or timing
    const bool em = emit != nullptr;
    if (!em) {
        if (!c->resolved)
            k_resolve<<<1, 64, 0, c->stream>>>(d_event, R, wall, c->canonical, c->d_Rj.p, c->d_Cj.p, c->d_misc);
        c->resolved = false;
        ev_record(c, kEvApply);
        c->windows.clear();
        c->apply_total = 1;
        if (c->timing) ev_record(c, ev_window(0, false));
    }
    const bool two = c->cap > (1ull << 20);
    const uint32_t shift1 = two ? 20u : (uint32_t)kSBits;
    const size_t ns_all = sg.j.size();
    // order-free form: packed 12-B payloads and the packed resolve when the scan's frame of the
    // batch fits the 64-bit key (one read-back of Misc per call), else wide payloads + lists
    PackFrame pf{};
    bool pk = false;
    if (cols.packed_in || (c->packed_resolve && c->frame_on)) {
        HIPCHK(hipMemcpyAsync(c->h_misc, c->d_misc, sizeof(Misc), hipMemcpyDeviceToHost, c->stream));
        SYNCHK(c, c->stream);
        pf = frame_of(c);
        pk = pf.ok;
        if (cols.packed_in && !pk) return CRDT_E_INVALID;           // routed packed under this same frame
    }
    if ((fl || em) && (!pk || cols.packed_in)) return CRDT_E_INVALID;   // the callers checked the frame
    // the ordered packed form: the flagged form's kernels, for win flags and / or exact per-record
    // counts (without flags: no positions kept, no flags carried back)
    const bool ord = !em && (fl || (c->counts && pk && !cols.packed_in));
    c->last_ordered = ord;
    c->last_packed = pk;
    c->key_end_valid = true;                 // k_bucket_items bounds the rows every window writes
    c->last_hist1_fused = false;
    c->sorted_phases = false;
    // final records with a 1-B key column when the packed key leaves 4 bits free (two levels)
    const bool k8 = pk && two && pf.key4 && !(c->form_off & kFormNoKey8);
    const bool k16 = k8 && !(c->form_off & kFormNoKey16);     // ... and 2-B level-1 key columns
    // the compact form (round 6; sorted_path.inc PackFrame::cb): on one ctx's order-free packed form, when the
    // records' lt & 0xFFFF (the scan's fr_cmax) leave the lt field short enough, 12-B records that carry their
    // whole 20-bit level-1 slot (+ a 1-B level-2 digit column at level 1) instead of 14 + 13 B
    bool cmp = false;
    if (k16 && (ord || !c->counts) && !em && !c->has_comm && !cols.packed_in && c->frame_on &&
        !(c->form_off & (kFormNoCompact | kFormNoHistW | kFormBigTile2 | kFormNoWholeLines | kFormNoVecLoads))) {
        const PackFrame cf = compact_frame(pf, (uint32_t)std::min<unsigned long long>(c->h_misc->fr_cmax, 0xFFFFull),
                                           c->plan_R);
        if (cf.cb) {
            pf = cf;
            cmp = true;
        }
    }
    c->last_compact = cmp;
    c->last_key8 = k8;
    c->last_key16 = k16;
    c->last_hw = pk && (!c->counts || ord) && c->hw_read < c->cap;     // (in the first window)
    // flagged, compact, one window, the default level-1 flag pass: the level-1 positions tile-strided (kPT)
    const uint32_t win0 = pk ? pf.jwin : kWindow;
    const bool pt1 = fl && cmp && ns_all && sg.j[0] / win0 == sg.j[ns_all - 1] / win0 &&
                     !(c->form_off & (kFormNoPosT | kFormNoFbackPre | kFormFbackWide)) &&
                     !(c->xcd_map && (c->form_off & kFormFbackXcd));
    if (fl && !pt1) {
        uint64_t ncol = 0;                                           // input index space of pos1
        for (size_t s = 0; s < ns_all; ++s) ncol = std::max<uint64_t>(ncol, sg.end[s]);
        HIPALLOC(c->f_pos1.ensure((ncol ? ncol : 1) + 8));   // + 8: k_flags_back_pre's clamped loads
    }
    for (size_t sb = 0; sb < ns_all;) {
        // window [jb, jb + win): kWindow changesets (the kj word's field), the packed key's W
        const uint32_t win = pk ? pf.jwin : kWindow;
        const uint32_t jb = sg.j[sb] - sg.j[sb] % win;
        size_t se = sb;
        uint64_t nw = 0;
        while (se < ns_all && sg.j[se] < jb + win) { nw += sg.end[se] - sg.beg[se]; ++se; }
        const uint32_t nseg = (uint32_t)(se - sb);
        const size_t s0 = sb;
        sb = se;
        if (nw == 0) continue;
        // host plan: segment bounds and changesets, level-1 tile prefix, the one-segment scan map
        // (the pinned staging buffer is reused: the previous window's copy must have run)
        if (s0 > 0) SYNCHK(c, c->stream);
        const size_t u32_words = (2 * (size_t)nseg + 2) / 2;        // seg_j [nseg] + tb [nseg + 1]
        const size_t words = 2 * (size_t)nseg + u32_words + 3;
        HIPALLOC(c->h_pplan.ensure(words));
        HIPALLOC(c->p_plan.ensure(words));
        uint64_t* h_beg = c->h_pplan.p;
        uint64_t* h_end = c->h_pplan.p + nseg;
        uint32_t* h_sj = reinterpret_cast<uint32_t*>(c->h_pplan.p + 2 * (size_t)nseg);
        uint32_t* tb = h_sj + nseg;
        uint32_t nt1 = 0;
        // level-1 tile (CRDT_L1_TILE, A/B): kPTile, whose level-1 histogram the scan counts; another size
        // (a multiple of 1024) takes the histogram pass
        const uint32_t l1t = !c->l1_tile ? l1_plan_tile(c) : c->l1_tile;
        for (uint32_t s = 0; s <= nseg; ++s) {
            tb[s] = nt1;
            if (s < nseg) {
                h_beg[s] = sg.beg[s0 + s];
                h_end[s] = sg.end[s0 + s];
                h_sj[s] = sg.j[s0 + s];
                nt1 += (uint32_t)((h_end[s] - h_beg[s] + l1t - 1) / l1t);
            }
        }
        const uint32_t nc1 = (nt1 + kChunkTiles - 1) / kChunkTiles;
        const size_t tail = 2 * (size_t)nseg + u32_words;
        uint32_t* sm_t = reinterpret_cast<uint32_t*>(c->h_pplan.p + tail);
        sm_t[0] = 0; sm_t[1] = nt1;                                   // scan tbase {0, nt1}
        uint32_t* sm_c = reinterpret_cast<uint32_t*>(c->h_pplan.p + tail + 1);
        sm_c[0] = 0; sm_c[1] = nc1;                                   // scan cbase {0, nc1}
        c->h_pplan.p[tail + 2] = 0;                                   // seg_pos {0}
        HIPCHK(hipMemcpyAsync(c->p_plan.p, c->h_pplan.p, words * sizeof(uint64_t), hipMemcpyHostToDevice,
                              c->stream));
        const uint32_t nt2 = two ? (uint32_t)((nw + kPTile2 - 1) / kPTile2) + kDigits : 0;
        const uint32_t nc2 = two ? (nt2 + kChunkTiles - 1) / kChunkTiles + kDigits : 0;
        const uint32_t ntm = std::max(nt1, nt2), ncm = std::max(nc1, nc2);
        HIPALLOC(c->p_hist.ensure((size_t)ntm * kDigits));
        HIPALLOC(c->p_toff.ensure((size_t)ntm * kDigits));
        HIPALLOC(c->p_part.ensure((size_t)ncm * kDigits));
        HIPALLOC(c->p_choff.ensure((size_t)ncm * kDigits));
        HIPALLOC(c->p_dstart1.ensure(kDigits + 1));
        // the partition buffers hold this form's records: packed payloads 12 B (Rec12), key columns 2 B at
        // level 1 (k16) and 1 B at level 2 (k8); the wide form 16 + 4 B
        const size_t rec_units = (pk ? (3 * (size_t)nw + 3) / 4 : (size_t)nw) + kPartPad;      // u32x4
        const size_t kj1_units = (k16 ? ((size_t)nw + 1) / 2 : (size_t)nw) + kPartPad;          // uint32
        const size_t kj2_units = (k8 ? ((size_t)nw + 3) / 4 : (size_t)nw) + kPartPad;
        // a placement trial (PlaceTune): candidate place_trial stands in as p1 for this call, every window
        // of it (swapped back in place_finish); the candidates are taken by the warm-up merge, sized for its
        // form and capped (place_take)
        if (c->place_k > 1 && c->place_trial < 0 && !c->has_comm && s0 == 0 && !c->place_warm) {
            c->place_warm = true;
            place_take(c, rec_units, kj1_units);
        }
        if (c->place_k > 1 && c->place_trial >= 0 && c->place_trial < 2 * c->place_k && !c->has_comm && s0 == 0 &&
            !c->place_timed) {
            const int k = c->place_trial % c->place_k;
            if (k) {                                  // (grown like p1 itself when this call holds more records)
                HIPALLOC(c->pc_rec[k].ensure(rec_units));
                HIPALLOC(c->pc_kj[k].ensure(kj1_units));
                std::swap(c->p1_rec, c->pc_rec[k]);
                std::swap(c->p1_kj, c->pc_kj[k]);
            }
            for (hipEvent_t& e : c->place_ev)
                if (!e) HIPCHK(hipEventCreate(&e));
            c->place_timed = true;
        }
        HIPALLOC(c->p1_rec.ensure(rec_units)); HIPALLOC(c->p1_kj.ensure(kj1_units));
        u32x4* p1r = c->p1_rec.p;
        uint32_t* p1k = c->p1_kj.p;
        u32x4* p2r = nullptr;
        uint32_t* p2k = nullptr;
        const uint64_t* d_beg = c->p_plan.p;
        const uint64_t* d_end = c->p_plan.p + nseg;
        const uint32_t* d_sj = reinterpret_cast<const uint32_t*>(c->p_plan.p + 2 * (size_t)nseg);
        const uint32_t* d_tb1 = d_sj + nseg;
        HIPALLOC(c->p_tseg.ensure(ntm));
        k_seg_index<<<std::min<uint32_t>(grid_for(nt1, 256), 4096), 256, 0, c->stream>>>(d_tb1, nseg, nt1, c->p_tseg.p);
        const TileMap tm1{d_beg, d_end, d_tb1, c->p_tseg.p, d_sj, nseg, l1t};
        const ScanMap sm1{reinterpret_cast<const uint32_t*>(c->p_plan.p + tail),
                          reinterpret_cast<const uint32_t*>(c->p_plan.p + tail + 1), c->p_plan.p + tail + 2, 1};
        if (two) HIPALLOC(c->p_l1beg.ensure(kDigits + 1));
        // level-1 histogram: counted by the scan (then only the changesets >= stop are cleared)
        // or here
        // (the same key map — not route_l1's owner-major one, ADVICE r4 — and the same tile boundaries)
        const bool h1 = c->hist1_fused && !c->hist1_routed && s0 == 0 && se == ns_all && !cols.packed_in &&
                        cols.key == c->hist1_key && c->hist1_shift == shift1 && nt1 == c->plan_ptiles &&
                        l1t == l1_plan_tile(c);
        const uint32_t* hist1 = h1 ? c->p_hist1.p : c->p_hist.p;
        if (h1)
            k_hist_trim<<<256, 256, 0, c->stream>>>(c->p_hist1.p, c->d_ptb, R, c->d_misc);
        else
            k_part_hist<true><<<nt1, kHThreads, 0, c->stream>>>(cols.key, tm1, jb, c->d_misc,
                                                                 c->cap, shift1, c->p_hist.p);
        c->last_hist1_fused = h1;
        k_scan_part<<<nc1, 256, 0, c->stream>>>(hist1, sm1, c->p_part.p);
        k_scan_seg<<<1, 256, 0, c->stream>>>(c->p_part.p, sm1, c->p_choff.p, c->p_dstart1.p,
                                             two ? c->p_l1beg.p : nullptr);
        k_scan_tiles<<<nc1, 256, 0, c->stream>>>(hist1, c->p_choff.p, sm1, c->p_dstart1.p, c->p_toff.p);
        const bool ph = c->timing && s0 == 0 && !em;   // phase events: the first window
        if (ph) ev_record(c, ev_window(1, false));
        if (c->place_timed && s0 == 0) HIPCHK(hipEventRecord(c->place_ev[0], c->stream));   // (the first window)
        const uint32_t xper1 = c->xcd_map ? (nt1 + kXcds - 1) / kXcds : 0;
        const bool rev1 = c->xcd_map && !(c->form_off & kFormNoReverse);
        if (pt1) HIPALLOC(c->f_pos1.ensure((size_t)nt1 * kPTile + 16));   // tile t's positions at t * kPTile
        if (pt1)                // ... tile-strided, stored from registers
            k_part_scatter1<true, false, true, kL1Items, true, true, true, true, true>
                <<<xcd_grid(nt1, c->xcd_map), kPThreads, 0, c->stream>>>(
                cols.key, cols.lt, cols.rank, cols.val, tm1, jb, c->d_misc, c->cap, shift1, c->p_toff.p, p1r,
                p1k, xper1, pf, rev1 ? hist1 : nullptr, c->f_pos1.p, hist1);
        else if (cmp && fl)     // the compact form's flagged level 1 (with positions)
            k_part_scatter1<true, false, true, kL1Items, true, true, true, true>
                <<<xcd_grid(nt1, c->xcd_map), kPThreads, 0, c->stream>>>(
                cols.key, cols.lt, cols.rank, cols.val, tm1, jb, c->d_misc, c->cap, shift1, c->p_toff.p, p1r,
                p1k, xper1, pf, rev1 ? hist1 : nullptr, c->f_pos1.p, hist1);
        else if (cmp)           // the compact form: 12-B records + the 1-B level-2 digit column
            k_part_scatter1<true, false, true, kL1Items, true, true, false, true>
                <<<xcd_grid(nt1, c->xcd_map), kPThreads, 0, c->stream>>>(
                cols.key, cols.lt, cols.rank, cols.val, tm1, jb, c->d_misc, c->cap, shift1, c->p_toff.p, p1r,
                p1k, xper1, pf, rev1 ? hist1 : nullptr);
        else if (fl && k16)     // the flagged form: each record's level-1 position kept at its input index
            k_part_scatter1<true, false, true, kL1Items, true, true, true>
                <<<xcd_grid(nt1, c->xcd_map), kPThreads, 0, c->stream>>>(
                cols.key, cols.lt, cols.rank, cols.val, tm1, jb, c->d_misc, c->cap, shift1, c->p_toff.p, p1r,
                p1k, xper1, pf, rev1 ? hist1 : nullptr, c->f_pos1.p, hist1);
        else if (fl)
            k_part_scatter1<true, false, false, kL1Items, true, false, true>
                <<<xcd_grid(nt1, c->xcd_map), kPThreads, 0, c->stream>>>(
                cols.key, cols.lt, cols.rank, cols.val, tm1, jb, c->d_misc, c->cap, shift1, c->p_toff.p, p1r,
                p1k, xper1, pf, rev1 ? hist1 : nullptr, c->f_pos1.p, hist1);
        else if (cols.packed_in && k16)
            k_part_scatter1<true, true, true, kL1Items, true><<<xcd_grid(nt1, c->xcd_map), kPThreads, 0, c->stream>>>(
                cols.key, cols.lt, cols.rank, cols.val, tm1, jb, c->d_misc, c->cap, shift1, c->p_toff.p, p1r,
                p1k, xper1, pf, rev1 ? hist1 : nullptr);
        else if (cols.packed_in)
            k_part_scatter1<true, true, false, kL1Items, true><<<xcd_grid(nt1, c->xcd_map), kPThreads, 0, c->stream>>>(
                cols.key, cols.lt, cols.rank, cols.val, tm1, jb, c->d_misc, c->cap, shift1, c->p_toff.p, p1r,
                p1k, xper1, pf, rev1 ? hist1 : nullptr);
        else if (k16 && !(c->form_off & kFormNoVecLoads))
            k_part_scatter1<true, false, true, kL1Items, true><<<xcd_grid(nt1, c->xcd_map), kPThreads, 0, c->stream>>>(
                cols.key, cols.lt, cols.rank, cols.val, tm1, jb, c->d_misc, c->cap, shift1, c->p_toff.p, p1r,
                p1k, xper1, pf, rev1 ? hist1 : nullptr);
        else if (k16)
            k_part_scatter1<true, false, true><<<xcd_grid(nt1, c->xcd_map), kPThreads, 0, c->stream>>>(
                cols.key, cols.lt, cols.rank, cols.val, tm1, jb, c->d_misc, c->cap, shift1, c->p_toff.p, p1r,
                p1k, xper1, pf, rev1 ? hist1 : nullptr);
        else if (pk)
            k_part_scatter1<true, false, false, kL1Items, true><<<xcd_grid(nt1, c->xcd_map), kPThreads, 0, c->stream>>>(
                cols.key, cols.lt, cols.rank, cols.val, tm1, jb, c->d_misc, c->cap, shift1, c->p_toff.p, p1r,
                p1k, xper1, pf, rev1 ? hist1 : nullptr);
        else
            k_part_scatter1<false, false, false, kL1Items, true><<<xcd_grid(nt1, c->xcd_map), kPThreads, 0, c->stream>>>(
                cols.key, cols.lt, cols.rank, cols.val, tm1, jb, c->d_misc, c->cap, shift1, c->p_toff.p, p1r,
                p1k, xper1, pf, rev1 ? hist1 : nullptr);
        if (ph) ev_record(c, ev_window(1, true));
        if (c->place_timed && s0 == 0) HIPCHK(hipEventRecord(c->place_ev[1], c->stream));
        if (ph) ev_record(c, ev_window(2, false));
        TileMap tm2f{};                              // level 2's tiling and counts (the flag pass)
        uint32_t nt2f = 0;
        const uint32_t* h2f = nullptr;
        const uint32_t* t2f = nullptr;
        if (two) {
            HIPALLOC(c->p_l2map.ensure(2 * (kDigits + 1)));
            HIPALLOC(c->p_dstart2.ensure(kDigits * kDigits + 1));
            HIPALLOC(c->p2_rec.ensure(rec_units)); HIPALLOC(c->p2_kj.ensure(kj2_units));
            p2r = c->p2_rec.p;
            p2k = c->p2_kj.p;
            uint32_t* tb2 = c->p_l2map.p;
            uint32_t* cb2 = c->p_l2map.p + kDigits + 1;
            // level-2 tiles of the packed form: kPTile2 records (one sub-tile each) — 256 workgroups
            // then cover a short stretch of each level-1 bucket at a time
            const uint32_t ts2 = k16 && !(c->form_off & kFormNoHistW) && !(c->form_off & kFormBigTile2)
                                 ? (uint32_t)kPTile2 : (uint32_t)kPTile;
            // (the flagged form keeps level 1's tile histogram and offsets for its flag pass: level 2
            // counts into buffers of its own)
            if (fl) {
                HIPALLOC(c->f_hist2.ensure((size_t)nt2 * kDigits));
                HIPALLOC(c->f_toff2.ensure((size_t)nt2 * kDigits));
            }
            uint32_t* h2p = fl ? c->f_hist2.p : c->p_hist.p;
            uint32_t* t2p = fl ? c->f_toff2.p : c->p_toff.p;
            h2f = h2p;
            t2f = t2p;
            k_l2_plan<<<1, 256, 0, c->stream>>>(c->p_l1beg.p, tb2, cb2, ts2);
            k_seg_index<<<std::min<uint32_t>(grid_for(nt2, 256), 4096), 256, 0, c->stream>>>(tb2, kDigits, nt2,
                                                                                            c->p_tseg.p);
            const TileMap tm2{c->p_l1beg.p, c->p_l1beg.p + 1, tb2, c->p_tseg.p, nullptr, kDigits, ts2};
            tm2f = tm2;
            nt2f = (uint32_t)((nw + ts2 - 1) / ts2) + kDigits;
            const ScanMap sm2{tb2, cb2, c->p_l1beg.p, kDigits};
            if (cmp)                                     // the compact form's 1-B level-2 digits
                k_part_hist16w<256, kPTile2, true><<<nt2, 256, 0, c->stream>>>(
                    reinterpret_cast<const uint16_t*>(p1k), tm2, 0, h2p);
            else if (k16 && !(c->form_off & kFormNoHistW) && ts2 == (uint32_t)kPTile2)   // key bits [4, 20) in 2 B:
                k_part_hist16w<256, kPTile2><<<nt2, 256, 0, c->stream>>>(   // the level-2 digit (bits [12, 20))
                    reinterpret_cast<const uint16_t*>(p1k), tm2, kSBits - 4, h2p);   // is its high byte
            else if (k16 && !(c->form_off & kFormNoHistW))
                k_part_hist16w<<<nt2, kHThreads, 0, c->stream>>>(
                    reinterpret_cast<const uint16_t*>(p1k), tm2, kSBits - 4, h2p);
            else if (k16)
                k_part_hist<false, true><<<nt2, kHThreads, 0, c->stream>>>(p1k, tm2, 0, c->d_misc, c->cap,
                                                                          kSBits - 4, h2p);
            else
                k_part_hist<false><<<nt2, kHThreads, 0, c->stream>>>(p1k, tm2, 0, c->d_misc, c->cap, kSBits,
                                                                      h2p);
            k_scan_part<<<nc2, 256, 0, c->stream>>>(h2p, sm2, c->p_part.p);
            k_scan_seg<<<kDigits, 256, 0, c->stream>>>(c->p_part.p, sm2, c->p_choff.p, c->p_dstart2.p, nullptr);
            k_scan_tiles<<<nc2, 256, 0, c->stream>>>(h2p, c->p_choff.p, sm2, c->p_dstart2.p, t2p);
            // (nt2 is an upper bound of the level-2 tiles; the real count is on the device)
            // (the grid and the XCD-contiguous mapping from a tile bound for THIS tile size: a loose
            // bound would leave the upper XCDs' ranges past the last tile, idle)
            const uint32_t nt2s = (uint32_t)((nw + ts2 - 1) / ts2) + kDigits;
            const uint32_t xper2 = c->xcd_map ? (nt2s + kXcds - 1) / kXcds : 0;
            if (ord) {         // changeset order kept in every final bucket; level-2 run offsets kept
                if (fl) HIPALLOC(c->f_pos2.ensure(nw + 8));
                uint16_t* pos2 = fl ? c->f_pos2.p : nullptr;
                const Rec12* i12 = reinterpret_cast<const Rec12*>(p1r);
                Rec12* o12 = reinterpret_cast<Rec12*>(p2r);
                const uint32_t jm = (uint32_t)pack_jmask(pf);
                if (cmp)
                    k_part_scatter2_seg<true, true, true><<<xcd_grid(nt2s, c->xcd_map), kPThreads, 0, c->stream>>>(
                        i12, nullptr, tm2, 24, t2p, o12, nullptr, xper2, jm, pos2, h2p);
                else if (k16)
                    k_part_scatter2_seg<true, true><<<xcd_grid(nt2s, c->xcd_map), kPThreads, 0, c->stream>>>(
                        i12, p1k, tm2, kSBits - 4, t2p, o12, p2k, xper2, jm, pos2, h2p);
                else if (k8)
                    k_part_scatter2_seg<true, false><<<xcd_grid(nt2s, c->xcd_map), kPThreads, 0, c->stream>>>(
                        i12, p1k, tm2, kSBits, t2p, o12, p2k, xper2, jm, pos2, h2p);
                else
                    k_part_scatter2_seg<false, false><<<xcd_grid(nt2s, c->xcd_map), kPThreads, 0, c->stream>>>(
                        i12, p1k, tm2, kSBits, t2p, o12, p2k, xper2, jm, pos2, h2p);
            } else if (c->counts)
                k_part_scatter2<true, false><<<xcd_grid(nt2s, c->xcd_map), kPThreads, 0, c->stream>>>(
                    p1r, p1k, tm2, kSBits, t2p, p2r, p2k, xper2, rev1 ? h2p : nullptr);
            else if (pk)
                if (cmp)       // (the record moves as it is: its digit is the word's top byte)
                    k_part_scatter2<false, true, true, true, true, true>
                        <<<xcd_grid(nt2s, c->xcd_map), kPThreads, 0, c->stream>>>(
                        p1r, nullptr, tm2, 24, t2p, p2r, nullptr, xper2, rev1 ? h2p : nullptr);
                else if (k16)
                    k_part_scatter2<false, true, true, true><<<xcd_grid(nt2s, c->xcd_map), kPThreads, 0, c->stream>>>(
                        p1r, p1k, tm2, kSBits - 4, t2p, p2r, p2k, xper2, rev1 ? h2p : nullptr);
                else if (k8)
                    k_part_scatter2<false, true, true><<<xcd_grid(nt2s, c->xcd_map), kPThreads, 0, c->stream>>>(
                        p1r, p1k, tm2, kSBits, t2p, p2r, p2k, xper2, rev1 ? h2p : nullptr);
                else
                    k_part_scatter2<false, true><<<xcd_grid(nt2s, c->xcd_map), kPThreads, 0, c->stream>>>(
                        p1r, p1k, tm2, kSBits, t2p, p2r, p2k, xper2, rev1 ? h2p : nullptr);
            else
                k_part_scatter2<false, false><<<xcd_grid(nt2s, c->xcd_map), kPThreads, 0, c->stream>>>(
                    p1r, p1k, tm2, kSBits, t2p, p2r, p2k, xper2, rev1 ? h2p : nullptr);
        }
        if (ph) ev_record(c, ev_window(2, true));
        // resolve: items = parts of buckets (hot buckets split into kRPart-record parts)
        const uint32_t nb = two ? kDigits * kDigits : kDigits;
        const uint32_t* bst = two ? c->p_dstart2.p : c->p_dstart1.p;
        const u32x4* rec = two ? p2r : p1r;
        const uint32_t* rv = two ? p2k : p1k;
        const uint32_t max_items = nb + (uint32_t)(nw / kRPart) + 1;
        const size_t ksn = (size_t)(2 * (nw / kRPart) + 2) * kSKeys;     // part-state slots of split buckets
        const uint32_t max_hot = std::min<uint32_t>(nb, (uint32_t)(nw / kRPart) + 1);   // split buckets hold > kRPart
        HIPALLOC(c->p_ibase.ensure(2 * (nb + 1) + 1 + max_hot));
        HIPALLOC(c->p_kslt.ensure(2 * ksn));
        HIPALLOC(c->p_ksu32.ensure(6 * ksn));
        uint32_t* d_ib = c->p_ibase.p;
        uint32_t* d_hb = c->p_ibase.p + nb + 1;
        uint32_t* d_hot = c->p_ibase.p + 2 * (nb + 1);                           // [0] count, [1..] buckets
        KeyState ps{c->p_kslt.p, c->p_ksu32.p, c->p_ksu32.p + ksn, c->p_ksu32.p + 2 * ksn};
        KeyState cy{c->p_kslt.p + ksn, c->p_ksu32.p + 3 * ksn, c->p_ksu32.p + 4 * ksn, c->p_ksu32.p + 5 * ksn};
        HIPALLOC(c->p_ibucket.ensure(max_items));
        // split buckets (parts folded apart, then carried) beside the unsplit buckets' resolve: two streams
        const bool ov = !em && pk && (ord || !c->counts) && two && (c->form_off & kFormOverlap);
        if (ph) ev_record(c, ev_window(3, false));
        if (em) HIPALLOC(c->e_bbase.ensure(nb));
        k_bucket_items<<<(nb + 1023) / 1024, 1024, 0, c->stream>>>(bst, nb, d_ib, d_hb, d_hot, c->d_misc,
                                                                    em ? c->e_bbase.p : nullptr);
        k_seg_index<<<std::min<uint32_t>(grid_for(max_items, 256), 4096), 256, 0, c->stream>>>(d_ib, nb, max_items,
                                                                                               c->p_ibucket.p);
        // k_item_lists, then the host's wait for its counts (the packed resolve's kernels on exactly their items)
        auto item_lists = [&](uint64_t hw_s, uint32_t sparse_s, uint32_t* n_fold, uint32_t* n_dense, uint32_t* n_sparse,
                              uint32_t* n_hot, uint32_t* n_items) -> int {
            HIPALLOC(c->p_ilist.ensure(kListHead + 3 * (size_t)max_items));
            HIPALLOC(c->h_ilist.ensure(kListHead));
            k_item_lists<<<(nb + 1023) / 1024, 1024, 0, c->stream>>>(bst, nb, d_ib, d_hb, d_hot, hw_s, sparse_s,
                                                                    c->p_ilist.p, max_items);
            HIPCHK(hipMemcpyAsync(c->h_ilist.p, c->p_ilist.p, kListHead * sizeof(uint32_t), hipMemcpyDeviceToHost,
                                  c->stream));
            HIPCHK(hipStreamSynchronize(c->stream));
            const uint32_t* h = c->h_ilist.p;
            if (h[0] > max_items || h[1] > max_items || h[2] > max_items || h[3] > max_hot || h[4] > max_items)
                return CRDT_E_HIP;                              // (cannot happen: the lists hold <= max_items)
            *n_fold = h[0]; *n_dense = h[1]; *n_sparse = h[2]; *n_hot = h[3]; *n_items = h[4];
            return CRDT_OK;
        };
        if (em) {          // map-side combine: part folds, then every key's maximum emitted
            // emit items: the resolve's max_items, then 16 carry blocks per hot bucket; the slots are the
            // buckets' (k_bucket_items' ebase: min(kSKeys, records) each), so at most min(records, key range)
            const uint32_t n_items = max_items + max_hot * (kSKeys / 256);
            const size_t slots = (size_t)std::min<uint64_t>(nw, (uint64_t)nb * kSKeys) + 1;
            HIPALLOC(c->e_key.ensure(slots));
            HIPALLOC(c->e_pk.ensure(slots));
            HIPALLOC(c->e_val.ensure(slots));
            HIPALLOC(c->e_icnt.ensure((size_t)n_items * (2 + emit->G)));
            HIPCHK(hipMemsetAsync(c->e_icnt.p, 0, (size_t)n_items * (2 + emit->G) * sizeof(uint32_t), c->stream));
            emit->key = c->e_key.p;
            emit->pk = c->e_pk.p;
            emit->val = c->e_val.p;
            emit->bbase = c->e_bbase.p;
            emit->icount = c->e_icnt.p;
            emit->ibase = c->e_icnt.p + n_items;
            emit->ocount = c->e_icnt.p + 2 * (size_t)n_items;
            emit->item0 = max_items;
            emit->n_items = n_items;
            uint64_t* ps_key = reinterpret_cast<uint64_t*>(c->p_kslt.p);
            uint32_t* ps_val = c->p_ksu32.p;
            const Rec12* rec12 = reinterpret_cast<const Rec12*>(rec);
            if (k8) {
                k_resolve_packed<true, true, true><<<max_items, kQThreads, 0, c->stream>>>(
                    bst, d_ib, d_hb, c->p_ibucket.p, nb, rec12, rv, c->table, c->cap, 0, c->d_Rj.p, jb, ps_key, ps_val,
                    pf, c->d_misc);
                k_resolve_packed<false, false, true, true><<<max_items, kQThreads, 0, c->stream>>>(
                    bst, d_ib, d_hb, c->p_ibucket.p, nb, rec12, rv, c->table, c->cap, 0, c->d_Rj.p, jb, ps_key, ps_val,
                    pf, c->d_misc, *emit);
            } else {
                k_resolve_packed<true><<<max_items, kQThreads, 0, c->stream>>>(
                    bst, d_ib, d_hb, c->p_ibucket.p, nb, rec12, rv, c->table, c->cap, 0, c->d_Rj.p, jb, ps_key, ps_val,
                    pf, c->d_misc);
                k_resolve_packed<false, false, false, true><<<max_items, kQThreads, 0, c->stream>>>(
                    bst, d_ib, d_hb, c->p_ibucket.p, nb, rec12, rv, c->table, c->cap, 0, c->d_Rj.p, jb, ps_key, ps_val,
                    pf, c->d_misc, *emit);
            }
            k_part_carry_packed<true><<<dim3(kSKeys / 256, max_hot), 256, 0, c->stream>>>(
                d_hot, d_ib, d_hb, c->table, c->cap, 0, ps_key, ps_val, c->d_Rj.p, jb, pf, c->d_misc, *emit);
        } else if (ord) {  // the ordered packed resolve: flags and / or counts (sorted_path.inc, "win flags")
            uint64_t* ps_key = reinterpret_cast<uint64_t*>(c->p_kslt.p);
            uint32_t* ps_val = c->p_ksu32.p;
            const Rec12* rec12 = reinterpret_cast<const Rec12*>(rec);
            HIPALLOC(c->f_cin_key.ensure(ksn));
            HIPALLOC(c->f_cin_val.ensure(ksn));
            HIPALLOC(c->f_cin_pres.ensure(ksn));
            if (fl) HIPALLOC(c->f_flag2.ensure(nw + 8));
            uint8_t* fl2 = fl ? c->f_flag2.p : nullptr;
            // the split buckets' part folds and carry-ins on the side stream, beside the unsplit buckets' ordered
            // resolve (disjoint buckets: their rows, states and flags do not meet); then the split buckets' walk
            // the fold and the carry-ins on exactly their items (k_item_lists), the walk on the items there are
            int st = CRDT_OK;
            uint32_t g_fold = max_items, g_hot = max_hot, g_items = max_items, g_d, g_s;
            const uint32_t* l_fold = nullptr;
            if (!c->has_comm && !(c->form_off & kFormNoItemLists)) {
                if ((st = item_lists(0, 0, &g_fold, &g_d, &g_s, &g_hot, &g_items))) return st;
                l_fold = c->p_ilist.p + kListHead;
            }
            if ((st = ov ? overlap_fork(c) : CRDT_OK)) return st;
            const hipStream_t fs = ov ? c->sstream : c->stream;
            if (!g_fold) {
            } else if (cmp)
                k_resolve_packed<true, true, false, false, true><<<g_fold, kQThreads, 0, fs>>>(
                    bst, d_ib, d_hb, c->p_ibucket.p, nb, rec12, nullptr, c->table, c->cap, c->hw_read, c->d_Rj.p, jb,
                    ps_key, ps_val, pf, c->d_misc, EmitOut{}, 0, false, l_fold);
            else if (k8)
                k_resolve_packed<true, true, true><<<g_fold, kQThreads, 0, fs>>>(
                    bst, d_ib, d_hb, c->p_ibucket.p, nb, rec12, rv, c->table, c->cap, c->hw_read, c->d_Rj.p, jb, ps_key,
                    ps_val, pf, c->d_misc, EmitOut{}, 0, false, l_fold);
            else
                k_resolve_packed<true><<<g_fold, kQThreads, 0, fs>>>(
                    bst, d_ib, d_hb, c->p_ibucket.p, nb, rec12, rv, c->table, c->cap, c->hw_read, c->d_Rj.p, jb, ps_key,
                    ps_val, pf, c->d_misc, EmitOut{}, 0, false, l_fold);
            if (g_hot)
                k_part_cin_packed<<<dim3(kSKeys / 256, g_hot), 256, 0, fs>>>(
                    d_hot, d_ib, d_hb, c->table, c->cap, c->hw_read, ps_key, ps_val, pf, c->d_misc,
                    reinterpret_cast<uint64_t*>(c->f_cin_key.p), c->f_cin_val.p, c->f_cin_pres.p);
            const uint64_t* cink = reinterpret_cast<const uint64_t*>(c->f_cin_key.p);
            for (uint32_t which = ov ? 1u : 0u; which <= (ov ? 2u : 0u); ++which) {
                if (which == 2 && (st = overlap_join(c))) return st;
                if (!g_items) {
                } else if (cmp)
                    k_resolve_pflags<false, true><<<g_items, kRThreads, 0, c->stream>>>(
                        bst, d_ib, d_hb, c->p_ibucket.p, nb, rec12, nullptr, c->table, c->cap, c->hw_read, c->d_Rj.p,
                        jb, cink, c->f_cin_val.p, c->f_cin_pres.p, pf, c->d_misc, fl2, which);
                else if (k8)
                    k_resolve_pflags<true><<<g_items, kRThreads, 0, c->stream>>>(
                        bst, d_ib, d_hb, c->p_ibucket.p, nb, rec12, rv, c->table, c->cap, c->hw_read, c->d_Rj.p, jb,
                        cink, c->f_cin_val.p, c->f_cin_pres.p, pf, c->d_misc, fl2, which);
                else
                    k_resolve_pflags<false><<<g_items, kRThreads, 0, c->stream>>>(
                        bst, d_ib, d_hb, c->p_ibucket.p, nb, rec12, rv, c->table, c->cap, c->hw_read, c->d_Rj.p, jb,
                        cink, c->f_cin_val.p, c->f_cin_pres.p, pf, c->d_misc, fl2, which);
            }
            // flags back: level-2 order -> level-1 order (two levels) -> input order
            const uint8_t* f1 = c->f_flag2.p;
            if (fl && two) {
                HIPALLOC(c->f_flag1.ensure(nw + 8));
                const bool fx = c->xcd_map && (c->form_off & kFormFbackXcd);
                const uint32_t xf2 = fx ? (nt2f + kXcds - 1) / kXcds : 0;
#define CRDT_FBACK2(CHK, W)                                                                               \
    if (tm2f.tsize == (uint32_t)kPTile2)                                                                  \
        k_flags_back<false, CHK, kPTile2, W><<<xcd_grid(nt2f, fx), 512, 0, c->stream>>>(                  \
            tm2f, h2f, t2f, c->f_pos2.p, c->f_flag2.p, c->f_flag1.p, c->d_misc, xf2);                     \
    else                                                                                                  \
        k_flags_back<false, CHK, kPTile, W><<<xcd_grid(nt2f, fx), 512, 0, c->stream>>>(                   \
            tm2f, h2f, t2f, c->f_pos2.p, c->f_flag2.p, c->f_flag1.p, c->d_misc, xf2)
                const bool pre2 = !(c->form_off & (kFormNoFbackPre | kFormFbackWide)) && !fx &&
                                  tm2f.tsize == (uint32_t)kPTile2;
                if (pre2 && (c->form_off & kFormFbackPre512))
                    k_flags_back_pre<false, 6, kPTile2, 16><<<nt2f, 512, 0, c->stream>>>(
                        tm2f, h2f, t2f, c->f_pos2.p, c->f_flag2.p, c->f_flag1.p, c->d_misc);
                else if (pre2)
                    k_flags_back_pre<false, 6, kPTile2, 32, 256><<<nt2f, 256, 0, c->stream>>>(
                        tm2f, h2f, t2f, c->f_pos2.p, c->f_flag2.p, c->f_flag1.p, c->d_misc);
                else if (c->form_off & kFormFbackWide) { CRDT_FBACK2(6, true); }
                else if (c->fback_chk == 4) { CRDT_FBACK2(4, false); }
                else if (c->fback_chk == 6) { CRDT_FBACK2(6, false); }
                else { CRDT_FBACK2(0, false); }
#undef CRDT_FBACK2
                f1 = c->f_flag1.p;
                // level 2 reused the tile -> segment index: rebuild level 1's
                k_seg_index<<<std::min<uint32_t>(grid_for(nt1, 256), 4096), 256, 0, c->stream>>>(d_tb1, nseg, nt1,
                                                                                                 c->p_tseg.p);
            }
            const bool fx1 = c->xcd_map && (c->form_off & kFormFbackXcd);
            const uint32_t xf1 = fx1 ? (nt1 + kXcds - 1) / kXcds : 0;
#define CRDT_FBACK1(CHK, W)                                                                               \
    k_flags_back<true, CHK, kPTile, W><<<xcd_grid(nt1, fx1), 512, 0, c->stream>>>(                        \
        tm1, hist1, c->p_toff.p, c->f_pos1.p, f1, dflags, c->d_misc, xf1)
            if (fl) {
                if (pt1)
                    k_flags_back_pre<true, 6, kPTile, 14, 512, true><<<nt1, 512, 0, c->stream>>>(
                        tm1, hist1, c->p_toff.p, c->f_pos1.p, f1, dflags, c->d_misc);
                else if (!(c->form_off & (kFormNoFbackPre | kFormFbackWide)) && !fx1)
                    k_flags_back_pre<true, 6, kPTile, 14><<<nt1, 512, 0, c->stream>>>(
                        tm1, hist1, c->p_toff.p, c->f_pos1.p, f1, dflags, c->d_misc);
                else if (c->form_off & kFormFbackWide) { CRDT_FBACK1(6, true); }
                else if (c->fback_chk == 4) { CRDT_FBACK1(4, false); }
                else if (c->fback_chk == 6) { CRDT_FBACK1(6, false); }
                else { CRDT_FBACK1(0, false); }
            }
#undef CRDT_FBACK1
        } else if (c->counts) {
            k_resolve<true><<<max_items, kRThreads, 0, c->stream>>>(bst, d_ib, d_hb, c->p_ibucket.p, nb, rec, rv,
                                                                    c->table, c->cap, c->d_Rj.p, jb, ps, cy, c->d_misc);
            k_part_carry<false><<<dim3(kSKeys / 256, max_hot), 256, 0, c->stream>>>(d_hot, d_ib, d_hb, c->table,
                                                                                    c->cap, ps, cy, c->d_Rj.p, jb, c->d_misc);
            k_resolve<false><<<max_items, kRThreads, 0, c->stream>>>(bst, d_ib, d_hb, c->p_ibucket.p, nb, rec, rv,
                                                                     c->table, c->cap, c->d_Rj.p, jb, ps, cy, c->d_misc);
        } else if (pk) {   // packed order-free form: one LDS 64-bit max per record (sorted_path.inc)
            uint64_t* ps_key = reinterpret_cast<uint64_t*>(c->p_kslt.p);
            uint32_t* ps_val = c->p_ksu32.p;
            const Rec12* rec12 = reinterpret_cast<const Rec12*>(rec);
            // the split buckets' part folds + carry (they write the split buckets' rows) on the side stream, beside
            // the unsplit buckets' resolve (the other rows): disjoint buckets, joined before the next window
            // the sparse buckets in k_resolve_sparse's small workgroups (the dense ones skip them)
            const bool spk = c->sparse_t > 0 && !(c->form_off & (kFormNoSparseK | kFormNoWholeLines));
            // each kernel on exactly its items (k_item_lists; the host waits for the four counts — by then the GPU is
            // at the resolve, and the launches below follow at once)
            int st = CRDT_OK;
            const bool lists = !c->has_comm && !(c->form_off & (kFormNoItemLists | kFormNoWholeLines));
            uint32_t g_fold = max_items, g_dense = max_items, g_sparse = max_items, g_hot = max_hot;
            const uint32_t *l_fold = nullptr, *l_dense = nullptr, *l_sparse = nullptr;
            if (lists) {
                uint32_t g_items;
                if ((st = item_lists(spk ? c->hw_read : 0, spk ? c->sparse_t : 0, &g_fold, &g_dense, &g_sparse, &g_hot,
                                     &g_items)))
                    return st;
                l_fold = c->p_ilist.p + kListHead;
                l_dense = l_fold + max_items;
                l_sparse = l_dense + max_items;
            }
            if ((st = ov ? overlap_fork(c) : CRDT_OK)) return st;
            const hipStream_t fs = ov ? c->sstream : c->stream;
            if (g_fold) {
                if (cmp)
                    k_resolve_packed<true, true, false, false, true><<<g_fold, kQThreads, 0, fs>>>(
                        bst, d_ib, d_hb, c->p_ibucket.p, nb, rec12, nullptr, c->table, c->cap, c->hw_read, c->d_Rj.p, jb,
                        ps_key, ps_val, pf, c->d_misc, EmitOut{}, 0, false, l_fold);
                else if (k8)
                    k_resolve_packed<true, true, true><<<g_fold, kQThreads, 0, fs>>>(
                        bst, d_ib, d_hb, c->p_ibucket.p, nb, rec12, rv, c->table, c->cap, c->hw_read, c->d_Rj.p, jb, ps_key,
                        ps_val, pf, c->d_misc, EmitOut{}, 0, false, l_fold);
                else
                    k_resolve_packed<true><<<g_fold, kQThreads, 0, fs>>>(
                        bst, d_ib, d_hb, c->p_ibucket.p, nb, rec12, rv, c->table, c->cap, c->hw_read, c->d_Rj.p, jb, ps_key,
                        ps_val, pf, c->d_misc, EmitOut{}, 0, false, l_fold);
            }
            if (g_hot)
                k_part_carry_packed<false><<<dim3(kSKeys / 256, g_hot), 256, 0, fs>>>(
                    d_hot, d_ib, d_hb, c->table, c->cap, c->hw_read, ps_key, ps_val, c->d_Rj.p, jb, pf, c->d_misc);
            if (!g_dense) {
            } else if (cmp)
                k_resolve_packed<false, true, false, false, true><<<g_dense, kQThreads, 0, c->stream>>>(
                    bst, d_ib, d_hb, c->p_ibucket.p, nb, rec12, nullptr, c->table, c->cap, c->hw_read, c->d_Rj.p, jb,
                    ps_key, ps_val, pf, c->d_misc, EmitOut{}, c->sparse_t, spk, l_dense);
            else if ((c->form_off & kFormNoWholeLines) && k8)      // (13-B records: 1-B key column)
                k_resolve_packed<false, false, true><<<max_items, kQThreads, 0, c->stream>>>(
                    bst, d_ib, d_hb, c->p_ibucket.p, nb, rec12, rv, c->table, c->cap, c->hw_read, c->d_Rj.p, jb, ps_key, ps_val,
                    pf, c->d_misc);
            else if (c->form_off & kFormNoWholeLines)
                k_resolve_packed<false, false><<<max_items, kQThreads, 0, c->stream>>>(
                    bst, d_ib, d_hb, c->p_ibucket.p, nb, rec12, rv, c->table, c->cap, c->hw_read, c->d_Rj.p, jb, ps_key, ps_val,
                    pf, c->d_misc);
            else if (k8)
                k_resolve_packed<false, true, true><<<g_dense, kQThreads, 0, c->stream>>>(
                    bst, d_ib, d_hb, c->p_ibucket.p, nb, rec12, rv, c->table, c->cap, c->hw_read, c->d_Rj.p, jb, ps_key, ps_val,
                    pf, c->d_misc, EmitOut{}, c->sparse_t, spk, l_dense);
            else
                k_resolve_packed<false><<<g_dense, kQThreads, 0, c->stream>>>(
                    bst, d_ib, d_hb, c->p_ibucket.p, nb, rec12, rv, c->table, c->cap, c->hw_read, c->d_Rj.p, jb, ps_key, ps_val,
                    pf, c->d_misc, EmitOut{}, c->sparse_t, spk, l_dense);
            if (!spk || !g_sparse) {
            } else if (cmp)
                k_resolve_sparse<false, true><<<g_sparse, kSpThreads, 0, c->stream>>>(
                    bst, d_ib, c->p_ibucket.p, nb, rec12, nullptr, c->table, c->hw_read, c->d_Rj.p, jb, pf, c->d_misc,
                    c->sparse_t, l_sparse);
            else if (k8)
                k_resolve_sparse<true, false><<<g_sparse, kSpThreads, 0, c->stream>>>(
                    bst, d_ib, c->p_ibucket.p, nb, rec12, rv, c->table, c->hw_read, c->d_Rj.p, jb, pf, c->d_misc,
                    c->sparse_t, l_sparse);
            else
                k_resolve_sparse<false, false><<<g_sparse, kSpThreads, 0, c->stream>>>(
                    bst, d_ib, c->p_ibucket.p, nb, rec12, rv, c->table, c->hw_read, c->d_Rj.p, jb, pf, c->d_misc,
                    c->sparse_t, l_sparse);
            if (ov && (st = overlap_join(c))) return st;
        } else {           // order-free list form; split buckets finished by k_part_carry<true>
            k_resolve<true, true><<<max_items, kRThreads, 0, c->stream>>>(bst, d_ib, d_hb, c->p_ibucket.p, nb, rec,
                                                                          rv, c->table, c->cap, c->d_Rj.p, jb, ps, cy,
                                                                          c->d_misc);
            k_part_carry<true><<<dim3(kSKeys / 256, max_hot), 256, 0, c->stream>>>(d_hot, d_ib, d_hb, c->table,
                                                                                   c->cap, ps, cy, c->d_Rj.p, jb, c->d_misc);
            k_resolve<false, true><<<max_items, kRThreads, 0, c->stream>>>(bst, d_ib, d_hb, c->p_ibucket.p, nb, rec,
                                                                           rv, c->table, c->cap, c->d_Rj.p, jb, ps, cy,
                                                                           c->d_misc);
        }
        if (ph) {
            ev_record(c, ev_window(3, true));
            c->sorted_phases = true;
            c->p1_records = nw;
        }
        HIPCHK(hipGetLastError());
        // the next window reads rows this one may have written anywhere below the capacity
        c->hw_read = c->cap;
    }
    if (em) return CRDT_OK;
    if (c->timing) {
        ev_record(c, ev_window(0, true));
        c->windows.push_back(1u);
    }
    HIPCHK(hipGetLastError());
#ifdef CRDT_PROF_RESOLVE
    HIPCHK(hipStreamSynchronize(c->stream));
    prof_resolve_report();
#endif
    return finish_apply(c, nullptr, nullptr, 0, true, out);
}

// The sorted path runs for crdt_merge when its preconditions hold (sorted_path.inc
// header) and either CRDT_MERGE_PATH=sorted or the batch is a multi-changeset fan-in
// large enough to amortise the partition passes.  R = changesets of the call.
bool use_sorted(const crdt_ctx* c, const Segs& sg, uint32_t R, const uint8_t* win_flags) {
    if (c->merge_path == 1 || c->canonical < 0 || c->cap > kSortedMaxCap) return false;
    // per-record win flags: the flagged form (packed records, one ctx; apply_segs checks the frame)
    if (win_flags && (!c->flags_sorted || !c->packed_resolve)) return false;
    uint64_t n = 0, nw = 0;
    uint32_t jb = 0;
    for (size_t s = 0; s < sg.j.size(); ++s) {              // < 2^31 records per kWindow changesets
        if (sg.j[s] >= jb + kWindow) { jb = sg.j[s] - sg.j[s] % kWindow; nw = 0; }
        nw += sg.end[s] - sg.beg[s];
        n += sg.end[s] - sg.beg[s];
        if (nw >= (1ull << 31)) return false;
    }
    if (c->merge_path == 2) return true;
    // auto: a many-changeset fan-in.  Order-free (no per-record counts): the partitioned passes
    // beat R K2 launches from 64 changesets and 8M records on (1B fan-in: 31.4 vs 34.1 ms,
    // DESIGN.md §5); with exact counts only while changesets are small (cfg3), where K2's
    // launches are latency-bound; the ordered packed form counts exactly (its resolve walks in
    // order) and serves flags — apply_segs sends a batch whose frame does not fit it to K2
    return R >= 64 && n >= (8ull << 20) &&
           (win_flags || !c->counts || c->packed_resolve || n / R <= (256ull << 10));
}

// Apply phase over columns whose changeset segments are c->segs (n = column length).
int apply_segs(crdt_ctx* c, const Cols& cols, uint64_t n, int32_t mem, int64_t wall, const long long* d_event,
               uint8_t* win_flags, crdt_result* out, bool allow_sorted) {
    if (c->timing) HIPCHK(ensure_events(c, events_for(c->segs.j.size())));
    c->last_sorted = allow_sorted && use_sorted(c, c->segs, c->plan_R, win_flags);
    c->last_flagged = false;
    // flags, or exact counts on large changesets (admitted for the ordered packed form): the scan's
    // frame must fit the packed key, else K2
    const uint64_t nrec = c->segs.j.empty() ? 0 : n;
    const bool big_cs = c->counts && c->merge_path != 2 && c->plan_R && nrec / c->plan_R > (256ull << 10);
    if (c->last_sorted && (win_flags || big_cs)) {
        bool ok = mem == CRDT_MEM_DEVICE && c->frame_on && !cols.packed_in;
        if (ok) {
            HIPCHK(hipMemcpyAsync(c->h_misc, c->d_misc, sizeof(Misc), hipMemcpyDeviceToHost, c->stream));
            SYNCHK(c, c->stream);
            ok = frame_of(c).ok;
        }
        c->last_sorted = ok;
    }
    if (c->last_sorted) {
        int st = kv_copy_all(c);
        if (st) return st;
        if (win_flags) {
            if (n) HIPCHK(hipMemsetAsync(win_flags, 0, n, c->stream));
            c->last_flagged = true;
        }
        return apply_sorted(c, cols, c->segs, wall, d_event, out, win_flags);
    }
    return apply_ranges(c, cols, c->segs, n, mem, wall, d_event, win_flags, out);
}

int phase_apply(crdt_ctx* c, const crdt_batch* owned, int64_t wall, const long long* d_event,
                uint8_t* win_flags, crdt_result* out, bool allow_sorted = false) {
    int st = validate_batch(owned);
    if (st) return st;
    const uint32_t R = c->plan_R;
    if (owned->n_changesets != R) return CRDT_E_INVALID;
    Cols cols;
    if ((st = stage_apply_cols(c, owned, &cols))) return st;
    c->segs.from_offsets(owned->offsets, R);
    return apply_segs(c, cols, owned->offsets[R], owned->mem, wall, d_event, win_flags, out, allow_sorted);
}

// After a merge's final synchronisation: the timed candidate's level-1 scatter; after the last trial, the
// fastest candidate becomes p1 for good and the others are freed.
void place_finish(crdt_ctx* c, bool ok) {
    if (c->place_warm) {
        c->place_warm = false;
        if (ok) c->place_trial = 0;
        return;
    }
    if (!c->place_timed) return;
    c->place_timed = false;
    const int k = c->place_trial % c->place_k;
    if (k) { std::swap(c->p1_rec, c->pc_rec[k]); std::swap(c->p1_kj, c->pc_kj[k]); }   // back in its slot
    float ms = 0.f;
    if (!ok || hipEventSynchronize(c->place_ev[1]) != hipSuccess ||
        hipEventElapsedTime(&ms, c->place_ev[0], c->place_ev[1]) != hipSuccess)
        return;                                   // (a failed call times nothing: the candidate is tried again)
    c->place_ms[k] = c->place_trial < c->place_k ? ms : std::min(c->place_ms[k], ms);
    if (++c->place_trial < 2 * c->place_k) return;
    int b = 0;
    for (int i = 1; i < c->place_k; ++i) b = c->place_ms[i] < c->place_ms[b] ? i : b;
    if (b) { std::swap(c->p1_rec, c->pc_rec[b]); std::swap(c->p1_kj, c->pc_kj[b]); }
    for (int i = 1; i < crdt_ctx::kPlaceMax; ++i) { c->pc_rec[i].release(); c->pc_kj[i].release(); }
    c->place_best = b;
}

void collect_timing(crdt_ctx* c) {
    crdt_timing t{};
    if (c->timing) {
        float ms = 0;
        auto el = [&](size_t a, size_t b) {
            return hipEventElapsedTime(&ms, c->events[a], c->events[b]) == hipSuccess ? (double)ms : 0.0;
        };
        t.scan_ms = el(kEvStart, kEvScan);
        t.clock_ms = el(kEvScan, kEvClock);
        t.route_ms = el(kEvClock, kEvApply);
        for (size_t k = 0; k < c->windows.size(); ++k) {
            t.apply_ms += el(ev_window(k, false), ev_window(k, true));
            t.apply_launches += c->windows[k];
        }
        t.apply_total = c->apply_total;
        t.total_ms = el(kEvStart, kEvEnd);
        if (c->last_sorted && c->sorted_phases) {
            t.part1_ms = el(ev_window(1, false), ev_window(1, true));
            t.part2_ms = el(ev_window(2, false), ev_window(2, true));
            t.resolve_ms = el(ev_window(3, false), ev_window(3, true));
            t.part1_records = c->p1_records;
        }
    }
    t.sent_bytes = c->sent_bytes;
    c->last_timing = t;
}

#include "comm_path.inc"

}  // namespace

// ============================================================== C-ABI entry points
extern "C" {

int crdt_abi_version(void) { return CRDT_ABI_VERSION; }

const char* crdt_status_string(int s) {
    switch (s) {
        case CRDT_OK: return "ok";
        case CRDT_CLOCK_DRIFT: return "clock drift";
        case CRDT_DUPLICATE_NODE: return "duplicate node";
        case CRDT_OVERFLOW: return "counter overflow";
        case CRDT_E_INVALID: return "invalid argument";
        case CRDT_E_HIP: return "HIP runtime error";
        case CRDT_E_NOMEM: return "device out of memory";
        case CRDT_E_KEY_RANGE: return "key id out of range";
        case CRDT_E_NO_DEVICE: return "no gfx950 device";
        case CRDT_E_COMM: return "communicator error";
        default: return "unknown status";
    }
}

int crdt_device_count(int* out) {
    if (!out) return CRDT_E_INVALID;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
    *out = n;
    return CRDT_OK;
}

// Tuning switches; with CRDT_ENV_DYNAMIC=1 re-read at every crdt_merge, so one
// process can alternate them step by step (A/B runs on one memory placement: tools/ab_steps.sh).
static void read_env_knobs(crdt_ctx* c) {
    if (const char* e = getenv("CRDT_NO_FUSE")) c->no_fuse = atoi(e) != 0;
    if (const char* e = getenv("CRDT_XCD_MAP")) c->xcd_map = atoi(e) != 0;
    if (const char* e = getenv("CRDT_PACKED")) c->packed_resolve = atoi(e) != 0;
    if (const char* e = getenv("CRDT_FLAGS_SORTED")) c->flags_sorted = atoi(e) != 0;
    if (const char* e = getenv("CRDT_COMBINE")) c->combine = std::min(std::max(atoi(e), 0), 2);
    if (const char* e = getenv("CRDT_ROUTE_L1")) c->route_l1 = std::min(std::max(atoi(e), 0), 3);
    if (const char* e = getenv("CRDT_RL1_SPLIT")) {   // 0: one piece, 1: two (the default), n: n pieces
        const int v = atoi(e);
        c->rl1_pieces = std::min<uint32_t>(v <= 0 ? 1u : v == 1 ? 2u : (uint32_t)v, kRl1MaxPieces);
    }
    if (const char* e = getenv("CRDT_ROUTE_TUNE")) c->route_tune = atoi(e) != 0;
    if (const char* e = getenv("CRDT_SPARSE_T")) c->sparse_t = (uint32_t)std::max(atoi(e), 0);
    if (const char* e = getenv("CRDT_FBACK_CHK")) c->fback_chk = atoi(e) == 4 ? 4 : atoi(e) == 0 ? 0 : 6;
    if (const char* e = getenv("CRDT_HIST_FUSE")) c->hist_fuse = atoi(e) != 0;
    if (const char* e = getenv("CRDT_L1_TILE"))
        c->l1_tile = std::min<uint32_t>((uint32_t)std::max(atoi(e), 0) / 1024u * 1024u, (uint32_t)kPTile);
    if (const char* e = getenv("CRDT_SORTED_FORM")) c->form_off = (uint32_t)strtoul(e, nullptr, 10);
    if (const char* e = getenv("CRDT_APPLY_ITEMS")) {
        const int v = atoi(e);
        c->apply_items = (v == 1 || v == 2 || v == 4 || v == 8) ? v : 0;
    }
    c->fail_rank = -1;
    c->fail_at = 0;
    if (const char* e = getenv("CRDT_TEST_FAIL")) {     // "rank:point" (comm_path.inc, kFail*)
        int r = -1, at = 0;
        if (sscanf(e, "%d:%d", &r, &at) == 2) { c->fail_rank = r; c->fail_at = at; }
    }
    c->stall_rank = -1;
    c->stall_at = c->stall_ms = 0;
    c->stall_dev = false;
    if (const char* e = getenv("CRDT_TEST_STALL")) {    // "rank:point:ms[:d]" (comm_path.inc, test_stall)
        int r = -1, at = 0, ms = 0;
        char d = 0;
        const int k = sscanf(e, "%d:%d:%d:%c", &r, &at, &ms, &d);
        if (k >= 3) { c->stall_rank = r; c->stall_at = at; c->stall_ms = ms; c->stall_dev = k == 4 && d == 'd'; }
    }
}

int crdt_create(int device, uint32_t local_rank, uint64_t capacity, crdt_ctx** out) {
    if (!out) return CRDT_E_INVALID;
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n) return CRDT_E_NO_DEVICE;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess) return CRDT_E_NO_DEVICE;
    if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) return CRDT_E_NO_DEVICE;
    HIPCHK(hipSetDevice(device));
    crdt_ctx* c = new (std::nothrow) crdt_ctx();
    if (!c) return CRDT_E_NOMEM;
    c->device = device;
    c->local_rank = local_rank;
    if (const char* e = getenv("CRDT_MERGE_PATH")) {
        c->merge_path = strcmp(e, "gather") == 0 ? 1 : strcmp(e, "sorted") == 0 ? 2 : 0;
    }
    read_env_knobs(c);
    if (const char* e = getenv("CRDT_ENV_DYNAMIC")) c->env_dynamic = atoi(e) != 0;
    if (const char* e = getenv("CRDT_COMM_TIMEOUT_MS")) c->comm_timeout_ms = (uint32_t)std::max(atoll(e), 0ll);
    if (const char* e = getenv("CRDT_KV_WINDOW")) {
        const long long v = atoll(e);
        if (v > 0) c->kv_window = (uint64_t)v;
    }
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
        hipMalloc(&c->d_misc, sizeof(Misc)) != hipSuccess ||
        hipHostMalloc(&c->h_misc, sizeof(Misc), hipHostMallocDefault) != hipSuccess ||
        c->d_M.ensure(1024) != hipSuccess || c->d_event.ensure(8) != hipSuccess ||
        c->d_word.ensure(4) != hipSuccess) {
        crdt_destroy(c);
        return CRDT_E_HIP;
    }
    int st = crdt_reserve(c, capacity);
    if (st) { crdt_destroy(c); return st; }
    *out = c;
    return CRDT_OK;
}

void crdt_destroy(crdt_ctx* c) {
    if (!c) return;
    hipSetDevice(c->device);
    if (c->stream) hipStreamSynchronize(c->stream);
    comm_release(c);
    for (auto* b : {&c->r_skey, &c->r_srank, &c->r_sval, &c->r_key, &c->r_rank, &c->r_val}) b->release();
    c->r_slt.release(); c->r_lt.release(); c->r_perm.release(); c->r_flags.release(); c->r_sflags.release();
    c->d_gsend.release(); c->d_grecv.release(); c->d_pbase.release(); c->d_sum.release(); c->d_tune.release(); c->h_tune.release();
    c->d_rcnt.release(); c->d_rrecv.release(); c->h_rcnt.release(); c->h_stage.release(); c->h_sum.release();
    c->d_rcur.release(); c->d_agree.release(); c->h_agree.release(); c->d_rl1cnt.release(); c->h_rl1cnt.release();
    if (c->route_ev) hipEventDestroy(c->route_ev);
    for (hipEvent_t e : c->rl_evs) if (e) hipEventDestroy(e);
    for (hipEvent_t e : c->rl_evx) if (e) hipEventDestroy(e);
    if (c->rl_evo) hipEventDestroy(c->rl_evo);
    if (c->rl_evh) hipEventDestroy(c->rl_evh);
    for (hipEvent_t e : c->ov_ev) if (e) hipEventDestroy(e);
    if (c->sstream) hipStreamDestroy(c->sstream);
    if (c->ostream) hipStreamDestroy(c->ostream);
    if (c->table.base) hipFree(c->table.base);
    if (c->d_misc) hipFree(c->d_misc);
    if (c->h_misc) hipHostFree(c->h_misc);
    c->d_M.release(); c->d_event.release(); c->d_plan.release();
    c->h_plan.release();
    c->d_T.release(); c->d_Cprev.release(); c->d_Rj.release(); c->d_Cj.release();
    c->d_candP.release(); c->d_candms.release(); c->d_candtile.release(); c->d_candkind.release();
    c->d_candkey.release();
    c->s_key.release(); c->s_rank.release(); c->s_val.release(); c->s_lt.release();
    c->s_millis.release(); c->s_mod.release(); c->s_flags.release(); c->s_out.release();
    c->d_word.release();
    c->d_ibase.release();
    c->p1_rec.release(); c->p1_kj.release(); c->p2_rec.release(); c->p2_kj.release();
    for (int i = 0; i < crdt_ctx::kPlaceMax; ++i) { c->pc_rec[i].release(); c->pc_kj[i].release(); }
    for (hipEvent_t e : c->place_ev) if (e) hipEventDestroy(e);
    c->p_hist.release(); c->p_hist1.release(); c->p_toff.release(); c->p_part.release(); c->p_choff.release();
    c->p_dstart1.release(); c->p_dstart2.release(); c->p_l2map.release();
    c->p_plan.release(); c->p_l1beg.release(); c->h_pplan.release();
    c->p_ibase.release(); c->p_ksu32.release(); c->p_kslt.release(); c->p_tseg.release();
    c->p_ibucket.release(); c->p_ilist.release(); c->h_ilist.release();
    c->f_pos1.release(); c->f_pos2.release(); c->f_flag1.release(); c->f_flag2.release();
    c->f_cin_key.release(); c->f_cin_val.release(); c->f_cin_pres.release();
    c->f_hist2.release(); c->f_toff2.release();
    c->e_key.release(); c->e_val.release(); c->e_pk.release(); c->e_cnt.release(); c->e_cur.release();
    c->e_icnt.release(); c->e_off.release(); c->e_csum.release(); c->e_bbase.release();
    c->h_ebase.release();
    c->rl_rec.release(); c->rl_k16.release(); for (Rl1Scratch& os : c->rl_os) os.release();
    c->rl_hf.release(); c->rl_hrec.release(); c->rl_hk16.release(); c->rl_hcnt.release(); c->h_hcnt.release();
    for (hipEvent_t e : c->events) hipEventDestroy(e);
    for (hipEvent_t e : c->cevents) hipEventDestroy(e);
    if (c->cstream) hipStreamDestroy(c->cstream);
    if (c->stream) hipStreamDestroy(c->stream);
    delete c;
}

int crdt_reserve(crdt_ctx* c, uint64_t capacity) {
    if (!c) return CRDT_E_INVALID;
    if (capacity <= c->cap && c->table.base) return CRDT_OK;
    if (capacity > (1ull << 32)) return CRDT_E_INVALID;   // key ids are uint32
    HIPCHK(hipSetDevice(c->device));
    const uint64_t newcap = std::max<uint64_t>(capacity, 16);
    const uint64_t rb = c->table.stride;
    Table t{nullptr, c->table.stride};
    HIPALLOC(hipMalloc(&t.base, newcap * rb));
    if (c->table.base && c->cap)
        HIPCHK(hipMemcpyAsync(t.base, c->table.base, c->cap * rb, hipMemcpyDeviceToDevice, c->stream));
    // absent rows: mod_hi 0x80808080 < 0 (and mod = 0x8080808080808080)
    HIPCHK(hipMemsetAsync(t.base + c->cap * rb, 0x80, (newcap - c->cap) * rb, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    if (c->table.base) hipFree(c->table.base);
    c->table = t;
    c->cap = newcap;
    return CRDT_OK;
}

int crdt_set_row_bytes(crdt_ctx* c, uint32_t row_bytes) {
    if (!c || (row_bytes != 24 && row_bytes != 32)) return CRDT_E_INVALID;
    if (row_bytes == c->table.stride) return CRDT_OK;
    HIPCHK(hipSetDevice(c->device));
    Table t{nullptr, row_bytes};
    HIPALLOC(hipMalloc(&t.base, c->cap * (uint64_t)row_bytes));
    if (c->cap) {
        k_relayout<<<std::min<uint32_t>(grid_for(c->cap, 256), 65536), 256, 0, c->stream>>>(c->table, t, c->cap);
        HIPCHK(hipGetLastError());
    }
    HIPCHK(hipStreamSynchronize(c->stream));
    hipFree(c->table.base);
    c->table = t;
    return CRDT_OK;
}

int crdt_reserve_scratch(crdt_ctx* c, uint64_t n_records) {
    if (!c) return CRDT_E_INVALID;
    if (n_records == 0) return CRDT_OK;
    HIPCHK(hipSetDevice(c->device));
    // sized for the packed two-level form (12-B payloads, 2-B / 1-B key columns: the fan-in's); another
    // form grows them in its first merge
    HIPALLOC(c->p1_rec.ensure((3 * n_records + 3) / 4 + kPartPad));
    HIPALLOC(c->p1_kj.ensure((n_records + 1) / 2 + kPartPad));
    HIPALLOC(c->p2_rec.ensure((3 * n_records + 3) / 4 + kPartPad));
    HIPALLOC(c->p2_kj.ensure((n_records + 3) / 4 + kPartPad));
    // PlaceTune: CRDT_PLACE_TRIES candidate level-1 buffers (default 3; 1 = off), taken by the next sorted
    // merge (place_take: capped at 1/8 of HBM) and timed in the merges after it
    int tries = 3;
    if (const char* e = getenv("CRDT_PLACE_TRIES")) tries = std::min(std::max(atoi(e), 1), crdt_ctx::kPlaceMax);
    if (c->has_comm) tries = 1;                   // (a sharded ctx partitions elsewhere: route_l1, the fold)
    c->place_k = tries;
    c->place_idle = 0;
    c->place_trial = tries > 1 ? -1 : 0;
    c->place_best = tries > 1 ? -1 : 0;
    return CRDT_OK;
}



int crdt_capacity(const crdt_ctx* c, uint64_t* out) {
    if (!c || !out) return CRDT_E_INVALID;
    *out = c->cap;
    return CRDT_OK;
}

int crdt_set_local_rank(crdt_ctx* c, uint32_t rank) {
    if (!c) return CRDT_E_INVALID;
    c->local_rank = rank;
    return CRDT_OK;
}

int crdt_get_canonical(const crdt_ctx* c, int64_t* lt) {
    if (!c || !lt) return CRDT_E_INVALID;
    *lt = c->canonical;
    return CRDT_OK;
}

int crdt_set_canonical(crdt_ctx* c, int64_t lt) {
    if (!c) return CRDT_E_INVALID;
    c->canonical = lt;
    return CRDT_OK;
}

int crdt_put_rows(crdt_ctx* c, const uint32_t* key_id, const int64_t* lt, const uint32_t* rank,
                  const uint32_t* val, const int64_t* mod, uint64_t n, int32_t mem) {
    if (!c) return CRDT_E_INVALID;
    if (n == 0) return CRDT_OK;
    if (!key_id || !lt || !rank || !val || !mod) return CRDT_E_INVALID;
    HIPCHK(hipSetDevice(c->device));
    const uint32_t *dk, *dr, *dv;
    const int64_t *dl, *dm;
    int st;
    if ((st = stage(c, c->s_key, key_id, n, mem, &dk))) return st;
    if ((st = stage(c, c->s_lt, lt, n, mem, &dl))) return st;
    if ((st = stage(c, c->s_rank, rank, n, mem, &dr))) return st;
    if ((st = stage(c, c->s_val, val, n, mem, &dv))) return st;
    if ((st = stage(c, c->s_mod, mod, n, mem, &dm))) return st;
    if ((st = reset_misc(c))) return st;
    k_put_rows<<<std::min<uint32_t>(grid_for(n, 256), kPutGrid), 256, 0, c->stream>>>(dk, dl, dr, dv, dm, n,
                                                                                     c->table, c->cap, c->d_misc);
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpyAsync(c->h_misc, c->d_misc, sizeof(Misc), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    raise_hw(c, c->h_misc->key_end);
    return c->h_misc->err ? CRDT_E_KEY_RANGE : CRDT_OK;
}

int crdt_put_stamped(crdt_ctx* c, const uint32_t* key_id, const uint32_t* val, uint64_t n, int64_t wall,
                     int32_t mem, crdt_result* out) {
    if (!c) return CRDT_E_INVALID;
    crdt_result res;
    memset(&res, 0, sizeof(res));
    res.exc_index = UINT64_MAX;
    res.canonical_lt = c->canonical;
    if (n == 0) { if (out) *out = res; return CRDT_OK; }     // crdt.dart:48
    if (!key_id || !val) return CRDT_E_INVALID;
    // Hlc.send (hlc.dart:51-74), once for the whole call (crdt.dart:40, 50)
    const int64_t cm = c->canonical >> kShift, cc = c->canonical & kMaxCounter;
    const int64_t mn = imax(cm, wall);
    const int64_t cn = (cm == mn) ? cc + 1 : 0;
    if (wsub(mn, wall) > kMaxDrift) {
        res.status = CRDT_CLOCK_DRIFT;
        res.drift_ms = wsub(mn, wall);
        if (out) *out = res;
        return res.status;
    }
    if (cn > kMaxCounter) {
        res.status = CRDT_OVERFLOW;
        res.counter = cn;
        if (out) *out = res;
        return res.status;
    }
    const int64_t stamp = (int64_t)(((uint64_t)mn << kShift) + (uint64_t)cn);
    HIPCHK(hipSetDevice(c->device));
    const uint32_t *dk, *dv;
    int st;
    if ((st = stage(c, c->s_key, key_id, n, mem, &dk))) return st;
    if ((st = stage(c, c->s_val, val, n, mem, &dv))) return st;
    if ((st = reset_misc(c))) return st;
    k_put_stamped<<<std::min<uint32_t>(grid_for(n, 256), kPutGrid), 256, 0, c->stream>>>(
        dk, dv, n, stamp, c->local_rank, c->table, c->cap, c->d_misc);
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpyAsync(c->h_misc, c->d_misc, sizeof(Misc), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    raise_hw(c, c->h_misc->key_end);
    if (c->h_misc->err) return CRDT_E_KEY_RANGE;
    c->canonical = stamp;
    res.canonical_lt = stamp;
    res.n_won = n;
    if (out) *out = res;
    return CRDT_OK;
}

int crdt_read_rows(crdt_ctx* c, const uint32_t* key_id, uint64_t n, int64_t* lt, uint32_t* rank,
                   uint32_t* val, int64_t* mod, int32_t mem) {
    if (!c) return CRDT_E_INVALID;
    if (n == 0) return CRDT_OK;
    if (!key_id) return CRDT_E_INVALID;
    HIPCHK(hipSetDevice(c->device));
    const uint32_t* dk;
    int st;
    if ((st = stage(c, c->s_key, key_id, n, mem, &dk))) return st;
    int64_t *dl = lt, *dm = mod;
    uint32_t *dr = rank, *dv = val;
    if (mem == CRDT_MEM_HOST) {
        HIPALLOC(c->s_lt.ensure(n));
        HIPALLOC(c->s_mod.ensure(n));
        HIPALLOC(c->s_rank.ensure(n));
        HIPALLOC(c->s_val.ensure(n));
        dl = lt ? c->s_lt.p : nullptr;
        dm = mod ? c->s_mod.p : nullptr;
        dr = rank ? c->s_rank.p : nullptr;
        dv = val ? c->s_val.p : nullptr;
    }
    if ((st = reset_misc(c))) return st;
    k_read_rows<<<grid_for(n, 256), 256, 0, c->stream>>>(dk, n, c->table, c->cap, dl, dr, dv, dm, c->d_misc);
    HIPCHK(hipGetLastError());
    if (mem == CRDT_MEM_HOST) {
        if (lt) HIPCHK(hipMemcpyAsync(lt, dl, n * sizeof(int64_t), hipMemcpyDeviceToHost, c->stream));
        if (mod) HIPCHK(hipMemcpyAsync(mod, dm, n * sizeof(int64_t), hipMemcpyDeviceToHost, c->stream));
        if (rank) HIPCHK(hipMemcpyAsync(rank, dr, n * sizeof(uint32_t), hipMemcpyDeviceToHost, c->stream));
        if (val) HIPCHK(hipMemcpyAsync(val, dv, n * sizeof(uint32_t), hipMemcpyDeviceToHost, c->stream));
    }
    HIPCHK(hipMemcpyAsync(c->h_misc, c->d_misc, sizeof(Misc), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    return c->h_misc->err ? CRDT_E_KEY_RANGE : CRDT_OK;
}

int crdt_refresh_canonical(crdt_ctx* c, uint64_t n_rows, int64_t* out_lt) {
    if (!c || n_rows > c->cap) return CRDT_E_INVALID;
    HIPCHK(hipSetDevice(c->device));
    k_fill_i64<<<1, 64, 0, c->stream>>>(c->d_word.p, 1, INT64_MIN);
    if (n_rows) {
        const unsigned g = std::min<unsigned>(grid_for(n_rows, 256), 2048);
        k_refresh<<<g, 256, 0, c->stream>>>(c->table, n_rows, c->d_word.p);
        HIPCHK(hipGetLastError());
    }
    long long w = 0;
    HIPCHK(hipMemcpyAsync(&w, c->d_word.p, sizeof(w), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    const int64_t lt = (w == INT64_MIN) ? 0 : (int64_t)w;  // empty recordMap -> 0 (crdt.dart:118)
    c->canonical = lt;                                 // fromLogicalTime(max, nodeId)
    if (out_lt) *out_lt = lt;
    return CRDT_OK;
}

int crdt_modified_since(crdt_ctx* c, uint64_t n_rows, int64_t since_lt, uint32_t* out_ids, uint64_t* n_out) {
    if (!c || !n_out || n_rows > c->cap) return CRDT_E_INVALID;
    *n_out = 0;
    if (n_rows == 0) return CRDT_OK;
    if (!out_ids) return CRDT_E_INVALID;
    HIPCHK(hipSetDevice(c->device));
    const unsigned nb = grid_for(n_rows, kMsPerBlock);
    HIPALLOC(c->s_out.ensure(n_rows + nb));
    uint32_t* counts = c->s_out.p + n_rows;
    k_ms_count<<<nb, 256, 0, c->stream>>>(c->table, n_rows, since_lt, counts);
    k_ms_scan<<<1, 1024, 0, c->stream>>>(counts, nb, c->d_word.p);
    k_ms_write<<<nb, 256, 0, c->stream>>>(c->table, n_rows, since_lt, counts, c->s_out.p);
    HIPCHK(hipGetLastError());
    long long total = 0;
    HIPCHK(hipMemcpyAsync(&total, c->d_word.p, sizeof(total), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    if (total) HIPCHK(hipMemcpy(out_ids, c->s_out.p, total * sizeof(uint32_t), hipMemcpyDeviceToHost));
    *n_out = total;
    return CRDT_OK;
}

int crdt_clear_rows(crdt_ctx* c, uint64_t first, uint64_t count) {
    if (!c || first > c->cap || count > c->cap - first) return CRDT_E_INVALID;
    if (count == 0) return CRDT_OK;
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipMemsetAsync(row_ptr(c->table, first), 0x80, count * c->table.stride, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    if (first <= c->hw && first + count >= c->hw) c->hw = first;   // the rows from first on are fill
    return CRDT_OK;
}

int crdt_remap_ranks(crdt_ctx* c, uint64_t n_rows, const uint32_t* old_to_new, uint32_t n_ranks) {
    if (!c || n_rows > c->cap || (!old_to_new && n_ranks)) return CRDT_E_INVALID;
    if (n_rows == 0 || n_ranks == 0) return CRDT_OK;
    HIPCHK(hipSetDevice(c->device));
    const uint32_t* dl;
    int st;
    if ((st = stage(c, c->s_rank, old_to_new, n_ranks, CRDT_MEM_HOST, &dl))) return st;
    k_remap<<<grid_for(n_rows, 256), 256, 0, c->stream>>>(c->table, n_rows, dl, n_ranks);
    if (n_ranks > 0x80808080u) raise_hw(c, n_rows);      // the fill's rank 0x80808080 would be remapped
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(c->stream));
    return CRDT_OK;
}

int crdt_merge(crdt_ctx* c, const crdt_batch* batch, int64_t wall, uint8_t* win_flags, crdt_result* out) {
    if (!c) return CRDT_E_INVALID;
    int st = validate_batch(batch);
    if (st) return st;
    const uint32_t R = batch->n_changesets;
    if (R == 0) {                                            // no merge() call at all
        crdt_result res;
        memset(&res, 0, sizeof(res));
        res.exc_index = UINT64_MAX;
        res.canonical_lt = c->canonical;
        if (out) *out = res;
        return CRDT_OK;
    }
    HIPCHK(hipSetDevice(c->device));
    if (c->env_dynamic) read_env_knobs(c);
    // rows >= hw_read are read as the fill by this merge; afterwards hw moves to hw_next (the
    // capacity unless finish_apply learned the batch's key bound) on every return path
    c->hw_read = (c->form_off & kFormNoHw) ? c->cap : c->hw;
    c->hw_next = c->cap;
    c->key_end_valid = false;
    struct HwUpdate {
        crdt_ctx* c;
        ~HwUpdate() { c->hw = std::max(c->hw, c->hw_next); }
    } hw_update{c};
    c->sent_bytes = 0;
    if (c->has_comm) return merge_sharded(c, batch, wall, win_flags, out);
    c->place_timed = c->place_warm = false;                  // (set by this call's first sorted window)
    // Host batches are staged once; every phase then sees device columns.
    crdt_batch dev = *batch;
    uint8_t* dflags = win_flags;
    const uint64_t n = batch->offsets[R];
    struct KvReset {                                         // no window outlives this call
        crdt_ctx* c;
        ~KvReset() { c->kv_key = c->kv_val = nullptr; c->kv_n = c->kv_done = 0; c->kv_win = 0; }
    } kv_reset{c};
    if (batch->mem == CRDT_MEM_HOST) {
        // lt / rank / millis now (the scan reads every record); key / val window by window
        // under K2 on the copy stream (kv_copy_next)
        if (n > 0 && (!batch->key_id || !batch->val)) return CRDT_E_INVALID;
        Cols cols;
        if ((st = stage_check_cols(c, batch, &cols))) return st;
        HIPALLOC(c->s_key.ensure(n ? n : 1));
        HIPALLOC(c->s_val.ensure(n ? n : 1));
        if (n) {
            if (!c->cstream) HIPCHK(hipStreamCreateWithFlags(&c->cstream, hipStreamNonBlocking));
            c->kv_key = batch->key_id;
            c->kv_val = batch->val;
            c->kv_n = n;
        }
        dev.key_id = c->s_key.p; dev.lt = cols.lt; dev.rank = cols.rank; dev.val = c->s_val.p;
        dev.millis = cols.millis;
        dev.mem = CRDT_MEM_DEVICE;
        if (win_flags) {
            HIPALLOC(c->s_flags.ensure(n ? n : 1));
            dflags = c->s_flags.p;
        }
    }
    HIPALLOC(c->d_M.ensure(R));
    if (c->timing) HIPCHK(ensure_events(c, events_for(R)));
    // the sorted path's packed form needs the records' frame: the scan reduces it on the way
    c->segs.from_offsets(batch->offsets, R);
    const bool frame = c->packed_resolve && use_sorted(c, c->segs, R, win_flags);
    ev_record(c, kEvStart);
    if ((st = phase_scan(c, &dev, wall, c->d_M.p, true, frame, true, batch->mem == CRDT_MEM_DEVICE))) return st;
    ev_record(c, kEvScan);
    if ((st = phase_clock(c, &dev, wall, c->d_M.p, c->d_event.p))) return st;
    if (!c->resolved && (st = phase_resolve(c, c->d_event.p))) return st;
    ev_record(c, kEvClock);
    st = phase_apply(c, &dev, wall, c->d_event.p, dflags, out, true);
    if (c->place_k > 1 && c->place_best < 0 && !c->last_sorted && ++c->place_idle >= 2) place_drop(c);
    if (c->timing) {
        ev_record(c, kEvEnd);
        hipStreamSynchronize(c->stream);
    }
    if (st >= 0 && win_flags && batch->mem == CRDT_MEM_HOST && n)
        HIPCHK(hipMemcpy(win_flags, dflags, n, hipMemcpyDeviceToHost));
    place_finish(c, st >= 0);
    collect_timing(c);
    return st;
}

int crdt_set_rank_bound(crdt_ctx* c, uint32_t bound) {
    if (!c) return CRDT_E_INVALID;
    c->rank_bound = bound;
    return CRDT_OK;
}

int crdt_set_counts(crdt_ctx* c, int exact) {
    if (!c || (exact != 0 && exact != 1)) return CRDT_E_INVALID;
    c->counts = exact != 0;
    return CRDT_OK;
}

int crdt_set_merge_path(crdt_ctx* c, int path) {
    if (!c || path < CRDT_PATH_AUTO || path > CRDT_PATH_SORTED) return CRDT_E_INVALID;
    c->merge_path = path;
    return CRDT_OK;
}

int crdt_last_path(const crdt_ctx* c, int* path) {
    if (!c || !path) return CRDT_E_INVALID;
    *path = c->last_sorted ? CRDT_PATH_SORTED : CRDT_PATH_GATHER;
    return CRDT_OK;
}

int crdt_last_plan(const crdt_ctx* c, uint32_t* flags) {
    if (!c || !flags) return CRDT_E_INVALID;
    uint32_t f = 0;
    if (c->last_sorted) {
        f |= CRDT_PLAN_SORTED;
        if (c->last_packed) f |= CRDT_PLAN_PACKED;
        if (c->cap > (1ull << 20)) f |= CRDT_PLAN_TWO_LEVEL;
        if (c->last_hist1_fused) f |= CRDT_PLAN_HIST_IN_SCAN;
        if (c->last_key8) f |= CRDT_PLAN_KEY8;
        if (c->last_key16) f |= CRDT_PLAN_KEY16;
        if (c->last_hw) f |= CRDT_PLAN_HIGH_WATER;
        if (c->last_flagged) f |= CRDT_PLAN_FLAGGED;
        if (c->last_ordered) f |= CRDT_PLAN_ORDERED;
        if (c->last_combined) f |= CRDT_PLAN_COMBINED;
        if (c->last_route_l1) f |= CRDT_PLAN_ROUTE_L1;
        if (c->last_compact) f |= CRDT_PLAN_COMPACT;
    }
    if (c->last_wire_pk) f |= CRDT_PLAN_WIRE_PACKED;
    if (c->last_own_in_place) f |= CRDT_PLAN_OWN_IN_PLACE;
    if (c->tune_trial) f |= CRDT_PLAN_ROUTE_TUNED;
    if (c->last_route_l1) f |= (c->last_rl1_pieces & 7u) << CRDT_PLAN_RL1_PIECES_SHIFT;
    if (c->last_route_l1 && c->last_rl1_head) f |= CRDT_PLAN_RL1_HEAD;
    *flags = f;
    return CRDT_OK;
}

int crdt_place_info(const crdt_ctx* c, int32_t* n, int32_t* kept, int32_t* done, float* ms) {
    if (!c || !n || !kept || !done || !ms) return CRDT_E_INVALID;
    *n = c->place_k;
    *kept = c->place_best;
    *done = c->place_k > 1 ? c->place_trial + 1 : 0;
    for (int i = 0; i < crdt_ctx::kPlaceMax; ++i) ms[i] = i < c->place_k ? c->place_ms[i] : 0.f;
    return CRDT_OK;
}

int crdt_route_tune_info(const crdt_ctx* c, int32_t* best, int64_t* us) {
    if (!c || !best || !us) return CRDT_E_INVALID;
    *best = c->rt.best;
    for (int w = 0; w < 5; ++w) us[w] = c->rt.us[w];
    return CRDT_OK;
}

int crdt_set_timing(crdt_ctx* c, int enable) {
    if (!c) return CRDT_E_INVALID;
    c->timing = enable != 0;
    return CRDT_OK;
}

int crdt_get_timing(const crdt_ctx* c, crdt_timing* out) {
    if (!c || !out) return CRDT_E_INVALID;
    *out = c->last_timing;
    return CRDT_OK;
}

}  // extern "C"
