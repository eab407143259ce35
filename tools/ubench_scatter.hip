// Microbenchmark: the level-1 partition scatter (k_part_scatter1's job) over 1B records,
// 256 digits of key bits [20, 28), 32K-record tiles, per-(tile, digit) output cursors given.
//   staged : k_part_scatter1's scheme — 4096-record sub-tiles ranked by LDS atomics, staged in
//            LDS in digit order (16-B + 4-B + 1-B writes at random LDS addresses), then written out
//            as contiguous runs
//   direct : no staging: one LDS atomic per record on the tile's digit cursor, the record stored
//            from registers at that position (L2 assembles the runs' lines)
//   directw: direct with wave-aggregated ranks (ballot match, one atomic per digit per wave)
//   carry  : staged, but every digit's output written in whole 128-B lines only (a partial last
//            line waits in an LDS carry for the next sub-tile): 15 % faster than staged, at the
//            cost of scattered whole-line writes (~9.5 ms), still far from sequential (6.9 ms)
//   copy   : 20 B in, 20 B out streaming (the ceiling)
// staged write modes (MODE): 0 as k_part_scatter1; 1 every sub-tile written to its own input
// range (sequential, wrong order: the kernel's cost without the scatter); 3 / 4 only rec / only kj;
// 7 whole 128-B lines at random line-aligned places; 5 / 6 only lines (128 / 64 B) a run fully
// covers; no-write = loads + LDS work alone.  Modes 5-7 leave a wrong output (timing only).
// Keys uniform, then skewed (a third of them in digit 0, as the fan-in's level 1).
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/ubench_scatter tools/ubench_scatter.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <algorithm>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
constexpr int kTile = 32768;
constexpr int kShift = 20;

__device__ inline uint64_t mix(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__global__ void k_gen(uint32_t* key, int64_t* lt, uint32_t* rank, uint32_t* val, uint64_t n, int skew) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t h = mix(i * 0x9E3779B97F4A7C15ull + 12345);
        uint32_t k = (uint32_t)(h >> 36);
        if (skew && (h & 0xFF) < 85) k &= (1u << kShift) - 1;     // ~1/3 into digit 0
        key[i] = k;
        lt[i] = (int64_t)((1700000000000ll + (h & 0xFFFF)) << 16);
        rank[i] = (uint32_t)(h >> 8) & 1023;
        val[i] = (uint32_t)i;
    }
}

__global__ __launch_bounds__(1024) void k_hist(const uint32_t* __restrict__ key, uint64_t n, uint32_t* __restrict__ hist) {
    __shared__ uint32_t h[256];
    if (threadIdx.x < 256) h[threadIdx.x] = 0;
    __syncthreads();
    const uint64_t beg = (uint64_t)blockIdx.x * kTile;
    for (int q = 0; q < kTile / 1024; ++q) {
        const uint64_t i = beg + q * 1024 + threadIdx.x;
        if (i < n) atomicAdd(&h[(key[i] >> kShift) & 255], 1u);
    }
    __syncthreads();
    if (threadIdx.x < 256) hist[(uint64_t)blockIdx.x * 256 + threadIdx.x] = h[threadIdx.x];
}

__device__ inline uint32_t scan256_excl(uint32_t v, uint32_t* s_w, uint32_t* total) {
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    uint32_t inc = v;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t u = __shfl_up(inc, off, 64);
        if (lane >= off) inc += u;
    }
    if (tid < 256 && lane == 63) s_w[w] = inc;
    __syncthreads();
    uint32_t wp = 0;
    for (int k = 0; k < w && k < 4; ++k) wp += s_w[k];
    *total = s_w[0] + s_w[1] + s_w[2] + s_w[3];
    return wp + inc - v;
}

__device__ inline uint32_t digit_count(uint32_t* bins, uint32_t d, bool act, int lane) {
    const unsigned long long a = __ballot(act);
    if (!a) return 0;
    const uint32_t d0 = __shfl(d, __ffsll((long long)a) - 1, 64);
    if (__all(!act || d == d0)) {
        uint32_t base = 0;
        const unsigned long long below = (1ull << lane) - 1;
        if (act && (a & below) == 0) base = atomicAdd(&bins[d0], (uint32_t)__popcll(a));
        base = __shfl(base, __ffsll((long long)a) - 1, 64);
        return base + (uint32_t)__popcll(a & below);
    }
    return act ? atomicAdd(&bins[d], 1u) : 0u;
}

__device__ inline unsigned long long match_digit(uint32_t d, bool active) {
    unsigned long long m = __ballot(active);
#pragma unroll
    for (int b = 0; b < 8; ++b) {
        const bool bit = (d >> b) & 1u;
        const unsigned long long bb = __ballot(active && bit);
        m &= bit ? bb : ~bb;
    }
    return m;
}

// k_part_scatter1's scheme; G: stage each record's global destination (u32) instead of its
// digit, so the write-out reads one conflict-free word instead of s_dig + cur[d] + dst[d];
// W: write nothing (LDS + barrier cost alone, loads kept)
// xper != 0: XCD-contiguous tile order (workgroup i on XCD i % 8 takes tile (i % 8) * xper + i / 8)
template <int T, int Q, bool G, bool W, int MODE = 0, uint32_t DMASK = 255>
__global__ __launch_bounds__(T) void k_staged(const uint32_t* __restrict__ keyw, const int64_t* __restrict__ lt,
                                              const uint32_t* __restrict__ rank, const uint32_t* __restrict__ val,
                                              uint64_t n, const uint32_t* __restrict__ toff, u32x4* __restrict__ orec,
                                              uint32_t* __restrict__ okj, uint32_t xper = 0) {
    constexpr int SUB = T * Q;
    __shared__ uint32_t cur[256], cnt[256], dst[257], s_w[4];
    __shared__ u32x4 s_rec[SUB];
    __shared__ uint32_t s_kj[SUB];
    __shared__ uint32_t s_g[G ? SUB : 1];
    __shared__ uint8_t s_dig[G ? 1 : SUB];
    const uint32_t t = xper ? (blockIdx.x % 8) * xper + blockIdx.x / 8 : blockIdx.x;
    if ((uint64_t)t * kTile >= n) return;
    const uint64_t beg = (uint64_t)t * kTile;
    const uint32_t len = (uint32_t)min<uint64_t>(kTile, n - beg);
    const int tid = threadIdx.x, lane = tid & 63;
    for (int d = tid; d < 256; d += T) cur[d] = toff[(uint64_t)t * 256 + d];
    u32x4 nrec[Q];
    uint32_t nk[Q];
    auto load_sub = [&](uint32_t sb) {
#pragma unroll
        for (int q = 0; q < Q; ++q) {
            const uint32_t i = sb + q * T + tid;
            const uint64_t gi = beg + (i < len ? i : 0);
            const int64_t l = __builtin_nontemporal_load(lt + gi);
            nrec[q].x = (uint32_t)l; nrec[q].y = (uint32_t)((uint64_t)l >> 32);
            nrec[q].z = __builtin_nontemporal_load(rank + gi);
            nrec[q].w = __builtin_nontemporal_load(val + gi);
            nk[q] = __builtin_nontemporal_load(keyw + gi);
        }
    };
    load_sub(0);
    uint32_t acc = 0;
    for (uint32_t sb = 0; sb < len; sb += SUB) {
        for (int d = tid; d < 256; d += T) cnt[d] = 0;
        u32x4 rec[Q];
        uint32_t k[Q], d[Q], slot[Q];
        bool act[Q];
#pragma unroll
        for (int q = 0; q < Q; ++q) { act[q] = sb + q * T + tid < len; rec[q] = nrec[q]; k[q] = nk[q]; }
        if (sb + SUB < len) load_sub(sb + SUB);
        __syncthreads();
#pragma unroll
        for (int q = 0; q < Q; ++q) {
            d[q] = (k[q] >> kShift) & DMASK;
            slot[q] = digit_count(cnt, d[q], act[q], lane);
        }
        __syncthreads();
        if (T >= 256) {
            uint32_t all;
            const uint32_t tv = tid < 256 ? cnt[tid] : 0u;
            const uint32_t ex = scan256_excl(tv, s_w, &all);
            if (tid < 256) { dst[tid] = ex; if (tid == 255) dst[256] = ex + tv; }
        }
        __syncthreads();
#pragma unroll
        for (int q = 0; q < Q; ++q)
            if (act[q]) {
                const uint32_t pos = dst[d[q]] + slot[q];
                s_rec[pos] = rec[q]; s_kj[pos] = k[q];
                if (G) s_g[pos] = cur[d[q]] + slot[q]; else s_dig[pos] = (uint8_t)d[q];
            }
        __syncthreads();
        const uint32_t staged = dst[256];
#pragma unroll
        for (int q = 0; q < Q; ++q) {
            const uint32_t s = q * T + tid;
            if (s < staged) {
                uint64_t g;
                if (G) g = s_g[s];
                else { const uint32_t dd = s_dig[s]; g = (uint64_t)cur[dd] + (s - dst[dd]); }
                if (MODE == 1) g = beg + sb + s;                       // sequential destination
                if (W) {
                    if (MODE == 2) { __builtin_nontemporal_store(s_rec[s], orec + g); __builtin_nontemporal_store(s_kj[s], okj + g); }
                    else if (MODE == 3) orec[g] = s_rec[s];
                    else if (MODE == 4) okj[g] = s_kj[s];
                    else if (MODE == 7) {                    // whole lines at scattered line-aligned places
                        const uint64_t u = beg + sb + s;
                        const uint64_t lr = mix(u >> 3) % (n >> 3), lk = mix((u >> 5) + 77) % (n >> 5);
                        orec[(lr << 3) | (u & 7)] = s_rec[s];
                        okj[(lk << 5) | (u & 31)] = s_kj[s];
                    }
                    else if (MODE == 5 || MODE == 6) {      // only records of fully covered lines (output wrong:
                        const uint32_t dd = s_dig[s];         // measures scattered whole-line writes)
                        const uint64_t r0 = cur[dd], r1 = r0 + (dst[dd + 1] - dst[dd]);
                        constexpr uint64_t AR = MODE == 5 ? 8 : 4, AK = MODE == 5 ? 32 : 16;
                        const uint64_t lr = g & ~(AR - 1), lk = g & ~(AK - 1);
                        if (lr >= r0 && lr + AR <= r1) orec[g] = s_rec[s];
                        if (lk >= r0 && lk + AK <= r1) okj[g] = s_kj[s];
                    }
                    else { orec[g] = s_rec[s]; okj[g] = s_kj[s]; }
                }
                else acc ^= s_rec[s].x ^ s_kj[s] ^ (uint32_t)g;
            }
        }
        __syncthreads();
        for (int dd = tid; dd < 256; dd += T) cur[dd] += dst[dd + 1] - dst[dd];
    }
    if (!W && acc == 0x12345678u) okj[0] = acc;
}


// write-combining form of "staged": each digit's output is only written in whole 128-B lines
// (8 records of rec, 32 of kj); a digit's partial last line waits in an LDS carry for the next
// sub-tile (the tile-run's first and last lines excepted).
__global__ __launch_bounds__(1024) void k_carry(const uint32_t* __restrict__ keyw, const int64_t* __restrict__ lt,
                                                const uint32_t* __restrict__ rank, const uint32_t* __restrict__ val,
                                                uint64_t n, const uint32_t* __restrict__ toff, u32x4* __restrict__ orec,
                                                uint32_t* __restrict__ okj) {
    constexpr int T = 1024, Q = 4, SUB = T * Q, AR = 8, AK = 32;
    __shared__ uint32_t cur[256], cnt[256], dst[257], s_w[4], wpR[256], wpK[256], feR[256], feK[256];
    __shared__ u32x4 s_rec[SUB];
    __shared__ uint32_t s_kj[SUB];
    __shared__ uint8_t s_dig[SUB];
    __shared__ u32x4 cR[256 * (AR - 1)];
    __shared__ uint32_t cK[256 * (AK - 1)];
    const uint32_t t = blockIdx.x;
    const uint64_t beg = (uint64_t)t * kTile;
    const uint32_t len = (uint32_t)min<uint64_t>(kTile, n - beg);
    const int tid = threadIdx.x, lane = tid & 63;
    if (tid < 256) { const uint32_t c0 = toff[(uint64_t)t * 256 + tid]; cur[tid] = c0; wpR[tid] = c0; wpK[tid] = c0; }
    u32x4 nrec[Q];
    uint32_t nk[Q];
    auto load_sub = [&](uint32_t sb) {
#pragma unroll
        for (int q = 0; q < Q; ++q) {
            const uint32_t i = sb + q * T + tid;
            const uint64_t gi = beg + (i < len ? i : 0);
            const int64_t l = __builtin_nontemporal_load(lt + gi);
            nrec[q].x = (uint32_t)l; nrec[q].y = (uint32_t)((uint64_t)l >> 32);
            nrec[q].z = __builtin_nontemporal_load(rank + gi);
            nrec[q].w = __builtin_nontemporal_load(val + gi);
            nk[q] = __builtin_nontemporal_load(keyw + gi);
        }
    };
    load_sub(0);
    for (uint32_t sb = 0; sb < len; sb += SUB) {
        if (tid < 256) cnt[tid] = 0;
        u32x4 rec[Q];
        uint32_t k[Q], d[Q], slot[Q];
        bool act[Q];
#pragma unroll
        for (int q = 0; q < Q; ++q) { act[q] = sb + q * T + tid < len; rec[q] = nrec[q]; k[q] = nk[q]; }
        if (sb + SUB < len) load_sub(sb + SUB);
        __syncthreads();
#pragma unroll
        for (int q = 0; q < Q; ++q) {
            d[q] = (k[q] >> kShift) & 255;
            slot[q] = digit_count(cnt, d[q], act[q], lane);
        }
        __syncthreads();
        uint32_t all;
        const uint32_t tv = tid < 256 ? cnt[tid] : 0u;
        const uint32_t ex = scan256_excl(tv, s_w, &all);
        if (tid < 256) {
            dst[tid] = ex;
            if (tid == 255) dst[256] = ex + tv;
            // flush end per array: whole lines only, unless the run has not reached its first
            // line boundary yet (then everything: the head line is partial anyway)
            const uint32_t end = cur[tid] + tv;
            uint32_t fr = end & ~(AR - 1), fk = end & ~(AK - 1);
            if (fr <= wpR[tid]) fr = (wpR[tid] & (AR - 1)) ? end : wpR[tid];
            if (fk <= wpK[tid]) fk = (wpK[tid] & (AK - 1)) ? end : wpK[tid];
            feR[tid] = fr; feK[tid] = fk;
        }
        __syncthreads();
#pragma unroll
        for (int q = 0; q < Q; ++q)
            if (act[q]) {
                const uint32_t pos = dst[d[q]] + slot[q];
                s_rec[pos] = rec[q]; s_kj[pos] = k[q]; s_dig[pos] = (uint8_t)d[q];
            }
        __syncthreads();
        // F1: carried entries below the flush end, and new records below it, go out
        for (int e = tid; e < 256 * AR; e += T) {
            const int dd = e / AR, kk = e % AR;
            const uint32_t g = wpR[dd] + kk;
            if (kk < AR - 1 && g < cur[dd] && g < feR[dd]) orec[g] = cR[dd * (AR - 1) + kk];
        }
        for (int e = tid; e < 256 * AK; e += T) {
            const int dd = e / AK, kk = e % AK;
            const uint32_t g = wpK[dd] + kk;
            if (kk < AK - 1 && g < cur[dd] && g < feK[dd]) okj[g] = cK[dd * (AK - 1) + kk];
        }
        const uint32_t staged = dst[256];
#pragma unroll
        for (int q = 0; q < Q; ++q) {
            const uint32_t s = q * T + tid;
            if (s < staged) {
                const uint32_t dd = s_dig[s];
                const uint32_t g = cur[dd] + (s - dst[dd]);
                if (g < feR[dd]) orec[g] = s_rec[s];
                if (g < feK[dd]) okj[g] = s_kj[s];
            }
        }
        __syncthreads();
        // F2: the rest of every digit into its carry (old carried entries never move: when
        // the flush end passed them they were all written, otherwise it stayed at wp)
#pragma unroll
        for (int q = 0; q < Q; ++q) {
            const uint32_t s = q * T + tid;
            if (s < staged) {
                const uint32_t dd = s_dig[s];
                const uint32_t g = cur[dd] + (s - dst[dd]);
                if (g >= feR[dd]) cR[dd * (AR - 1) + (g - feR[dd])] = s_rec[s];
                if (g >= feK[dd]) cK[dd * (AK - 1) + (g - feK[dd])] = s_kj[s];
            }
        }
        __syncthreads();
        if (tid < 256) { cur[tid] += dst[tid + 1] - dst[tid]; wpR[tid] = feR[tid]; wpK[tid] = feK[tid]; }
    }
    // the runs' last partial lines
    for (int e = tid; e < 256 * AR; e += T) {
        const int dd = e / AR, kk = e % AR;
        const uint32_t g = wpR[dd] + kk;
        if (kk < AR - 1 && g < cur[dd]) orec[g] = cR[dd * (AR - 1) + kk];
    }
    for (int e = tid; e < 256 * AK; e += T) {
        const int dd = e / AK, kk = e % AK;
        const uint32_t g = wpK[dd] + kk;
        if (kk < AK - 1 && g < cur[dd]) okj[g] = cK[dd * (AK - 1) + kk];
    }
}

// direct: LDS atomic cursor per record, store from registers.  B records per thread in flight.
template <int T, int B, bool WAVE_AGG>
__global__ __launch_bounds__(T) void k_direct(const uint32_t* __restrict__ keyw, const int64_t* __restrict__ lt,
                                              const uint32_t* __restrict__ rank, const uint32_t* __restrict__ val,
                                              uint64_t n, const uint32_t* __restrict__ toff, u32x4* __restrict__ orec,
                                              uint32_t* __restrict__ okj) {
    __shared__ uint32_t cur[256];
    const uint32_t t = blockIdx.x;
    const uint64_t beg = (uint64_t)t * kTile;
    const uint32_t len = (uint32_t)min<uint64_t>(kTile, n - beg);
    const int tid = threadIdx.x, lane = tid & 63;
    for (int d = tid; d < 256; d += T) cur[d] = toff[(uint64_t)t * 256 + d];
    __syncthreads();
    const unsigned long long below = (1ull << lane) - 1;
    for (uint32_t i0 = 0; i0 < len; i0 += T * B) {
        u32x4 rec[B];
        uint32_t k[B];
#pragma unroll
        for (int q = 0; q < B; ++q) {
            const uint32_t i = i0 + q * T + tid;
            const uint64_t gi = beg + (i < len ? i : 0);
            const int64_t l = __builtin_nontemporal_load(lt + gi);
            rec[q].x = (uint32_t)l; rec[q].y = (uint32_t)((uint64_t)l >> 32);
            rec[q].z = __builtin_nontemporal_load(rank + gi);
            rec[q].w = __builtin_nontemporal_load(val + gi);
            k[q] = __builtin_nontemporal_load(keyw + gi);
        }
#pragma unroll
        for (int q = 0; q < B; ++q) {
            const bool act = i0 + q * T + tid < len;
            const uint32_t d = (k[q] >> kShift) & 255;
            uint32_t pos;
            if (WAVE_AGG) {
                const unsigned long long m = match_digit(d, act);
                const int leader = m ? __ffsll((long long)m) - 1 : 0;
                uint32_t base = 0;
                if (act && lane == leader) base = atomicAdd(&cur[d], (uint32_t)__popcll(m));
                // every lane of the group reads its leader's base
                base = __shfl(base, leader, 64);
                pos = base + (uint32_t)__popcll(m & below);
            } else {
                pos = act ? atomicAdd(&cur[d], 1u) : 0u;
            }
            if (act) { orec[pos] = rec[q]; okj[pos] = k[q]; }
        }
    }
}

__global__ void k_copy(const uint32_t* __restrict__ key, const int64_t* __restrict__ lt,
                       const uint32_t* __restrict__ rank, const uint32_t* __restrict__ val, uint64_t n,
                       u32x4* __restrict__ rec, uint32_t* __restrict__ kj) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        int64_t l = __builtin_nontemporal_load(lt + i);
        u32x4 o;
        o.x = (uint32_t)l; o.y = (uint32_t)((uint64_t)l >> 32);
        o.z = __builtin_nontemporal_load(rank + i); o.w = __builtin_nontemporal_load(val + i);
        rec[i] = o;
        kj[i] = __builtin_nontemporal_load(key + i);
    }
}

// digit order violations + a checksum of val
__global__ void k_check(const u32x4* __restrict__ rec, const uint32_t* __restrict__ kj, uint64_t n,
                        unsigned long long* __restrict__ out) {
    unsigned long long bad = 0, sum = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        if (i && ((kj[i] >> kShift) & 255) < ((kj[i - 1] >> kShift) & 255)) ++bad;
        sum += rec[i].w;
    }
    atomicAdd(&out[0], bad);
    atomicAdd(&out[1], sum);
}

struct Timer {
    hipEvent_t a, b;
    Timer() { CK(hipEventCreate(&a)); CK(hipEventCreate(&b)); }
    void start() { CK(hipEventRecord(a)); }
    float stop() { CK(hipEventRecord(b)); CK(hipEventSynchronize(b)); float ms; CK(hipEventElapsedTime(&ms, a, b)); return ms; }
};

int main() {
    const uint64_t n = 1000000512ull;
    const uint32_t tiles = (uint32_t)((n + kTile - 1) / kTile);
    uint32_t *key, *rank, *val, *kj, *hist, *toff;
    int64_t* lt;
    u32x4* rec;
    unsigned long long* chk;
    CK(hipMalloc(&key, n * 4)); CK(hipMalloc(&lt, n * 8)); CK(hipMalloc(&rank, n * 4)); CK(hipMalloc(&val, n * 4));
    CK(hipMalloc(&rec, n * 16)); CK(hipMalloc(&kj, n * 4));
    CK(hipMalloc(&hist, (uint64_t)tiles * 256 * 4)); CK(hipMalloc(&toff, (uint64_t)tiles * 256 * 4));
    CK(hipMalloc(&chk, 16));
    std::vector<uint32_t> h((size_t)tiles * 256), o((size_t)tiles * 256);
    const unsigned long long expect = (unsigned long long)n * (n - 1) / 2;
    Timer tm;
    for (int skew = 0; skew < 2; ++skew) {
        k_gen<<<8192, 256>>>(key, lt, rank, val, n, skew);
        k_hist<<<tiles, 1024>>>(key, n, hist);
        CK(hipMemcpy(h.data(), hist, h.size() * 4, hipMemcpyDeviceToHost));
        uint64_t run = 0;
        for (int d = 0; d < 256; ++d)
            for (uint32_t t = 0; t < tiles; ++t) { o[(size_t)t * 256 + d] = (uint32_t)run; run += h[(size_t)t * 256 + d]; }
        CK(hipMemcpy(toff, o.data(), o.size() * 4, hipMemcpyHostToDevice));
        auto run_check = [&](const char* name, auto launch) {
            float best = 1e9;
            for (int r = 0; r < 4; ++r) { tm.start(); launch(); float ms = tm.stop(); if (r) best = best < ms ? best : ms; }
            CK(hipGetLastError());
            CK(hipMemset(chk, 0, 16));
            k_check<<<4096, 256>>>(rec, kj, n, chk);
            unsigned long long c[2];
            CK(hipMemcpy(c, chk, 16, hipMemcpyDeviceToHost));
            printf("skew %d %-22s %7.3f ms  %5.0f GB/s r+w  order-violations %llu  checksum %s\n", skew, name, best,
                   n * 40 / best / 1e6, c[0], c[1] == expect ? "ok" : "BAD");
        };
        run_check("copy", [&] { k_copy<<<8192, 256>>>(key, lt, rank, val, n, rec, kj); });
        // output placement variants (same kernel, other cursor tables): XCD-contiguous tile order;
        // tile-local (each tile's records digit-sorted inside the tile's own range); super-regions of
        // S consecutive tiles (digit-major inside the region)
        const uint32_t xper = (tiles + 7) / 8;
        run_check("staged global+xcd", [&] { k_staged<1024, 4, false, true><<<xper * 8, 1024>>>(key, lt, rank, val, n, toff, rec, kj, xper); });
        // fewer level-1 digits (longer runs per sub-tile): cursors of the digit-masked histogram
        for (uint32_t D : {16u, 64u, 128u}) {
            std::vector<uint32_t> o3((size_t)tiles * 256, 0);
            uint64_t r3 = 0;
            for (uint32_t d = 0; d < D; ++d)
                for (uint32_t t = 0; t < tiles; ++t) {
                    o3[(size_t)t * 256 + d] = (uint32_t)r3;
                    for (uint32_t e = d; e < 256; e += D) r3 += h[(size_t)t * 256 + e];
                }
            CK(hipMemcpy(toff, o3.data(), o3.size() * 4, hipMemcpyHostToDevice));
            char nm[64];
            snprintf(nm, sizeof(nm), "staged %u digits +xcd", D);
            if (D == 16) run_check(nm, [&] { k_staged<1024, 4, false, true, 0, 15><<<xper * 8, 1024>>>(key, lt, rank, val, n, toff, rec, kj, xper); });
            if (D == 64) run_check(nm, [&] { k_staged<1024, 4, false, true, 0, 63><<<xper * 8, 1024>>>(key, lt, rank, val, n, toff, rec, kj, xper); });
            if (D == 128) run_check(nm, [&] { k_staged<1024, 4, false, true, 0, 127><<<xper * 8, 1024>>>(key, lt, rank, val, n, toff, rec, kj, xper); });
        }
        CK(hipMemcpy(toff, o.data(), o.size() * 4, hipMemcpyHostToDevice));
        for (uint32_t S : {1u, 4u, 16u, 64u}) {
            std::vector<uint32_t> o2((size_t)tiles * 256);
            for (uint32_t g0 = 0; g0 < tiles; g0 += S) {
                const uint32_t g1 = std::min<uint32_t>(tiles, g0 + S);
                uint64_t r2 = (uint64_t)g0 * kTile;
                for (int d = 0; d < 256; ++d)
                    for (uint32_t t = g0; t < g1; ++t) { o2[(size_t)t * 256 + d] = (uint32_t)r2; r2 += h[(size_t)t * 256 + d]; }
            }
            CK(hipMemcpy(toff, o2.data(), o2.size() * 4, hipMemcpyHostToDevice));
            char nm[64];
            snprintf(nm, sizeof(nm), "staged region %u tiles", S);
            run_check(nm, [&] { k_staged<1024, 4, false, true><<<tiles, 1024>>>(key, lt, rank, val, n, toff, rec, kj); });
            snprintf(nm, sizeof(nm), "staged region %u +xcd", S);
            run_check(nm, [&] { k_staged<1024, 4, false, true><<<xper * 8, 1024>>>(key, lt, rank, val, n, toff, rec, kj, xper); });
        }
        CK(hipMemcpy(toff, o.data(), o.size() * 4, hipMemcpyHostToDevice));
        run_check("staged 1024x4 (cur.)", [&] { k_staged<1024, 4, false, true><<<tiles, 1024>>>(key, lt, rank, val, n, toff, rec, kj); });
        run_check("carry (whole lines)", [&] { k_carry<<<tiles, 1024>>>(key, lt, rank, val, n, toff, rec, kj); });
        run_check("staged seq-dest", [&] { k_staged<1024, 4, false, true, 1><<<tiles, 1024>>>(key, lt, rank, val, n, toff, rec, kj); });
        if (0) run_check("staged nt-store", [&] { k_staged<1024, 4, false, true, 2><<<tiles, 1024>>>(key, lt, rank, val, n, toff, rec, kj); });
        run_check("staged rec-only", [&] { k_staged<1024, 4, false, true, 3><<<tiles, 1024>>>(key, lt, rank, val, n, toff, rec, kj); });
        run_check("staged kj-only", [&] { k_staged<1024, 4, false, true, 4><<<tiles, 1024>>>(key, lt, rank, val, n, toff, rec, kj); });
        run_check("staged scattered-lines", [&] { k_staged<1024, 4, false, true, 7><<<tiles, 1024>>>(key, lt, rank, val, n, toff, rec, kj); });
        run_check("staged full-lines-128", [&] { k_staged<1024, 4, false, true, 5><<<tiles, 1024>>>(key, lt, rank, val, n, toff, rec, kj); });
        run_check("staged full-lines-64", [&] { k_staged<1024, 4, false, true, 6><<<tiles, 1024>>>(key, lt, rank, val, n, toff, rec, kj); });
        run_check("staged 1024x4 no-write", [&] { k_staged<1024, 4, false, false><<<tiles, 1024>>>(key, lt, rank, val, n, toff, rec, kj); });
        if (0) run_check("direct 1024 B8", [&] { k_direct<1024, 8, false><<<tiles, 1024>>>(key, lt, rank, val, n, toff, rec, kj); });
    }
    return 0;
}
