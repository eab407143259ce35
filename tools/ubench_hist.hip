// Microbenchmark: why does the partition histogram (k_part_hist) read 4 GB of keys at
// ~1.5 TB/s?  Variants over 1B random 28-bit keys, 256 digits of key >> 20:
//   A  1024-thread workgroups, 32 keys per thread, nontemporal loads, ballot-aggregated LDS atomics
//   B  A with plain loads
//   C  A's loads only (xor of the keys, no histogram)
//   D  256-thread workgroups, 32 keys per thread (8K-key tiles)
//   E  A with uint4 loads (4 keys per lane per load)
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/ubench_hist tools/ubench_hist.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#ifndef SHIFT_BITS
#define SHIFT_BITS 20
#endif
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

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

template <int T, int Q, bool NT, bool HIST>
__global__ __launch_bounds__(T) void k_hist(const uint32_t* __restrict__ key, uint64_t n, uint32_t* __restrict__ hist) {
    __shared__ uint32_t h[256];
    const int tid = threadIdx.x, lane = tid & 63;
    for (int d = tid; d < 256; d += T) h[d] = 0;
    const uint64_t beg = (uint64_t)blockIdx.x * T * Q;
    uint32_t k[Q];
#pragma unroll
    for (int q = 0; q < Q; ++q) {
        const uint64_t i = beg + (uint64_t)q * T + tid;
        k[q] = i < n ? (NT ? __builtin_nontemporal_load(key + i) : key[i]) : 0u;
    }
    __syncthreads();
    if (!HIST) {
        uint32_t x = 0;
#pragma unroll
        for (int q = 0; q < Q; ++q) x ^= k[q];
        if (x == 0x12345678u) hist[0] = x;
        return;
    }
    const unsigned long long below = (1ull << lane) - 1;
#pragma unroll
    for (int q = 0; q < Q; ++q) {
        const uint64_t i = beg + (uint64_t)q * T + tid;
        const bool act = i < n;
        const uint32_t d = (k[q] >> 20) & 255;
        const unsigned long long m = match_digit(d, act);
        if (act && (m & below) == 0) atomicAdd(&h[d], (uint32_t)__popcll(m));
    }
    __syncthreads();
    for (int d = tid; d < 256; d += T) hist[(uint64_t)blockIdx.x * 256 + d] = h[d];
}

// G/H: one LDS atomic per key, no ballot aggregation (H returns the old value = a slot,
// as a non-stable scatter would use it)
template <int T, int Q, bool RET>
__global__ __launch_bounds__(T) void k_hist_atomic(const uint32_t* __restrict__ key, uint64_t n,
                                                   uint32_t* __restrict__ hist) {
    __shared__ uint32_t h[256];
    const int tid = threadIdx.x;
    for (int d = tid; d < 256; d += T) h[d] = 0;
    const uint64_t beg = (uint64_t)blockIdx.x * T * Q;
    uint32_t k[Q];
#pragma unroll
    for (int q = 0; q < Q; ++q) {
        const uint64_t i = beg + (uint64_t)q * T + tid;
        k[q] = i < n ? __builtin_nontemporal_load(key + i) : 0u;
    }
    __syncthreads();
    uint32_t acc = 0;
#pragma unroll
    for (int q = 0; q < Q; ++q) {
        const uint32_t d = (k[q] >> SHIFT_BITS) & 255;
        if (RET) acc += atomicAdd(&h[d], 1u);
        else atomicAdd(&h[d], 1u);
    }
    if (RET && acc == 0x12345678u) hist[0] = acc;
    __syncthreads();
    for (int d = tid; d < 256; d += T) hist[(uint64_t)blockIdx.x * 256 + d] = h[d];
}

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
template <int T, int Q>
__global__ __launch_bounds__(T) void k_hist4(const u32x4* __restrict__ key4, uint64_t n4, uint32_t* __restrict__ hist) {
    __shared__ uint32_t h[256];
    const int tid = threadIdx.x, lane = tid & 63;
    for (int d = tid; d < 256; d += T) h[d] = 0;
    const uint64_t beg = (uint64_t)blockIdx.x * T * Q;
    u32x4 k[Q];
#pragma unroll
    for (int q = 0; q < Q; ++q) {
        const uint64_t i = beg + (uint64_t)q * T + tid;
        k[q] = i < n4 ? __builtin_nontemporal_load(key4 + i) : u32x4{0u, 0u, 0u, 0u};
    }
    __syncthreads();
    const unsigned long long below = (1ull << lane) - 1;
#pragma unroll
    for (int q = 0; q < Q; ++q) {
        const uint64_t i = beg + (uint64_t)q * T + tid;
        const bool act = i < n4;
        const uint32_t kk[4] = {k[q].x, k[q].y, k[q].z, k[q].w};
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const uint32_t d = (kk[c] >> 20) & 255;
            const unsigned long long m = match_digit(d, act);
            if (act && (m & below) == 0) atomicAdd(&h[d], (uint32_t)__popcll(m));
        }
    }
    __syncthreads();
    for (int d = tid; d < 256; d += T) hist[(uint64_t)blockIdx.x * 256 + d] = h[d];
}

__global__ void k_gen(uint32_t* key, uint64_t n) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t z = (i + 1) * 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        key[i] = (uint32_t)((z ^ (z >> 31)) >> 36);
    }
}

template <typename F>
float timeit(F f) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    f();
    CK(hipEventRecord(a));
    for (int r = 0; r < 3; ++r) f();
    CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
    float ms; CK(hipEventElapsedTime(&ms, a, b));
    return ms / 3;
}

int main() {
    const uint64_t n = 1ull << 30;
    uint32_t *key, *hist;
    CK(hipMalloc(&key, n * 4));
    CK(hipMalloc(&hist, (n / 4096 + 16) * 256 * 4));   // largest grid: variant F, n / 4096 blocks
    k_gen<<<8192, 256>>>(key, n);
    CK(hipDeviceSynchronize());
    const double gb = n * 4 / 1e9;
    float a = timeit([&] { k_hist<1024, 32, true, true><<<n / 32768, 1024>>>(key, n, hist); });
    float b = timeit([&] { k_hist<1024, 32, false, true><<<n / 32768, 1024>>>(key, n, hist); });
    float c = timeit([&] { k_hist<1024, 32, true, false><<<n / 32768, 1024>>>(key, n, hist); });
    float d = timeit([&] { k_hist<256, 32, true, true><<<n / 8192, 256>>>(key, n, hist); });
    float e = timeit([&] { k_hist4<1024, 8><<<n / 32768, 1024>>>((const u32x4*)key, n / 4, hist); });
    float f = timeit([&] { k_hist<256, 16, true, true><<<n / 4096, 256>>>(key, n, hist); });
    float g = timeit([&] { k_hist_atomic<1024, 32, false><<<n / 32768, 1024>>>(key, n, hist); });
    float h2 = timeit([&] { k_hist_atomic<1024, 32, true><<<n / 32768, 1024>>>(key, n, hist); });
    // skewed digits: a third of the keys in digit 0 (the fan-in's level-1 shape)
    CK(hipGetLastError());
    printf("G atomic/key %.3f ms (%.0f GB/s)  H atomic-with-return %.3f (%.0f)\n", g, gb / g * 1e3, h2, gb / h2 * 1e3);
    printf("1B keys (4.3 GB): A %.3f ms (%.0f GB/s)  B plain %.3f (%.0f)  C loads-only %.3f (%.0f)  "
           "D 256thr %.3f (%.0f)  E uint4 %.3f (%.0f)  F 256thr/16 %.3f (%.0f)\n",
           a, gb / a * 1e3, b, gb / b * 1e3, c, gb / c * 1e3, d, gb / d * 1e3, e, gb / e * 1e3, f, gb / f * 1e3);
    return 0;
}
