// Microbenchmark: what bounds K2's random row reads — a per-CU limit on outstanding misses,
// or the memory system as a whole?  Random 16-B reads of a 2^28 x 32-B table (K2's gather)
// from a persistent grid restricted to C CUs (one workgroup of 256 threads per slot, `occ`
// workgroups per CU, grid-stride), plus a variant where every wave also issues S uniform
// scalar loads (s_load_dwordx4 through the scalar cache) for extra records, i.e. a second
// miss path beside the vector L1.
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/ubench_mshr tools/ubench_mshr.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef const __attribute__((address_space(4))) u32x4* cptr4;

// vector path: each thread reads 4 random rows per iteration
__global__ __launch_bounds__(256) void k_vec(const uint32_t* __restrict__ idx, uint64_t n, const uint8_t* table,
                                             uint32_t* sink) {
    uint32_t acc = 0;
    const uint64_t stride = (uint64_t)gridDim.x * 1024;
    for (uint64_t base = (uint64_t)blockIdx.x * 1024 + threadIdx.x; base < n; base += stride) {
        uint32_t k[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const uint64_t i = base + q * 256;
            k[q] = i < n ? __builtin_nontemporal_load(idx + i) : 0u;
        }
        u32x4 r[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) r[q] = *reinterpret_cast<const u32x4*>(table + (uint64_t)k[q] * 32);
#pragma unroll
        for (int q = 0; q < 4; ++q) acc ^= r[q].x ^ r[q].w;
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

// vector + scalar: per iteration a wave handles 256 rows by vector loads and S more by s_load
template <int S>
__global__ __launch_bounds__(256) void k_mix(const uint32_t* __restrict__ idx, uint64_t n, const uint8_t* table,
                                             uint32_t* sink) {
    uint32_t acc = 0;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    constexpr int PER = 1024 + 4 * S;                      // records per workgroup iteration
    const uint64_t stride = (uint64_t)gridDim.x * PER;
    for (uint64_t b0 = (uint64_t)blockIdx.x * PER; b0 < n; b0 += stride) {
        uint32_t k[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const uint64_t i = b0 + q * 256 + threadIdx.x;
            k[q] = i < n ? __builtin_nontemporal_load(idx + i) : 0u;
        }
        const uint64_t si = b0 + 1024 + wave * S + lane;
        const uint32_t ks = (lane < S && si < n) ? idx[si] : 0u;
        u32x4 r[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) r[q] = *reinterpret_cast<const u32x4*>(table + (uint64_t)k[q] * 32);
        u32x4 sv[S];
#pragma unroll
        for (int s = 0; s < S; ++s) {
            const uint32_t kk = __builtin_amdgcn_readlane(ks, s);
            sv[s] = *(cptr4)(table + (uint64_t)kk * 32);
        }
        uint32_t sacc = 0;
#pragma unroll
        for (int s = 0; s < S; ++s) sacc ^= sv[s].x ^ sv[s].w;
#pragma unroll
        for (int q = 0; q < 4; ++q) acc ^= r[q].x ^ r[q].w;
        acc ^= sacc;
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

__global__ void k_fill(uint32_t* idx, uint64_t n, uint64_t rows, uint64_t seed) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint64_t z = (i + seed) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    idx[i] = (uint32_t)(z % rows);
}

template <typename F>
float timeit(F f) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    f();
    CK(hipEventRecord(a));
    for (int r = 0; r < 5; ++r) f();
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    return ms / 5;
}

int main() {
    const uint64_t n = 16ull << 20;
    uint32_t *idx, *sink;
    uint8_t* table;
    int ncu = 0;
    CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
    CK(hipMalloc(&idx, n * 4)); CK(hipMalloc(&sink, 64));
    printf("16M random 16-B reads of 32-B rows; %d CUs; G rows/s\n", ncu);
    for (uint64_t rows : {1ull << 20, 1ull << 28}) {
        CK(hipMalloc(&table, rows * 32));
        CK(hipMemset(table, 0, rows * 32));
        k_fill<<<(n + 255) / 256, 256>>>(idx, n, rows, 17);
        CK(hipDeviceSynchronize());
        printf("table %llu rows (%llu MB)\n", (unsigned long long)rows, (unsigned long long)(rows * 32 >> 20));
        for (int occ : {2, 4, 8}) {
            for (int cus : {32, 64, 128, 256}) {
                if (cus > ncu) continue;
                const unsigned g = (unsigned)(cus * occ);
                float t = timeit([&] { k_vec<<<g, 256>>>(idx, n, table, sink); });
                printf("  vec  occ %d  wgs %5u (%3d CUs)  %7.1f us  %6.2f G/s\n", occ, g, cus, t * 1e3, n / t / 1e6);
            }
        }
        for (int occ : {4, 8}) {
            const unsigned g = (unsigned)(ncu * occ);
            float t4 = timeit([&] { k_mix<4><<<g, 256>>>(idx, n, table, sink); });
            float t16 = timeit([&] { k_mix<16><<<g, 256>>>(idx, n, table, sink); });
            float t32 = timeit([&] { k_mix<8><<<g, 256>>>(idx, n, table, sink); });
            printf("  mix  occ %d  S=4 %7.1f us %6.2f G/s | S=16 %7.1f us %6.2f G/s | S=8 %7.1f us %6.2f G/s\n", occ,
                   t4 * 1e3, n / t4 / 1e6, t16 * 1e3, n / t16 / 1e6, t32 * 1e3, n / t32 / 1e6);
        }
        CK(hipFree(table));
    }
    return 0;
}
