// Microbenchmark: is there HBM headroom under K2 for K3a's scan?  K2's access pattern (random
// 16-B row reads, 25 % of rows rewritten, 2^28 x 32-B rows; one launch per 976K-record
// changeset) back to back on one stream, a streaming max-reduction of an int64 column (the
// scan's lt stream) on another: alone, then concurrently.  Scale: 256 changesets (1/4 of the
// fan-in) and a 2 GB column (1/4 of its 8 GB lt stream).
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/ubench_overlap tools/ubench_overlap.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x8 __attribute__((ext_vector_type(8)));

__global__ __launch_bounds__(256) void k_rmw(const uint32_t* __restrict__ idx, uint64_t n, uint8_t* table,
                                             uint32_t* sink) {
    const uint64_t base = (uint64_t)blockIdx.x * 1024 + threadIdx.x;
    uint32_t k[4];
    u32x4 r[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const uint64_t i = base + q * 256;
        k[q] = i < n ? __builtin_nontemporal_load(idx + i) : 0u;
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) r[q] = *reinterpret_cast<const u32x4*>(table + (uint64_t)k[q] * 32);
    uint32_t acc = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        acc ^= r[q].x;
        const uint64_t i = base + q * 256;
        if (i < n && (k[q] & 3) == 0) {
            u32x8 v = {r[q].x + 1, r[q].y, r[q].z, r[q].w, 1u, 2u, 0u, 0u};
            *reinterpret_cast<u32x8*>(table + (uint64_t)k[q] * 32) = v;
        }
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

__global__ __launch_bounds__(256) void k_max(const int64_t* __restrict__ a, uint64_t n, int64_t* out) {
    int64_t m = INT64_MIN;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256 * 4) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const uint64_t j = i + (uint64_t)q * gridDim.x * 256;
            if (j < n) { const int64_t v = __builtin_nontemporal_load(a + j); m = v > m ? v : m; }
        }
    }
    if (m == 0x123456789ll) out[0] = m;
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

int main() {
    const uint64_t rows = 1ull << 28, per = 976563, R = 256, n = per * R, ncol = 256ull << 20;   // 2 GB of int64
    uint32_t *idx, *sink;
    uint8_t* table;
    int64_t *col, *out;
    CK(hipMalloc(&idx, n * 4)); CK(hipMalloc(&sink, 64)); CK(hipMalloc(&table, rows * 32));
    CK(hipMalloc(&col, ncol * 8)); CK(hipMalloc(&out, 64));
    CK(hipMemset(table, 0, rows * 32)); CK(hipMemset(col, 1, ncol * 8));
    k_fill<<<(n + 255) / 256, 256>>>(idx, n, rows, 17);
    CK(hipDeviceSynchronize());
    hipStream_t s1, s2;
    CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking)); CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    const unsigned g = (unsigned)((per + 1023) / 1024);
    auto k2 = [&](hipStream_t s) { for (uint64_t j = 0; j < R; ++j) k_rmw<<<g, 256, 0, s>>>(idx + j * per, per, table, sink); };
    auto scan = [&](hipStream_t s, unsigned blocks, int parts) {
        const uint64_t pc = ncol / parts;
        for (int p = 0; p < parts; ++p) k_max<<<blocks, 256, 0, s>>>(col + p * pc, pc, out);
    };
    auto timed = [&](auto f) {
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(a, s1));
        CK(hipStreamWaitEvent(s2, a, 0));
        f();
        hipEvent_t c;
        CK(hipEventCreate(&c));
        CK(hipEventRecord(c, s2));
        CK(hipStreamWaitEvent(s1, c, 0));
        CK(hipEventRecord(b, s1));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        return ms;
    };
    for (int rep = 0; rep < 2; ++rep) {
        const float t_k2 = timed([&] { k2(s1); });
        const float t_scan = timed([&] { scan(s2, 4096, 1); });
        const float t_both = timed([&] { k2(s1); scan(s2, 4096, 1); });
        const float t_both256 = timed([&] { k2(s1); scan(s2, 256, 1); });
        const float t_both_parts = timed([&] { k2(s1); scan(s2, 1024, 16); });
        printf("K2 x%lu %.3f ms | scan 2 GB %.3f ms (%.0f GB/s) | sum %.3f | concurrent: scan 4096 WGs %.3f, "
               "256 WGs %.3f, 16 parts of 1024 WGs %.3f ms\n",
               (unsigned long)R, t_k2, t_scan, ncol * 8 / t_scan / 1e6, t_k2 + t_scan, t_both, t_both256, t_both_parts);
    }
    return 0;
}
