// Microbenchmark: K2's access pattern — random 16-B row read, then a write of the row
// for ~25 % of the records — with 32-B rows (write 32 B = half of a 64-B DRAM burst)
// vs 64-B rows (write the whole 64 B), on a 2^28-row table.  Answers whether partial
// 32-B writes cost a read-modify-write in the memory system.
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/ubench_rowwrite tools/ubench_rowwrite.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x8 __attribute__((ext_vector_type(8)));
typedef unsigned int u32x16 __attribute__((ext_vector_type(16)));

template <int ROWB, int WRITEB>
__global__ __launch_bounds__(256) void k_rmw(const uint32_t* __restrict__ idx, uint64_t n, uint8_t* table,
                                             uint32_t wmod, uint32_t* sink) {
    const uint64_t base = (uint64_t)blockIdx.x * 1024 + threadIdx.x;
    uint32_t k[4];
    u32x4 r[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const uint64_t i = base + q * 256;
        k[q] = i < n ? __builtin_nontemporal_load(idx + i) : 0u;
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) r[q] = *reinterpret_cast<const u32x4*>(table + (uint64_t)k[q] * ROWB);
    uint32_t acc = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        acc ^= r[q].x;
        const uint64_t i = base + q * 256;
        if (i < n && (k[q] % wmod) == 0) {
            uint8_t* p = table + (uint64_t)k[q] * ROWB;
            if (WRITEB == 32) {
                u32x8 v = {r[q].x + 1, r[q].y, r[q].z, r[q].w, 1u, 2u, 0u, 0u};
                *reinterpret_cast<u32x8*>(p) = v;
            } else if (WRITEB == 64) {
                u32x16 v = {r[q].x + 1, r[q].y, r[q].z, r[q].w, 1u, 2u, 0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u};
                *reinterpret_cast<u32x16*>(p) = v;
            }
        }
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

template <int ROWB, int WRITEB>
float run(const uint32_t* idx, uint64_t n, uint8_t* table, uint32_t wmod, uint32_t* sink) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    const unsigned g = (unsigned)((n + 1023) / 1024);
    k_rmw<ROWB, WRITEB><<<g, 256>>>(idx, n, table, wmod, sink);
    CK(hipEventRecord(a));
    for (int r = 0; r < 5; ++r) k_rmw<ROWB, WRITEB><<<g, 256>>>(idx, n, table, wmod, sink);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    return ms / 5;
}

int main() {
    const uint64_t rows = 1ull << 28, n = 16ull << 20;
    uint32_t *idx, *sink;
    uint8_t* table;
    CK(hipMalloc(&idx, n * 4)); CK(hipMalloc(&sink, 64));
    CK(hipMalloc(&table, rows * 64));
    CK(hipMemset(table, 0, rows * 64));
    k_fill<<<(n + 255) / 256, 256>>>(idx, n, rows, 17);
    CK(hipDeviceSynchronize());
    printf("16M random records over 2^28 rows; time per launch (us) and G records/s\n");
    for (uint32_t wmod : {1000000000u, 4u, 1u}) {
        const char* w = wmod == 1u ? "100%" : wmod == 4u ? "25%" : "0%";
        float a = run<32, 0>(idx, n, table, wmod, sink);
        float b = run<32, 32>(idx, n, table, wmod, sink);
        float c = run<64, 0>(idx, n, table, wmod, sink);
        float d = run<64, 64>(idx, n, table, wmod, sink);
        float e = run<64, 32>(idx, n, table, wmod, sink);
        printf("writes %-5s | 32-B rows read-only %7.1f (%5.1f)  write 32 B %7.1f (%5.1f) | 64-B rows read-only %7.1f (%5.1f)"
               "  write 64 B %7.1f (%5.1f)  write 32 B %7.1f (%5.1f)\n",
               w, a * 1e3, n / a / 1e6, b * 1e3, n / b / 1e6, c * 1e3, n / c / 1e6, d * 1e3, n / d / 1e6, e * 1e3,
               n / e / 1e6);
    }
    return 0;
}
