// Microbenchmark: the packed-key variant SURVEY section 7 step 4 suggests for the fan-in —
// one 64-bit atomic max per record on an 8-B field of the record's 32-B row (a batch-relative
// (lt, rank, changeset) key) — against K2's plain random 16-B row read, on a 2^28-row table and
// on a cache-sized 2^20-row one.  The atomic variant then needs a second pass (read the row and
// the max, the record that equals it writes), so it only pays if an atomic costs well under a read.
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/ubench_atomic tools/ubench_atomic.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// MODE 0: random 16-B row read; 1: atomic max (no return) on the row's bytes 24..31;
// 2: atomic max with the old value returned
template <int MODE>
__global__ __launch_bounds__(256) void k_op(const uint32_t* __restrict__ idx, uint64_t n, uint8_t* table,
                                            uint32_t* sink) {
    const uint64_t base = (uint64_t)blockIdx.x * 1024 + threadIdx.x;
    uint32_t k[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const uint64_t i = base + q * 256;
        k[q] = i < n ? __builtin_nontemporal_load(idx + i) : 0u;
    }
    uint32_t acc = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const uint64_t i = base + q * 256;
        uint8_t* p = table + (uint64_t)k[q] * 32;
        if (MODE == 0) {
            const u32x4 r = *reinterpret_cast<const u32x4*>(p);
            acc ^= r.x;
        } else if (i < n) {
            const unsigned long long v = ((unsigned long long)(i * 0x9E3779B97F4A7C15ull) >> 8);
            if (MODE == 1) {
                atomicMax(reinterpret_cast<unsigned long long*>(p + 24), v);
            } else {
                acc ^= (uint32_t)atomicMax(reinterpret_cast<unsigned long long*>(p + 24), v);
            }
        }
    }
    if (acc == 0x12345678u) sink[threadIdx.x] = acc;
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

template <int MODE>
float run(const uint32_t* idx, uint64_t n, uint8_t* table, uint32_t* sink) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    const unsigned g = (unsigned)((n + 1023) / 1024);
    k_op<MODE><<<g, 256>>>(idx, n, table, sink);
    CK(hipEventRecord(a));
    for (int r = 0; r < 5; ++r) k_op<MODE><<<g, 256>>>(idx, n, table, sink);
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
    CK(hipMalloc(&idx, n * 4)); CK(hipMalloc(&sink, 4096));
    CK(hipMalloc(&table, (1ull << 28) * 32));
    CK(hipMemset(table, 0, (1ull << 28) * 32));
    printf("16M random operations; time per launch (us) and G ops/s\n");
    for (uint64_t rows : {1ull << 28, 1ull << 20}) {
        k_fill<<<(n + 255) / 256, 256>>>(idx, n, rows, 17);
        CK(hipDeviceSynchronize());
        const float a = run<0>(idx, n, table, sink);
        const float b = run<1>(idx, n, table, sink);
        const float c = run<2>(idx, n, table, sink);
        printf("rows 2^%d | read 16 B %7.1f (%5.1f) | atomic max %7.1f (%5.1f) | atomic max + return %7.1f (%5.1f)\n",
               rows == (1ull << 28) ? 28 : 20, a * 1e3, n / a / 1e6, b * 1e3, n / b / 1e6, c * 1e3, n / c / 1e6);
    }
    return 0;
}
