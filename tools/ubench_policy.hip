// Microbenchmark: does the cache policy of a random 16-B gather change the L2
// fill granularity (128-B line vs 32-B sector) and the gather rate on MI355X?
// aux = CPol bits of the buffer load (gfx940+): sc0 = 1, nt = 2, sc1 = 16.
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/ubench_policy tools/ubench_policy.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__device__ inline __amdgpu_buffer_rsrc_t make_rsrc(const void* base, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
}

// table viewed as 64 chunks of 128 MiB (buffer offsets are 32-bit): chunk = row >> 23 for 16-B rows
template <int AUX>
__global__ __launch_bounds__(256) void k_policy(const uint32_t* __restrict__ idx, uint64_t n, const uint8_t* table,
                                                uint32_t* sink) {
    const uint64_t base = (uint64_t)blockIdx.x * 1024 + threadIdx.x;
    uint32_t acc = 0;
    u32x4 r[4];
    uint32_t k[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        uint64_t i = base + q * 256;
        k[q] = idx[i < n ? i : 0];
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const uint8_t* chunk = table + ((uint64_t)(k[q] >> 23) << 27);
        __amdgpu_buffer_rsrc_t rs = make_rsrc(chunk, 1u << 27);
        r[q] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, (k[q] & ((1u << 23) - 1)) * 16, 0, AUX));
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) acc ^= r[q].x + r[q].w;
    if (acc == 0x12345678u) sink[0] = acc;
}

__global__ void k_fill(uint32_t* idx, uint64_t n, uint64_t rows, uint64_t seed) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint64_t z = (i + seed) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    idx[i] = (uint32_t)((z ^ (z >> 31)) % rows);
}

template <int AUX>
void run(const char* name, const uint32_t* idx, uint64_t n, const uint8_t* t, uint32_t* sink) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    unsigned g = (unsigned)((n + 1023) / 1024);
    k_policy<AUX><<<g, 256>>>(idx, n, t, sink);
    CK(hipEventRecord(a));
    for (int r = 0; r < 5; ++r) k_policy<AUX><<<g, 256>>>(idx, n, t, sink);
    CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
    float ms; CK(hipEventElapsedTime(&ms, a, b)); ms /= 5;
    printf("aux=%-3d %-14s %8.1f us  %6.2f G rows/s\n", AUX, name, ms * 1e3, n / (ms / 1e3) / 1e9);
}

int main() {
    const uint64_t n = 16ull << 20, T = 8ull << 30, rows = T / 16;
    uint32_t *idx, *sink;
    uint8_t* t;
    CK(hipMalloc(&idx, n * 4)); CK(hipMalloc(&sink, 64)); CK(hipMalloc(&t, T));
    CK(hipMemset(t, 0x11, T));
    k_fill<<<(n + 255) / 256, 256>>>(idx, n, rows, 3);
    CK(hipDeviceSynchronize());
    run<0>("default", idx, n, t, sink);
    run<1>("sc0", idx, n, t, sink);
    run<2>("nt", idx, n, t, sink);
    run<3>("sc0|nt", idx, n, t, sink);
    run<16>("sc1", idx, n, t, sink);
    run<17>("sc0|sc1", idx, n, t, sink);
    run<18>("sc1|nt", idx, n, t, sink);
    run<19>("sc0|sc1|nt", idx, n, t, sink);
    return 0;
}
