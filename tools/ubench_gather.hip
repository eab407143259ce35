// Microbenchmark: random row gather / read-modify-write throughput on MI355X.
// Answers: what does a random 16/32/64-B row access cost on an 8.6 GB table
// (the K2 access pattern), vs table size (L2 / MALL / HBM / TLB reach)?
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/ubench_gather tools/ubench_gather.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <stdlib.h>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

template <int ROWB, int ITEMS, bool WRITE>
__global__ __launch_bounds__(256) void k_gather(const uint32_t* __restrict__ idx, uint64_t n, uint8_t* table,
                                                uint32_t* __restrict__ sink) {
    constexpr int V = ROWB / 16;
    const uint64_t base = (uint64_t)blockIdx.x * 256 * ITEMS + threadIdx.x;
    uint32_t k[ITEMS];
    uint4 r[ITEMS][V];
#pragma unroll
    for (int q = 0; q < ITEMS; ++q) {
        uint64_t i = base + q * 256;
        k[q] = i < n ? __builtin_nontemporal_load(idx + i) : 0xFFFFFFFFu;
    }
#pragma unroll
    for (int q = 0; q < ITEMS; ++q) {
        if (k[q] != 0xFFFFFFFFu) {
            const uint4* p = reinterpret_cast<const uint4*>(table + (uint64_t)k[q] * ROWB);
#pragma unroll
            for (int v = 0; v < V; ++v) r[q][v] = p[v];
        }
    }
    uint32_t acc = 0;
#pragma unroll
    for (int q = 0; q < ITEMS; ++q) {
        if (k[q] != 0xFFFFFFFFu) {
#pragma unroll
            for (int v = 0; v < V; ++v) acc ^= r[q][v].x + r[q][v].w;
            if (WRITE && (r[q][0].x & 1)) {
                uint4* p = reinterpret_cast<uint4*>(table + (uint64_t)k[q] * ROWB);
#pragma unroll
                for (int v = 0; v < V; ++v) p[v] = make_uint4(r[q][v].x + 1, r[q][v].y, r[q][v].z, acc);
            }
        }
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
__global__ void k_stream(const u32x4* __restrict__ a, uint64_t n16, uint32_t* sink) {
    uint32_t acc = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * blockDim.x) {
        u32x4 v = __builtin_nontemporal_load(a + i);
        acc ^= v.x ^ v.w;
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

template <int ROWB, int ITEMS, bool WRITE>
double run(const uint32_t* idx, uint64_t n, uint8_t* table, uint32_t* sink, int reps) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    unsigned g = (unsigned)((n + 256 * ITEMS - 1) / (256 * ITEMS));
    k_gather<ROWB, ITEMS, WRITE><<<g, 256>>>(idx, n, table, sink);
    CK(hipEventRecord(a));
    for (int r = 0; r < reps; ++r) k_gather<ROWB, ITEMS, WRITE><<<g, 256>>>(idx, n, table, sink);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    return ms / reps;
}

int main(int argc, char** argv) {
    const uint64_t n = 16ull << 20;               // 16M random accesses
    uint32_t *idx, *sink;
    CK(hipMalloc(&idx, n * 4));
    CK(hipMalloc(&sink, 64));
    std::vector<uint64_t> sizes = {64ull << 20, 256ull << 20, 1ull << 30, 4ull << 30, 8ull << 30, 16ull << 30};
    uint8_t* table;
    CK(hipMalloc(&table, 16ull << 30));
    CK(hipMemset(table, 0x11, 16ull << 30));
    {   // streaming read ceiling
        hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
        uint64_t n16 = (8ull << 30) / 16;
        k_stream<<<4096, 256>>>((const u32x4*)table, n16, sink);
        CK(hipEventRecord(a));
        for (int r = 0; r < 5; ++r) k_stream<<<4096, 256>>>((const u32x4*)table, n16, sink);
        CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
        float ms; CK(hipEventElapsedTime(&ms, a, b));
        printf("stream read 8 GiB: %.1f GB/s\n", (8ull << 30) * 5 / (ms / 1e3) / 1e9);
    }
    printf("%-10s %-6s %-5s %-5s %10s %12s %12s\n", "table", "rowB", "items", "write", "us", "Grows/s", "GB/s(rows)");
    for (uint64_t T : sizes) {
        for (int rowb : {16, 32, 64}) {
            uint64_t rows = T / rowb;
            k_fill<<<(n + 255) / 256, 256>>>(idx, n, rows, T + rowb);
            CK(hipDeviceSynchronize());
            for (int w = 0; w < 2; ++w) {
                double ms;
                if (rowb == 16) ms = w ? run<16, 4, true>(idx, n, table, sink, 5) : run<16, 4, false>(idx, n, table, sink, 5);
                else if (rowb == 32) ms = w ? run<32, 4, true>(idx, n, table, sink, 5) : run<32, 4, false>(idx, n, table, sink, 5);
                else ms = w ? run<64, 4, true>(idx, n, table, sink, 5) : run<64, 4, false>(idx, n, table, sink, 5);
                printf("%-10llu %-6d %-5d %-5d %10.1f %12.2f %12.1f\n", (unsigned long long)(T >> 20), rowb, 4, w,
                       ms * 1e3, n / (ms / 1e3) / 1e9, n * (double)rowb / (ms / 1e3) / 1e9);
            }
        }
    }
    // ordering check: read-only again after the RMW runs
    {
        uint64_t rows = (8ull << 30) / 32;
        k_fill<<<(n + 255) / 256, 256>>>(idx, n, rows, 99);
        CK(hipDeviceSynchronize());
        double r0 = run<32, 4, false>(idx, n, table, sink, 5), w0 = run<32, 4, true>(idx, n, table, sink, 5),
               r1 = run<32, 4, false>(idx, n, table, sink, 5), h = run<16, 4, false>(idx, n, table, sink, 5);
        printf("8GiB/32B: read %.1fus rmw %.1fus read-again %.1fus | 16B-of-32B-row stride read %.1fus\n",
               r0 * 1e3, w0 * 1e3, r1 * 1e3, h * 1e3);
    }
    // physically contiguous allocation (larger translation fragments?)
    {
        uint8_t* t2 = nullptr;
        hipError_t e = hipExtMallocWithFlags((void**)&t2, 8ull << 30, hipDeviceMallocContiguous);
        if (e == hipSuccess) {
            CK(hipMemset(t2, 0x11, 8ull << 30));
            for (int rowb : {16, 32}) {
                uint64_t rows = (8ull << 30) / rowb;
                k_fill<<<(n + 255) / 256, 256>>>(idx, n, rows, 5 + rowb);
                CK(hipDeviceSynchronize());
                double a = rowb == 16 ? run<16, 4, false>(idx, n, t2, sink, 5) : run<32, 4, false>(idx, n, t2, sink, 5);
                double b = rowb == 16 ? run<16, 4, false>(idx, n, table, sink, 5) : run<32, 4, false>(idx, n, table, sink, 5);
                printf("contiguous 8GiB/%dB read: %.1fus (%.2f Grows/s) vs plain %.1fus (%.2f)\n", rowb, a * 1e3,
                       n / a / 1e6, b * 1e3, n / b / 1e6);
            }
            CK(hipFree(t2));
        } else {
            printf("hipDeviceMallocContiguous failed: %s\n", hipGetErrorString(e));
        }
    }
    // ITEMS sensitivity at 8 GiB / 32 B
    {
        uint64_t rows = (8ull << 30) / 32;
        k_fill<<<(n + 255) / 256, 256>>>(idx, n, rows, 7);
        CK(hipDeviceSynchronize());
        double m1 = run<32, 1, false>(idx, n, table, sink, 5), m2 = run<32, 2, false>(idx, n, table, sink, 5),
               m8 = run<32, 8, false>(idx, n, table, sink, 5), m16 = run<32, 16, false>(idx, n, table, sink, 5);
        printf("items sweep 8GiB/32B read: 1:%.1fus 2:%.1fus 8:%.1fus 16:%.1fus\n", m1 * 1e3, m2 * 1e3, m8 * 1e3, m16 * 1e3);
    }
    return 0;
}
