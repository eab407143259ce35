// Microbenchmark: the HBM streaming ceilings of MI355X that DESIGN.md §5.5's bytes-floor model prices the
// sorted path's passes against (the round-1 figures, 5.7 TB/s read / 5.2 TB/s copy, sat
// under the guide's 6.0-6.3 TB/s).  For a 8 GiB buffer (far past the 256 MiB Infinity Cache):
//   read  : 16-B loads, U loads in flight per lane before any is used, grid-stride, summed into a sink
//   copy  : 16-B loads + 16-B stores (plain or nontemporal stores), U in flight
//   write : 16-B stores only
// over workgroups per CU x unroll, best of 5 runs each; GB/s counts the bytes moved (copy: read + write).
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/ubench_stream tools/ubench_stream.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <int U, bool kNt>
__global__ __launch_bounds__(256) void k_read(const u32x4* __restrict__ a, uint64_t n, uint32_t* __restrict__ sink) {
    const uint64_t stride = (uint64_t)gridDim.x * 256 * U;
    uint32_t acc = 0;
    for (uint64_t b = (uint64_t)blockIdx.x * 256 * U + threadIdx.x; b < n; b += stride) {
        u32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t i = b + (uint64_t)u * 256;
            v[u] = i < n ? (kNt ? __builtin_nontemporal_load(a + i) : a[i]) : u32x4{0, 0, 0, 0};
        }
#pragma unroll
        for (int u = 0; u < U; ++u) acc ^= v[u].x + v[u].y + v[u].z + v[u].w;
    }
    if (acc == 0x12345678u) sink[0] = acc;                 // (never: keeps the loads)
}

template <int U, bool kNtSt>
__global__ __launch_bounds__(256) void k_copy(const u32x4* __restrict__ a, u32x4* __restrict__ b, uint64_t n) {
    const uint64_t stride = (uint64_t)gridDim.x * 256 * U;
    for (uint64_t s = (uint64_t)blockIdx.x * 256 * U + threadIdx.x; s < n; s += stride) {
        u32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t i = s + (uint64_t)u * 256;
            if (i < n) v[u] = __builtin_nontemporal_load(a + i);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t i = s + (uint64_t)u * 256;
            if (i < n) {
                if (kNtSt) __builtin_nontemporal_store(v[u], b + i);
                else b[i] = v[u];
            }
        }
    }
}

// Block-contiguous copy (round 6): workgroup g copies the contiguous chunk [g * per, + per)
// instead of striding over the grid — each workgroup streams one region of DRAM pages, as a partition tile does.
template <int U>
__global__ __launch_bounds__(256) void k_copy_blk(const u32x4* __restrict__ a, u32x4* __restrict__ b, uint64_t n,
                                                  uint64_t per) {
    const uint64_t c0 = (uint64_t)blockIdx.x * per, c1 = c0 + per < n ? c0 + per : n;
    for (uint64_t s = c0 + threadIdx.x; s < c1; s += 256 * U) {
        u32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t i = s + (uint64_t)u * 256;
            if (i < c1) v[u] = __builtin_nontemporal_load(a + i);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t i = s + (uint64_t)u * 256;
            if (i < c1) b[i] = v[u];
        }
    }
}

// The level-1 scatter's shape without its ranking (round 6): a tile of T records (16 B each) read contiguously,
// written as 256 runs of T / 256 records to 256 far-apart places — run d of tile t at d * (tiles * run) + t * run,
// so the tiles' runs of one digit are adjacent, as in a partition.  Records of 16 B or (kNarrow) 12 + 2 B
// (the 14-B level-1 record: payload column + key column).  XCD-contiguous tile order as in the library.
template <int T, bool kNarrow>
__global__ __launch_bounds__(1024) void k_scatter_runs(const u32x4* __restrict__ a, u32x4* __restrict__ b,
                                                       uint32_t* __restrict__ b12, uint16_t* __restrict__ bk,
                                                       uint32_t tiles, uint32_t per) {
    const uint32_t t = (blockIdx.x % 8) * per + blockIdx.x / 8;
    if (t >= tiles) return;
    constexpr uint32_t run = T / 256;
    for (uint32_t i = threadIdx.x; i < T; i += 1024) {
        const u32x4 v = a[(uint64_t)t * T + i];
        const uint32_t d = i / run, k = i % run;
        const uint64_t o = (uint64_t)d * tiles * run + (uint64_t)t * run + k;
        if (kNarrow) {
            b12[3 * o] = v.x; b12[3 * o + 1] = v.y; b12[3 * o + 2] = v.z;
            bk[o] = (uint16_t)v.w;
        } else {
            b[o] = v;
        }
    }
}

template <int U>
__global__ __launch_bounds__(256) void k_write(u32x4* __restrict__ b, uint64_t n) {
    const uint64_t stride = (uint64_t)gridDim.x * 256 * U;
    for (uint64_t s = (uint64_t)blockIdx.x * 256 * U + threadIdx.x; s < n; s += stride)
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t i = s + (uint64_t)u * 256;
            if (i < n) b[i] = u32x4{(uint32_t)i, 1u, 2u, 3u};
        }
}

template <typename F>
float best_ms(F launch) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    launch();
    CK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int r = 0; r < 5; ++r) {
        CK(hipEventRecord(e0));
        launch();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        best = ms < best ? ms : best;
    }
    CK(hipEventDestroy(e0));
    CK(hipEventDestroy(e1));
    return best;
}

int main(int argc, char** argv) {
    const uint64_t bytes = (argc > 1 ? strtoull(argv[1], nullptr, 10) : 8ull) << 30;
    const uint64_t n = bytes / 16;
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    const int cus = prop.multiProcessorCount;
    u32x4 *a, *b;
    uint32_t* sink;
    CK(hipMalloc(&a, bytes));
    CK(hipMalloc(&b, bytes));
    CK(hipMalloc(&sink, 64));
    CK(hipMemset(a, 1, bytes));
    CK(hipMemset(b, 2, bytes));
    printf("buffer %.1f GiB, %d CUs\n", bytes / double(1ull << 30), cus);
    const double gb = bytes / 1e9;
    double best_r = 0, best_c = 0, best_w = 0;
    for (int wpc : {1, 2, 4, 8}) {
        const int grid = cus * wpc;
#define RD(U, NT) { float ms = best_ms([&] { k_read<U, NT><<<grid, 256>>>(a, n, sink); }); double r = gb / (ms * 1e-3); \
                    printf("read  wg/CU %d U %d nt %d : %7.3f ms %7.0f GB/s\n", wpc, U, NT, ms, r); if (r > best_r) best_r = r; }
#define CP(U, NT) { float ms = best_ms([&] { k_copy<U, NT><<<grid, 256>>>(a, b, n); }); double r = 2 * gb / (ms * 1e-3); \
                    printf("copy  wg/CU %d U %d ntst %d : %7.3f ms %7.0f GB/s (r+w)\n", wpc, U, NT, ms, r); if (r > best_c) best_c = r; }
#define WR(U) { float ms = best_ms([&] { k_write<U><<<grid, 256>>>(b, n); }); double r = gb / (ms * 1e-3); \
                printf("write wg/CU %d U %d : %7.3f ms %7.0f GB/s\n", wpc, U, ms, r); if (r > best_w) best_w = r; }
        RD(1, false) RD(4, false) RD(8, false) RD(4, true) RD(8, true)
        CP(1, false) CP(4, false) CP(8, false) CP(4, true) CP(8, true)
        WR(1) WR(4)
    }
    printf("BEST read %.0f GB/s, copy %.0f GB/s (r+w), write %.0f GB/s\n", best_r, best_c, best_w);
    // round 6: block-contiguous copies, the runtime's device-to-device copy (what torch's copy_ and the bench's
    // copy_GBs use), smaller buffers, and the level-1 scatter's own shape
    double best_b = 0;
    for (int wpc : {1, 2, 4}) {
        const int grid = cus * wpc;
        const uint64_t per = (n + grid - 1) / grid;
#define CB(U) { float ms = best_ms([&] { k_copy_blk<U><<<grid, 256>>>(a, b, n, per); }); double r = 2 * gb / (ms * 1e-3); \
                printf("copy-blk wg/CU %d U %d : %7.3f ms %7.0f GB/s (r+w)\n", wpc, U, ms, r); if (r > best_b) best_b = r; }
        CB(4) CB(8)
    }
    {
        float ms = best_ms([&] { CK(hipMemcpyAsync(b, a, bytes, hipMemcpyDeviceToDevice, 0)); });
        printf("hipMemcpy D2D : %7.3f ms %7.0f GB/s (r+w)\n", ms, 2 * gb / (ms * 1e-3));
    }
    for (uint64_t sub : {1ull << 30, 2ull << 30, 4ull << 30}) {
        const uint64_t ns = sub / 16;
        const int grid = cus * 2;
        float ms = best_ms([&] { k_copy<8, true><<<grid, 256>>>(a, b, ns); });
        printf("copy %4.1f GiB wg/CU 2 U 8 ntst : %7.3f ms %7.0f GB/s (r+w)\n", sub / double(1ull << 30), ms,
               2 * (sub / 1e9) / (ms * 1e-3));
    }
    {
        constexpr int T = 7168;                       // one level-1 sub-tile; runs of 28 records
        const uint32_t tiles = (uint32_t)(n / T);
        const uint32_t per = (tiles + 7) / 8;
        const double recs = (double)tiles * T;
        uint32_t* b12 = reinterpret_cast<uint32_t*>(b);
        uint16_t* bk = reinterpret_cast<uint16_t*>(reinterpret_cast<uint8_t*>(b) + (uint64_t)(recs * 12) + 256);
        float ms = best_ms([&] { k_scatter_runs<T, false><<<per * 8, 1024>>>(a, b, nullptr, nullptr, tiles, per); });
        printf("scatter-runs 16B (256 runs of %d) : %7.3f ms %7.0f GB/s (r+w)\n", T / 256, ms, recs * 32 / 1e9 / (ms * 1e-3));
        ms = best_ms([&] { k_scatter_runs<T, true><<<per * 8, 1024>>>(a, nullptr, b12, bk, tiles, per); });
        printf("scatter-runs 12+2B (256 runs of %d) : %7.3f ms %7.0f GB/s (r+w)\n", T / 256, ms, recs * 30 / 1e9 / (ms * 1e-3));
        const double seq = 2 * gb;
        (void)seq;
    }
    printf("BEST copy-blk %.0f GB/s (r+w)\n", best_b);
    return 0;
}
