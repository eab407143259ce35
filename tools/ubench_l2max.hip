// Microbenchmark for a round-6 candidate: resolving level-1 buckets straight from records with
// the bucket's per-key state held in an XCD's L2 (no level-2 scatter).  Measures the rate of 64-bit
// atomicMax (global, no return) into an L2-resident state: each XCD (workgroup i runs on XCD i % 8) owns
// its own S-key array of 8-B maxima (S = 256K keys = 2 MB, inside the 4 MB L2), and the grid performs
// N atomics at keys drawn by a counter-based hash — uniform, or skewed to low keys (u^4: a Zipf-like head) —
// with values from the hash:
//   gen  : keys / values generated in registers (the atomic rate alone)
//   read : keys (4 B) / values (8 B) streamed from HBM as a level-1 bucket's records would be (12 B each)
// best of 5 runs each; G atomics per second.  No scalar stores: every write is a vector global atomic.
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/ubench_l2max tools/ubench_l2max.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

__device__ __host__ inline uint64_t mix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

__device__ inline uint32_t pick(uint64_t h, uint32_t S, bool skew) {
    if (!skew) return (uint32_t)(h % S);
    const double u = (double)(h >> 11) * (1.0 / 9007199254740992.0);
    const double u4 = u * u * u * u;
    return (uint32_t)(u4 * S) % S;
}

template <int U>
__global__ __launch_bounds__(256) void k_gen(unsigned long long* __restrict__ st, uint32_t S, uint64_t n, bool skew) {
    unsigned long long* my = st + (uint64_t)(blockIdx.x % 8) * S;
    const uint64_t stride = (uint64_t)gridDim.x * 256 * U;
    for (uint64_t b = (uint64_t)blockIdx.x * 256 * U + threadIdx.x; b < n; b += stride) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t i = b + (uint64_t)u * 256;
            if (i < n) {
                const uint64_t h = mix64(i);
                atomicMax(my + pick(h, S, skew), (unsigned long long)mix64(h));
            }
        }
    }
}

template <int U>
__global__ __launch_bounds__(256) void k_read(const uint32_t* __restrict__ key, const unsigned long long* __restrict__ v,
                                              unsigned long long* __restrict__ st, uint32_t S, uint64_t n) {
    unsigned long long* my = st + (uint64_t)(blockIdx.x % 8) * S;
    const uint64_t stride = (uint64_t)gridDim.x * 256 * U;
    for (uint64_t b = (uint64_t)blockIdx.x * 256 * U + threadIdx.x; b < n; b += stride) {
        uint32_t k[U];
        unsigned long long x[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t i = b + (uint64_t)u * 256;
            k[u] = i < n ? __builtin_nontemporal_load(key + i) : 0u;
            x[u] = i < n ? __builtin_nontemporal_load(v + i) : 0ull;
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (b + (uint64_t)u * 256 < n) atomicMax(my + (k[u] % S), x[u]);
    }
}

__global__ void k_fill(uint32_t* __restrict__ key, unsigned long long* __restrict__ v, uint64_t n, uint32_t S, bool skew) {
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
        const uint64_t h = mix64(i ^ 0x5EEDull);
        key[i] = pick(h, S, skew);
        v[i] = mix64(h);
    }
}

int main(int argc, char** argv) {
    const uint64_t n = argc > 1 ? strtoull(argv[1], nullptr, 10) : (1ull << 30);
    const uint32_t S = argc > 2 ? (uint32_t)strtoul(argv[2], nullptr, 10) : (1u << 18);
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    unsigned long long* st;
    uint32_t* key;
    unsigned long long* v;
    CK(hipMalloc(&st, (size_t)8 * S * 8));
    CK(hipMalloc(&key, n * 4));
    CK(hipMalloc(&v, n * 8));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    printf("records %llu, state %u keys per XCD (%u KB), %d CUs\n", (unsigned long long)n, S, S * 8 / 1024, cus);
    for (int skew = 0; skew < 2; ++skew) {
        k_fill<<<4096, 256>>>(key, v, n, S, skew);
        CK(hipDeviceSynchronize());
        for (int wpc = 2; wpc <= 8; wpc *= 2) {
            const int grid = cus * wpc;
            for (int mode = 0; mode < 2; ++mode) {
                float best = 1e30f;
                for (int r = 0; r < 5; ++r) {
                    CK(hipMemset(st, 0, (size_t)8 * S * 8));
                    CK(hipEventRecord(a));
                    if (mode == 0) k_gen<4><<<grid, 256>>>(st, S, n, skew);
                    else k_read<4><<<grid, 256>>>(key, v, st, S, n);
                    CK(hipEventRecord(b));
                    CK(hipEventSynchronize(b));
                    CK(hipGetLastError());
                    float ms;
                    CK(hipEventElapsedTime(&ms, a, b));
                    best = ms < best ? ms : best;
                }
                printf("%-4s %-7s wg/CU %d : %8.3f ms  %6.1f G atomics/s%s\n", mode ? "read" : "gen",
                       skew ? "skewed" : "uniform", wpc, best, n / (best * 1e-3) / 1e9,
                       mode ? "  (+12 B/record streamed)" : "");
                fflush(stdout);
            }
        }
    }
    CK(hipFree(st));
    CK(hipFree(key));
    CK(hipFree(v));
    return 0;
}
