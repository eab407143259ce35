// Microbenchmark: cost of partitioning the 1B-record fan-in into 4096-key buckets
// (the K1 half of a sort-then-resolve merge) on MI355X.
//   hist    : per changeset (one workgroup), LDS histogram of 65,536 buckets (u16 in u32)
//   offsets : off[j][b] = start of cell (b, j) in a bucket-major [b][j] layout
//   scatter : per changeset (one workgroup), LDS cursors; 16-B {lt, rank, val} + 4-B {key_lo | j << 12}
//   read    : stream of the partitioned output (proxy for the resolve pass)
//   copy    : 20 B read + 20 B write streaming copy (the ideal the scatter is measured against)
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/ubench_bucket tools/ubench_bucket.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

constexpr int kBucketBits = 12;
constexpr uint32_t kBuckets = 1u << 16;   // 2^28 keys / 4096

__device__ inline uint64_t mix(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__global__ void k_gen(uint32_t* key, int64_t* lt, uint32_t* rank, uint32_t* val, uint64_t n, uint64_t per) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t h = mix(i * 0x9E3779B97F4A7C15ull + 12345);
        key[i] = (uint32_t)(h >> 36);                       // 28 bits
        lt[i] = (int64_t)((1700000000000ll + (h & 0xFFFF)) << 16) + (int64_t)((h >> 16) & 15);
        rank[i] = (uint32_t)(i / per) + 1;
        val[i] = (uint32_t)i;
    }
}

__global__ __launch_bounds__(1024) void k_hist(const uint32_t* __restrict__ key, uint64_t per, uint64_t n,
                                               uint32_t* __restrict__ cnt /* [R][kBuckets/2] u16 pairs */) {
    extern __shared__ uint32_t h[];
    for (uint32_t b = threadIdx.x; b < kBuckets / 2; b += 1024) h[b] = 0;
    __syncthreads();
    const uint64_t beg = (uint64_t)blockIdx.x * per, end = min(beg + per, n);
    for (uint64_t i = beg + threadIdx.x; i < end; i += 1024) {
        const uint32_t b = __builtin_nontemporal_load(key + i) >> kBucketBits;
        atomicAdd(&h[b >> 1], 1u << ((b & 1) * 16));
    }
    __syncthreads();
    uint32_t* row = cnt + (uint64_t)blockIdx.x * (kBuckets / 2);
    for (uint32_t b = threadIdx.x; b < kBuckets / 2; b += 1024) row[b] = h[b];
}

// tot[b] = sum_j cnt[j][b]
__global__ void k_colsum(const uint32_t* __restrict__ cnt, uint32_t R, uint32_t* __restrict__ tot) {
    const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= kBuckets) return;
    const uint16_t* c = reinterpret_cast<const uint16_t*>(cnt);
    uint32_t s = 0;
    for (uint32_t j = 0; j < R; ++j) s += c[(uint64_t)j * kBuckets + b];
    tot[b] = s;
}

// exclusive scan of tot (one workgroup of 1024, 64 per thread)
__global__ __launch_bounds__(1024) void k_bscan(const uint32_t* __restrict__ tot, uint32_t* __restrict__ bstart) {
    __shared__ uint32_t part[1024];
    const uint32_t t = threadIdx.x;
    uint32_t s = 0;
    for (int q = 0; q < 64; ++q) s += tot[t * 64 + q];
    part[t] = s;
    __syncthreads();
    for (int off = 1; off < 1024; off <<= 1) {
        uint32_t v = t >= (uint32_t)off ? part[t - off] : 0;
        __syncthreads();
        part[t] += v;
        __syncthreads();
    }
    uint32_t run = part[t] - s;
    for (int q = 0; q < 64; ++q) { bstart[t * 64 + q] = run; run += tot[t * 64 + q]; }
}

// off[j][b] = bstart[b] + sum_{j' < j} cnt[j'][b]
__global__ void k_offsets(const uint32_t* __restrict__ cnt, const uint32_t* __restrict__ bstart, uint32_t R,
                          uint32_t* __restrict__ off) {
    const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= kBuckets) return;
    const uint16_t* c = reinterpret_cast<const uint16_t*>(cnt);
    uint32_t s = bstart[b];
    for (uint32_t j = 0; j < R; ++j) { off[(uint64_t)j * kBuckets + b] = s; s += c[(uint64_t)j * kBuckets + b]; }
}

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <int kItems>
__global__ __launch_bounds__(1024) void k_scatter(const uint32_t* __restrict__ key, const int64_t* __restrict__ lt,
                                                  const uint32_t* __restrict__ rank, const uint32_t* __restrict__ val,
                                                  uint64_t per, uint64_t n, const uint32_t* __restrict__ off,
                                                  u32x4* __restrict__ rec, uint32_t* __restrict__ kj) {
    extern __shared__ uint32_t h[];
    for (uint32_t b = threadIdx.x; b < kBuckets / 2; b += 1024) h[b] = 0;
    __syncthreads();
    const uint32_t j = blockIdx.x;
    const uint64_t beg = (uint64_t)j * per, end = min(beg + per, n);
    const uint32_t* orow = off + (uint64_t)j * kBuckets;
    for (uint64_t i0 = beg + threadIdx.x; i0 < end; i0 += 1024 * kItems) {
        uint32_t k[kItems], r[kItems], v[kItems];
        int64_t l[kItems];
#pragma unroll
        for (int q = 0; q < kItems; ++q) {
            const uint64_t i = i0 + (uint64_t)q * 1024;
            const uint64_t ii = i < end ? i : beg;
            k[q] = __builtin_nontemporal_load(key + ii);
            l[q] = __builtin_nontemporal_load(lt + ii);
            r[q] = __builtin_nontemporal_load(rank + ii);
            v[q] = __builtin_nontemporal_load(val + ii);
        }
#pragma unroll
        for (int q = 0; q < kItems; ++q) {
            const uint64_t i = i0 + (uint64_t)q * 1024;
            if (i >= end) continue;
            const uint32_t b = k[q] >> kBucketBits;
            const uint32_t old = atomicAdd(&h[b >> 1], 1u << ((b & 1) * 16));
            const uint32_t slot = (old >> ((b & 1) * 16)) & 0xFFFF;
            const uint32_t pos = orow[b] + slot;
            u32x4 o;
            o.x = (uint32_t)l[q]; o.y = (uint32_t)((uint64_t)l[q] >> 32); o.z = r[q]; o.w = v[q];
            rec[pos] = o;
            kj[pos] = (k[q] & ((1u << kBucketBits) - 1)) | (j << kBucketBits);
        }
    }
}

__global__ void k_read(const u32x4* __restrict__ rec, const uint32_t* __restrict__ kj, uint64_t n, uint32_t* sink) {
    uint32_t acc = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        u32x4 v = __builtin_nontemporal_load(rec + i);
        acc ^= v.x ^ v.w ^ __builtin_nontemporal_load(kj + i);
    }
    if (acc == 0x12345678u) sink[0] = acc;
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

struct Timer {
    hipEvent_t a, b;
    Timer() { CK(hipEventCreate(&a)); CK(hipEventCreate(&b)); }
    void start() { CK(hipEventRecord(a)); }
    float stop() { CK(hipEventRecord(b)); CK(hipEventSynchronize(b)); float ms; CK(hipEventElapsedTime(&ms, a, b)); return ms; }
};

int main(int argc, char** argv) {
    const uint32_t R = argc > 1 ? atoi(argv[1]) : 1024;
    const uint64_t per = argc > 2 ? strtoull(argv[2], 0, 10) : 976563;
    const uint64_t n = (uint64_t)R * per;
    printf("R %u per %lu n %lu\n", R, per, n);
    uint32_t *key, *rank, *val, *cnt, *tot, *bstart, *off, *kj, *sink;
    int64_t* lt;
    u32x4* rec;
    CK(hipMalloc(&key, n * 4)); CK(hipMalloc(&lt, n * 8)); CK(hipMalloc(&rank, n * 4)); CK(hipMalloc(&val, n * 4));
    CK(hipMalloc(&cnt, (uint64_t)R * kBuckets * 2)); CK(hipMalloc(&tot, kBuckets * 4)); CK(hipMalloc(&bstart, kBuckets * 4));
    CK(hipMalloc(&off, (uint64_t)R * kBuckets * 4)); CK(hipMalloc(&rec, n * 16)); CK(hipMalloc(&kj, n * 4));
    CK(hipMalloc(&sink, 64));
    k_gen<<<8192, 256>>>(key, lt, rank, val, n, per);
    CK(hipDeviceSynchronize());
    CK(hipFuncSetAttribute((const void*)k_hist, hipFuncAttributeMaxDynamicSharedMemorySize, kBuckets * 2));
    CK(hipFuncSetAttribute((const void*)k_scatter<4>, hipFuncAttributeMaxDynamicSharedMemorySize, kBuckets * 2));
    CK(hipFuncSetAttribute((const void*)k_scatter<8>, hipFuncAttributeMaxDynamicSharedMemorySize, kBuckets * 2));
    Timer t;
    for (int rep = 0; rep < 3; ++rep) {
        t.start(); k_hist<<<R, 1024, kBuckets * 2>>>(key, per, n, cnt); float th = t.stop();
        t.start();
        k_colsum<<<kBuckets / 256, 256>>>(cnt, R, tot);
        k_bscan<<<1, 1024>>>(tot, bstart);
        k_offsets<<<kBuckets / 256, 256>>>(cnt, bstart, R, off);
        float to = t.stop();
        t.start(); k_scatter<4><<<R, 1024, kBuckets * 2>>>(key, lt, rank, val, per, n, off, rec, kj); float ts4 = t.stop();
        t.start(); k_scatter<8><<<R, 1024, kBuckets * 2>>>(key, lt, rank, val, per, n, off, rec, kj); float ts8 = t.stop();
        t.start(); k_read<<<8192, 256>>>(rec, kj, n, sink); float tr = t.stop();
        t.start(); k_copy<<<8192, 256>>>(key, lt, rank, val, n, rec, kj); float tc = t.stop();
        CK(hipGetLastError());
        printf("hist %.3f ms (%.0f GB/s)  offsets %.3f ms  scatter4 %.3f ms  scatter8 %.3f ms (%.0f GB/s r+w)  "
               "read %.3f ms (%.0f GB/s)  copy %.3f ms (%.0f GB/s r+w)\n",
               th, n * 4 / th / 1e6, to, ts4, ts8, n * 40 / ts4 / 1e6, tr, n * 20 / tr / 1e6, tc, n * 40 / tc / 1e6);
    }
    // sanity: cell (b=0) sizes
    return 0;
}
