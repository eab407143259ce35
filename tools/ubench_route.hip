// Microbenchmark of the sharded merge's routing kernels (comm_path.inc step 4) at one rank's share
// of config 4 on 8 GPUs: 125M records in 128 changesets, G = 8 owners (and G = 2): the library's
// k_route_count / k_route_scatter<true> against their vector-load, wave-aggregated forms
// (k_route_count_v / k_route_scatter_v), same inputs; outputs compared per owner as order-free sums.
// Build: hipcc -O3 --offload-arch=gfx950 -std=c++17 -I include -ldl -o tools/ubench_route tools/ubench_route.hip
#include "../crdt_amd/csrc/crdt_merge.hip"

#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

__global__ void k_fill(uint32_t* key, int64_t* lt, uint32_t* rank, uint32_t* val, uint64_t n) {
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
        uint64_t h = (i + 1) * 0x9E3779B97F4A7C15ull;
        h ^= h >> 29; h *= 0xBF58476D1CE4E5B9ull; h ^= h >> 32;
        key[i] = (uint32_t)(h & ((1u << 28) - 1));
        lt[i] = (int64_t)(((1735689600000ull + (h >> 40) % 65536) << 16) | ((h >> 20) & 15));
        rank[i] = 1 + (uint32_t)((h >> 8) % 1024);
        val[i] = (uint32_t)i;
    }
}

static uint64_t mix(uint64_t x) { x ^= x >> 31; x *= 0x7FB5D329728EA185ull; x ^= x >> 27; return x; }

int main() {
    const uint64_t n = 125000064;
    const uint32_t R = 128;
    const uint64_t per = n / R;
    uint32_t *key, *rank, *val, *o_slot, *o_rank, *o_val;
    int64_t *lt, *o_lt;
    uint64_t *o_perm, *d_offs;
    uint32_t* d_tstart;
    unsigned long long *cnt, *cur;
    CK(hipMalloc(&key, n * 4)); CK(hipMalloc(&lt, n * 8)); CK(hipMalloc(&rank, n * 4)); CK(hipMalloc(&val, n * 4));
    CK(hipMalloc(&o_slot, n * 4)); CK(hipMalloc(&o_lt, n * 8)); CK(hipMalloc(&o_rank, n * 4)); CK(hipMalloc(&o_val, n * 4));
    CK(hipMalloc(&o_perm, n * 8));
    k_fill<<<4096, 256>>>(key, lt, rank, val, n);
    std::vector<uint64_t> offs(R + 1);
    std::vector<uint32_t> ts(R + 1);
    uint32_t mt = 0, tiles = 0;
    for (uint32_t j = 0; j <= R; ++j) {
        offs[j] = std::min<uint64_t>(n, (uint64_t)j * per) + (j == R ? n - R * per : 0);
        if (j == R) offs[j] = n;
        ts[j] = tiles;
        if (j < R) {
            const uint64_t nj = std::min<uint64_t>(n, (uint64_t)(j + 1) * per) - (uint64_t)j * per + (j == R - 1 ? n - R * per : 0);
            const uint32_t t = (uint32_t)((nj + kTile - 1) / kTile);
            tiles += t;
            mt = std::max(mt, t);
        }
    }
    CK(hipMalloc(&d_offs, (R + 1) * 8)); CK(hipMalloc(&d_tstart, (R + 1) * 4));
    CK(hipMemcpy(d_offs, offs.data(), (R + 1) * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_tstart, ts.data(), (R + 1) * 4, hipMemcpyHostToDevice));
    // the frame words the library's scatter reads (Misc::fr_*: lt over the fill's range, ranks 0..1025)
    Misc hm{};
    hm.fr_lo = ~ord64((int64_t)(1735689600000ull << 16));
    hm.fr_hi = ord64((int64_t)(((1735689600000ull + 65536) << 16) | 15));
    hm.fr_rlo = ~0u;
    hm.fr_rhi = 1025;
    Misc* fm;
    CK(hipMalloc(&fm, sizeof(Misc)));
    CK(hipMemcpy(fm, &hm, sizeof(Misc), hipMemcpyHostToDevice));
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    for (uint32_t G : {8u, 2u}) {
        uint32_t nbits = 0;
        while ((1u << nbits) < G) ++nbits;
        const size_t cells = (size_t)G * R;
        CK(hipMalloc(&cnt, cells * 8)); CK(hipMalloc(&cur, cells * 8));
        const uint32_t gx = std::max<uint32_t>(1, std::min<uint32_t>(mt, std::max<uint32_t>(1, 65536u / R)));
        const dim3 grid(gx, R);
        std::vector<unsigned long long> hc[2];
        double sums[2][8] = {};
        for (int v = 0; v < 2; ++v) {
            float best_c = 1e9f, best_s = 1e9f;
            for (int rep = 0; rep < 4; ++rep) {
                CK(hipMemset(cnt, 0, cells * 8));
                CK(hipEventRecord(a));
                if (v == 0) k_route_count<<<grid, kScanThreads>>>(key, d_offs, d_tstart, 0, R, G, cnt);
                else k_route_count_v<<<grid, kScanThreads>>>(key, d_offs, d_tstart, 0, R, G, nbits, cnt);
                CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
                float ms; CK(hipEventElapsedTime(&ms, a, b)); best_c = std::min(best_c, ms);
                hc[v].resize(cells);
                CK(hipMemcpy(hc[v].data(), cnt, cells * 8, hipMemcpyDeviceToHost));
                std::vector<unsigned long long> hcur(cells);
                unsigned long long so = 0;
                for (uint32_t d = 0; d < G; ++d)
                    for (uint32_t j = 0; j < R; ++j) { hcur[(size_t)d * R + j] = so; so += hc[v][(size_t)d * R + j]; }
                CK(hipMemcpy(cur, hcur.data(), cells * 8, hipMemcpyHostToDevice));
                CK(hipEventRecord(a));
                const RouteCols snd{o_slot, o_lt, o_rank, o_val}, none{nullptr, nullptr, nullptr, nullptr};
                if (v == 0) k_route_scatter<<<grid, kScanThreads>>>(key, lt, rank, val, d_offs, d_tstart, 0, R, G, cur,
                                                                    snd, none, 0, o_perm, fm, 1u);
                else k_route_scatter_v<<<grid, kScanThreads>>>(key, lt, rank, val, d_offs, d_tstart, 0, R, G, nbits, cur,
                                                               snd, none, 0, o_perm, fm, 1u);
                CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
                CK(hipEventElapsedTime(&ms, a, b)); best_s = std::min(best_s, ms);
            }
            // order-free check: per owner, sum of mix(perm, slot, lt, val)
            std::vector<uint32_t> hs(n), hv(n);
            std::vector<int64_t> hl(n);
            std::vector<uint64_t> hp(n);
            CK(hipMemcpy(hs.data(), o_slot, n * 4, hipMemcpyDeviceToHost));
            CK(hipMemcpy(hv.data(), o_val, n * 4, hipMemcpyDeviceToHost));
            CK(hipMemcpy(hl.data(), o_lt, n * 8, hipMemcpyDeviceToHost));
            CK(hipMemcpy(hp.data(), o_perm, n * 8, hipMemcpyDeviceToHost));
            uint64_t o = 0;
            for (uint32_t d = 0; d < G; ++d) {
                uint64_t tot = 0;
                for (uint32_t j = 0; j < R; ++j) tot += hc[v][(size_t)d * R + j];
                uint64_t acc = 0;
                for (uint64_t x = o; x < o + tot; ++x) acc += mix(hp[x] ^ ((uint64_t)hs[x] << 40) ^ mix((uint64_t)hl[x]) ^ ((uint64_t)hv[x] << 7));
                sums[v][d] = (double)(acc >> 11);
                o += tot;
            }
            printf("G=%u %-22s count %.3f ms  scatter %.3f ms  (%.1f GB/s read+write in the scatter)\n", G,
                   v ? "vector + aggregated" : "as built", best_c, best_s, n * 36.0 / (best_s * 1e6));
        }
        bool same = hc[0] == hc[1];
        for (uint32_t d = 0; d < G; ++d) same = same && sums[0][d] == sums[1][d];
        printf("G=%u counts and per-owner outputs equal: %s\n", G, same ? "yes" : "NO");
        CK(hipFree(cnt)); CK(hipFree(cur));
    }
    return 0;
}
