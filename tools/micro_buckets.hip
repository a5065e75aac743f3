// Microbenchmark: does the number of destination buckets change the rate of the staging scatter?
// 48-B SoA changes staged as 64-B records (k_scatter's 4x4 permlane transpose, LDS cursors) into
// per-tile bucket slices, for 2^LGB buckets and several tile counts. If far fewer buckets stage
// near the sequential rate, a two-level (coarse scatter + in-merge split) design could pay.
// Build: hipcc -O3 --offload-arch=gfx950 tools/micro_buckets.hip -o tools/micro_buckets
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#define CK(x)                                                                  \
    do {                                                                       \
        hipError_t e = (x);                                                    \
        if (e != hipSuccess) {                                                 \
            printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__);    \
            return 1;                                                          \
        }                                                                      \
    } while (0)

__device__ inline uint64_t mix64(uint64_t x) {
    x ^= x >> 33; x *= 0xff51afd7ed558ccdULL; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ULL; x ^= x >> 33;
    return x;
}
__device__ inline void swap32(uint32_t &a, uint32_t &b) { auto r = __builtin_amdgcn_permlane32_swap(a, b, false, false); a = r[0]; b = r[1]; }
__device__ inline void swap16(uint32_t &a, uint32_t &b) { auto r = __builtin_amdgcn_permlane16_swap(a, b, false, false); a = r[0]; b = r[1]; }

constexpr int TH = 512;

template <int LGB, bool SEQ>
__global__ void __launch_bounds__(TH) k_stage(const uint64_t *pk, const int64_t *cv, const int64_t *dbv,
                                               const uint64_t *v0, const uint32_t *tc, const uint32_t *cl,
                                               const uint32_t *seq, const uint32_t *site, uint4 *out,
                                               uint32_t n, uint32_t tile, uint32_t ptb) {
    constexpr uint32_t NB = 1u << LGB;
    __shared__ uint32_t cur[NB];
    const uint32_t ntiles = gridDim.x;
    for (uint32_t b = threadIdx.x; b < NB; b += TH) cur[b] = b * (ptb * ntiles) + blockIdx.x * ptb;
    __syncthreads();
    const uint32_t begin = blockIdx.x * tile, end = min(n, begin + tile);
    const uint32_t lane = threadIdx.x & 63;
    for (uint32_t base = begin; base < end; base += TH * 4) {
        uint4 q[4][4];
        uint32_t d[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const uint32_t i = base + u * TH + threadIdx.x;
            const uint64_t p = pk[i], c = (uint64_t)cv[i], b = (uint64_t)dbv[i], v = v0[i];
            const uint32_t t = tc[i], l = cl[i], s = seq[i], st = site[i];
            q[u][0] = make_uint4((uint32_t)p, (uint32_t)(p >> 32), (uint32_t)c, (uint32_t)(c >> 32));
            q[u][1] = make_uint4((uint32_t)b, (uint32_t)(b >> 32), (uint32_t)v, (uint32_t)(v >> 32));
            q[u][2] = make_uint4(0, 0, t, l);
            q[u][3] = make_uint4(s, st, i, 1);
            d[u] = SEQ ? i : 0;
        }
#pragma unroll
        for (int u = 0; u < 4; u++) {
            if (!SEQ) {
                const uint64_t p = ((uint64_t)q[u][0].y << 32) | q[u][0].x;
                d[u] = atomicAdd(&cur[(uint32_t)(mix64(p) >> (64 - LGB))], 1u);
            }
            uint4 *qq = q[u];
            swap32(qq[0].x, qq[2].x); swap32(qq[0].y, qq[2].y); swap32(qq[0].z, qq[2].z); swap32(qq[0].w, qq[2].w);
            swap32(qq[1].x, qq[3].x); swap32(qq[1].y, qq[3].y); swap32(qq[1].z, qq[3].z); swap32(qq[1].w, qq[3].w);
            swap16(qq[0].x, qq[1].x); swap16(qq[0].y, qq[1].y); swap16(qq[0].z, qq[1].z); swap16(qq[0].w, qq[1].w);
            swap16(qq[2].x, qq[3].x); swap16(qq[2].y, qq[3].y); swap16(qq[2].z, qq[3].z); swap16(qq[2].w, qq[3].w);
            const uint32_t j = lane >> 4, l = lane & 15;
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const uint32_t sidx = __shfl(d[u], (int)l + 16 * k);
                out[(size_t)sidx * 4 + j] = qq[k];
            }
        }
    }
}

int main() {
    const uint32_t n = 1u << 26;
    size_t sizes[8] = {8, 8, 8, 8, 4, 4, 4, 4};
    void *in[8];
    for (int k = 0; k < 8; k++) CK(hipMalloc(&in[k], sizes[k] * n));
    {
        uint64_t *h = (uint64_t *)malloc(8ULL * n);
        uint64_t x = 12345;
        for (uint32_t i = 0; i < n; i++) { x ^= x << 13; x ^= x >> 7; x ^= x << 17; h[i] = x & 0x3FFFFF; }
        CK(hipMemcpy(in[0], h, 8ULL * n, hipMemcpyHostToDevice));
        free(h);
        for (int k = 1; k < 8; k++) CK(hipMemset(in[k], k, sizes[k] * n));
    }
    const size_t out_recs = 5ULL * n;
    uint4 *out;
    CK(hipMalloc(&out, 64ULL * out_recs));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto time_it = [&](const char *name, int lgb, uint32_t ntiles, double bytes, auto launch) {
        for (int w = 0; w < 2; w++) launch();
        CK(hipEventRecord(e0));
        const int reps = 5;
        for (int r = 0; r < reps; r++) launch();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        ms /= reps;
        printf("%-12s buckets 2^%-2d tiles %4u  %8.3f ms  %7.2f TB/s\n", name, lgb, ntiles, ms, bytes / (ms * 1e-3) / 1e12);
        return 0;
    };
    auto run = [&](auto kern, int lgb, uint32_t ntiles, bool seq) {
        const uint32_t tile = n / ntiles;
        // slice per (tile, bucket): expected tile/NB records, 1.5x + 16 slack (uniform keys); timing only
        const uint32_t ptb = (uint32_t)((double)tile / (1u << lgb) * 1.5) + 16;
        if ((size_t)ptb * ntiles * (1u << lgb) > out_recs) { printf("skip 2^%d x %u\n", lgb, ntiles); return 0; }
        return time_it(seq ? "sequential" : "slices", lgb, ntiles, 112.0 * n, [&] {
            hipLaunchKernelGGL(kern, dim3(ntiles), dim3(TH), 0, 0, (uint64_t *)in[0], (int64_t *)in[1], (int64_t *)in[2],
                               (uint64_t *)in[3], (uint32_t *)in[4], (uint32_t *)in[5], (uint32_t *)in[6],
                               (uint32_t *)in[7], out, n, tile, ptb);
        });
    };
    run(k_stage<15, true>, 15, 256, true);
    for (uint32_t nt : {256u, 1024u}) {
        run(k_stage<8, false>, 8, nt, false);
        run(k_stage<10, false>, 10, nt, false);
        run(k_stage<11, false>, 11, nt, false);
        run(k_stage<12, false>, 12, nt, false);
        run(k_stage<13, false>, 13, nt, false);
        run(k_stage<14, false>, 14, nt, false);
        run(k_stage<15, false>, 15, nt, false);
    }
    return 0;
}
