// Microbenchmark: two-pass MSD bucket partition of 2^26 SoA changes (48 B) into 32-B records,
// 512 coarse buckets (pass 1) x 64 fine buckets each (pass 2) = 32 K merge buckets, each pass an
// LDS counting sort of 4 K-record sub-tiles so that global writes are runs, not scattered records.
// Checks that every record lands in its fine bucket. Compare with one-pass 64-B scatter (2.17 ms).
// Build: hipcc -O3 --offload-arch=gfx950 tools/micro_msd.hip -o tools/micro_msd
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <vector>

#define CK(x)                                                                  \
    do {                                                                       \
        hipError_t e = (x);                                                    \
        if (e != hipSuccess) {                                                 \
            printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__);    \
            return 1;                                                          \
        }                                                                      \
    } while (0)

__host__ __device__ inline uint64_t mix64(uint64_t x) {
    x ^= x >> 33; x *= 0xff51afd7ed558ccdULL; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ULL; x ^= x >> 33;
    return x;
}
__device__ inline uint32_t fine_of(uint64_t pk) { return (uint32_t)(mix64(pk + 0x9E3779B97F4A7C15ULL) >> 49); }

constexpr int TH = 512;
constexpr uint32_t NF = 1u << 15, NC = 512, FPC = NF / NC;  // fine, coarse, fine per coarse
constexpr uint32_t SUB = 4096, PER = SUB / TH;             // records per LDS sub-tile, per thread

struct Soa {
    const uint64_t *pk; const int64_t *cv; const int64_t *dbv; const uint64_t *v0;
    const uint32_t *tc; const uint32_t *cl; const uint32_t *seq; const uint32_t *site;
};

// hist: per tile LDS fine histogram; fine totals by coalesced atomics; per (tile, coarse) counts
__global__ void __launch_bounds__(TH) k_hist(Soa in, uint32_t n, uint32_t tile, uint32_t *tc_cnt, uint32_t *fine_tot) {
    __shared__ uint32_t h[NF];
    for (uint32_t i = threadIdx.x; i < NF; i += TH) h[i] = 0;
    __syncthreads();
    const uint32_t begin = blockIdx.x * tile, end = min(n, begin + tile);
    for (uint32_t base = begin; base < end; base += TH * 8) {
        uint64_t p[8];
#pragma unroll
        for (int u = 0; u < 8; u++) { const uint32_t i = base + u * TH + threadIdx.x; p[u] = i < end ? in.pk[i] : 0; }
#pragma unroll
        for (int u = 0; u < 8; u++) { const uint32_t i = base + u * TH + threadIdx.x; if (i < end) atomicAdd(&h[fine_of(p[u])], 1u); }
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < NF; i += TH) if (h[i]) atomicAdd(&fine_tot[i], h[i]);
    // coarse counts of this tile: 64 fine counters per coarse digit
    const uint32_t c = threadIdx.x;  // TH == NC
    uint32_t s = 0;
    for (uint32_t k = 0; k < FPC; k++) s += h[c * FPC + k];
    tc_cnt[(size_t)blockIdx.x * NC + c] = s;
}

// scans: coarse per-(tile, coarse) offsets (column prefix), coarse starts, fine starts, pass-2 tiles
__global__ void __launch_bounds__(1024) k_scan(uint32_t *tc_cnt, uint32_t ntiles, const uint32_t *fine_tot,
                                              uint32_t *fine_off, uint32_t *fine_cur, uint32_t *coarse_off,
                                              uint32_t *coarse_cnt, uint32_t *p2_tile_start) {
    __shared__ uint32_t tot[NC], st[NC];
    for (uint32_t c = threadIdx.x; c < NC; c += blockDim.x) {
        uint32_t run = 0;
        for (uint32_t t = 0; t < ntiles; t++) { const uint32_t x = tc_cnt[(size_t)t * NC + c]; tc_cnt[(size_t)t * NC + c] = run; run += x; }
        tot[c] = run;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t run = 0, tiles = 0;
        for (uint32_t c = 0; c < NC; c++) {
            st[c] = run; coarse_off[c] = run; coarse_cnt[c] = tot[c]; p2_tile_start[c] = tiles;
            run += tot[c]; tiles += (tot[c] + SUB - 1) / SUB;
        }
        p2_tile_start[NC] = tiles;
    }
    __syncthreads();
    {   // fine starts: 32 consecutive counters per thread, block scan of the thread sums
        __shared__ uint32_t ws[16];
        const uint32_t f0 = threadIdx.x * (NF / 1024);
        uint32_t loc = 0;
        for (uint32_t k = 0; k < NF / 1024; k++) loc += fine_tot[f0 + k];
        const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
        uint32_t inc = loc;
        for (int d = 1; d < 64; d <<= 1) { const uint32_t y = __shfl_up(inc, d); if (lane >= (uint32_t)d) inc += y; }
        if (lane == 63) ws[w] = inc;
        __syncthreads();
        uint32_t run = inc - loc;
        for (uint32_t k = 0; k < w; k++) run += ws[k];
        for (uint32_t k = 0; k < NF / 1024; k++) { fine_off[f0 + k] = run; fine_cur[f0 + k] = run; run += fine_tot[f0 + k]; }
    }
    for (uint32_t i = threadIdx.x; i < (size_t)ntiles * NC; i += blockDim.x) tc_cnt[i] += st[i % NC];
}

__device__ inline uint32_t block_excl_scan512(uint32_t x, uint32_t *wsum) {
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint32_t inc = x;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) { const uint32_t y = __shfl_up(inc, d); if (lane >= (uint32_t)d) inc += y; }
    if (lane == 63) wsum[w] = inc;
    __syncthreads();
    uint32_t add = 0;
    for (uint32_t k = 0; k < w; k++) add += wsum[k];
    return add + inc - x;
}

// pass 1: tile -> 32 sub-tiles of 4 K; LDS counting sort by coarse digit; runs written at cursors
__global__ void __launch_bounds__(TH) k_pass1(Soa in, uint32_t n, uint32_t tile, const uint32_t *tc_off, uint4 *out) {
    __shared__ uint4 rec[SUB * 2];
    __shared__ uint32_t cnt[NC], off[NC], cur[NC], wsum[8];
    cur[threadIdx.x] = tc_off[(size_t)blockIdx.x * NC + threadIdx.x];
    cnt[threadIdx.x] = 0;
    __syncthreads();
    const uint32_t begin = blockIdx.x * tile, end = min(n, begin + tile);
    for (uint32_t base = begin; base < end; base += SUB) {
        uint4 q0[PER], q1[PER];
        uint32_t dg[PER], rk[PER];
#pragma unroll
        for (int u = 0; u < PER; u++) {
            const uint32_t i = base + u * TH + threadIdx.x;
            if (i < end) {
                const uint64_t p = in.pk[i], v = in.v0[i], c = (uint64_t)in.cv[i], b = (uint64_t)in.dbv[i];
                const uint32_t t = in.tc[i], l = in.cl[i], s = in.seq[i], st = in.site[i];
                q0[u] = make_uint4((uint32_t)p, (uint32_t)(p >> 32), (uint32_t)v, (uint32_t)(v >> 32));
                q1[u] = make_uint4((uint32_t)c ^ (l << 31), (uint32_t)b, i, (s << 16) ^ st ^ t);
            }
        }
#pragma unroll
        for (int u = 0; u < PER; u++) {
            const uint32_t i = base + u * TH + threadIdx.x;
            if (i < end) {
                dg[u] = fine_of(((uint64_t)q0[u].y << 32) | q0[u].x) / FPC;
                rk[u] = atomicAdd(&cnt[dg[u]], 1u);
            }
        }
        __syncthreads();
        const uint32_t c = cnt[threadIdx.x];
        off[threadIdx.x] = block_excl_scan512(c, wsum);
        __syncthreads();
#pragma unroll
        for (int u = 0; u < PER; u++) {
            const uint32_t i = base + u * TH + threadIdx.x;
            if (i < end) { const uint32_t s = off[dg[u]] + rk[u]; rec[2 * s] = q0[u]; rec[2 * s + 1] = q1[u]; }
        }
        __syncthreads();
        const uint32_t m = min(SUB, end - base);
        for (uint32_t q = threadIdx.x; q < 2 * m; q += TH) {
            const uint32_t r = q >> 1;
            const uint4 x = rec[q];
            const uint4 h0 = rec[2 * r];
            const uint32_t d = fine_of(((uint64_t)h0.y << 32) | h0.x) / FPC;
            out[2 * (size_t)(cur[d] + r - off[d]) + (q & 1)] = x;
        }
        __syncthreads();
        cur[threadIdx.x] += c;
        cnt[threadIdx.x] = 0;
        __syncthreads();
    }
}

// pass 2: tiles of 4 K records inside one coarse bucket; LDS counting sort by fine digit; one
// global atomic reservation per (tile, fine digit)
__global__ void __launch_bounds__(TH) k_pass2(const uint4 *in, const uint32_t *coarse_off, const uint32_t *coarse_cnt,
                                            const uint32_t *p2_tile_start, uint32_t *fine_cur, uint4 *out) {
    __shared__ uint4 rec[SUB * 2];
    __shared__ uint32_t cnt[FPC], off[FPC], gb[FPC], s_c;
    const uint32_t t = blockIdx.x;
    if (t >= p2_tile_start[NC]) return;
    if (threadIdx.x == 0) {  // coarse bucket of this tile (binary search)
        uint32_t lo = 0, hi = NC;
        while (hi - lo > 1) { const uint32_t mid = (lo + hi) / 2; if (p2_tile_start[mid] <= t) lo = mid; else hi = mid; }
        s_c = lo;
    }
    if (threadIdx.x < FPC) cnt[threadIdx.x] = 0;
    __syncthreads();
    const uint32_t c = s_c;
    const uint32_t j = t - p2_tile_start[c];
    const uint32_t begin = coarse_off[c] + j * SUB, end = min(coarse_off[c] + coarse_cnt[c], begin + SUB);
    const uint32_t m = end - begin;
    uint4 q0[PER], q1[PER];
    uint32_t dg[PER], rk[PER];
#pragma unroll
    for (int u = 0; u < PER; u++) {
        const uint32_t r = u * TH + threadIdx.x;
        if (r < m) { q0[u] = in[2 * (size_t)(begin + r)]; q1[u] = in[2 * (size_t)(begin + r) + 1]; }
    }
#pragma unroll
    for (int u = 0; u < PER; u++) {
        const uint32_t r = u * TH + threadIdx.x;
        if (r < m) { dg[u] = fine_of(((uint64_t)q0[u].y << 32) | q0[u].x) % FPC; rk[u] = atomicAdd(&cnt[dg[u]], 1u); }
    }
    __syncthreads();
    if (threadIdx.x < 64) {
        const uint32_t x = cnt[threadIdx.x];
        uint32_t inc = x;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) { const uint32_t y = __shfl_up(inc, d); if (threadIdx.x >= (uint32_t)d) inc += y; }
        off[threadIdx.x] = inc - x;
        gb[threadIdx.x] = x ? atomicAdd(&fine_cur[c * FPC + threadIdx.x], x) : 0;
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < PER; u++) {
        const uint32_t r = u * TH + threadIdx.x;
        if (r < m) { const uint32_t s = off[dg[u]] + rk[u]; rec[2 * s] = q0[u]; rec[2 * s + 1] = q1[u]; }
    }
    __syncthreads();
    for (uint32_t q = threadIdx.x; q < 2 * m; q += TH) {
        const uint32_t r = q >> 1;
        const uint4 x = rec[q];
        const uint4 h0 = rec[2 * r];
        const uint32_t d = fine_of(((uint64_t)h0.y << 32) | h0.x) % FPC;
        out[2 * (size_t)(gb[d] + r - off[d]) + (q & 1)] = x;
    }
}

__global__ void k_check(const uint4 *recs, const uint32_t *fine_off, const uint32_t *fine_tot, unsigned long long *bad,
                        unsigned long long *possum) {
    const uint32_t f = blockIdx.x;
    unsigned long long nb = 0, ps = 0;
    for (uint32_t i = threadIdx.x; i < fine_tot[f]; i += blockDim.x) {
        const uint4 h0 = recs[2 * (size_t)(fine_off[f] + i)];
        const uint4 h1 = recs[2 * (size_t)(fine_off[f] + i) + 1];
        if (fine_of(((uint64_t)h0.y << 32) | h0.x) != f) nb++;
        ps += h1.z;
    }
    if (nb) atomicAdd(bad, nb);
    atomicAdd(possum, ps);
}

int main() {
    const uint32_t n = 1u << 26, ntiles = 512, tile = n / ntiles;
    size_t sizes[8] = {8, 8, 8, 8, 4, 4, 4, 4};
    void *b[8];
    for (int k = 0; k < 8; k++) CK(hipMalloc(&b[k], sizes[k] * n));
    {
        std::vector<uint64_t> h(n);
        uint64_t x = 12345;
        for (uint32_t i = 0; i < n; i++) { x ^= x << 13; x ^= x >> 7; x ^= x << 17; h[i] = 1 + (x & 0x3FFFFF); }
        CK(hipMemcpy(b[0], h.data(), 8ULL * n, hipMemcpyHostToDevice));
        for (int k = 1; k < 8; k++) CK(hipMemset(b[k], k, sizes[k] * n));
    }
    Soa in{(uint64_t *)b[0], (int64_t *)b[1], (int64_t *)b[2], (uint64_t *)b[3], (uint32_t *)b[4], (uint32_t *)b[5], (uint32_t *)b[6], (uint32_t *)b[7]};
    uint32_t *tc_cnt, *fine_tot, *fine_off, *fine_cur, *coarse_off, *coarse_cnt, *p2s;
    CK(hipMalloc(&tc_cnt, 4ULL * ntiles * NC));
    CK(hipMalloc(&fine_tot, 4ULL * NF)); CK(hipMalloc(&fine_off, 4ULL * NF)); CK(hipMalloc(&fine_cur, 4ULL * NF));
    CK(hipMalloc(&coarse_off, 4ULL * NC)); CK(hipMalloc(&coarse_cnt, 4ULL * NC)); CK(hipMalloc(&p2s, 4ULL * (NC + 1)));
    uint4 *mid, *fin;
    CK(hipMalloc(&mid, 32ULL * n)); CK(hipMalloc(&fin, 32ULL * n));
    unsigned long long *chk;
    CK(hipMalloc(&chk, 16));
    hipEvent_t ev[6];
    for (auto &evk : ev) CK(hipEventCreate(&evk));
    const uint32_t p2_grid = n / SUB + NC;
    float acc[5] = {0, 0, 0, 0, 0};
    const int reps = 7;
    for (int r = 0; r < reps; r++) {
        CK(hipMemset(fine_tot, 0, 4ULL * NF));
        CK(hipEventRecord(ev[0]));
        hipLaunchKernelGGL(k_hist, dim3(ntiles), dim3(TH), 0, 0, in, n, tile, tc_cnt, fine_tot);
        CK(hipEventRecord(ev[1]));
        hipLaunchKernelGGL(k_scan, dim3(1), dim3(1024), 0, 0, tc_cnt, ntiles, fine_tot, fine_off, fine_cur, coarse_off, coarse_cnt, p2s);
        CK(hipEventRecord(ev[2]));
        hipLaunchKernelGGL(k_pass1, dim3(ntiles), dim3(TH), 0, 0, in, n, tile, tc_cnt, mid);
        CK(hipEventRecord(ev[3]));
        hipLaunchKernelGGL(k_pass2, dim3(p2_grid), dim3(TH), 0, 0, mid, coarse_off, coarse_cnt, p2s, fine_cur, fin);
        CK(hipEventRecord(ev[4]));
        CK(hipEventSynchronize(ev[4]));
        if (r >= 2)
            for (int k = 0; k < 4; k++) { float ms; CK(hipEventElapsedTime(&ms, ev[k], ev[k + 1])); acc[k] += ms; }
    }
    const char *nm[4] = {"hist (pk 8 B/change)", "scan (1 WG; unoptimised)", "pass1 48B->32B coarse runs", "pass2 32B->32B fine runs"};
    const double bytes[4] = {8.0 * n, 0, 80.0 * n, 64.0 * n};
    for (int k = 0; k < 4; k++) {
        const double ms = acc[k] / (reps - 2);
        printf("%-34s %8.3f ms  %6.2f TB/s\n", nm[k], ms, bytes[k] ? bytes[k] / (ms * 1e-3) / 1e12 : 0.0);
    }
    CK(hipMemset(chk, 0, 16));
    hipLaunchKernelGGL(k_check, dim3(NF), dim3(256), 0, 0, fin, fine_off, fine_tot, chk, chk + 1);
    unsigned long long hc[2];
    CK(hipMemcpy(hc, chk, 16, hipMemcpyDeviceToHost));
    const unsigned long long want = (unsigned long long)n * (n - 1) / 2;
    printf("check: misplaced=%llu possum %s\n", hc[0], hc[1] == want ? "ok" : "MISMATCH");
    return 0;
}
