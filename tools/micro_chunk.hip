// Microbenchmark: chunked two-pass partition that keeps the intermediate in the Infinity Cache.
// The batch (2^26 SoA changes, 48 B) is cut into chunks of C changes. Per chunk:
//   pass 1: 48-B SoA -> 32-B records, LDS counting sort of a sub-tile by coarse digit (512), runs
//           reserved by one atomic per (sub-tile, digit) in a chunk-sized staging buffer that is
//           re-used by every chunk (so it can stay resident in the 256 MB MALL);
//   pass 2: staging -> final 32 K fine buckets (64 per coarse), LDS counting sort, one atomic per
//           (tile, fine digit) on global fine cursors (from a whole-batch fine histogram).
// Build: hipcc -O3 --offload-arch=gfx950 tools/micro_chunk.hip -o tools/micro_chunk
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <vector>

#define CK(x)                                                                  \
    do {                                                                       \
        hipError_t e_ = (x);                                                   \
        if (e_ != hipSuccess) {                                                \
            printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__);   \
            return 1;                                                          \
        }                                                                      \
    } while (0)

__host__ __device__ inline uint64_t mix64(uint64_t x) {
    x ^= x >> 33; x *= 0xff51afd7ed558ccdULL; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ULL; x ^= x >> 33;
    return x;
}
__device__ inline uint32_t fine_of(uint64_t pk) { return (uint32_t)(mix64(pk + 0x9E3779B97F4A7C15ULL) >> 49); }

constexpr int TH = 512;
constexpr uint32_t NF = 1u << 15, NC = 512, FPC = NF / NC;

struct Soa {
    const uint64_t *pk; const int64_t *cv; const int64_t *dbv; const uint64_t *v0;
    const uint32_t *tc; const uint32_t *cl; const uint32_t *seq; const uint32_t *site;
};

template <class T> __device__ inline T ldg(const T *p, bool nt) { return nt ? __builtin_nontemporal_load(p) : *p; }
__device__ inline void st4(uint4 *p, uint4 v, bool nt) {
    typedef uint32_t v4u __attribute__((ext_vector_type(4)));
    if (nt) { const v4u t = {v.x, v.y, v.z, v.w}; __builtin_nontemporal_store(t, reinterpret_cast<v4u *>(p)); }
    else *p = v;
}

// hist over tiles of HT changes; every tile lies in one chunk
__global__ void __launch_bounds__(TH) k_hist(Soa in, uint32_t n, uint32_t ht, uint32_t chunk, uint32_t *fine_tot,
                                             uint32_t *ch_coarse) {
    __shared__ uint32_t h[NF];
    for (uint32_t i = threadIdx.x; i < NF; i += TH) h[i] = 0;
    __syncthreads();
    const uint32_t begin = blockIdx.x * ht, end = min(n, begin + ht);
    for (uint32_t base = begin; base < end; base += TH * 8) {
        uint64_t p[8];
#pragma unroll
        for (int u = 0; u < 8; u++) { const uint32_t i = base + u * TH + threadIdx.x; p[u] = i < end ? in.pk[i] : 0; }
#pragma unroll
        for (int u = 0; u < 8; u++) { const uint32_t i = base + u * TH + threadIdx.x; if (i < end) atomicAdd(&h[fine_of(p[u])], 1u); }
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < NF; i += TH) if (h[i]) atomicAdd(&fine_tot[i], h[i]);
    uint32_t s = 0;
    for (uint32_t k = 0; k < FPC; k++) s += h[threadIdx.x * FPC + k];
    if (s) atomicAdd(&ch_coarse[(size_t)(begin / chunk) * NC + threadIdx.x], s);
}

// fine starts (whole batch); per chunk: coarse starts in the staging buffer + pass-2 tile lists
template <uint32_t SUB2>
__global__ void __launch_bounds__(1024) k_scan(const uint32_t *fine_tot, uint32_t *fine_cur, uint32_t *fine_off,
                                              const uint32_t *ch_coarse, uint32_t nch, uint32_t *ch_off,
                                              uint32_t *ch_cur, uint32_t *ch_tiles) {
    __shared__ uint32_t ws[16];
    {
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
    // one thread per chunk (few chunks)
    for (uint32_t c = threadIdx.x; c < nch; c += blockDim.x) {
        uint32_t run = 0, tiles = 0;
        for (uint32_t d = 0; d < NC; d++) {
            const uint32_t x = ch_coarse[(size_t)c * NC + d];
            ch_off[(size_t)c * (NC + 1) + d] = run;
            ch_cur[(size_t)c * NC + d] = run;
            ch_tiles[(size_t)c * (NC + 1) + d] = tiles;
            run += x;
            tiles += (x + SUB2 - 1) / SUB2;
        }
        ch_off[(size_t)c * (NC + 1) + NC] = run;
        ch_tiles[(size_t)c * (NC + 1) + NC] = tiles;
    }
}

__device__ inline uint32_t block_excl_scan(uint32_t x, uint32_t *wsum) {
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

// pass 1: one sub-tile of SUB changes per workgroup
template <uint32_t SUB, bool NTL>
__global__ void __launch_bounds__(TH) k_pass1(Soa in, uint32_t cbeg, uint32_t cend, uint32_t *ccur, uint4 *stg) {
    constexpr uint32_t PER = SUB / TH;
    __shared__ uint4 rec[SUB * 2];
    __shared__ uint32_t cnt[NC], off[NC], gb[NC], wsum[8];
    cnt[threadIdx.x] = 0;
    __syncthreads();
    const uint32_t base = cbeg + blockIdx.x * SUB;
    const uint32_t m = min(SUB, cend - base);
    uint4 q0[PER], q1[PER];
    uint32_t dg[PER], rk[PER];
#pragma unroll
    for (int u = 0; u < PER; u++) {
        const uint32_t r = u * TH + threadIdx.x, i = base + r;
        if (r < m) {
            const uint64_t p = ldg(in.pk + i, NTL), v = ldg(in.v0 + i, NTL);
            const uint64_t c = (uint64_t)ldg(in.cv + i, NTL), b = (uint64_t)ldg(in.dbv + i, NTL);
            const uint32_t t = ldg(in.tc + i, NTL), l = ldg(in.cl + i, NTL), s = ldg(in.seq + i, NTL), st = ldg(in.site + i, NTL);
            q0[u] = make_uint4((uint32_t)p, (uint32_t)(p >> 32), (uint32_t)v, (uint32_t)(v >> 32));
            q1[u] = make_uint4((uint32_t)c ^ (l << 31), (uint32_t)b, i, (s << 16) ^ st ^ t);
        }
    }
#pragma unroll
    for (int u = 0; u < PER; u++) {
        const uint32_t r = u * TH + threadIdx.x;
        if (r < m) { dg[u] = fine_of(((uint64_t)q0[u].y << 32) | q0[u].x) / FPC; rk[u] = atomicAdd(&cnt[dg[u]], 1u); }
    }
    __syncthreads();
    const uint32_t c = cnt[threadIdx.x];
    off[threadIdx.x] = block_excl_scan(c, wsum);
    gb[threadIdx.x] = c ? atomicAdd(&ccur[threadIdx.x], c) : 0;
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
        const uint32_t d = fine_of(((uint64_t)h0.y << 32) | h0.x) / FPC;
        stg[2 * (size_t)(gb[d] + r - off[d]) + (q & 1)] = x;
    }
}

// pass 2: one tile of <= SUB records of one coarse bucket of the chunk per workgroup
template <uint32_t SUB, bool NTS>
__global__ void __launch_bounds__(TH) k_pass2(const uint4 *stg, const uint32_t *off_c, const uint32_t *tiles_c,
                                            uint32_t *fine_cur, uint4 *out) {
    constexpr uint32_t PER = SUB / TH;
    __shared__ uint4 rec[SUB * 2];
    __shared__ uint32_t cnt[FPC], off[FPC], gb[FPC], s_c;
    const uint32_t t = blockIdx.x;
    if (t >= tiles_c[NC]) return;
    if (threadIdx.x == 0) {
        uint32_t lo = 0, hi = NC;
        while (hi - lo > 1) { const uint32_t mid = (lo + hi) / 2; if (tiles_c[mid] <= t) lo = mid; else hi = mid; }
        s_c = lo;
    }
    if (threadIdx.x < FPC) cnt[threadIdx.x] = 0;
    __syncthreads();
    const uint32_t c = s_c;
    const uint32_t begin = off_c[c] + (t - tiles_c[c]) * SUB, end = min(off_c[c + 1], begin + SUB);
    const uint32_t m = end - begin;
    uint4 q0[PER], q1[PER];
    uint32_t dg[PER], rk[PER];
#pragma unroll
    for (int u = 0; u < PER; u++) {
        const uint32_t r = u * TH + threadIdx.x;
        if (r < m) { q0[u] = stg[2 * (size_t)(begin + r)]; q1[u] = stg[2 * (size_t)(begin + r) + 1]; }
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
        st4(&out[2 * (size_t)(gb[d] + r - off[d]) + (q & 1)], x, NTS);
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

struct Bufs {
    Soa in;
    uint32_t *fine_tot, *fine_cur, *fine_off, *ch_coarse, *ch_off, *ch_cur, *ch_tiles;
    uint4 *stg, *fin;
    unsigned long long *chk;
};

template <uint32_t SUB1, uint32_t SUB2, bool NTL, bool NTS>
int run(const Bufs &b, uint32_t n, uint32_t chunk, const char *name) {
    const uint32_t nch = n / chunk;
    const uint32_t ht = std::min<uint32_t>(chunk, 1u << 17);
    hipEvent_t e0, e1, e2, e3;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1)); CK(hipEventCreate(&e2)); CK(hipEventCreate(&e3));
    std::vector<uint32_t> tiles((size_t)nch * (NC + 1));
    float th = 0, tp = 0;
    const int reps = 6;
    for (int r = 0; r < reps; r++) {
        CK(hipMemsetAsync(b.fine_tot, 0, 4ULL * NF));
        CK(hipMemsetAsync(b.ch_coarse, 0, 4ULL * nch * NC));
        CK(hipEventRecord(e0));
        hipLaunchKernelGGL(k_hist, dim3(n / ht), dim3(TH), 0, 0, b.in, n, ht, chunk, b.fine_tot, b.ch_coarse);
        hipLaunchKernelGGL(k_scan<SUB2>, dim3(1), dim3(1024), 0, 0, b.fine_tot, b.fine_cur, b.fine_off, b.ch_coarse, nch,
                           b.ch_off, b.ch_cur, b.ch_tiles);
        CK(hipEventRecord(e1));
        // the host would not need this copy: the pass-2 grid can be an upper bound (early exit)
        for (uint32_t c = 0; c < nch; c++) {
            hipLaunchKernelGGL((k_pass1<SUB1, NTL>), dim3((chunk + SUB1 - 1) / SUB1), dim3(TH), 0, 0, b.in, c * chunk,
                               (c + 1) * chunk, b.ch_cur + (size_t)c * NC, b.stg);
            hipLaunchKernelGGL((k_pass2<SUB2, NTS>), dim3(chunk / SUB2 + NC), dim3(TH), 0, 0, b.stg,
                               b.ch_off + (size_t)c * (NC + 1), b.ch_tiles + (size_t)c * (NC + 1), b.fine_cur, b.fin);
        }
        CK(hipEventRecord(e2));
        CK(hipEventSynchronize(e2));
        if (r >= 2) {
            float a, c2;
            CK(hipEventElapsedTime(&a, e0, e1));
            CK(hipEventElapsedTime(&c2, e1, e2));
            th += a; tp += c2;
        }
    }
    th /= reps - 2; tp /= reps - 2;
    CK(hipMemset(b.chk, 0, 16));
    hipLaunchKernelGGL(k_check, dim3(NF), dim3(256), 0, 0, b.fin, b.fine_off, b.fine_tot, b.chk, b.chk + 1);
    unsigned long long hc[2];
    CK(hipMemcpy(hc, b.chk, 16, hipMemcpyDeviceToHost));
    const unsigned long long want = (unsigned long long)n * (n - 1) / 2;
    printf("%-44s chunk %5uK  hist+scan %6.3f ms  passes %6.3f ms  total %6.3f ms  %s\n", name, chunk >> 10, th, tp,
           th + tp, (hc[0] == 0 && hc[1] == want) ? "ok" : "BAD");
    return 0;
}

int main() {
    const uint32_t n = 1u << 26;
    size_t sizes[8] = {8, 8, 8, 8, 4, 4, 4, 4};
    void *p[8];
    for (int k = 0; k < 8; k++) CK(hipMalloc(&p[k], sizes[k] * n));
    {
        std::vector<uint64_t> h(n);
        uint64_t x = 12345;
        for (uint32_t i = 0; i < n; i++) { x ^= x << 13; x ^= x >> 7; x ^= x << 17; h[i] = 1 + (x & 0x3FFFFF); }
        CK(hipMemcpy(p[0], h.data(), 8ULL * n, hipMemcpyHostToDevice));
        for (int k = 1; k < 8; k++) CK(hipMemset(p[k], k, sizes[k] * n));
    }
    Bufs b;
    b.in = Soa{(uint64_t *)p[0], (int64_t *)p[1], (int64_t *)p[2], (uint64_t *)p[3], (uint32_t *)p[4], (uint32_t *)p[5], (uint32_t *)p[6], (uint32_t *)p[7]};
    const uint32_t maxch = 256;
    CK(hipMalloc(&b.fine_tot, 4ULL * NF)); CK(hipMalloc(&b.fine_cur, 4ULL * NF)); CK(hipMalloc(&b.fine_off, 4ULL * NF));
    CK(hipMalloc(&b.ch_coarse, 4ULL * maxch * NC)); CK(hipMalloc(&b.ch_off, 4ULL * maxch * (NC + 1)));
    CK(hipMalloc(&b.ch_cur, 4ULL * maxch * NC)); CK(hipMalloc(&b.ch_tiles, 4ULL * maxch * (NC + 1)));
    CK(hipMalloc(&b.stg, 32ULL * n)); CK(hipMalloc(&b.fin, 32ULL * n)); CK(hipMalloc(&b.chk, 16));
    run<4096, 4096, false, false>(b, n, n, "unchunked (= two full passes)");
    for (uint32_t ch : {1u << 21, 1u << 22, 1u << 23}) {
        run<4096, 4096, false, false>(b, n, ch, "sub 4K/4K");
        run<4096, 4096, true, false>(b, n, ch, "sub 4K/4K nt input loads");
        run<4096, 4096, true, true>(b, n, ch, "sub 4K/4K nt loads + nt final stores");
        run<2048, 2048, false, false>(b, n, ch, "sub 2K/2K");
        run<2048, 2048, true, true>(b, n, ch, "sub 2K/2K nt loads + nt final stores");
    }
    return 0;
}
