// Microbenchmark: would a cache-resident atomic cell reduction (SURVEY §7 "viable design 2") beat
// the partition + bucket merge for cl = 1 batches? Config-2 shape: 2^26 changes, uniform over 2^22
// pks x 4 cids = 16.8 M cells. Best case for the atomic design: the cell index is known without a
// hash probe (dense pk * 4 + cid) and the 8-B slot table (128 MB) fits the 256 MB Infinity Cache.
// The lexicographic argmax of (cv, value, site rank) with the earliest position among equals needs
// one atomic pass per 64-bit key word after the first, each re-reading the batch:
//   pass 1  atomicMax(slot_a[cell], cv)                        reads pk, tc, cv
//   pass 2  cv == slot_a ? atomicMax(slot_b[cell], value)      + gather slot_a
//   pass 3  both equal ? atomicMax(slot_c[cell], rank:~pos)    + gather slot_a, slot_b
//   pass 4  winner (all equal) writes its 64-B clock row at the cell
// Each pass is timed alone; the sum is the atomic design's floor on this shape.
// Build: hipcc -O3 --offload-arch=gfx950 tools/micro_atomic.hip -o tools/micro_atomic
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                  \
    do {                                                                       \
        hipError_t e = (x);                                                    \
        if (e != hipSuccess) {                                                 \
            printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__);    \
            return 1;                                                          \
        }                                                                      \
    } while (0)

constexpr int TH = 256;

__global__ void __launch_bounds__(TH) k_pass1(const uint64_t *pk, const uint32_t *tc, const uint64_t *cv,
                                              unsigned long long *sa, uint32_t n) {
    const uint32_t i = blockIdx.x * TH + threadIdx.x;
    if (i >= n) return;
    const uint64_t cell = pk[i] * 4 + (tc[i] & 3);
    atomicMax(&sa[cell], (unsigned long long)cv[i]);
}

__global__ void __launch_bounds__(TH) k_pass2(const uint64_t *pk, const uint32_t *tc, const uint64_t *cv,
                                              const uint64_t *v0, const unsigned long long *sa,
                                              unsigned long long *sb, uint32_t n) {
    const uint32_t i = blockIdx.x * TH + threadIdx.x;
    if (i >= n) return;
    const uint64_t cell = pk[i] * 4 + (tc[i] & 3);
    if (sa[cell] == cv[i]) atomicMax(&sb[cell], (unsigned long long)v0[i]);
}

__global__ void __launch_bounds__(TH) k_pass3(const uint64_t *pk, const uint32_t *tc, const uint64_t *cv,
                                              const uint64_t *v0, const uint32_t *site,
                                              const unsigned long long *sa, const unsigned long long *sb,
                                              unsigned long long *sc, uint32_t n) {
    const uint32_t i = blockIdx.x * TH + threadIdx.x;
    if (i >= n) return;
    const uint64_t cell = pk[i] * 4 + (tc[i] & 3);
    if (sa[cell] == cv[i] && sb[cell] == v0[i])
        atomicMax(&sc[cell], ((unsigned long long)site[i] << 32) | (uint32_t)~i);
}

__global__ void __launch_bounds__(TH) k_pass4(const uint64_t *pk, const uint32_t *tc, const uint64_t *cv,
                                              const uint64_t *v0, const uint64_t *dbv, const uint32_t *seq,
                                              const uint32_t *site, const unsigned long long *sc, uint4 *rows,
                                              uint32_t n) {
    const uint32_t i = blockIdx.x * TH + threadIdx.x;
    if (i >= n) return;
    const uint64_t cell = pk[i] * 4 + (tc[i] & 3);
    if ((uint32_t)~sc[cell] != i) return;
    const uint64_t p = pk[i], c = cv[i], v = v0[i], b = dbv[i];
    uint4 *r = rows + cell * 4;
    r[0] = make_uint4((uint32_t)p, (uint32_t)(p >> 32), (uint32_t)c, (uint32_t)(c >> 32));
    r[1] = make_uint4((uint32_t)b, (uint32_t)(b >> 32), (uint32_t)v, (uint32_t)(v >> 32));
    r[2] = make_uint4(0, 0, tc[i], 1);
    r[3] = make_uint4(seq[i], site[i], i, 1);
}

int main() {
    const uint32_t n = 1u << 26, npk = 1u << 22;
    const size_t cells = (size_t)(npk + 1) * 4;
    uint64_t *pk, *cv, *v0, *dbv;
    uint32_t *tc, *seq, *site;
    unsigned long long *sa, *sb, *sc;
    uint4 *rows;
    CK(hipMalloc(&pk, 8ULL * n)); CK(hipMalloc(&cv, 8ULL * n)); CK(hipMalloc(&v0, 8ULL * n));
    CK(hipMalloc(&dbv, 8ULL * n)); CK(hipMalloc(&tc, 4ULL * n)); CK(hipMalloc(&seq, 4ULL * n));
    CK(hipMalloc(&site, 4ULL * n));
    CK(hipMalloc(&sa, 8 * cells)); CK(hipMalloc(&sb, 8 * cells)); CK(hipMalloc(&sc, 8 * cells));
    CK(hipMalloc(&rows, 64 * cells));
    {
        uint64_t *h = (uint64_t *)malloc(8ULL * n);
        uint32_t *h4 = (uint32_t *)malloc(4ULL * n);
        uint64_t x = 12345;
        auto nx = [&] { x ^= x << 13; x ^= x >> 7; x ^= x << 17; return x; };
        for (uint32_t i = 0; i < n; i++) h[i] = 1 + (nx() & (npk - 1));
        CK(hipMemcpy(pk, h, 8ULL * n, hipMemcpyHostToDevice));
        for (uint32_t i = 0; i < n; i++) h[i] = 1 + (nx() % 8);
        CK(hipMemcpy(cv, h, 8ULL * n, hipMemcpyHostToDevice));
        for (uint32_t i = 0; i < n; i++) h[i] = nx() % 1000;
        CK(hipMemcpy(v0, h, 8ULL * n, hipMemcpyHostToDevice));
        CK(hipMemcpy(dbv, h, 8ULL * n, hipMemcpyHostToDevice));
        for (uint32_t i = 0; i < n; i++) h4[i] = nx() & 3;
        CK(hipMemcpy(tc, h4, 4ULL * n, hipMemcpyHostToDevice));
        for (uint32_t i = 0; i < n; i++) h4[i] = nx() % 1000;
        CK(hipMemcpy(site, h4, 4ULL * n, hipMemcpyHostToDevice));
        CK(hipMemcpy(seq, h4, 4ULL * n, hipMemcpyHostToDevice));
        free(h);
        free(h4);
    }
    hipEvent_t evs[6];
    for (auto &ev : evs) CK(hipEventCreate(&ev));
    const dim3 g((n + TH - 1) / TH);
    const int reps = 5;
    float tot[4] = {0, 0, 0, 0}, tres = 0;
    for (int r = 0; r < reps + 2; r++) {
        CK(hipEventRecord(evs[0]));
        CK(hipMemsetAsync(sa, 0, 8 * cells)); CK(hipMemsetAsync(sb, 0, 8 * cells)); CK(hipMemsetAsync(sc, 0, 8 * cells));
        CK(hipEventRecord(evs[1]));
        hipLaunchKernelGGL(k_pass1, g, dim3(TH), 0, 0, pk, tc, cv, sa, n);
        CK(hipEventRecord(evs[2]));
        hipLaunchKernelGGL(k_pass2, g, dim3(TH), 0, 0, pk, tc, cv, v0, sa, sb, n);
        CK(hipEventRecord(evs[3]));
        hipLaunchKernelGGL(k_pass3, g, dim3(TH), 0, 0, pk, tc, cv, v0, site, sa, sb, sc, n);
        CK(hipEventRecord(evs[4]));
        hipLaunchKernelGGL(k_pass4, g, dim3(TH), 0, 0, pk, tc, cv, v0, dbv, seq, site, sc, rows, n);
        CK(hipEventRecord(evs[5]));
        CK(hipEventSynchronize(evs[5]));
        if (r < 2) continue;
        float ms;
        CK(hipEventElapsedTime(&ms, evs[0], evs[1])); tres += ms;
        for (int k = 0; k < 4; k++) { CK(hipEventElapsedTime(&ms, evs[k + 1], evs[k + 2])); tot[k] += ms; }
    }
    const char *names[4] = {"pass1 atomicMax cv", "pass2 atomicMax value", "pass3 atomicMax rank:pos",
                            "pass4 winner row write"};
    float sum = 0;
    printf("2^26 changes, 2^22 pks x 4 cids (%zu cells, 8-B slot tables %zu MB each)\n", cells, 8 * cells >> 20);
    printf("%-26s %8.3f ms\n", "slot reset (3 memsets)", tres / reps);
    for (int k = 0; k < 4; k++) {
        printf("%-26s %8.3f ms  %6.2f G atomics-or-changes/s\n", names[k], tot[k] / reps, n / (tot[k] / reps * 1e-3) / 1e9);
        sum += tot[k] / reps;
    }
    printf("%-26s %8.3f ms (excluding reset; no hash probe, no prior state, no impacts)\n", "atomic design floor", sum);
    return 0;
}
