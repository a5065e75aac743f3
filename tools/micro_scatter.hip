// Microbenchmark: what does MI355X give for the staging pass's memory pattern?
// N changes, SoA input 48 B/change, 64-B records written to (a) sequential (b) bucket-slice
// positions like k_scatter (c) a random permutation; plus read-only / write-only baselines.
// Build: hipcc -O3 --offload-arch=gfx950 tools/micro_scatter.hip -o tools/micro_scatter
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

__device__ inline uint64_t mix64(uint64_t x) {
    x ^= x >> 33; x *= 0xff51afd7ed558ccdULL; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ULL; x ^= x >> 33;
    return x;
}

__device__ inline void swap32(uint32_t &a, uint32_t &b) { auto r = __builtin_amdgcn_permlane32_swap(a, b, false, false); a = r[0]; b = r[1]; }
__device__ inline void swap16(uint32_t &a, uint32_t &b) { auto r = __builtin_amdgcn_permlane16_swap(a, b, false, false); a = r[0]; b = r[1]; }

template <bool NT>
__device__ inline void store64_wave(uint4 *base, uint32_t idx, uint4 q0, uint4 q1, uint4 q2, uint4 q3) {
    uint4 q[4] = {q0, q1, q2, q3};
    swap32(q[0].x, q[2].x); swap32(q[0].y, q[2].y); swap32(q[0].z, q[2].z); swap32(q[0].w, q[2].w);
    swap32(q[1].x, q[3].x); swap32(q[1].y, q[3].y); swap32(q[1].z, q[3].z); swap32(q[1].w, q[3].w);
    swap16(q[0].x, q[1].x); swap16(q[0].y, q[1].y); swap16(q[0].z, q[1].z); swap16(q[0].w, q[1].w);
    swap16(q[2].x, q[3].x); swap16(q[2].y, q[3].y); swap16(q[2].z, q[3].z); swap16(q[2].w, q[3].w);
    const uint32_t lane = threadIdx.x & 63, j = lane >> 4, l = lane & 15;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const uint32_t sidx = __shfl(idx, (int)l + 16 * k);
        typedef uint32_t v4u __attribute__((ext_vector_type(4)));
        const v4u t = {q[k].x, q[k].y, q[k].z, q[k].w};
        if (NT) __builtin_nontemporal_store(t, reinterpret_cast<v4u *>(&base[(size_t)sidx * 4 + j]));
        else base[(size_t)sidx * 4 + j] = q[k];
    }
}

// mode 0: dest = i; 1: dest = bucket-slice position (hash bucket, 32K buckets, per-WG slice cursor
// emulated by dest = bucket * per + (i % per)); 2: dest = random permutation (xor-shift bijection)
__global__ void k_stage(const uint64_t *pk, const int64_t *cv, const int64_t *dbv, const uint64_t *v0,
                        const uint32_t *tc, const uint32_t *cl, const uint32_t *seq, const uint32_t *site,
                        uint4 *out, uint32_t n, int mode, uint32_t lgn) {
    for (uint32_t base = blockIdx.x * blockDim.x; base < n; base += gridDim.x * blockDim.x) {
        const uint32_t i = base + threadIdx.x;
        uint4 q0{}, q1{}, q2{}, q3{};
        uint32_t d = 0;
        if (i < n) {
            const uint64_t p = pk[i], c = (uint64_t)cv[i], b = (uint64_t)dbv[i], v = v0[i];
            q0 = make_uint4((uint32_t)p, (uint32_t)(p >> 32), (uint32_t)c, (uint32_t)(c >> 32));
            q1 = make_uint4((uint32_t)b, (uint32_t)(b >> 32), (uint32_t)v, (uint32_t)(v >> 32));
            q2 = make_uint4(0, 0, tc[i], cl[i]);
            q3 = make_uint4(seq[i], site[i], i, 1);
            if (mode == 0 || mode == 3) d = i;
            else if (mode == 1) {
                const uint32_t bk = (uint32_t)(mix64(p) >> 49);  // 32K buckets
                const uint32_t per = n >> 15;
                d = bk * per + (uint32_t)(mix64(i) % per);       // random slot within the bucket slice
            } else {
                d = (uint32_t)(mix64(i) & ((1u << lgn) - 1));    // not a bijection; fine for bandwidth
            }
        }
        if (mode >= 3) store64_wave<true>(out, d, q0, q1, q2, q3);
        else store64_wave<false>(out, d, q0, q1, q2, q3);
    }
}

__global__ void k_read(const uint64_t *pk, const int64_t *cv, const int64_t *dbv, const uint64_t *v0,
                       const uint32_t *tc, const uint32_t *cl, const uint32_t *seq, const uint32_t *site,
                       uint64_t *sink, uint32_t n) {
    uint64_t acc = 0;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
        acc += pk[i] + cv[i] + dbv[i] + v0[i] + tc[i] + cl[i] + seq[i] + site[i];
    if (acc == 0x123456789ULL) sink[0] = acc;
}

__global__ void k_read_rec(const uint4 *in, uint64_t *sink, uint32_t n) {
    uint64_t acc = 0;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n * 4; i += gridDim.x * blockDim.x) {
        const uint4 q = in[i];
        acc += q.x + q.y + q.z + q.w;
    }
    if (acc == 0x123456789ULL) sink[0] = acc;
}

int main(int argc, char **argv) {
    const uint32_t lgn = 26, n = 1u << lgn;
    std::vector<void *> bufs;
    size_t sizes[8] = {8, 8, 8, 8, 4, 4, 4, 4};
    void *in[8];
    for (int k = 0; k < 8; k++) {
        CK(hipMalloc(&in[k], sizes[k] * n));
        CK(hipMemset(in[k], k + 1, sizes[k] * n));
    }
    uint4 *out;
    CK(hipMalloc(&out, 64ULL * n));
    uint64_t *sink;
    CK(hipMalloc(&sink, 64));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto time_it = [&](const char *name, double bytes, auto launch) {
        for (int w = 0; w < 2; w++) launch();
        (void)hipEventRecord(e0);
        const int reps = 5;
        for (int r = 0; r < reps; r++) launch();
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, e0, e1);
        ms /= reps;
        printf("%-40s %8.3f ms  %7.2f TB/s\n", name, ms, bytes / (ms * 1e-3) / 1e12);
    };
    const dim3 grid(4096), blk(256);
    time_it("read SoA 48B", 48.0 * n, [&] {
        hipLaunchKernelGGL(k_read, grid, blk, 0, 0, (uint64_t *)in[0], (int64_t *)in[1], (int64_t *)in[2],
                           (uint64_t *)in[3], (uint32_t *)in[4], (uint32_t *)in[5], (uint32_t *)in[6],
                           (uint32_t *)in[7], sink, n);
    });
    time_it("read records 64B", 64.0 * n, [&] { hipLaunchKernelGGL(k_read_rec, grid, blk, 0, 0, out, sink, n); });
    const char *names[5] = {"stage 48B->64B sequential", "stage 48B->64B bucket slices", "stage 48B->64B random",
                            "stage sequential, nt stores", "stage random, nt stores"};
    for (int mode = 0; mode < 5; mode++)
        time_it(names[mode], 112.0 * n, [&] {
            hipLaunchKernelGGL(k_stage, grid, blk, 0, 0, (uint64_t *)in[0], (int64_t *)in[1], (int64_t *)in[2],
                               (uint64_t *)in[3], (uint32_t *)in[4], (uint32_t *)in[5], (uint32_t *)in[6],
                               (uint32_t *)in[7], out, n, mode, lgn);
        });
    return 0;
}
