// Microbenchmark for the staging pass's record width: what does MI355X give when 48-B SoA changes
// are staged as 64-B records vs 48-B or 32-B records into per-tile bucket slices (32 K buckets, LDS
// cursors exactly like k_scatter), and how should a wave lay out the narrower stores?
// Build: hipcc -O3 --offload-arch=gfx950 tools/micro_stage32.hip -o tools/micro_stage32
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
constexpr uint32_t LGB = 15, NB = 1u << LGB;

// layout 0: 64-B record, 4x4 permlane transpose (k_scatter today)
// layout 1: 32-B record, each lane stores its own record with two dwordx4
// layout 2: 32-B record, permlane32 transpose: lanes L and L+32 store the two halves of a record
// layout 3: 32-B record, shuffles so that lanes 2r, 2r+1 store the two halves of one record
// layout 4: 32-B record as two 16-B SoA planes (quad 0 array, quad 1 array), one dwordx4 each
// layout 5: 48-B record (a PLAIN batch's record without v1 / meta), each lane stores its own 3 quads
// layout 6: 48-B record, wave-cooperative: the wave's 64 records are 192 consecutive-per-record
//           quads; store instruction k has lane L write quad 64k + L (record (64k+L)/3, part %3)
template <int LAYOUT, bool SEQ>
__global__ void __launch_bounds__(TH) k_stage(const uint64_t *pk, const int64_t *cv, const int64_t *dbv,
                                               const uint64_t *v0, const uint32_t *tc, const uint32_t *cl,
                                               const uint32_t *seq, const uint32_t *site, uint4 *out,
                                               uint32_t n, uint32_t tile, uint32_t per_tile_bucket) {
    __shared__ uint32_t cur[NB];
    const uint32_t ntiles = gridDim.x;
    for (uint32_t b = threadIdx.x; b < NB; b += TH) cur[b] = b * (per_tile_bucket * ntiles) + blockIdx.x * per_tile_bucket;
    __syncthreads();
    const uint32_t begin = blockIdx.x * tile, end = min(n, begin + tile);
    const uint32_t lane = threadIdx.x & 63;
    for (uint32_t base = begin; base < end; base += TH * 4) {
        uint4 q[4][4] = {};
        uint32_t d[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const uint32_t i = base + u * TH + threadIdx.x;
            const uint64_t p = pk[i], c = (uint64_t)cv[i], b = (uint64_t)dbv[i], v = v0[i];
            const uint32_t t = tc[i], l = cl[i], s = seq[i], st = site[i];
            if (LAYOUT >= 5) {
                q[u][0] = make_uint4((uint32_t)p, (uint32_t)(p >> 32), (uint32_t)c, (uint32_t)(c >> 32));
                q[u][1] = make_uint4((uint32_t)b, (uint32_t)(b >> 32), (uint32_t)v, (uint32_t)(v >> 32));
                q[u][2] = make_uint4(t, l ^ s, st, i);
            } else if (LAYOUT == 0) {
                q[u][0] = make_uint4((uint32_t)p, (uint32_t)(p >> 32), (uint32_t)c, (uint32_t)(c >> 32));
                q[u][1] = make_uint4((uint32_t)b, (uint32_t)(b >> 32), (uint32_t)v, (uint32_t)(v >> 32));
                q[u][2] = make_uint4(0, 0, t, l);
                q[u][3] = make_uint4(s, st, i, 1);
            } else {
                q[u][0] = make_uint4((uint32_t)p, (uint32_t)(p >> 32), (uint32_t)v, (uint32_t)(v >> 32));
                q[u][1] = make_uint4((uint32_t)c ^ l, (uint32_t)b, i, (s & 0xFFFF) | (st << 16) ^ t);
            }
            d[u] = SEQ ? i : 0;
        }
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const uint32_t i = base + u * TH + threadIdx.x;
            if (!SEQ) {
                const uint64_t p = ((uint64_t)q[u][0].y << 32) | q[u][0].x;
                d[u] = atomicAdd(&cur[(uint32_t)(mix64(p) >> (64 - LGB))], 1u);
            }
            (void)i;
            if (LAYOUT == 0) {
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
            } else if (LAYOUT == 1) {
                out[(size_t)d[u] * 2] = q[u][0];
                out[(size_t)d[u] * 2 + 1] = q[u][1];
            } else if (LAYOUT == 2) {
                uint4 *qq = q[u];
                swap32(qq[0].x, qq[1].x); swap32(qq[0].y, qq[1].y); swap32(qq[0].z, qq[1].z); swap32(qq[0].w, qq[1].w);
                const uint32_t j = lane >> 5, l = lane & 31;
#pragma unroll
                for (int k = 0; k < 2; k++) {
                    const uint32_t sidx = __shfl(d[u], (int)l + 32 * k);
                    out[(size_t)sidx * 2 + j] = qq[k];
                }
            } else if (LAYOUT == 3) {
                // instruction k: lane L writes quad (L&1) of the record of lane 32k + (L>>1)
                const uint32_t j = lane & 1;
#pragma unroll
                for (int k = 0; k < 2; k++) {
                    const int src = 32 * k + (int)(lane >> 1);
                    uint4 a, b;
                    a.x = __shfl(q[u][0].x, src); a.y = __shfl(q[u][0].y, src); a.z = __shfl(q[u][0].z, src); a.w = __shfl(q[u][0].w, src);
                    b.x = __shfl(q[u][1].x, src); b.y = __shfl(q[u][1].y, src); b.z = __shfl(q[u][1].z, src); b.w = __shfl(q[u][1].w, src);
                    const uint32_t sidx = __shfl(d[u], src);
                    out[(size_t)sidx * 2 + j] = j ? b : a;
                }
            } else if (LAYOUT == 5) {
                out[(size_t)d[u] * 3] = q[u][0];
                out[(size_t)d[u] * 3 + 1] = q[u][1];
                out[(size_t)d[u] * 3 + 2] = q[u][2];
            } else if (LAYOUT == 6) {
#pragma unroll
                for (int k = 0; k < 3; k++) {
                    const uint32_t qi = 64 * k + lane, src = qi / 3, part = qi % 3;
                    uint4 a0, a1, a2;
                    a0.x = __shfl(q[u][0].x, (int)src); a0.y = __shfl(q[u][0].y, (int)src); a0.z = __shfl(q[u][0].z, (int)src); a0.w = __shfl(q[u][0].w, (int)src);
                    a1.x = __shfl(q[u][1].x, (int)src); a1.y = __shfl(q[u][1].y, (int)src); a1.z = __shfl(q[u][1].z, (int)src); a1.w = __shfl(q[u][1].w, (int)src);
                    a2.x = __shfl(q[u][2].x, (int)src); a2.y = __shfl(q[u][2].y, (int)src); a2.z = __shfl(q[u][2].z, (int)src); a2.w = __shfl(q[u][2].w, (int)src);
                    const uint32_t sidx = __shfl(d[u], (int)src);
                    out[(size_t)sidx * 3 + part] = part == 0 ? a0 : (part == 1 ? a1 : a2);
                }
            } else {
                out[d[u]] = q[u][0];
                out[(size_t)n + (1u << 20) + d[u]] = q[u][1];
            }
        }
    }
}

// read 32-B records back with coalesced 16-B loads (the merge's load pattern)
__global__ void k_read_rec(const uint4 *in, uint64_t *sink, size_t nq) {
    uint64_t acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < nq; i += (size_t)gridDim.x * blockDim.x) {
        const uint4 q = in[i];
        acc += q.x + q.y + q.z + q.w;
    }
    if (acc == 0x123456789ULL) sink[0] = acc;
}

__global__ void k_read_soa(const uint64_t *pk, const int64_t *cv, const int64_t *dbv, const uint64_t *v0,
                           const uint32_t *tc, const uint32_t *cl, const uint32_t *seq, const uint32_t *site,
                           uint64_t *sink, uint32_t n) {
    uint64_t acc = 0;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
        acc += pk[i] + cv[i] + dbv[i] + v0[i] + tc[i] + cl[i] + seq[i] + site[i];
    if (acc == 0x123456789ULL) sink[0] = acc;
}

int main() {
    const uint32_t n = 1u << 26;
    const uint32_t ntiles = 512, tile = n / ntiles;
    const uint32_t per_tile_bucket = 4;  // expected count per (tile, bucket); overflow spills into the neighbour (timing only)
    size_t sizes[8] = {8, 8, 8, 8, 4, 4, 4, 4};
    void *in[8];
    for (int k = 0; k < 8; k++) CK(hipMalloc(&in[k], sizes[k] * n));
    // pk = random so buckets are uniform
    {
        uint64_t *h = (uint64_t *)malloc(8ULL * n);
        uint64_t x = 12345;
        for (uint32_t i = 0; i < n; i++) { x ^= x << 13; x ^= x >> 7; x ^= x << 17; h[i] = x & 0x3FFFFF; }
        CK(hipMemcpy(in[0], h, 8ULL * n, hipMemcpyHostToDevice));
        free(h);
        for (int k = 1; k < 8; k++) CK(hipMemset(in[k], k, sizes[k] * n));
    }
    const size_t out_recs = (size_t)NB * per_tile_bucket * ntiles + (1u << 20);  // + slack for spills
    uint4 *out;
    CK(hipMalloc(&out, 64ULL * out_recs));
    uint64_t *sink;
    CK(hipMalloc(&sink, 64));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto time_it = [&](const char *name, double bytes, auto launch) {
        for (int w = 0; w < 2; w++) launch();
        CK(hipEventRecord(e0));
        const int reps = 5;
        for (int r = 0; r < reps; r++) launch();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        ms /= reps;
        printf("%-52s %8.3f ms  %7.2f TB/s\n", name, ms, bytes / (ms * 1e-3) / 1e12);
        return 0;
    };
#define ARGS (uint64_t *)in[0], (int64_t *)in[1], (int64_t *)in[2], (uint64_t *)in[3], (uint32_t *)in[4], \
             (uint32_t *)in[5], (uint32_t *)in[6], (uint32_t *)in[7], out, n, tile, per_tile_bucket
    time_it("read SoA 48B", 48.0 * n, [&] {
        hipLaunchKernelGGL(k_read_soa, dim3(4096), dim3(256), 0, 0, (uint64_t *)in[0], (int64_t *)in[1],
                           (int64_t *)in[2], (uint64_t *)in[3], (uint32_t *)in[4], (uint32_t *)in[5],
                           (uint32_t *)in[6], (uint32_t *)in[7], sink, n);
    });
    time_it("read 32-B records (2 GB)", 32.0 * n, [&] { hipLaunchKernelGGL(k_read_rec, dim3(4096), dim3(256), 0, 0, out, sink, (size_t)n * 2); });
    time_it("read 48-B records (3 GB)", 48.0 * n, [&] { hipLaunchKernelGGL(k_read_rec, dim3(4096), dim3(256), 0, 0, out, sink, (size_t)n * 3); });
    time_it("read 64-B records (4 GB)", 64.0 * n, [&] { hipLaunchKernelGGL(k_read_rec, dim3(4096), dim3(256), 0, 0, out, sink, (size_t)n * 4); });
    const dim3 g(ntiles), b(TH);
    time_it("stage 64B, sequential", 112.0 * n, [&] { hipLaunchKernelGGL((k_stage<0, true>), g, b, 0, 0, ARGS); });
    time_it("stage 64B, bucket slices (k_scatter today)", 112.0 * n, [&] { hipLaunchKernelGGL((k_stage<0, false>), g, b, 0, 0, ARGS); });
    time_it("stage 32B per-lane 2x16B, sequential", 80.0 * n, [&] { hipLaunchKernelGGL((k_stage<1, true>), g, b, 0, 0, ARGS); });
    time_it("stage 32B per-lane 2x16B, bucket slices", 80.0 * n, [&] { hipLaunchKernelGGL((k_stage<1, false>), g, b, 0, 0, ARGS); });
    time_it("stage 32B permlane32 halves, sequential", 80.0 * n, [&] { hipLaunchKernelGGL((k_stage<2, true>), g, b, 0, 0, ARGS); });
    time_it("stage 32B permlane32 halves, bucket slices", 80.0 * n, [&] { hipLaunchKernelGGL((k_stage<2, false>), g, b, 0, 0, ARGS); });
    time_it("stage 32B adjacent-lane halves, sequential", 80.0 * n, [&] { hipLaunchKernelGGL((k_stage<3, true>), g, b, 0, 0, ARGS); });
    time_it("stage 32B adjacent-lane halves, bucket slices", 80.0 * n, [&] { hipLaunchKernelGGL((k_stage<3, false>), g, b, 0, 0, ARGS); });
    time_it("stage 2x16B SoA planes, sequential", 80.0 * n, [&] { hipLaunchKernelGGL((k_stage<4, true>), g, b, 0, 0, ARGS); });
    time_it("stage 48B per-lane 3x16B, sequential", 96.0 * n, [&] { hipLaunchKernelGGL((k_stage<5, true>), g, b, 0, 0, ARGS); });
    time_it("stage 48B per-lane 3x16B, bucket slices", 96.0 * n, [&] { hipLaunchKernelGGL((k_stage<5, false>), g, b, 0, 0, ARGS); });
    time_it("stage 48B wave-cooperative quads, sequential", 96.0 * n, [&] { hipLaunchKernelGGL((k_stage<6, true>), g, b, 0, 0, ARGS); });
    time_it("stage 48B wave-cooperative quads, bucket slices", 96.0 * n, [&] { hipLaunchKernelGGL((k_stage<6, false>), g, b, 0, 0, ARGS); });
    time_it("stage 2x16B SoA planes, bucket slices", 80.0 * n, [&] { hipLaunchKernelGGL((k_stage<4, false>), g, b, 0, 0, ARGS); });
    return 0;
}
