// Device half of corro_process_multiple_changes (agent.cpp; interface in agent_dev.h).
//
// /root/reference/crates/corro-agent/src/agent/util.rs:765-884 walks every change of every
// changeset on the host (a SAVEPOINT per version, an INSERT per change). Here the host walks only
// the changeset headers; each per-change pass is one kernel over the caller's device batch:
//   k_cs_bad       one lane per changeset: does any change name an unknown table/column (the INSERT
//                  would fail and the version's SAVEPOINT roll back, util.rs:839-860)?
//   k_span_gather  one wave per applied changeset: its changes into the applied batch (skipped when
//                  the applied changesets are one contiguous run of the input: zero-copy)
//   k_first_imp    the first batch position whose INSERT grew crsql_rows_impacted()
//   k_impactful    per application position (k_span_blocks): impactful flags with the transaction-cumulative
//                  counter rule (util.rs:1218-1261), per-changeset "any", per-table committed counts
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstddef>
#include <cstring>

#include "agent_dev.h"
#include <chrono>
#include <cstdio>
#include <cstdlib>

#include "internal.h"

extern "C" uint64_t corro_detail_chunk_changes(const corro_ctx *ctx);  // engine.hip (apply chunk size)

namespace corro {

// prims.hip (rocPRIM)
int ovf_sort_pairs(void *temp, size_t *temp_bytes, const uint64_t *ki, uint64_t *ko, const uint32_t *vi,
                   uint32_t *vo, uint32_t n, uint32_t end_bit, hipStream_t s);
int prim_inclusive_scan_u32(void *temp, size_t *temp_bytes, const uint32_t *in, uint32_t *out, uint32_t n,
                            hipStream_t s);
int prim_segmax_scan_u64(void *temp, size_t *temp_bytes, const uint32_t *keys, const uint64_t *in, uint64_t *out,
                         uint32_t n, hipStream_t s);

namespace {

constexpr int AG_T = 256;                   // threads per workgroup: 4 waves, one changeset each
constexpr uint32_t AG_GRID_MAX = 16384;

dim3 wave_grid(uint64_t nspans) {
    return dim3((uint32_t)std::max<uint64_t>(1, std::min<uint64_t>((nspans + 3) / 4, AG_GRID_MAX)));
}

// one lane per changeset: its span's table_cids, 16-B loads when the span start is 4-aligned
// (a wave per changeset leaves each lane one 4-B load per 64 changes: latency-bound)
__device__ inline bool span_has_unknown(const uint32_t *__restrict__ tcid, uint64_t o, uint64_t c) {
    bool b = false;
    uint64_t k = 0;
    if ((o & 3) == 0) {
        const uint4 *q = reinterpret_cast<const uint4 *>(tcid + o);
        for (; k + 16 <= c; k += 16) {
            uint4 x[4];
#pragma unroll
            for (int u = 0; u < 4; u++) x[u] = q[k / 4 + u];
#pragma unroll
            for (int u = 0; u < 4; u++)
                b |= (x[u].x == CORRO_TCID_UNKNOWN) | (x[u].y == CORRO_TCID_UNKNOWN) | (x[u].z == CORRO_TCID_UNKNOWN) |
                     (x[u].w == CORRO_TCID_UNKNOWN);
        }
    }
    for (; k < c; k++) b |= tcid[o + k] == CORRO_TCID_UNKNOWN;
    return b;
}

__global__ void __launch_bounds__(AG_T) k_cs_bad(const uint32_t *__restrict__ tcid, const uint64_t *__restrict__ off,
                                                  const uint64_t *__restrict__ cnt, uint64_t nspans,
                                                  uint8_t *__restrict__ bad) {
    for (uint64_t j = (uint64_t)blockIdx.x * AG_T + threadIdx.x; j < nspans; j += (uint64_t)gridDim.x * AG_T)
        bad[j] = span_has_unknown(tcid, off[j], cnt[j]) ? 1 : 0;
}

struct GatherArgs {
    corro_changes src;   // device view of the input
    corro_changes dst;   // batch arrays (writable through const_cast)
    const uint64_t *s_src, *s_dst, *s_cnt, *s_ts;
    uint64_t nspans;
    uint32_t fill_ts;    // dst.ts from s_ts (the input has no ts array)
};

template <class T>
__device__ inline void mv(const T *s, const T *d, uint64_t i, uint64_t o) {
    if (s) const_cast<T *>(d)[o] = s[i];
}

__global__ void __launch_bounds__(AG_T) k_span_gather(GatherArgs g) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t w0 = ((uint64_t)blockIdx.x * AG_T + threadIdx.x) >> 6, nw = (uint64_t)gridDim.x * (AG_T / 64);
    for (uint64_t j = w0; j < g.nspans; j += nw) {
        const uint64_t s = g.s_src[j], d = g.s_dst[j], c = g.s_cnt[j], ts = g.s_ts[j];
        for (uint64_t k = lane; k < c; k += 64) {
            const uint64_t i = s + k, o = d + k;
            mv(g.src.pk, g.dst.pk, i, o);
            mv(g.src.table_cid, g.dst.table_cid, i, o);
            mv(g.src.col_version, g.dst.col_version, i, o);
            mv(g.src.db_version, g.dst.db_version, i, o);
            mv(g.src.cl, g.dst.cl, i, o);
            mv(g.src.seq, g.dst.seq, i, o);
            mv(g.src.site, g.dst.site, i, o);
            mv(g.src.val0, g.dst.val0, i, o);
            mv(g.src.val1, g.dst.val1, i, o);
            mv(g.src.val_type, g.dst.val_type, i, o);
            mv(g.src.val_len, g.dst.val_len, i, o);
            mv(g.src.val_off, g.dst.val_off, i, o);
            mv(g.src.val_size, g.dst.val_size, i, o);
            if (g.fill_ts) const_cast<uint64_t *>(g.dst.ts)[o] = ts;
            else mv(g.src.ts, g.dst.ts, i, o);
        }
    }
}

// first[0] = min batch position with impact > 0 (stays ~0 when none)
__global__ void __launch_bounds__(AG_T) k_first_imp(const uint8_t *__restrict__ imp, uint64_t n,
                                                     unsigned long long *first) {
    unsigned long long best = ~0ULL;
    const uint64_t nv = n / 16;
    const uint64_t t0 = (uint64_t)blockIdx.x * AG_T + threadIdx.x, nt = (uint64_t)gridDim.x * AG_T;
    for (uint64_t v = t0; v < nv; v += nt) {
        const uint4 x = reinterpret_cast<const uint4 *>(imp)[v];
        const uint32_t w[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
        for (int q = 0; q < 4; q++)
            if (w[q]) {
                best = 16 * v + 4 * q + (__ffs(w[q]) - 1) / 8;
                break;
            }
        if (best != ~0ULL) break;  // later vectors of this thread are further on
    }
    for (uint64_t i = 16 * nv + t0; i < n; i += nt)
        if (imp[i] && i < best) best = i;
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        const unsigned long long y = __shfl_xor(best, d);
        best = y < best ? y : best;
    }
    __shared__ unsigned long long l_b[AG_T / 64];
    if ((threadIdx.x & 63) == 0) l_b[threadIdx.x >> 6] = best;
    __syncthreads();
    if (threadIdx.x == 0) {  // one atomic per workgroup (same-address atomics serialise at the L2)
        for (int k = 1; k < AG_T / 64; k++) best = l_b[k] < best ? l_b[k] : best;
        if (best != ~0ULL) atomicMin(first, best);
    }
}

// Per-position passes over the applied batch. Application positions [0, nbatch) are covered by the
// spans in order (s_dst ascending, every count >= 1). A workgroup takes SPB consecutive positions:
// k_span_blocks gives it its first span, it stages the spans it overlaps in LDS and each lane finds
// the span of its positions by binary search there -- loads and stores run along positions (and
// along input indices inside a span), not one wave-latency chain per span.
constexpr uint32_t SPB = 2048;                  // positions per workgroup
constexpr uint32_t SP_PER = SPB / AG_T;         // positions per lane

__global__ void __launch_bounds__(AG_T) k_span_blocks(const uint64_t *__restrict__ s_dst, const uint64_t *__restrict__ s_cnt,
                                                       uint64_t nspans, uint32_t *__restrict__ first) {
    for (uint64_t j = (uint64_t)blockIdx.x * AG_T + threadIdx.x; j < nspans; j += (uint64_t)gridDim.x * AG_T) {
        const uint64_t d = s_dst[j], c = s_cnt[j];
        for (uint64_t b = (d + SPB - 1) / SPB; b * SPB < d + c; b++) first[b] = (uint32_t)j;
    }
}

struct SpanTile {
    uint32_t j0, ns;        // first span, spans staged
    uint64_t p0, p1;        // positions [p0, p1)
    bool head0;             // the first staged span starts inside [p0, p1)
};

// stage the spans of workgroup blockIdx.x: dst (relative to p0, clamped at 0), src, and optionally ts / cs
__device__ inline SpanTile stage_spans(const uint32_t *__restrict__ first, uint64_t nspans, uint64_t nbatch,
                                       const uint64_t *__restrict__ s_dst, const uint64_t *__restrict__ s_src,
                                       const uint64_t *__restrict__ s_ts, const uint32_t *__restrict__ s_cs,
                                       uint32_t *l_dst, uint64_t *l_src, uint64_t *l_ts, uint32_t *l_cs) {
    const uint64_t nblocks = (nbatch + SPB - 1) / SPB;
    SpanTile t;
    t.p0 = (uint64_t)blockIdx.x * SPB;
    t.p1 = t.p0 + SPB < nbatch ? t.p0 + SPB : nbatch;
    t.j0 = first[blockIdx.x];
    const uint32_t j1 = blockIdx.x + 1 < nblocks ? first[blockIdx.x + 1] : (uint32_t)(nspans - 1);
    t.ns = j1 - t.j0 + 1;
    t.head0 = s_dst[t.j0] == t.p0;
    for (uint32_t k = threadIdx.x; k < t.ns; k += AG_T) {
        const uint64_t d = s_dst[t.j0 + k];
        l_dst[k] = d > t.p0 ? (uint32_t)(d - t.p0) : 0u;
        l_src[k] = s_src[t.j0 + k] + (d < t.p0 ? t.p0 - d : 0);  // input index of the span's first position here
        if (l_ts) l_ts[k] = s_ts[t.j0 + k];
        if (l_cs) l_cs[k] = s_cs[t.j0 + k];
    }
    __syncthreads();
    return t;
}

// position -> local span map of the tile: each wave writes the positions of every 4th span (no
// per-position binary search: one LDS read per position afterwards)
__device__ inline void fill_pspan(const uint32_t *l_dst, const SpanTile &t, uint16_t *pspan) {
    const uint32_t w = threadIdx.x >> 6, lane = threadIdx.x & 63, len = (uint32_t)(t.p1 - t.p0);
    for (uint32_t k = w; k < t.ns; k += AG_T / 64) {
        const uint32_t a = l_dst[k], b = k + 1 < t.ns ? l_dst[k + 1] : len;
        for (uint32_t r = a + lane; r < b && r < len; r += 64) pspan[r] = (uint16_t)k;
    }
    __syncthreads();
}

struct ImpArgs {
    const uint8_t *imp;
    const uint32_t *tcid;
    const uint64_t *s_src, *s_dst;
    const uint32_t *s_cs;              // changeset of each span
    const uint32_t *first_span;        // k_span_blocks
    uint64_t nspans, nbatch;
    const unsigned long long *first;
    uint8_t *out;                      // impactful per input change (nullable)
    uint8_t *any;                      // per changeset
    unsigned long long *committed;     // per table (ntables > IMP_TLDS: atomics)
    unsigned long long *part;          // per (workgroup, table) counts (ntables <= IMP_TLDS)
    uint32_t ntables;
    bool tcid_by_src;                  // tcid indexed by input index (position mode), else by batch position
};
constexpr uint32_t IMP_TLDS = 32;

// impactful flag of every applied change: its own growth, except a version's first change, which
// takes the transaction-cumulative counter (any growth at or before it in the batch)
__global__ void __launch_bounds__(AG_T) k_impactful(ImpArgs a) {
    __shared__ uint32_t l_dst[SPB + 1];
    __shared__ uint64_t l_src[SPB + 1];
    __shared__ uint32_t l_cs[SPB + 1];
    __shared__ uint8_t l_any[SPB + 1];
    __shared__ uint32_t l_cnt[IMP_TLDS];
    __shared__ uint16_t pspan[SPB];
    const SpanTile t = stage_spans(a.first_span, a.nspans, a.nbatch, a.s_dst, a.s_src, nullptr, a.s_cs, l_dst, l_src,
                                   nullptr, l_cs);
    fill_pspan(l_dst, t, pspan);
    for (uint32_t k = threadIdx.x; k < t.ns; k += AG_T) l_any[k] = 0;
    if (threadIdx.x < IMP_TLDS) l_cnt[threadIdx.x] = 0;
    __syncthreads();
    const unsigned long long first = *a.first;
    const bool lds_t = a.ntables <= IMP_TLDS;
    const uint32_t lane = threadIdx.x & 63;
    // the lane's SP_PER positions: spans from LDS first, then every flag load in flight at once,
    // then the table loads of the hits, then the stores (memory-level parallelism per lane)
    uint32_t kk[SP_PER];
    uint64_t src[SP_PER];
    uint8_t st[SP_PER];  // bit 0 active, bit 1 head of its span, bit 2 hit
#pragma unroll
    for (uint32_t u = 0; u < SP_PER; u++) {
        const uint32_t r = u * AG_T + threadIdx.x;
        const uint64_t p = t.p0 + r;
        st[u] = 0;
        kk[u] = 0;
        src[u] = 0;
        if (p < t.p1) {
            const uint32_t k = pspan[r];
            kk[u] = k;
            src[u] = l_src[k] + (r - l_dst[k]);
            st[u] = 1 | ((r == l_dst[k] && (k > 0 || t.head0)) ? 2 : 0);
        }
    }
    uint8_t im[SP_PER];
#pragma unroll
    for (uint32_t u = 0; u < SP_PER; u++) im[u] = (st[u] & 1) && !(st[u] & 2) ? a.imp[t.p0 + u * AG_T + threadIdx.x] : 0;
    uint32_t tb[SP_PER];
#pragma unroll
    for (uint32_t u = 0; u < SP_PER; u++) {
        const uint64_t p = t.p0 + u * AG_T + threadIdx.x;
        const bool hit = (st[u] & 1) && ((st[u] & 2) ? first <= p : im[u] != 0);
        if (hit) st[u] |= 4;
        tb[u] = hit ? a.tcid[a.tcid_by_src ? src[u] : p] : 0xFFFFFFFFu;
    }
#pragma unroll
    for (uint32_t u = 0; u < SP_PER; u++) {
        const bool hit = st[u] & 4;
        if (a.out && (st[u] & 1)) a.out[src[u]] = hit ? 1 : 0;
        if (hit) l_any[kk[u]] = 1;
        uint32_t t_ = hit ? tb[u] >> 16 : 0xFFFFFFFFu;
        if (t_ >= a.ntables) t_ = 0xFFFFFFFFu;
        // one atomic per (wave, table): LDS counters when the tables fit, else global
        unsigned long long m = __ballot(t_ != 0xFFFFFFFFu);
        while (m) {
            const uint32_t leader = (uint32_t)__ffsll(m) - 1;
            const uint32_t tl = __shfl(t_, leader);
            const unsigned long long mt = __ballot(t_ == tl);
            if (lane == leader) {
                if (lds_t) atomicAdd(&l_cnt[tl], (uint32_t)__popcll(mt));
                else atomicAdd(&a.committed[tl], (unsigned long long)__popcll(mt));
            }
            m &= ~mt;
            if (t_ == tl) t_ = 0xFFFFFFFFu;
        }
    }
    __syncthreads();
    for (uint32_t k = threadIdx.x; k < t.ns; k += AG_T)
        if (l_any[k]) a.any[l_cs[k]] = 1;  // (spans straddling workgroups: the same value from each)
    if (lds_t && threadIdx.x < a.ntables) a.part[(uint64_t)blockIdx.x * a.ntables + threadIdx.x] = l_cnt[threadIdx.x];
}

// committed[t] += sum over workgroups of part[wg * ntables + t] (one workgroup per table)
__global__ void __launch_bounds__(AG_T) k_imp_reduce(const unsigned long long *__restrict__ part, uint64_t nwg,
                                                      uint32_t ntables, unsigned long long *__restrict__ committed) {
    __shared__ unsigned long long l[AG_T / 64];
    unsigned long long sum = 0;
    for (uint64_t w = threadIdx.x; w < nwg; w += AG_T) sum += part[w * ntables + blockIdx.x];
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) sum += __shfl_xor(sum, d);
    if ((threadIdx.x & 63) == 0) l[threadIdx.x >> 6] = sum;
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long s = 0;
        for (int k = 0; k < AG_T / 64; k++) s += l[k];
        committed[blockIdx.x] += s;
    }
}

// Position mode: the impactful flags streamed along the positions (no span staging): src_of gives
// each position's input index and whether it heads its span (a version's first change), so a lane
// needs only imp[p], src_of[p] and, for a hit, its table. Hits are stored into the zeroed output
// (out[src] = 1) and into a per-position byte map for k_span_any; table counts per (workgroup,
// table) in LDS (global atomics past IMP_TLDS tables).
constexpr uint32_t IP_U = 8;      // positions per lane per iteration
constexpr uint32_t IP_GRID = 2048;
__global__ void __launch_bounds__(AG_T) k_imp_pos(const uint8_t *__restrict__ imp, const uint32_t *__restrict__ src_of,
                                                  const uint32_t *__restrict__ tcid, uint64_t nbatch,
                                                  const unsigned long long *first_p, uint8_t *__restrict__ out,
                                                  uint8_t *__restrict__ hitp, unsigned long long *committed,
                                                  unsigned long long *part, uint32_t ntables) {
    __shared__ uint32_t l_cnt[IMP_TLDS];
    if (threadIdx.x < IMP_TLDS) l_cnt[threadIdx.x] = 0;
    __syncthreads();
    const unsigned long long first = *first_p;
    const bool lds_t = ntables <= IMP_TLDS;
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t step = (uint64_t)gridDim.x * AG_T * IP_U;
    for (uint64_t base = (uint64_t)blockIdx.x * AG_T * IP_U; base < nbatch; base += step) {
        uint32_t sv[IP_U];
        uint8_t im[IP_U];
#pragma unroll
        for (uint32_t u = 0; u < IP_U; u++) {
            const uint64_t p = base + u * AG_T + threadIdx.x;
            const uint64_t pc = p < nbatch ? p : nbatch - 1;
            sv[u] = src_of[pc];
            im[u] = imp[pc];
        }
        uint32_t tb[IP_U];
        bool hit[IP_U];
#pragma unroll
        for (uint32_t u = 0; u < IP_U; u++) {
            const uint64_t p = base + u * AG_T + threadIdx.x;
            hit[u] = p < nbatch && ((sv[u] >> 31) ? first <= p : im[u] != 0);
            tb[u] = hit[u] ? tcid[sv[u] & 0x7FFFFFFFu] : 0xFFFFFFFFu;
        }
#pragma unroll
        for (uint32_t u = 0; u < IP_U; u++) {
            const uint64_t p = base + u * AG_T + threadIdx.x;
            if (hit[u]) {
                if (out) out[sv[u] & 0x7FFFFFFFu] = 1;
                hitp[p] = 1;
            }
            uint32_t t_ = hit[u] ? tb[u] >> 16 : 0xFFFFFFFFu;
            if (t_ >= ntables) t_ = 0xFFFFFFFFu;
            unsigned long long m = __ballot(t_ != 0xFFFFFFFFu);
            while (m) {
                const uint32_t leader = (uint32_t)__ffsll(m) - 1;
                const uint32_t tl = __shfl(t_, leader);
                const unsigned long long mt = __ballot(t_ == tl);
                if (lane == leader) {
                    if (lds_t) atomicAdd(&l_cnt[tl], (uint32_t)__popcll(mt));
                    else atomicAdd(&committed[tl], (unsigned long long)__popcll(mt));
                }
                m &= ~mt;
                if (t_ == tl) t_ = 0xFFFFFFFFu;
            }
        }
    }
    __syncthreads();
    if (lds_t && threadIdx.x < ntables) part[(uint64_t)blockIdx.x * ntables + threadIdx.x] = l_cnt[threadIdx.x];
}

// any[cs of span j] = 1 when a position of span j was a hit (k_imp_pos's byte map)
__global__ void __launch_bounds__(AG_T) k_span_any(const uint8_t *__restrict__ hitp, const uint64_t *__restrict__ s_dst,
                                                   const uint64_t *__restrict__ s_cnt, const uint32_t *__restrict__ s_cs,
                                                   uint64_t nspans, uint8_t *__restrict__ any) {
    for (uint64_t j = (uint64_t)blockIdx.x * AG_T + threadIdx.x; j < nspans; j += (uint64_t)gridDim.x * AG_T) {
        const uint64_t d = s_dst[j], e = d + s_cnt[j];
        uint32_t acc = 0;
        uint64_t q = d;
        for (; q < e && (q & 3); q++) acc |= hitp[q];
        for (; q + 4 <= e && !acc; q += 4) acc |= *reinterpret_cast<const uint32_t *>(hitp + q);
        for (; q < e && !acc; q++) acc |= hitp[q];
        if (acc) any[s_cs[j]] = 1;
    }
}

// Application order of the applied changesets: key = site rank (ActorId byte order) for an applied
// changeset, past every rank otherwise; value = arrival index. A stable radix sort keeps arrival
// order inside an actor.
__global__ void __launch_bounds__(AG_T) k_span_keys(const uint32_t *__restrict__ site, const uint8_t *__restrict__ flag,
                                                     const uint32_t *__restrict__ site_rank, uint64_t ncs, uint64_t last,
                                                     uint64_t *__restrict__ key, uint32_t *__restrict__ val) {
    for (uint64_t i = (uint64_t)blockIdx.x * AG_T + threadIdx.x; i < ncs; i += (uint64_t)gridDim.x * AG_T) {
        key[i] = flag[i] ? site_rank[site[i]] : last;
        val[i] = (uint32_t)i;
    }
}

// span j (application order) of changeset val[j]
__global__ void __launch_bounds__(AG_T) k_span_build(const uint32_t *__restrict__ val, uint64_t nspans,
                                                      const uint64_t *__restrict__ off, const uint64_t *__restrict__ cnt,
                                                      const uint64_t *__restrict__ ts, uint64_t *__restrict__ s_src,
                                                      uint32_t *__restrict__ cnt32, uint64_t *__restrict__ s_ts) {
    for (uint64_t j = (uint64_t)blockIdx.x * AG_T + threadIdx.x; j < nspans; j += (uint64_t)gridDim.x * AG_T) {
        const uint32_t i = val[j];
        s_src[j] = off[i];
        cnt32[j] = (uint32_t)cnt[i];
        s_ts[j] = ts[i];
    }
}

// dst from the inclusive scan of the counts; info[0] |= 1 when the spans are not one contiguous run
__global__ void __launch_bounds__(AG_T) k_span_fin(const uint64_t *__restrict__ s_src, const uint32_t *__restrict__ cnt32,
                                                    const uint32_t *__restrict__ incl, uint64_t nspans,
                                                    uint64_t *__restrict__ s_dst, uint64_t *__restrict__ s_cnt,
                                                    unsigned int *info) {
    bool gap = false;
    for (uint64_t j = (uint64_t)blockIdx.x * AG_T + threadIdx.x; j < nspans; j += (uint64_t)gridDim.x * AG_T) {
        s_dst[j] = incl[j] - cnt32[j];
        s_cnt[j] = cnt32[j];
        if (j && s_src[j] != s_src[j - 1] + cnt32[j - 1]) gap = true;
    }
    if (__any(gap) && (threadIdx.x & 63) == 0) *info = 1u;  // (a plain store: every writer stores 1)
}

size_t al256(size_t x) { return (x + 255) & ~(size_t)255; }

struct Field {
    size_t off;   // offsetof(corro_changes, <array>)
    size_t elem;  // bytes per change
};
#define CORRO_FIELD(f, e) Field{offsetof(corro_changes, f), e}
// every per-change array of corro_changes (val_data is not per change)
const Field kFields[] = {
    CORRO_FIELD(pk, 8),  CORRO_FIELD(table_cid, 4), CORRO_FIELD(col_version, 8), CORRO_FIELD(db_version, 8),
    CORRO_FIELD(cl, 4),  CORRO_FIELD(seq, 4),       CORRO_FIELD(site, 4),         CORRO_FIELD(val0, 8),
    CORRO_FIELD(val1, 8), CORRO_FIELD(val_type, 1), CORRO_FIELD(val_len, 1),      CORRO_FIELD(ts, 8),
    CORRO_FIELD(val_off, 8), CORRO_FIELD(val_size, 4),
};
#undef CORRO_FIELD
constexpr size_t TS_OFF = offsetof(corro_changes, ts);

const void *&fld(corro_changes &c, const Field &f) {
    return *reinterpret_cast<const void **>(reinterpret_cast<char *>(&c) + f.off);
}
const void *fld(const corro_changes &c, const Field &f) {
    return *reinterpret_cast<const void *const *>(reinterpret_cast<const char *>(&c) + f.off);
}

// carve every field present in `like` (plus ts when with_ts) for n changes out of buf
int carve_fields(DevBuf &buf, const corro_changes &like, uint64_t n, bool with_ts, corro_changes &out) {
    auto wanted = [&](const Field &f) { return fld(like, f) != nullptr || (with_ts && f.off == TS_OFF); };
    size_t total = 0;
    for (const Field &f : kFields)
        if (wanted(f)) total += al256(std::max<uint64_t>(n, 1) * f.elem);
    if (int rc = buf.ensure(total + 256)) return rc;
    uint8_t *p = buf.as<uint8_t>();
    out = corro_changes{};
    out.n = n;
    for (const Field &f : kFields) {
        if (!wanted(f)) continue;
        fld(out, f) = p;
        p += al256(std::max<uint64_t>(n, 1) * f.elem);
    }
    out.val_data = like.val_data;
    out.val_data_len = like.val_data_len;
    return CORRO_OK;
}

// Device layout of a call's per-changeset and per-span arrays in d_agent_spans (n = agent_ncs):
//   0 off u64 | 1 cnt u64 | 2 ts u64 | 3 site u32 | 4 flag u8 | 5 bad u8 | 6 any u8
//   7 key u64 | 8 key' u64 | 9 val u32 | 10 val' u32 (the sort) | 11 s_src u64 | 12 s_dst u64 | 13 s_cnt u64
//   14 s_ts u64 | 15 cnt32 u32 | 16 incl u32 | 17 info u32 | 18 rocPRIM temp
struct DevCols {
    uint64_t *off, *cnt, *ts;
    uint32_t *site;
    uint8_t *flag, *bad, *any;
    uint64_t *key, *key2;
    uint32_t *val, *val2;
    uint64_t *s_src, *s_dst, *s_cnt, *s_ts;
    uint32_t *cnt32, *incl, *info;
    uint32_t *first_span;    // k_span_blocks: first span of each SPB-position workgroup
    void *temp;
    size_t temp_bytes;
};

size_t sort_temp_bytes(uint64_t n) {
    size_t t0 = 0, t1 = 0, t2 = 0;
    const uint32_t m = (uint32_t)std::max<uint64_t>(n, 1);
    ovf_sort_pairs(nullptr, &t0, nullptr, nullptr, nullptr, nullptr, m, 64, nullptr);
    prim_inclusive_scan_u32(nullptr, &t1, nullptr, nullptr, m, nullptr);
    prim_segmax_scan_u64(nullptr, &t2, nullptr, nullptr, nullptr, m, nullptr);
    return std::max(std::max(t0, t1), t2);
}

DevCols dev_cols(corro_ctx *ctx, size_t *total = nullptr) {
    const uint64_t n = std::max<uint64_t>(ctx->agent_ncs, 1);
    const size_t elem[] = {8, 8, 8, 4, 1, 1, 1, 8, 8, 4, 4, 8, 8, 8, 8, 4, 4, 4};  // (+ first_span, below)
    DevCols c{};
    void **slot[] = {(void **)&c.off, (void **)&c.cnt, (void **)&c.ts, (void **)&c.site, (void **)&c.flag,
                     (void **)&c.bad, (void **)&c.any, (void **)&c.key, (void **)&c.key2, (void **)&c.val,
                     (void **)&c.val2, (void **)&c.s_src, (void **)&c.s_dst, (void **)&c.s_cnt, (void **)&c.s_ts,
                     (void **)&c.cnt32, (void **)&c.incl, (void **)&c.info};
    uint8_t *base = ctx->d_agent_spans.as<uint8_t>();
    size_t o = 0;
    for (size_t k = 0; k < sizeof(elem) / sizeof(elem[0]); k++) {
        *slot[k] = base + o;
        o += al256(n * elem[k]);
    }
    c.first_span = reinterpret_cast<uint32_t *>(base + o);
    o += al256((ctx->agent_nbatch_max / SPB + 2) * 4);
    c.temp_bytes = sort_temp_bytes(n);
    c.temp = base + o;
    o += al256(c.temp_bytes);
    if (total) *total = o;
    return c;
}

// gather spans (device columns src/dst/cnt/ts) of dv into buf
int gather_dev(corro_ctx *ctx, const corro_changes *dv, const uint64_t *src, const uint64_t *dst, const uint64_t *cnt,
               const uint64_t *ts, uint64_t nspans, uint64_t n, bool fill_ts, DevBuf &buf, corro_changes &out) {
    if (int rc = carve_fields(buf, *dv, n, fill_ts, out)) return rc;
    if (!nspans) return CORRO_OK;
    GatherArgs g{};
    g.src = *dv;
    g.dst = out;
    g.s_src = src;
    g.s_dst = dst;
    g.s_cnt = cnt;
    g.s_ts = ts;
    g.nspans = nspans;
    g.fill_ts = fill_ts && !dv->ts;
    hipLaunchKernelGGL(k_span_gather, wave_grid(nspans), dim3(AG_T), 0, ctx->stream, g);
    CORRO_HIP_TRY(hipGetLastError());
    return CORRO_OK;
}

// position mode: ap[src] = p, src_of[p] = src | (first position of its span) << 31 and, when wanted,
// the ts of application position p (the input's per-change ts, else the changeset's), positions along
// the workgroup's spans (position mode takes inputs of < 2^31 changes)
__global__ void __launch_bounds__(AG_T) k_span_pos(const uint32_t *__restrict__ first_span, const uint64_t *__restrict__ s_src,
                                                    const uint64_t *__restrict__ s_dst, const uint64_t *__restrict__ s_ts,
                                                    uint64_t nspans, uint64_t nbatch, const uint64_t *__restrict__ in_ts,
                                                    uint32_t *__restrict__ ap, uint32_t *__restrict__ src_of,
                                                    uint64_t *__restrict__ ts_out) {
    __shared__ uint32_t l_dst[SPB + 1];
    __shared__ uint64_t l_src[SPB + 1];
    __shared__ uint64_t l_ts[SPB + 1];
    __shared__ uint16_t pspan[SPB];
    const SpanTile t = stage_spans(first_span, nspans, nbatch, s_dst, s_src, ts_out && !in_ts ? s_ts : nullptr, nullptr,
                                   l_dst, l_src, ts_out && !in_ts ? l_ts : nullptr, nullptr);
    fill_pspan(l_dst, t, pspan);
    // spans from LDS for all of the lane's positions, then every ts load in flight, then the stores
    uint64_t src[SP_PER], tv[SP_PER];
    uint32_t kk[SP_PER], hd[SP_PER];
#pragma unroll
    for (uint32_t u = 0; u < SP_PER; u++) {
        const uint32_t r = u * AG_T + threadIdx.x;
        const uint32_t k = t.p0 + r < t.p1 ? pspan[r] : 0u;
        kk[u] = k;
        src[u] = l_src[k] + (r - l_dst[k]);
        hd[u] = (r == l_dst[k] && (k > 0 || t.head0)) ? 0x80000000u : 0u;
    }
#pragma unroll
    for (uint32_t u = 0; u < SP_PER; u++) {
        const bool act = t.p0 + u * AG_T + threadIdx.x < t.p1;
        tv[u] = ts_out && act ? (in_ts ? in_ts[src[u]] : l_ts[kk[u]]) : 0ULL;
    }
#pragma unroll
    for (uint32_t u = 0; u < SP_PER; u++) {
        const uint64_t p = t.p0 + u * AG_T + threadIdx.x;
        if (p >= t.p1) continue;
        ap[src[u]] = (uint32_t)p;
        src_of[p] = (uint32_t)src[u] | hd[u];
        if (ts_out) ts_out[p] = tv[u];
    }
}

dim3 flat_grid(uint64_t n) { return dim3((uint32_t)std::max<uint64_t>(1, std::min<uint64_t>((n + AG_T - 1) / AG_T, 8192))); }

}  // namespace

int agent_dev_begin(corro_ctx *ctx, uint64_t ncs, uint64_t nchanges, AgentPinned *p) {
    static const bool prof = std::getenv("CORRO_AGENT_PROFILE") != nullptr;
    const auto t0 = std::chrono::steady_clock::now();
    auto ms = [&]() { return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count(); };
    CORRO_HIP_TRY(hipSetDevice(ctx->device));
    const double t_set = ms();
    const bool busy = prof && hipStreamQuery(ctx->stream) == hipErrorNotReady;
    CORRO_HIP_TRY(hipStreamSynchronize(ctx->stream));  // (the pinned area may still feed a copy)
    const double t_sync = ms();
    const uint64_t n = std::max<uint64_t>(ncs, 1);
    const size_t c8 = al256(n * 8), c4 = al256(n * 4), c1 = al256(n);
    const size_t total = 3 * c8 + c4 + 3 * c1 + 8 * 65536;
    if (total > ctx->h_agent_bytes) {
        if (ctx->h_agent) (void)hipHostFree(ctx->h_agent);
        ctx->h_agent = nullptr;
        ctx->h_agent_bytes = 0;
        const size_t want = total + total / 4;
        CORRO_HIP_TRY(hipHostMalloc(&ctx->h_agent, want, hipHostMallocDefault));
        ctx->h_agent_bytes = want;
    }
    uint8_t *h = static_cast<uint8_t *>(ctx->h_agent);
    p->off = reinterpret_cast<uint64_t *>(h);
    p->cnt = reinterpret_cast<uint64_t *>(h + c8);
    p->ts = reinterpret_cast<uint64_t *>(h + 2 * c8);
    p->site = reinterpret_cast<uint32_t *>(h + 3 * c8);
    p->flag = h + 3 * c8 + c4;
    p->bad = p->flag + c1;
    p->any = p->bad + c1;
    p->committed = reinterpret_cast<uint64_t *>(p->any + c1);
    ctx->agent_ncs = ncs;
    ctx->agent_nbatch_max = nchanges;
    ctx->agent_sorted_mode = false;
    const double t_pin = ms();
    size_t dtotal = 0;
    (void)dev_cols(ctx, &dtotal);
    const double t_cols = ms();
    if (int rc = ctx->d_agent_spans.ensure(dtotal + 256)) return rc;
    const int rc = ctx->d_agent_out.ensure(256 + 8 * 65536);
    if (prof)
        fprintf(stderr, "[corro agent dev begin] set=%.3f sync=%.3f (stream busy %d) pinned=%.3f cols=%.3f ensure=%.3f ms\n",
                t_set, t_sync - t_set, (int)busy, t_pin - t_sync, t_cols - t_pin, ms() - t_cols);
    return rc;
}

int agent_dev_input(corro_ctx *ctx, const corro_changes *in, int mem, corro_changes *dv) {
    CORRO_HIP_TRY(hipSetDevice(ctx->device));
    if (mem == CORRO_MEM_DEVICE) {
        *dv = *in;
        return CORRO_OK;
    }
    // host input: every field once into device scratch (pageable copies), val_data after them
    corro_changes d{};
    if (int rc = carve_fields(ctx->d_agent_in, *in, in->n, false, d)) return rc;
    for (const Field &f : kFields) {
        const void *src = fld(*in, f);
        if (!src || !in->n) continue;
        CORRO_HIP_TRY(hipMemcpyAsync(const_cast<void *>(fld(d, f)), src, in->n * f.elem, hipMemcpyHostToDevice,
                                     ctx->stream));
    }
    d.val_data = nullptr;
    d.val_data_len = 0;
    if (in->val_data && in->val_data_len) {
        if (int rc = ctx->d_agent_aux.ensure(in->val_data_len)) return rc;
        CORRO_HIP_TRY(hipMemcpyAsync(ctx->d_agent_aux.p, in->val_data, in->val_data_len, hipMemcpyHostToDevice,
                                     ctx->stream));
        d.val_data = ctx->d_agent_aux.as<uint8_t>();
        d.val_data_len = in->val_data_len;
    }
    CORRO_HIP_TRY(hipStreamSynchronize(ctx->stream));  // (pageable sources: the caller may reuse them)
    *dv = d;
    return CORRO_OK;
}

int agent_dev_bad(corro_ctx *ctx, const corro_changes *dv, const AgentPinned &p, uint64_t ncs) {
    if (!ncs) return CORRO_OK;
    hipStream_t s = ctx->stream;
    const DevCols c = dev_cols(ctx);
    CORRO_HIP_TRY(hipMemcpyAsync(c.off, p.off, ncs * 8, hipMemcpyHostToDevice, s));
    CORRO_HIP_TRY(hipMemcpyAsync(c.cnt, p.cnt, ncs * 8, hipMemcpyHostToDevice, s));
    hipLaunchKernelGGL(k_cs_bad, flat_grid(ncs), dim3(AG_T), 0, s, dv->table_cid, c.off, c.cnt, ncs, c.bad);
    CORRO_HIP_TRY(hipGetLastError());
    CORRO_HIP_TRY(hipMemcpyAsync(p.bad, c.bad, ncs, hipMemcpyDeviceToHost, s));
    CORRO_HIP_TRY(hipStreamSynchronize(s));
    return CORRO_OK;
}

int agent_dev_fetch(corro_ctx *ctx, const corro_changes *dv, const std::vector<AgentSpan> &spans, HostSpanRows &o) {
    const uint64_t ns = spans.size();
    std::vector<uint64_t> cols(4 * ns);
    uint64_t n = 0;
    for (uint64_t j = 0; j < ns; j++) {
        cols[j] = spans[j].src;
        cols[ns + j] = n;
        cols[2 * ns + j] = spans[j].count;
        cols[3 * ns + j] = spans[j].ts;
        n += spans[j].count;
    }
    if (int rc = ctx->d_agent_fetch.ensure(std::max<uint64_t>(ns, 1) * 32 + 256)) return rc;
    uint64_t *dc = ctx->d_agent_fetch.as<uint64_t>();
    if (ns) CORRO_HIP_TRY(hipMemcpy(dc, cols.data(), ns * 32, hipMemcpyHostToDevice));
    DevBuf &rows = ctx->d_agent_aux2;
    corro_changes g{};
    if (int rc = gather_dev(ctx, dv, dc, dc + ns, dc + 2 * ns, dc + 3 * ns, ns, n, false, rows, g)) return rc;
    auto get = [&](auto &vec, const void *src, size_t elem) -> int {
        vec.assign(n, 0);
        if (src && n) CORRO_HIP_TRY(hipMemcpyAsync(vec.data(), src, n * elem, hipMemcpyDeviceToHost, ctx->stream));
        return CORRO_OK;
    };
    int rc = CORRO_OK;
    if (!rc) rc = get(o.pk, g.pk, 8);
    if (!rc) rc = get(o.tcid, g.table_cid, 4);
    if (!rc) rc = get(o.cv, g.col_version, 8);
    if (!rc) rc = get(o.dbv, g.db_version, 8);
    if (!rc) rc = get(o.cl, g.cl, 4);
    if (!rc) rc = get(o.seq, g.seq, 4);
    if (!rc) rc = get(o.site, g.site, 4);
    if (!rc) rc = get(o.v0, g.val0, 8);
    if (!rc) rc = get(o.v1, g.val1, 8);
    if (!rc) rc = get(o.vt, g.val_type, 1);
    if (!rc) rc = get(o.vl, g.val_len, 1);
    if (!rc) rc = get(o.ts, g.ts, 8);
    std::vector<uint64_t> voff;
    std::vector<uint32_t> vsz;
    if (!rc) rc = get(voff, g.val_off, 8);
    if (!rc) rc = get(vsz, g.val_size, 4);
    if (rc) return rc;
    CORRO_HIP_TRY(hipStreamSynchronize(ctx->stream));
    if (!g.val_type) o.vt.assign(n, (uint8_t)CORRO_INTEGER);
    o.lv_off.assign(n, 0);
    o.lv_len.assign(n, 0);
    o.lv_data.clear();
    if (g.val_off && g.val_size && dv->val_data) {
        for (uint64_t i = 0; i < n; i++) {
            const bool lng = o.vl[i] == CORRO_VAL_LONG && (o.vt[i] == CORRO_TEXT || o.vt[i] == CORRO_BLOB);
            // a malformed span is passed on empty: the apply rejects it
            if (!lng || vsz[i] <= 16 || voff[i] > dv->val_data_len || vsz[i] > dv->val_data_len - voff[i]) continue;
            o.lv_off[i] = o.lv_data.size();
            o.lv_len[i] = vsz[i];
            o.lv_data.resize(o.lv_data.size() + vsz[i]);
            CORRO_HIP_TRY(hipMemcpy(o.lv_data.data() + o.lv_off[i], dv->val_data + voff[i], vsz[i],
                                    hipMemcpyDeviceToHost));
        }
    }
    return CORRO_OK;
}

// spans (s_src, cnt32, s_ts, s_cs written for nspans) -> their batch offsets, workgroup span table,
// then the batch: zero-copy, position mode or a gather
int spans_to_batch(corro_ctx *ctx, const corro_changes *dv, uint64_t nspans, uint64_t nbatch, bool need_ts,
                   corro_changes *batch, bool *gathered, AgentPositions *pm) {
    *gathered = false;
    if (pm) *pm = AgentPositions{};
    ctx->agent_src_of = nullptr;
    hipStream_t s = ctx->stream;
    const DevCols c = dev_cols(ctx);
    if (nspans) {
        size_t tb = c.temp_bytes;
        if (int rc = prim_inclusive_scan_u32(c.temp, &tb, c.cnt32, c.incl, (uint32_t)nspans, s)) return rc;
        CORRO_HIP_TRY(hipMemsetAsync(c.info, 0, 4, s));
        hipLaunchKernelGGL(k_span_fin, flat_grid(nspans), dim3(AG_T), 0, s, c.s_src, c.cnt32, c.incl, nspans, c.s_dst,
                           c.s_cnt, c.info);
        CORRO_HIP_TRY(hipGetLastError());
        hipLaunchKernelGGL(k_span_blocks, flat_grid(nspans), dim3(AG_T), 0, s, c.s_dst, c.s_cnt, nspans, c.first_span);
        CORRO_HIP_TRY(hipGetLastError());
    }
    // zero-copy: one contiguous run, pairs of changes 16-B aligned (the scatter's paired loads), and
    // the timestamps already per change (or none needed)
    uint32_t info = 1;
    uint64_t s0 = 0;
    if (nspans) {
        CORRO_HIP_TRY(hipMemcpyAsync(&info, c.info, 4, hipMemcpyDeviceToHost, s));
        CORRO_HIP_TRY(hipMemcpyAsync(&s0, c.s_src, 8, hipMemcpyDeviceToHost, s));
        CORRO_HIP_TRY(hipStreamSynchronize(s));
    }
    if (nspans && info == 0 && (s0 & 1) == 0 && (!need_ts || dv->ts)) {
        corro_changes b = *dv;
        b.n = nbatch;
        for (const Field &f : kFields) {
            const void *q = fld(*dv, f);
            if (q) fld(b, f) = static_cast<const uint8_t *>(q) + s0 * f.elem;
        }
        if (!need_ts && !dv->ts) b.ts = nullptr;
        *batch = b;
        return CORRO_OK;
    }
    // position mode: the merge stages the input where it lies, each change with its application
    // position, instead of a gather of every field into application order (one chunk, the apply's
    // alignment of device batches)
    auto aligned = [](const void *q, uintptr_t a) { return !q || ((uintptr_t)q % a) == 0; };
    const char *fg = std::getenv("CORRO_AGENT_GATHER");  // tests: force the gather path
    if (pm && nspans && !(fg && fg[0] == '1') && dv->n <= corro_detail_chunk_changes(ctx) && dv->n < (1ULL << 31) &&
        aligned(dv->pk, 16) && aligned(dv->col_version, 16) &&
        aligned(dv->db_version, 16) && aligned(dv->val0, 16) && aligned(dv->val1, 16) && aligned(dv->table_cid, 8) &&
        aligned(dv->cl, 8) && aligned(dv->seq, 8) && aligned(dv->site, 8)) {
        // per-position ts only from the changesets: an input with per-change ts is staged with them
        // (the apply puts an INTEGER batch's ts in its staged records, else gathers them by position)
        const bool want_ts = need_ts && !dv->ts;
        const size_t o_src = al256(dv->n * 4), o_ts = o_src + al256(nbatch * 4);
        if (int rc = ctx->d_agent_batch.ensure(o_ts + (want_ts ? nbatch * 8 : 0) + 256)) return rc;
        uint8_t *base = ctx->d_agent_batch.as<uint8_t>();
        uint32_t *ap = reinterpret_cast<uint32_t *>(base), *src_of = reinterpret_cast<uint32_t *>(base + o_src);
        uint64_t *ts = want_ts ? reinterpret_cast<uint64_t *>(base + o_ts) : nullptr;
        CORRO_HIP_TRY(hipMemsetAsync(ap, 0xFF, dv->n * 4, s));
        hipLaunchKernelGGL(k_span_pos, dim3((uint32_t)((nbatch + SPB - 1) / SPB)), dim3(AG_T), 0, s, c.first_span, c.s_src,
                           c.s_dst, c.s_ts, nspans, nbatch, dv->ts, ap, src_of, ts);
        CORRO_HIP_TRY(hipGetLastError());
        *batch = *dv;
        ctx->agent_src_of = src_of;
        pm->on = true;
        pm->ap = ap;
        pm->src = src_of;
        pm->ts = ts;
        pm->n = nbatch;
        return CORRO_OK;
    }
    corro_changes g{};
    if (int rc = gather_dev(ctx, dv, c.s_src, c.s_dst, c.s_cnt, c.s_ts, nspans, nbatch, need_ts, ctx->d_agent_batch, g))
        return rc;
    if (!need_ts && !dv->ts) g.ts = nullptr;
    *batch = g;
    *gathered = true;
    return CORRO_OK;
}

int agent_dev_batch(corro_ctx *ctx, const corro_changes *dv, const AgentPinned &p, uint64_t ncs, uint64_t nspans,
                    uint64_t nbatch, bool need_ts, corro_changes *batch, bool *gathered, AgentPositions *pm) {
    hipStream_t s = ctx->stream;
    const DevCols c = dev_cols(ctx);
    if (nspans) {
        // off / cnt are on the device already (the screen); the rest of the changeset columns once
        if (!dv->ts) CORRO_HIP_TRY(hipMemcpyAsync(c.ts, p.ts, ncs * 8, hipMemcpyHostToDevice, s));
        CORRO_HIP_TRY(hipMemcpyAsync(c.site, p.site, ncs * 4, hipMemcpyHostToDevice, s));
        CORRO_HIP_TRY(hipMemcpyAsync(c.flag, p.flag, ncs, hipMemcpyHostToDevice, s));
        uint32_t bits = 1;
        while ((1ULL << bits) <= ctx->sites.size()) bits++;
        hipLaunchKernelGGL(k_span_keys, flat_grid(ncs), dim3(AG_T), 0, s, c.site, c.flag, ctx->d_site_rank.as<uint32_t>(),
                           ncs, (uint64_t)((1ULL << bits) - 1), c.key, c.val);
        CORRO_HIP_TRY(hipGetLastError());
        size_t tb = c.temp_bytes;
        if (int rc = ovf_sort_pairs(c.temp, &tb, c.key, c.key2, c.val, c.val2, (uint32_t)ncs, bits, s)) return rc;
        hipLaunchKernelGGL(k_span_build, flat_grid(nspans), dim3(AG_T), 0, s, c.val2, nspans, c.off, c.cnt, c.ts,
                           c.s_src, c.cnt32, c.s_ts);
        CORRO_HIP_TRY(hipGetLastError());
    }
    return spans_to_batch(ctx, dv, nspans, nbatch, need_ts, batch, gathered, pm);
}

void agent_dev_set_positions(corro_ctx *ctx, const AgentPositions *pm) {
    ctx->pm_ap = pm ? pm->ap : nullptr;
    ctx->pm_src = pm ? pm->src : nullptr;
    ctx->pm_ts = pm ? pm->ts : nullptr;
    ctx->pm_n = pm ? pm->n : 0;
}

uint8_t *agent_dev_impact_buf(corro_ctx *ctx, uint64_t n, int *rc) {
    *rc = ctx->d_agent_imp.ensure(al256(std::max<uint64_t>(n, 1)) + 256);
    return *rc ? nullptr : ctx->d_agent_imp.as<uint8_t>();
}

int agent_dev_impacts(corro_ctx *ctx, const uint8_t *impact, const uint32_t *tcid, bool tcid_by_src, uint64_t nbatch,
                      const AgentPinned &p, uint64_t ncs, uint64_t nspans, uint8_t *impactful, uint64_t nin, int mem,
                      uint32_t ntables) {
    hipStream_t s = ctx->stream;
    if (ntables > 65536) return fail(CORRO_E_RANGE, "at most 65536 tables");
    const DevCols c = dev_cols(ctx);
    // scratch: first (8 B) | committed (8 per table) | host-mode impactful (nin) | per-workgroup table counts
    // position mode with span-head flags: the streamed pass (k_imp_pos + k_span_any)
    const bool streamed = tcid_by_src && ctx->agent_src_of && !std::getenv("CORRO_IMP_SPANS");  // (env: A/B)
    const uint64_t nwg = streamed ? std::max<uint64_t>(1, std::min<uint64_t>(IP_GRID, (nbatch + AG_T * IP_U - 1) / (AG_T * IP_U)))
                                  : (nbatch + SPB - 1) / SPB;
    const size_t o_cm = 256, o_out = o_cm + 8 * 65536;
    const size_t o_part = o_out + (mem == CORRO_MEM_HOST && impactful ? al256(nin) : 0);
    const size_t o_hit = o_part + (ntables <= IMP_TLDS ? al256(nwg * ntables * 8) : 0);
    const size_t total = o_hit + (streamed ? al256(nbatch) : 0);
    if (int rc = ctx->d_agent_out.ensure(total)) return rc;
    uint8_t *base = ctx->d_agent_out.as<uint8_t>();
    unsigned long long *first = reinterpret_cast<unsigned long long *>(base);
    CORRO_HIP_TRY(hipMemsetAsync(first, 0xFF, 8, s));
    CORRO_HIP_TRY(hipMemsetAsync(base + o_cm, 0, 8ULL * std::max<uint32_t>(ntables, 1), s));
    uint8_t *out = nullptr;
    if (impactful) {
        out = mem == CORRO_MEM_HOST ? base + o_out : impactful;
        if (nin) CORRO_HIP_TRY(hipMemsetAsync(out, 0, nin, s));
    }
    if (nspans) {
        const uint32_t g1 = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>((nbatch / 16 + AG_T - 1) / AG_T, 2048));
        hipLaunchKernelGGL(k_first_imp, dim3(g1), dim3(AG_T), 0, s, impact, nbatch, first);
        CORRO_HIP_TRY(hipGetLastError());
        CORRO_HIP_TRY(hipMemsetAsync(c.any, 0, ncs, s));
        ImpArgs a{};
        a.imp = impact;
        a.tcid = tcid;
        a.s_src = c.s_src;
        a.s_dst = c.s_dst;
        a.s_cs = ctx->agent_sorted_mode ? c.val : c.val2;
        a.first_span = c.first_span;
        a.nspans = nspans;
        a.nbatch = nbatch;
        a.first = first;
        a.out = out;
        a.any = c.any;
        a.committed = reinterpret_cast<unsigned long long *>(base + o_cm);
        a.part = reinterpret_cast<unsigned long long *>(base + o_part);
        a.ntables = ntables;
        a.tcid_by_src = tcid_by_src;
        if (streamed) {
            uint8_t *hitp = base + o_hit;
            CORRO_HIP_TRY(hipMemsetAsync(hitp, 0, nbatch, s));
            hipLaunchKernelGGL(k_imp_pos, dim3((uint32_t)nwg), dim3(AG_T), 0, s, impact, ctx->agent_src_of, tcid, nbatch,
                               first, out, hitp, a.committed, a.part, ntables);
            CORRO_HIP_TRY(hipGetLastError());
            hipLaunchKernelGGL(k_span_any, flat_grid(nspans), dim3(AG_T), 0, s, hitp, c.s_dst, c.s_cnt, a.s_cs, nspans,
                               c.any);
        } else {
            hipLaunchKernelGGL(k_impactful, dim3((uint32_t)nwg), dim3(AG_T), 0, s, a);
        }
        CORRO_HIP_TRY(hipGetLastError());
        if (ntables && ntables <= IMP_TLDS) {
            hipLaunchKernelGGL(k_imp_reduce, dim3(ntables), dim3(AG_T), 0, s, a.part, nwg, ntables, a.committed);
            CORRO_HIP_TRY(hipGetLastError());
        }
        // (device-resident headers: the outcome pass reads c.any on the device)
        if (!ctx->agent_sorted_mode) CORRO_HIP_TRY(hipMemcpyAsync(p.any, c.any, ncs, hipMemcpyDeviceToHost, s));
    }
    CORRO_HIP_TRY(hipMemcpyAsync(p.committed, base + o_cm, 8ULL * ntables, hipMemcpyDeviceToHost, s));
    if (out && mem == CORRO_MEM_HOST && nin) CORRO_HIP_TRY(hipMemcpyAsync(impactful, out, nin, hipMemcpyDeviceToHost, s));
    CORRO_HIP_TRY(hipStreamSynchronize(s));
    return CORRO_OK;
}

// ---- device-resident headers ------------------------------------------------------------------
namespace {

// One changeset's header fields the decision passes read, packed (32 B: one line fetch per gather)
struct HdrPack {
    uint64_t vs, ve;     // versions(): Full v..=v, Empty its range, EmptySet the dummy 0..=0
    uint32_t site, cnt;  // site ordinal; change count of a non-empty Full (clamped to 32 bits)
    uint32_t kd;         // kind byte (KD_*)
    uint32_t pad;
};
static_assert(sizeof(HdrPack) == 32, "HdrPack is 32 B");
struct RunRec {          // a version run of decided changesets
    uint64_t start, end;
    uint32_t site, pad;
};
static_assert(sizeof(RunRec) == 24, "RunRec is 24 B");

// kind byte: bits 0-1 the CORRO_CS_* kind, bit 2 a complete Full version, bit 3 the unknown-name screen
constexpr uint32_t KD_COMPLETE = 4, KD_BAD = 8;

// Header-mode columns in d_agent_hdr (n = changesets, m = sites), per changeset i unless noted
// ([q]: per slot of order2, the (site rank, version start) sort):
//   pack HdrPack | dec u8 (decided on the device) | inrun u8 [q] | emp u8 (set_db_version(ve) at
//   commit) | rflag u32 [q] | rincl u32 [q] | runs RunRec | key2 u64 | key2' u64 | val2 u32 | val2'
//   u32 (order2) | segk u32 [q] | ver2 u64 [q] | vend2 u64 [q] | rmax u64 [q] | kd2 u8 [q] | cnt2 u32
//   [q] | ghead u32 [q] | gincl u32 [q] | gfirst u32 | glast u32 | site_max i64[m] | then, adjacent
//   (one readback): ctl u64[8] (0 err, 1 ts_any, 2 nspans, 3 nchanges, 4 max version start, 6 runs,
//   7 host changesets) | gstart u32[m] | gend u32[m]
struct HdrCols {
    HdrPack *pack;
    uint8_t *dec, *inrun, *emp;
    uint32_t *rflag, *rincl;
    RunRec *runs;
    uint64_t *key2, *key2b;
    uint32_t *val2, *val2b, *segk;
    uint64_t *ver2, *vend2, *rmax;
    uint8_t *kd2;
    uint32_t *cnt2;
    uint32_t *ghead, *gincl, *gfirst, *glast;
    int64_t *site_max;
    unsigned long long *part;  // per-workgroup partials: [0, 8192) max version start, then nspans, nchanges
    unsigned long long *ctl;
    uint32_t *gstart, *gend;
    size_t summary_bytes;  // ctl .. gend
};

HdrCols hdr_cols(corro_ctx *ctx, uint64_t ncs, uint32_t nsites, size_t *total = nullptr) {
    const uint64_t n = std::max<uint64_t>(ncs, 1), m = std::max<uint32_t>(nsites, 1);
    const size_t sz[] = {n * 32, n, n, n, n * 4, n * 4, n * 24, n * 8, n * 8, n * 4, n * 4, n * 4, n * 8, n * 8, n * 8,
                         n, n * 4, n * 4, n * 4, n * 4, n * 4, m * 8, 3 * 8192 * 8, 64, m * 4, m * 4};
    HdrCols h{};
    void **dst[] = {(void **)&h.pack,  (void **)&h.dec,   (void **)&h.inrun, (void **)&h.emp,   (void **)&h.rflag,
                    (void **)&h.rincl, (void **)&h.runs,  (void **)&h.key2,  (void **)&h.key2b, (void **)&h.val2,
                    (void **)&h.val2b, (void **)&h.segk,  (void **)&h.ver2,  (void **)&h.vend2, (void **)&h.rmax,
                    (void **)&h.kd2,   (void **)&h.cnt2,  (void **)&h.ghead, (void **)&h.gincl, (void **)&h.gfirst,
                    (void **)&h.glast, (void **)&h.site_max, (void **)&h.part, (void **)&h.ctl, (void **)&h.gstart,
                    (void **)&h.gend};
    static_assert(sizeof(sz) / sizeof(sz[0]) == sizeof(dst) / sizeof(dst[0]), "one size per column");
    uint8_t *base = ctx->d_agent_hdr.as<uint8_t>();
    size_t o = 0;
    for (size_t k = 0; k < sizeof(sz) / sizeof(sz[0]); k++) {
        if (base) *dst[k] = base + o;
        o += al256(sz[k]);
    }
    h.summary_bytes = al256(64) + 2 * al256(m * 4);
    if (total) *total = o;
    return h;
}

struct HdrArgs {
    const corro_changeset *cs;
    uint64_t ncs, nchanges;
    uint32_t nsites;
    const uint32_t *tcid;          // the input's table_cid (device)
    const uint32_t *site_rank;
    uint64_t *off, *cnt, *ts, *key;
    uint32_t *site, *val;
    uint8_t *flag, *bad, *emp, *dec;
    int32_t *known;
    unsigned long long *ctl, *part;
    HdrPack *pack;
};

// versions at or above 2^40 - 1 share one sort key (arrival order among them): never decided
constexpr uint64_t VCLAMP40 = (1ULL << 40) - 1;

// one thread per changeset: span check, unknown-name screen, the per-changeset columns, the first
// sort's key, the largest version start below 2^40 - 1 (sizes the second sort's key)
__global__ void __launch_bounds__(AG_T) k_hdr(HdrArgs a) {
    bool tsb = false;
    uint32_t err = 0;
    unsigned long long vmax = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * AG_T + threadIdx.x; i < a.ncs; i += (uint64_t)gridDim.x * AG_T) {
        const corro_changeset c = a.cs[i];
        const bool full = c.kind == CORRO_CS_FULL && c.change_count;
        bool ok = true;
        if (full && (c.change_off > a.nchanges || c.change_count > a.nchanges - c.change_off)) {
            err |= 1u;
            ok = false;
        }
        if (c.site >= a.nsites) err |= 2u;
        a.off[i] = full ? c.change_off : 0;
        a.cnt[i] = full ? c.change_count : 0;
        a.ts[i] = c.ts;
        a.site[i] = c.site;
        a.flag[i] = 0;
        a.emp[i] = 0;
        a.dec[i] = 0;
        a.known[i] = CORRO_KNOWN_SKIPPED;
        const bool comp = c.kind == CORRO_CS_FULL && c.seq_start == 0 && c.seq_end == c.last_seq;
        const bool bad = full && ok && span_has_unknown(a.tcid, c.change_off, c.change_count);
        a.bad[i] = bad ? 1 : 0;
        HdrPack pk;
        pk.vs = c.kind == CORRO_CS_EMPTY_SET ? 0 : c.version_start;
        pk.ve = c.kind == CORRO_CS_EMPTY_SET ? 0 : (c.kind == CORRO_CS_EMPTY ? c.version_end : c.version_start);
        pk.site = c.site;
        pk.cnt = full ? (uint32_t)(c.change_count < 0xFFFFFFFFULL ? c.change_count : 0xFFFFFFFFULL) : 0u;
        pk.kd = (c.kind & 3u) | (comp ? KD_COMPLETE : 0u) | (bad ? KD_BAD : 0u);
        pk.pad = 0;
        a.pack[i] = pk;
        if (pk.vs < VCLAMP40 && pk.vs > vmax) vmax = pk.vs;
        a.key[i] = c.site < a.nsites ? a.site_rank[c.site] : 0;
        a.val[i] = (uint32_t)i;
        tsb |= c.ts != 0;
    }
    __shared__ unsigned long long l_v[AG_T / 64];
    const unsigned long long anyts = __ballot(tsb);
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        err |= __shfl_xor(err, d);
        const unsigned long long y = __shfl_xor(vmax, d);
        vmax = y > vmax ? y : vmax;
    }
    if ((threadIdx.x & 63) == 0) {
        if (err) atomicOr(&a.ctl[0], (unsigned long long)err);  // (rare: a malformed call)
        if (anyts) a.ctl[1] = 1;                                // (a plain store of 1)
        l_v[threadIdx.x >> 6] = vmax;
    }
    __syncthreads();
    if (threadIdx.x == 0) {  // one partial per workgroup (no same-address atomics), k_hdr_reduce folds them
        unsigned long long m = 0;
        for (int k = 0; k < AG_T / 64; k++) m = l_v[k] > m ? l_v[k] : m;
        a.part[blockIdx.x] = m;
    }
}

// fold per-workgroup partials: ctl[4] = max of part[0, nb); with sums, ctl[2] += sum part[8192 + ..],
// ctl[3] += sum part[16384 + ..]
__global__ void __launch_bounds__(1024) k_hdr_reduce(const unsigned long long *__restrict__ part, uint32_t nb, int sums,
                                                      unsigned long long *__restrict__ ctl) {
    __shared__ unsigned long long l[3][1024 / 64];
    unsigned long long m = 0, x = 0, y = 0;
    for (uint32_t b = threadIdx.x; b < nb; b += 1024) {
        if (sums) {
            x += part[8192 + b];
            y += part[16384 + b];
        } else {
            m = part[b] > m ? part[b] : m;
        }
    }
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        const unsigned long long q = __shfl_xor(m, d);
        m = q > m ? q : m;
        x += __shfl_xor(x, d);
        y += __shfl_xor(y, d);
    }
    if ((threadIdx.x & 63) == 0) {
        l[0][threadIdx.x >> 6] = m;
        l[1][threadIdx.x >> 6] = x;
        l[2][threadIdx.x >> 6] = y;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int k = 1; k < 1024 / 64; k++) {
            m = l[0][k] > l[0][0] ? l[0][k] : l[0][0];
            l[0][0] = m;
            l[1][0] += l[1][k];
            l[2][0] += l[2][k];
        }
        if (sums) {
            ctl[2] += l[1][0];
            ctl[3] += l[2][0];
        } else {
            ctl[4] = l[0][0];
        }
    }
}

// the second sort's key: site rank << vbits | version start (clamped at vclamp = 2^vbits - 1)
__global__ void __launch_bounds__(AG_T) k_hdr_key2(uint64_t ncs, const HdrPack *__restrict__ pack,
                                                    const uint32_t *__restrict__ site_rank, uint32_t nsites,
                                                    uint32_t vbits, uint64_t *__restrict__ key2, uint32_t *__restrict__ val2) {
    const uint64_t vclamp = (1ULL << vbits) - 1;
    for (uint64_t i = (uint64_t)blockIdx.x * AG_T + threadIdx.x; i < ncs; i += (uint64_t)gridDim.x * AG_T) {
        const HdrPack pk = pack[i];
        const uint64_t rank = pk.site < nsites ? site_rank[pk.site] : 0;
        key2[i] = rank << vbits | (pk.vs < vclamp ? pk.vs : vclamp);
        val2[i] = (uint32_t)i;
    }
}

// per sorted slot (order: site rank, arrival): each actor's slots [gstart, gend]
__global__ void __launch_bounds__(AG_T) k_hdr_sites(const uint32_t *__restrict__ order, uint64_t ncs,
                                                     const uint32_t *__restrict__ site, uint32_t *__restrict__ gstart,
                                                     uint32_t *__restrict__ gend) {
    for (uint64_t j = (uint64_t)blockIdx.x * AG_T + threadIdx.x; j < ncs; j += (uint64_t)gridDim.x * AG_T) {
        const uint32_t st = site[order[j]];
        if (j == 0 || site[order[j - 1]] != st) gstart[st] = (uint32_t)j;
        if (j + 1 == ncs || site[order[j + 1]] != st) gend[st] = (uint32_t)j;
    }
}

// ---- per-changeset decisions (order2: site rank, version start, arrival) ------------------------
// A changeset is decided on the device when nothing else of its actor in the call touches its
// versions and they are all above the actor's booked max: then util.rs:704-884 treats it on its
// own -- contains_all is false (no version above max is known), no earlier changeset of the actor
// has seen a version of it -- so a complete Full version merges (or rolls back on an unknown name),
// an empty one or an Empty range clears (crsql_set_db_version of its end, :810-824). Changesets with
// the same dedup key (actor, versions, seqs: util.rs:711) form one group: the first to arrive is the
// one processed, the rest are skipped by pass 1's seen set. versions() == 0..=0 (EmptySet, and any
// changeset of version 0) is always contained (agent.rs:1353-1361): skipped. Everything else -- an
// overlap, an incomplete (partial) version, a version at or below the max -- is walked by the host
// with the reference's per-actor code, and never touches the versions of a decided changeset.
__device__ inline bool same_key(const corro_changeset *cs, const HdrPack &x, const HdrPack &y, uint32_t a, uint32_t b) {
    if (x.vs != y.vs || x.ve != y.ve) return false;
    const bool sa = (x.kd & 3u) == CORRO_CS_FULL, sb = (y.kd & 3u) == CORRO_CS_FULL;  // seqs: Full only
    if (sa != sb) return false;
    return !sa || (cs[a].seq_start == cs[b].seq_start && cs[a].seq_end == cs[b].seq_end);
}

// the slot-ordered copies the decision reads (one 32-B gather per slot) and the dedup-group heads
__global__ void __launch_bounds__(AG_T) k_iso_prep(const corro_changeset *__restrict__ cs, const uint32_t *__restrict__ order2,
                                                    uint64_t n, const HdrPack *__restrict__ pack, uint32_t *__restrict__ segk,
                                                    uint64_t *__restrict__ ver2, uint64_t *__restrict__ vend2,
                                                    uint8_t *__restrict__ kd2, uint32_t *__restrict__ cnt2,
                                                    uint32_t *__restrict__ ghead) {
    for (uint64_t q = (uint64_t)blockIdx.x * AG_T + threadIdx.x; q < n; q += (uint64_t)gridDim.x * AG_T) {
        const uint32_t i = order2[q];
        const HdrPack x = pack[i];
        segk[q] = x.site;
        ver2[q] = x.vs;
        vend2[q] = x.ve;
        kd2[q] = (uint8_t)x.kd;
        cnt2[q] = x.cnt;
        bool head = q == 0;
        if (!head) {
            const uint32_t p = order2[q - 1];
            const HdrPack y = pack[p];
            head = y.site != x.site || !same_key(cs, y, x, p, i);
        }
        ghead[q] = head ? 1u : 0u;
    }
}

__global__ void __launch_bounds__(AG_T) k_iso_groups(uint64_t n, const uint32_t *__restrict__ ghead,
                                                      const uint32_t *__restrict__ gincl, uint32_t *__restrict__ gfirst,
                                                      uint32_t *__restrict__ glast) {
    for (uint64_t q = (uint64_t)blockIdx.x * AG_T + threadIdx.x; q < n; q += (uint64_t)gridDim.x * AG_T) {
        const uint32_t g = gincl[q] - 1;
        if (ghead[q]) gfirst[g] = (uint32_t)q;
        if (q + 1 == n || ghead[q + 1]) glast[g] = (uint32_t)q;
    }
}

struct IsoArgs {
    const uint32_t *order2, *segk, *gincl, *gfirst, *glast, *cnt2;
    const uint64_t *ver2, *vend2, *rmax;
    const uint8_t *kd2;
    const int64_t *site_max;
    uint8_t *dec, *flag, *emp, *inrun;
    int32_t *known;
    unsigned long long *part;
    uint64_t n, vclamp;
};

__global__ void __launch_bounds__(AG_T) k_iso_decide(IsoArgs a) {
    __shared__ unsigned long long l_sp[AG_T / 64], l_ch[AG_T / 64];
    unsigned long long nsp = 0, nch = 0;
    for (uint64_t q = (uint64_t)blockIdx.x * AG_T + threadIdx.x; q < a.n; q += (uint64_t)gridDim.x * AG_T) {
        const uint32_t i = a.order2[q];
        const uint64_t vs_q = a.ver2[q], ve_q = a.vend2[q];
        uint8_t in = 0;
        if (vs_q == 0 && ve_q == 0) {
            a.dec[i] = 1;  // versions() == 0..=0: always contained (pass 1 skips it)
        } else if (vs_q != 0 && vs_q <= ve_q && vs_q < a.vclamp) {
            const uint32_t g = a.gincl[q] - 1, f = a.gfirst[g], l = a.glast[g];
            const uint64_t vs = a.ver2[f], ve = a.vend2[f];
            const bool prev_ov = f > 0 && a.segk[f - 1] == a.segk[f] && a.rmax[f - 1] >= vs;
            bool next_ov = false;
            if (l + 1 < a.n && a.segk[l + 1] == a.segk[l]) {
                const uint64_t nv = a.ver2[l + 1];
                next_ov = nv <= ve || (nv >= a.vclamp && ve >= a.vclamp);
            }
            const int64_t mx = a.site_max[a.segk[q]];
            const uint32_t kd = a.kd2[f], kind = kd & 3u;
            const bool decidable = !prev_ov && !next_ov && (mx < 0 || vs > (uint64_t)mx) &&
                                   (kind == CORRO_CS_EMPTY || (kind == CORRO_CS_FULL && (kd & KD_COMPLETE)));
            if (decidable && q != f) {
                a.dec[i] = 1;  // a later copy of the group's key: pass 1's seen set skips it
            } else if (decidable) {
                a.dec[i] = 1;
                if (kind == CORRO_CS_EMPTY || a.cnt2[q] == 0) {  // process_empty_version (above the max)
                    a.known[i] = CORRO_KNOWN_CLEARED;
                    a.emp[i] = 1;
                    in = 1;
                } else if (kd & KD_BAD) {  // the version's SAVEPOINT rolls back alone (util.rs:839-860)
                    a.known[i] = CORRO_E_UNKNOWN_COLUMN;
                } else {
                    a.flag[i] = 1;
                    a.known[i] = CORRO_KNOWN_CURRENT;  // final value decided after the merge
                    in = 1;
                    nsp++;
                    nch += a.cnt2[q];
                }
            }
        }  // (else: a range from version 0, an inverted or clamped range -- the host walks it)
        a.inrun[q] = in;
    }
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        nsp += __shfl_xor(nsp, d);
        nch += __shfl_xor(nch, d);
    }
    if ((threadIdx.x & 63) == 0) {
        l_sp[threadIdx.x >> 6] = nsp;
        l_ch[threadIdx.x >> 6] = nch;
    }
    __syncthreads();
    if (threadIdx.x == 0) {  // one partial per workgroup (k_hdr_reduce)
        unsigned long long x = 0, y = 0;
        for (int k = 0; k < AG_T / 64; k++) {
            x += l_sp[k];
            y += l_ch[k];
        }
        a.part[8192 + blockIdx.x] = x;
        a.part[16384 + blockIdx.x] = y;
    }
}

// version runs of the decided (merged or cleared) changesets, in order2: a slot starts a run unless
// the previous slot is in a run of the same actor ending right before it
__global__ void __launch_bounds__(AG_T) k_hdr_runflag(uint64_t n, const uint32_t *__restrict__ segk,
                                                       const uint64_t *__restrict__ ver2, const uint64_t *__restrict__ vend2,
                                                       const uint8_t *__restrict__ inrun, uint32_t *__restrict__ rflag) {
    for (uint64_t q = (uint64_t)blockIdx.x * AG_T + threadIdx.x; q < n; q += (uint64_t)gridDim.x * AG_T) {
        const bool cont = q > 0 && inrun[q - 1] && segk[q - 1] == segk[q] && vend2[q - 1] + 1 == ver2[q];
        rflag[q] = inrun[q] && !cont ? 1u : 0u;
    }
}

__global__ void __launch_bounds__(AG_T) k_hdr_runs(uint64_t n, const uint32_t *__restrict__ segk,
                                                    const uint64_t *__restrict__ ver2, const uint64_t *__restrict__ vend2,
                                                    const uint8_t *__restrict__ inrun, const uint32_t *__restrict__ rflag,
                                                    const uint32_t *__restrict__ rincl, RunRec *__restrict__ runs) {
    for (uint64_t q = (uint64_t)blockIdx.x * AG_T + threadIdx.x; q < n; q += (uint64_t)gridDim.x * AG_T) {
        if (!inrun[q]) continue;
        const uint32_t r = rincl[q] - 1;
        if (rflag[q]) {
            runs[r].site = segk[q];
            runs[r].start = ver2[q];
        }
        const bool ends = q + 1 >= n || !inrun[q + 1] || rflag[q + 1];
        if (ends) runs[r].end = vend2[q];
    }
}

// the host's changesets (dec 0) among the sorted slots (order: site rank, arrival): flags for the scan
__global__ void __launch_bounds__(AG_T) k_hdr_hmark(const uint32_t *__restrict__ order, uint64_t n,
                                                     const uint8_t *__restrict__ dec, uint32_t *__restrict__ hm) {
    for (uint64_t j = (uint64_t)blockIdx.x * AG_T + threadIdx.x; j < n; j += (uint64_t)gridDim.x * AG_T)
        hm[j] = dec[order[j]] ? 0u : 1u;
}

__global__ void __launch_bounds__(AG_T) k_hdr_hlist(uint64_t n, const uint32_t *__restrict__ hm,
                                                     const uint32_t *__restrict__ hincl, uint32_t *__restrict__ hslot) {
    for (uint64_t j = (uint64_t)blockIdx.x * AG_T + threadIdx.x; j < n; j += (uint64_t)gridDim.x * AG_T)
        if (hm[j]) hslot[hincl[j] - 1] = (uint32_t)j;
}

// run and host-changeset counts into ctl[6], ctl[7] (read back with the summary)
__global__ void k_hdr_counts(uint64_t n, const uint32_t *__restrict__ rincl, const uint32_t *__restrict__ hincl,
                             unsigned long long *__restrict__ ctl) {
    if (threadIdx.x == 0) {
        ctl[6] = rincl ? rincl[n - 1] : 0u;
        ctl[7] = hincl[n - 1];
    }
}

// the host's changesets: header, arrival index, unknown-name flag, and whether a partial one is
// canonical (bufpool.hip: its k-th change has seq = seq_start + k, its own site and version, no long
// value -- its rows then stay in HBM)
struct HGatherArgs {
    const corro_changeset *cs;
    const uint32_t *order, *slot;
    const uint8_t *bad;
    corro_changes in;
    uint64_t n;
    corro_changeset *out;
    uint32_t *idx;
    uint8_t *obad, *ocanon;
    uint32_t *otab;  // a canonical one's table index when all its changes share it, else HDR_TAB_MIXED
};

// one wave per changeset: lane 0 copies the header, the lanes check its changes 64 at a time (the
// canonical test reads five fields of every change: a lane-serial loop of them was a chain of
// dependent latencies per changeset)
__global__ void __launch_bounds__(AG_T) k_hdr_gather(HGatherArgs a) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t w0 = ((uint64_t)blockIdx.x * AG_T + threadIdx.x) >> 6, nw = (uint64_t)gridDim.x * (AG_T / 64);
    for (uint64_t k = w0; k < a.n; k += nw) {  // (wave-uniform)
        const uint32_t i = a.order[a.slot[k]];
        const corro_changeset c = a.cs[i];
        bool canon = c.kind == CORRO_CS_FULL && c.change_count && !(c.seq_start == 0 && c.seq_end == c.last_seq) &&
                     !a.bad[i] && c.seq_start <= c.seq_end && c.seq_end < 0xFFFFFFFFULL &&
                     c.change_count == c.seq_end - c.seq_start + 1 && c.version_start <= (uint64_t)INT64_MAX &&
                     c.change_off <= a.in.n && c.change_count <= a.in.n - c.change_off && a.in.seq && a.in.site &&
                     a.in.db_version;
        uint32_t tab = HDR_TAB_MIXED;
        if (canon && a.in.table_cid) tab = a.in.table_cid[c.change_off] >> 16;
        for (uint64_t q0 = 0; canon && q0 < c.change_count; q0 += 64) {  // (canon is wave-uniform)
            const uint64_t q = q0 + lane;
            bool ok = true;
            if (q < c.change_count) {
                const uint64_t r = c.change_off + q;
                const uint8_t vt = a.in.val_type ? a.in.val_type[r] : (uint8_t)CORRO_INTEGER;
                const uint8_t vl = a.in.val_len ? a.in.val_len[r] : 0;
                ok = a.in.seq[r] == c.seq_start + q && a.in.site[r] == c.site &&
                     (uint64_t)a.in.db_version[r] == c.version_start &&
                     !(vl == CORRO_VAL_LONG && (vt == CORRO_TEXT || vt == CORRO_BLOB));
                if (tab != HDR_TAB_MIXED && a.in.table_cid && (a.in.table_cid[r] >> 16) != tab) tab = HDR_TAB_MIXED;
            }
            canon = __all(ok);
            if (!__all(tab != HDR_TAB_MIXED)) tab = HDR_TAB_MIXED;
        }
        if (lane == 0) {
            a.out[k] = c;
            a.idx[k] = i;
            a.obad[k] = a.bad[i];
            a.ocanon[k] = canon ? 1 : 0;
            a.otab[k] = canon ? tab : HDR_TAB_MIXED;
        }
    }
}

__global__ void __launch_bounds__(AG_T) k_hdr_put(const uint32_t *__restrict__ idx, const uint8_t *__restrict__ f,
                                                   const int32_t *__restrict__ kn, uint64_t n, uint8_t *__restrict__ flag,
                                                   int32_t *__restrict__ known) {
    for (uint64_t k = (uint64_t)blockIdx.x * AG_T + threadIdx.x; k < n; k += (uint64_t)gridDim.x * AG_T) {
        flag[idx[k]] = f[k];
        known[idx[k]] = kn[k];
    }
}

// applied spans in sorted order: slot j's changeset when flagged -> span rincl[j] - 1
__global__ void __launch_bounds__(AG_T) k_hdr_flagged(const uint32_t *__restrict__ order, uint64_t ncs,
                                                       const uint8_t *__restrict__ flag, uint32_t *__restrict__ fl) {
    for (uint64_t j = (uint64_t)blockIdx.x * AG_T + threadIdx.x; j < ncs; j += (uint64_t)gridDim.x * AG_T)
        fl[j] = flag[order[j]];
}

__global__ void __launch_bounds__(AG_T) k_hdr_spans(const uint32_t *__restrict__ order, uint64_t ncs,
                                                     const uint8_t *__restrict__ flag, const uint32_t *__restrict__ incl,
                                                     const uint64_t *__restrict__ off, const uint64_t *__restrict__ cnt,
                                                     const uint64_t *__restrict__ ts, uint64_t *__restrict__ s_src,
                                                     uint32_t *__restrict__ cnt32, uint64_t *__restrict__ s_ts,
                                                     uint32_t *__restrict__ s_cs) {
    for (uint64_t j = (uint64_t)blockIdx.x * AG_T + threadIdx.x; j < ncs; j += (uint64_t)gridDim.x * AG_T) {
        const uint32_t i = order[j];
        if (!flag[i]) continue;
        const uint32_t k = incl[j] - 1;
        s_src[k] = off[i];
        cnt32[k] = (uint32_t)cnt[i];
        s_ts[k] = ts[i];
        s_cs[k] = i;
    }
}

// commit: known of flagged changesets, crsql_set_db_version of the decided empty versions / ranges
__global__ void __launch_bounds__(AG_T) k_hdr_commit(uint64_t ncs, const uint8_t *__restrict__ flag,
                                                      const uint8_t *__restrict__ any, const uint8_t *__restrict__ emp,
                                                      const HdrPack *__restrict__ pack, int32_t *__restrict__ known,
                                                      unsigned long long *__restrict__ dbv) {
    for (uint64_t i = (uint64_t)blockIdx.x * AG_T + threadIdx.x; i < ncs; i += (uint64_t)gridDim.x * AG_T) {
        if (flag[i]) known[i] = any[i] ? CORRO_KNOWN_CURRENT : CORRO_KNOWN_CLEARED;
        if (emp[i]) {
            const HdrPack pk = pack[i];
            atomicMax(&dbv[pk.site], (unsigned long long)(pk.ve + 1));
        }
    }
}

// flagged changeset i whose site << 40 | version is among the sorted keys -> hit list
__global__ void __launch_bounds__(AG_T) k_hdr_clearprobe(uint64_t ncs, const uint8_t *__restrict__ flag,
                                                          const HdrPack *__restrict__ pack, const uint64_t *__restrict__ keys,
                                                          uint64_t nk, uint64_t *__restrict__ hit,
                                                          unsigned long long *__restrict__ nhit) {
    for (uint64_t i = (uint64_t)blockIdx.x * AG_T + threadIdx.x; i < ncs; i += (uint64_t)gridDim.x * AG_T) {
        if (!flag[i]) continue;
        const HdrPack pk = pack[i];
        if (pk.vs >= (1ULL << 40)) continue;
        const uint64_t k = (uint64_t)pk.site << 40 | pk.vs;
        uint64_t lo = 0, hi = nk;  // first key >= k
        while (lo < hi) {
            const uint64_t m = (lo + hi) >> 1;
            if (keys[m] < k) lo = m + 1;
            else hi = m;
        }
        if (lo < nk && keys[lo] == k) hit[atomicAdd(nhit, 1ULL)] = k;
    }
}

}  // namespace

int agent_dev_headers(corro_ctx *ctx, const corro_changeset *dcs, uint64_t ncs, const corro_changes *dv,
                      const std::vector<int64_t> &site_max, int32_t *dknown, DevHdrResult &res) {
    hipStream_t s = ctx->stream;
    const uint32_t nsites = (uint32_t)ctx->sites.size();
    // CORRO_AGENT_PROFILE: host-visible phase times of this pass on stderr
    static const bool prof = std::getenv("CORRO_AGENT_PROFILE") != nullptr;
    const auto t0 = std::chrono::steady_clock::now();
    auto ms = [&]() { return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count(); };
    double t_launch = 0, t_ctl0 = 0, t_sum = 0;
    res = DevHdrResult{};
    res.sites.assign(nsites, DevHdrSite{0xFFFFFFFFu, 0xFFFFFFFFu});
    ctx->agent_sorted_mode = true;
    if (!ncs) return CORRO_OK;
    size_t total = 0;
    (void)hdr_cols(ctx, ncs, nsites, &total);
    if (int rc = ctx->d_agent_hdr.ensure(total + 256)) return rc;
    const HdrCols h = hdr_cols(ctx, ncs, nsites);
    const DevCols c = dev_cols(ctx);
    CORRO_HIP_TRY(hipMemsetAsync(h.ctl, 0, 64, s));
    CORRO_HIP_TRY(hipMemsetAsync(h.gstart, 0xFF, 4ULL * std::max<uint32_t>(nsites, 1), s));
    if (nsites) CORRO_HIP_TRY(hipMemcpyAsync(h.site_max, site_max.data(), 8ULL * nsites, hipMemcpyHostToDevice, s));
    HdrArgs a{};
    a.cs = dcs;
    a.ncs = ncs;
    a.nchanges = dv ? dv->n : 0;
    a.nsites = nsites;
    a.tcid = dv ? dv->table_cid : nullptr;
    a.site_rank = ctx->d_site_rank.as<uint32_t>();
    a.off = c.off;
    a.cnt = c.cnt;
    a.ts = c.ts;
    a.key = c.key;
    a.site = c.site;
    a.val = c.val;
    a.flag = c.flag;
    a.bad = c.bad;
    a.emp = h.emp;
    a.dec = h.dec;
    a.known = dknown;
    a.ctl = h.ctl;
    a.part = h.part;
    a.pack = h.pack;
    t_launch = ms();
    hipLaunchKernelGGL(k_hdr, flat_grid(ncs), dim3(AG_T), 0, s, a);
    CORRO_HIP_TRY(hipGetLastError());
    hipLaunchKernelGGL(k_hdr_reduce, dim3(1), dim3(1024), 0, s, h.part, flat_grid(ncs).x, 0, h.ctl);
    CORRO_HIP_TRY(hipGetLastError());
    unsigned long long ctl0[5] = {0, 0, 0, 0, 0};
    CORRO_HIP_TRY(hipMemcpyAsync(ctl0, h.ctl, sizeof(ctl0), hipMemcpyDeviceToHost, s));
    CORRO_HIP_TRY(hipStreamSynchronize(s));
    t_ctl0 = ms();
    if (ctl0[0]) {  // nothing decided: every changeset stays Skipped
        res.err = (uint32_t)ctl0[0];
        return CORRO_OK;
    }
    uint32_t bits = 1;
    while ((1ULL << bits) <= nsites) bits++;
    // the second sort's version field: wide enough that only versions >= 2^40 - 1 reach its clamp
    uint32_t vbits = 1;
    while (vbits < 40 && (1ULL << vbits) - 1 <= ctl0[4]) vbits++;
    const uint32_t n32 = (uint32_t)ncs;
    // the application order (site rank, arrival) and each actor's slots in it
    size_t tb = c.temp_bytes;
    if (int rc = ovf_sort_pairs(c.temp, &tb, c.key, c.key2, c.val, c.val2, n32, bits, s)) return rc;
    const uint32_t *order = c.val2;
    hipLaunchKernelGGL(k_hdr_sites, flat_grid(ncs), dim3(AG_T), 0, s, order, ncs, c.site, h.gstart, h.gend);
    CORRO_HIP_TRY(hipGetLastError());
    // per-changeset decisions over (site rank, version start, arrival): dedup groups, the running max
    // of version ends per actor (overlaps), then the decided changesets' version runs
    const bool decide = bits + vbits <= 64;  // (else the host walks every changeset)
    if (decide) {
        hipLaunchKernelGGL(k_hdr_key2, flat_grid(ncs), dim3(AG_T), 0, s, ncs, h.pack, a.site_rank, nsites, vbits, h.key2,
                           h.val2);
        CORRO_HIP_TRY(hipGetLastError());
        tb = c.temp_bytes;
        if (int rc = ovf_sort_pairs(c.temp, &tb, h.key2, h.key2b, h.val2, h.val2b, n32, bits + vbits, s)) return rc;
        const uint32_t *order2 = h.val2b;
        hipLaunchKernelGGL(k_iso_prep, flat_grid(ncs), dim3(AG_T), 0, s, dcs, order2, ncs, h.pack, h.segk, h.ver2, h.vend2,
                           h.kd2, h.cnt2, h.ghead);
        CORRO_HIP_TRY(hipGetLastError());
        tb = c.temp_bytes;
        if (int rc = prim_inclusive_scan_u32(c.temp, &tb, h.ghead, h.gincl, n32, s)) return rc;
        hipLaunchKernelGGL(k_iso_groups, flat_grid(ncs), dim3(AG_T), 0, s, ncs, h.ghead, h.gincl, h.gfirst, h.glast);
        CORRO_HIP_TRY(hipGetLastError());
        tb = c.temp_bytes;
        if (int rc = prim_segmax_scan_u64(c.temp, &tb, h.segk, h.vend2, h.rmax, n32, s)) return rc;
        IsoArgs d{};
        d.order2 = order2;
        d.segk = h.segk;
        d.gincl = h.gincl;
        d.gfirst = h.gfirst;
        d.glast = h.glast;
        d.cnt2 = h.cnt2;
        d.ver2 = h.ver2;
        d.vend2 = h.vend2;
        d.rmax = h.rmax;
        d.kd2 = h.kd2;
        d.site_max = h.site_max;
        d.dec = h.dec;
        d.flag = c.flag;
        d.emp = h.emp;
        d.inrun = h.inrun;
        d.known = dknown;
        d.part = h.part;
        d.n = ncs;
        d.vclamp = vbits >= 40 ? VCLAMP40 : (1ULL << vbits) - 1;
        hipLaunchKernelGGL(k_iso_decide, flat_grid(ncs), dim3(AG_T), 0, s, d);
        CORRO_HIP_TRY(hipGetLastError());
        hipLaunchKernelGGL(k_hdr_reduce, dim3(1), dim3(1024), 0, s, h.part, flat_grid(ncs).x, 1, h.ctl);
        CORRO_HIP_TRY(hipGetLastError());
        hipLaunchKernelGGL(k_hdr_runflag, flat_grid(ncs), dim3(AG_T), 0, s, ncs, h.segk, h.ver2, h.vend2, h.inrun, h.rflag);
        CORRO_HIP_TRY(hipGetLastError());
        tb = c.temp_bytes;
        if (int rc = prim_inclusive_scan_u32(c.temp, &tb, h.rflag, h.rincl, n32, s)) return rc;
        hipLaunchKernelGGL(k_hdr_runs, flat_grid(ncs), dim3(AG_T), 0, s, ncs, h.segk, h.ver2, h.vend2, h.inrun, h.rflag,
                           h.rincl, h.runs);
        CORRO_HIP_TRY(hipGetLastError());
    }
    // the host's changesets: their sorted slots (grouped by actor, arrival order inside)
    hipLaunchKernelGGL(k_hdr_hmark, flat_grid(ncs), dim3(AG_T), 0, s, order, ncs, h.dec, c.cnt32);
    CORRO_HIP_TRY(hipGetLastError());
    tb = c.temp_bytes;
    if (int rc = prim_inclusive_scan_u32(c.temp, &tb, c.cnt32, c.incl, n32, s)) return rc;
    uint32_t *hslot = h.gfirst;  // (free once the decisions are made)
    hipLaunchKernelGGL(k_hdr_hlist, flat_grid(ncs), dim3(AG_T), 0, s, ncs, c.cnt32, c.incl, hslot);
    CORRO_HIP_TRY(hipGetLastError());
    hipLaunchKernelGGL(k_hdr_counts, dim3(1), dim3(64), 0, s, ncs, decide ? h.rincl : nullptr, c.incl, h.ctl);
    CORRO_HIP_TRY(hipGetLastError());
    // one readback: counters, run count, host changeset count, per-site groups
    std::vector<uint8_t> sum(h.summary_bytes);
    CORRO_HIP_TRY(hipMemcpyAsync(sum.data(), h.ctl, h.summary_bytes, hipMemcpyDeviceToHost, s));
    CORRO_HIP_TRY(hipStreamSynchronize(s));
    t_sum = ms();
    const unsigned long long *ctl = reinterpret_cast<const unsigned long long *>(sum.data());
    const uint32_t *gs = reinterpret_cast<const uint32_t *>(sum.data() + al256(64));
    const uint32_t *ge = reinterpret_cast<const uint32_t *>(sum.data() + al256(64) + al256(std::max<uint32_t>(nsites, 1) * 4ULL));
    res.ts_any = ctl[1] != 0;
    res.nspans = ctl[2];
    res.nchanges = ctl[3];
    const uint64_t nruns = ctl[6], nh = ctl[7];
    for (uint32_t t = 0; t < nsites; t++) res.sites[t] = DevHdrSite{gs[t], ge[t]};
    res.run_site.resize(nruns);
    res.run_start.resize(nruns);
    res.run_end.resize(nruns);
    res.nh = nh;
    // one pinned readback area for the version runs and (when there are host changesets) their headers,
    // arrival index, unknown-name and canonical flags; one wait for both copies (a pageable copy of the
    // runs blocked on its own)
    size_t o_idx = 0, o_bad = 0, o_can = 0, o_tab = 0, total_b = 0;
    if (nh) {
        o_idx = al256((uint64_t)nh * sizeof(corro_changeset));
        o_bad = o_idx + al256(nh * 4ULL);
        o_can = o_bad + al256(nh);
        o_tab = o_can + al256(nh);
        total_b = o_tab + al256(nh * 4ULL);
    }
    const size_t o_runs = total_b, pin_b = o_runs + al256(nruns * sizeof(RunRec));
    if (pin_b > ctx->h_hfetch_bytes) {
        if (ctx->h_hfetch) (void)hipHostFree(ctx->h_hfetch);
        ctx->h_hfetch = nullptr;
        ctx->h_hfetch_bytes = 0;
        CORRO_HIP_TRY(hipHostMalloc(&ctx->h_hfetch, pin_b + pin_b / 4, hipHostMallocDefault));
        ctx->h_hfetch_bytes = pin_b + pin_b / 4;
    }
    uint8_t *hp = static_cast<uint8_t *>(ctx->h_hfetch);
    if (nruns) CORRO_HIP_TRY(hipMemcpyAsync(hp + o_runs, h.runs, nruns * sizeof(RunRec), hipMemcpyDeviceToHost, s));
    if (nh) {
        if (int rc = ctx->d_agent_fetch.ensure(total_b + 256)) return rc;
        uint8_t *base = ctx->d_agent_fetch.as<uint8_t>();
        HGatherArgs g{};
        g.cs = dcs;
        g.order = order;
        g.slot = hslot;
        g.bad = c.bad;
        if (dv) g.in = *dv;
        g.n = nh;
        g.out = reinterpret_cast<corro_changeset *>(base);
        g.idx = reinterpret_cast<uint32_t *>(base + o_idx);
        g.obad = base + o_bad;
        g.ocanon = base + o_can;
        g.otab = reinterpret_cast<uint32_t *>(base + o_tab);
        hipLaunchKernelGGL(k_hdr_gather, wave_grid(nh), dim3(AG_T), 0, s, g);
        CORRO_HIP_TRY(hipGetLastError());
        CORRO_HIP_TRY(hipMemcpyAsync(hp, base, total_b, hipMemcpyDeviceToHost, s));
        res.hcs = reinterpret_cast<const corro_changeset *>(hp);
        res.hidx = reinterpret_cast<const uint32_t *>(hp + o_idx);
        res.hbad = hp + o_bad;
        res.hcanon = hp + o_can;
        res.hctab = reinterpret_cast<const uint32_t *>(hp + o_tab);
    }
    const RunRec *runs = reinterpret_cast<const RunRec *>(hp + o_runs);
    if (nruns || nh) CORRO_HIP_TRY(hipStreamSynchronize(s));
    for (uint64_t r = 0; r < nruns; r++) {
        res.run_site[r] = runs[r].site;
        res.run_start[r] = runs[r].start;
        res.run_end[r] = runs[r].end;
    }
    if (prof)
        fprintf(stderr, "[corro agent dev headers] setup=%.3f k_hdr+sync=%.3f passes+sync=%.3f fetch=%.3f ms\n", t_launch,
                t_ctl0 - t_launch, t_sum - t_ctl0, ms() - t_sum);
    return CORRO_OK;
}

int agent_dev_put_host(corro_ctx *ctx, const uint32_t *idx, uint64_t n, const std::vector<uint8_t> &flag,
                       const std::vector<int32_t> &known, int32_t *dknown) {
    if (!n) return CORRO_OK;
    hipStream_t s = ctx->stream;
    const size_t o_f = al256(n * 4), o_k = o_f + al256(n);
    if (int rc = ctx->d_agent_aux2.ensure(o_k + al256(n * 4))) return rc;
    uint8_t *base = ctx->d_agent_aux2.as<uint8_t>();
    CORRO_HIP_TRY(hipMemcpyAsync(base, idx, n * 4, hipMemcpyHostToDevice, s));
    CORRO_HIP_TRY(hipMemcpyAsync(base + o_f, flag.data(), n, hipMemcpyHostToDevice, s));
    CORRO_HIP_TRY(hipMemcpyAsync(base + o_k, known.data(), n * 4, hipMemcpyHostToDevice, s));
    const DevCols c = dev_cols(ctx);
    hipLaunchKernelGGL(k_hdr_put, flat_grid(n), dim3(AG_T), 0, s, reinterpret_cast<const uint32_t *>(base), base + o_f,
                       reinterpret_cast<const int32_t *>(base + o_k), n, c.flag, dknown);
    CORRO_HIP_TRY(hipGetLastError());
    CORRO_HIP_TRY(hipStreamSynchronize(s));  // (host sources)
    return CORRO_OK;
}

int agent_dev_batch_sorted(corro_ctx *ctx, const corro_changes *dv, uint64_t ncs, uint64_t nspans, uint64_t nbatch,
                           bool need_ts, corro_changes *batch, bool *gathered, AgentPositions *pm) {
    CORRO_HIP_TRY(hipSetDevice(ctx->device));  // (callable from a second host thread)
    hipStream_t s = ctx->stream;
    const DevCols c = dev_cols(ctx);
    if (nspans) {
        hipLaunchKernelGGL(k_hdr_flagged, flat_grid(ncs), dim3(AG_T), 0, s, c.val2, ncs, c.flag, c.cnt32);
        CORRO_HIP_TRY(hipGetLastError());
        size_t tb = c.temp_bytes;
        if (int rc = prim_inclusive_scan_u32(c.temp, &tb, c.cnt32, c.incl, (uint32_t)ncs, s)) return rc;
        hipLaunchKernelGGL(k_hdr_spans, flat_grid(ncs), dim3(AG_T), 0, s, c.val2, ncs, c.flag, c.incl, c.off, c.cnt, c.ts,
                           c.s_src, c.cnt32, c.s_ts, c.val);
        CORRO_HIP_TRY(hipGetLastError());
    }
    return spans_to_batch(ctx, dv, nspans, nbatch, need_ts, batch, gathered, pm);
}

int agent_dev_commit_headers(corro_ctx *ctx, uint64_t ncs, int32_t *dknown, const std::vector<uint64_t> *keys,
                             std::vector<std::pair<uint32_t, uint64_t>> *hits) {
    if (hits) hits->clear();
    if (!ncs) return CORRO_OK;
    hipStream_t s = ctx->stream;
    const HdrCols h = hdr_cols(ctx, ncs, (uint32_t)ctx->sites.size());
    const DevCols c = dev_cols(ctx);
    hipLaunchKernelGGL(k_hdr_commit, flat_grid(ncs), dim3(AG_T), 0, s, ncs, c.flag, c.any, h.emp, h.pack, dknown,
                       ctx->d_dbv.as<unsigned long long>());
    CORRO_HIP_TRY(hipGetLastError());
    if (keys && !keys->empty() && hits) {
        // the merged changesets whose (site, version) holds buffered meta: keys uploaded once, a
        // binary search per flagged changeset, the hits appended (a few) and read back
        const uint64_t nk = keys->size();
        const size_t o_hit = al256(nk * 8), o_cnt = o_hit + al256(ncs * 8);
        if (int rc = ctx->d_agent_aux2.ensure(o_cnt + 256)) return rc;
        uint8_t *base = ctx->d_agent_aux2.as<uint8_t>();
        uint64_t *dk = reinterpret_cast<uint64_t *>(base);
        uint64_t *dh = reinterpret_cast<uint64_t *>(base + o_hit);  // the hits' keys
        unsigned long long *dc = reinterpret_cast<unsigned long long *>(base + o_cnt);
        CORRO_HIP_TRY(hipMemcpyAsync(dk, keys->data(), nk * 8, hipMemcpyHostToDevice, s));
        CORRO_HIP_TRY(hipMemsetAsync(dc, 0, 8, s));
        hipLaunchKernelGGL(k_hdr_clearprobe, flat_grid(ncs), dim3(AG_T), 0, s, ncs, c.flag, h.pack, dk, nk, dh, dc);
        CORRO_HIP_TRY(hipGetLastError());
        unsigned long long nh = 0;
        CORRO_HIP_TRY(hipMemcpyAsync(&nh, dc, 8, hipMemcpyDeviceToHost, s));
        CORRO_HIP_TRY(hipStreamSynchronize(s));
        if (nh) {
            std::vector<uint64_t> hk(nh);
            CORRO_HIP_TRY(hipMemcpyAsync(hk.data(), dh, nh * 8, hipMemcpyDeviceToHost, s));
            CORRO_HIP_TRY(hipStreamSynchronize(s));
            for (uint64_t k : hk) hits->emplace_back((uint32_t)(k >> 40), k & ((1ULL << 40) - 1));
        }
    }
    CORRO_HIP_TRY(hipStreamSynchronize(s));
    return CORRO_OK;
}

// The pinned host areas a call of `ncs` changesets uses (the per-changeset columns and the staged host
// headers), allocated ahead of the first call: hipHostMalloc of ~100 MB inside a call doubled the
// process's first host-header call. corro_ctx_create reserves them from its capacity hint.
int agent_dev_reserve(corro_ctx *ctx, uint64_t ncs) {
    CORRO_HIP_TRY(hipSetDevice(ctx->device));
    const uint64_t n = std::max<uint64_t>(ncs, 1);
    const size_t c8 = al256(n * 8), c4 = al256(n * 4), c1 = al256(n);
    const size_t total = 3 * c8 + c4 + 3 * c1 + 8 * 65536;
    if (total > ctx->h_agent_bytes) {
        if (ctx->h_agent) (void)hipHostFree(ctx->h_agent);
        ctx->h_agent = nullptr;
        ctx->h_agent_bytes = 0;
        CORRO_HIP_TRY(hipHostMalloc(&ctx->h_agent, total + total / 4, hipHostMallocDefault));
        ctx->h_agent_bytes = total + total / 4;
    }
    // the readback of the decided version runs and of the host changesets' headers (agent_dev_headers):
    // sized for runs of a quarter of the changesets and headers of an eighth
    const size_t fb = al256(n / 4 * 24) + al256(n / 8 * (sizeof(corro_changeset) + 10));
    if (fb > ctx->h_hfetch_bytes) {
        if (ctx->h_hfetch) (void)hipHostFree(ctx->h_hfetch);
        ctx->h_hfetch = nullptr;
        ctx->h_hfetch_bytes = 0;
        CORRO_HIP_TRY(hipHostMalloc(&ctx->h_hfetch, fb, hipHostMallocDefault));
        ctx->h_hfetch_bytes = fb;
    }
    const size_t hb = n * sizeof(corro_changeset);
    if (hb > ctx->h_hdr_bytes) {
        if (ctx->h_hdr) (void)hipHostFree(ctx->h_hdr);
        ctx->h_hdr = nullptr;
        ctx->h_hdr_bytes = 0;
        CORRO_HIP_TRY(hipHostMalloc(&ctx->h_hdr, hb + hb / 4, hipHostMallocDefault));
        ctx->h_hdr_bytes = hb + hb / 4;
    }
    // the buffered-row pool's copy jobs (bufpool_append): sized for jobs of a sixteenth of the changesets
    const size_t pb = 5 * al256(std::max<uint64_t>(n / 16, 1) * 8);
    if (pb > ctx->h_pool_bytes) {
        if (ctx->h_pool) (void)hipHostFree(ctx->h_pool);
        ctx->h_pool = nullptr;
        ctx->h_pool_bytes = 0;
        CORRO_HIP_TRY(hipHostMalloc(&ctx->h_pool, pb, hipHostMallocDefault));
        ctx->h_pool_bytes = pb;
    }
    return CORRO_OK;
}

int agent_dev_stage_begin(corro_ctx *ctx, uint64_t ncs, HdrStage *st) {
    CORRO_HIP_TRY(hipSetDevice(ctx->device));
    const size_t hb = std::max<uint64_t>(ncs, 1) * sizeof(corro_changeset);
    if (hb > ctx->h_hdr_bytes) {
        if (ctx->h_hdr) (void)hipHostFree(ctx->h_hdr);
        ctx->h_hdr = nullptr;
        ctx->h_hdr_bytes = 0;
        CORRO_HIP_TRY(hipHostMalloc(&ctx->h_hdr, hb + hb / 4, hipHostMallocDefault));
        ctx->h_hdr_bytes = hb + hb / 4;
    }
    if (int rc = ctx->d_hdr_stage.ensure(al256(hb) + al256(std::max<uint64_t>(ncs, 1) * 4))) return rc;
    st->pinned = static_cast<corro_changeset *>(ctx->h_hdr);
    st->dev = ctx->d_hdr_stage.as<corro_changeset>();
    st->dknown = reinterpret_cast<int32_t *>(ctx->d_hdr_stage.as<uint8_t>() + al256(hb));
    return CORRO_OK;
}

int agent_dev_stage_upload(corro_ctx *ctx, const HdrStage &st, uint64_t lo, uint64_t hi) {
    if (hi <= lo) return CORRO_OK;
    CORRO_HIP_TRY(hipSetDevice(ctx->device));  // (pool threads have their own current device)
    CORRO_HIP_TRY(hipMemcpyAsync(st.dev + lo, st.pinned + lo, (hi - lo) * sizeof(corro_changeset), hipMemcpyHostToDevice,
                                 ctx->stream));
    return CORRO_OK;
}

int agent_dev_stage_known(corro_ctx *ctx, const HdrStage &st, int32_t *known, uint64_t ncs) {
    if (ncs) CORRO_HIP_TRY(hipMemcpyAsync(known, st.dknown, ncs * 4, hipMemcpyDeviceToHost, ctx->stream));
    CORRO_HIP_TRY(hipStreamSynchronize(ctx->stream));
    return CORRO_OK;
}

int agent_dev_clear_known(corro_ctx *ctx, int32_t *dknown, uint64_t ncs) {
    if (ncs) CORRO_HIP_TRY(hipMemsetAsync(dknown, 0, ncs * 4, ctx->stream));  // (CORRO_KNOWN_SKIPPED = 0)
    CORRO_HIP_TRY(hipStreamSynchronize(ctx->stream));
    return CORRO_OK;
}

bool agent_site_id(corro_ctx *ctx, uint32_t site, uint8_t out[16]) {
    if (site >= ctx->sites.size()) return false;
    std::memcpy(out, ctx->sites[site].data(), 16);
    return true;
}

uint32_t agent_site_count(corro_ctx *ctx) { return (uint32_t)ctx->sites.size(); }

uint32_t agent_table_count(corro_ctx *ctx) { return (uint32_t)ctx->tables.size(); }

}  // namespace corro
