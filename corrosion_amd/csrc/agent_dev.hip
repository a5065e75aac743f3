// Device half of corro_process_multiple_changes (agent.cpp; interface in agent_dev.h).
//
// /root/reference/crates/corro-agent/src/agent/util.rs:765-884 walks every change of every
// changeset on the host (a SAVEPOINT per version, an INSERT per change). Here the host walks only
// the changeset headers; each per-change pass is one kernel over the caller's device batch:
//   k_cs_bad       one wave per changeset: does any change name an unknown table/column (the INSERT
//                  would fail and the version's SAVEPOINT roll back, util.rs:839-860)?
//   k_span_gather  one wave per applied changeset: its changes into the applied batch (skipped when
//                  the applied changesets are one contiguous run of the input: zero-copy)
//   k_first_imp    the first batch position whose INSERT grew crsql_rows_impacted()
//   k_impactful    one wave per applied changeset: impactful flags with the transaction-cumulative
//                  counter rule (util.rs:1218-1261), per-changeset "any", per-table committed counts
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstddef>
#include <cstring>

#include "agent_dev.h"
#include <cstdlib>

#include "internal.h"

extern "C" uint64_t corro_detail_chunk_changes(const corro_ctx *ctx);  // engine.hip (apply chunk size)

namespace corro {

// prims.hip (rocPRIM)
int ovf_sort_pairs(void *temp, size_t *temp_bytes, const uint64_t *ki, uint64_t *ko, const uint32_t *vi,
                   uint32_t *vo, uint32_t n, uint32_t end_bit, hipStream_t s);
int prim_inclusive_scan_u32(void *temp, size_t *temp_bytes, const uint32_t *in, uint32_t *out, uint32_t n,
                            hipStream_t s);

namespace {

constexpr int AG_T = 256;                   // threads per workgroup: 4 waves, one changeset each
constexpr uint32_t AG_GRID_MAX = 16384;

dim3 wave_grid(uint64_t nspans) {
    return dim3((uint32_t)std::max<uint64_t>(1, std::min<uint64_t>((nspans + 3) / 4, AG_GRID_MAX)));
}

__global__ void __launch_bounds__(AG_T) k_cs_bad(const uint32_t *__restrict__ tcid, const uint64_t *__restrict__ off,
                                                  const uint64_t *__restrict__ cnt, uint64_t nspans,
                                                  uint8_t *__restrict__ bad) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t w0 = ((uint64_t)blockIdx.x * AG_T + threadIdx.x) >> 6, nw = (uint64_t)gridDim.x * (AG_T / 64);
    for (uint64_t j = w0; j < nspans; j += nw) {
        const uint64_t o = off[j], c = cnt[j];
        bool b = false;
        for (uint64_t k = lane; k < c; k += 64) b |= tcid[o + k] == CORRO_TCID_UNKNOWN;
        b = __any(b);
        if (lane == 0) bad[j] = b ? 1 : 0;
    }
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
    if ((threadIdx.x & 63) == 0 && best != ~0ULL) atomicMin(first, best);
}

struct ImpArgs {
    const uint8_t *imp;
    const uint32_t *tcid;
    const uint64_t *s_src, *s_dst, *s_cnt;
    const uint32_t *s_cs;              // changeset of each span
    uint64_t nspans;
    const unsigned long long *first;
    uint8_t *out;                      // impactful per input change (nullable)
    uint8_t *any;                      // per changeset
    unsigned long long *committed;     // per table
    uint32_t ntables;
    bool tcid_by_src;                  // tcid indexed by input index (position mode), else by batch position
};

__global__ void __launch_bounds__(AG_T) k_impactful(ImpArgs a) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t w0 = ((uint64_t)blockIdx.x * AG_T + threadIdx.x) >> 6, nw = (uint64_t)gridDim.x * (AG_T / 64);
    const unsigned long long first = *a.first;
    // committed counts: the wave's running (table, count), one atomic per table change and at the end
    uint32_t run_t = 0xFFFFFFFFu;
    unsigned long long run_c = 0;
    for (uint64_t j = w0; j < a.nspans; j += nw) {
        const uint64_t s = a.s_src[j], d = a.s_dst[j], c = a.s_cnt[j];
        bool anyb = false;
        for (uint64_t base = 0; base < c; base += 64) {  // (wave-uniform trip count)
            const uint64_t k = base + lane;
            const bool act = k < c;
            bool hit = false;
            if (act) hit = k == 0 ? first <= d : a.imp[d + k] != 0;
            if (act && a.out) a.out[s + k] = hit ? 1 : 0;
            const uint32_t t = hit ? a.tcid[(a.tcid_by_src ? s : d) + k] >> 16 : 0xFFFFFFFFu;
            unsigned long long m = __ballot(hit && t < a.ntables);
            anyb |= __ballot(hit) != 0;
            while (m) {
                const uint32_t leader = (uint32_t)__ffsll(m) - 1;
                const uint32_t tl = __shfl(t, leader);
                const unsigned long long mt = __ballot(hit && t == tl);
                if (tl != run_t) {
                    if (lane == 0 && run_c) atomicAdd(&a.committed[run_t], run_c);
                    run_t = tl;
                    run_c = 0;
                }
                run_c += (unsigned long long)__popcll(mt);
                m &= ~mt;
            }
        }
        if (lane == 0) a.any[a.s_cs[j]] = anyb ? 1 : 0;
    }
    if (lane == 0 && run_c) atomicAdd(&a.committed[run_t], run_c);
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
    if (__any(gap) && (threadIdx.x & 63) == 0) atomicOr(info, 1u);
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
    void *temp;
    size_t temp_bytes;
};

size_t sort_temp_bytes(uint64_t n) {
    size_t t0 = 0, t1 = 0;
    ovf_sort_pairs(nullptr, &t0, nullptr, nullptr, nullptr, nullptr, (uint32_t)std::max<uint64_t>(n, 1), 32, nullptr);
    prim_inclusive_scan_u32(nullptr, &t1, nullptr, nullptr, (uint32_t)std::max<uint64_t>(n, 1), nullptr);
    return std::max(t0, t1);
}

DevCols dev_cols(corro_ctx *ctx, size_t *total = nullptr) {
    const uint64_t n = std::max<uint64_t>(ctx->agent_ncs, 1);
    const size_t elem[] = {8, 8, 8, 4, 1, 1, 1, 8, 8, 4, 4, 8, 8, 8, 8, 4, 4, 4};
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

// position mode: ap[src + k] = dst + k, src_of[dst + k] = src + k and, when wanted, the ts of
// application position dst + k (the input's per-change ts, else the changeset's), a wave per span
__global__ void __launch_bounds__(AG_T) k_span_pos(const uint64_t *__restrict__ s_src, const uint64_t *__restrict__ s_dst,
                                                    const uint64_t *__restrict__ s_cnt, const uint64_t *__restrict__ s_ts,
                                                    uint64_t nspans, const uint64_t *__restrict__ in_ts,
                                                    uint32_t *__restrict__ ap, uint32_t *__restrict__ src_of,
                                                    uint64_t *__restrict__ ts_out) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t w0 = ((uint64_t)blockIdx.x * AG_T + threadIdx.x) >> 6, nw = (uint64_t)gridDim.x * (AG_T / 64);
    for (uint64_t j = w0; j < nspans; j += nw) {
        const uint64_t s = s_src[j], d = s_dst[j], c = s_cnt[j], t = s_ts[j];
        for (uint64_t k = lane; k < c; k += 64) {
            ap[s + k] = (uint32_t)(d + k);
            src_of[d + k] = (uint32_t)(s + k);
            if (ts_out) ts_out[d + k] = in_ts ? in_ts[s + k] : t;
        }
    }
}

dim3 flat_grid(uint64_t n) { return dim3((uint32_t)std::max<uint64_t>(1, std::min<uint64_t>((n + AG_T - 1) / AG_T, 8192))); }

}  // namespace

int agent_dev_begin(corro_ctx *ctx, uint64_t ncs, AgentPinned *p) {
    CORRO_HIP_TRY(hipSetDevice(ctx->device));
    CORRO_HIP_TRY(hipStreamSynchronize(ctx->stream));  // (the pinned area may still feed a copy)
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
    size_t dtotal = 0;
    (void)dev_cols(ctx, &dtotal);
    if (int rc = ctx->d_agent_spans.ensure(dtotal + 256)) return rc;
    return ctx->d_agent_out.ensure(256 + 8 * 65536);
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
    hipLaunchKernelGGL(k_cs_bad, wave_grid(ncs), dim3(AG_T), 0, s, dv->table_cid, c.off, c.cnt, ncs, c.bad);
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

int agent_dev_batch(corro_ctx *ctx, const corro_changes *dv, const AgentPinned &p, uint64_t ncs, uint64_t nspans,
                    uint64_t nbatch, bool need_ts, corro_changes *batch, bool *gathered, AgentPositions *pm) {
    *gathered = false;
    if (pm) *pm = AgentPositions{};
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
        tb = c.temp_bytes;
        if (int rc = prim_inclusive_scan_u32(c.temp, &tb, c.cnt32, c.incl, (uint32_t)nspans, s)) return rc;
        CORRO_HIP_TRY(hipMemsetAsync(c.info, 0, 4, s));
        hipLaunchKernelGGL(k_span_fin, flat_grid(nspans), dim3(AG_T), 0, s, c.s_src, c.cnt32, c.incl, nspans, c.s_dst,
                           c.s_cnt, c.info);
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
    if (pm && nspans && !(fg && fg[0] == '1') && dv->n <= corro_detail_chunk_changes(ctx) && aligned(dv->pk, 16) && aligned(dv->col_version, 16) &&
        aligned(dv->db_version, 16) && aligned(dv->val0, 16) && aligned(dv->val1, 16) && aligned(dv->table_cid, 8) &&
        aligned(dv->cl, 8) && aligned(dv->seq, 8) && aligned(dv->site, 8)) {
        const bool want_ts = need_ts || dv->ts;
        const size_t o_src = al256(dv->n * 4), o_ts = o_src + al256(nbatch * 4);
        if (int rc = ctx->d_agent_batch.ensure(o_ts + (want_ts ? nbatch * 8 : 0) + 256)) return rc;
        uint8_t *base = ctx->d_agent_batch.as<uint8_t>();
        uint32_t *ap = reinterpret_cast<uint32_t *>(base), *src_of = reinterpret_cast<uint32_t *>(base + o_src);
        uint64_t *ts = want_ts ? reinterpret_cast<uint64_t *>(base + o_ts) : nullptr;
        CORRO_HIP_TRY(hipMemsetAsync(ap, 0xFF, dv->n * 4, s));
        hipLaunchKernelGGL(k_span_pos, wave_grid(nspans), dim3(AG_T), 0, s, c.s_src, c.s_dst, c.s_cnt, c.s_ts, nspans,
                           dv->ts, ap, src_of, ts);
        CORRO_HIP_TRY(hipGetLastError());
        *batch = *dv;
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
    // scratch: first (8 B) | committed (8 per table) | host-mode impactful (nin)
    const size_t o_cm = 256, o_out = o_cm + 8 * 65536;
    const size_t total = o_out + (mem == CORRO_MEM_HOST && impactful ? al256(nin) : 0);
    if (int rc = ctx->d_agent_out.ensure(total)) return rc;
    uint8_t *base = ctx->d_agent_out.as<uint8_t>();
    unsigned long long *first = reinterpret_cast<unsigned long long *>(base);
    CORRO_HIP_TRY(hipMemsetAsync(first, 0xFF, 8, s));
    CORRO_HIP_TRY(hipMemsetAsync(base + o_cm, 0, 8ULL * std::max<uint32_t>(ntables, 1), s));
    uint8_t *out = nullptr;
    if (impactful) {
        out = mem == CORRO_MEM_DEVICE ? impactful : base + o_out;
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
        a.s_cnt = c.s_cnt;
        a.s_cs = c.val2;
        a.nspans = nspans;
        a.first = first;
        a.out = out;
        a.any = c.any;
        a.committed = reinterpret_cast<unsigned long long *>(base + o_cm);
        a.ntables = ntables;
        a.tcid_by_src = tcid_by_src;
        hipLaunchKernelGGL(k_impactful, wave_grid(nspans), dim3(AG_T), 0, s, a);
        CORRO_HIP_TRY(hipGetLastError());
        CORRO_HIP_TRY(hipMemcpyAsync(p.any, c.any, ncs, hipMemcpyDeviceToHost, s));
    }
    CORRO_HIP_TRY(hipMemcpyAsync(p.committed, base + o_cm, 8ULL * ntables, hipMemcpyDeviceToHost, s));
    if (out && mem == CORRO_MEM_HOST && nin) CORRO_HIP_TRY(hipMemcpyAsync(impactful, out, nin, hipMemcpyDeviceToHost, s));
    CORRO_HIP_TRY(hipStreamSynchronize(s));
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
