// Device-resident __corro_buffered_changes rows (interface in agent_dev.h).
//
// process_incomplete_version (/root/reference/crates/corro-agent/src/agent/util.rs:1053-1186)
// INSERTs every change of a partial changeset into __corro_buffered_changes ON CONFLICT (site_id,
// db_version, seq) DO NOTHING, and process_fully_buffered_changes (:541-688) later reads them back
// ordered by seq. When the call's changes are already in HBM, a partial changeset in the usual
// form -- its k-th change has seq = seq_start + k, the actor's own site and the changeset's version,
// no long value ("canonical") -- never needs its rows on the host: they are copied once into this
// pool, and the bookie keeps per (site, db_version) the pool segments with their seq ranges, which
// are disjoint and exact, so the conflict rule is range arithmetic on the host (agent.cpp). (The
// canonical test runs in the header gather, agent_dev.hip k_hdr_gather.)
//   k_pool_gather one wave per copy job: input changes -> pool rows (ts from the changeset when the
//                 input has none, optional fields defaulted as the host rows default them)
//   k_tab_count   per-table counts of the buffered changes (corro.changes.committed, util.rs:1101)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>

#include "agent_dev.h"
#include "internal.h"

namespace corro {

struct DevBufPool {
    int device = -1;
    DevBuf buf;
    uint64_t cap = 0, top = 0;
};

namespace {

constexpr int BP_T = 256;

size_t al256(size_t x) { return (x + 255) & ~(size_t)255; }

dim3 bp_wave_grid(uint64_t n) { return dim3((uint32_t)std::max<uint64_t>(1, std::min<uint64_t>((n + 3) / 4, 16384))); }

// pool columns for `cap` rows: pk v0 v1 ts (u64) cv dbv (i64) tcid cl seq site (u32) vt vl (u8)
corro_changes pool_view(void *base, uint64_t cap) {
    uint8_t *p = static_cast<uint8_t *>(base);
    const uint64_t c = std::max<uint64_t>(cap, 1);
    corro_changes v{};
    v.n = cap;
    size_t o = 0;
    auto take = [&](size_t elem) {
        void *q = p + o;
        o += al256(c * elem);
        return q;
    };
    v.pk = static_cast<const uint64_t *>(take(8));
    v.val0 = static_cast<const uint64_t *>(take(8));
    v.val1 = static_cast<const uint64_t *>(take(8));
    v.ts = static_cast<const uint64_t *>(take(8));
    v.col_version = static_cast<const int64_t *>(take(8));
    v.db_version = static_cast<const int64_t *>(take(8));
    v.table_cid = static_cast<const uint32_t *>(take(4));
    v.cl = static_cast<const uint32_t *>(take(4));
    v.seq = static_cast<const uint32_t *>(take(4));
    v.site = static_cast<const uint32_t *>(take(4));
    v.val_type = static_cast<const uint8_t *>(take(1));
    v.val_len = static_cast<const uint8_t *>(take(1));
    return v;
}

size_t pool_bytes(uint64_t cap) {
    const uint64_t c = std::max<uint64_t>(cap, 1);
    return 6 * al256(c * 8) + 4 * al256(c * 4) + 2 * al256(c) + 256;
}

template <class T>
__device__ inline T *wr(const T *p) {
    return const_cast<T *>(p);
}

struct PoolGatherArgs {
    corro_changes in, out;
    const uint64_t *src, *dst, *cnt, *ts;
    uint64_t n;
};

__global__ void __launch_bounds__(BP_T) k_pool_gather(PoolGatherArgs g) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t w0 = ((uint64_t)blockIdx.x * BP_T + threadIdx.x) >> 6, nw = (uint64_t)gridDim.x * (BP_T / 64);
    for (uint64_t j = w0; j < g.n; j += nw) {
        const uint64_t s = g.src[j], d = g.dst[j], c = g.cnt[j], ts = g.ts[j];
        for (uint64_t k = lane; k < c; k += 64) {
            const uint64_t i = s + k, o = d + k;
            wr(g.out.pk)[o] = g.in.pk[i];
            wr(g.out.val0)[o] = g.in.val0[i];
            wr(g.out.val1)[o] = g.in.val1 ? g.in.val1[i] : 0;
            wr(g.out.ts)[o] = g.in.ts ? g.in.ts[i] : ts;
            wr(g.out.col_version)[o] = g.in.col_version[i];
            wr(g.out.db_version)[o] = g.in.db_version[i];
            wr(g.out.table_cid)[o] = g.in.table_cid[i];
            wr(g.out.cl)[o] = g.in.cl[i];
            wr(g.out.seq)[o] = g.in.seq[i];
            wr(g.out.site)[o] = g.in.site[i];
            wr(g.out.val_type)[o] = g.in.val_type ? g.in.val_type[i] : (uint8_t)CORRO_INTEGER;
            wr(g.out.val_len)[o] = g.in.val_len ? g.in.val_len[i] : 0;
        }
    }
}

// per-table counts of the changes of spans (off, cnt): an LDS histogram per workgroup when the
// tables fit, one atomic per (workgroup, table)
constexpr uint32_t TC_LDS = 4096;
__global__ void __launch_bounds__(BP_T) k_tab_count(const uint32_t *__restrict__ tcid, const uint64_t *__restrict__ off,
                                                    const uint64_t *__restrict__ cnt, uint64_t n, uint32_t ntables,
                                                    unsigned long long *__restrict__ out) {
    __shared__ uint32_t h[TC_LDS];
    const bool lds = ntables <= TC_LDS;
    if (lds)
        for (uint32_t t = threadIdx.x; t < ntables; t += BP_T) h[t] = 0;
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t w0 = ((uint64_t)blockIdx.x * BP_T + threadIdx.x) >> 6, nw = (uint64_t)gridDim.x * (BP_T / 64);
    for (uint64_t j = w0; j < n; j += nw) {
        const uint64_t o = off[j], c = cnt[j];
        for (uint64_t k = lane; k < c; k += 64) {
            const uint32_t t = tcid[o + k] >> 16;
            if (t >= ntables) continue;
            if (lds) atomicAdd(&h[t], 1u);
            else atomicAdd(&out[t], 1ULL);
        }
    }
    __syncthreads();
    if (lds)
        for (uint32_t t = threadIdx.x; t < ntables; t += BP_T)
            if (h[t]) atomicAdd(&out[t], (unsigned long long)h[t]);
}

// k-column staging of host arrays into d_agent_fetch: k arrays of n u64 each
int stage_cols(corro_ctx *ctx, const std::vector<const std::vector<uint64_t> *> &cols, uint64_t n, uint64_t **dev) {
    const size_t k = cols.size();
    if (int rc = ctx->d_agent_fetch.ensure(k * al256(std::max<uint64_t>(n, 1) * 8) + 256)) return rc;
    uint8_t *p = ctx->d_agent_fetch.as<uint8_t>();
    for (size_t q = 0; q < k; q++) {
        dev[q] = reinterpret_cast<uint64_t *>(p + q * al256(std::max<uint64_t>(n, 1) * 8));
        if (n) CORRO_HIP_TRY(hipMemcpyAsync(dev[q], cols[q]->data(), n * 8, hipMemcpyHostToDevice, ctx->stream));
    }
    return CORRO_OK;
}

}  // namespace

DevBufPool *bufpool_new() { return new DevBufPool(); }

void bufpool_free(DevBufPool *p) {
    if (!p) return;
    if (p->buf.p && p->device >= 0) {
        int cur = 0;
        (void)hipGetDevice(&cur);
        (void)hipSetDevice(p->device);
        p->buf.release();
        (void)hipSetDevice(cur);
    }
    delete p;
}

bool bufpool_usable(corro_ctx *ctx, const DevBufPool *p) { return p && (p->device < 0 || p->device == ctx->device); }

uint64_t bufpool_top(const DevBufPool *p) { return p ? p->top : 0; }

int agent_dev_table_counts(corro_ctx *ctx, const corro_changes *dv, const std::vector<AgentSpan> &spans,
                           uint32_t ntables, std::vector<uint64_t> &counts) {
    counts.assign(ntables, 0);
    const uint64_t n = spans.size();
    if (!n || !ntables) return CORRO_OK;
    std::vector<uint64_t> off(n), cnt(n);
    for (uint64_t j = 0; j < n; j++) {
        off[j] = spans[j].src;
        cnt[j] = spans[j].count;
    }
    std::vector<uint64_t> zero(ntables, 0);
    uint64_t *d[2];
    if (int rc = stage_cols(ctx, {&off, &cnt}, n, d)) return rc;
    if (int rc = ctx->d_agent_aux2.ensure(8ULL * ntables + 256)) return rc;
    unsigned long long *dc = ctx->d_agent_aux2.as<unsigned long long>();
    CORRO_HIP_TRY(hipMemsetAsync(dc, 0, 8ULL * ntables, ctx->stream));
    hipLaunchKernelGGL(k_tab_count, bp_wave_grid(n), dim3(BP_T), 0, ctx->stream, dv->table_cid, d[0], d[1], n, ntables, dc);
    CORRO_HIP_TRY(hipGetLastError());
    CORRO_HIP_TRY(hipMemcpyAsync(counts.data(), dc, 8ULL * ntables, hipMemcpyDeviceToHost, ctx->stream));
    CORRO_HIP_TRY(hipStreamSynchronize(ctx->stream));
    return CORRO_OK;
}

// Room for `need` more rows at the pool's top. When the dead rows (below top, in no live segment)
// are at least half of top, the live segments are compacted into a fresh buffer (offs rewritten in
// place, in the order given); otherwise the buffer grows, keeping [0, top).
int bufpool_reserve(corro_ctx *ctx, DevBufPool *p, uint64_t need, std::vector<uint64_t *> &offs,
                    const std::vector<uint64_t> &lens) {
    if (!bufpool_usable(ctx, p)) return fail(CORRO_E_INVALID, "buffered-row pool belongs to another device");
    if (p->top + need <= p->cap) return CORRO_OK;
    uint64_t live = 0;
    for (uint64_t l : lens) live += l;
    const bool compact = p->top - live >= p->top / 2;
    const uint64_t keep = compact ? live : p->top;
    const uint64_t cap = std::max<uint64_t>({2 * (keep + need), 1ULL << 16});
    DevBuf nb;
    if (int rc = nb.ensure(pool_bytes(cap))) return rc;
    const corro_changes nv = pool_view(nb.p, cap);
    hipStream_t s = ctx->stream;
    if (p->buf.p && keep) {
        const corro_changes ov = pool_view(p->buf.p, p->cap);
        if (compact) {  // live segments, in the given order, packed from 0
            const uint64_t n = offs.size();
            std::vector<uint64_t> src(n), dst(n), cnt(n), ts(n, 0);
            uint64_t o = 0;
            for (uint64_t k = 0; k < n; k++) {
                src[k] = *offs[k];
                dst[k] = o;
                cnt[k] = lens[k];
                o += lens[k];
            }
            uint64_t *d[4];
            if (int rc = stage_cols(ctx, {&src, &dst, &cnt, &ts}, n, d)) {
                nb.release();
                return rc;
            }
            PoolGatherArgs g{};
            g.in = ov;
            g.out = nv;
            g.src = d[0];
            g.dst = d[1];
            g.cnt = d[2];
            g.ts = d[3];
            g.n = n;
            hipLaunchKernelGGL(k_pool_gather, bp_wave_grid(n), dim3(BP_T), 0, s, g);
            CORRO_HIP_TRY(hipGetLastError());
            for (uint64_t k = 0; k < n; k++) *offs[k] = dst[k];
        } else {
            const void *from[12] = {ov.pk, ov.val0, ov.val1, ov.ts, ov.col_version, ov.db_version,
                                    ov.table_cid, ov.cl, ov.seq, ov.site, ov.val_type, ov.val_len};
            const void *to[12] = {nv.pk, nv.val0, nv.val1, nv.ts, nv.col_version, nv.db_version,
                                  nv.table_cid, nv.cl, nv.seq, nv.site, nv.val_type, nv.val_len};
            const size_t elem[12] = {8, 8, 8, 8, 8, 8, 4, 4, 4, 4, 1, 1};
            for (int f = 0; f < 12; f++)
                CORRO_HIP_TRY(hipMemcpyAsync(const_cast<void *>(to[f]), from[f], keep * elem[f], hipMemcpyDeviceToDevice, s));
        }
    }
    CORRO_HIP_TRY(hipStreamSynchronize(s));
    p->buf.release();
    p->buf = nb;
    p->cap = cap;
    p->top = keep;
    p->device = ctx->device;
    return CORRO_OK;
}

// input changes -> pool rows at [top, top + sum(count)) in job order; dst written per job
int bufpool_append(corro_ctx *ctx, DevBufPool *p, const corro_changes *dv, std::vector<PoolCopy> &jobs) {
    const uint64_t n = jobs.size();
    if (!n) return CORRO_OK;
    uint64_t total = 0;
    for (const PoolCopy &j : jobs) total += j.count;
    if (p->top + total > p->cap) return fail(CORRO_E_INVALID, "buffered-row pool not reserved");
    // the four job columns written straight into one pinned area and sent up in one copy (four pageable
    // copies of a mixed call's 5 x 10^4 jobs cost ~0.4 ms)
    const size_t col = al256(n * 8);
    if (4 * col > ctx->h_pool_bytes) {
        if (ctx->h_pool) (void)hipHostFree(ctx->h_pool);  // (the previous append synchronised before returning)
        ctx->h_pool = nullptr;
        ctx->h_pool_bytes = 0;
        CORRO_HIP_TRY(hipHostMalloc(&ctx->h_pool, 4 * col + col, hipHostMallocDefault));
        ctx->h_pool_bytes = 4 * col + col;
    }
    if (int rc = ctx->d_agent_fetch.ensure(4 * col + 256)) return rc;
    uint8_t *hp = static_cast<uint8_t *>(ctx->h_pool);
    uint64_t *hc[4];
    for (int q = 0; q < 4; q++) hc[q] = reinterpret_cast<uint64_t *>(hp + q * col);
    for (uint64_t k = 0; k < n; k++) {
        jobs[k].dst = p->top;
        p->top += jobs[k].count;
        hc[0][k] = jobs[k].src;
        hc[1][k] = jobs[k].dst;
        hc[2][k] = jobs[k].count;
        hc[3][k] = jobs[k].ts;
    }
    uint8_t *db = ctx->d_agent_fetch.as<uint8_t>();
    CORRO_HIP_TRY(hipMemcpyAsync(db, hp, 4 * col, hipMemcpyHostToDevice, ctx->stream));
    uint64_t *d[4];
    for (int q = 0; q < 4; q++) d[q] = reinterpret_cast<uint64_t *>(db + q * col);
    PoolGatherArgs g{};
    g.in = *dv;
    g.out = pool_view(p->buf.p, p->cap);
    g.src = d[0];
    g.dst = d[1];
    g.cnt = d[2];
    g.ts = d[3];
    g.n = n;
    hipLaunchKernelGGL(k_pool_gather, bp_wave_grid(n), dim3(BP_T), 0, ctx->stream, g);
    CORRO_HIP_TRY(hipGetLastError());
    CORRO_HIP_TRY(hipStreamSynchronize(ctx->stream));  // (the staging area is reused by the next call)
    return CORRO_OK;
}

// pool rows [off, off + n) -> host arrays (synchronous, on the pool's device; no context needed)
int bufpool_read(const DevBufPool *p, uint64_t off, uint64_t n, HostSpanRows &o) {
    o = HostSpanRows{};
    if (!n) return CORRO_OK;
    if (!p || !p->buf.p || off + n > p->top) return fail(CORRO_E_INVALID, "buffered-row pool read out of range");
    int cur = 0;
    CORRO_HIP_TRY(hipGetDevice(&cur));
    CORRO_HIP_TRY(hipSetDevice(p->device));
    const corro_changes v = pool_view(p->buf.p, p->cap);
    auto get = [&](auto &vec, const void *src, size_t elem) -> hipError_t {
        vec.assign(n, 0);
        return hipMemcpy(vec.data(), static_cast<const uint8_t *>(src) + off * elem, n * elem, hipMemcpyDeviceToHost);
    };
    hipError_t e = hipSuccess;
    if (e == hipSuccess) e = get(o.pk, v.pk, 8);
    if (e == hipSuccess) e = get(o.v0, v.val0, 8);
    if (e == hipSuccess) e = get(o.v1, v.val1, 8);
    if (e == hipSuccess) e = get(o.ts, v.ts, 8);
    if (e == hipSuccess) e = get(o.cv, v.col_version, 8);
    if (e == hipSuccess) e = get(o.dbv, v.db_version, 8);
    if (e == hipSuccess) e = get(o.tcid, v.table_cid, 4);
    if (e == hipSuccess) e = get(o.cl, v.cl, 4);
    if (e == hipSuccess) e = get(o.seq, v.seq, 4);
    if (e == hipSuccess) e = get(o.site, v.site, 4);
    if (e == hipSuccess) e = get(o.vt, v.val_type, 1);
    if (e == hipSuccess) e = get(o.vl, v.val_len, 1);
    (void)hipSetDevice(cur);
    if (e != hipSuccess) return fail(CORRO_E_DEVICE, std::string("buffered-row pool read: ") + hipGetErrorString(e));
    o.lv_off.assign(n, 0);
    o.lv_len.assign(n, 0);
    return CORRO_OK;
}

int agent_dev_gaps(corro_ctx *ctx, const GapsHost &in, GapsHostOut &out) {
    const uint64_t n = in.max.size();
    out = GapsHostOut{};
    if (!n) return CORRO_OK;
    const uint64_t ng = in.gap_off[n], nv = in.ver_off[n], nw = ng + nv + n;
    // one device area: inputs, then outputs
    const size_t sz[] = {n * 8, (n + 1) * 8, ng * 8, ng * 8, (n + 1) * 8, nv * 8, nv * 8,                // in
                         n * 8, n * 8, n * 8, n * 8, ng * 8, ng * 8, nw * 8, nw * 8, nw * 8, nw * 8, n * 4};  // out
    size_t off[18], total = 0;
    for (int k = 0; k < 18; k++) {
        off[k] = total;
        total += al256(std::max<size_t>(sz[k], 8));
    }
    if (int rc = ctx->d_agent_aux2.ensure(total + 256)) return rc;
    uint8_t *d = ctx->d_agent_aux2.as<uint8_t>();
    hipStream_t s = ctx->stream;
    const void *src[7] = {in.max.data(), in.gap_off.data(), in.gap_start.data(), in.gap_end.data(),
                          in.ver_off.data(), in.ver_start.data(), in.ver_end.data()};
    for (int k = 0; k < 7; k++)
        if (sz[k]) CORRO_HIP_TRY(hipMemcpyAsync(d + off[k], src[k], sz[k], hipMemcpyHostToDevice, s));
    corro_gaps_in gi{};
    gi.n = n;
    gi.max = reinterpret_cast<const int64_t *>(d + off[0]);
    gi.gap_off = reinterpret_cast<const uint64_t *>(d + off[1]);
    gi.gap_start = reinterpret_cast<const uint64_t *>(d + off[2]);
    gi.gap_end = reinterpret_cast<const uint64_t *>(d + off[3]);
    gi.ver_off = reinterpret_cast<const uint64_t *>(d + off[4]);
    gi.ver_start = reinterpret_cast<const uint64_t *>(d + off[5]);
    gi.ver_end = reinterpret_cast<const uint64_t *>(d + off[6]);
    corro_gaps_out go{};
    go.max = reinterpret_cast<int64_t *>(d + off[7]);
    go.rm_count = reinterpret_cast<uint64_t *>(d + off[8]);
    go.ins_count = reinterpret_cast<uint64_t *>(d + off[9]);
    go.gap_count = reinterpret_cast<uint64_t *>(d + off[10]);
    go.rm_start = reinterpret_cast<uint64_t *>(d + off[11]);
    go.rm_end = reinterpret_cast<uint64_t *>(d + off[12]);
    go.ins_start = reinterpret_cast<uint64_t *>(d + off[13]);
    go.ins_end = reinterpret_cast<uint64_t *>(d + off[14]);
    go.new_start = reinterpret_cast<uint64_t *>(d + off[15]);
    go.new_end = reinterpret_cast<uint64_t *>(d + off[16]);
    go.status = reinterpret_cast<int32_t *>(d + off[17]);
    if (int rc = corro_booked_insert_db_batch(ctx, &gi, &go)) return rc;
    out.max.resize(n);
    out.rm_count.resize(n);
    out.ins_count.resize(n);
    out.gap_count.resize(n);
    out.rm_start.resize(ng);
    out.rm_end.resize(ng);
    out.ins_start.resize(nw);
    out.ins_end.resize(nw);
    out.new_start.resize(nw);
    out.new_end.resize(nw);
    out.status.resize(n);
    void *dst[11] = {out.max.data(), out.rm_count.data(), out.ins_count.data(), out.gap_count.data(),
                     out.rm_start.data(), out.rm_end.data(), out.ins_start.data(), out.ins_end.data(),
                     out.new_start.data(), out.new_end.data(), out.status.data()};
    for (int k = 0; k < 11; k++)
        if (sz[7 + k]) CORRO_HIP_TRY(hipMemcpyAsync(dst[k], d + off[7 + k], sz[7 + k], hipMemcpyDeviceToHost, s));
    CORRO_HIP_TRY(hipStreamSynchronize(s));
    return CORRO_OK;
}

}  // namespace corro
