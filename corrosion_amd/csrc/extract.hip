// Server-side changeset extraction for sync: the device half of
// handle_need (/root/reference/crates/corro-agent/src/api/peer/mod.rs:371-727).
//
// For every need (actor, db_version range, optional seq range) the reference runs
//   SELECT db_version, MAX(seq), MAX(ts) FROM crsql_changes WHERE site_id = :actor
//     AND db_version BETWEEN :start AND :end GROUP BY db_version ORDER BY db_version DESC  (:385-394)
// and per version found
//   SELECT ... FROM crsql_changes WHERE site_id = :actor AND db_version = :version
//     [AND seq BETWEEN :s AND :e] ORDER BY seq ASC                                         (:423-431, :603-611)
// Here both are answered from an index over the device state's clock rows:
//   * index build (once per state epoch): one radix sort of every clock row by
//     (site, db_version, seq) packed into one 64-bit key (two stable sorts when the three do not fit
//     64 bits), then group boundaries (site, db_version) with a scan, and per group MAX(seq) (its
//     last row) and MAX(ts);
//   * extraction (two passes, like the need diff): one lane per need binary-searches its
//     [(site, start), (site, end)] slice of the sorted keys and counts groups / rows (seq filter by
//     binary search inside each group); the fill pass writes the groups in DESCENDING version order
//     and one wave per group gathers its rows (seq ascending) from the state into crsql_changes form.
// Ties on seq inside one version (a resurrecting column change also writes the row's sentinel
// clock with its own site/db_version/seq) come out in (state) index order; SQLite's order for such
// ties is unspecified by the query (parity compares them as a set).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <string>
#include <vector>

#include "internal.h"

namespace corro {

int ovf_sort_pairs(void *temp, size_t *temp_bytes, const uint64_t *ki, uint64_t *ko, const uint32_t *vi,
                   uint32_t *vo, uint32_t n, uint32_t end_bit, hipStream_t s);
int prim_inclusive_scan_u32(void *temp, size_t *temp_bytes, const uint32_t *in, uint32_t *out, uint32_t n,
                            hipStream_t s);
int state_dense_view(corro_ctx *ctx, DenseView &v);

namespace {

__device__ inline Rec x_load(const Rec *p) {
    const uint4 *q = reinterpret_cast<const uint4 *>(p);
    Rec r;
    uint4 *o = reinterpret_cast<uint4 *>(&r);
    o[0] = q[0];
    o[1] = q[1];
    o[2] = q[2];
    o[3] = q[3];
    return r;
}

struct XIndex {
    uint64_t *hkey;     // sorted (site << dbv_bits | db_version)
    uint32_t *seq;      // sorted rows' seq
    uint32_t *ref;      // sorted rows' state index
    uint32_t *gid;      // group id of sorted row i
    uint32_t *gstart;   // G + 1 group starts
    uint32_t *glast;    // MAX(seq) per group
    uint64_t *gts;      // MAX(ts) per group
};

// max db_version and max seq over the state's clock rows: per-bucket maxima (no contended
// atomics: one word per block), then one block folds them
__device__ inline void block_max2(uint64_t &a, uint64_t &b) {
    __shared__ uint64_t sa[16], sb[16];
    for (int d = 32; d >= 1; d >>= 1) {
        a = max(a, (uint64_t)__shfl_xor(a, d));
        b = max(b, (uint64_t)__shfl_xor(b, d));
    }
    const uint32_t w = threadIdx.x >> 6, nw = blockDim.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        sa[w] = a;
        sb[w] = b;
    }
    __syncthreads();
    if (threadIdx.x == 0)
        for (uint32_t k = 1; k < nw; k++) {
            a = max(a, sa[k]);
            b = max(b, sb[k]);
        }
}

__global__ void k_xmax(const Rec *st, const uint64_t *off, const uint32_t *cnt, uint64_t *part) {
    const uint32_t b = blockIdx.x;
    const uint32_t n = cnt[b];
    uint64_t md = 0, ms = 0;
    for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) {
        const Rec r = x_load(st + off[b] + i);
        md = max(md, (uint64_t)r.dbv);
        ms = max(ms, (uint64_t)r.seq);
    }
    block_max2(md, ms);
    if (threadIdx.x == 0) {
        part[2 * b] = md;
        part[2 * b + 1] = ms;
    }
}

__global__ void k_xmax_fold(const uint64_t *part, uint32_t B, uint64_t *mx) {
    uint64_t md = 0, ms = 0;
    for (uint32_t b = threadIdx.x; b < B; b += blockDim.x) {
        md = max(md, part[2 * b]);
        ms = max(ms, part[2 * b + 1]);
    }
    block_max2(md, ms);
    if (threadIdx.x == 0) {
        mx[0] = md;
        mx[1] = ms;
    }
}

// sort keys of every clock row: composite (site, dbv, seq) or, for the first of two stable sorts, seq
__global__ void k_xkeys(const Rec *st, const uint64_t *off, const uint32_t *cnt, const uint64_t *dense,
                        uint32_t db, uint32_t sb, int composite, uint64_t *keys, uint32_t *refs) {
    const uint32_t b = blockIdx.x;
    const uint32_t n = cnt[b];
    for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) {
        const uint64_t g = off[b] + i;
        const Rec r = x_load(st + g);
        const uint64_t k = dense[b] + i;
        keys[k] = composite ? (((uint64_t)r.site << (db + sb)) | ((uint64_t)r.dbv << sb) | r.seq) : (uint64_t)r.seq;
        refs[k] = (uint32_t)g;
    }
}

// second stable sort of the two-sort path: (site, dbv) keys in the seq-sorted order
__global__ void k_xkeys2(const Rec *st, const uint32_t *refs_in, uint64_t m, uint32_t db, uint64_t *keys,
                         uint32_t *refs) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    const uint32_t g = refs_in[i];
    const Rec r = x_load(st + g);
    keys[i] = ((uint64_t)r.site << db) | (uint64_t)r.dbv;
    refs[i] = g;
}

// sorted keys -> hkey / seq arrays and group-start flags (scanned afterwards)
__global__ void k_xpost(const Rec *st, const uint64_t *keys, uint64_t m, uint32_t sb, int composite, XIndex x,
                        uint32_t *flags) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    uint64_t h;
    uint32_t s;
    if (composite) {
        h = keys[i] >> sb;
        s = (uint32_t)(keys[i] & ((1ULL << sb) - 1));
    } else {
        h = keys[i];
        s = x_load(st + x.ref[i]).seq;
    }
    x.hkey[i] = h;
    x.seq[i] = s;
    const uint64_t hp = i == 0 ? ~h : (composite ? keys[i - 1] >> sb : keys[i - 1]);
    flags[i] = (i == 0 || hp != h) ? 1u : 0u;
}

// scn = inclusive scan of the start flags
__global__ void k_xgroups(XIndex x, const uint32_t *scn, uint64_t m) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    const uint32_t g = scn[i] - 1;
    if (i == 0 || scn[i - 1] != scn[i]) x.gstart[g] = (uint32_t)i;
    x.gid[i] = g;
    if (i == m - 1) x.gstart[g + 1] = (uint32_t)m;
}

__global__ void k_xgmeta(XIndex x, const uint64_t *st_ts, uint32_t G) {
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= G) return;
    const uint32_t a = x.gstart[g], b = x.gstart[g + 1];
    x.glast[g] = x.seq[b - 1];
    uint64_t t = 0;
    if (st_ts)
        for (uint32_t i = a; i < b; i++) t = max(t, st_ts[x.ref[i]]);
    x.gts[g] = t;
}

// clustered copy of the clock rows in index order (and their ts): extraction then reads each
// group's rows as one contiguous run instead of one random 64-B line per row
__global__ void k_xcluster(const Rec *st, const uint64_t *st_ts, const uint32_t *ref, uint64_t m, Rec *crec,
                           uint64_t *cts) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    const uint32_t g = ref[i];
    const Rec r = x_load(st + g);
    uint4 *o = reinterpret_cast<uint4 *>(crec + i);
    const uint4 *q = reinterpret_cast<const uint4 *>(&r);
    o[0] = q[0];
    o[1] = q[1];
    o[2] = q[2];
    o[3] = q[3];
    if (cts) cts[i] = st_ts ? st_ts[g] : 0ULL;
}

// ---- extraction ----------------------------------------------------------------------------

struct XNeeds {
    uint64_t n;
    const uint32_t *site;
    const uint64_t *start, *end;
    const uint32_t *ss, *se;  // optional seq filter
};

struct XParams {
    uint64_t m;           // indexed rows
    uint32_t db;          // dbv bits
    uint32_t nsites;
    uint64_t max_dbv;
};

__device__ inline uint64_t lower_bound64(const uint64_t *a, uint64_t n, uint64_t v) {
    uint64_t lo = 0, hi = n;
    while (lo < hi) {
        const uint64_t mid = (lo + hi) >> 1;
        if (a[mid] < v) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}
__device__ inline uint32_t lower_bound32(const uint32_t *a, uint32_t lo, uint32_t hi, uint64_t v) {
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (a[mid] < v) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

// [lo, hi) of the need's rows in the sorted index
__device__ inline void need_slice(const XIndex &x, const XParams &p, const XNeeds &nd, uint64_t e, uint64_t &lo,
                                  uint64_t &hi) {
    lo = hi = 0;
    const uint32_t site = nd.site[e];
    const uint64_t s = nd.start[e];
    uint64_t t = nd.end[e];
    if (site >= p.nsites || s > t || s > p.max_dbv || p.m == 0) return;
    if (t > p.max_dbv) t = p.max_dbv;
    const uint64_t base = (uint64_t)site << p.db;
    lo = lower_bound64(x.hkey, p.m, base | s);
    hi = lower_bound64(x.hkey, p.m, (base | t) + 1);
}

__global__ void k_xcount(XIndex x, XParams p, XNeeds nd, uint64_t *gcnt, uint64_t *rcnt) {
    const uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= nd.n) return;
    uint64_t lo, hi;
    need_slice(x, p, nd, e, lo, hi);
    uint64_t groups = 0, rows = 0;
    if (hi > lo) {
        const uint32_t g0 = x.gid[lo], g1 = x.gid[hi - 1];
        groups = g1 - g0 + 1;
        if (!nd.ss) {
            rows = hi - lo;
        } else {
            const uint64_t a0 = nd.ss[e], b0 = (uint64_t)nd.se[e];
            for (uint32_t g = g0; g <= g1; g++) {
                const uint32_t ga = x.gstart[g], gb = x.gstart[g + 1];
                if (a0 <= b0) rows += lower_bound32(x.seq, ga, gb, b0 + 1) - lower_bound32(x.seq, ga, gb, a0);
            }
        }
    }
    gcnt[e] = groups;
    rcnt[e] = rows;
}

struct XOut {
    const uint64_t *grp_off, *row_off;
    int64_t *version;
    uint64_t *last_seq, *ts, *grp_row_off, *grp_rows;
    uint32_t *out_src;   // scratch: index-order position of every output row
    corro_rows rows;
};

__global__ void k_xfill(XIndex x, XParams p, XNeeds nd, XOut o) {
    const uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= nd.n) return;
    uint64_t lo, hi;
    need_slice(x, p, nd, e, lo, hi);
    if (hi <= lo) return;
    const uint32_t g0 = x.gid[lo], g1 = x.gid[hi - 1];
    uint64_t k = o.grp_off[e], cur = o.row_off[e];
    const uint64_t dmask = (p.db >= 64) ? ~0ULL : ((1ULL << p.db) - 1);
    for (uint32_t g = g1 + 1; g-- > g0;) {  // db_version DESC
        const uint32_t ga = x.gstart[g], gb = x.gstart[g + 1];
        uint32_t a = ga, b = gb;
        if (nd.ss) {
            const uint64_t a0 = nd.ss[e], b0 = (uint64_t)nd.se[e];
            if (a0 <= b0) {
                a = lower_bound32(x.seq, ga, gb, a0);
                b = lower_bound32(x.seq, ga, gb, b0 + 1);
            } else {
                a = b = ga;
            }
        }
        o.version[k] = (int64_t)(x.hkey[ga] & dmask);
        o.last_seq[k] = x.glast[g];
        o.ts[k] = x.gts[g];
        o.grp_row_off[k] = cur;
        o.grp_rows[k] = b - a;
        for (uint32_t i = a; i < b; i++) o.out_src[cur + (i - a)] = i;
        cur += b - a;
        k++;
    }
}

// one thread per output row: rows copied from the index's clustered copy (runs of a group are
// contiguous there), into crsql_changes form
__global__ void k_xgather(const Rec *crec, const uint64_t *cts, XOut o, uint64_t R) {
    const uint64_t q = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= R) return;
    const uint32_t i = o.out_src[q];
    const Rec r = x_load(crec + i);
    const corro_rows &w = o.rows;
    if (w.pk) w.pk[q] = r.pk;
    if (w.table_cid) w.table_cid[q] = r.tcid;
    if (w.col_version) w.col_version[q] = r.cv;
    if (w.db_version) w.db_version[q] = r.dbv;
    if (w.cl) w.cl[q] = (int64_t)r.cl;
    if (w.seq) w.seq[q] = r.seq;
    if (w.site) w.site[q] = r.site;
    if (w.ts) w.ts[q] = cts ? cts[i] : 0ULL;
    if (w.val0) w.val0[q] = r.v0;
    if (w.val1) w.val1[q] = r.v1;
    if (w.val_type) w.val_type[q] = (uint8_t)(r.meta & 0xFFu);
    if (w.val_len) w.val_len[q] = (uint8_t)((r.meta >> 8) & 0xFFu);
}

uint32_t bits_for(uint64_t v) {
    uint32_t b = 1;
    while (b < 64 && (v >> b)) b++;
    return b;
}

size_t al(size_t bytes) { return ((bytes + 255) / 256) * 256; }

// Build (or reuse) the (site, db_version, seq) index of the current state.
int ensure_index(corro_ctx *ctx, XIndex &x, XParams &p) {
    hipStream_t s = ctx->stream;
    const uint64_t m = ctx->state_total;
    if (m >= (1ULL << 32)) return fail(CORRO_E_RANGE, "extraction index holds at most 2^32-1 clock rows");
    if (ctx->xidx_epoch != ctx->state_epoch) {
        if (ctx->profiling) CORRO_HIP_TRY(hipEventRecord(ctx->ev[2], s));
        // the row store's clock records, materialised densely in pseudo-buckets
        DenseView dv{};
        if (int rc = state_dense_view(ctx, dv)) return rc;
        const uint32_t B = dv.nb;
        const Rec *st = dv.st;
        const uint64_t *off = dv.off;
        const uint32_t *cnt = dv.cnt;
        // scratch: keys in/out, refs in, dense offsets, max words; rocPRIM temp after
        size_t sort_tmp = 0, scan_tmp = 0;
        if (m) {
            if (int rc = ovf_sort_pairs(nullptr, &sort_tmp, nullptr, nullptr, nullptr, nullptr, (uint32_t)m, 64, s))
                return rc;
            if (int rc = prim_inclusive_scan_u32(nullptr, &scan_tmp, nullptr, nullptr, (uint32_t)m, s)) return rc;
        }
        const size_t idx_bytes = al(m * 8) + 5 * al(m * 4 + 4) + al(m * 8 + 8) + al(m * 64) + al(m * 8);
        const size_t scr_bytes = 2 * al(m * 8) + al(m * 4) + al(B * 8ULL) + al(B * 16ULL) + 256 +
                                 al(std::max(sort_tmp, scan_tmp) + 256);
        if (int rc = ctx->d_xidx.ensure(idx_bytes + scr_bytes)) return rc;
        uint8_t *q = ctx->d_xidx.as<uint8_t>();
        auto carve = [&](size_t bytes) {
            uint8_t *r = q;
            q += al(bytes);
            return r;
        };
        ctx->x.hkey = (uint64_t *)carve(m * 8);
        ctx->x.seq = (uint32_t *)carve(m * 4 + 4);
        ctx->x.ref = (uint32_t *)carve(m * 4 + 4);
        ctx->x.gid = (uint32_t *)carve(m * 4 + 4);
        ctx->x.gstart = (uint32_t *)carve(m * 4 + 4);
        ctx->x.glast = (uint32_t *)carve(m * 4 + 4);
        ctx->x.gts = (uint64_t *)carve(m * 8 + 8);
        ctx->x.crec = (Rec *)carve(m * 64);
        ctx->x.cts = (uint64_t *)carve(m * 8);
        uint64_t *kin = (uint64_t *)carve(m * 8), *kout = (uint64_t *)carve(m * 8);
        uint32_t *rin = (uint32_t *)carve(m * 4);
        uint64_t *d_dense = (uint64_t *)carve(B * 8ULL);
        uint64_t *part = (uint64_t *)carve(B * 16ULL);
        uint64_t *mx = (uint64_t *)carve(256);
        void *tmp = carve(std::max(sort_tmp, scan_tmp) + 256);
        XIndex X{ctx->x.hkey, ctx->x.seq, ctx->x.ref, ctx->x.gid, ctx->x.gstart, ctx->x.glast, ctx->x.gts};
        uint64_t hm[2] = {0, 0};
        uint32_t G = 0;
        uint32_t db = 1, sb = 1;
        if (m) {
            std::vector<uint32_t> c(B);
            CORRO_HIP_TRY(hipMemcpy(c.data(), cnt, B * 4ULL, hipMemcpyDeviceToHost));
            std::vector<uint64_t> dense(B);
            uint64_t run = 0;
            for (uint32_t b = 0; b < B; b++) {
                dense[b] = run;
                run += c[b];
            }
            if (run != m) return fail(CORRO_E_DEVICE, "internal: state count mismatch");
            CORRO_HIP_TRY(hipMemcpyAsync(d_dense, dense.data(), B * 8ULL, hipMemcpyHostToDevice, s));
            hipLaunchKernelGGL(k_xmax, dim3(B), dim3(256), 0, s, st, off, cnt, part);
            hipLaunchKernelGGL(k_xmax_fold, dim3(1), dim3(1024), 0, s, part, B, mx);
            CORRO_HIP_TRY(hipMemcpyAsync(hm, mx, 16, hipMemcpyDeviceToHost, s));
            CORRO_HIP_TRY(hipStreamSynchronize(s));
            db = bits_for(hm[0]);
            sb = bits_for(hm[1]);
            const uint32_t stb = bits_for(ctx->sites.empty() ? 0 : ctx->sites.size() - 1);
            if (db + stb > 64) return fail(CORRO_E_RANGE, "db_version and site ordinal bits exceed 64");
            const bool composite = db + sb + stb <= 64;
            hipLaunchKernelGGL(k_xkeys, dim3(B), dim3(256), 0, s, st, off, cnt, d_dense, db, sb, composite ? 1 : 0,
                               kin, rin);
            const uint32_t mb = (uint32_t)((m + 255) / 256);
            if (composite) {
                if (int rc = ovf_sort_pairs(tmp, &sort_tmp, kin, kout, rin, X.ref, (uint32_t)m, db + sb + stb, s))
                    return rc;
            } else {
                if (int rc = ovf_sort_pairs(tmp, &sort_tmp, kin, kout, rin, X.ref, (uint32_t)m, sb, s)) return rc;
                hipLaunchKernelGGL(k_xkeys2, dim3(mb), dim3(256), 0, s, st, X.ref, m, db, kin, rin);
                if (int rc = ovf_sort_pairs(tmp, &sort_tmp, kin, kout, rin, X.ref, (uint32_t)m, db + stb, s)) return rc;
            }
            hipLaunchKernelGGL(k_xpost, dim3(mb), dim3(256), 0, s, st, kout, m, sb, composite ? 1 : 0, X, rin);
            uint32_t *scn = reinterpret_cast<uint32_t *>(kin);  // free after the sorts
            if (int rc = prim_inclusive_scan_u32(tmp, &scan_tmp, rin, scn, (uint32_t)m, s)) return rc;
            hipLaunchKernelGGL(k_xgroups, dim3(mb), dim3(256), 0, s, X, scn, m);
            CORRO_HIP_TRY(hipMemcpyAsync(&G, X.gid + (m - 1), 4, hipMemcpyDeviceToHost, s));
            CORRO_HIP_TRY(hipStreamSynchronize(s));
            G += 1;
            const uint64_t *sts = dv.ts;
            hipLaunchKernelGGL(k_xgmeta, dim3((G + 255) / 256), dim3(256), 0, s, X, sts, G);
            hipLaunchKernelGGL(k_xcluster, dim3(mb), dim3(256), 0, s, st, sts, X.ref, m, ctx->x.crec,
                               sts ? ctx->x.cts : nullptr);
            CORRO_HIP_TRY(hipGetLastError());
        }
        if (ctx->profiling) {
            CORRO_HIP_TRY(hipEventRecord(ctx->ev[3], s));
            CORRO_HIP_TRY(hipEventSynchronize(ctx->ev[3]));
            CORRO_HIP_TRY(hipEventElapsedTime(&ctx->last_ms[8], ctx->ev[2], ctx->ev[3]));
        }
        ctx->x_db = db;
        ctx->x_max_dbv = hm[0];
        ctx->x_groups = G;
        ctx->xidx_epoch = ctx->state_epoch;
    }
    x = XIndex{ctx->x.hkey, ctx->x.seq, ctx->x.ref, ctx->x.gid, ctx->x.gstart, ctx->x.glast, ctx->x.gts};
    p = XParams{m, ctx->x_db, (uint32_t)ctx->sites.size(), ctx->x_max_dbv};
    return CORRO_OK;
}

}  // namespace
}  // namespace corro

using namespace corro;

extern "C" int corro_extract_changes(corro_ctx *ctx, const corro_extract_in *in, int mem, corro_extract_out *out,
                                     int pass) {
    if (!ctx || !in || !out) return fail(CORRO_E_INVALID, "NULL argument");
    if (pass != 0 && pass != 1) return fail(CORRO_E_INVALID, "pass must be 0 or 1");
    if (mem != CORRO_MEM_HOST && mem != CORRO_MEM_DEVICE) return fail(CORRO_E_INVALID, "bad mem kind");
    if ((in->seq_start == nullptr) != (in->seq_end == nullptr))
        return fail(CORRO_E_INVALID, "seq_start and seq_end must both be given or both be NULL");
    const uint64_t n = in->n;
    if (n == 0) return CORRO_OK;
    if (!in->site || !in->start || !in->end) return fail(CORRO_E_INVALID, "a required need array is NULL");
    if (pass == 0 && (!out->grp_count || !out->row_count)) return fail(CORRO_E_INVALID, "count outputs are NULL");
    if (pass == 1 && (!out->grp_off || !out->row_off)) return fail(CORRO_E_INVALID, "grp_off / row_off are NULL");
    CORRO_HIP_TRY(hipSetDevice(ctx->device));
    hipStream_t s = ctx->stream;
    XIndex x;
    XParams p;
    if (int rc = ensure_index(ctx, x, p)) return rc;
    XNeeds nd{n, in->site, in->start, in->end, in->seq_start, in->seq_end};
    uint64_t G = 0, R = 0;
    if (pass == 1) {
        if (mem == CORRO_MEM_HOST) {
            G = out->grp_off[n];
            R = out->row_off[n];
        } else {
            CORRO_HIP_TRY(hipMemcpy(&G, out->grp_off + n, 8, hipMemcpyDeviceToHost));
            CORRO_HIP_TRY(hipMemcpy(&R, out->row_off + n, 8, hipMemcpyDeviceToHost));
        }
    }
    // device scratch: staged needs (host mode), outputs (host mode), out_src
    const bool has_seq = in->seq_start != nullptr;
    size_t need_bytes = mem == CORRO_MEM_HOST ? al(n * 4) + 2 * al(n * 8) + (has_seq ? 2 * al(n * 4) : 0) : 0;
    size_t out_bytes = 0;
    if (mem == CORRO_MEM_HOST)
        out_bytes = pass == 0 ? 2 * al(n * 8) : 2 * al((n + 1) * 8) + 5 * al(G * 8) + al(R * 8) * 7 + al(R * 4) * 3 + al(R) * 2;
    const size_t src_bytes = pass == 1 ? al(R * 4 + 4) : 0;
    if (int rc = ctx->d_xout.ensure(need_bytes + out_bytes + src_bytes + 1024)) return rc;
    uint8_t *q = ctx->d_xout.as<uint8_t>();
    auto carve = [&](size_t bytes) {
        uint8_t *r = q;
        q += al(bytes);
        return r;
    };
    if (mem == CORRO_MEM_HOST) {
        uint32_t *d_site = (uint32_t *)carve(n * 4);
        uint64_t *d_s = (uint64_t *)carve(n * 8), *d_e = (uint64_t *)carve(n * 8);
        CORRO_HIP_TRY(hipMemcpyAsync(d_site, in->site, n * 4, hipMemcpyHostToDevice, s));
        CORRO_HIP_TRY(hipMemcpyAsync(d_s, in->start, n * 8, hipMemcpyHostToDevice, s));
        CORRO_HIP_TRY(hipMemcpyAsync(d_e, in->end, n * 8, hipMemcpyHostToDevice, s));
        nd.site = d_site;
        nd.start = d_s;
        nd.end = d_e;
        if (has_seq) {
            uint32_t *a = (uint32_t *)carve(n * 4), *b = (uint32_t *)carve(n * 4);
            CORRO_HIP_TRY(hipMemcpyAsync(a, in->seq_start, n * 4, hipMemcpyHostToDevice, s));
            CORRO_HIP_TRY(hipMemcpyAsync(b, in->seq_end, n * 4, hipMemcpyHostToDevice, s));
            nd.ss = a;
            nd.se = b;
        }
    }
    const uint32_t nb = (uint32_t)((n + 255) / 256);
    if (ctx->profiling) CORRO_HIP_TRY(hipEventRecord(ctx->ev[0], s));
    if (pass == 0) {
        uint64_t *gc = out->grp_count, *rc = out->row_count;
        if (mem == CORRO_MEM_HOST) {
            gc = (uint64_t *)carve(n * 8);
            rc = (uint64_t *)carve(n * 8);
        }
        hipLaunchKernelGGL(k_xcount, dim3(nb), dim3(256), 0, s, x, p, nd, gc, rc);
        if (ctx->profiling) CORRO_HIP_TRY(hipEventRecord(ctx->ev[1], s));
        CORRO_HIP_TRY(hipGetLastError());
        if (mem == CORRO_MEM_HOST) {
            CORRO_HIP_TRY(hipMemcpyAsync(out->grp_count, gc, n * 8, hipMemcpyDeviceToHost, s));
            CORRO_HIP_TRY(hipMemcpyAsync(out->row_count, rc, n * 8, hipMemcpyDeviceToHost, s));
        }
    } else {
        XOut o{};
        o.out_src = (uint32_t *)carve(R * 4 + 4);
        if (mem == CORRO_MEM_DEVICE) {
            o.grp_off = out->grp_off;
            o.row_off = out->row_off;
            o.version = out->version;
            o.last_seq = out->last_seq;
            o.ts = out->ts;
            o.grp_row_off = out->grp_row_off;
            o.grp_rows = out->grp_rows;
            o.rows = out->rows;
        } else {
            uint64_t *go = (uint64_t *)carve((n + 1) * 8), *ro = (uint64_t *)carve((n + 1) * 8);
            CORRO_HIP_TRY(hipMemcpyAsync(go, out->grp_off, (n + 1) * 8, hipMemcpyHostToDevice, s));
            CORRO_HIP_TRY(hipMemcpyAsync(ro, out->row_off, (n + 1) * 8, hipMemcpyHostToDevice, s));
            o.grp_off = go;
            o.row_off = ro;
            o.version = (int64_t *)carve(G * 8);
            o.last_seq = (uint64_t *)carve(G * 8);
            o.ts = (uint64_t *)carve(G * 8);
            o.grp_row_off = (uint64_t *)carve(G * 8);
            o.grp_rows = (uint64_t *)carve(G * 8);
            corro_rows &w = o.rows;
            const corro_rows &h = out->rows;
            w.pk = h.pk ? (uint64_t *)carve(R * 8) : nullptr;
            w.col_version = h.col_version ? (int64_t *)carve(R * 8) : nullptr;
            w.db_version = h.db_version ? (int64_t *)carve(R * 8) : nullptr;
            w.cl = h.cl ? (int64_t *)carve(R * 8) : nullptr;
            w.ts = h.ts ? (uint64_t *)carve(R * 8) : nullptr;
            w.val0 = h.val0 ? (uint64_t *)carve(R * 8) : nullptr;
            w.val1 = h.val1 ? (uint64_t *)carve(R * 8) : nullptr;
            w.table_cid = h.table_cid ? (uint32_t *)carve(R * 4) : nullptr;
            w.seq = h.seq ? (uint32_t *)carve(R * 4) : nullptr;
            w.site = h.site ? (uint32_t *)carve(R * 4) : nullptr;
            w.val_type = h.val_type ? (uint8_t *)carve(R) : nullptr;
            w.val_len = h.val_len ? (uint8_t *)carve(R) : nullptr;
        }
        hipLaunchKernelGGL(k_xfill, dim3(nb), dim3(256), 0, s, x, p, nd, o);
        if (R)
            hipLaunchKernelGGL(k_xgather, dim3((uint32_t)((R + 255) / 256)), dim3(256), 0, s, ctx->x.crec,
                               ctx->track_ts ? ctx->x.cts : nullptr, o, R);
        if (ctx->profiling) CORRO_HIP_TRY(hipEventRecord(ctx->ev[1], s));
        CORRO_HIP_TRY(hipGetLastError());
        if (mem == CORRO_MEM_HOST) {
            struct Cp { void *dst; const void *src; size_t bytes; } cp[] = {
                {out->version, o.version, G * 8},         {out->last_seq, o.last_seq, G * 8},
                {out->ts, o.ts, G * 8},                   {out->grp_row_off, o.grp_row_off, G * 8},
                {out->grp_rows, o.grp_rows, G * 8},       {out->rows.pk, o.rows.pk, R * 8},
                {out->rows.col_version, o.rows.col_version, R * 8}, {out->rows.db_version, o.rows.db_version, R * 8},
                {out->rows.cl, o.rows.cl, R * 8},         {out->rows.ts, o.rows.ts, R * 8},
                {out->rows.val0, o.rows.val0, R * 8},     {out->rows.val1, o.rows.val1, R * 8},
                {out->rows.table_cid, o.rows.table_cid, R * 4}, {out->rows.seq, o.rows.seq, R * 4},
                {out->rows.site, o.rows.site, R * 4},     {out->rows.val_type, o.rows.val_type, R},
                {out->rows.val_len, o.rows.val_len, R}};
            for (auto &c : cp)
                if (c.dst && c.bytes) CORRO_HIP_TRY(hipMemcpyAsync(c.dst, c.src, c.bytes, hipMemcpyDeviceToHost, s));
        }
    }
    CORRO_HIP_TRY(hipStreamSynchronize(s));
    if (ctx->profiling) CORRO_HIP_TRY(hipEventElapsedTime(&ctx->last_ms[6 + pass], ctx->ev[0], ctx->ev[1]));
    return CORRO_OK;
}
