// libcorro_hip.so — context, site registry and the apply_batch pipeline (C ABI, corro_hip.h).
//
// corro_apply_batch replaces, for one `process_multiple_changes` call, the nest
//   for actor { for changeset { SAVEPOINT; for change { INSERT INTO crsql_changes; ... } } }
// of /root/reference/crates/corro-agent/src/agent/util.rs:765-884 + :1222-1262 with one batched
// device merge. Kernels: merge_kernels.h. Host bookkeeping stays with the caller.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <numeric>

#include "internal.h"
#include "merge_kernels.h"

namespace corro {

static thread_local std::string g_last_error;

void set_error(const std::string &msg) { g_last_error = msg; }

int fail(int code, const std::string &msg) {
    g_last_error = msg;
    return code;
}

int DevBuf::ensure(size_t want) {
    if (want <= bytes && p) return CORRO_OK;
    release();
    size_t alloc = std::max<size_t>(want, 256);
    hipError_t e = hipMalloc(&p, alloc);
    if (e != hipSuccess) {
        p = nullptr;
        bytes = 0;
        return fail(CORRO_E_NOMEM, std::string("hipMalloc(") + std::to_string(alloc) + "): " + hipGetErrorString(e));
    }
    bytes = alloc;
    return CORRO_OK;
}

void DevBuf::release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    bytes = 0;
}

}  // namespace corro

using namespace corro;

#define TRY(x)                       \
    do {                             \
        int rc_ = (x);               \
        if (rc_ != CORRO_OK) return rc_; \
    } while (0)

namespace corro {
int ovf_sort_pairs(void *temp, size_t *temp_bytes, const uint64_t *ki, uint64_t *ko, const uint32_t *vi,
                   uint32_t *vo, uint32_t n, uint32_t end_bit, hipStream_t s);

int ovf_scans(void *temp, size_t *temp_bytes, const OvfDev &d, int which, hipStream_t s);
int prim_inclusive_scan_u32(void *temp, size_t *temp_bytes, const uint32_t *in, uint32_t *out, uint32_t n,
                            hipStream_t s);
int ovf_scan_tiles(void *temp, size_t *temp_bytes, const OvfDev &d, const CsAgg *in, CsAgg *out, uint32_t n,
                   hipStream_t s);

// Oversized buckets (after the first merge pass queued them), all at once and device-wide (the
// phases of ovf_kernels.h): fields + row ids -> sort by (bucket base + row, position) -> L scan ->
// classify -> epoch scan -> candidate keys -> sort -> argmax / group-start scans -> link -> walk
// -> [impacts] -> per-bucket counts.
static int run_overflow(corro_ctx *ctx, MergeArgs &a, uint64_t novf, uint64_t nbatch, bool prof) {
    hipStream_t s = ctx->stream;
    const uint32_t B = ctx->B;
    std::vector<uint32_t> list(novf), pc(B), nc(B);
    CORRO_HIP_TRY(hipMemcpy(list.data(), ctx->d_ovf_list.p, novf * 4, hipMemcpyDeviceToHost));
    CORRO_HIP_TRY(hipMemcpy(pc.data(), ctx->d_state_cnt.p, B * 4ULL, hipMemcpyDeviceToHost));
    CORRO_HIP_TRY(hipMemcpy(nc.data(), ctx->d_new_cnt.p, B * 4ULL, hipMemcpyDeviceToHost));
    std::vector<uint32_t> koff(novf + 1), soff(novf);
    uint64_t K = 0, S = 0, PM = 0;
    for (uint64_t k = 0; k < novf; k++) {
        const uint64_t n = (uint64_t)pc[list[k]] + nc[list[k]];
        PM = std::max<uint64_t>(PM, pc[list[k]]);
        uint64_t sl = 1;
        while (sl < 2 * n) sl <<= 1;
        koff[k] = (uint32_t)K;
        soff[k] = (uint32_t)S;
        K += n;
        S += sl;
        if (K >= (1ULL << 31) || S >= (1ULL << 32))
            return fail(CORRO_E_RANGE, "oversized buckets hold more than 2^31 records");
    }
    koff[novf] = (uint32_t)K;
    // row ids (< K) take rb bits with one spare value above them, so that ~0 sorts last
    uint32_t rb = 1;
    while ((1ULL << rb) <= K) rb++;
    // compact positions: prior slice index < PM, batch change i -> PM + i
    uint32_t pbits = 1;
    while ((1ULL << pbits) < PM + nbatch) pbits++;
    uint32_t maxc = 0, cid_bits = 1;
    for (const auto &t : ctx->tables) maxc = std::max<uint32_t>(maxc, (uint32_t)t.cols.size());
    while ((1u << cid_bits) <= maxc) cid_bits++;
    const uint32_t ckey_bits = rb + cid_bits;
    auto al = [](uint64_t x) { return (x + 255) & ~255ULL; };
    // pass 0 sizes the arrays, pass 1 carves them out of d_ovf_sort
    OvfDev d{};
    d.G = (uint32_t)novf;
    d.K = (uint32_t)K;
    d.cid_bits = cid_bits;
    d.rshift = pbits;
    d.pm = (uint32_t)PM;
    uint64_t bytes = 0;
    uint8_t *base = nullptr;
    auto take = [&](uint64_t n) {
        uint8_t *r = base ? base + bytes : nullptr;
        bytes += al(n);
        return r;
    };
    void *d_temp = nullptr;
    size_t temp = 0;
    uint32_t nt = 0, *cs_first = nullptr;
    CsAgg *cs_agg = nullptr, *cs_incl = nullptr;
    for (int pass = 0; pass < 2; pass++) {
        bytes = 0;
        d.koff = (const uint32_t *)take((novf + 1) * 4);
        d.slot_off = (const uint32_t *)take(novf * 4);
        d.ocnt = (uint32_t *)take(novf * 4);
        d.oflag = (uint32_t *)take(novf * 4);
        d.slots = (uint32_t *)take(S * 4);
        uint64_t **u64s[] = {&d.pk, &d.key, &d.key_s, &d.ckey, &d.ckey_s};
        for (uint64_t **p : u64s) *p = (uint64_t *)take(K * 8);
        d.cv = (int64_t *)take(K * 8);
        d.ccv = (int64_t *)take(K * 8);
        d.qkey = (OvfKey *)take(K * sizeof(OvfKey));
        uint32_t **u32s[] = {&d.tc,    &d.cl,     &d.pos,   &d.val,    &d.val_s, &d.rowid,
                             &d.cl_s,  &d.lx,     &d.recf,  &d.epc,   &d.kind,  &d.pb,     &d.rstart, &d.rbad,
                             &d.rnrec, &d.recs,   &d.head,  &d.scid,  &d.spos,  &d.sz,     &d.ccid,  &d.csrc,
                             &d.cval,  &d.cval_s, &d.cbest, &d.cgs,   &d.nxt,   &d.fstg};
        for (uint32_t **p : u32s) *p = (uint32_t *)take(K * 4);
        if (pass == 0) {
            size_t t0 = 0, t1 = 0, t2 = 0, t3 = 0;
            TRY(ovf_sort_pairs(nullptr, &t0, nullptr, nullptr, nullptr, nullptr, d.K, 64, s));
            TRY(ovf_sort_pairs(nullptr, &t1, nullptr, nullptr, nullptr, nullptr, d.K, ckey_bits, s));
            TRY(ovf_scans(nullptr, &t2, d, 0, s));
            TRY(prim_inclusive_scan_u32(nullptr, &t3, nullptr, nullptr, d.K, s));
            size_t t4 = 0;
            TRY(ovf_scan_tiles(nullptr, &t4, d, nullptr, nullptr, (uint32_t)((K + CS_TILE - 1) / CS_TILE), s));
            temp = std::max(std::max(std::max(t0, t1), std::max(t2, t3)), t4);
        }
        nt = (uint32_t)((K + CS_TILE - 1) / CS_TILE);
        cs_agg = (CsAgg *)take(nt * 8ULL);
        cs_incl = (CsAgg *)take(nt * 8ULL);
        cs_first = (uint32_t *)take(nt * 4ULL);
        d_temp = take(temp);
        if (pass == 0) {
            TRY(ctx->d_ovf_sort.ensure(bytes + 256));
            base = ctx->d_ovf_sort.as<uint8_t>();
        }
    }
    CORRO_HIP_TRY(hipMemcpyAsync((void *)d.koff, koff.data(), (novf + 1) * 4, hipMemcpyHostToDevice, s));
    CORRO_HIP_TRY(hipMemcpyAsync((void *)d.slot_off, soff.data(), novf * 4, hipMemcpyHostToDevice, s));
    CORRO_HIP_TRY(hipMemsetAsync(d.ocnt, 0, novf * 4, s));
    CORRO_HIP_TRY(hipMemsetAsync(d.oflag, 0, novf * 4, s));
    CORRO_HIP_TRY(hipMemsetAsync(d.slots, 0, S * 4, s));
    if (prof) (void)hipEventRecord(ctx->ev[6], s);
    const dim3 blk(256), grid((uint32_t)std::min<uint64_t>((K + 255) / 256, 8192));
    auto launched = [&]() -> int {
        CORRO_HIP_TRY(hipGetLastError());
        return CORRO_OK;
    };
    hipLaunchKernelGGL(k_ovf_load, grid, blk, 0, s, a, d);
    hipLaunchKernelGGL(k_ovf_rowhash, grid, blk, 0, s, d);
    TRY(launched());
    // dense row ids: the row count sizes the sort's key
    TRY(prim_inclusive_scan_u32(d_temp, &temp, d.recf, d.epc, d.K, s));
    uint32_t nrows = 0;
    CORRO_HIP_TRY(hipMemcpyAsync(&nrows, d.epc + (K - 1), 4, hipMemcpyDeviceToHost, s));
    CORRO_HIP_TRY(hipStreamSynchronize(s));
    uint32_t rbits = 1;
    while ((1ULL << rbits) < nrows) rbits++;
    const uint32_t key_bits = rbits + pbits;
    d.nrows = nrows;
    if (key_bits > 64) return fail(CORRO_E_RANGE, "overflow sort key exceeds 64 bits");
    static const bool dbg = std::getenv("CORRO_HIP_OVF_DEBUG") != nullptr;
    if (dbg)
        fprintf(stderr, "[corro ovf] buckets %llu records %llu rows %u key bits %u (+%u) cand key bits %u\n",
                (unsigned long long)novf, (unsigned long long)K, nrows, key_bits, rbits, ckey_bits);
    hipLaunchKernelGGL(k_ovf_rowkey, grid, blk, 0, s, d);
    TRY(launched());
    TRY(ovf_sort_pairs(d_temp, &temp, d.key, d.key_s, d.val, d.val_s, d.K, key_bits, s));
    hipLaunchKernelGGL(k_ovf_gather, grid, blk, 0, s, d);
    TRY(launched());
    TRY(ovf_scans(d_temp, &temp, d, 0, s));
    hipLaunchKernelGGL(k_ovf_classify, grid, blk, 0, s, a, d);
    TRY(launched());
    TRY(ovf_scans(d_temp, &temp, d, 1, s));
    hipLaunchKernelGGL(k_ovf_epochs, grid, blk, 0, s, d);
    hipLaunchKernelGGL(k_ovf_ckeys, grid, blk, 0, s, d);
    TRY(launched());
    // only the candidates are sorted (a minority of the records): compact them first
    TRY(prim_inclusive_scan_u32(d_temp, &temp, d.slots, d.slots + K, d.K, s));
    uint32_t ncand = 0;
    CORRO_HIP_TRY(hipMemcpyAsync(&ncand, d.slots + K + (K - 1), 4, hipMemcpyDeviceToHost, s));
    CORRO_HIP_TRY(hipStreamSynchronize(s));
    hipLaunchKernelGGL(k_ovf_ccompact, grid, blk, 0, s, d);
    TRY(launched());
    if (ncand) TRY(ovf_sort_pairs(d_temp, &temp, d.key, d.ckey_s, d.val, d.cval_s, ncand, ckey_bits, s));
    if (ncand < K) CORRO_HIP_TRY(hipMemsetAsync(d.ckey_s + ncand, 0xFF, (K - ncand) * 8, s));
    if (dbg) fprintf(stderr, "[corro ovf] candidates %u\n", ncand);
    d.ncand = ncand;
    const dim3 cgrid((uint32_t)std::max<uint64_t>(1, std::min<uint64_t>((ncand + 255) / 256, 8192)));
    hipLaunchKernelGGL(k_ovf_cgather, cgrid, blk, 0, s, a, d);
    TRY(launched());
    if (ncand) {
        const uint32_t ntc = (ncand + CS_TILE - 1) / CS_TILE;  // <= nt
        hipLaunchKernelGGL(k_cscan_tile, dim3(ntc), dim3(CS_T), 0, s, d, cs_agg, cs_first);
        TRY(launched());
        TRY(ovf_scan_tiles(d_temp, &temp, d, cs_agg, cs_incl, ntc, s));
        hipLaunchKernelGGL(k_cscan_fix, dim3(ntc), dim3(CS_T), 0, s, d, cs_incl, cs_first);
    }
    TRY(launched());
    if (ncand) TRY(ovf_scans(d_temp, &temp, d, 2, s));
    hipLaunchKernelGGL(k_ovf_link, cgrid, blk, 0, s, d);
    // carried cells in registers when no table has WALK_MAXC or more columns (cids 1..ncols)
    auto walk = maxc + 1 <= WALK_MAXC ? k_ovf_walk<true> : k_ovf_walk<false>;
    hipLaunchKernelGGL(walk, dim3((uint32_t)std::max<uint64_t>(1, std::min<uint64_t>((nrows + 255) / 256, 8192))),
                       blk, 0, s, a, d);
    if (a.impact) hipLaunchKernelGGL(k_ovf_impacts, cgrid, blk, 0, s, a, d);
    hipLaunchKernelGGL(k_ovf_finish, dim3((uint32_t)((novf + 255) / 256)), blk, 0, s, a, d);
    TRY(launched());
    if (prof) (void)hipEventRecord(ctx->ev[7], s);
    CORRO_HIP_TRY(hipMemcpyAsync(ctx->h_misc, a.misc, 4 * 8, hipMemcpyDeviceToHost, s));
    CORRO_HIP_TRY(hipStreamSynchronize(s));
    if (prof) CORRO_HIP_TRY(hipEventElapsedTime(&ctx->last_ms[5], ctx->ev[6], ctx->ev[7]));
    return CORRO_OK;
}
}  // namespace corro

extern "C" {

const char *corro_last_error(void) { return g_last_error.c_str(); }

int corro_abi_version(void) { return CORRO_HIP_ABI_VERSION; }

int corro_device_count(int *count) {
    if (!count) return fail(CORRO_E_INVALID, "count is NULL");
    int c = 0;
    hipError_t e = hipGetDeviceCount(&c);
    if (e != hipSuccess) c = 0;
    *count = c;
    return CORRO_OK;
}

static int ctx_prepare_device(corro_ctx *ctx) {
    int c = 0;
    if (hipGetDeviceCount(&c) != hipSuccess || c == 0)
        return fail(CORRO_E_NO_DEVICE, "no HIP device visible: the merge engine has no CPU fallback");
    if (ctx->device < 0 || ctx->device >= c) return fail(CORRO_E_INVALID, "device ordinal out of range");
    CORRO_HIP_TRY(hipSetDevice(ctx->device));
    hipDeviceProp_t prop;
    CORRO_HIP_TRY(hipGetDeviceProperties(&prop, ctx->device));
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        return fail(CORRO_E_NO_DEVICE, std::string("libcorro_hip is built for gfx950, device is ") + prop.gcnArchName);
    CORRO_HIP_TRY(hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking));
    CORRO_HIP_TRY(hipHostMalloc((void **)&ctx->h_misc, 8 * sizeof(uint64_t), hipHostMallocDefault));
    for (auto &e : ctx->ev) CORRO_HIP_TRY(hipEventCreate(&e));
    const size_t lds_max = 160 * 1024;
    CORRO_HIP_TRY(hipFuncSetAttribute((const void *)k_hist, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_max));
    for (const void *f : {(const void *)k_scatter<true, true>, (const void *)k_scatter<true, false>,
                          (const void *)k_scatter<false, true>, (const void *)k_scatter<false, false>})
        CORRO_HIP_TRY(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_max));
    return CORRO_OK;
}

int corro_ctx_create(const corro_table_desc *tables, uint32_t ntables, uint64_t capacity_hint, int device,
                     corro_ctx **out) {
    if (!out) return fail(CORRO_E_INVALID, "out is NULL");
    *out = nullptr;
    if (!tables && ntables) return fail(CORRO_E_INVALID, "tables is NULL");
    if (ntables > 65535) return fail(CORRO_E_RANGE, "at most 65535 tables");
    corro_ctx *ctx = new corro_ctx();
    ctx->device = device;
    for (uint32_t t = 0; t < ntables; t++) {
        if (!tables[t].name) {
            delete ctx;
            return fail(CORRO_E_INVALID, "table name is NULL");
        }
        if (tables[t].ncols > 65535) {
            delete ctx;
            return fail(CORRO_E_RANGE, "at most 65535 columns per table");
        }
        Table tb;
        tb.name = tables[t].name;
        for (uint32_t c = 0; c < tables[t].ncols; c++) tb.cols.emplace_back(tables[t].col_names[c]);
        ctx->table_index[tb.name] = t;
        ctx->tables.push_back(std::move(tb));
    }
    // bucket count: ~1280 records per bucket at the hinted merge size, at most 2^15 buckets
    uint64_t per = std::max<uint64_t>(1, capacity_hint / 1280);
    uint32_t lg = 0;
    while ((1ULL << lg) < per && lg < 15) lg++;
    ctx->log2B = lg;
    ctx->B = 1u << lg;
    int rc = ctx_prepare_device(ctx);
    if (rc != CORRO_OK) {
        corro_ctx_destroy(ctx);
        return rc;
    }
    const uint32_t B = ctx->B;
    rc = ctx->d_state_off.ensure(B * 8ULL);
    if (!rc) rc = ctx->d_state_cnt.ensure(B * 4ULL);
    if (!rc) rc = ctx->d_state_flags.ensure(B * 4ULL);
    if (!rc) rc = ctx->d_out_off.ensure(B * 8ULL);
    if (!rc) rc = ctx->d_out_cnt.ensure(B * 4ULL);
    if (!rc) rc = ctx->d_out_flags.ensure(B * 4ULL);
    if (!rc) rc = ctx->d_new_cnt.ensure(B * 4ULL);
    if (!rc) rc = ctx->d_stage_off.ensure(B * 4ULL);
    if (!rc) rc = ctx->d_bflags.ensure(((B + 31) / 32) * 4ULL);
    if (!rc) rc = ctx->d_misc.ensure(8 * 8);
    if (!rc) rc = ctx->d_ovf_list.ensure(B * 4ULL);
    if (!rc) rc = ctx->d_gen_list.ensure(3 * B * 4ULL);
    if (!rc) rc = ctx->d_wide_list.ensure(B * 4ULL);
    if (!rc) rc = ctx->d_state[0].ensure(64);
    if (!rc) rc = ctx->d_state[1].ensure(64);
    if (rc != CORRO_OK) {
        corro_ctx_destroy(ctx);
        return rc;
    }
    {
        std::vector<uint16_t> ncols(ctx->tables.size() + 1, 0);
        for (size_t t = 0; t < ctx->tables.size(); t++) ncols[t] = (uint16_t)ctx->tables[t].cols.size();
        rc = ctx->d_ncols.ensure(ncols.size() * 2);
        if (rc == CORRO_OK && hipMemcpy(ctx->d_ncols.p, ncols.data(), ncols.size() * 2, hipMemcpyHostToDevice) != hipSuccess)
            rc = fail(CORRO_E_DEVICE, "upload of the schema failed");
        if (rc != CORRO_OK) {
            corro_ctx_destroy(ctx);
            return rc;
        }
    }
    (void)hipMemsetAsync(ctx->d_state_off.p, 0, B * 8ULL, ctx->stream);
    (void)hipMemsetAsync(ctx->d_state_cnt.p, 0, B * 4ULL, ctx->stream);
    (void)hipMemsetAsync(ctx->d_state_flags.p, 0, B * 4ULL, ctx->stream);
    if (hipStreamSynchronize(ctx->stream) != hipSuccess) {
        corro_ctx_destroy(ctx);
        return fail(CORRO_E_DEVICE, "stream synchronize failed");
    }
    *out = ctx;
    return CORRO_OK;
}

void corro_ctx_destroy(corro_ctx *ctx) {
    if (!ctx) return;
    if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
    DevBuf *bufs[] = {&ctx->d_site_rank, &ctx->d_dbv, &ctx->d_dbv_batch, &ctx->d_state[0], &ctx->d_state[1],
                      &ctx->d_state_ts[0], &ctx->d_state_ts[1], &ctx->d_state_off, &ctx->d_state_cnt,
                      &ctx->d_state_flags, &ctx->d_out_off, &ctx->d_out_cnt, &ctx->d_out_flags, &ctx->d_in,
                      &ctx->d_hist, &ctx->d_new_cnt, &ctx->d_stage_off, &ctx->d_bflags, &ctx->d_stage,
                      &ctx->d_misc, &ctx->d_ovf_list, &ctx->d_gen_list, &ctx->d_wide_list, &ctx->d_ovf_sort, &ctx->d_scan_tmp, &ctx->d_impact, &ctx->d_export,
                      &ctx->d_needs, &ctx->d_needs1, &ctx->d_xidx, &ctx->d_xout, &ctx->d_wire, &ctx->d_wire_schema, &ctx->d_wire_sites, &ctx->d_ncols, &ctx->d_part};
    for (DevBuf *b : bufs) b->release();
    if (ctx->h_misc) (void)hipHostFree(ctx->h_misc);
    for (auto &e : ctx->ev)
        if (e) (void)hipEventDestroy(e);
    if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
    delete ctx;
}

int corro_lookup_cid(corro_ctx *ctx, const char *table, const char *cid, uint32_t *table_cid) {
    if (!ctx || !table || !cid || !table_cid) return fail(CORRO_E_INVALID, "NULL argument");
    auto it = ctx->table_index.find(table);
    if (it == ctx->table_index.end()) return fail(CORRO_E_UNKNOWN_TABLE, std::string("no such table: ") + table);
    const Table &tb = ctx->tables[it->second];
    if (std::strcmp(cid, "-1") == 0) {
        *table_cid = it->second << 16;
        return CORRO_OK;
    }
    for (size_t c = 0; c < tb.cols.size(); c++)
        if (tb.cols[c] == cid) {
            *table_cid = (it->second << 16) | (uint32_t)(c + 1);
            return CORRO_OK;
        }
    return fail(CORRO_E_UNKNOWN_COLUMN, std::string("SQL logic error: no column ") + cid + " in " + table);
}

static int upload_site_tables(corro_ctx *ctx) {
    const uint32_t n = (uint32_t)ctx->sites.size();
    std::vector<uint32_t> order(n), rank(n);
    std::iota(order.begin(), order.end(), 0u);
    std::sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) {
        return std::memcmp(ctx->sites[a].data(), ctx->sites[b].data(), 16) < 0;
    });
    for (uint32_t r = 0; r < n; r++) rank[order[r]] = r;
    TRY(ctx->d_site_rank.ensure(std::max<size_t>(n, 1) * 4));
    CORRO_HIP_TRY(hipMemcpyAsync(ctx->d_site_rank.p, rank.data(), n * 4ULL, hipMemcpyHostToDevice, ctx->stream));
    if (n > ctx->dbv_cap) {
        size_t cap = std::max<size_t>(n, 2 * ctx->dbv_cap);
        DevBuf nb;
        TRY(nb.ensure(cap * 8));
        CORRO_HIP_TRY(hipMemsetAsync(nb.p, 0, cap * 8, ctx->stream));
        if (ctx->dbv_cap)
            CORRO_HIP_TRY(hipMemcpyAsync(nb.p, ctx->d_dbv.p, ctx->dbv_cap * 8, hipMemcpyDeviceToDevice, ctx->stream));
        CORRO_HIP_TRY(hipStreamSynchronize(ctx->stream));
        ctx->d_dbv.release();
        ctx->d_dbv = nb;
        nb.p = nullptr;
        ctx->dbv_cap = cap;
        TRY(ctx->d_dbv_batch.ensure(cap * 8));
    }
    CORRO_HIP_TRY(hipStreamSynchronize(ctx->stream));
    return CORRO_OK;
}

int corro_site_register(corro_ctx *ctx, const uint8_t *site_ids, uint64_t n, uint32_t *ordinals) {
    if (!ctx || (!site_ids && n)) return fail(CORRO_E_INVALID, "NULL argument");
    bool added = false;
    for (uint64_t i = 0; i < n; i++) {
        std::array<uint8_t, 16> id;
        std::memcpy(id.data(), site_ids + 16 * i, 16);
        auto it = ctx->site_ordinal.find(id);
        uint32_t ord;
        if (it == ctx->site_ordinal.end()) {
            ord = (uint32_t)ctx->sites.size();
            ctx->sites.push_back(id);
            ctx->site_ordinal[id] = ord;
            added = true;
        } else {
            ord = it->second;
        }
        if (ordinals) ordinals[i] = ord;
    }
    if (added) return upload_site_tables(ctx);
    return CORRO_OK;
}

int corro_site_ids(corro_ctx *ctx, uint8_t *ids, uint32_t cap, uint32_t *count) {
    if (!ctx || !count || (cap && !ids)) return fail(CORRO_E_INVALID, "NULL argument");
    const uint32_t n = (uint32_t)ctx->sites.size();
    for (uint32_t i = 0; i < n && i < cap; i++) std::memcpy(ids + 16ULL * i, ctx->sites[i].data(), 16);
    *count = n;
    return CORRO_OK;
}

int corro_site_count(corro_ctx *ctx, uint32_t *count) {
    if (!ctx || !count) return fail(CORRO_E_INVALID, "NULL argument");
    *count = (uint32_t)ctx->sites.size();
    return CORRO_OK;
}

// Copy a host batch into one device slab; returns device views.
static int stage_host_batch(corro_ctx *ctx, const corro_changes *in, BatchDev &bd) {
    const uint64_t n = in->n;
    struct F { const void *src; size_t elem; const void **dst; };
    const void *pk = nullptr, *tc = nullptr, *cv = nullptr, *dbv = nullptr, *cl = nullptr, *seq = nullptr,
               *site = nullptr, *v0 = nullptr, *v1 = nullptr, *vt = nullptr, *vl = nullptr, *ts = nullptr;
    F f[] = {{in->pk, 8, &pk},   {in->col_version, 8, &cv}, {in->db_version, 8, &dbv}, {in->val0, 8, &v0},
             {in->val1, 8, &v1}, {in->ts, 8, &ts},          {in->table_cid, 4, &tc},   {in->cl, 4, &cl},
             {in->seq, 4, &seq}, {in->site, 4, &site},      {in->val_type, 1, &vt},    {in->val_len, 1, &vl}};
    size_t total = 0;
    for (auto &x : f)
        if (x.src) total += ((n * x.elem + 255) / 256) * 256;
    TRY(ctx->d_in.ensure(total));
    size_t off = 0;
    for (auto &x : f) {
        if (!x.src) continue;
        uint8_t *d = ctx->d_in.as<uint8_t>() + off;
        CORRO_HIP_TRY(hipMemcpyAsync(d, x.src, n * x.elem, hipMemcpyHostToDevice, ctx->stream));
        *x.dst = d;
        off += ((n * x.elem + 255) / 256) * 256;
    }
    bd.pk = (const uint64_t *)pk;
    bd.tcid = (const uint32_t *)tc;
    bd.cv = (const int64_t *)cv;
    bd.dbv = (const int64_t *)dbv;
    bd.cl = (const uint32_t *)cl;
    bd.seq = (const uint32_t *)seq;
    bd.site = (const uint32_t *)site;
    bd.v0 = (const uint64_t *)v0;
    bd.v1 = (const uint64_t *)v1;
    bd.vt = (const uint8_t *)vt;
    bd.vl = (const uint8_t *)vl;
    bd.ts = (const uint64_t *)ts;
    return CORRO_OK;
}

static int error_from_bits(uint64_t bits) {
    if (bits & ERR_NAME) return fail(CORRO_E_UNKNOWN_COLUMN, "batch references an unknown table or cid");
    if (bits & ERR_SITE) return fail(CORRO_E_INVALID, "batch references an unregistered site ordinal");
    if (bits & ERR_RANGE)
        return fail(CORRO_E_RANGE, "causal length / sentinel col_version / db_version outside the engine encoding");
    return fail(CORRO_E_INVALID, "malformed value (type, length or NaN REAL)");
}

// One apply of a device-resident chunk (bd: n changes in application order) into the state.
// imp_buf: device impact flags of this chunk (or null). Returns with the state committed.
static int apply_chunk(corro_ctx *ctx, BatchDev bd, uint8_t *imp_buf) {
    hipStream_t s = ctx->stream;
    const uint32_t n = bd.n;
    const uint32_t B = ctx->B, log2B = ctx->log2B;
    const uint32_t nsites = (uint32_t)ctx->sites.size();
    if (bd.ts && !ctx->track_ts) {
        // timestamps start being tracked: give the current state zero timestamps
        const size_t cap_rows = ctx->d_state[ctx->cur].bytes / sizeof(Rec);
        TRY(ctx->d_state_ts[ctx->cur].ensure(std::max<size_t>(cap_rows, 1) * 8));
        CORRO_HIP_TRY(hipMemsetAsync(ctx->d_state_ts[ctx->cur].p, 0, std::max<size_t>(cap_rows, 1) * 8, s));
        ctx->track_ts = true;
    }

    // tiles: one workgroup per CU (the 128-KB LDS histogram admits one), 256 CUs
    static const uint32_t tiles_max = [] {
        const char *e = std::getenv("CORRO_HIP_TILES");  // tuning knob for experiments
        const long v = e ? std::atol(e) : 0;
        return v > 0 && v <= 4096 ? (uint32_t)v : TILES_MAX;
    }();
    uint32_t ntiles = std::max<uint32_t>(1, std::min<uint32_t>(tiles_max, (n + 4095) / 4096));
    uint32_t tile = (n + ntiles - 1) / ntiles;
    tile = (tile + HIST_THREADS - 1) / HIST_THREADS * HIST_THREADS;
    ntiles = (n + tile - 1) / tile;

    const int nxt = ctx->cur ^ 1;
    const uint64_t out_cap = ctx->state_total + 2ULL * n;
    TRY(ctx->d_hist.ensure((size_t)ntiles * B * 4));
    TRY(ctx->d_stage.ensure((size_t)n * sizeof(Rec)));
    TRY(ctx->d_state[nxt].ensure(out_cap * sizeof(Rec)));
    if (ctx->track_ts) TRY(ctx->d_state_ts[nxt].ensure(out_cap * 8));

    CORRO_HIP_TRY(hipMemsetAsync(ctx->d_bflags.p, 0, ((B + 31) / 32) * 4ULL, s));
    CORRO_HIP_TRY(hipMemsetAsync(ctx->d_misc.p, 0, 8 * 8, s));
    CORRO_HIP_TRY(hipMemsetAsync(ctx->d_dbv_batch.p, 0, (size_t)nsites * 8, s));
    if (imp_buf) CORRO_HIP_TRY(hipMemsetAsync(imp_buf, 0, n, s));

    unsigned long long *misc = ctx->d_misc.as<unsigned long long>();
    const bool prof = ctx->profiling;
    auto mark = [&](int i) {
        if (prof) (void)hipEventRecord(ctx->ev[i], s);
    };
    for (int k = 0; k < 6; k++) ctx->last_ms[k] = 0.f;
    mark(0);
    const uint32_t one_table = ctx->tables.size() == 1 ? 1u : 0u;
    hipLaunchKernelGGL(k_hist, dim3(ntiles), dim3(HIST_THREADS), (size_t)B * 4, s, bd, tile, log2B, one_table,
                       ctx->d_hist.as<uint32_t>());
    CORRO_HIP_TRY(hipGetLastError());
    mark(1);
    hipLaunchKernelGGL(k_colscan, dim3((B + 255) / 256), dim3(256), 0, s, ctx->d_hist.as<uint32_t>(), ntiles, B,
                       ctx->d_new_cnt.as<uint32_t>());
    mark(2);
    hipLaunchKernelGGL(k_plan, dim3(1), dim3(1024), 0, s, ctx->d_new_cnt.as<uint32_t>(),
                       ctx->d_state_cnt.as<uint32_t>(), B, ctx->d_stage_off.as<uint32_t>(),
                       ctx->d_out_off.as<uint64_t>());
    mark(3);
    {
        static const bool nt_stores = std::getenv("CORRO_HIP_NT") && std::atoi(std::getenv("CORRO_HIP_NT")) != 0;
        const bool plain = !bd.v1 && !bd.vt && !bd.vl;
        auto kern = plain ? (nt_stores ? k_scatter<true, true> : k_scatter<true, false>)
                          : (nt_stores ? k_scatter<false, true> : k_scatter<false, false>);
        hipLaunchKernelGGL(kern, dim3(ntiles), dim3(HIST_THREADS), (size_t)B * 4 + ((B + 31) / 32) * 4, s, bd,
                           tile, log2B, one_table, ctx->d_hist.as<uint32_t>(), ctx->d_stage_off.as<uint32_t>(),
                           ctx->d_stage.as<Rec>(), ctx->d_bflags.as<uint32_t>(),
                           ctx->d_dbv_batch.as<unsigned long long>(), nsites, ctx->d_ncols.as<uint16_t>(),
                           (uint32_t)ctx->tables.size(), misc);
    }
    CORRO_HIP_TRY(hipGetLastError());
    mark(4);

    MergeArgs a{};
    a.prior = ctx->d_state[ctx->cur].as<Rec>();
    a.prior_off = ctx->d_state_off.as<uint64_t>();
    a.prior_cnt = ctx->d_state_cnt.as<uint32_t>();
    a.prior_flags = ctx->d_state_flags.as<uint32_t>();
    a.prior_ts = ctx->track_ts && ctx->state_total ? ctx->d_state_ts[ctx->cur].as<uint64_t>() : nullptr;
    a.stage = ctx->d_stage.as<Rec>();
    a.stage_off = ctx->d_stage_off.as<uint32_t>();
    a.new_cnt = ctx->d_new_cnt.as<uint32_t>();
    a.bflags = ctx->d_bflags.as<uint32_t>();
    a.batch_ts = bd.ts;
    a.out = ctx->d_state[nxt].as<Rec>();
    a.out_ts = ctx->track_ts ? ctx->d_state_ts[nxt].as<uint64_t>() : nullptr;
    a.out_off = ctx->d_out_off.as<uint64_t>();
    a.out_cnt = ctx->d_out_cnt.as<uint32_t>();
    a.out_flags = ctx->d_out_flags.as<uint32_t>();
    a.site_rank = ctx->d_site_rank.as<uint32_t>();
    a.nsites = nsites;
    a.impact = imp_buf;
    a.misc = misc;
    a.ovf_list = ctx->d_ovf_list.as<uint32_t>();
    // CORRO_HIP_FORCE_GENERAL=1 sends every bucket through the sequential body (cross-checks)
    static const bool force_general = std::getenv("CORRO_HIP_FORCE_GENERAL") &&
                                      std::atoi(std::getenv("CORRO_HIP_FORCE_GENERAL")) != 0;
    a.force_general = force_general ? 1u : 0u;
    a.track_ts = ctx->track_ts ? 1u : 0u;
    a.state_wide = ctx->state_wide ? 1u : 0u;
    a.gen_list = ctx->d_gen_list.as<uint32_t>();
    a.wide_list = ctx->d_wide_list.as<uint32_t>();
    if (a.impact) {
        hipLaunchKernelGGL(k_merge_fast_int<true>, dim3(B), dim3(MERGE_THREADS), 0, s, a);
        CORRO_HIP_TRY(hipGetLastError());
        hipLaunchKernelGGL(k_merge_fast_wide<true>, dim3(std::min(B, LIST_GRID)), dim3(MERGE_THREADS), 0, s, a);
    } else {
        hipLaunchKernelGGL(k_merge_fast_int<false>, dim3(B), dim3(MERGE_THREADS), 0, s, a);
        CORRO_HIP_TRY(hipGetLastError());
        hipLaunchKernelGGL(k_merge_fast_wide<false>, dim3(std::min(B, LIST_GRID)), dim3(MERGE_THREADS), 0, s, a);
    }
    CORRO_HIP_TRY(hipGetLastError());
    hipLaunchKernelGGL(k_merge_gen_small, dim3(std::min(B, 4 * LIST_GRID)), dim3(GEN_SMALL_THREADS), 0, s, a, B);
    CORRO_HIP_TRY(hipGetLastError());
    hipLaunchKernelGGL(k_merge_gen_mid, dim3(std::min(B, 2 * LIST_GRID)), dim3(MERGE_THREADS), 0, s, a, B);
    CORRO_HIP_TRY(hipGetLastError());
    hipLaunchKernelGGL(k_merge_gen, dim3(std::min(B, LIST_GRID)), dim3(MERGE_THREADS), 0, s, a);
    CORRO_HIP_TRY(hipGetLastError());
    mark(5);
    CORRO_HIP_TRY(hipMemcpyAsync(ctx->h_misc, misc, 4 * 8, hipMemcpyDeviceToHost, s));
    CORRO_HIP_TRY(hipStreamSynchronize(s));
    if (ctx->h_misc[0]) return error_from_bits(ctx->h_misc[0]);
    if (prof)
        for (int i = 0; i < 5; i++) CORRO_HIP_TRY(hipEventElapsedTime(&ctx->last_ms[i], ctx->ev[i], ctx->ev[i + 1]));

    const uint64_t novf = ctx->h_misc[1];
    if (novf) TRY(run_overflow(ctx, a, novf, n, prof));
    hipLaunchKernelGGL(k_dbv_fold, dim3((nsites + 255) / 256), dim3(256), 0, s,
                       ctx->d_dbv.as<unsigned long long>(), ctx->d_dbv_batch.as<unsigned long long>(), nsites);
    CORRO_HIP_TRY(hipStreamSynchronize(s));

    // commit: the next state becomes current
    std::swap(ctx->d_state_off, ctx->d_out_off);
    std::swap(ctx->d_state_cnt, ctx->d_out_cnt);
    std::swap(ctx->d_state_flags, ctx->d_out_flags);
    ctx->cur = nxt;
    ctx->state_total = ctx->h_misc[2];
    ctx->state_epoch++;
    if (ctx->h_misc[3]) ctx->state_wide = true;
    return CORRO_OK;
}

// Changes per chunk: the bucket count sizes the merge for ~2048 records per bucket, so a larger
// batch is applied as consecutive chunks of it, in application order -- the same result as one
// apply, since the merge is a left fold over the changes (each INSERT sees the state its
// predecessors left). The whole batch is validated before the first chunk commits.
static uint64_t chunk_changes(const corro_ctx *ctx) {
    const char *e = std::getenv("CORRO_HIP_CHUNK");  // tests: force chunking of small batches
    const uint64_t env = e ? (uint64_t)std::atoll(e) : 0ULL;
    if (env) return std::max<uint64_t>(1024, env & ~1023ULL);
    return std::max<uint64_t>(1ULL << 16, (uint64_t)ctx->B * 2048ULL);
}

int corro_apply_batch(corro_ctx *ctx, const corro_changes *in, int mem, corro_apply_out *out) {
    if (!ctx || !in) return fail(CORRO_E_INVALID, "NULL argument");
    if (in->n == 0) return CORRO_OK;
    if (in->n >= (1ULL << 31)) return fail(CORRO_E_RANGE, "at most 2^31-1 changes per batch");
    if (!in->pk || !in->table_cid || !in->col_version || !in->db_version || !in->cl || !in->seq || !in->site ||
        !in->val0)
        return fail(CORRO_E_INVALID, "a required batch array is NULL");
    if (mem != CORRO_MEM_HOST && mem != CORRO_MEM_DEVICE) return fail(CORRO_E_INVALID, "bad mem kind");
    CORRO_HIP_TRY(hipSetDevice(ctx->device));
    hipStream_t s = ctx->stream;
    const uint32_t n = (uint32_t)in->n;
    const uint32_t nsites = (uint32_t)ctx->sites.size();
    if (nsites == 0) return fail(CORRO_E_INVALID, "no sites registered");

    BatchDev bd{};
    if (mem == CORRO_MEM_HOST) {
        TRY(stage_host_batch(ctx, in, bd));
    } else {
        // k_scatter reads pairs of changes with 16-B (64-bit fields) / 8-B (32-bit fields) loads
        auto misaligned = [](const void *p, uintptr_t a) { return p && ((uintptr_t)p % a) != 0; };
        if (misaligned(in->pk, 16) || misaligned(in->col_version, 16) || misaligned(in->db_version, 16) ||
            misaligned(in->val0, 16) || misaligned(in->val1, 16) || misaligned(in->table_cid, 8) ||
            misaligned(in->cl, 8) || misaligned(in->seq, 8) || misaligned(in->site, 8))
            return fail(CORRO_E_INVALID, "device batch arrays must be 16-byte (64-bit fields) / 8-byte aligned");
        bd.pk = in->pk;
        bd.tcid = in->table_cid;
        bd.cv = in->col_version;
        bd.dbv = in->db_version;
        bd.cl = in->cl;
        bd.seq = in->seq;
        bd.site = in->site;
        bd.v0 = in->val0;
        bd.v1 = in->val1;
        bd.vt = in->val_type;
        bd.vl = in->val_len;
        bd.ts = in->ts;
    }
    bd.n = n;
    // impact output: a device batch gets its flags written straight into the caller's device
    // buffer; a host batch through a device staging buffer + one copy
    const bool imp_dev = out && out->impact && mem == CORRO_MEM_DEVICE;
    if (out && out->impact && !imp_dev) TRY(ctx->d_impact.ensure(n));
    uint8_t *imp_buf = !(out && out->impact) ? nullptr : (imp_dev ? out->impact : ctx->d_impact.as<uint8_t>());

    const uint64_t chunk = chunk_changes(ctx);
    if (n > chunk) {
        CORRO_HIP_TRY(hipMemsetAsync(ctx->d_misc.p, 0, 8 * 8, s));
        hipLaunchKernelGGL(k_validate, dim3((uint32_t)std::min<uint64_t>((n + 255) / 256, 8192)), dim3(256), 0, s, bd,
                           nsites, ctx->d_ncols.as<uint16_t>(), (uint32_t)ctx->tables.size(),
                           ctx->d_misc.as<unsigned long long>());
        CORRO_HIP_TRY(hipGetLastError());
        CORRO_HIP_TRY(hipMemcpyAsync(ctx->h_misc, ctx->d_misc.p, 8, hipMemcpyDeviceToHost, s));
        CORRO_HIP_TRY(hipStreamSynchronize(s));
        if (ctx->h_misc[0]) return error_from_bits(ctx->h_misc[0]);
    }
    float ms[6] = {};
    for (uint64_t off = 0; off < n; off += chunk) {
        BatchDev c = bd;
        const uint32_t m = (uint32_t)std::min<uint64_t>(chunk, n - off);
        auto adv = [&](auto *&p) {
            if (p) p += off;
        };
        adv(c.pk), adv(c.tcid), adv(c.cv), adv(c.dbv), adv(c.cl), adv(c.seq), adv(c.site), adv(c.v0), adv(c.v1);
        adv(c.vt), adv(c.vl), adv(c.ts);
        c.n = m;
        TRY(apply_chunk(ctx, c, imp_buf ? imp_buf + off : nullptr));
        for (int k = 0; k < 6; k++) ms[k] += ctx->last_ms[k];
    }
    for (int k = 0; k < 6; k++) ctx->last_ms[k] = ms[k];
    if (out && out->impact && !imp_dev) {
        CORRO_HIP_TRY(hipMemcpyAsync(out->impact, ctx->d_impact.p, n, hipMemcpyDeviceToHost, s));
        CORRO_HIP_TRY(hipStreamSynchronize(s));
    }
    return CORRO_OK;
}

}  // extern "C"

namespace corro {
// crsql_set_db_version(site, v) for an empty complete changeset (util.rs:1040-1050)
int set_db_version(corro_ctx *ctx, uint32_t site, uint64_t version) {
    if (site >= ctx->sites.size()) return fail(CORRO_E_INVALID, "unregistered site ordinal");
    CORRO_HIP_TRY(hipSetDevice(ctx->device));
    uint64_t cur = 0;
    uint64_t *p = ctx->d_dbv.as<uint64_t>() + site;
    CORRO_HIP_TRY(hipMemcpy(&cur, p, 8, hipMemcpyDeviceToHost));
    if (version + 1 > cur) {
        const uint64_t nv = version + 1;
        CORRO_HIP_TRY(hipMemcpy(p, &nv, 8, hipMemcpyHostToDevice));
    }
    return CORRO_OK;
}
}  // namespace corro

extern "C" {

int corro_ctx_set_profiling(corro_ctx *ctx, int on) {
    if (!ctx) return fail(CORRO_E_INVALID, "NULL argument");
    ctx->profiling = on != 0;
    return CORRO_OK;
}

int corro_last_timings(corro_ctx *ctx, float *ms, uint32_t cap, uint32_t *count) {
    if (!ctx || !count || (!ms && cap)) return fail(CORRO_E_INVALID, "NULL argument");
    const uint32_t n = 9;
    for (uint32_t i = 0; i < n && i < cap; i++) ms[i] = ctx->last_ms[i];
    *count = n;
    return CORRO_OK;
}

int corro_state_count(corro_ctx *ctx, uint64_t *count) {
    if (!ctx || !count) return fail(CORRO_E_INVALID, "NULL argument");
    *count = ctx->state_total;
    return CORRO_OK;
}

int corro_state_reset(corro_ctx *ctx) {
    if (!ctx) return fail(CORRO_E_INVALID, "NULL argument");
    CORRO_HIP_TRY(hipSetDevice(ctx->device));
    CORRO_HIP_TRY(hipMemsetAsync(ctx->d_state_cnt.p, 0, ctx->B * 4ULL, ctx->stream));
    CORRO_HIP_TRY(hipMemsetAsync(ctx->d_state_off.p, 0, ctx->B * 8ULL, ctx->stream));
    CORRO_HIP_TRY(hipMemsetAsync(ctx->d_state_flags.p, 0, ctx->B * 4ULL, ctx->stream));
    CORRO_HIP_TRY(hipStreamSynchronize(ctx->stream));
    ctx->state_total = 0;
    ctx->state_epoch++;
    return CORRO_OK;
}

int corro_state_export(corro_ctx *ctx, corro_rows *o, uint64_t cap, uint64_t *written) {
    if (!ctx || !o || !written) return fail(CORRO_E_INVALID, "NULL argument");
    const uint64_t m = ctx->state_total;
    *written = 0;
    if (cap < m) return fail(CORRO_E_INVALID, "export capacity too small");
    if (m == 0) return CORRO_OK;
    CORRO_HIP_TRY(hipSetDevice(ctx->device));
    hipStream_t s = ctx->stream;
    const uint32_t B = ctx->B;
    std::vector<uint32_t> cnt(B);
    CORRO_HIP_TRY(hipMemcpy(cnt.data(), ctx->d_state_cnt.p, B * 4ULL, hipMemcpyDeviceToHost));
    std::vector<uint64_t> dense(B);
    uint64_t run = 0;
    for (uint32_t b = 0; b < B; b++) {
        dense[b] = run;
        run += cnt[b];
    }
    if (run != m) return fail(CORRO_E_DEVICE, "internal: state count mismatch");
    // device SoA: 8*6 + 4*3 + 1*2 bytes per row
    const size_t per = 8 * 7 + 4 * 3 + 2;
    TRY(ctx->d_export.ensure(m * per + B * 8 + 4096));
    uint8_t *p = ctx->d_export.as<uint8_t>();
    corro_rows d{};
    auto carve = [&](size_t elem) {
        uint8_t *q = p;
        p += ((m * elem + 255) / 256) * 256;
        return q;
    };
    d.pk = (uint64_t *)carve(8);
    d.col_version = (int64_t *)carve(8);
    d.db_version = (int64_t *)carve(8);
    d.cl = (int64_t *)carve(8);
    d.ts = (uint64_t *)carve(8);
    d.val0 = (uint64_t *)carve(8);
    d.val1 = (uint64_t *)carve(8);
    d.table_cid = (uint32_t *)carve(4);
    d.seq = (uint32_t *)carve(4);
    d.site = (uint32_t *)carve(4);
    d.val_type = (uint8_t *)carve(1);
    d.val_len = (uint8_t *)carve(1);
    uint64_t *d_dense = (uint64_t *)p;
    CORRO_HIP_TRY(hipMemcpyAsync(d_dense, dense.data(), B * 8ULL, hipMemcpyHostToDevice, s));
    const uint64_t *sts = ctx->track_ts ? ctx->d_state_ts[ctx->cur].as<uint64_t>() : nullptr;
    hipLaunchKernelGGL(k_export, dim3(B), dim3(256), 0, s, ctx->d_state[ctx->cur].as<Rec>(), sts,
                       ctx->d_state_off.as<uint64_t>(), ctx->d_state_cnt.as<uint32_t>(), d_dense, d);
    CORRO_HIP_TRY(hipGetLastError());
    struct C { void *dst; const void *src; size_t elem; } cp[] = {
        {o->pk, d.pk, 8},         {o->col_version, d.col_version, 8}, {o->db_version, d.db_version, 8},
        {o->cl, d.cl, 8},         {o->ts, d.ts, 8},                   {o->val0, d.val0, 8},
        {o->val1, d.val1, 8},     {o->table_cid, d.table_cid, 4},     {o->seq, d.seq, 4},
        {o->site, d.site, 4},     {o->val_type, d.val_type, 1},       {o->val_len, d.val_len, 1}};
    for (auto &c : cp)
        if (c.dst) CORRO_HIP_TRY(hipMemcpyAsync(c.dst, c.src, m * c.elem, hipMemcpyDeviceToHost, s));
    CORRO_HIP_TRY(hipStreamSynchronize(s));
    *written = m;
    return CORRO_OK;
}

int corro_db_versions(corro_ctx *ctx, int64_t *out, uint32_t nsites) {
    if (!ctx || (!out && nsites)) return fail(CORRO_E_INVALID, "NULL argument");
    if (nsites > ctx->sites.size()) return fail(CORRO_E_INVALID, "nsites exceeds registered sites");
    if (nsites == 0) return CORRO_OK;
    std::vector<uint64_t> v(nsites);
    CORRO_HIP_TRY(hipMemcpy(v.data(), ctx->d_dbv.p, nsites * 8ULL, hipMemcpyDeviceToHost));
    for (uint32_t i = 0; i < nsites; i++) out[i] = v[i] ? (int64_t)(v[i] - 1) : -1;
    return CORRO_OK;
}

}  // extern "C"
