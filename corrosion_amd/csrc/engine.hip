// libcorro_hip.so — context, site registry and the apply_batch pipeline (C ABI, corro_hip.h).
//
// corro_apply_batch replaces, for one `process_multiple_changes` call, the nest
//   for actor { for changeset { SAVEPOINT; for change { INSERT INTO crsql_changes; ... } } }
// of /root/reference/crates/corro-agent/src/agent/util.rs:765-884 + :1222-1262 with one batched
// device merge. Kernels: merge_kernels.h. Host bookkeeping stays with the caller.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
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

int grow_regions(corro_ctx *ctx, uint32_t new_log2S);
int grow_heap(corro_ctx *ctx, uint64_t want_records);
RowStore row_store(corro_ctx *ctx);
int affinity_convert(corro_ctx *ctx, BatchDev &bd);  // affinity.hip

// The overflow fold reduces rows to their last epoch (k_ovf_lookup's comment) unless asked not to
// (CORRO_OVF_REDUCE=0; CORRO_OVF_RIMP=0 only with impacts: A/B runs) or a table has 32 or more
// columns (the summary's cid bits cover cids < 32).
static bool ovf_reduce_ok(const corro_ctx *ctx, bool impact) {
    static const bool no_reduce = std::getenv("CORRO_OVF_REDUCE") && std::atoi(std::getenv("CORRO_OVF_REDUCE")) == 0;
    static const bool no_rimp = std::getenv("CORRO_OVF_RIMP") && std::atoi(std::getenv("CORRO_OVF_RIMP")) == 0;
    return !no_reduce && ctx->max_stride <= 32 && !(impact && no_rimp);
}

// Oversized buckets (queued by a merge round), all at once and device-wide (the phases of
// ovf_kernels.h): batch fields + row owners (one pass) -> region lookups (prior records appended, new rows
// counted; the store grows here if they do not fit, before anything is written) -> sort by (row,
// position) -> L scan -> classify -> epoch scan -> candidate keys -> sort -> argmax / group-start
// scans -> link -> walk (rows written back to the heap) -> [impacts] -> region fill counts.
static int run_overflow(corro_ctx *ctx, MergeArgs &a, uint64_t novf, uint64_t nbatch, bool prof) {
    hipStream_t s = ctx->stream;
    const uint32_t B = ctx->B;
    // readbacks land in pinned memory: async copies, one wait per group (pageable ones block per copy)
    if (!ctx->h_ovf) CORRO_HIP_TRY(hipHostMalloc((void **)&ctx->h_ovf, (8ULL * B + 32) * 4, hipHostMallocDefault));
    uint32_t *const hw = ctx->h_ovf + 8ULL * B;  // (32 readback words; hw + 8: the plan's totals, 8-B aligned)
    // the plan (k_ovf_plan): bucket offsets and row-table slices on the device, totals back
    if (novf > (uint64_t)PLAN_T * PLAN_PER) return fail(CORRO_E_RANGE, "internal: more oversized buckets than k_ovf_plan takes");
    TRY(ctx->d_ovf_plan.ensure((2ULL * B + 2) * 4 + 16 * 8 + 256));
    uint32_t *const p_koff = ctx->d_ovf_plan.as<uint32_t>(), *const p_soff = p_koff + B + 1;
    unsigned long long *const p_tot = (unsigned long long *)(((uintptr_t)(p_soff + B) + 15) & ~(uintptr_t)15);
    unsigned long long *const hq = (unsigned long long *)(hw + 8);  // (pinned: tot[0..4])
    hipLaunchKernelGGL(k_ovf_plan, dim3(1), dim3(PLAN_T), 0, s, ctx->d_ovf_list.as<uint32_t>(), ctx->d_new_cnt.as<uint32_t>(),
                       ctx->d_used.as<uint32_t>(), (uint32_t)novf, p_koff, p_soff, p_tot);
    CORRO_HIP_TRY(hipGetLastError());
    CORRO_HIP_TRY(hipMemcpyAsync(hq, p_tot, 3 * 8, hipMemcpyDeviceToHost, s));
    // CORRO_OVF_HOSTPROF=1: the host's own time between the fold's waits, to stderr (diagnostics)
    static const bool hostprof = std::getenv("CORRO_OVF_HOSTPROF") != nullptr;
    auto hp_t0 = std::chrono::steady_clock::now();
    std::string hp_line;
    auto hp = [&](const char *what) {
        if (!hostprof) return;
        const auto t = std::chrono::steady_clock::now();
        hp_line += std::string(" ") + what + "=" +
                   std::to_string(std::chrono::duration<double, std::micro>(t - hp_t0).count()).substr(0, 6);
        hp_t0 = t;
    };
    CORRO_HIP_TRY(hipStreamSynchronize(s));
    hp("wait1");
    const uint64_t Kb = hq[0], S = hq[1];
    // prior records: at most one heap row per batch row, at most the rows the oversized buckets'
    // regions hold (each at most max_stride records), at most the whole state -- the region bound
    // keeps a hot-row batch into a large state from sizing (and failing) for the whole state
    const uint64_t region_rows = hq[2];
    const uint64_t Kmax = Kb + std::min<uint64_t>(std::min<uint64_t>(ctx->state_total, region_rows * ctx->max_stride),
                                                  Kb * (uint64_t)ctx->max_stride);
    if (Kmax >= (1ULL << 31) || S >= (1ULL << 32))
        return fail(CORRO_E_RANGE, "oversized buckets hold more than 2^31 records");
    // compact positions: prior slots [0, pm), batch change i -> pm + i
    const uint32_t pm = ctx->max_stride;
    uint32_t pbits = 1;
    while ((1ULL << pbits) < pm + nbatch) pbits++;
    uint32_t rb = 1;  // record positions (< Kmax) with one spare value above them, so that ~0 sorts last
    while ((1ULL << rb) <= Kmax) rb++;
    uint32_t cid_bits = 1;
    while ((1u << cid_bits) <= ctx->max_stride - 1) cid_bits++;
    const uint32_t ckey_bits = rb + cid_bits;
    hp("koff");
    auto al = [](uint64_t x) { return (x + 255) & ~255ULL; };
    // pass 0 sizes the arrays, pass 1 carves them out of d_ovf_sort
    OvfDev d{};
    d.G = (uint32_t)novf;
    d.K = (uint32_t)Kmax;
    d.Kb = (uint32_t)Kb;
    d.cid_bits = cid_bits;
    d.pm = pm;
    d.arena = a.arena;
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
    uint8_t *rowblk = nullptr;
    CsAgg *cs_agg = nullptr, *cs_incl = nullptr;
    const uint64_t K = Kmax, R = std::max<uint64_t>(Kb, 1);
    for (int pass = 0; pass < 2; pass++) {
        bytes = 0;
        d.koff = p_koff;
        d.slot_off = p_soff;
        d.bnew = (uint32_t *)take(novf * 4);
        d.bnrec = (uint32_t *)take(novf * 4);
        d.slots = (uint32_t *)take(std::max<uint64_t>(S, 2 * K) * 4);
        uint64_t **u64s[] = {&d.pk, &d.key, &d.key_s, &d.ckey, &d.ckey_s};
        for (uint64_t **p : u64s) *p = (uint64_t *)take(K * 8);
        d.cv = (int64_t *)take(K * 8);
        d.ccv = (int64_t *)take(K * 8);
        d.qkey = (OvfKey *)take(K * sizeof(OvfKey));
        d.pkey = (OvfKey *)take((K - Kb + 1) * sizeof(OvfKey));
        uint32_t **u32s[] = {&d.tc,    &d.cl,    &d.pos,   &d.src,   &d.val,   &d.val_s, &d.rowid, &d.cl_s,
                             &d.lx,    &d.recf,  &d.epc,   &d.kind,  &d.pb,    &d.rstart, &d.rbad, &d.rnrec,
                             &d.recs,  &d.head,  &d.scid,  &d.spos,  &d.sz,    &d.ccid,  &d.csrc,  &d.cval,
                             &d.cval_s, &d.cbest, &d.cgs,  &d.nxt,   &d.fstg};
        for (uint32_t **p : u32s) *p = (uint32_t *)take(K * 4);
        uint32_t **rows[] = {&d.rowner, &d.rb, &d.rheap, &d.rprior, &d.rpoff};
        for (uint32_t **p : rows) *p = (uint32_t *)take(R * 4);
        d.rbits = (uint64_t *)take(R * 16);
        rowblk = take(R * 20 + 64);  // row summaries, laid out once the row count is known
        d.cbk = (uint32_t *)take((Kb / 64 + 2) * 32);
        if (pass == 0 && K <= ctx->ovf_temp_k) {
            temp = ctx->ovf_temp;  // (rocPRIM's temp sizes grow with n; the 64-bit sort bounds the others)
        } else if (pass == 0) {
            size_t t0 = 0, t1 = 0, t2 = 0, t3 = 0;
            TRY(ovf_sort_pairs(nullptr, &t0, nullptr, nullptr, nullptr, nullptr, d.K, 64, s));
            TRY(ovf_sort_pairs(nullptr, &t1, nullptr, nullptr, nullptr, nullptr, d.K, ckey_bits, s));
            TRY(ovf_scans(nullptr, &t2, d, 0, s));
            TRY(prim_inclusive_scan_u32(nullptr, &t3, nullptr, nullptr, d.K, s));
            size_t t4 = 0;
            TRY(ovf_scan_tiles(nullptr, &t4, d, nullptr, nullptr, (uint32_t)((K + CS_TILE - 1) / CS_TILE), s));
            temp = std::max(std::max(std::max(t0, t1), std::max(t2, t3)), t4);
            ctx->ovf_temp_k = K;
            ctx->ovf_temp = temp;
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
    hp("carve");
    CORRO_HIP_TRY(hipMemsetAsync(d.bnew, 0, novf * 4, s));
    CORRO_HIP_TRY(hipMemsetAsync(d.bnrec, 0, novf * 4, s));
    CORRO_HIP_TRY(hipMemsetAsync(d.slots, 0, S * 4, s));
    if (prof) (void)hipEventRecord(ctx->ev[6], s);
    auto grid_for = [](uint64_t n) { return dim3((uint32_t)std::max<uint64_t>(1, std::min<uint64_t>((n + 255) / 256, 8192))); };
    const dim3 blk(256), gridb = grid_for(Kb);
    auto launched = [&]() -> int {
        CORRO_HIP_TRY(hipGetLastError());
        return CORRO_OK;
    };
    // Row reduction (k_ovf_lookup's comment), with impacts in its impact form (k_ovf_keep's comment:
    // the dropped records' flags from per-row causal-length slots, the dropped candidates sorted by
    // group); off when asked (A/B runs) or when the dropped candidates' key would not fit 64 bits.
    uint32_t kbits = 1;  // (nrows <= Kb)
    while ((1ULL << kbits) < Kb) kbits++;
    const bool rimp_fits = kbits + 3 + cid_bits + pbits <= 64;
    d.reduce = ovf_reduce_ok(ctx, a.impact != nullptr) && (!a.impact || rimp_fits) ? 1u : 0u;
    d.rimp = d.reduce && a.impact ? 1u : 0u;
    static const bool split = !std::getenv("CORRO_OVF_SPLIT") || std::atoi(std::getenv("CORRO_OVF_SPLIT")) != 0;
    // fused plain form (OvfDev::fuse; CORRO_OVF_FUSE=0: the separate summary pass, A/B runs)
    static const bool no_fuse = std::getenv("CORRO_OVF_FUSE") && std::atoi(std::getenv("CORRO_OVF_FUSE")) == 0;
    d.fuse = d.reduce && !d.rimp && split && !no_fuse ? 1u : 0u;
    if (d.fuse) {
        // summaries by owner record: zero between applies (each walk clears its rows' words); a fresh
        // area, or one an apply left before its walk (an error return), is cleared here
        void *const was = ctx->d_ovf_sum.p;
        const size_t was_bytes = ctx->d_ovf_sum.bytes;  // (a regrown area may come back at the same address)
        TRY(ctx->d_ovf_sum.ensure(Kb * sizeof(OvfSum) + 256));
        if (ctx->d_ovf_sum.p != was || ctx->d_ovf_sum.bytes != was_bytes || ctx->ovf_sum_dirty)
            CORRO_HIP_TRY(hipMemsetAsync(ctx->d_ovf_sum.p, 0, ctx->d_ovf_sum.bytes, s));
        ctx->ovf_sum_dirty = true;  // (until this apply's walk has run)
        d.osum = ctx->d_ovf_sum.as<OvfSum>();
        d.cstride = ctx->max_stride;
        d.obits = 1;
        while ((1ULL << d.obits) < Kb) d.obits++;
    }
    hp("h2d");
    hipLaunchKernelGGL(k_ovf_chunkmap, grid_for((Kb + 63) / 64), blk, 0, s, a, d);
    if (d.fuse)
        hipLaunchKernelGGL(k_ovf_loadsum, dim3((uint32_t)((Kb + RS_CHUNK - 1) / RS_CHUNK)), dim3(RS_T), 0, s, a, d);
    else
        hipLaunchKernelGGL(k_ovf_loadhash, gridb, blk, 0, s, a, d);
    TRY(launched());
    // dense row ids: the row count sizes the sort's key
    TRY(prim_inclusive_scan_u32(d_temp, &temp, d.recf, d.epc, d.Kb, s));
    CORRO_HIP_TRY(hipMemcpyAsync(&hw[0], d.epc + (Kb - 1), 4, hipMemcpyDeviceToHost, s));
    hp("enq2");
    CORRO_HIP_TRY(hipStreamSynchronize(s));
    hp("wait2");
    const uint32_t nrows = hw[0];
    d.nrows = nrows;
    d.rshift = pbits;
    if (d.fuse) {  // (summaries by owner record: the per-row block holds the counters)
        d.nkeep = (uint32_t *)rowblk;
        CORRO_HIP_TRY(hipMemsetAsync(d.nkeep, 0, 16, s));
        TRY(ctx->d_ovf_rcl.ensure((uint64_t)nrows * 4 * 7 + 256));
        d.rsum = ctx->d_ovf_rcl.as<uint64_t>();
        d.rowE = reinterpret_cast<uint32_t *>(d.rsum + nrows);
        d.rlist = d.rowE + nrows;
        d.flist = d.rlist + nrows;
        d.rhb = d.flist + nrows;
        d.rclw = d.rhb + nrows;
    } else {
        uint8_t *blk = rowblk;
        d.rw1 = (uint64_t *)blk;
        d.rw2 = (uint32_t *)(blk + 8ULL * nrows);
        d.nkeep = (uint32_t *)(blk + 12ULL * nrows);
        if (d.reduce) CORRO_HIP_TRY(hipMemsetAsync(blk, 0, 12ULL * nrows + 8, s));
    }
    if (d.rimp) {  // causal-length slots (free = ~0) and their first records
        TRY(ctx->d_ovf_rcl.ensure((uint64_t)nrows * OVF_NCL * 12 + 256));
        d.rcl = ctx->d_ovf_rcl.as<uint64_t>();
        d.rclr = reinterpret_cast<uint32_t *>(d.rcl + (uint64_t)nrows * OVF_NCL);
        CORRO_HIP_TRY(hipMemsetAsync(d.rcl, 0xFF, (uint64_t)nrows * OVF_NCL * 8, s));
    }
    // every row looked up in its region; prior records counted, new rows counted per bucket (and
    // every batch record's sort key)
    d.split = split ? 1u : 0u;
    if (d.fuse)
        hipLaunchKernelGGL(k_ovf_owners, gridb, blk, 0, s, a, d);
    else
        hipLaunchKernelGGL(d.rimp ? k_ovf_lookup<true> : k_ovf_lookup<false>, dim3((uint32_t)((Kb + RS_CHUNK - 1) / RS_CHUNK)),
                           dim3(RS_T), 0, s, a, d);
    if (split) hipLaunchKernelGGL(k_ovf_rlook, grid_for(nrows), blk, 0, s, a, d);
    TRY(launched());
    TRY(prim_inclusive_scan_u32(d_temp, &temp, d.rprior, d.rpoff, nrows, s));
    CORRO_HIP_TRY(hipMemcpyAsync(&hw[0], d.rpoff + (nrows - 1), 4, hipMemcpyDeviceToHost, s));
    hipLaunchKernelGGL(k_ovf_room, dim3(1), dim3(PLAN_T), 0, s, ctx->d_ovf_list.as<uint32_t>(), ctx->d_used.as<uint32_t>(),
                       d.bnew, d.bnrec, (uint32_t)novf, p_tot);
    CORRO_HIP_TRY(hipGetLastError());
    CORRO_HIP_TRY(hipMemcpyAsync(hq + 3, p_tot + 3, 2 * 8, hipMemcpyDeviceToHost, s));
    CORRO_HIP_TRY(hipMemcpyAsync(&hw[2], ctx->d_heap_top.p, 8, hipMemcpyDeviceToHost, s));
    hp("enq3");
    CORRO_HIP_TRY(hipStreamSynchronize(s));
    hp("wait3");
    const uint32_t P = hw[0];
    const unsigned long long top = (unsigned long long)hw[2] | ((unsigned long long)hw[3] << 32);
    if (Kb + (uint64_t)P > Kmax) return fail(CORRO_E_DEVICE, "internal: overflow prior records exceed their bound");
    // room for the new rows (region fill, heap) before the walk writes anything
    const uint64_t need_heap = hq[4], want = hq[3];  // (k_ovf_room: the largest fill asked of a region)
    uint32_t need_log2S = ctx->log2S;
    while (want > ((7ULL << need_log2S) >> 3)) need_log2S++;
    if (need_log2S != ctx->log2S) TRY(grow_regions(ctx, need_log2S));
    if (top + need_heap > ctx->heap_cap) TRY(grow_heap(ctx, top + need_heap));
    a.rs = row_store(ctx);
    d.K = (uint32_t)(Kb + P);
    uint32_t rbits = 1;
    while ((1ULL << rbits) < nrows) rbits++;
    const uint32_t key_bits = rbits + pbits;
    d.rshift = pbits;
    if (key_bits > 64) return fail(CORRO_E_RANGE, "overflow sort key exceeds 64 bits");
    static const bool dbg = std::getenv("CORRO_HIP_OVF_DEBUG") != nullptr;
    if (dbg)
        fprintf(stderr, "[corro ovf] buckets %llu batch records %llu prior %u rows %u key bits %u (+%u) cand key bits %u\n",
                (unsigned long long)novf, (unsigned long long)Kb, P, nrows, key_bits, rbits, ckey_bits);
    hp("room");
    hipLaunchKernelGGL(k_ovf_pload, grid_for(nrows), blk, 0, s, a, d);
    TRY(launched());
    if (d.reduce) {
        // rows reduced to their last epoch's records (k_ovf_lookup's comment); the rest sort as before
        const uint32_t kcap = d.K;
        hipLaunchKernelGGL(d.fuse ? k_ovf_keep<true> : k_ovf_keep<false>, dim3((d.K + KEEP_CHUNK - 1) / KEEP_CHUNK),
                           dim3(KEEP_T), 0, s, a, d, kcap);
        TRY(launched());
        CORRO_HIP_TRY(hipMemcpyAsync(&hw[4], d.nkeep, 8, hipMemcpyDeviceToHost, s));
        hp("enq4");
        CORRO_HIP_TRY(hipStreamSynchronize(s));
        hp("wait4");
        const uint32_t kept = hw[4], ndc = d.rimp ? hw[5] : 0u, nc = d.fuse ? hw[5] : 0u;
        if ((kept == 0 && !d.fuse) || (uint64_t)kept + ndc + nc > kcap)
            return fail(CORRO_E_DEVICE, "internal: overflow row reduction kept no records");
        if (dbg)
            fprintf(stderr, "[corro ovf] row reduction keeps %u of %u records (%u dropped candidates, %u reduced rows' cell records)\n",
                    kept, d.K, ndc, nc);
        if (nc) {
            // fused form: the reduced rows' cells -- sorted by (owner record, cid), each cell's winner by the
            // argmax scan with the position as the last tie-break -- before the kept records' sort
            // reuses key_s / val_s / qkey / cbest
            TRY(ovf_sort_pairs(d_temp, &temp, d.ckey + (kcap - nc), d.key_s, d.cval + (kcap - nc), d.val_s, nc,
                               d.obits + cid_bits, s));
            const dim3 rgrid = grid_for(nc);
            hipLaunchKernelGGL(k_ovf_rgather, rgrid, blk, 0, s, a, d, nc, d.pb);
            TRY(launched());
            OvfDev dd = d;
            dd.ckey_s = d.key_s;
            dd.K = nc;
            dd.qpos = d.pb;
            const uint32_t ntc = (nc + CS_TILE - 1) / CS_TILE;  // <= nt
            hipLaunchKernelGGL(k_cscan_tile<true>, dim3(ntc), dim3(CS_T), 0, s, dd, cs_agg, cs_first);
            TRY(launched());
            TRY(ovf_scan_tiles(d_temp, &temp, dd, cs_agg, cs_incl, ntc, s));
            hipLaunchKernelGGL(k_cscan_fix<true>, dim3(ntc), dim3(CS_T), 0, s, dd, cs_incl, cs_first);
            TRY(launched());
        }
        // the reduced rows written now (their sentinels and slots, then their cells, one lane per cell),
        // while the cell sort's results are in key_s / val_s / cbest; the other rows' pipeline below
        // reads no heap or region word these write
        if (d.fuse) {
            void (*const walk1)(MergeArgs, OvfDev) = ctx->max_stride <= WALK_MAXC ? k_ovf_walk<true, 1> : k_ovf_walk<false, 1>;
            hipLaunchKernelGGL(walk1, grid_for(nrows), blk, 0, s, a, d);
            if (nc) hipLaunchKernelGGL(k_ovf_rcells, grid_for(nc), blk, 0, s, a, d, nc);
            TRY(launched());
        }
        if (ndc) {
            // dropped candidates (impact form): sorted by (row, slot, cid, position), running argmax by
            // group with the candidate scan's kernels, then their flags -- all before the kept records'
            // sort reuses key_s / val_s / key / qkey / cbest
            const uint32_t dbits = kbits + 3 + cid_bits + pbits;
            TRY(ovf_sort_pairs(d_temp, &temp, d.ckey + (kcap - ndc), d.key_s, d.cval + (kcap - ndc), d.val_s, ndc, dbits, s));
            const dim3 dgrid = grid_for(ndc);
            hipLaunchKernelGGL(k_ovf_dgather, dgrid, blk, 0, s, a, d, ndc, d.key_s, d.val_s, d.key, d.qkey);
            TRY(launched());
            OvfDev dd = d;  // the scan reads (ckey_s: group keys, qkey: cell keys, K, cbest)
            dd.ckey_s = d.key;
            dd.K = ndc;
            const uint32_t ntc = (ndc + CS_TILE - 1) / CS_TILE;  // <= nt
            hipLaunchKernelGGL(k_cscan_tile<false>, dim3(ntc), dim3(CS_T), 0, s, dd, cs_agg, cs_first);
            TRY(launched());
            TRY(ovf_scan_tiles(d_temp, &temp, dd, cs_agg, cs_incl, ntc, s));
            hipLaunchKernelGGL(k_cscan_fix<false>, dim3(ntc), dim3(CS_T), 0, s, dd, cs_incl, cs_first);
            hipLaunchKernelGGL(k_ovf_dimp, dgrid, blk, 0, s, a, d, ndc, d.key, d.val_s, d.qkey, d.cbest);
            TRY(launched());
        }
        d.K = kept;
        if (kept) TRY(ovf_sort_pairs(d_temp, &temp, d.ckey, d.key_s, d.cval, d.val_s, d.K, key_bits, s));
    } else {
        TRY(ovf_sort_pairs(d_temp, &temp, d.key, d.key_s, d.val, d.val_s, d.K, key_bits, s));
    }
    d.ncand = 0;
    if (d.K) {  // (fused form: none when every row reduced)
    const dim3 grid = grid_for(d.K);
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
    TRY(prim_inclusive_scan_u32(d_temp, &temp, d.slots, d.slots + d.K, d.K, s));
    CORRO_HIP_TRY(hipMemcpyAsync(&hw[5], d.slots + d.K + (d.K - 1), 4, hipMemcpyDeviceToHost, s));
    hp("enq5");
    CORRO_HIP_TRY(hipStreamSynchronize(s));
    hp("wait5");
    const uint32_t ncand = hw[5];
    hipLaunchKernelGGL(k_ovf_ccompact, grid, blk, 0, s, d);
    TRY(launched());
    if (ncand) TRY(ovf_sort_pairs(d_temp, &temp, d.key, d.ckey_s, d.val, d.cval_s, ncand, ckey_bits, s));
    if (ncand < d.K) CORRO_HIP_TRY(hipMemsetAsync(d.ckey_s + ncand, 0xFF, (d.K - ncand) * 8ULL, s));
    if (dbg) fprintf(stderr, "[corro ovf] candidates %u\n", ncand);
    d.ncand = ncand;
    const dim3 cgrid = grid_for(ncand);
    hipLaunchKernelGGL(k_ovf_cgather, cgrid, blk, 0, s, a, d);
    TRY(launched());
    if (ncand) {
        const uint32_t ntc = (ncand + CS_TILE - 1) / CS_TILE;  // <= nt
        hipLaunchKernelGGL(k_cscan_tile<false>, dim3(ntc), dim3(CS_T), 0, s, d, cs_agg, cs_first);
        TRY(launched());
        TRY(ovf_scan_tiles(d_temp, &temp, d, cs_agg, cs_incl, ntc, s));
        hipLaunchKernelGGL(k_cscan_fix<false>, dim3(ntc), dim3(CS_T), 0, s, d, cs_incl, cs_first);
    }
    TRY(launched());
    if (ncand && a.impact) TRY(ovf_scans(d_temp, &temp, d, 2, s));  // (group starts: impacts only)
    hipLaunchKernelGGL(k_ovf_link, cgrid, blk, 0, s, d);
    }
    // carried cells in registers when no table has WALK_MAXC or more columns (cids 1..ncols)
    const bool wreg = ctx->max_stride <= WALK_MAXC;
    using WalkK = void (*)(MergeArgs, OvfDev);
    const WalkK walk0 = wreg ? k_ovf_walk<true, 0> : k_ovf_walk<false, 0>;
    const WalkK walk2 = wreg ? k_ovf_walk<true, 2> : k_ovf_walk<false, 2>;
    if (d.fuse) {  // the rows that are not reduced (the reduced ones were written after the cell scan)
        hipLaunchKernelGGL(walk2, grid_for(nrows), blk, 0, s, a, d);
    } else {
        hipLaunchKernelGGL(walk0, grid_for(nrows), blk, 0, s, a, d);
    }
    if (a.impact && d.ncand) hipLaunchKernelGGL(k_ovf_impacts, grid_for(d.ncand), blk, 0, s, a, d);
    hipLaunchKernelGGL(k_ovf_finish, grid_for(novf), blk, 0, s, a, d);
    TRY(launched());
    hp("enq6");
    if (hostprof) fprintf(stderr, "[corro ovf host us]%s\n", hp_line.c_str());
    if (prof) (void)hipEventRecord(ctx->ev[7], s);
    CORRO_HIP_TRY(hipStreamSynchronize(s));
    if (d.fuse) ctx->ovf_sum_dirty = false;  // (the walk cleared every row's summary words)
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
    CORRO_HIP_TRY(hipHostMalloc((void **)&ctx->h_misc, MISC_WORDS * sizeof(uint64_t), hipHostMallocDefault));
    for (auto &e : ctx->ev) CORRO_HIP_TRY(hipEventCreate(&e));
    const size_t lds_max = 160 * 1024;
    for (const void *f : {(const void *)k_hist<8>, (const void *)k_hist<16>, (const void *)k_hist<32>,
                          (const void *)k_hist<16, true>, (const void *)k_hist<16, false, true>})
        CORRO_HIP_TRY(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_max));
    for (const void *f : {(const void *)k_scatter<true, true>, (const void *)k_scatter<true, false>,
                          (const void *)k_scatter<true, false, 8>,
                          (const void *)k_scatter<false, true>, (const void *)k_scatter<false, false>})
        CORRO_HIP_TRY(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_max));
    return CORRO_OK;
}

}  // extern "C"

// Initial row-store sizes from the capacity hint (expected changes per apply): regions at about half
// fill for hint/16 rows, a heap of hint/2 records; both grow on demand.
static int store_alloc(corro_ctx *ctx, uint64_t capacity_hint) {
    const uint32_t B = ctx->B;
    const uint64_t rows = std::max<uint64_t>(1024, capacity_hint / 16);  // (~4 changes per row, half of them new)
    uint32_t lg = 4;
    // (region entries are named by 32-bit indices: B << log2S stays <= 2^31)
    while (((uint64_t)B << lg) < 2 * rows && lg < 20 && ((uint64_t)B << (lg + 1)) <= (1ULL << 31)) lg++;
    ctx->log2S = lg;
    TRY(ctx->d_ent.ensure(((size_t)B << lg) * sizeof(RowEnt)));
    TRY(ctx->d_used.ensure(B * 4ULL));
    TRY(ctx->d_gen.ensure(B * 4ULL));
    TRY(ctx->d_heap_top.ensure(8));
    ctx->heap_cap = std::min<uint64_t>(1ULL << 31, std::max<uint64_t>(1ULL << 16, capacity_hint / 2));
    TRY(ctx->d_heap.ensure(ctx->heap_cap * sizeof(Rec)));
    return CORRO_OK;
}

static int store_clear(corro_ctx *ctx) {
    hipStream_t s = ctx->stream;
    CORRO_HIP_TRY(hipMemsetAsync(ctx->d_ent.p, 0, ((size_t)ctx->B << ctx->log2S) * sizeof(RowEnt), s));
    CORRO_HIP_TRY(hipMemsetAsync(ctx->d_used.p, 0, ctx->B * 4ULL, s));
    CORRO_HIP_TRY(hipMemsetAsync(ctx->d_gen.p, 0, ctx->B * 4ULL, s));
    CORRO_HIP_TRY(hipMemsetAsync(ctx->d_heap_top.p, 0, 8, s));  // (stream-ordered before the next apply)
    if (ctx->d_touch_n.p) CORRO_HIP_TRY(hipMemsetAsync(ctx->d_touch_n.p, 0, 8, s));
    ctx->touch_bound = 0;
    ctx->state_total = 0;
    ctx->state_rows = 0;
    ctx->arena_top = 0;
    ctx->state_epoch++;
    ctx->poisoned = false;
    return CORRO_OK;
}

namespace corro {
RowStore row_store(corro_ctx *ctx) {
    RowStore rs{};
    rs.ent = ctx->d_ent.as<RowEnt>();
    rs.used = ctx->d_used.as<uint32_t>();
    rs.gen = ctx->d_gen.as<uint32_t>();
    rs.heap = ctx->d_heap.as<Rec>();
    rs.heap_ts = ctx->track_ts ? ctx->d_heap_ts.as<uint64_t>() : nullptr;
    rs.heap_top = ctx->d_heap_top.as<unsigned long long>();
    rs.heap_cap = ctx->heap_cap;
    rs.log2S = ctx->log2S;
    rs.fill = (uint32_t)((7ULL << ctx->log2S) >> 3);
    rs.stride = ctx->d_stride.as<uint16_t>();
    return rs;
}

// Room for `add` more bytes in the value arena (contents kept: handles are offsets into it).
static constexpr uint64_t ARENA_MAX = 1ULL << 40;  // a value handle holds a 40-bit offset
int arena_reserve(corro_ctx *ctx, uint64_t add) {
    const uint64_t need = ctx->arena_top + add;
    if (need > ARENA_MAX) return fail(CORRO_E_RANGE, "value arena would exceed 2^40 bytes");
    if (need <= ctx->d_arena.bytes && ctx->d_arena.p) return CORRO_OK;
    DevBuf nb;
    TRY(nb.ensure(std::max<uint64_t>(need + (need >> 1), 1ULL << 20)));
    if (ctx->arena_top)
        CORRO_HIP_TRY(hipMemcpyAsync(nb.p, ctx->d_arena.p, ctx->arena_top, hipMemcpyDeviceToDevice, ctx->stream));
    CORRO_HIP_TRY(hipStreamSynchronize(ctx->stream));
    ctx->d_arena.release();
    ctx->d_arena = nb;
    nb.p = nullptr;
    return CORRO_OK;
}

// Regions rehashed to 2^new_log2S slots (between merge rounds / before an overflow walk: no apply
// writes are in flight). Entry indices change; heap indices and presence bits move with the rows.
int grow_regions(corro_ctx *ctx, uint32_t new_log2S) {
    if (new_log2S <= ctx->log2S) return CORRO_OK;
    ctx->metrics.region_growths++;
    if (new_log2S > 26 || ((uint64_t)ctx->B << new_log2S) > (1ULL << 31))
        return fail(CORRO_E_NOMEM, "row store regions would exceed 2^31 entries");
    hipStream_t s = ctx->stream;
    DevBuf nb;
    TRY(nb.ensure(((size_t)ctx->B << new_log2S) * sizeof(RowEnt)));
    CORRO_HIP_TRY(hipMemsetAsync(nb.p, 0, ((size_t)ctx->B << new_log2S) * sizeof(RowEnt), s));
    const uint32_t old_log2S = ctx->log2S;
    DevBuf old = ctx->d_ent;
    ctx->d_ent = nb;
    nb.p = nullptr;
    ctx->log2S = new_log2S;
    hipLaunchKernelGGL(k_rehash, dim3(ctx->B), dim3(256), 0, s, old.as<RowEnt>(), old_log2S, row_store(ctx));
    CORRO_HIP_TRY(hipGetLastError());
    CORRO_HIP_TRY(hipStreamSynchronize(s));
    old.release();
    return CORRO_OK;
}

// Heap reallocated to hold at least want_records (doubling), contents copied.
int grow_heap(corro_ctx *ctx, uint64_t want_records) {
    if (want_records <= ctx->heap_cap) return CORRO_OK;
    ctx->metrics.heap_growths++;
    uint64_t cap = ctx->heap_cap;
    while (cap < want_records) cap *= 2;
    // (heap indices stay below 2^31: the fast bodies mark a new row's heap offset with the top bit)
    if (cap > (1ULL << 31)) cap = 1ULL << 31;
    if (cap < want_records) return fail(CORRO_E_RANGE, "row store heap would exceed 2^31 records");
    if (ctx->heap_limit && cap > ctx->heap_limit) {
        if (want_records > ctx->heap_limit)
            return fail(CORRO_E_NOMEM, "row store heap would exceed the context's store limit");
        cap = ctx->heap_limit;
    }
    hipStream_t s = ctx->stream;
    unsigned long long top = 0;
    CORRO_HIP_TRY(hipMemcpyAsync(&top, ctx->d_heap_top.p, 8, hipMemcpyDeviceToHost, s));
    CORRO_HIP_TRY(hipStreamSynchronize(s));
    top = std::min<unsigned long long>(top, ctx->heap_cap);
    DevBuf nh;
    TRY(nh.ensure(cap * sizeof(Rec)));
    CORRO_HIP_TRY(hipMemcpyAsync(nh.p, ctx->d_heap.p, top * sizeof(Rec), hipMemcpyDeviceToDevice, s));
    DevBuf nts;
    if (ctx->track_ts) {
        TRY(nts.ensure(cap * 8));
        CORRO_HIP_TRY(hipMemsetAsync(nts.p, 0, cap * 8, s));
        CORRO_HIP_TRY(hipMemcpyAsync(nts.p, ctx->d_heap_ts.p, top * 8, hipMemcpyDeviceToDevice, s));
    }
    CORRO_HIP_TRY(hipStreamSynchronize(s));
    ctx->d_heap.release();
    ctx->d_heap = nh;
    nh.p = nullptr;
    if (ctx->track_ts) {
        ctx->d_heap_ts.release();
        ctx->d_heap_ts = nts;
        nts.p = nullptr;
    }
    ctx->heap_cap = cap;
    return CORRO_OK;
}
}  // namespace corro

extern "C" {

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
        if (tables[t].ncols > MAX_COLS) {
            delete ctx;
            return fail(CORRO_E_RANGE, "at most 127 non-pk columns per table (the row store's presence bits)");
        }
        Table tb;
        tb.name = tables[t].name;
        for (uint32_t c = 0; c < tables[t].ncols; c++) tb.cols.emplace_back(tables[t].col_names[c]);
        ctx->max_stride = std::max<uint32_t>(ctx->max_stride, tables[t].ncols + 1);
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
    rc = ctx->d_new_cnt.ensure(B * 4ULL);
    if (!rc) rc = ctx->d_stage_off.ensure(B * 4ULL);
    if (!rc) rc = ctx->d_bflags.ensure(((B + 31) / 32) * 4ULL);
    if (!rc) rc = ctx->d_misc.ensure(MISC_WORDS * 8);
    if (!rc) rc = ctx->d_ovf_list.ensure(B * 4ULL);
    if (!rc) rc = ctx->d_gen_list.ensure(3 * B * 4ULL);
    if (!rc) rc = ctx->d_wide_list.ensure(B * 4ULL);
    if (!rc) rc = ctx->d_defer.ensure(B * 4ULL);
    if (!rc) rc = ctx->d_relist.ensure(B * 4ULL);
    if (!rc) rc = store_alloc(ctx, capacity_hint);
    if (rc != CORRO_OK) {
        corro_ctx_destroy(ctx);
        return rc;
    }
    {
        std::vector<uint16_t> ncols(ctx->tables.size() + 1, 0), stride(ctx->tables.size() + 1, 1);
        for (size_t t = 0; t < ctx->tables.size(); t++) {
            ncols[t] = (uint16_t)ctx->tables[t].cols.size();
            stride[t] = (uint16_t)(ctx->tables[t].cols.size() + 1);
        }
        rc = ctx->d_ncols.ensure(ncols.size() * 2);
        if (!rc) rc = ctx->d_stride.ensure(stride.size() * 2);
        if (rc == CORRO_OK &&
            (hipMemcpy(ctx->d_ncols.p, ncols.data(), ncols.size() * 2, hipMemcpyHostToDevice) != hipSuccess ||
             hipMemcpy(ctx->d_stride.p, stride.data(), stride.size() * 2, hipMemcpyHostToDevice) != hipSuccess))
            rc = fail(CORRO_E_DEVICE, "upload of the schema failed");
        if (rc == CORRO_OK) rc = store_clear(ctx);
        if (rc == CORRO_OK) rc = prims_warm(ctx);
        // (the agent's pinned host areas for a call of the hinted size: ~64 changes per changeset)
        if (rc == CORRO_OK) rc = agent_dev_reserve(ctx, std::max<uint64_t>(4096, capacity_hint / 64));
        if (rc != CORRO_OK) {
            corro_ctx_destroy(ctx);
            return rc;
        }
    }
    *out = ctx;
    return CORRO_OK;
}

void corro_ctx_destroy(corro_ctx *ctx) {
    if (!ctx) return;
    if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
    DevBuf *bufs[] = {&ctx->d_site_rank, &ctx->d_dbv, &ctx->d_dbv_batch, &ctx->d_ent, &ctx->d_used, &ctx->d_gen,
                      &ctx->d_heap, &ctx->d_heap_ts, &ctx->d_heap_top, &ctx->d_stride, &ctx->d_defer,
                      &ctx->d_relist, &ctx->d_dense, &ctx->d_dense_ts, &ctx->d_dense_view, &ctx->d_in,
                      &ctx->d_hist, &ctx->d_new_cnt, &ctx->d_stage_off, &ctx->d_bflags, &ctx->d_stage,
                      &ctx->d_misc, &ctx->d_ovf_list, &ctx->d_gen_list, &ctx->d_wide_list, &ctx->d_fast_of, &ctx->d_ovf_sort, &ctx->d_ovf_rcl, &ctx->d_ovf_sum, &ctx->d_ovf_plan, &ctx->d_setdbv,
                      &ctx->d_scan_tmp, &ctx->d_impact, &ctx->d_export, &ctx->d_needs, &ctx->d_needs1,
                      &ctx->d_xidx, &ctx->d_xout, &ctx->d_wire, &ctx->d_wire_schema, &ctx->d_wire_sites,
                      &ctx->d_ncols, &ctx->d_part, &ctx->d_arena, &ctx->d_aff, &ctx->d_affflag,
                      &ctx->d_agent_in, &ctx->d_agent_batch, &ctx->d_agent_spans, &ctx->d_agent_imp,
                      &ctx->d_agent_out, &ctx->d_agent_aux, &ctx->d_agent_fetch, &ctx->d_agent_aux2, &ctx->d_touch, &ctx->d_touch_n, &ctx->d_touch_stamp, &ctx->d_touch_tmp,
                      &ctx->d_aff_conv, &ctx->d_aff_vals, &ctx->d_gaps_big, &ctx->d_agent_hdr, &ctx->d_wire_map,
                      &ctx->d_hdr_stage, &ctx->d_pm_ts};
    for (DevBuf *b : bufs) b->release();
    ctx->d_pkdir.release();
    ctx->d_pk_scratch.release();
    ctx->d_pk_bad.release();
    ctx->d_part_var.release();
    for (PkTable &t : ctx->pk) {
        t.d_off.release();
        t.d_bytes.release();
        t.d_hash.release();
        t.d_slots.release();
    }
    if (ctx->h_misc) (void)hipHostFree(ctx->h_misc);
    if (ctx->h_ovf) (void)hipHostFree(ctx->h_ovf);
    if (ctx->h_agent) (void)hipHostFree(ctx->h_agent);
    if (ctx->h_hdr) (void)hipHostFree(ctx->h_hdr);
    if (ctx->h_hfetch) (void)hipHostFree(ctx->h_hfetch);
    if (ctx->h_pool) (void)hipHostFree(ctx->h_pool);
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
               *site = nullptr, *v0 = nullptr, *v1 = nullptr, *vt = nullptr, *vl = nullptr, *ts = nullptr,
               *voff = nullptr, *vsz = nullptr;
    F f[] = {{in->pk, 8, &pk},   {in->col_version, 8, &cv}, {in->db_version, 8, &dbv}, {in->val0, 8, &v0},
             {in->val1, 8, &v1}, {in->ts, 8, &ts},          {in->table_cid, 4, &tc},   {in->cl, 4, &cl},
             {in->seq, 4, &seq}, {in->site, 4, &site},      {in->val_type, 1, &vt},    {in->val_len, 1, &vl},
             {in->val_off, 8, &voff}, {in->val_size, 4, &vsz}};
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
    bd.voff = (const uint64_t *)voff;
    bd.vsz = (const uint32_t *)vsz;
    return CORRO_OK;
}

// position mode, value words in the batch: ts[p] = input ts of application position p
static __global__ void k_ts_by_pos(const uint64_t *__restrict__ in_ts, const uint32_t *__restrict__ src_of, uint64_t n,
                                   uint64_t *__restrict__ out) {
    for (uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; p < n; p += (uint64_t)gridDim.x * blockDim.x)
        out[p] = in_ts[src_of[p] & 0x7FFFFFFFu];  // (bit 31: span head flag)
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
// Merge rounds: the first covers every bucket; a bucket that could not take its new rows (region
// or heap full) deferred itself before writing anything, the store grows, and the next round
// merges only the deferred buckets.
static int apply_chunk(corro_ctx *ctx, BatchDev bd, uint8_t *imp_buf) {
    hipStream_t s = ctx->stream;
    const uint32_t n = bd.n;
    const uint32_t B = ctx->B, log2B = ctx->log2B;
    const uint32_t nsites = (uint32_t)ctx->sites.size();
    if (bd.ts && !ctx->track_ts) {
        // timestamps start being tracked: the state so far has zero timestamps
        TRY(ctx->d_heap_ts.ensure(ctx->heap_cap * 8));
        CORRO_HIP_TRY(hipMemsetAsync(ctx->d_heap_ts.p, 0, ctx->heap_cap * 8, s));
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

    TRY(ctx->d_hist.ensure((size_t)ntiles * B * 4));
    TRY(ctx->d_stage.ensure((size_t)n * sizeof(Rec)));
    // (bucket general bits, misc counters and per-site db_version maxima are zeroed by k_hist)
    ApplyZero z{ctx->d_bflags.as<uint32_t>(), ctx->d_misc.as<unsigned long long>(),
                ctx->d_dbv_batch.as<unsigned long long>(), (B + 31) / 32, (uint32_t)MISC_WORDS, nsites};
    // (0: every body stores only the nonzero flags -- in Zipf-hot batches most changes are no-ops,
    // and each flag store is a random byte)
    if (imp_buf) CORRO_HIP_TRY(hipMemsetAsync(imp_buf, 0, bd.ap ? ctx->pm_n : n, s));

    unsigned long long *misc = ctx->d_misc.as<unsigned long long>();
    const bool prof = ctx->profiling;
    auto mark = [&](int i) {
        if (prof) (void)hipEventRecord(ctx->ev[i], s);
    };
    for (int k = 0; k < 6; k++) ctx->last_ms[k] = 0.f;
    mark(0);
    const uint32_t one_table = ctx->tables.size() == 1 ? 1u : 0u;
    // changes per lane in flight (CORRO_HIST_U: A/B knob)
    static const int hist_u = std::getenv("CORRO_HIST_U") ? std::atoi(std::getenv("CORRO_HIST_U")) : 16;
    using HistK = void (*)(BatchDev, uint32_t, uint32_t, uint32_t, uint32_t *, ApplyZero);
    const HistK hk = bd.slot_rec ? k_hist<16, true>
                     : !one_table ? (HistK)k_hist<16, false, true>
                     : hist_u == 8 ? k_hist<8> : hist_u == 32 ? k_hist<32> : k_hist<16>;
    hipLaunchKernelGGL(hk, dim3(ntiles), dim3(HIST_THREADS), (size_t)B * 4, s, bd, tile, log2B, one_table,
                       ctx->d_hist.as<uint32_t>(), z);
    CORRO_HIP_TRY(hipGetLastError());
    mark(1);
    hipLaunchKernelGGL(k_colscan, dim3((B + 255) / 256), dim3(256), 0, s, ctx->d_hist.as<uint32_t>(), ntiles, B,
                       ctx->d_new_cnt.as<uint32_t>());
    mark(2);
    hipLaunchKernelGGL(k_plan, dim3(1), dim3(1024), 0, s, ctx->d_new_cnt.as<uint32_t>(), B,
                       ctx->d_stage_off.as<uint32_t>());
    mark(3);
    {
        static const bool nt_stores = std::getenv("CORRO_HIP_NT") && std::atoi(std::getenv("CORRO_HIP_NT")) != 0;
        const bool plain = !bd.v1 && !bd.vt && !bd.vl && !bd.conv;
        if (bd.ts_v1 && !plain) return fail(CORRO_E_INVALID, "internal: ts_v1 on a batch with value words");
        static const bool scat8 = std::getenv("CORRO_SCAT_U") && std::atoi(std::getenv("CORRO_SCAT_U")) == 8;  // A/B knob
        auto kern = plain ? (nt_stores ? k_scatter<true, true> : scat8 ? k_scatter<true, false, 8> : k_scatter<true, false>)
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
    a.stage = ctx->d_stage.as<Rec>();
    a.stage_off = ctx->d_stage_off.as<uint32_t>();
    a.new_cnt = ctx->d_new_cnt.as<uint32_t>();
    a.bflags = ctx->d_bflags.as<uint32_t>();
    a.batch_ts = bd.ts;
    a.rs = row_store(ctx);
    a.site_rank = ctx->d_site_rank.as<uint32_t>();
    a.nsites = nsites;
    a.impact = imp_buf;
    a.misc = misc;
    a.ovf_list = ctx->d_ovf_list.as<uint32_t>();
    a.gen_list = ctx->d_gen_list.as<uint32_t>();
    a.wide_list = ctx->d_wide_list.as<uint32_t>();
    a.defer_list = ctx->d_defer.as<uint32_t>();
    a.bucket_list = nullptr;
    a.B = B;
    // CORRO_HIP_FORCE_GENERAL=1 sends every bucket through the sequential body (cross-checks)
    static const bool force_general = std::getenv("CORRO_HIP_FORCE_GENERAL") &&
                                      std::atoi(std::getenv("CORRO_HIP_FORCE_GENERAL")) != 0;
    a.force_general = force_general ? 1u : 0u;
    // General buckets of more than 512 records go to the device-wide fold when the batch is large
    // enough that the fold runs anyway and no impacts are asked for (the fold then reduces hot rows):
    // config 5 12.3 -> 11.5 ms (256 / 1024 / all: 12.4 / 11.8 / 12.8, profiles/history/r03_c5_gen_ovf_min.log).
    // A small batch keeps its LDS bodies (one bucket past 512 records would pull in the whole fold).
    static const char *gom = std::getenv("CORRO_GEN_OVF_MIN");  // (A/B knob)
    a.gen_ovf_min = gom ? (uint32_t)std::atoi(gom)
                        : (ovf_reduce_ok(ctx, imp_buf != nullptr) && bd.n >= (1ULL << 24) ? 512u : 0xFFFFFFFFu);
    a.track_ts = ctx->track_ts ? 1u : 0u;
    a.state_wide = ctx->state_wide ? 1u : 0u;
    a.arena = ctx->d_arena.as<uint8_t>();
    a.touch = ctx->track_touched ? ctx->d_touch.as<uint4>() : nullptr;
    a.touch_n = ctx->track_touched ? ctx->d_touch_n.as<unsigned long long>() : nullptr;
    if (bd.conv) {  // converted values: incoming changes compare by their raw values
        a.raw = bd;
        a.raw.arena = ctx->d_arena.as<uint8_t>();
    }
    a.pos_src = bd.ap ? ctx->pm_src : nullptr;
    a.ts_v1 = bd.ts_v1;
    uint32_t nblocks = B;
    float merge_ms = 0.f, ovf_ms = 0.f;
    // A batch that failed validation (k_scatter's error bits in misc[0]) is never merged: the merge
    // and the db_version fold check the bits on the device, so the non-impact path needs no host
    // round trip between the scatter and the merge (the impact path reads MISC_CVBIG first: it picks
    // one of two kernels). The region fill sum and the db_version fold are launched behind the first
    // merge round; the host reads everything once, and re-runs the sum only after further rounds.
    if (a.impact) {
        CORRO_HIP_TRY(hipMemcpyAsync(ctx->h_misc, misc, (MISC_CVBIG + 1) * 8, hipMemcpyDeviceToHost, s));
        CORRO_HIP_TRY(hipStreamSynchronize(s));
        if (ctx->h_misc[0]) return error_from_bits(ctx->h_misc[0]);
    }
    bool extra_rounds = false;
    for (int round = 0;; round++) {
        if (round > 40) return fail(CORRO_E_NOMEM, "internal: the row store did not take the batch's rows");
        mark(4);
        // triage in one pass, queue appends per wave (k_triage); the fast body's workgroups skip it
        static const bool no_triage = std::getenv("CORRO_TRIAGE") && std::atoi(std::getenv("CORRO_TRIAGE")) == 0;
        if (!no_triage) {
            TRY(ctx->d_fast_of.ensure(B + 256));
            a.fast_of = ctx->d_fast_of.as<uint8_t>();
            hipLaunchKernelGGL(k_triage, dim3(std::min<uint32_t>((nblocks + 255) / 256, 1024)), dim3(256), 0, s, a, nblocks,
                               ctx->d_fast_of.as<uint8_t>());
            CORRO_HIP_TRY(hipGetLastError());
        }
        if (a.impact) {
            // the packed two-word keys of the INTEGER impact body: col_versions < 2^15, <= 2^16 sites
            const bool packed = ctx->h_misc[MISC_CVBIG] == 0 && nsites <= 65536;
            auto kern = packed ? k_merge_fast_int<true, true> : k_merge_fast_int<true, false>;
            hipLaunchKernelGGL(kern, dim3(nblocks), dim3(FAST_T), 0, s, a);
            CORRO_HIP_TRY(hipGetLastError());
            hipLaunchKernelGGL(k_merge_fast_wide<true>, dim3(std::min(nblocks, LIST_GRID)), dim3(FAST_T), 0, s, a);
        } else {
            hipLaunchKernelGGL(k_merge_fast_int<false>, dim3(nblocks), dim3(FAST_T), 0, s, a);
            CORRO_HIP_TRY(hipGetLastError());
            hipLaunchKernelGGL(k_merge_fast_wide<false>, dim3(std::min(nblocks, LIST_GRID)), dim3(FAST_T), 0, s, a);
        }
        CORRO_HIP_TRY(hipGetLastError());
        hipLaunchKernelGGL(k_merge_gen_small, dim3(std::min(nblocks, 4 * LIST_GRID)), dim3(GEN_SMALL_THREADS), 0, s, a);
        CORRO_HIP_TRY(hipGetLastError());
        hipLaunchKernelGGL(k_merge_gen_mid, dim3(std::min(nblocks, 2 * LIST_GRID)), dim3(MERGE_THREADS), 0, s, a);
        CORRO_HIP_TRY(hipGetLastError());
        hipLaunchKernelGGL(k_merge_gen, dim3(std::min(nblocks, LIST_GRID)), dim3(MERGE_THREADS), 0, s, a);
        CORRO_HIP_TRY(hipGetLastError());
        mark(5);
        if (round == 0) {
            hipLaunchKernelGGL(k_dbv_fold, dim3((nsites + 255) / 256), dim3(256), 0, s,
                               ctx->d_dbv.as<unsigned long long>(), ctx->d_dbv_batch.as<unsigned long long>(), nsites,
                               (const unsigned long long *)misc);
            CORRO_HIP_TRY(hipMemsetAsync(misc + MISC_ROWS, 0, 8, s));
            hipLaunchKernelGGL(k_sum_used, dim3(1), dim3(1024), 0, s, ctx->d_used.as<uint32_t>(), B, misc);
        }
        CORRO_HIP_TRY(hipMemcpyAsync(ctx->h_misc, misc, MISC_WORDS * 8, hipMemcpyDeviceToHost, s));
        CORRO_HIP_TRY(hipStreamSynchronize(s));
        if (round == 0) {
            if (ctx->h_misc[0]) return error_from_bits(ctx->h_misc[0]);  // (nothing merged)
            ctx->apply_wrote = true;  // from here on a failure leaves the state part-merged
            if (prof)
                for (int i = 0; i < 4; i++) CORRO_HIP_TRY(hipEventElapsedTime(&ctx->last_ms[i], ctx->ev[i], ctx->ev[i + 1]));
        }
        if (prof) {
            float ms = 0.f;
            CORRO_HIP_TRY(hipEventElapsedTime(&ms, ctx->ev[4], ctx->ev[5]));
            merge_ms += ms;
        }
        const uint64_t novf = ctx->h_misc[MISC_OVF];
        if (novf) {
            extra_rounds = true;
            TRY(run_overflow(ctx, a, novf, n, prof));
            ctx->metrics.overflow_rounds++;
            ovf_ms += ctx->last_ms[5];
        }
        const uint64_t ndefer = ctx->h_misc[MISC_DEFER];
        if (!ndefer) break;
        extra_rounds = true;
        // grow what ran out, then merge the deferred buckets again
        const uint64_t why = ctx->h_misc[MISC_DEFER_WHY];
        ctx->metrics.deferred_rounds++;
        if (why & DEFER_REGION) TRY(grow_regions(ctx, ctx->log2S + 1));
        if (why & DEFER_HEAP) {
            unsigned long long top = 0;
            CORRO_HIP_TRY(hipMemcpy(&top, ctx->d_heap_top.p, 8, hipMemcpyDeviceToHost));
            TRY(grow_heap(ctx, std::max<uint64_t>(ctx->heap_cap * 2, top + (top >> 2))));
        }
        CORRO_HIP_TRY(hipMemcpyAsync(ctx->d_relist.p, ctx->d_defer.p, ndefer * 4, hipMemcpyDeviceToDevice, s));
        for (int w : {MISC_OVF, MISC_GEN, MISC_WIDEQ, MISC_GEN_SMALL, MISC_GEN_MID, MISC_DEFER, MISC_DEFER_WHY})
            CORRO_HIP_TRY(hipMemsetAsync(misc + w, 0, 8, s));
        a.rs = row_store(ctx);
        a.bucket_list = ctx->d_relist.as<uint32_t>();
        nblocks = (uint32_t)ndefer;
    }
    if (prof) {
        ctx->last_ms[4] = merge_ms;
        ctx->last_ms[5] = ovf_ms;
    }
    if (extra_rounds) {  // the overflow fold / deferred rounds changed the region fills
        CORRO_HIP_TRY(hipMemsetAsync(misc + MISC_ROWS, 0, 8, s));
        hipLaunchKernelGGL(k_sum_used, dim3(1), dim3(1024), 0, s, ctx->d_used.as<uint32_t>(), B, misc);
        CORRO_HIP_TRY(hipMemcpyAsync(ctx->h_misc, misc, MISC_WORDS * 8, hipMemcpyDeviceToHost, s));
        CORRO_HIP_TRY(hipStreamSynchronize(s));
    }
    ctx->state_total += ctx->h_misc[MISC_LIVE];  // (a signed delta in two's complement)
    ctx->state_rows = ctx->h_misc[MISC_ROWS];
#if CORRO_DIAG & 256
    fprintf(stderr, "DIAG impact phases (us per bucket; packed body: loads claims rows counts place walk region winners): %.3f %.3f %.3f %.3f %.3f %.3f %.3f %.3f\n",
            ctx->h_misc[MISC_DIAG] / 100.0 / B, ctx->h_misc[MISC_DIAG + 1] / 100.0 / B,
            ctx->h_misc[MISC_DIAG + 2] / 100.0 / B, ctx->h_misc[MISC_DIAG + 3] / 100.0 / B,
            ctx->h_misc[MISC_DIAG + 4] / 100.0 / B, ctx->h_misc[MISC_DIAG + 5] / 100.0 / B,
            ctx->h_misc[MISC_DIAG + 6] / 100.0 / B, ctx->h_misc[MISC_DIAG + 7] / 100.0 / B);
#endif
#if CORRO_DIAG & 64
    fprintf(stderr, "DIAG phases (us per bucket): load %.3f claims %.3f rows_count %.3f stage1 %.3f stages %.3f fast_rows %.3f winners %.3f publish %.3f\n",
            ctx->h_misc[MISC_DIAG] / 100.0 / B, ctx->h_misc[MISC_DIAG + 1] / 100.0 / B,
            ctx->h_misc[MISC_DIAG + 6] / 100.0 / B, ctx->h_misc[MISC_DIAG + 7] / 100.0 / B,
            ctx->h_misc[MISC_DIAG + 2] / 100.0 / B, ctx->h_misc[MISC_DIAG + 3] / 100.0 / B,
            ctx->h_misc[MISC_DIAG + 4] / 100.0 / B, ctx->h_misc[MISC_DIAG + 5] / 100.0 / B);
#endif
    ctx->state_epoch++;
    if (ctx->h_misc[MISC_WIDE]) ctx->state_wide = true;
    // keep the regions' average fill at most 5/8 for the next batch (rows, not clock records: a
    // row's cells share one entry); growth takes them back to at most half
    const uint64_t slots = (uint64_t)B << ctx->log2S;
    if (ctx->state_rows * 8 > slots * 5) {
        uint32_t lg = ctx->log2S;
        while (((uint64_t)B << lg) / 2 < ctx->state_rows && lg < 26 && ((uint64_t)B << (lg + 1)) <= (1ULL << 31)) lg++;
        TRY(grow_regions(ctx, lg));
    }
    return CORRO_OK;
}

// Changes per chunk: the bucket count sizes the merge for ~2048 records per bucket, so a larger
// batch is applied as consecutive chunks of it, in application order -- the same result as one
// apply, since the merge is a left fold over the changes (each INSERT sees the state its
// predecessors left). The whole batch is validated before the first chunk commits.
uint64_t corro_detail_chunk_changes(const corro_ctx *ctx) {
    const char *e = std::getenv("CORRO_HIP_CHUNK");  // tests: force chunking of small batches
    const uint64_t env = e ? (uint64_t)std::atoll(e) : 0ULL;
    if (env) return std::max<uint64_t>(1024, env & ~1023ULL);
    return std::max<uint64_t>(1ULL << 16, (uint64_t)ctx->B * 2048ULL);
}

// Room in the touched-row list for a batch of n changes (at most n rows): the bound grows by n per
// apply; when it would pass the capacity the exact count is read and the list regrown (contents kept).
static int touch_reserve(corro_ctx *ctx, uint64_t n) {
    if (!ctx->d_touch_n.p) {
        TRY(ctx->d_touch_n.ensure(8));
        CORRO_HIP_TRY(hipMemsetAsync(ctx->d_touch_n.p, 0, 8, ctx->stream));
    }
    if (ctx->touch_bound + n > ctx->touch_cap) {
        unsigned long long cur = 0;
        CORRO_HIP_TRY(hipMemcpyAsync(&cur, ctx->d_touch_n.p, 8, hipMemcpyDeviceToHost, ctx->stream));
        CORRO_HIP_TRY(hipStreamSynchronize(ctx->stream));
        ctx->touch_bound = cur;
        if (cur + n > ctx->touch_cap) {
            const uint64_t cap = std::max<uint64_t>(cur + n, std::min<uint64_t>(2 * ctx->touch_cap, cur + 4 * n));
            DevBuf nb;
            TRY(nb.ensure(cap * 16));
            if (cur) CORRO_HIP_TRY(hipMemcpyAsync(nb.p, ctx->d_touch.p, cur * 16, hipMemcpyDeviceToDevice, ctx->stream));
            CORRO_HIP_TRY(hipStreamSynchronize(ctx->stream));
            ctx->d_touch.release();
            ctx->d_touch = nb;
            nb.p = nullptr;
            ctx->touch_cap = cap;
        }
    }
    ctx->touch_bound += n;
    return CORRO_OK;
}

static int apply_batch_impl(corro_ctx *ctx, const corro_changes *in, int mem, corro_apply_out *out);
static const char *poisoned_msg =
    "context poisoned: an earlier apply failed after it began writing the state; call corro_state_reset";

int corro_apply_batch(corro_ctx *ctx, const corro_changes *in, int mem, corro_apply_out *out) {
    if (!ctx || !in) return fail(CORRO_E_INVALID, "NULL argument");
    if (ctx->poisoned) return fail(CORRO_E_DEVICE, poisoned_msg);
    if (in->n == 0) return CORRO_OK;
    if (fault_armed("apply")) return fail(CORRO_E_NOMEM, "injected fault (CORRO_FAULT): apply");
    const auto t0 = std::chrono::steady_clock::now();
    ctx->apply_wrote = false;
    const int rc = apply_batch_impl(ctx, in, mem, out);
    if (rc != CORRO_OK && ctx->apply_wrote) {
        // the merge had begun writing: the state is no longer the pre-call state
        ctx->poisoned = true;
        corro::set_error(corro_last_error() + std::string(" (mid-apply: the context is poisoned until corro_state_reset)"));
    }
    if (rc == CORRO_OK) {
        corro_metrics &m = ctx->metrics;
        m.applies++;
        m.changes += in->n;
        m.max_batch = std::max<uint64_t>(m.max_batch, in->n);
        m.apply_seconds += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    }
    return rc;
}

static int apply_batch_impl(corro_ctx *ctx, const corro_changes *in, int mem, corro_apply_out *out) {
    if (in->n >= (1ULL << 31)) return fail(CORRO_E_RANGE, "at most 2^31-1 changes per batch");
    if (!ctx->slot_rec && (!in->pk || !in->table_cid || !in->col_version || !in->db_version || !in->cl || !in->seq ||
                           !in->site || !in->val0))
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
        bd.voff = in->val_off;
        bd.vsz = in->val_size;
    }
    bd.n = n;
    if (ctx->slot_rec) {  // slot mode (corro_apply_slots): positions = slot indices (chunk-relative)
        bd.slot_rec = static_cast<const SlotRec *>(ctx->slot_rec);
        bd.slot_cnt = ctx->slot_cnt;
        bd.slot_cap = ctx->slot_cap;
        bd.slot_nsrc = ctx->slot_nsrc;
        bd.slot_over = ctx->slot_over;
    }
    // (a slot layout -- corro_apply_mapped -- may pass the chunk size by its padding: one chunk still)
    const uint64_t chunk_cap = corro_detail_chunk_changes(ctx) +
                               (ctx->pm_slack || ctx->slot_rec ? corro_detail_chunk_changes(ctx) / 4 : 0);
    if (ctx->pm_ap) {  // position mode (agent): one chunk, per-position ts
        if (mem != CORRO_MEM_DEVICE || n > chunk_cap)
            return fail(CORRO_E_INVALID, "internal: position mode needs one device-resident chunk");
        bd.ap = ctx->pm_ap;
        // (positions [0, pm_n) cover every input change; a mapped apply's skips are anywhere)
        bd.ap_all = ctx->pm_n == n && !ctx->pm_slack ? 1u : 0u;
        // per-position timestamps (pm_ts), else the input's own per-change ones (by input index)
        bd.ts = ctx->pm_ts ? ctx->pm_ts : in->ts;
        bd.ts_pos = ctx->pm_ts ? 1u : 0u;
    }
    // long values: the batch's value bytes are appended to the arena once; every chunk's changes
    // name their bytes relative to that base. A failed batch leaves them unreferenced.
    if (in->val_off) {
        if (!in->val_size || !in->val_type || !in->val_len || (in->val_data_len && !in->val_data))
            return fail(CORRO_E_INVALID, "long values need val_size, val_type, val_len and val_data");
        TRY(arena_reserve(ctx, in->val_data_len));
        if (in->val_data_len)
            CORRO_HIP_TRY(hipMemcpyAsync(ctx->d_arena.as<uint8_t>() + ctx->arena_top, in->val_data, in->val_data_len,
                                         mem == CORRO_MEM_HOST ? hipMemcpyHostToDevice : hipMemcpyDeviceToDevice, s));
        bd.arena = ctx->d_arena.as<uint8_t>();
        bd.lbase = ctx->arena_top;
        bd.ldata = in->val_data_len;
        // (claimed before the first chunk: a chunk that commits may reference them)
        ctx->arena_top = (ctx->arena_top + in->val_data_len + 7) & ~7ULL;
    }
    // impact output: a device batch gets its flags written straight into the caller's device
    // buffer; a host batch through a device staging buffer + one copy
    const bool imp_dev = out && out->impact && mem == CORRO_MEM_DEVICE;
    if (out && out->impact && !imp_dev) TRY(ctx->d_impact.ensure(n));
    uint8_t *imp_buf = !(out && out->impact) ? nullptr : (imp_dev ? out->impact : ctx->d_impact.as<uint8_t>());

    TRY(affinity_convert(ctx, bd));
    // INTEGER-only batch: the scatter stages each change's ts in its record's v1 word (BatchDev::ts_v1;
    // CORRO_TS_V1=0 keeps the per-position ts array, A/B). Otherwise ts must be per position: a
    // position-mode batch that brought its input's per-change ts gets them gathered into that order.
    static const bool no_ts_v1 = std::getenv("CORRO_TS_V1") && std::atoi(std::getenv("CORRO_TS_V1")) == 0;
    const bool plain = !bd.v1 && !bd.vt && !bd.vl && !bd.conv;
    static const bool no_ts_pair = std::getenv("CORRO_TS_PAIR") && std::atoi(std::getenv("CORRO_TS_PAIR")) == 0;  // (A/B)
    bd.ts_v1 = bd.ts && plain && !no_ts_v1 ? 1u : 0u;
    // (chunks start at multiples of the chunk size, a multiple of 1024 changes: alignment carries over)
    if (bd.ts_v1 && !no_ts_pair && ((uintptr_t)bd.ts % 16) == 0) bd.ts_v1 |= 2u;
    if (bd.ap && bd.ts && !bd.ts_pos && !bd.ts_v1) {
        if (!ctx->pm_src) return fail(CORRO_E_INVALID, "internal: position mode without a position -> input map");
        TRY(ctx->d_pm_ts.ensure(ctx->pm_n * 8 + 8));
        hipLaunchKernelGGL(k_ts_by_pos, dim3((uint32_t)std::min<uint64_t>((ctx->pm_n + 255) / 256, 8192)), dim3(256), 0,
                           ctx->stream, bd.ts, ctx->pm_src, ctx->pm_n, ctx->d_pm_ts.as<uint64_t>());
        CORRO_HIP_TRY(hipGetLastError());
        bd.ts = ctx->d_pm_ts.as<uint64_t>();
        bd.ts_pos = 1;
    }
    if (ctx->track_touched) TRY(touch_reserve(ctx, n));
    // (a slot layout carries its padding: up to a quarter more slots than applied records, one chunk still)
    const uint64_t chunk = ctx->pm_ap ? std::max<uint64_t>(n, 1) : ctx->slot_rec ? chunk_cap : corro_detail_chunk_changes(ctx);
    // (slot mode: corro_partition_slots validated the records it packed and marks a failed batch's
    // counts, so the layout needs no validation pass before its first chunk commits)
    if (n > chunk && !bd.slot_rec) {
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
        adv(c.vt), adv(c.vl), adv(c.ts), adv(c.voff), adv(c.vsz);
        adv(c.conv), adv(c.cv0), adv(c.cv1), adv(c.cmeta), adv(c.slot_rec);
        c.slot_base = (uint32_t)off;
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

// The received slots of the stream-ordered exchange merged where they lie: k_hist / k_scatter read the
// 48-B records themselves (BatchDev slot mode), so the receiver runs no unpack pass.
int corro_apply_slots(corro_ctx *ctx, const void *recs, uint32_t nsrc, uint64_t cap, const uint64_t *src_counts_dev,
                      corro_apply_out *out, uint32_t *overflow_dev) {
    if (!ctx || !recs || !src_counts_dev) return fail(CORRO_E_INVALID, "NULL argument");
    if (nsrc == 0 || nsrc > 64) return fail(CORRO_E_RANGE, "1..64 source ranks");
    if (cap == 0 || (uint64_t)nsrc * cap >= (1ULL << 31)) return fail(CORRO_E_RANGE, "slots: nsrc * cap < 2^31 records");
    if ((uintptr_t)recs % 16) return fail(CORRO_E_INVALID, "slot records must be 16-byte aligned");
    if (ctx->pm_ap || ctx->slot_rec) return fail(CORRO_E_INVALID, "a position map is already set on this context");
    if (ctx->aff_any) return fail(CORRO_E_INVALID, "slots carry INTEGER values: no column affinity may convert them");
    if (fault_armed("apply_slots")) return fail(CORRO_E_NOMEM, "injected fault (CORRO_FAULT): apply_slots");
    corro_changes in{};
    in.n = (uint64_t)nsrc * cap;
    ctx->slot_rec = recs;
    ctx->slot_cnt = src_counts_dev;
    ctx->slot_cap = (uint32_t)cap;
    ctx->slot_nsrc = nsrc;
    ctx->slot_over = overflow_dev;
    const int rc = corro_apply_batch(ctx, &in, CORRO_MEM_DEVICE, out);
    ctx->slot_rec = nullptr;
    ctx->slot_cnt = nullptr;
    ctx->slot_over = nullptr;
    return rc;
}

int corro_apply_mapped(corro_ctx *ctx, const corro_changes *in, const uint32_t *ap, corro_apply_out *out) {
    if (!ctx || !in || !ap) return fail(CORRO_E_INVALID, "NULL argument");
    if (ctx->pm_ap) return fail(CORRO_E_INVALID, "a position map is already set on this context");
    // position mode with position = index: skipped changes are not applied, the rest in index order
    ctx->pm_ap = ap;
    ctx->pm_src = nullptr;
    ctx->pm_ts = in->ts;
    ctx->pm_n = in->n;
    ctx->pm_slack = true;
    const int rc = corro_apply_batch(ctx, in, CORRO_MEM_DEVICE, out);
    ctx->pm_ap = nullptr;
    ctx->pm_ts = nullptr;
    ctx->pm_n = 0;
    ctx->pm_slack = false;
    return rc;
}

}  // extern "C"

namespace corro {
// The state's clock records as one dense array (+ ts), split into pseudo-buckets of 4096 records
// for the extraction index's per-bucket kernels; rebuilt once per state epoch.
int state_dense_view(corro_ctx *ctx, DenseView &v) {
    const uint64_t m = ctx->state_total;
    const uint32_t chunk = 4096;
    const uint32_t nb = (uint32_t)std::max<uint64_t>(1, (m + chunk - 1) / chunk);
    hipStream_t s = ctx->stream;
    if (ctx->dense_epoch != ctx->state_epoch) {
        TRY(ctx->d_dense.ensure(std::max<uint64_t>(m, 1) * sizeof(Rec)));
        if (ctx->track_ts) TRY(ctx->d_dense_ts.ensure(std::max<uint64_t>(m, 1) * 8));
        TRY(ctx->d_dense_view.ensure(nb * 12ULL + 256));
        std::vector<uint64_t> off(nb);
        std::vector<uint32_t> cnt(nb);
        for (uint32_t b = 0; b < nb; b++) {
            off[b] = (uint64_t)b * chunk;
            cnt[b] = (uint32_t)std::min<uint64_t>(chunk, m - std::min<uint64_t>(m, off[b]));
        }
        uint8_t *p = ctx->d_dense_view.as<uint8_t>();
        CORRO_HIP_TRY(hipMemcpyAsync(p, off.data(), nb * 8ULL, hipMemcpyHostToDevice, s));
        CORRO_HIP_TRY(hipMemcpyAsync(p + nb * 8ULL, cnt.data(), nb * 4ULL, hipMemcpyHostToDevice, s));
        unsigned long long *c = (unsigned long long *)(p + ((nb * 12ULL + 7) / 8) * 8);
        CORRO_HIP_TRY(hipMemsetAsync(c, 0, 8, s));
        const uint64_t nent = (uint64_t)ctx->B << ctx->log2S;
        if (m)
            hipLaunchKernelGGL(k_materialize, dim3((uint32_t)std::min<uint64_t>((nent + 255) / 256, 8192)), dim3(256),
                               0, s, row_store(ctx), nent, c, ctx->d_dense.as<Rec>(),
                               ctx->track_ts ? ctx->d_dense_ts.as<uint64_t>() : nullptr);
        CORRO_HIP_TRY(hipGetLastError());
        CORRO_HIP_TRY(hipStreamSynchronize(s));
        ctx->dense_epoch = ctx->state_epoch;
    }
    uint8_t *p = ctx->d_dense_view.as<uint8_t>();
    v.st = ctx->d_dense.as<Rec>();
    v.ts = ctx->track_ts ? ctx->d_dense_ts.as<uint64_t>() : nullptr;
    v.off = (const uint64_t *)p;
    v.cnt = (const uint32_t *)(p + nb * 8ULL);
    v.nb = nb;
    return CORRO_OK;
}

// crsql_set_db_version(site, v) for an empty complete changeset (util.rs:1040-1050)
// crsql_set_db_version for many (site, version) pairs at once: the per-site maxima on the host, one
// atomicMax per site on the device (d_dbv holds version + 1), queued on the context's stream
static __global__ void k_set_dbv(const uint64_t *__restrict__ sv, uint32_t n, unsigned long long *__restrict__ dbv) {
    for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k < n; k += gridDim.x * blockDim.x)
        atomicMax(&dbv[(uint32_t)(sv[2 * k])], (unsigned long long)sv[2 * k + 1]);
}

int set_db_versions(corro_ctx *ctx, const std::vector<std::pair<uint32_t, uint64_t>> &sv) {
    if (sv.empty()) return CORRO_OK;
    std::vector<uint64_t> best(ctx->sites.size(), 0);
    for (const auto &[site, v] : sv) {
        if (site >= ctx->sites.size()) return fail(CORRO_E_INVALID, "unregistered site ordinal");
        best[site] = std::max<uint64_t>(best[site], v + 1);
    }
    std::vector<uint64_t> flat;
    for (uint32_t t = 0; t < best.size(); t++)
        if (best[t]) flat.insert(flat.end(), {(uint64_t)t, best[t]});
    const uint32_t n = (uint32_t)(flat.size() / 2);
    CORRO_HIP_TRY(hipSetDevice(ctx->device));
    TRY(ctx->d_setdbv.ensure(flat.size() * 8 + 256));
    hipStream_t s = ctx->stream;
    CORRO_HIP_TRY(hipMemcpyAsync(ctx->d_setdbv.p, flat.data(), flat.size() * 8, hipMemcpyHostToDevice, s));
    hipLaunchKernelGGL(k_set_dbv, dim3((n + 255) / 256), dim3(256), 0, s, ctx->d_setdbv.as<uint64_t>(), n,
                       ctx->d_dbv.as<unsigned long long>());
    CORRO_HIP_TRY(hipGetLastError());
    ctx->dbv_writes++;
    CORRO_HIP_TRY(hipStreamSynchronize(s));  // (the host vector is the copy's source)
    return CORRO_OK;
}

uint64_t ctx_write_mark(const corro_ctx *ctx) { return ctx->metrics.applies + ctx->dbv_writes; }

bool ctx_poisoned(const corro_ctx *ctx) { return ctx->poisoned; }

void ctx_poison(corro_ctx *ctx, const char *why) {
    if (ctx->poisoned) return;
    ctx->poisoned = true;
    set_error(corro_last_error() + std::string(why));
}

int set_db_version(corro_ctx *ctx, uint32_t site, uint64_t version) {
    if (site >= ctx->sites.size()) return fail(CORRO_E_INVALID, "unregistered site ordinal");
    CORRO_HIP_TRY(hipSetDevice(ctx->device));
    uint64_t cur = 0;
    uint64_t *p = ctx->d_dbv.as<uint64_t>() + site;
    CORRO_HIP_TRY(hipMemcpy(&cur, p, 8, hipMemcpyDeviceToHost));
    if (version + 1 > cur) {
        const uint64_t nv = version + 1;
        ctx->dbv_writes++;
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

int corro_ctx_metrics(corro_ctx *ctx, corro_metrics *out) {
    if (!ctx || !out) return fail(CORRO_E_INVALID, "NULL argument");
    *out = ctx->metrics;
    out->state_rows = ctx->state_rows;
    out->state_records = ctx->state_total;
    out->arena_bytes = ctx->arena_top;
    out->aff_sensitive = ctx->metrics.aff_sensitive;
    return CORRO_OK;
}

}  // extern "C"

void corro_detail_add_committed(corro_ctx *ctx, const uint64_t *counts, size_t n) {
    if (ctx->committed.size() < ctx->tables.size()) ctx->committed.resize(ctx->tables.size(), 0);
    for (size_t t = 0; t < n && t < ctx->committed.size(); t++) ctx->committed[t] += counts[t];
}

extern "C" {

int corro_table_committed(corro_ctx *ctx, uint32_t table, uint64_t *count) {
    if (!ctx || !count) return fail(CORRO_E_INVALID, "NULL argument");
    if (table >= ctx->tables.size()) return fail(CORRO_E_UNKNOWN_TABLE, "no such table");
    *count = table < ctx->committed.size() ? ctx->committed[table] : 0;
    return CORRO_OK;
}

int corro_state_reset(corro_ctx *ctx) {
    if (!ctx) return fail(CORRO_E_INVALID, "NULL argument");
    CORRO_HIP_TRY(hipSetDevice(ctx->device));
    return store_clear(ctx);
}

int corro_state_export(corro_ctx *ctx, corro_rows *o, uint64_t cap, uint64_t *written) {
    if (!ctx || !o || !written) return fail(CORRO_E_INVALID, "NULL argument");
    if (ctx->poisoned) return fail(CORRO_E_DEVICE, poisoned_msg);
    const uint64_t m = ctx->state_total;
    *written = 0;
    if (cap < m) return fail(CORRO_E_INVALID, "export capacity too small");
    if (m == 0) return CORRO_OK;
    CORRO_HIP_TRY(hipSetDevice(ctx->device));
    hipStream_t s = ctx->stream;
    // device SoA: 8*7 + 4*3 + 1*2 bytes per row
    const size_t per = 8 * 7 + 4 * 3 + 2;
    TRY(ctx->d_export.ensure(m * per + 13 * 256 + 256));
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
    unsigned long long *cnt = (unsigned long long *)p;
    CORRO_HIP_TRY(hipMemsetAsync(cnt, 0, 8, s));
    const uint64_t nent = (uint64_t)ctx->B << ctx->log2S;
    hipLaunchKernelGGL(k_export, dim3((uint32_t)std::min<uint64_t>((nent + 255) / 256, 8192)), dim3(256), 0, s,
                       row_store(ctx), nent, cnt, d);
    CORRO_HIP_TRY(hipGetLastError());
    unsigned long long got = 0;
    CORRO_HIP_TRY(hipMemcpyAsync(&got, cnt, 8, hipMemcpyDeviceToHost, s));
    CORRO_HIP_TRY(hipStreamSynchronize(s));
    if (got != m) return fail(CORRO_E_DEVICE, "internal: state count mismatch");
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

}  // extern "C"

// value i's bytes (handle = offset << 24 | length) to out + off[i]: one workgroup per value
static __global__ void k_gather_values(const uint8_t *__restrict__ arena, const uint64_t *__restrict__ handles,
                                       const uint64_t *__restrict__ off, uint64_t n, uint8_t *__restrict__ out) {
    for (uint64_t i = blockIdx.x; i < n; i += gridDim.x) {
        const uint64_t h = handles[i], src = h >> 24, len = h & 0xFFFFFFu, dst = off[i];
        for (uint64_t k = threadIdx.x; k < len; k += blockDim.x) out[dst + k] = arena[src + k];
    }
}

extern "C" {

int corro_value_bytes(corro_ctx *ctx, const uint64_t *handles, uint64_t n, uint8_t *bytes, uint64_t cap,
                      uint64_t *out_off) {
    if (!ctx || !out_off || (n && !handles) || (cap && !bytes)) return fail(CORRO_E_INVALID, "NULL argument");
    out_off[0] = 0;
    for (uint64_t i = 0; i < n; i++) {
        const uint64_t src = handles[i] >> 24, len = handles[i] & 0xFFFFFFu;
        if (src + len > ctx->arena_top) return fail(CORRO_E_INVALID, "value handle outside the value arena");
        out_off[i + 1] = out_off[i] + len;
    }
    const uint64_t total = out_off[n];
    if (total > cap) return fail(CORRO_E_RANGE, "value bytes exceed cap");
    if (total == 0) return CORRO_OK;
    CORRO_HIP_TRY(hipSetDevice(ctx->device));
    hipStream_t s = ctx->stream;
    DevBuf &tmp = ctx->d_export;  // (scratch shared with corro_state_export)
    TRY(tmp.ensure(16 * n + total + 256));
    uint64_t *dh = tmp.as<uint64_t>(), *doff = dh + n;
    uint8_t *dout = reinterpret_cast<uint8_t *>(doff + n);
    CORRO_HIP_TRY(hipMemcpyAsync(dh, handles, 8 * n, hipMemcpyHostToDevice, s));
    CORRO_HIP_TRY(hipMemcpyAsync(doff, out_off, 8 * n, hipMemcpyHostToDevice, s));
    hipLaunchKernelGGL(k_gather_values, dim3((uint32_t)std::min<uint64_t>(n, 4096)), dim3(256), 0, s,
                       ctx->d_arena.as<uint8_t>(), dh, doff, n, dout);
    CORRO_HIP_TRY(hipGetLastError());
    CORRO_HIP_TRY(hipMemcpyAsync(bytes, dout, total, hipMemcpyDeviceToHost, s));
    CORRO_HIP_TRY(hipStreamSynchronize(s));
    return CORRO_OK;
}

int corro_ctx_track_touched(corro_ctx *ctx, int on) {
    if (!ctx) return fail(CORRO_E_INVALID, "NULL argument");
    CORRO_HIP_TRY(hipSetDevice(ctx->device));
    ctx->track_touched = on != 0;
    TRY(ctx->d_touch_n.ensure(8));
    CORRO_HIP_TRY(hipMemsetAsync(ctx->d_touch_n.p, 0, 8, ctx->stream));
    CORRO_HIP_TRY(hipStreamSynchronize(ctx->stream));
    ctx->touch_bound = 0;
    return CORRO_OK;
}

int corro_ctx_set_store_limit(corro_ctx *ctx, uint64_t max_heap_records) {
    if (!ctx) return fail(CORRO_E_INVALID, "NULL argument");
    ctx->heap_limit = max_heap_records;
    return CORRO_OK;
}

int corro_state_export_touched(corro_ctx *ctx, corro_rows *o, uint64_t cap, uint64_t *written) {
    if (!ctx || !o || !written) return fail(CORRO_E_INVALID, "NULL argument");
    *written = 0;
    if (ctx->poisoned) return fail(CORRO_E_DEVICE, poisoned_msg);
    if (!ctx->track_touched) return fail(CORRO_E_INVALID, "touched-row tracking is off (corro_ctx_track_touched)");
    CORRO_HIP_TRY(hipSetDevice(ctx->device));
    hipStream_t s = ctx->stream;
    unsigned long long m = 0;
    CORRO_HIP_TRY(hipMemcpyAsync(&m, ctx->d_touch_n.p, 8, hipMemcpyDeviceToHost, s));
    CORRO_HIP_TRY(hipStreamSynchronize(s));
    if (m == 0) return CORRO_OK;
    if (m * (uint64_t)ctx->max_stride >= (1ULL << 32))
        return fail(CORRO_E_RANGE, "touched rows exceed one export (2^32 clock rows): export after every apply");
    // dedup stamps per region entry: reallocated (zeroed) when the regions changed size
    const uint64_t nent = (uint64_t)ctx->B << ctx->log2S;
    if (ctx->touch_stamp_n != nent || ++ctx->touch_epoch == 0) {
        TRY(ctx->d_touch_stamp.ensure(nent * 4));
        CORRO_HIP_TRY(hipMemsetAsync(ctx->d_touch_stamp.p, 0, nent * 4, s));
        ctx->touch_stamp_n = nent;
        ctx->touch_epoch = 1;
    }
    size_t temp = 0;
    TRY(prim_inclusive_scan_u32(nullptr, &temp, nullptr, nullptr, (uint32_t)m, s));
    const size_t col = ((m * 4 + 255) / 256) * 256;
    TRY(ctx->d_touch_tmp.ensure(3 * col + temp + 256));
    uint32_t *ent = ctx->d_touch_tmp.as<uint32_t>();
    uint32_t *cnt = (uint32_t *)((uint8_t *)ent + col), *incl = (uint32_t *)((uint8_t *)ent + 2 * col);
    void *tmp = (uint8_t *)ent + 3 * col;
    const dim3 grid((uint32_t)std::min<uint64_t>((m + 255) / 256, 8192));
    hipLaunchKernelGGL(k_touch_count, grid, dim3(256), 0, s, row_store(ctx), ctx->log2B, ctx->d_touch.as<uint4>(), m,
                       ctx->d_touch_stamp.as<uint32_t>(), ctx->touch_epoch, ent, cnt);
    CORRO_HIP_TRY(hipGetLastError());
    TRY(prim_inclusive_scan_u32(tmp, &temp, cnt, incl, (uint32_t)m, s));
    uint32_t total = 0;
    CORRO_HIP_TRY(hipMemcpyAsync(&total, incl + (m - 1), 4, hipMemcpyDeviceToHost, s));
    CORRO_HIP_TRY(hipStreamSynchronize(s));
    if (total > cap) {  // the list is kept: a retry with room exports the same rows
        *written = total;
        return fail(CORRO_E_RANGE, "touched rows exceed cap (*written = the row count)");
    }
    const size_t per = 8 * 7 + 4 * 3 + 2;
    TRY(ctx->d_export.ensure((uint64_t)total * per + 13 * 256 + 256));
    uint8_t *p = ctx->d_export.as<uint8_t>();
    corro_rows d{};
    auto carve = [&](size_t elem) {
        uint8_t *q = p;
        p += (((uint64_t)total * elem + 255) / 256) * 256;
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
    hipLaunchKernelGGL(k_touch_rows, grid, dim3(256), 0, s, row_store(ctx), ent, cnt, incl, m, d);
    CORRO_HIP_TRY(hipGetLastError());
    struct C { void *dst; const void *src; size_t elem; } cp[] = {
        {o->pk, d.pk, 8},         {o->col_version, d.col_version, 8}, {o->db_version, d.db_version, 8},
        {o->cl, d.cl, 8},         {o->ts, d.ts, 8},                   {o->val0, d.val0, 8},
        {o->val1, d.val1, 8},     {o->table_cid, d.table_cid, 4},     {o->seq, d.seq, 4},
        {o->site, d.site, 4},     {o->val_type, d.val_type, 1},       {o->val_len, d.val_len, 1}};
    for (auto &c : cp)
        if (c.dst && total) CORRO_HIP_TRY(hipMemcpyAsync(c.dst, c.src, (uint64_t)total * c.elem, hipMemcpyDeviceToHost, s));
    CORRO_HIP_TRY(hipMemsetAsync(ctx->d_touch_n.p, 0, 8, s));
    CORRO_HIP_TRY(hipStreamSynchronize(s));
    ctx->touch_bound = 0;
    *written = total;
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
