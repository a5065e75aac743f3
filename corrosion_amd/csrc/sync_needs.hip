// Batched SyncStateV1::compute_available_needs (/root/reference/crates/corro-types/src/sync.rs:127-249)
// over CSR (node-pair, actor) entries: one lane per entry, two passes (count, fill).
//
// Per entry, with `holes` = their need ranges ∪ {their partial versions}:
//   haves = {1..=head} − holes                                   (sync.rs:141-162)
//   Full(r ∩ h) for every our-need range r, for every maximal haves range h overlapping r,
//     in our range order, ascending inside each                   (sync.rs:164-174)
//   for every our partial (v, seqs):                              (sync.rs:176-226)
//     v ∈ haves                -> Partial(v, seqs)
//     else they have partial v -> Partial(v, seqs ∩ ({0..=max end} − their seqs)) if non-empty
//   Full(our_head+1..=head) if head > our_head, Full(1..=head) if we have no head (sync.rs:229-245)
// "maximal haves range" is realised by a sweep that jumps over holes, so no set is materialised.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <string>
#include <vector>

#include "internal.h"

namespace corro {

struct SyncDev {
    uint64_t n;
    const uint64_t *their_head;
    const int64_t *our_head;
    const uint64_t *tn_off, *tn_start, *tn_end;
    const uint64_t *tp_off, *tp_ver;
    const uint64_t *tps_off, *tps_start, *tps_end;
    const uint64_t *on_off, *on_start, *on_end;
    const uint64_t *op_off, *op_ver;
    const uint64_t *ops_off, *ops_start, *ops_end;
};

// Array views indexed by GLOBAL CSR index k: element k lives at p[k - base] (base = the start of
// the workgroup's staged segment when p points into LDS, 0 for global memory). The bias is applied
// to the index, never to the pointer: an LDS pointer moved outside the LDS window is not a valid
// flat address.
// SPACE tags the instantiation (0 global, 1 LDS): a workgroup picks one uniformly, so every
// access in an instantiation has a single known address space (LDS views compile to ds_read /
// ds_write; a view that could be either would be a flat access, issued through the vector memory
// pipeline lane by lane).
template <int SPACE> struct V64S {
    const uint64_t *p;
    uint64_t base;
    __device__ inline uint64_t operator[](uint64_t k) const { return p[k - base]; }
};
using V64 = V64S<0>;
template <class T, int SPACE = 0> struct WView {
    T *p;
    uint64_t base;
    __device__ inline T &operator[](uint64_t k) const { return p[k - base]; }
};

// Holes of an entry's version space: their need ranges [tn] and their partial versions [tp].
template <class V> struct VerHolesT {
    V hs, he;                 // ranges
    uint64_t h0, h1;
    const uint64_t *pv;       // points
    uint64_t p0, p1;
    // if x lies in a hole, return the hole end (max over holes containing x) else return false
    __device__ inline bool covering(uint64_t x, uint64_t &end) const {
        bool hit = false;
        for (uint64_t k = h0; k < h1; k++)
            if (hs[k] <= x && x <= he[k] && (!hit || he[k] > end)) {
                end = he[k];
                hit = true;
            }
        for (uint64_t k = p0; k < p1; k++)
            if (pv[k] == x && (!hit || x > end)) {
                end = x;
                hit = true;
            }
        return hit;
    }
    // smallest hole start > x (UINT64_MAX if none)
    __device__ inline uint64_t next_start(uint64_t x) const {
        uint64_t m = ~0ULL;
        for (uint64_t k = h0; k < h1; k++)
            if (hs[k] > x && hs[k] < m) m = hs[k];
        for (uint64_t k = p0; k < p1; k++)
            if (pv[k] > x && pv[k] < m) m = pv[k];
        return m;
    }
};

struct SeqHoles {
    V64 hs, he;
    uint64_t h0, h1;
    __device__ inline bool covering(uint64_t x, uint64_t &end) const {
        bool hit = false;
        for (uint64_t k = h0; k < h1; k++)
            if (hs[k] <= x && x <= he[k] && (!hit || he[k] > end)) {
                end = he[k];
                hit = true;
            }
        return hit;
    }
    __device__ inline uint64_t next_start(uint64_t x) const {
        uint64_t m = ~0ULL;
        for (uint64_t k = h0; k < h1; k++)
            if (hs[k] > x && hs[k] < m) m = hs[k];
        return m;
    }
};

// Visit maximal pieces of ([lo, hi] ∩ universe[ulo, uhi]) − holes in ascending order.
template <class H, class F>
__device__ inline void sweep(const H &holes, uint64_t lo, uint64_t hi, uint64_t ulo, uint64_t uhi, F &&emit) {
    uint64_t x = lo > ulo ? lo : ulo;
    const uint64_t top = hi < uhi ? hi : uhi;
    while (x <= top) {
        uint64_t e;
        if (holes.covering(x, e)) {
            if (e >= top) return;
            x = e + 1;
            continue;
        }
        const uint64_t ns = holes.next_start(x);
        const uint64_t pe = (ns == ~0ULL || ns - 1 > top) ? top : ns - 1;
        emit(x, pe);
        if (pe >= top) return;
        x = pe + 1;
    }
}

// One workgroup = NEEDS_T consecutive entries, one lane per entry. The workgroup's CSR segments of
// their/our need ranges are contiguous, so they are staged into LDS with coalesced 16-B loads
// (lanes then walk LDS, not scattered global lines); in the fill pass the workgroup's output
// range [need_off[e0], need_off[e1]) is contiguous too, so outputs are assembled in LDS and
// written out coalesced. Segments larger than the LDS caps fall back to global memory (same code,
// generic pointers). Partials (5 % of entries) are read from global memory directly.
constexpr uint32_t NEEDS_T = 256;
constexpr uint32_t NEEDS_CAP_R = 640;    // staged ranges per side (avg 2 per entry -> 512, sd ~32)
constexpr uint32_t NEEDS_CAP_O = 960;    // staged output needs (avg ~2.5 per entry -> ~650); 3 WGs/CU

__device__ inline void stage_ranges(const uint64_t *gs, const uint64_t *ge, uint64_t lo, uint64_t cnt, uint64_t *ls,
                                    uint64_t *le) {
    // 16-B loads of pairs of ranges starting at an even global index (the CSR arrays are
    // 16-B aligned: corro_compute_needs checks device pointers)
    const uint64_t a0 = lo & ~1ULL;
    const uint64_t npair = (lo + cnt - a0 + 1) / 2;
    for (uint64_t q = threadIdx.x; q < npair; q += blockDim.x) {
        const uint64_t g = a0 + 2 * q;
        ulonglong2 s2, e2;
        if (g + 1 < lo + cnt) {  // never read past the segment (it may end the array)
            s2 = *reinterpret_cast<const ulonglong2 *>(gs + g);
            e2 = *reinterpret_cast<const ulonglong2 *>(ge + g);
        } else {
            s2.x = gs[g];
            e2.x = ge[g];
            s2.y = e2.y = 0;
        }
        if (g >= lo && g < lo + cnt) {
            ls[g - lo] = s2.x;
            le[g - lo] = e2.x;
        }
        if (g + 1 >= lo && g + 1 < lo + cnt) {
            ls[g + 1 - lo] = s2.y;
            le[g + 1 - lo] = e2.y;
        }
    }
}

template <bool FILL>
__global__ void __launch_bounds__(NEEDS_T) k_needs(SyncDev in, corro_needs_out o) {
    __shared__ uint64_t l_tns[NEEDS_CAP_R], l_tne[NEEDS_CAP_R], l_ons[NEEDS_CAP_R], l_one[NEEDS_CAP_R];
    __shared__ uint64_t l_start[FILL ? NEEDS_CAP_O : 1], l_end[FILL ? NEEDS_CAP_O : 1];
    __shared__ uint64_t l_sro[FILL ? NEEDS_CAP_O : 1], l_srn[FILL ? NEEDS_CAP_O : 1];
    __shared__ uint8_t l_kind[FILL ? NEEDS_CAP_O : 1];
    const uint64_t e0 = (uint64_t)blockIdx.x * NEEDS_T;
    const uint64_t e1 = min(in.n, e0 + NEEDS_T);
    const uint64_t e = e0 + threadIdx.x;
    const bool live = e < in.n;
    // per-lane words first, so their latency overlaps the staging below
    const uint64_t el = live ? e : e0;
    const uint64_t head = in.their_head[el];
    const int64_t ours = in.our_head[el];
    const uint64_t tne0 = in.tn_off[el], tne1 = in.tn_off[el + 1], one0 = in.on_off[el], one1 = in.on_off[el + 1];
    const uint64_t tpe0 = in.tp_off[el], tpe1 = in.tp_off[el + 1], ope0 = in.op_off[el], ope1 = in.op_off[el + 1];
    const uint64_t nbase = FILL ? o.need_off[el] : 0, sbase = FILL ? o.seq_off[el] : 0;
    // workgroup segments (uniform scalar loads)
    const uint64_t tn_lo = in.tn_off[e0], tn_hi = in.tn_off[e1];
    const uint64_t on_lo = in.on_off[e0], on_hi = in.on_off[e1];
    const bool tn_lds = tn_hi - tn_lo <= NEEDS_CAP_R, on_lds = on_hi - on_lo <= NEEDS_CAP_R;
    if (tn_lds) stage_ranges(in.tn_start, in.tn_end, tn_lo, tn_hi - tn_lo, l_tns, l_tne);
    if (on_lds) stage_ranges(in.on_start, in.on_end, on_lo, on_hi - on_lo, l_ons, l_one);
    uint64_t o_lo = 0, o_hi = 0;
    bool o_lds = false;
    if (FILL) {
        o_lo = o.need_off[e0];
        o_hi = o.need_off[e1];
        o_lds = o_hi - o_lo <= NEEDS_CAP_O;
    }
    __syncthreads();
    // the per-lane walk, instantiated once for LDS-staged views and once for global ones
    auto lane = [&](auto tns, auto tne, auto ons, auto one, auto okind, auto ostart, auto oend, auto osro,
                    auto osrn) {
        VerHolesT<decltype(tns)> vh{tns, tne, tne0, tne1, in.tp_ver, tpe0, tpe1};
        uint64_t nn = 0, ns = 0;
        auto full = [&](uint64_t s, uint64_t t) {
            if (FILL) {
                const uint64_t k = nbase + nn;
                okind[k] = 0;
                ostart[k] = s;
                oend[k] = t;
                osro[k] = sbase + ns;
                osrn[k] = 0;
            }
            nn++;
        };
        for (uint64_t k = one0; k < one1; k++) sweep(vh, ons[k], one[k], 1, head, full);

        for (uint64_t k = ope0; k < ope1; k++) {
            const uint64_t v = in.op_ver[k];
            uint64_t dummy;
            const bool have = v >= 1 && v <= head && !vh.covering(v, dummy);
            const uint64_t q0 = in.ops_off[k], q1 = in.ops_off[k + 1];
            if (have) {
                if (FILL) {
                    const uint64_t q = nbase + nn;
                    okind[q] = 1;
                    ostart[q] = v;
                    oend[q] = v;
                    osro[q] = sbase + ns;
                    osrn[q] = q1 - q0;
                    for (uint64_t j = q0; j < q1; j++) {
                        o.s_start[sbase + ns + (j - q0)] = in.ops_start[j];
                        o.s_end[sbase + ns + (j - q0)] = in.ops_end[j];
                    }
                }
                ns += q1 - q0;
                nn++;
                continue;
            }
            int64_t tk = -1;
            for (uint64_t j = tpe0; j < tpe1; j++)
                if (in.tp_ver[j] == v) {
                    tk = (int64_t)j;
                    break;
                }
            if (tk < 0) continue;
            bool have_end = false;
            uint64_t end = 0;
            for (uint64_t j = in.tps_off[tk]; j < in.tps_off[tk + 1]; j++)
                if (!have_end || in.tps_end[j] > end) {
                    end = in.tps_end[j];
                    have_end = true;
                }
            for (uint64_t j = q0; j < q1; j++)
                if (!have_end || in.ops_end[j] > end) {
                    end = in.ops_end[j];
                    have_end = true;
                }
            if (!have_end) continue;
            SeqHoles sh{V64{in.tps_start, 0}, V64{in.tps_end, 0}, in.tps_off[tk], in.tps_off[tk + 1]};
            const uint64_t first = sbase + ns;
            uint64_t cnt = 0;
            auto piece = [&](uint64_t s, uint64_t t) {
                if (FILL) {
                    o.s_start[first + cnt] = s;
                    o.s_end[first + cnt] = t;
                }
                cnt++;
            };
            for (uint64_t j = q0; j < q1; j++) sweep(sh, in.ops_start[j], in.ops_end[j], 0, end, piece);
            if (cnt) {
                if (FILL) {
                    const uint64_t q = nbase + nn;
                    okind[q] = 1;
                    ostart[q] = v;
                    oend[q] = v;
                    osro[q] = first;
                    osrn[q] = cnt;
                }
                nn++;
                ns += cnt;
            }
        }
        if (ours < 0) full(1, head);
        else if (head > (uint64_t)ours) full((uint64_t)ours + 1, head);
        if (!FILL) {
            o.need_count[e] = nn;
            o.seq_count[e] = ns;
        }
    };
    const bool all_lds = tn_lds && on_lds && (!FILL || o_lds);
    if (live) {
        if (all_lds) {
            lane(V64S<1>{l_tns, tn_lo}, V64S<1>{l_tne, tn_lo}, V64S<1>{l_ons, on_lo}, V64S<1>{l_one, on_lo},
                 WView<uint8_t, 1>{l_kind, o_lo}, WView<uint64_t, 1>{l_start, o_lo}, WView<uint64_t, 1>{l_end, o_lo},
                 WView<uint64_t, 1>{l_sro, o_lo}, WView<uint64_t, 1>{l_srn, o_lo});
        } else {
            lane(V64{in.tn_start, 0}, V64{in.tn_end, 0}, V64{in.on_start, 0}, V64{in.on_end, 0},
                 WView<uint8_t>{o.kind, 0}, WView<uint64_t>{o.start, 0}, WView<uint64_t>{o.end, 0},
                 WView<uint64_t>{o.sr_off, 0}, WView<uint64_t>{o.sr_n, 0});
        }
    }
    if (FILL && all_lds) {
        __syncthreads();
        const uint64_t m = o_hi - o_lo;
        for (uint64_t k = threadIdx.x; k < m; k += NEEDS_T) {
            o.start[o_lo + k] = l_start[k];
            o.end[o_lo + k] = l_end[k];
            o.sr_off[o_lo + k] = l_sro[k];
            o.sr_n[o_lo + k] = l_srn[k];
            o.kind[o_lo + k] = l_kind[k];
        }
    }
}

}  // namespace corro

using namespace corro;

extern "C" int corro_compute_needs(corro_ctx *ctx, const corro_sync_entries *in, int mem, corro_needs_out *out,
                                   int pass) {
    if (!ctx || !in || !out) return fail(CORRO_E_INVALID, "NULL argument");
    if (pass != 0 && pass != 1) return fail(CORRO_E_INVALID, "pass must be 0 or 1");
    if (mem != CORRO_MEM_HOST && mem != CORRO_MEM_DEVICE) return fail(CORRO_E_INVALID, "bad mem kind");
    const uint64_t n = in->n;
    if (n == 0) return CORRO_OK;
    CORRO_HIP_TRY(hipSetDevice(ctx->device));
    hipStream_t s = ctx->stream;
    SyncDev d{};
    d.n = n;
    corro_needs_out od = *out;
    if (mem == CORRO_MEM_DEVICE) {
        for (const void *q : {(const void *)in->tn_start, (const void *)in->tn_end, (const void *)in->on_start,
                              (const void *)in->on_end})
            if (q && ((uintptr_t)q % 16) != 0)
                return fail(CORRO_E_INVALID, "device need-range arrays must be 16-byte aligned");
        d.their_head = in->their_head; d.our_head = in->our_head;
        d.tn_off = in->tn_off; d.tn_start = in->tn_start; d.tn_end = in->tn_end;
        d.tp_off = in->tp_off; d.tp_ver = in->tp_ver;
        d.tps_off = in->tps_off; d.tps_start = in->tps_start; d.tps_end = in->tps_end;
        d.on_off = in->on_off; d.on_start = in->on_start; d.on_end = in->on_end;
        d.op_off = in->op_off; d.op_ver = in->op_ver;
        d.ops_off = in->ops_off; d.ops_start = in->ops_start; d.ops_end = in->ops_end;
    } else {
        // element counts of every CSR array
        const uint64_t ntn = in->tn_off[n], ntp = in->tp_off[n], nop = in->op_off[n], non = in->on_off[n];
        const uint64_t ntps = ntp ? in->tps_off[ntp] : 0, nops = nop ? in->ops_off[nop] : 0;
        struct F { const void *src; uint64_t cnt; const void **dst; };
        F f[] = {{in->their_head, n, (const void **)&d.their_head}, {in->our_head, n, (const void **)&d.our_head},
                 {in->tn_off, n + 1, (const void **)&d.tn_off},     {in->tn_start, ntn, (const void **)&d.tn_start},
                 {in->tn_end, ntn, (const void **)&d.tn_end},       {in->tp_off, n + 1, (const void **)&d.tp_off},
                 {in->tp_ver, ntp, (const void **)&d.tp_ver},       {in->tps_off, ntp + 1, (const void **)&d.tps_off},
                 {in->tps_start, ntps, (const void **)&d.tps_start}, {in->tps_end, ntps, (const void **)&d.tps_end},
                 {in->on_off, n + 1, (const void **)&d.on_off},     {in->on_start, non, (const void **)&d.on_start},
                 {in->on_end, non, (const void **)&d.on_end},       {in->op_off, n + 1, (const void **)&d.op_off},
                 {in->op_ver, nop, (const void **)&d.op_ver},       {in->ops_off, nop + 1, (const void **)&d.ops_off},
                 {in->ops_start, nops, (const void **)&d.ops_start}, {in->ops_end, nops, (const void **)&d.ops_end}};
        uint64_t total = 0;
        for (size_t i = 0; i < sizeof(f) / sizeof(f[0]); i++) {
            // nested offsets (tps_off / ops_off) may be NULL when there are no partials
            if (!f[i].src && ((i == 7 && ntp == 0) || (i == 15 && nop == 0))) f[i].cnt = 0;
            if (!f[i].src && f[i].cnt) return fail(CORRO_E_INVALID, "a required sync entry array is NULL");
            total += ((f[i].cnt * 8 + 255) / 256) * 256;
        }
        // outputs
        uint64_t tneeds = 0, tseqs = 0;
        if (pass == 1) {
            tneeds = out->need_off[n];
            tseqs = out->seq_off[n];
        }
        const uint64_t out_bytes = pass == 0 ? 2 * ((n * 8 + 255) / 256) * 256
                                             : 2 * (((n + 1) * 8 + 255) / 256) * 256 + ((tneeds + 255) / 256) * 256 +
                                                   4 * ((tneeds * 8 + 255) / 256) * 256 +
                                                   2 * ((tseqs * 8 + 255) / 256) * 256;
        if (int rc = ctx->d_needs.ensure(total + out_bytes + 4096)) return rc;
        uint8_t *p = ctx->d_needs.as<uint8_t>();
        for (auto &x : f) {
            *x.dst = p;
            if (x.cnt && x.src) CORRO_HIP_TRY(hipMemcpyAsync(p, x.src, x.cnt * 8, hipMemcpyHostToDevice, s));
            p += ((x.cnt * 8 + 255) / 256) * 256;
        }
        auto carve = [&](uint64_t bytes) {
            uint8_t *q = p;
            p += ((bytes + 255) / 256) * 256;
            return q;
        };
        if (pass == 0) {
            od.need_count = (uint64_t *)carve(n * 8);
            od.seq_count = (uint64_t *)carve(n * 8);
        } else {
            uint64_t *no = (uint64_t *)carve((n + 1) * 8), *so = (uint64_t *)carve((n + 1) * 8);
            CORRO_HIP_TRY(hipMemcpyAsync(no, out->need_off, (n + 1) * 8, hipMemcpyHostToDevice, s));
            CORRO_HIP_TRY(hipMemcpyAsync(so, out->seq_off, (n + 1) * 8, hipMemcpyHostToDevice, s));
            od.need_off = no;
            od.seq_off = so;
            od.kind = (uint8_t *)carve(tneeds);
            od.start = (uint64_t *)carve(tneeds * 8);
            od.end = (uint64_t *)carve(tneeds * 8);
            od.sr_off = (uint64_t *)carve(tneeds * 8);
            od.sr_n = (uint64_t *)carve(tneeds * 8);
            od.s_start = (uint64_t *)carve(tseqs * 8);
            od.s_end = (uint64_t *)carve(tseqs * 8);
        }
    }
    const uint64_t blocks = (n + NEEDS_T - 1) / NEEDS_T;
    if (blocks > 0x7FFFFFFFULL) return fail(CORRO_E_RANGE, "too many sync entries");
    if (ctx->profiling) CORRO_HIP_TRY(hipEventRecord(ctx->ev[0], s));
    if (pass == 0)
        hipLaunchKernelGGL(k_needs<false>, dim3((uint32_t)blocks), dim3(NEEDS_T), 0, s, d, od);
    else
        hipLaunchKernelGGL(k_needs<true>, dim3((uint32_t)blocks), dim3(NEEDS_T), 0, s, d, od);
    if (ctx->profiling) CORRO_HIP_TRY(hipEventRecord(ctx->ev[1], s));
    CORRO_HIP_TRY(hipGetLastError());
    if (mem == CORRO_MEM_HOST) {
        if (pass == 0) {
            CORRO_HIP_TRY(hipMemcpyAsync(out->need_count, od.need_count, n * 8, hipMemcpyDeviceToHost, s));
            CORRO_HIP_TRY(hipMemcpyAsync(out->seq_count, od.seq_count, n * 8, hipMemcpyDeviceToHost, s));
        } else {
            const uint64_t tneeds = out->need_off[n], tseqs = out->seq_off[n];
            if (tneeds) {
                CORRO_HIP_TRY(hipMemcpyAsync(out->kind, od.kind, tneeds, hipMemcpyDeviceToHost, s));
                CORRO_HIP_TRY(hipMemcpyAsync(out->start, od.start, tneeds * 8, hipMemcpyDeviceToHost, s));
                CORRO_HIP_TRY(hipMemcpyAsync(out->end, od.end, tneeds * 8, hipMemcpyDeviceToHost, s));
                CORRO_HIP_TRY(hipMemcpyAsync(out->sr_off, od.sr_off, tneeds * 8, hipMemcpyDeviceToHost, s));
                CORRO_HIP_TRY(hipMemcpyAsync(out->sr_n, od.sr_n, tneeds * 8, hipMemcpyDeviceToHost, s));
            }
            if (tseqs) {
                CORRO_HIP_TRY(hipMemcpyAsync(out->s_start, od.s_start, tseqs * 8, hipMemcpyDeviceToHost, s));
                CORRO_HIP_TRY(hipMemcpyAsync(out->s_end, od.s_end, tseqs * 8, hipMemcpyDeviceToHost, s));
            }
        }
    }
    CORRO_HIP_TRY(hipStreamSynchronize(s));
    if (ctx->profiling) CORRO_HIP_TRY(hipEventElapsedTime(&ctx->last_ms[6 + pass], ctx->ev[0], ctx->ev[1]));
    return CORRO_OK;
}
