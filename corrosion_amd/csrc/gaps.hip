// Batched gap bookkeeping: VersionsSnapshot::compute_gaps_change + insert_db
// (/root/reference/crates/corro-types/src/agent.rs:1108-1235) for many actors in one launch, one
// lane per actor. The host form (booked.h, one std::map walk per actor) costs ~20-30 us per actor
// (tools/time_bookkeeping.py); a process_multiple_changes call or a sync round touching 10^5 actors
// spends seconds there against a few ms of merge.
//
// Per actor, with G = its needed gaps (canonical RangeInclusiveSet: sorted, disjoint, non-touching,
// all below max), V = the call's applied versions (canonical), M = max (has_max), gs = M + 1:
//   absorbed = { g in G : g overlaps or touches some v in V }       (the overlapping / s-1 / e+1
//              ∪ { g in G : g overlaps [gs, v.s] for a v with gs < v.s }  lookups of insert_db)
//   N        = [gs, max{v.s : v.s > gs}]  when such a v exists          (gap_start .. s)
//   inserted = (∪absorbed ∪ N) − ∪V       (the INSERT rows; each piece maximal)
//   removed  = absorbed                     (the DELETE rows)
//   needed'  = (G − absorbed) ∪ inserted,  max' = max(M, last v.e)
// All lists are produced by sorted two-pointer merges: no set is materialised. A piece of
// `inserted` starting where a kept gap starts is the reference's UNIQUE (actor_id, start) failure
// (status 1 in the ABI): pieces lie inside absorbed gaps or above max, kept gaps are disjoint from
// both, so canonical inputs never produce it and the kernel reports 0 or -1 (a non-canonical input).
#include <hip/hip_runtime.h>

#include "internal.h"

namespace corro {

constexpr uint32_t GAPS_T = 256;

struct GapsDev {
    corro_gaps_in in;
    corro_gaps_out out;
};

// true when [a, b] overlaps or touches [s, e] (s - 1 / e + 1 without wrapping)
__device__ inline bool touches(uint64_t a, uint64_t b, uint64_t s, uint64_t e) {
    const uint64_t lo = s > 0 ? s - 1 : 0, hi = e < ~0ULL ? e + 1 : e;
    return a <= hi && b >= lo;
}

__global__ void __launch_bounds__(GAPS_T) k_gaps(GapsDev d) {
    const uint64_t a = (uint64_t)blockIdx.x * GAPS_T + threadIdx.x;
    if (a >= d.in.n) return;
    const corro_gaps_in &in = d.in;
    const corro_gaps_out &o = d.out;
    const uint64_t g0 = in.gap_off[a], g1 = in.gap_off[a + 1];
    const uint64_t v0 = in.ver_off[a], v1 = in.ver_off[a + 1];
    const int64_t m_in = in.max[a];
    const bool has_max = m_in >= 0;
    const uint64_t M = has_max ? (uint64_t)m_in : 0, gs = M + 1;
    // output windows reserved by the input sizes (corro_gaps_out)
    const uint64_t rbase = g0, ibase = g0 + v0 + a;
    int32_t st = 0;
    // canonical inputs: sorted, disjoint, non-touching
    for (uint64_t k = v0; k < v1; k++)
        if (in.ver_start[k] > in.ver_end[k] || (k > v0 && in.ver_start[k] <= in.ver_end[k - 1] + 1)) st = -1;
    for (uint64_t k = g0; k < g1; k++)
        if (in.gap_start[k] > in.gap_end[k] || (k > g0 && in.gap_start[k] <= in.gap_end[k - 1] + 1)) st = -1;
    if (st) {
        o.status[a] = st;
        o.max[a] = m_in;
        o.rm_count[a] = o.ins_count[a] = 0;
        o.gap_count[a] = 0;
        return;
    }
    // N = [gs, max s over versions with s > gs]
    bool hasN = false;
    uint64_t nEnd = 0;
    int64_t nmax = m_in;
    for (uint64_t k = v0; k < v1; k++) {
        const uint64_t s = in.ver_start[k], e = in.ver_end[k];
        if (nmax < 0 || e > (uint64_t)nmax) nmax = (int64_t)e;
        if (gs < s) {
            hasN = true;
            nEnd = s;  // ascending: the last such s is the largest
        }
    }
    // pass over G: absorbed gaps (two pointers over V), their pieces minus V, kept gaps; the pieces
    // and kept gaps come out in ascending order, merged on the fly into needed'
    uint64_t nr = 0, ni = 0, ng = 0;
    uint64_t vk = v0;  // first version range that can still touch the current gap
    auto emit_piece_minus_v = [&](uint64_t s, uint64_t e, uint64_t &vp) {
        // [s, e] − ∪V: V ranges from vp on (sorted); vp advances past ranges ending before s
        while (vp < v1 && in.ver_end[vp] < s) vp++;
        uint64_t x = s;
        uint64_t j = vp;
        while (x <= e) {
            if (j < v1 && in.ver_start[j] <= e) {
                const uint64_t vs = in.ver_start[j], ve = in.ver_end[j];
                if (vs > x) {
                    o.ins_start[ibase + ni] = x;
                    o.ins_end[ibase + ni] = vs - 1;
                    ni++;
                    o.new_start[ibase + ng] = x;
                    o.new_end[ibase + ng] = vs - 1;
                    ng++;
                }
                if (ve >= e) return;
                x = ve + 1;
                j++;
            } else {
                o.ins_start[ibase + ni] = x;
                o.ins_end[ibase + ni] = e;
                ni++;
                o.new_start[ibase + ng] = x;
                o.new_end[ibase + ng] = e;
                ng++;
                return;
            }
        }
    };
    uint64_t vp = v0;
    for (uint64_t k = g0; k < g1; k++) {
        const uint64_t s = in.gap_start[k], e = in.gap_end[k];
        // skip version ranges ending before s - 1 (sorted: none of them touches a later gap either)
        while (vk < v1 && s > 0 && in.ver_end[vk] < s - 1) vk++;
        const bool ab = vk < v1 && touches(s, e, in.ver_start[vk], in.ver_end[vk]);
        // or overlaps [gs, s] (never for gaps below max)
        if (ab || (hasN && e >= gs && s <= nEnd)) {
            o.rm_start[rbase + nr] = s;
            o.rm_end[rbase + nr] = e;
            nr++;
            emit_piece_minus_v(s, e, vp);
        } else {
            // a kept gap: an inserted piece never starts here for canonical inputs (disjoint)
            o.new_start[ibase + ng] = s;
            o.new_end[ibase + ng] = e;
            ng++;
        }
    }
    if (hasN) emit_piece_minus_v(gs, nEnd, vp);
    o.status[a] = st;
    o.max[a] = nmax;
    o.rm_count[a] = nr;
    o.ins_count[a] = ni;
    o.gap_count[a] = ng;
}

}  // namespace corro

using namespace corro;

extern "C" int corro_booked_insert_db_batch(corro_ctx *ctx, const corro_gaps_in *in, corro_gaps_out *out) {
    if (!ctx || !in || !out) return fail(CORRO_E_INVALID, "NULL argument");
    const uint64_t n = in->n;
    if (n == 0) return CORRO_OK;
    if (!in->max || !in->gap_off || !in->ver_off || !out->max || !out->rm_count || !out->ins_count ||
        !out->gap_count || !out->status)
        return fail(CORRO_E_INVALID, "a required array is NULL");
    const uint64_t blocks = (n + GAPS_T - 1) / GAPS_T;
    if (blocks > 0x7FFFFFFFULL) return fail(CORRO_E_RANGE, "too many actors");
    CORRO_HIP_TRY(hipSetDevice(ctx->device));
    hipStream_t s = ctx->stream;
    GapsDev d{*in, *out};
    if (ctx->profiling) CORRO_HIP_TRY(hipEventRecord(ctx->ev[0], s));
    hipLaunchKernelGGL(k_gaps, dim3((uint32_t)blocks), dim3(GAPS_T), 0, s, d);
    if (ctx->profiling) CORRO_HIP_TRY(hipEventRecord(ctx->ev[1], s));
    CORRO_HIP_TRY(hipGetLastError());
    CORRO_HIP_TRY(hipStreamSynchronize(s));
    if (ctx->profiling) {
        CORRO_HIP_TRY(hipEventElapsedTime(&ctx->last_ms[6], ctx->ev[0], ctx->ev[1]));
        ctx->last_ms[7] = 0.f;
    }
    return CORRO_OK;
}
