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
// All lists are produced by sorted two-pointer merges: no set is materialised. Actors with more
// than GAPS_BIG gaps + version ranges take a wave each instead of a lane (k_gaps_wave: the gaps in
// chunks of 64 lanes, each lane's absorption and pieces found by binary search over V, the output
// offsets by wave scans), so one long actor no longer serialises its wave. A piece of
// `inserted` starting where a kept gap starts is the reference's UNIQUE (actor_id, start) failure
// (status 1 in the ABI): pieces lie inside absorbed gaps or above max, kept gaps are disjoint from
// both, so canonical inputs never produce it and the kernel reports 0 or -1 (a non-canonical input).
#include <hip/hip_runtime.h>

#include "internal.h"

namespace corro {

constexpr uint32_t GAPS_T = 256;
constexpr uint64_t GAPS_BIG = 32;  // gaps + version ranges above which an actor takes a wave

struct GapsDev {
    corro_gaps_in in;
    corro_gaps_out out;
    uint32_t *big;               // actors handed to k_gaps_wave
    unsigned long long *nbig;
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
    if ((g1 - g0) + (v1 - v0) > GAPS_BIG) {
        d.big[atomicAdd(d.nbig, 1ULL)] = (uint32_t)a;
        return;
    }
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

// ---- one wave per long actor --------------------------------------------------------------------
__device__ inline uint64_t gw_scan(uint64_t x) {  // inclusive, over the wave
    const uint32_t lane = threadIdx.x & 63;
#pragma unroll
    for (int k = 1; k < 64; k <<= 1) {
        const uint64_t y = __shfl_up(x, k);
        if (lane >= (uint32_t)k) x += y;
    }
    return x;
}
// first k in [lo, hi) with a[k] >= x (a ascending)
__device__ inline uint64_t gw_lower(const uint64_t *a, uint64_t lo, uint64_t hi, uint64_t x) {
    while (lo < hi) {
        const uint64_t m = lo + (hi - lo) / 2;
        if (a[m] < x) lo = m + 1;
        else hi = m;
    }
    return lo;
}
// first k in [lo, hi) with a[k] > x
__device__ inline uint64_t gw_upper(const uint64_t *a, uint64_t lo, uint64_t hi, uint64_t x) {
    while (lo < hi) {
        const uint64_t m = lo + (hi - lo) / 2;
        if (a[m] <= x) lo = m + 1;
        else hi = m;
    }
    return lo;
}

// [s, e] − ∪V as maximal pieces (V ascending, disjoint): their number; with o non-null, each piece
// also written to ins[ib ..] and to new[nb ..]
__device__ inline uint64_t gw_pieces(const corro_gaps_in &in, uint64_t v0, uint64_t v1, uint64_t s, uint64_t e,
                                     const corro_gaps_out *o, uint64_t ib, uint64_t nb) {
    const uint64_t j0 = gw_lower(in.ver_end, v0, v1, s), j1 = gw_upper(in.ver_start, j0, v1, e);
    uint64_t x = s, n = 0;
    auto put = [&](uint64_t ps, uint64_t pe) {
        if (o) {
            o->ins_start[ib + n] = ps;
            o->ins_end[ib + n] = pe;
            o->new_start[nb + n] = ps;
            o->new_end[nb + n] = pe;
        }
        n++;
    };
    for (uint64_t j = j0; j < j1; j++) {
        const uint64_t vs = in.ver_start[j], ve = in.ver_end[j];
        if (vs > x) put(x, vs - 1);
        if (ve >= e) return n;
        x = ve + 1;
    }
    put(x, e);
    return n;
}

__global__ void __launch_bounds__(GAPS_T) k_gaps_wave(GapsDev d) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t nw = (uint64_t)gridDim.x * (GAPS_T / 64);
    const uint64_t nbig = *d.nbig;
    const corro_gaps_in &in = d.in;
    const corro_gaps_out &o = d.out;
    for (uint64_t w = (uint64_t)blockIdx.x * (GAPS_T / 64) + (threadIdx.x >> 6); w < nbig; w += nw) {
        const uint64_t a = d.big[w];
        const uint64_t g0 = in.gap_off[a], g1 = in.gap_off[a + 1];
        const uint64_t v0 = in.ver_off[a], v1 = in.ver_off[a + 1];
        const int64_t m_in = in.max[a];
        const uint64_t M = m_in >= 0 ? (uint64_t)m_in : 0, gs = M + 1;
        const uint64_t rbase = g0, ibase = g0 + v0 + a;
        bool bad = false;
        for (uint64_t k = v0 + lane; k < v1; k += 64)
            bad |= in.ver_start[k] > in.ver_end[k] || (k > v0 && in.ver_start[k] <= in.ver_end[k - 1] + 1);
        for (uint64_t k = g0 + lane; k < g1; k += 64)
            bad |= in.gap_start[k] > in.gap_end[k] || (k > g0 && in.gap_start[k] <= in.gap_end[k - 1] + 1);
        if (__any(bad)) {
            if (lane == 0) {
                o.status[a] = -1;
                o.max[a] = m_in;
                o.rm_count[a] = o.ins_count[a] = o.gap_count[a] = 0;
            }
            continue;
        }
        // max' and N = [gs, the largest version start above gs] (V ascending: its last range)
        int64_t nmax = m_in;
        bool hasN = false;
        uint64_t nEnd = 0;
        if (v1 > v0) {
            const uint64_t le = in.ver_end[v1 - 1], ls = in.ver_start[v1 - 1];
            if (nmax < 0 || le > (uint64_t)nmax) nmax = (int64_t)le;
            if (gs < ls) {
                hasN = true;
                nEnd = ls;
            }
        }
        uint64_t nr = 0, ni = 0, ng = 0;  // running output counts (wave-uniform)
        for (uint64_t c = g0; c < g1; c += 64) {
            const uint64_t k = c + lane;
            const bool act = k < g1;
            bool ab = false;
            uint64_t s = 0, e = 0, np = 0;
            if (act) {
                s = in.gap_start[k];
                e = in.gap_end[k];
                // a version range overlapping or touching [s, e]: the first one ending at or after s - 1
                const uint64_t vk = gw_lower(in.ver_end, v0, v1, s > 0 ? s - 1 : 0);
                ab = (vk < v1 && touches(s, e, in.ver_start[vk], in.ver_end[vk])) ||
                     (hasN && e >= gs && s <= nEnd);
                if (ab) np = gw_pieces(in, v0, v1, s, e, nullptr, 0, 0);
            }
            const uint64_t ng_own = act ? (ab ? np : 1) : 0;
            const uint64_t r_inc = gw_scan(ab ? 1 : 0), i_inc = gw_scan(np), g_inc = gw_scan(ng_own);
            if (ab) {
                o.rm_start[rbase + nr + r_inc - 1] = s;
                o.rm_end[rbase + nr + r_inc - 1] = e;
                gw_pieces(in, v0, v1, s, e, &o, ibase + ni + i_inc - np, ibase + ng + g_inc - np);
            } else if (act) {
                o.new_start[ibase + ng + g_inc - 1] = s;
                o.new_end[ibase + ng + g_inc - 1] = e;
            }
            nr += __shfl(r_inc, 63);
            ni += __shfl(i_inc, 63);
            ng += __shfl(g_inc, 63);
        }
        // N's pieces come after every gap (gaps lie below max < gs)
        if (hasN) {
            uint64_t np = 0;
            if (lane == 0) np = gw_pieces(in, v0, v1, gs, nEnd, &o, ibase + ni, ibase + ng);
            np = __shfl(np, 0);
            ni += np;
            ng += np;
        }
        if (lane == 0) {
            o.status[a] = 0;
            o.max[a] = nmax;
            o.rm_count[a] = nr;
            o.ins_count[a] = ni;
            o.gap_count[a] = ng;
        }
    }
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
    if (n >= (1ULL << 32)) return fail(CORRO_E_RANGE, "too many actors");
    if (int rc = ctx->d_gaps_big.ensure(n * 4 + 64)) return rc;
    GapsDev d{*in, *out, ctx->d_gaps_big.as<uint32_t>() + 16, ctx->d_gaps_big.as<unsigned long long>()};
    CORRO_HIP_TRY(hipMemsetAsync(d.nbig, 0, 8, s));
    if (ctx->profiling) CORRO_HIP_TRY(hipEventRecord(ctx->ev[0], s));
    hipLaunchKernelGGL(k_gaps, dim3((uint32_t)blocks), dim3(GAPS_T), 0, s, d);
    CORRO_HIP_TRY(hipGetLastError());
    // the long actors, a wave each (the grid strides over however many k_gaps listed)
    hipLaunchKernelGGL(k_gaps_wave, dim3((uint32_t)std::min<uint64_t>(blocks * (GAPS_T / 64), 2048)), dim3(GAPS_T), 0,
                       s, d);
    if (ctx->profiling) CORRO_HIP_TRY(hipEventRecord(ctx->ev[1], s));
    CORRO_HIP_TRY(hipGetLastError());
    CORRO_HIP_TRY(hipStreamSynchronize(s));
    if (ctx->profiling) {
        CORRO_HIP_TRY(hipEventElapsedTime(&ctx->last_ms[6], ctx->ev[0], ctx->ev[1]));
        ctx->last_ms[7] = 0.f;
    }
    return CORRO_OK;
}
