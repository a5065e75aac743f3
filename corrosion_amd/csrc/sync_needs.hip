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
#include <cstdio>
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
    V pv;                     // points
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

// The common entry -- a few need ranges of theirs, no partial of theirs -- keeps its holes in
// registers: the sweep tests every hole at every step, and from LDS that is a chain of dependent
// reads per step; from registers the tests are a few predicated compares.
#ifndef NEED_RH
#define NEED_RH 3
#endif
#ifndef NEED_RO  // > 0: an entry with at most NEED_RO need ranges of ours loads them all up front
#define NEED_RO 0
#endif
struct RegHoles {
    uint64_t hs[NEED_RH > 0 ? NEED_RH : 1], he[NEED_RH > 0 ? NEED_RH : 1];
    uint32_t n;
    __device__ inline bool covering(uint64_t x, uint64_t &end) const {
        bool hit = false;
#pragma unroll
        for (int k = 0; k < NEED_RH; k++)
            if ((uint32_t)k < n && hs[k] <= x && x <= he[k] && (!hit || he[k] > end)) {
                end = he[k];
                hit = true;
            }
        return hit;
    }
    __device__ inline uint64_t next_start(uint64_t x) const {
        uint64_t m = ~0ULL;
#pragma unroll
        for (int k = 0; k < NEED_RH; k++)
            if ((uint32_t)k < n && hs[k] > x && hs[k] < m) m = hs[k];
        return m;
    }
};

template <class V> struct SeqHolesT {
    V hs, he;
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

// One workgroup = NEEDS_T consecutive entries, one lane per entry. Every CSR segment a workgroup
// touches is contiguous (their/our need ranges, their/our partial versions, their seq offsets and
// seq ranges), so all of them are staged into LDS up front — one wave of coalesced loads per
// segment, three dependent latencies in total (offsets -> nested offsets -> ranges) — and the lanes
// then walk LDS only. In the fill pass the workgroup's output range is contiguous too, so outputs
// are assembled in LDS and written out coalesced. A workgroup with any segment above its LDS cap
// runs the same walk on global memory instead (views over global arrays).
constexpr uint32_t NEEDS_T = 256;
constexpr uint32_t NEEDS_CAP_R = 576;    // staged need ranges per side (avg 2 per entry -> 512, sd ~23)
constexpr uint32_t NEEDS_CAP_O = 800;    // staged output needs (avg ~2.55 per entry -> ~650, sd ~30)
constexpr uint32_t NEEDS_CAP_P = 64;     // staged partial versions per side (5 % of entries -> ~13)
constexpr uint32_t NEEDS_CAP_S = 160;    // staged partial seq ranges per side (~2 per partial -> ~26)

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

__device__ inline void stage_words(const uint64_t *g, uint64_t lo, uint64_t cnt, uint64_t *l) {
    for (uint64_t q = threadIdx.x; q < cnt; q += blockDim.x) l[q] = g[lo + q];
}

// Per-lane words of one entry.
struct EntryHdr {
    uint64_t head;
    int64_t ours;
    uint64_t tne0, tne1, one0, one1, tpe0, tpe1, ope0, ope1;
};

__device__ inline EntryHdr load_entry(const SyncDev &in, uint64_t e) {
    EntryHdr h;
    h.head = in.their_head[e];
    h.ours = in.our_head[e];
    h.tne0 = in.tn_off[e]; h.tne1 = in.tn_off[e + 1];
    h.one0 = in.on_off[e]; h.one1 = in.on_off[e + 1];
    h.tpe0 = in.tp_off[e]; h.tpe1 = in.tp_off[e + 1];
    h.ope0 = in.op_off[e]; h.ope1 = in.op_off[e + 1];
    return h;
}

// Every input array an entry walk reads, as views of one address space.
template <class V> struct InViews {
    V tns, tne, ons, one;          // need ranges
    V tpv, tpso, tpss, tpse;       // their partial versions, seq offsets, seq ranges
    V opv, opso, opss, opse;       // ours
};

// The walk of one entry (sync.rs:141-245). Counts its needs (nn) and partial seq ranges (ns); with
// FILL also writes them: needs at [nbase, nbase + nn) through the o* views, seq ranges straight to
// global memory at [sbase, sbase + ns).
// Output emitters of the fill walk. NeedsEmit: the five arrays of corro_needs_out (global or LDS
// views); need q, seq-range slot j.
template <class VK, class VU> struct NeedsEmit {
    VK okind;
    VU ostart, oend, osro, osrn;
    uint64_t *s_start, *s_end;
    __device__ inline void full(uint64_t q, uint64_t s, uint64_t t, uint64_t sr) const {
        okind[q] = 0;
        ostart[q] = s;
        oend[q] = t;
        osro[q] = sr;
        osrn[q] = 0;
    }
    __device__ inline void partial(uint64_t q, uint64_t v, uint64_t sr, uint64_t cnt) const {
        okind[q] = 1;
        ostart[q] = v;
        oend[q] = v;
        osro[q] = sr;
        osrn[q] = cnt;
    }
    __device__ inline void seq(uint64_t j, uint64_t s, uint64_t t) const {
        s_start[j] = s;
        s_end[j] = t;
    }
};

template <bool FILL, class V, class E, class H>
__device__ inline void walk_entry_h(const EntryHdr &h, const InViews<V> &iv, const H &vh, const E &em, uint64_t nbase,
                                    uint64_t sbase, uint64_t &nn_out, uint64_t &ns_out) {
    const uint64_t head = h.head;
    uint64_t nn = 0, ns = 0;
    auto full = [&](uint64_t s, uint64_t t) {
        if (FILL) em.full(nbase + nn, s, t, sbase + ns);
        nn++;
    };
    auto our_range = [&](uint64_t s, uint64_t t) {
        if (s > t) {
            // an inverted (empty) range, which no RangeInclusiveSet holds but a peer's message may:
            // rangemap's overlapping(s..=t) yields every stored range with end >= s and start <= t,
            // i.e. a have range spanning [t, s], and the reference then pushes Full(s..=t) as is
            if (t >= 1 && s <= head) {
                uint64_t dummy;
                if (!vh.covering(t, dummy) && vh.next_start(t) > s) full(s, t);
            }
            return;
        }
        sweep(vh, s, t, 1, head, full);
    };
#if NEED_RO > 0
    if (h.one1 - h.one0 <= (uint64_t)NEED_RO) {  // all loads issued before the first sweep
        uint64_t os[NEED_RO], oe[NEED_RO];
        const uint32_t no = (uint32_t)(h.one1 - h.one0);
#pragma unroll
        for (int k = 0; k < NEED_RO; k++) {
            os[k] = (uint32_t)k < no ? iv.ons[h.one0 + k] : 0;
            oe[k] = (uint32_t)k < no ? iv.one[h.one0 + k] : 0;
        }
#pragma unroll
        for (int k = 0; k < NEED_RO; k++)
            if ((uint32_t)k < no) our_range(os[k], oe[k]);
    } else
#endif
        for (uint64_t k = h.one0; k < h.one1; k++) our_range(iv.ons[k], iv.one[k]);

    for (uint64_t k = h.ope0; k < h.ope1; k++) {
        const uint64_t v = iv.opv[k];
        uint64_t dummy;
        const bool have = v >= 1 && v <= head && !vh.covering(v, dummy);
        const uint64_t q0 = iv.opso[k], q1 = iv.opso[k + 1];
        if (have) {
            if (FILL) {
                em.partial(nbase + nn, v, sbase + ns, q1 - q0);
                for (uint64_t j = q0; j < q1; j++) em.seq(sbase + ns + (j - q0), iv.opss[j], iv.opse[j]);
            }
            ns += q1 - q0;
            nn++;
            continue;
        }
        int64_t tk = -1;
        for (uint64_t j = h.tpe0; j < h.tpe1; j++)
            if (iv.tpv[j] == v) {
                tk = (int64_t)j;
                break;
            }
        if (tk < 0) continue;
        const uint64_t t0 = iv.tpso[tk], t1 = iv.tpso[tk + 1];
        bool have_end = false;
        uint64_t end = 0;
        for (uint64_t j = t0; j < t1; j++)
            if (!have_end || iv.tpse[j] > end) {
                end = iv.tpse[j];
                have_end = true;
            }
        for (uint64_t j = q0; j < q1; j++)
            if (!have_end || iv.opse[j] > end) {
                end = iv.opse[j];
                have_end = true;
            }
        if (!have_end) continue;
        SeqHolesT<V> sh{iv.tpss, iv.tpse, t0, t1};
        const uint64_t first = sbase + ns;
        uint64_t cnt = 0;
        auto piece = [&](uint64_t s, uint64_t t) {
            if (FILL) em.seq(first + cnt, s, t);
            cnt++;
        };
        for (uint64_t j = q0; j < q1; j++) sweep(sh, iv.opss[j], iv.opse[j], 0, end, piece);
        if (cnt) {
            if (FILL) em.partial(nbase + nn, v, first, cnt);
            nn++;
            ns += cnt;
        }
    }
    if (h.ours < 0) full(1, head);
    else if (head > (uint64_t)h.ours) full((uint64_t)h.ours + 1, head);
    nn_out = nn;
    ns_out = ns;
}

template <bool FILL, class V, class E>
__device__ inline void walk_entry(const EntryHdr &h, const InViews<V> &iv, const E &em, uint64_t nbase,
                                  uint64_t sbase, uint64_t &nn_out, uint64_t &ns_out) {
    if (NEED_RH > 0 && h.tpe1 == h.tpe0 && h.tne1 - h.tne0 <= (uint64_t)NEED_RH) {
        RegHoles rh;
        rh.n = (uint32_t)(h.tne1 - h.tne0);
#pragma unroll
        for (int k = 0; k < (NEED_RH > 0 ? NEED_RH : 1); k++) {
            const bool in = (uint32_t)k < rh.n;
            rh.hs[k] = in ? iv.tns[h.tne0 + k] : 0;
            rh.he[k] = in ? iv.tne[h.tne0 + k] : 0;
        }
        walk_entry_h<FILL>(h, iv, rh, em, nbase, sbase, nn_out, ns_out);
        return;
    }
    const VerHolesT<V> vh{iv.tns, iv.tne, h.tne0, h.tne1, iv.tpv, h.tpe0, h.tpe1};
    walk_entry_h<FILL>(h, iv, vh, em, nbase, sbase, nn_out, ns_out);
}

// LDS of one need workgroup: the staged inputs ...
struct NeedsLds {
    uint64_t tns[NEEDS_CAP_R], tne[NEEDS_CAP_R], ons[NEEDS_CAP_R], one[NEEDS_CAP_R];
    uint64_t tpv[NEEDS_CAP_P], tpso[NEEDS_CAP_P + 1], tpss[NEEDS_CAP_S], tpse[NEEDS_CAP_S];
    uint64_t opv[NEEDS_CAP_P], opso[NEEDS_CAP_P + 1], opss[NEEDS_CAP_S], opse[NEEDS_CAP_S];
};
// ... and, when outputs are staged (NEEDS_OSTAGE), the output needs.
struct NeedsOutLds {
    uint64_t start[NEEDS_CAP_O], end[NEEDS_CAP_O], sro[NEEDS_CAP_O], srn[NEEDS_CAP_O];
    uint8_t kind[NEEDS_CAP_O];
};

// Segment bounds of one workgroup [e0, e1) (global CSR indices).
struct WgSegs {
    uint64_t tn_lo, tn_hi, on_lo, on_hi, tp_lo, tp_hi, op_lo, op_hi, tps_lo, tps_hi, ops_lo, ops_hi;
    bool lds;
};

// Stage every input segment of the workgroup into LDS (or decide that one does not fit).
// Ends with __syncthreads().
__device__ inline WgSegs stage_inputs(const SyncDev &in, uint64_t e0, uint64_t e1, NeedsLds &L) {
    WgSegs g;
    g.tn_lo = in.tn_off[e0]; g.tn_hi = in.tn_off[e1];
    g.on_lo = in.on_off[e0]; g.on_hi = in.on_off[e1];
    g.tp_lo = in.tp_off[e0]; g.tp_hi = in.tp_off[e1];
    g.op_lo = in.op_off[e0]; g.op_hi = in.op_off[e1];
    const bool fit1 = g.tn_hi - g.tn_lo <= NEEDS_CAP_R && g.on_hi - g.on_lo <= NEEDS_CAP_R &&
                      g.tp_hi - g.tp_lo <= NEEDS_CAP_P && g.op_hi - g.op_lo <= NEEDS_CAP_P;
    g.tps_lo = g.tps_hi = g.ops_lo = g.ops_hi = 0;
    g.lds = false;
    if (!fit1) return g;  // uniform: no barrier skipped by part of the workgroup
    // nested offsets of the partial segments (uniform loads; NULL arrays only when empty)
    if (g.tp_hi > g.tp_lo) {
        g.tps_lo = in.tps_off[g.tp_lo];
        g.tps_hi = in.tps_off[g.tp_hi];
    }
    if (g.op_hi > g.op_lo) {
        g.ops_lo = in.ops_off[g.op_lo];
        g.ops_hi = in.ops_off[g.op_hi];
    }
    stage_ranges(in.tn_start, in.tn_end, g.tn_lo, g.tn_hi - g.tn_lo, L.tns, L.tne);
    stage_ranges(in.on_start, in.on_end, g.on_lo, g.on_hi - g.on_lo, L.ons, L.one);
    if (g.tp_hi > g.tp_lo) {
        stage_words(in.tp_ver, g.tp_lo, g.tp_hi - g.tp_lo, L.tpv);
        stage_words(in.tps_off, g.tp_lo, g.tp_hi - g.tp_lo + 1, L.tpso);
    }
    if (g.op_hi > g.op_lo) {
        stage_words(in.op_ver, g.op_lo, g.op_hi - g.op_lo, L.opv);
        stage_words(in.ops_off, g.op_lo, g.op_hi - g.op_lo + 1, L.opso);
    }
    g.lds = g.tps_hi - g.tps_lo <= NEEDS_CAP_S && g.ops_hi - g.ops_lo <= NEEDS_CAP_S;
    if (g.lds) {
        stage_words(in.tps_start, g.tps_lo, g.tps_hi - g.tps_lo, L.tpss);
        stage_words(in.tps_end, g.tps_lo, g.tps_hi - g.tps_lo, L.tpse);
        stage_words(in.ops_start, g.ops_lo, g.ops_hi - g.ops_lo, L.opss);
        stage_words(in.ops_end, g.ops_lo, g.ops_hi - g.ops_lo, L.opse);
    }
    __syncthreads();
    return g;
}

__device__ inline NeedsEmit<WView<uint8_t>, WView<uint64_t>> gemit(const corro_needs_out &o) {
    return {WView<uint8_t>{o.kind, 0},   WView<uint64_t>{o.start, 0}, WView<uint64_t>{o.end, 0},
            WView<uint64_t>{o.sr_off, 0}, WView<uint64_t>{o.sr_n, 0}, o.s_start, o.s_end};
}

// Run walk_entry on LDS views when the inputs are staged (and, with FILL, the outputs fit),
// else on global views.
template <bool FILL>
__device__ inline void walk_dispatch(const SyncDev &in, const corro_needs_out &o, const EntryHdr &h, NeedsLds &L,
                                     NeedsOutLds *Lo, const WgSegs &g, uint64_t o_lo, uint64_t nbase, uint64_t sbase,
                                     uint64_t &nn, uint64_t &ns) {
    if (g.lds && (!FILL || !Lo)) {  // staged inputs, outputs (if any) straight to global memory
        using VL = V64S<1>;
        const InViews<VL> iv{VL{L.tns, g.tn_lo},  VL{L.tne, g.tn_lo},  VL{L.ons, g.on_lo},  VL{L.one, g.on_lo},
                             VL{L.tpv, g.tp_lo},  VL{L.tpso, g.tp_lo}, VL{L.tpss, g.tps_lo}, VL{L.tpse, g.tps_lo},
                             VL{L.opv, g.op_lo},  VL{L.opso, g.op_lo}, VL{L.opss, g.ops_lo}, VL{L.opse, g.ops_lo}};
        walk_entry<FILL>(h, iv, gemit(o), nbase, sbase, nn, ns);
    } else if (g.lds) {
        using VL = V64S<1>;
        const InViews<VL> iv{VL{L.tns, g.tn_lo},  VL{L.tne, g.tn_lo},  VL{L.ons, g.on_lo},  VL{L.one, g.on_lo},
                             VL{L.tpv, g.tp_lo},  VL{L.tpso, g.tp_lo}, VL{L.tpss, g.tps_lo}, VL{L.tpse, g.tps_lo},
                             VL{L.opv, g.op_lo},  VL{L.opso, g.op_lo}, VL{L.opss, g.ops_lo}, VL{L.opse, g.ops_lo}};
        NeedsOutLds &O = *Lo;
        const NeedsEmit<WView<uint8_t, 1>, WView<uint64_t, 1>> em{
            WView<uint8_t, 1>{O.kind, o_lo}, WView<uint64_t, 1>{O.start, o_lo}, WView<uint64_t, 1>{O.end, o_lo},
            WView<uint64_t, 1>{O.sro, o_lo}, WView<uint64_t, 1>{O.srn, o_lo}, o.s_start, o.s_end};
        walk_entry<FILL>(h, iv, em, nbase, sbase, nn, ns);
    } else {
        const InViews<V64> iv{V64{in.tn_start, 0}, V64{in.tn_end, 0},  V64{in.on_start, 0},  V64{in.on_end, 0},
                              V64{in.tp_ver, 0},   V64{in.tps_off, 0}, V64{in.tps_start, 0}, V64{in.tps_end, 0},
                              V64{in.op_ver, 0},   V64{in.ops_off, 0}, V64{in.ops_start, 0}, V64{in.ops_end, 0}};
        walk_entry<FILL>(h, iv, gemit(o), nbase, sbase, nn, ns);
    }
}

__device__ inline void flush_needs(const corro_needs_out &o, const NeedsOutLds &L, uint64_t o_lo, uint64_t m) {
    for (uint64_t k = threadIdx.x; k < m; k += NEEDS_T) {
        o.start[o_lo + k] = L.start[k];
        o.end[o_lo + k] = L.end[k];
        o.sr_off[o_lo + k] = L.sro[k];
        o.sr_n[o_lo + k] = L.srn[k];
        o.kind[o_lo + k] = L.kind[k];
    }
}

// Output staging in LDS costs ~33 B of LDS per output need (3 -> 2 workgroups per CU); writing
// straight from the lanes keeps 6 workgroups per CU resident, which hides more latency.
#ifndef NEEDS_OSTAGE
#define NEEDS_OSTAGE 0
#endif
template <bool FILL> struct OutStage { __device__ NeedsOutLds *get() { return nullptr; } };
#if NEEDS_OSTAGE
template <> struct OutStage<true> {
    __device__ NeedsOutLds *get() {
        __shared__ NeedsOutLds Lo;
        return &Lo;
    }
};
#endif

// Two-pass form (corro_compute_needs): pass 0 counts, pass 1 fills at caller-scanned offsets.
template <bool FILL>
__global__ void __launch_bounds__(NEEDS_T) k_needs(SyncDev in, corro_needs_out o) {
    __shared__ NeedsLds L;
    const uint64_t e0 = (uint64_t)blockIdx.x * NEEDS_T;
    const uint64_t e1 = min(in.n, e0 + NEEDS_T);
    const uint64_t e = e0 + threadIdx.x;
    const bool live = e < in.n;
    // per-lane words first, so their latency overlaps the staging below
    const EntryHdr h = load_entry(in, live ? e : e0);
    const uint64_t nbase = FILL ? o.need_off[live ? e : e0] : 0, sbase = FILL ? o.seq_off[live ? e : e0] : 0;
    uint64_t o_lo = 0, o_hi = 0;
    if (FILL) {
        o_lo = o.need_off[e0];
        o_hi = o.need_off[e1];
    }
    const WgSegs g = stage_inputs(in, e0, e1, L);
    NeedsOutLds *Lo = OutStage<FILL>().get();
    if (o_hi - o_lo > NEEDS_CAP_O) Lo = nullptr;
    uint64_t nn = 0, ns = 0;
    if (live) walk_dispatch<FILL>(in, o, h, L, Lo, g, o_lo, nbase, sbase, nn, ns);
    if (!FILL && live) {
        o.need_count[e] = nn;
        o.seq_count[e] = ns;
    }
    if (FILL && g.lds && Lo) {
        __syncthreads();
        flush_needs(o, *Lo, o_lo, o_hi - o_lo);
    }
}

// ---- one-pass form (corro_compute_needs_onepass) ----------------------------------------------
// Each workgroup counts its entries' needs / seq ranges from LDS-staged inputs, scans them across
// the workgroup, obtains the global prefix of every earlier workgroup by a decoupled look-back
// over per-workgroup status words (one chain for needs, one for seq ranges), then re-walks the
// LDS-resident inputs writing its outputs at the now-known offsets. Inputs are read from HBM once.
// Workgroups take their logical index from a ticket counter, so a workgroup only ever waits on
// workgroups that are already running (no dependence on dispatch order).
constexpr uint64_t ST_A = 1ULL << 62, ST_P = 2ULL << 62, ST_VAL = (1ULL << 62) - 1;

__device__ inline uint64_t st_load(const uint64_t *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ inline void st_store(uint64_t *p, uint64_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ inline uint64_t wave_sum(uint64_t v) {
    for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d);
    return v;
}

// Called by one whole wave: sums of both chains over workgroups [0, wg). Status words of one
// workgroup are adjacent (needs, seqs) and published together, so one look-back serves both.
// Each lane inspects LB_PER consecutive predecessors, so one round covers 64 * LB_PER of them (the
// statuses sit in the device-coherent level, a round trip costs ~1-2 us: a wide window makes the
// inclusive-prefix frontier advance that many workgroups per round trip).
constexpr int LB_PER = 1;
__device__ inline void lookback2(const uint64_t *st, int64_t wg, uint64_t &xn, uint64_t &xs) {
    const int lane = threadIdx.x & 63;
    xn = xs = 0;
    int64_t base = wg - 1;  // nearest predecessor not yet summed
    while (true) {
        // lane's chunk: predecessors base - (lane * LB_PER + j), nearest first. Sum the run of
        // aggregates up to the first non-aggregate; a P (inclusive prefix) ends the look-back, an
        // X (not yet published, or the two words caught mid-update) stops the run there.
        uint64_t an = 0, as = 0;
        int first = LB_PER;
        bool isp = false;
#pragma unroll
        for (int j = 0; j < LB_PER; j++) {
            const int64_t idx = base - (lane * LB_PER + j);
            const uint64_t vn = idx >= 0 ? st_load(&st[2 * idx]) : ST_P;
            const uint64_t vs = idx >= 0 ? st_load(&st[2 * idx + 1]) : ST_P;
            const uint64_t sn = vn >> 62;
            const bool agg = sn == 1 && (vs >> 62) == 1;
            const bool pre = sn == 2 && (vs >> 62) == 2;
            if (first == LB_PER) {
                if (agg || pre) {
                    an += vn & ST_VAL;
                    as += vs & ST_VAL;
                }
                if (!agg) {
                    first = j;
                    isp = pre;
                }
            }
        }
        const unsigned long long stop = __ballot(first < LB_PER);
        if (!stop) {
            xn += wave_sum(an);
            xs += wave_sum(as);
            base -= 64 * LB_PER;
            continue;
        }
        const int k = __ffsll(stop) - 1;
        if (lane > k) an = as = 0;
        xn += wave_sum(an);
        xs += wave_sum(as);
        const bool kp = __shfl(isp ? 1 : 0, k);
        if (kp) return;
        const int kf = __shfl(first, k);
        base -= k * LB_PER + kf;  // resume at the unpublished predecessor
        __builtin_amdgcn_s_sleep(2);
    }
}

struct Needs1Args {
    uint64_t *st;        // 2 status words per workgroup (zeroed)
    uint64_t *ticket;    // [0] ticket counter (zeroed), [1] totals: needs, [2] seq ranges
    uint64_t need_cap, seq_cap;
};

__global__ void __launch_bounds__(NEEDS_T) k_needs1(SyncDev in, corro_needs_out o, Needs1Args a) {
    __shared__ NeedsLds L;
    __shared__ uint64_t s_wn[NEEDS_T / 64], s_ws[NEEDS_T / 64];
    __shared__ uint64_t s_base[2];
    __shared__ uint64_t s_wg;
    if (threadIdx.x == 0) s_wg = atomicAdd((unsigned long long *)a.ticket, 1ULL);
    __syncthreads();
    const uint64_t wg = s_wg;
    const uint64_t e0 = wg * NEEDS_T;
    const uint64_t e1 = min(in.n, e0 + NEEDS_T);
    const uint64_t e = e0 + threadIdx.x;
    const bool live = e < in.n;
    const EntryHdr h = load_entry(in, live ? e : e0);
    const WgSegs g = stage_inputs(in, e0, e1, L);
    // count walk (no output)
    uint64_t nn = 0, ns = 0;
    if (live) walk_dispatch<false>(in, o, h, L, nullptr, g, 0, 0, 0, nn, ns);
    // workgroup exclusive scan of (nn, ns)
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    uint64_t in_n = nn, in_s = ns;
    for (int d = 1; d < 64; d <<= 1) {
        const uint64_t yn = __shfl_up(in_n, d), ys = __shfl_up(in_s, d);
        if (lane >= d) {
            in_n += yn;
            in_s += ys;
        }
    }
    if (lane == 63) {
        s_wn[wv] = in_n;
        s_ws[wv] = in_s;
    }
    __syncthreads();
    uint64_t pre_n = 0, pre_s = 0, tot_n = 0, tot_s = 0;
    for (int w = 0; w < (int)(NEEDS_T / 64); w++) {
        if (w < wv) {
            pre_n += s_wn[w];
            pre_s += s_ws[w];
        }
        tot_n += s_wn[w];
        tot_s += s_ws[w];
    }
    const uint64_t lex_n = pre_n + in_n - nn, lex_s = pre_s + in_s - ns;
    // publish the aggregate, look back for the prefix, publish the inclusive prefix
    if (wv == 0) {
        uint64_t bn = 0, bs = 0;
        if (wg == 0) {
            if (lane == 0) {
                st_store(&a.st[0], ST_P | tot_n);
                st_store(&a.st[1], ST_P | tot_s);
            }
        } else {
            if (lane == 0) {
                st_store(&a.st[2 * wg], ST_A | tot_n);
                st_store(&a.st[2 * wg + 1], ST_A | tot_s);
            }
            lookback2(a.st, (int64_t)wg, bn, bs);
            if (lane == 0) {
                st_store(&a.st[2 * wg], ST_P | (bn + tot_n));
                st_store(&a.st[2 * wg + 1], ST_P | (bs + tot_s));
            }
        }
        if (lane == 0) {
            s_base[0] = bn;
            s_base[1] = bs;
        }
    }
    __syncthreads();
    const uint64_t wbn = s_base[0], wbs = s_base[1];
    if (live) {
        const_cast<uint64_t *>(o.need_off)[e] = wbn + lex_n;
        const_cast<uint64_t *>(o.seq_off)[e] = wbs + lex_s;
    }
    if (e1 == in.n && threadIdx.x == 0) {  // last workgroup: closing offsets and totals
        const_cast<uint64_t *>(o.need_off)[in.n] = wbn + tot_n;
        const_cast<uint64_t *>(o.seq_off)[in.n] = wbs + tot_s;
        a.ticket[1] = wbn + tot_n;
        a.ticket[2] = wbs + tot_s;
    }
    // capacity guard: a workgroup whose outputs would not fit writes none (the host reports the
    // totals and the caller re-runs with them)
    if (wbn + tot_n > a.need_cap || wbs + tot_s > a.seq_cap) return;
    NeedsOutLds *Lo = OutStage<true>().get();
    if (tot_n > NEEDS_CAP_O) Lo = nullptr;
    if (live) walk_dispatch<true>(in, o, h, L, Lo, g, wbn, wbn + lex_n, wbs + lex_s, nn, ns);
    if (g.lds && Lo) {
        __syncthreads();
        flush_needs(o, *Lo, wbn, tot_n);
    }
}

// Segment bounds of every workgroup boundary e = w * NEEDS_T (w = 0..nwg), computed by one tiny
// pre-pass so a workgroup reads its whole CSR window -- including the nested partial-seq offsets, a
// chain of two dependent loads -- with two 48-B loads (one latency) before staging its data.
struct WgBound {
    uint64_t tn, on, tp, op, tps, ops;
};
__global__ void __launch_bounds__(256) k_needs_bounds(SyncDev in, uint64_t nwg, WgBound *wb) {
    const uint64_t w = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (w > nwg) return;
    const uint64_t e = min(in.n, w * NEEDS_T);
    WgBound b;
    b.tn = in.tn_off[e];
    b.on = in.on_off[e];
    b.tp = in.tp_off[e];
    b.op = in.op_off[e];
    b.tps = in.tps_off ? in.tps_off[b.tp] : 0;
    b.ops = in.ops_off ? in.ops_off[b.op] : 0;
    wb[w] = b;
}

// stage_inputs with the workgroup's bounds given (one latency fewer per nesting level).
__device__ inline WgSegs stage_inputs_b(const SyncDev &in, const WgBound &b0, const WgBound &b1, NeedsLds &L) {
    WgSegs g;
    g.tn_lo = b0.tn; g.tn_hi = b1.tn;
    g.on_lo = b0.on; g.on_hi = b1.on;
    g.tp_lo = b0.tp; g.tp_hi = b1.tp;
    g.op_lo = b0.op; g.op_hi = b1.op;
    g.tps_lo = b0.tps; g.tps_hi = b1.tps;
    g.ops_lo = b0.ops; g.ops_hi = b1.ops;
    g.lds = g.tn_hi - g.tn_lo <= NEEDS_CAP_R && g.on_hi - g.on_lo <= NEEDS_CAP_R && g.tp_hi - g.tp_lo <= NEEDS_CAP_P &&
            g.op_hi - g.op_lo <= NEEDS_CAP_P && g.tps_hi - g.tps_lo <= NEEDS_CAP_S && g.ops_hi - g.ops_lo <= NEEDS_CAP_S;
#ifdef NEED_NOSTAGE  // experiment: the walk reads global memory (holes in registers)
    g.lds = false;
#endif
    if (!g.lds) return g;  // uniform
    stage_ranges(in.tn_start, in.tn_end, g.tn_lo, g.tn_hi - g.tn_lo, L.tns, L.tne);
    stage_ranges(in.on_start, in.on_end, g.on_lo, g.on_hi - g.on_lo, L.ons, L.one);
    if (g.tp_hi > g.tp_lo) {
        stage_words(in.tp_ver, g.tp_lo, g.tp_hi - g.tp_lo, L.tpv);
        stage_words(in.tps_off, g.tp_lo, g.tp_hi - g.tp_lo + 1, L.tpso);
        stage_words(in.tps_start, g.tps_lo, g.tps_hi - g.tps_lo, L.tpss);
        stage_words(in.tps_end, g.tps_lo, g.tps_hi - g.tps_lo, L.tpse);
    }
    if (g.op_hi > g.op_lo) {
        stage_words(in.op_ver, g.op_lo, g.op_hi - g.op_lo, L.opv);
        stage_words(in.ops_off, g.op_lo, g.op_hi - g.op_lo + 1, L.opso);
        stage_words(in.ops_start, g.ops_lo, g.ops_hi - g.ops_lo, L.opss);
        stage_words(in.ops_end, g.ops_lo, g.ops_hi - g.ops_lo, L.opse);
    }
    __syncthreads();
    return g;
}

// ---- packed one-pass form (corro_compute_needs_packed) ---------------------------------------
// No count pass and no look-back: a workgroup's outputs go to the slots its entries' output BOUNDS
// reserve (corro_needs_bound, per entry: our + their need ranges + their + our partial versions + 1
// need slots; our + their partial seq ranges seq slots -- prefix sums of the input CSR offsets, so
// the workgroup reads them off its own segment bounds), compacted within the workgroup: count walk
// over the LDS-staged inputs, workgroup scan, fill walk. Needs are written as one 16-B pair + a kind
// byte (Partial: {version, first seq slot << 24 | seq ranges}), so a wave's stores cover whole lines.
#ifndef NEED_DIAG  // diagnostics only (results not valid): 1 = no kind stores, 2 = no range stores
#define NEED_DIAG 0
#endif
#ifndef NEED_NT    // 1: non-temporal range stores (experiment)
#define NEED_NT 0
#endif
struct PackedEmit {
    uint64_t *range;
    uint8_t *kind;
    uint64_t *s_start, *s_end;
    __device__ inline void put(uint64_t q, uint64_t a, uint64_t b) const {
#if NEED_NT
        typedef uint64_t v2u __attribute__((ext_vector_type(2)));
        const v2u x = {a, b};
        __builtin_nontemporal_store(x, reinterpret_cast<v2u *>(range + 2 * q));
#else
        *reinterpret_cast<ulonglong2 *>(range + 2 * q) = make_ulonglong2(a, b);
#endif
    }
    __device__ inline void full(uint64_t q, uint64_t s, uint64_t t, uint64_t) const {
        if (!(NEED_DIAG & 2)) put(q, s, t);
        if (!(NEED_DIAG & 1)) kind[q] = 0;
    }
    __device__ inline void partial(uint64_t q, uint64_t v, uint64_t sr, uint64_t cnt) const {
        if (!(NEED_DIAG & 2)) put(q, v, (sr << 24) | cnt);
        if (!(NEED_DIAG & 1)) kind[q] = 1;
    }
    __device__ inline void seq(uint64_t j, uint64_t s, uint64_t t) const {
        s_start[j] = s;
        s_end[j] = t;
    }
};
struct NullEmit {
    __device__ inline void full(uint64_t, uint64_t, uint64_t, uint64_t) const {}
    __device__ inline void partial(uint64_t, uint64_t, uint64_t, uint64_t) const {}
    __device__ inline void seq(uint64_t, uint64_t, uint64_t) const {}
};
// NEED_NB > 0 (measured, not kept): the count walk keeps a lane's first NEED_NB needs in registers
// (Full needs only: a lane with a Partial, or with more needs, walks again to write them itself),
// and after the scan the wave writes the buffered needs of its contiguous output window with
// coalesced stores (each slot fetched from its lane by a cross-lane permute), without a second walk.
// At the 6-waves-per-SIMD register budget the buffers spill: config 4 5.52 ms (NEED_NB 0) vs 6.02 /
// 6.48 / 7.47 ms (2 / 3 / 4), and 10.6 GB written per diff at 4 (profiles/history/r03_sync_need_nb.log).
#ifndef NEED_NB
#define NEED_NB 0
#endif
#if NEED_NB > 0
struct BufEmit {
    uint64_t (&bs)[NEED_NB];
    uint64_t (&bt)[NEED_NB];
    bool &spill;
    __device__ inline void full(uint64_t q, uint64_t s, uint64_t t, uint64_t) const {
#pragma unroll
        for (int k = 0; k < NEED_NB; k++)
            if (q == (uint64_t)k) {
                bs[k] = s;
                bt[k] = t;
            }
        if (q >= NEED_NB) spill = true;
    }
    __device__ inline void partial(uint64_t, uint64_t, uint64_t, uint64_t) const { spill = true; }
    __device__ inline void seq(uint64_t, uint64_t, uint64_t) const {}
};
#endif

template <bool FILL, class E>
__device__ inline void walk_inputs(const SyncDev &in, const EntryHdr &h, const NeedsLds &L, const WgSegs &g,
                                   const E &em, uint64_t nbase, uint64_t sbase, uint64_t &nn, uint64_t &ns) {
    if (g.lds) {
        using VL = V64S<1>;
        const InViews<VL> iv{VL{L.tns, g.tn_lo},  VL{L.tne, g.tn_lo},  VL{L.ons, g.on_lo},  VL{L.one, g.on_lo},
                             VL{L.tpv, g.tp_lo},  VL{L.tpso, g.tp_lo}, VL{L.tpss, g.tps_lo}, VL{L.tpse, g.tps_lo},
                             VL{L.opv, g.op_lo},  VL{L.opso, g.op_lo}, VL{L.opss, g.ops_lo}, VL{L.opse, g.ops_lo}};
        walk_entry<FILL>(h, iv, em, nbase, sbase, nn, ns);
    } else {
        const InViews<V64> iv{V64{in.tn_start, 0}, V64{in.tn_end, 0},  V64{in.on_start, 0},  V64{in.on_end, 0},
                              V64{in.tp_ver, 0},   V64{in.tps_off, 0}, V64{in.tps_start, 0}, V64{in.tps_end, 0},
                              V64{in.op_ver, 0},   V64{in.ops_off, 0}, V64{in.ops_start, 0}, V64{in.ops_end, 0}};
        walk_entry<FILL>(h, iv, em, nbase, sbase, nn, ns);
    }
}

// err[0] |= 1: an entry's needs exceed its bound slots (overlapping input ranges); 2: a partial
// with >= 2^24 seq ranges or a seq slot >= 2^40 (not representable in the packed word)
#ifndef NEEDS_PACKED_WAVES
#define NEEDS_PACKED_WAVES 6  // waves per SIMD the compiler budgets registers for: LDS allows 6
                              // workgroups per CU
#endif
// PackedEmit bounded by the entry's own slots: nothing is written past them (an entry whose needs
// exceed its bound -- overlapping input ranges -- only sets the error)
struct BoundedEmit {
    PackedEmit e;
    uint64_t qlim, slim;
    bool *over;
    __device__ inline void full(uint64_t q, uint64_t s, uint64_t t, uint64_t sr) const {
        if (q < qlim) e.full(q, s, t, sr);
        else *over = true;
    }
    __device__ inline void partial(uint64_t q, uint64_t v, uint64_t sr, uint64_t cnt) const {
        if (q < qlim) e.partial(q, v, sr, cnt);
        else *over = true;
    }
    __device__ inline void seq(uint64_t j, uint64_t s, uint64_t t) const {
        if (j < slim) e.seq(j, s, t);
        else *over = true;
    }
};

// One walk per entry, written straight into the slots its own output bound reserves: entry e's
// needs start at tn_off[e] + on_off[e] + tp_off[e] + op_off[e] + e (the prefix of the per-entry
// bound our + their need ranges + their + our partial versions + 1), its seq ranges at
// tps_off[tp_off[e]] + ops_off[op_off[e]]. Every bound offset is a sum of CSR offsets the lane
// loads anyway, so there is no count walk and no scan (round 2 compacted the slots within each
// 256-entry run: a count walk, a workgroup scan, then the fill walk).
__global__ void __launch_bounds__(NEEDS_T, NEEDS_PACKED_WAVES) k_needs_packed(SyncDev in, corro_needs_packed_out o, uint64_t need_slots,
                                                          uint64_t seq_slots, unsigned long long *err,
                                                          const WgBound *__restrict__ wb) {
    __shared__ NeedsLds L;
#if defined(CORRO_DIAG) && (CORRO_DIAG & 128)
    unsigned long long dt0 = wall_clock64();
#define NDIAG(k) do { if (threadIdx.x == 0) { const unsigned long long t_ = wall_clock64(); atomicAdd(&err[1 + (k)], t_ - dt0); dt0 = t_; } } while (0)
#else
#define NDIAG(k) do { } while (0)
#endif
    const uint64_t e0 = (uint64_t)blockIdx.x * NEEDS_T;
    const uint64_t e = e0 + threadIdx.x;
    const bool live = e < in.n;
    const EntryHdr h = load_entry(in, live ? e : e0);
    const WgBound b0 = wb[blockIdx.x], b1 = wb[blockIdx.x + 1];
    const WgSegs g = stage_inputs_b(in, b0, b1, L);
    NDIAG(0);
    if (!live) return;
    // this entry's bound windows
    const uint64_t nbase = h.tne0 + h.one0 + h.tpe0 + h.ope0 + e;
    const uint64_t nend = h.tne1 + h.one1 + h.tpe1 + h.ope1 + e + 1;
    // nested seq offsets: staged in LDS for the workgroup's partials [lo, hi] (when it has any)
    auto soff = [&](const uint64_t *goff, const uint64_t *loff, uint64_t lo, uint64_t hi, uint64_t k) -> uint64_t {
        return g.lds && hi > lo ? loff[k - lo] : goff[k];
    };
    const uint64_t tps0 = in.tps_off ? soff(in.tps_off, L.tpso, g.tp_lo, g.tp_hi, h.tpe0) : 0;
    const uint64_t tps1 = in.tps_off ? soff(in.tps_off, L.tpso, g.tp_lo, g.tp_hi, h.tpe1) : 0;
    const uint64_t ops0 = in.ops_off ? soff(in.ops_off, L.opso, g.op_lo, g.op_hi, h.ope0) : 0;
    const uint64_t ops1 = in.ops_off ? soff(in.ops_off, L.opso, g.op_lo, g.op_hi, h.ope1) : 0;
    const uint64_t sbase = tps0 + ops0, send = tps1 + ops1;
    bool over = nend > need_slots || send > seq_slots;
    const BoundedEmit em{PackedEmit{o.range, o.kind, o.s_start, o.s_end}, over ? nbase : nend, over ? sbase : send,
                         &over};
    uint64_t nn = 0, ns = 0;
    walk_inputs<true>(in, h, L, g, em, nbase, sbase, nn, ns);
    NDIAG(1);
    o.need_off[e] = nbase;
    o.need_count[e] = (uint32_t)nn;
    if (over || nbase + nn > nend || sbase + ns > send) atomicOr(err, 1ULL);
    if (send >= (1ULL << 40) || nn > 0xFFFFFFFFULL || ns >= (1ULL << 24)) atomicOr(err, 2ULL);
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

extern "C" int corro_needs_bound(corro_ctx *ctx, const corro_sync_entries *in, int mem, uint64_t *need_cap,
                                 uint64_t *seq_cap) {
    if (!ctx || !in || !need_cap || !seq_cap) return fail(CORRO_E_INVALID, "NULL argument");
    if (mem != CORRO_MEM_HOST && mem != CORRO_MEM_DEVICE) return fail(CORRO_E_INVALID, "bad mem kind");
    const uint64_t n = in->n;
    if (n == 0) {
        *need_cap = *seq_cap = 0;
        return CORRO_OK;
    }
    uint64_t w[6] = {0, 0, 0, 0, 0, 0};  // tn, on, tp, op totals, then tps, ops totals
    const uint64_t *offs[4] = {in->tn_off, in->on_off, in->tp_off, in->op_off};
    for (int i = 0; i < 4; i++) {
        if (!offs[i]) return fail(CORRO_E_INVALID, "a required offset array is NULL");
        if (mem == CORRO_MEM_HOST) w[i] = offs[i][n];
        else CORRO_HIP_TRY(hipMemcpy(&w[i], offs[i] + n, 8, hipMemcpyDeviceToHost));
    }
    const uint64_t *soffs[2] = {in->tps_off, in->ops_off};
    const uint64_t sidx[2] = {w[2], w[3]};
    for (int i = 0; i < 2; i++) {
        if (!sidx[i]) continue;
        if (!soffs[i]) return fail(CORRO_E_INVALID, "a partial seq offset array is NULL");
        if (mem == CORRO_MEM_HOST) w[4 + i] = soffs[i][sidx[i]];
        else CORRO_HIP_TRY(hipMemcpy(&w[4 + i], soffs[i] + sidx[i], 8, hipMemcpyDeviceToHost));
    }
    // Full pieces <= our ranges + holes (their ranges + their partial versions) + 1 tail per entry,
    // plus one Partial per our partial version; seq pieces <= our + their partial seq ranges.
    // Exact for disjoint need ranges (RangeInclusiveSet output); the one-pass call reports the
    // true totals if overlapping ranges ever exceed it.
    *need_cap = w[0] + w[1] + w[2] + w[3] + n;
    *seq_cap = w[4] + w[5];
    return CORRO_OK;
}

extern "C" int corro_compute_needs_onepass(corro_ctx *ctx, const corro_sync_entries *in, corro_needs_out *out,
                                         uint64_t need_cap, uint64_t seq_cap, uint64_t *totals) {
    if (!ctx || !in || !out || !totals) return fail(CORRO_E_INVALID, "NULL argument");
    const uint64_t n = in->n;
    totals[0] = totals[1] = 0;
    if (n == 0) return CORRO_OK;
    if (!out->need_off || !out->seq_off) return fail(CORRO_E_INVALID, "need_off / seq_off are NULL");
    if ((need_cap && (!out->kind || !out->start || !out->end || !out->sr_off || !out->sr_n)) ||
        (seq_cap && (!out->s_start || !out->s_end)))
        return fail(CORRO_E_INVALID, "an output array is NULL");
    for (const void *q : {(const void *)in->tn_start, (const void *)in->tn_end, (const void *)in->on_start,
                          (const void *)in->on_end})
        if (q && ((uintptr_t)q % 16) != 0) return fail(CORRO_E_INVALID, "device need-range arrays must be 16-byte aligned");
    CORRO_HIP_TRY(hipSetDevice(ctx->device));
    hipStream_t s = ctx->stream;
    const uint64_t blocks = (n + NEEDS_T - 1) / NEEDS_T;
    if (blocks > 0x7FFFFFFFULL) return fail(CORRO_E_RANGE, "too many sync entries");
    const size_t scratch = (2 * blocks + 4) * 8;
    if (int rc = ctx->d_needs1.ensure(scratch)) return rc;
    uint64_t *ticket = ctx->d_needs1.as<uint64_t>();
    Needs1Args a{ticket + 4, ticket, need_cap, seq_cap};
    SyncDev d{};
    d.n = n;
    d.their_head = in->their_head; d.our_head = in->our_head;
    d.tn_off = in->tn_off; d.tn_start = in->tn_start; d.tn_end = in->tn_end;
    d.tp_off = in->tp_off; d.tp_ver = in->tp_ver;
    d.tps_off = in->tps_off; d.tps_start = in->tps_start; d.tps_end = in->tps_end;
    d.on_off = in->on_off; d.on_start = in->on_start; d.on_end = in->on_end;
    d.op_off = in->op_off; d.op_ver = in->op_ver;
    d.ops_off = in->ops_off; d.ops_start = in->ops_start; d.ops_end = in->ops_end;
    CORRO_HIP_TRY(hipMemsetAsync(ticket, 0, scratch, s));
    if (ctx->profiling) CORRO_HIP_TRY(hipEventRecord(ctx->ev[0], s));
    hipLaunchKernelGGL(k_needs1, dim3((uint32_t)blocks), dim3(NEEDS_T), 0, s, d, *out, a);
    if (ctx->profiling) CORRO_HIP_TRY(hipEventRecord(ctx->ev[1], s));
    CORRO_HIP_TRY(hipGetLastError());
    uint64_t t[2];
    CORRO_HIP_TRY(hipMemcpyAsync(t, ticket + 1, 16, hipMemcpyDeviceToHost, s));
    CORRO_HIP_TRY(hipStreamSynchronize(s));
    if (ctx->profiling) {
        CORRO_HIP_TRY(hipEventElapsedTime(&ctx->last_ms[6], ctx->ev[0], ctx->ev[1]));
        ctx->last_ms[7] = 0.f;
    }
    totals[0] = t[0];
    totals[1] = t[1];
    if (t[0] > need_cap || t[1] > seq_cap)
        return fail(CORRO_E_RANGE, "need output exceeds the given capacity (totals hold the sizes to re-run with)");
    return CORRO_OK;
}

extern "C" int corro_compute_needs_packed(corro_ctx *ctx, const corro_sync_entries *in, corro_needs_packed_out *out,
                                          uint64_t need_slots, uint64_t seq_slots) {
    if (!ctx || !in || !out) return fail(CORRO_E_INVALID, "NULL argument");
    const uint64_t n = in->n;
    if (n == 0) return CORRO_OK;
    if (!out->need_off || !out->need_count || (need_slots && (!out->range || !out->kind)) ||
        (seq_slots && (!out->s_start || !out->s_end)))
        return fail(CORRO_E_INVALID, "an output array is NULL");
    if ((uintptr_t)out->range % 16) return fail(CORRO_E_INVALID, "range must be 16-byte aligned");
    for (const void *q : {(const void *)in->tn_start, (const void *)in->tn_end, (const void *)in->on_start,
                          (const void *)in->on_end})
        if (q && ((uintptr_t)q % 16) != 0) return fail(CORRO_E_INVALID, "device need-range arrays must be 16-byte aligned");
    CORRO_HIP_TRY(hipSetDevice(ctx->device));
    hipStream_t s = ctx->stream;
    const uint64_t blocks = (n + NEEDS_T - 1) / NEEDS_T;
    if (blocks > 0x7FFFFFFFULL) return fail(CORRO_E_RANGE, "too many sync entries");
    if (int rc = ctx->d_needs1.ensure(64 + (blocks + 1) * sizeof(WgBound))) return rc;
    unsigned long long *err = ctx->d_needs1.as<unsigned long long>();
    WgBound *wb = reinterpret_cast<WgBound *>(ctx->d_needs1.as<uint8_t>() + 64);
    SyncDev d{};
    d.n = n;
    d.their_head = in->their_head; d.our_head = in->our_head;
    d.tn_off = in->tn_off; d.tn_start = in->tn_start; d.tn_end = in->tn_end;
    d.tp_off = in->tp_off; d.tp_ver = in->tp_ver;
    d.tps_off = in->tps_off; d.tps_start = in->tps_start; d.tps_end = in->tps_end;
    d.on_off = in->on_off; d.on_start = in->on_start; d.on_end = in->on_end;
    d.op_off = in->op_off; d.op_ver = in->op_ver;
    d.ops_off = in->ops_off; d.ops_start = in->ops_start; d.ops_end = in->ops_end;
    CORRO_HIP_TRY(hipMemsetAsync(err, 0, 64, s));
    if (ctx->profiling) CORRO_HIP_TRY(hipEventRecord(ctx->ev[0], s));
    hipLaunchKernelGGL(k_needs_bounds, dim3((uint32_t)((blocks + 1 + 255) / 256)), dim3(256), 0, s, d, blocks, wb);
    hipLaunchKernelGGL(k_needs_packed, dim3((uint32_t)blocks), dim3(NEEDS_T), 0, s, d, *out, need_slots, seq_slots, err,
                       (const WgBound *)wb);
    if (ctx->profiling) CORRO_HIP_TRY(hipEventRecord(ctx->ev[1], s));
    CORRO_HIP_TRY(hipGetLastError());
    unsigned long long e = 0;
    CORRO_HIP_TRY(hipMemcpyAsync(&e, err, 8, hipMemcpyDeviceToHost, s));
    CORRO_HIP_TRY(hipStreamSynchronize(s));
    if (ctx->profiling) {
        CORRO_HIP_TRY(hipEventElapsedTime(&ctx->last_ms[6], ctx->ev[0], ctx->ev[1]));
        ctx->last_ms[7] = 0.f;
    }
#if defined(CORRO_DIAG) && (CORRO_DIAG & 128)
    {
        unsigned long long ph[5];
        CORRO_HIP_TRY(hipMemcpy(ph, err, 40, hipMemcpyDeviceToHost));
        fprintf(stderr, "NDIAG us per workgroup: staging %.3f count %.3f scan %.3f fill %.3f\n", ph[1] / 100.0 / blocks,
                ph[2] / 100.0 / blocks, ph[3] / 100.0 / blocks, ph[4] / 100.0 / blocks);
    }
#endif
    if (e & 1) return fail(CORRO_E_RANGE, "needs exceed their bound slots (overlapping need ranges: use corro_compute_needs)");
    if (e & 2) return fail(CORRO_E_RANGE, "a partial's seq ranges do not fit the packed need word");
    return CORRO_OK;
}
