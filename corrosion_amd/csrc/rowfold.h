// Parallel per-row fold of the general merge body (causal lengths, deletes, resurrects), for the
// rows that make a bucket overflow (Zipf-hot rows: tens of thousands of changes in one row). The
// sequential body (gen_fold_row) walks a row one change at a time in one lane, which for such a
// row is a chain of dependent scratch loads; here every step over a row's CHANGES is a
// workgroup-wide scan or reduction, and only a walk over the row's RECORDS (the changes that
// raise the causal length: at most one per distinct cl value) is sequential.
//
// Per row, with changes sorted by application position (prior state first, as a prefix):
//   L_i     = exclusive running max of cl                          (segmented max-scan)
//   kind_i  = record (cl_i > L_i) | candidate (cl_i == L_i, odd, column change) | no-op
//   epoch_i = index of the last record at or before i              (segmented count)
//   W(e, c) = argmax over the epoch's candidates of cid c of (col_version, value, site id),
//             earliest on ties                                     (LDS/global atomic-max stages)
//   walk over records: a delete drops the cells, an odd record zeroes them (cv -> 0, value and
//   metadata kept) and a column record then sets its own cell; each W(e, c) replaces the carried
//   cell when strictly greater.
//   impacts: records 1 (2 for a column record that resurrects), candidates 1 iff strictly greater
//   than the epoch's first element of their cell and every earlier candidate of it (segmented
//   prefix argmax over the candidates sorted by (group, position)), everything else 0.
// This equals cr-sqlite's sequential rules whenever every sentinel and even-cl
// change carries col_version == cl (App. A.3, what cr-sqlite itself produces): L then only grows
// by max. Rows that break it keep the sequential fold. Checked against the oracle on random
// batches by tools/proto_rowfold.py (same formulation on the CPU) and tests/test_gpu_merge.py.
#pragma once
#include "internal.h"

namespace corro {

constexpr uint32_t RF_NONE = 0xFFFFFFFFu;

struct FoldArrays {
    uint32_t *lx;      // sorted position: L before the change
    uint32_t *ep;      // sorted position: epoch index (RF_NONE before the row's first record)
    uint32_t *kind;    // sorted position: 0 no-op, 1 record, 2 candidate
    uint32_t *rstart;  // row id: first sorted position
    uint32_t *rbad;    // row id: 1 = keep the sequential fold
    uint32_t *rnrec;   // row id: number of records
    uint32_t *recs;    // rstart + k: sorted position of the row's k-th record
    uint32_t *gid;     // sorted position (candidate): group owner position
    uint32_t *alive;   // sorted position (candidate): still a possible argmax
    uint32_t *win;     // group owner: winning candidate position
    uint32_t *fst;     // group owner: the epoch's first element of the cell (pos + 1 | zeroed << 31)
    uint32_t *head;    // record position: groups of its epoch (owner + 1), linked through nxt
    uint32_t *nxt;
    uint32_t *scid, *spos, *sz;  // walk state of a row: cells at [rstart, rstart + ncell)
    uint32_t *cval;              // candidate sort payload
    uint32_t *gslot;             // group hash slots
    uint32_t *vmeta, *srank;     // record index: value meta, site rank
    uint64_t *gk;                // group owner: stage key
    uint64_t *vk0, *vk1;         // record index: value words
    uint64_t *ckey;              // candidate sort keys: group << 32 | position
    uint32_t gslots, Pc;
    uint32_t kbase;              // added to row / group ids in the device-wide sort keys
};

// Block-wide segmented exclusive scan over [0, n) (all threads of the workgroup call it). A
// segment starts at j where start(j); elem(j) is combined left to right with comb; out(j, excl)
// receives the combination of the segment's elements before j (ident at a segment start).
// Chunked: C consecutive positions per thread, a Hillis-Steele scan of the chunk summaries in
// LDS (s_f, s_m: 2 x blockDim words each), then a local pass.
template <class Elem, class Comb, class Start, class Out>
__device__ inline void rf_seg_scan(uint32_t n, uint32_t ident, Elem elem, Comb comb, Start start, Out out,
                                   uint32_t *s_f, uint32_t *s_m) {
    const uint32_t tid = threadIdx.x, nth = blockDim.x;
    const uint32_t C = (n + nth - 1) / nth;
    const uint32_t j0 = min(n, tid * C), j1 = min(n, j0 + C);
    uint32_t f = 0, m = ident;
    for (uint32_t j = j0; j < j1; j++) {
        if (start(j)) {
            f = 1;
            m = ident;
        }
        m = comb(m, elem(j));
    }
    s_f[tid] = f;
    s_m[tid] = m;
    __syncthreads();
    // inclusive scan of (f, m) pairs: (f1, m1) . (f2, m2) = (f1 | f2, f2 ? m2 : comb(m1, m2))
    uint32_t cur = 0;
    for (uint32_t d = 1; d < nth; d <<= 1) {
        const uint32_t nf = cur ^ 1;
        uint32_t ff = s_f[cur * nth + tid], mm = s_m[cur * nth + tid];
        if (tid >= d) {
            const uint32_t pf = s_f[cur * nth + tid - d], pm = s_m[cur * nth + tid - d];
            mm = ff ? mm : comb(pm, mm);
            ff = ff | pf;
        }
        s_f[nf * nth + tid] = ff;
        s_m[nf * nth + tid] = mm;
        cur = nf;
        __syncthreads();
    }
    uint32_t run = tid ? s_m[cur * nth + tid - 1] : ident;  // exclusive carry into this chunk
    __syncthreads();
    for (uint32_t j = j0; j < j1; j++) {
        if (start(j)) run = ident;
        out(j, run);
        run = comb(run, elem(j));
    }
    __syncthreads();
}

// Carve the overflow scratch of one bucket (n records): the GenArrays of the sequential body plus
// the FoldArrays, except the sort arrays (g.key / g.val, F.ckey / F.cval), which live in the
// device-wide segmented-sort buffers. Host (base = nullptr) uses it for sizing; returns the bytes.
__host__ __device__ inline uint64_t carve_ovf(uint8_t *base, uint64_t n, GenArrays *g, FoldArrays *f) {
    uint64_t S = 1;
    while (S < 2 * n) S <<= 1;
    uint64_t off = 0;
    auto take = [&](uint64_t bytes) {
        uint8_t *q = base ? base + off : nullptr;
        off += (bytes + 15) & ~15ULL;
        return q;
    };
    GenArrays gg{};
    FoldArrays ff{};
    gg.pk = (uint64_t *)take(n * 8);
    gg.cv = (int64_t *)take(n * 8);
    gg.ccv = (int64_t *)take(n * 8);
    gg.own = (uint32_t *)take(S * 4);
    gg.tc = (uint32_t *)take(n * 4);
    gg.cl = (uint32_t *)take(n * 4);
    gg.pos = (uint32_t *)take(n * 4);
    gg.ccid = (uint32_t *)take(n * 4);
    gg.csrc = (uint32_t *)take(n * 4);
    gg.slots = (uint32_t)S;
    gg.P = (uint32_t)n;
    ff.lx = (uint32_t *)take(n * 4);
    ff.ep = (uint32_t *)take(n * 4);
    ff.kind = (uint32_t *)take(n * 4);
    ff.rstart = (uint32_t *)take(n * 4);
    ff.rbad = (uint32_t *)take(n * 4);
    ff.rnrec = (uint32_t *)take(n * 4);
    ff.recs = (uint32_t *)take(n * 4);
    ff.gid = (uint32_t *)take(n * 4);
    ff.alive = (uint32_t *)take(n * 4);
    ff.win = (uint32_t *)take(n * 4);
    ff.fst = (uint32_t *)take(n * 4);
    ff.head = (uint32_t *)take(n * 4);
    ff.nxt = (uint32_t *)take(n * 4);
    ff.scid = (uint32_t *)take(n * 4);
    ff.spos = (uint32_t *)take(n * 4);
    ff.sz = (uint32_t *)take(n * 4);
    ff.vmeta = (uint32_t *)take(n * 4);
    ff.srank = (uint32_t *)take(n * 4);
    ff.gslot = (uint32_t *)take(S * 4);
    ff.gk = (uint64_t *)take(n * 8);
    ff.vk0 = (uint64_t *)take(n * 8);
    ff.vk1 = (uint64_t *)take(n * 8);
    ff.gslots = (uint32_t)S;
    ff.Pc = (uint32_t)n;
    if (g) *g = gg;
    if (f) *f = ff;
    return off;
}

}  // namespace corro
