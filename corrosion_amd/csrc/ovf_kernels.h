// Overflow path, device-wide: the buckets too large for a workgroup's LDS, or holding a long row
// (Zipf-hot rows: tens of thousands of changes in one row), are folded by kernels that span the
// whole GPU, so a bucket of a million changes is not one CU's work, and a hot row is not a chain
// of dependent loads in one lane. Every per-record / per-position / per-row array is global.
// Records [0, Kb) are the oversized buckets' batch changes (bucket k at koff[k]); their rows get
// dense ids (bucket-major), each row is looked up once in its region, and the prior clock records
// of the rows found are appended as records [Kb, K) (read from the heap), so the sort by (row,
// position) places them first in their row -- the prior state as a prefix of the application order.
//
// Parallel row fold. Per row, with changes sorted by application position
// (prior state first, as a prefix):
//   L_i     = exclusive running max of cl                          (segmented max-scan)
//   kind_i  = record (cl_i > L_i) | candidate (cl_i == L_i, odd, column change) | no-op
//   epoch_i = index of the last record at or before i              (segmented count)
//   W(e, c) = argmax over the epoch's candidates of cid c of (col_version, value, site id),
//             earliest on ties                                     (segmented argmax-scan)
//   walk over records: a delete drops the cells, an odd record zeroes them (cv -> 0, value and
//   metadata kept) and a column record then sets its own cell; each W(e, c) replaces the carried
//   cell when strictly greater.
//   impacts: records 1 (2 for a column record that resurrects), candidates 1 iff strictly greater
//   than the epoch's first element of their cell and every earlier candidate of it, else 0.
// This equals cr-sqlite's sequential rules (App. A.1) whenever every sentinel and even-cl change
// carries col_version == cl (App. A.3, what cr-sqlite itself produces): L then only grows by max.
// Rows that break it keep the sequential fold (gen_fold_row). The formulation was checked against the oracle on random batches on the CPU
// (tools/proto_rowfold.py); tests/test_gpu_merge.py checks this implementation.
//
// Phases:
//   k_ovf_loadhash                  fields; row owners (open addressing per bucket, read-before-CAS)
//   scan of owner flags               dense row ids
//   k_ovf_lookup, scan, k_ovf_pload   each row looked up in its region (new rows counted per bucket
//                                     for the host's capacity check), prior records appended
//   [no impacts] (row summaries in k_ovf_lookup / k_ovf_pload), k_ovf_keep  row reduction: a row
//                                     whose last epoch covers every cid it holds keeps only the
//                                     records at its largest cl (below)
//   (k_ovf_lookup also writes the batch records' sort keys: dense row << rshift | compact position,
//   prior slots [0, pm), then the batch in application order: log2(rows) + log2(pm + batch) bits)
//   radix sort by (row, position)                                       [prims.hip, rocPRIM]
//   k_ovf_gather                    cl in sorted order, row starts
//   exclusive max-scan of cl by row -> L                                [rocPRIM scan_by_key]
//   k_ovf_classify                  record / candidate / no-op, record impacts, App. A.3 check
//   inclusive count of records by row -> epoch
//   k_ovf_epochs, k_ovf_ckeys       the row's record list; candidate keys (epoch's record, cid)
//   k_ovf_ccompact                  the candidates compacted (scan of flags), then a stable radix
//                                   sort by (epoch, cid): a group keeps application order; the
//                                   rest of the sorted key array is ~0
//   k_ovf_cgather                   the candidates' cell keys in candidate-sorted order
//   k_cscan_*                       inclusive argmax-scan by group (-> W and every prefix), keys
//                                   compared in registers; group start = plain max-scan of the
//                                   group heads' indices [prims.hip]
//   k_ovf_link                      each group's end is linked under its epoch's record
//   k_ovf_walk                      one thread per row: the walk over its records, the row written
//                                   back to its heap slot (found or inserted in its region); rows
//                                   outside App. A.3 run the sequential fold instead
//   k_ovf_impacts                   candidate impacts (strict prefix max, seeded by the epoch's
//                                   first element of the cell)
//   k_ovf_finish                    region fill counts
#pragma once

namespace corro {

// Cell key (col_version, value order, site rank) of a change; `z` = the carried cell of a
// resurrected row (col_version 0, value and metadata kept). 32 B: two 16-B loads from one line.
struct alignas(16) OvfKey {
    int64_t cv;
    uint64_t k0, k1;
    uint32_t m, sr;
};

// a row's summary words by its owner record (the fused form; one 32-B line: k_ovf_keep<true> reads
// them, and the row's dense id, with two 16-B loads)
struct alignas(32) OvfSum {
    unsigned long long w1, w3;  // rs_comb's word; Mx << 32 | ~(first compact position at Mx)
    uint32_t w2, row;           // cids | outside App. A.3; the dense row (k_ovf_owners)
    uint32_t pad[2];
};

struct OvfDev {
    uint32_t G, K;              // oversized buckets, their records (batch + prior)
    uint32_t Kb;                // batch records [0, Kb); prior records [Kb, K)
    uint32_t cid_bits;          // a candidate key is (epoch's record position) << cid_bits | cid
    uint32_t rshift;            // a record's sort key is dense row << rshift | compact position
    uint32_t pm;                // compact position of batch change i: pm + i (prior records: slot < pm)
    uint32_t ncand;             // candidates: candidate-sorted indices [0, ncand) (the rest of ckey_s is ~0)
    uint32_t nrows;             // rows (dense ids [0, nrows))
    const uint32_t *koff;       // [G + 1] bucket base offsets of the batch records
    const uint32_t *slot_off;   // [G] row-hash slot region, next_pow2(2 n) words each
    // per record (global index)
    uint64_t *pk;               // (row owners only)
    int64_t *cv;
    uint32_t *tc, *cl, *pos;
    uint32_t *src;              // batch record: its staged index; prior record: its heap index
    // per sorted position
    uint64_t *key, *key_s;
    uint32_t *val, *val_s;      // global record index
    uint32_t *rowid, *cl_s, *lx, *recf, *epc, *kind, *pb;
    // per row (dense id)
    uint32_t *rstart, *rbad, *rnrec, *recs, *head;
    uint32_t *rowner, *rb, *rheap, *rprior, *rpoff;  // owner record, bucket, prior heap slot, prior records
    uint64_t *rbits;                                 // [2 * nrows] prior presence bits
    uint32_t *scid, *spos, *sz;  // walk state at [rstart, rstart + ncell)
    uint32_t *ccid, *csrc;       // sequential-fold scratch (GenArrays)
    int64_t *ccv;
    // candidates
    uint64_t *ckey, *ckey_s;
    uint32_t *cval, *cval_s, *cbest, *cgs, *nxt, *fstg;
    // candidates' cell keys gathered in candidate-sorted order (the argmax scan reads neighbours)
    OvfKey *qkey;
    OvfKey *pkey;                // [K - Kb] the prior records' keys, read before the walk rewrites their slots
    uint32_t *slots;
    uint32_t *bnew, *bnrec;      // [G] new rows / their heap records per bucket
    const uint8_t *arena;        // long value bytes (MergeArgs::arena)
    // row reduction (no impacts): per row the largest cl, whether any record is outside App. A.3,
    // the cids of all its column records and of its column records at that cl with col_version > 0
    uint32_t reduce;             // 1: rows are reduced to their last epoch's records before the sort
    uint64_t *rw1;               // [nrows] Mx << 32 | cids at Mx (rs_comb)
    uint32_t *rw2;               // [nrows] cids | outside App. A.3
    uint32_t *nkeep;             // [1] records kept; [1]: dropped candidates (impact form)
    uint32_t *cbk;               // [8 (Kb / 64 + 1)] bucket of batch record 64 c and its words (k_ovf_chunkmap)
    // impact form of the reduction (rimp): per row OVF_NCL causal-length slots, the first compact
    // position of each causal length (cl << 32 | position, ~0 free) and the record at it; the
    // dropped candidates' sort key = ((row * OVF_NCL + slot) << cid_bits | cid) << rshift | position
    uint32_t rimp;
    uint32_t split;              // 1: the rows' region lookups run in k_ovf_rlook (one lane per row)
    uint64_t *rcl;               // [nrows * OVF_NCL]
    uint32_t *rclr;              // [nrows * OVF_NCL]
    // fused plain form (fuse = 1: row reduction without impacts). The summaries are built in the
    // pass that loads the records and finds their row owners, keyed by the owner record's index
    // (dense rows are not known yet): osum is a persistent [Kb] area that is zero between applies
    // (the walks clear each row's words after use). w3 = Mx << 32 | ~(first compact position at Mx)
    // (max monoid): the epoch record of a reduced row. Reduced rows then go around the
    // (row, position) sort: their column records at Mx are sorted by (owner record, cid) only and each
    // cell's winner is an argmax with the position as the last tie-break (earliest wins), so their
    // order in the sort does not matter.
    uint32_t fuse;
    OvfSum *osum;                // [Kb] (fuse; rs_put writes here when set)
    uint32_t obits;              // (fuse) bits of an owner record index: the cell key is owner << cid_bits | cid
    uint32_t *rlist, *flist;     // [nrows] reduced rows / the others (k_ovf_keep<true>), counts at nkeep[2..3]
    uint64_t *rsum;              // [nrows] a reduced row's Mx << 32 | cids (fuse)
    uint32_t *rowE;              // [nrows] a reduced row's epoch record (fuse)
    uint32_t *rhb, *rclw;        // [nrows] a reduced row's heap slot and clock-row cl (k_ovf_walk mode 1, for k_ovf_rcells)
    uint32_t cstride;
    const uint32_t *qpos;        // argmax tie-break positions, by sorted index (fuse; nullptr: order decides)
};

// a record's 64-B source: the staged batch change or the prior heap record
__device__ inline const Rec *ovf_rec(const MergeArgs &a, const OvfDev &d, uint32_t x) {
    return x < d.Kb ? a.stage + d.src[x] : a.rs.heap + d.src[x];
}

// the view gen_fold_row / heap_write_row read records through (record = global index)
struct OvfView {
    const MergeArgs *a;
    const OvfDev *d;
    __device__ inline const Rec *at(uint32_t x) const { return ovf_rec(*a, *d, x); }
    __device__ inline uint64_t prior_ts(const Rec &r) const { return a->rs.heap_ts ? a->rs.heap_ts[r.pos] : 0ULL; }
};

__device__ inline uint32_t ovf_bucket_of(const OvfDev &d, uint32_t r) {
    uint32_t lo = 0, hi = d.G;  // koff[lo] <= r < koff[hi]
    while (hi - lo > 1) {
        const uint32_t m = (lo + hi) >> 1;
        if (d.koff[m] <= r) lo = m;
        else hi = m;
    }
    return lo;
}

// by sorted position p
// (the value words, metadata and site of a record are read from its 64-B source record: only
// candidates and carried cells need them, a small part of the overflow records)
__device__ inline OvfKey ovf_key_rec(const MergeArgs &a, const OvfDev &d, uint32_t p, bool z) {
    const uint32_t x = d.val_s[p];
    if (x >= d.Kb) {  // a prior clock: its heap slot may already hold the row's new value
        OvfKey k = d.pkey[x - d.Kb];
        if (z) k.cv = 0;
        return k;
    }
    const Rec r = load_rec(ovf_rec(a, d, x));
    return OvfKey{z ? 0 : r.cv, r.v0, r.v1, r.meta, site_rank_of(a, r.site)};
}

__device__ inline OvfKey ovf_key_p(const MergeArgs &a, const OvfDev &d, uint32_t p, bool z) {
    return ovf_key_rec(a, d, p, z);
}

// by candidate-sorted index q
__device__ inline OvfKey ovf_key_q(const OvfDev &d, uint32_t q) {
    return d.qkey[q];
}

// >0: a greater
__device__ inline int ovf_kcmp(const OvfKey &a, const OvfKey &b, const uint8_t *arena) {
    if (a.cv != b.cv) return a.cv > b.cv ? 1 : -1;
    const int vc = value_cmp_f(a.m, a.k0, a.k1, b.m, b.k0, b.k1, arena);
    if (vc != 0) return vc;
    if (a.sr != b.sr) return a.sr > b.sr ? 1 : -1;
    return 0;
}

#define OVF_LOOP(i, N) for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < (N); i += gridDim.x * blockDim.x)

// ---- the fold's plan, on the device (one workgroup each; these were host loops over pinned
// readbacks of the bucket lists: ~0.25 ms and ~0.06 ms at 32 K buckets, the GPU idle meanwhile) ----
constexpr uint32_t PLAN_T = 1024;  // (x PLAN_PER buckets per thread: up to 32 K queued buckets)

// next_pow2(2 n), 1 for n = 0 (the host's former `while (sl < 2 n) sl <<= 1` from sl = 1)
__device__ inline unsigned long long ovf_slots_for(unsigned long long n) {
    return n ? 1ULL << (64 - __clzll((long long)(2 * n - 1))) : 1ULL;
}

// exclusive scan across the 1024-thread workgroup; `total` = the sum of every x
__device__ inline unsigned long long plan_scan(unsigned long long x, unsigned long long *s_w, unsigned long long &total) {
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    unsigned long long incl = x;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const unsigned long long y = __shfl_up(incl, o);
        if ((int)lane >= o) incl += y;
    }
    if (lane == 63) s_w[w] = incl;
    __syncthreads();
    if (w == 0) {
        unsigned long long v = lane < PLAN_T / 64 ? s_w[lane] : 0ULL;
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) {
            const unsigned long long y = __shfl_up(v, o);
            if ((int)lane >= o) v += y;
        }
        if (lane < PLAN_T / 64) s_w[lane] = v;
    }
    __syncthreads();
    total = s_w[PLAN_T / 64 - 1];
    return (w ? s_w[w - 1] : 0ULL) + incl - x;
}

// per queued bucket k (b = list[k]): its batch records at koff[k] (exclusive scan of the counts), its
// row-table slots next_pow2(2 n) at soff[k]; tot[0..2] = records, slots, the buckets' region rows
static __global__ void __launch_bounds__(PLAN_T) k_ovf_plan(const uint32_t *__restrict__ list, const uint32_t *__restrict__ nc,
                                                            const uint32_t *__restrict__ used, uint32_t novf,
                                                            uint32_t *__restrict__ koff, uint32_t *__restrict__ soff,
                                                            unsigned long long *__restrict__ tot) {
    __shared__ unsigned long long s_a[PLAN_T / 64], s_b[PLAN_T / 64], s_c[PLAN_T / 64];
    const uint32_t per = (novf + PLAN_T - 1) / PLAN_T;  // <= PLAN_PER (the host checks)
    const uint32_t k0 = min(novf, threadIdx.x * per), k1 = min(novf, k0 + per);
    // the buckets' counts staged in LDS by coalesced strided loads (independent, so they overlap),
    // then each thread scans its contiguous range from LDS
    __shared__ uint32_t s_n[PLAN_T * PLAN_PER];
    unsigned long long sn = 0, ss = 0, su = 0;
#pragma unroll 8
    for (uint32_t k = threadIdx.x; k < novf; k += PLAN_T) {
        const uint32_t b = list[k];
        s_n[k] = nc[b];
        su += used[b];
    }
    __syncthreads();
    for (uint32_t k = k0; k < k1; k++) {
        sn += s_n[k];
        ss += ovf_slots_for(s_n[k]);
    }
    unsigned long long tn, ts, tu;
    unsigned long long bn = plan_scan(sn, s_a, tn), bs = plan_scan(ss, s_b, ts);
    plan_scan(su, s_c, tu);
    for (uint32_t k = k0; k < k1; k++) {
        koff[k] = (uint32_t)bn;
        soff[k] = (uint32_t)bs;
        bn += s_n[k];
        bs += ovf_slots_for(s_n[k]);
    }
    if (threadIdx.x == 0) {
        koff[novf] = (uint32_t)tn;
        tot[0] = tn;
        tot[1] = ts;
        tot[2] = tu;
    }
}

// room for the new rows: tot[3] = the largest region fill the buckets' new rows ask for, tot[4] =
// their heap records
static __global__ void __launch_bounds__(PLAN_T) k_ovf_room(const uint32_t *__restrict__ list, const uint32_t *__restrict__ used,
                                                            const uint32_t *__restrict__ bnew, const uint32_t *__restrict__ bnrec,
                                                            uint32_t novf, unsigned long long *__restrict__ tot) {
    __shared__ unsigned long long s_m[PLAN_T / 64], s_r[PLAN_T / 64];
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    unsigned long long mx = 0, sr = 0;
    for (uint32_t k = threadIdx.x; k < novf; k += PLAN_T) {
        mx = max(mx, (unsigned long long)used[list[k]] + bnew[k]);
        sr += bnrec[k];
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
        mx = max(mx, (unsigned long long)__shfl_xor(mx, o));
        sr += __shfl_xor(sr, o);
    }
    if (lane == 0) {
        s_m[w] = mx;
        s_r[w] = sr;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (uint32_t v = 1; v < PLAN_T / 64; v++) {
            mx = max(mx, s_m[v]);
            sr += s_r[v];
        }
        tot[3] = mx;
        tot[4] = sr;
    }
}

// the bucket of every 64th batch record and the words its records need (a record's bucket is then
// its chunk's, or a step or two past it: the binary search over koff is one dependent chain of ~15
// loads, and the bucket's words -- record range, staged base, row-table slice -- another three)
// chunk c: b, koff[b], koff[b + 1], staged base, row-table offset, row-table size, -, -
struct ChunkB {
    uint32_t b, kb, ke, sbase, soff, S;
};

__device__ inline ChunkB ovf_chunk_words(const MergeArgs &a, const OvfDev &d, uint32_t b) {
    ChunkB c;
    c.b = b;
    c.kb = d.koff[b];
    c.ke = d.koff[b + 1];
    c.sbase = a.stage_off[a.ovf_list[b]];
    c.soff = d.slot_off[b];
    uint32_t S = 1;
    while (S < 2 * (c.ke - c.kb)) S <<= 1;
    c.S = S;
    return c;
}

static __global__ void k_ovf_chunkmap(MergeArgs a, OvfDev d) {
    OVF_LOOP(c, (d.Kb + 63) / 64) {
        const ChunkB x = ovf_chunk_words(a, d, ovf_bucket_of(d, c * 64));
        uint4 *o = (uint4 *)d.cbk + 2 * c;
        o[0] = make_uint4(x.b, x.kb, x.ke, x.sbase);
        o[1] = make_uint4(x.soff, x.S, 0u, 0u);
    }
}

// a batch record's bucket words: its chunk's, unless the chunk crosses into a later bucket
__device__ inline ChunkB ovf_chunk_of(const MergeArgs &a, const OvfDev &d, uint32_t r) {
    const uint4 *m = (const uint4 *)d.cbk + 2 * (r >> 6);
    const uint4 x = m[0], y = m[1];
    if (r < x.z) return ChunkB{x.x, x.y, x.z, x.w, y.x, y.y};
    uint32_t b = x.x + 1;
    while (d.koff[b + 1] <= r) b++;
    return ovf_chunk_words(a, d, b);
}

// A batch record's row owner (the bucket-local index of the row's first claimant): open addressing
// per bucket, a slot read before it is claimed; an occupied slot's row key is compared with the
// claimant's staged record (read-only while owners are found, so no ordering against the claimant's
// own field writes). Called by every lane of the wave (`todo`: the lane has a record).
__device__ inline uint32_t ovf_find_owner(const MergeArgs &a, const OvfDev &d, bool todo, uint32_t r, const ChunkB &cb,
                                          uint64_t pk, uint32_t t) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t kb = cb.kb, sbase = cb.sbase, S = cb.S;
    uint32_t *slots = d.slots + cb.soff;
    auto probe = [&]() -> uint32_t {
        uint32_t slot = row_hash(pk, t) & (S - 1);
        while (true) {
            // a plain read first: a claimed slot is only read afterwards
            uint32_t o = slots[slot];
            if (o == 0) o = atomicCAS(&slots[slot], 0u, r - kb + 1);
            if (o == 0) return r - kb;
            const Rec *q = a.stage + sbase + (o - 1);
            if (q->pk == pk && (q->tcid >> 16) == t) return o - 1;
            slot = (slot + 1) & (S - 1);
        }
    };
    // A Zipf-hot row fills whole waves, and all of its lanes start at once: every one of them
    // would read the unclaimed slot and CAS it, a chain of serialised same-address atomics
    // as long as the row. Lanes of one wave that share a row let one leader probe for them.
    uint32_t owner = 0;
    for (int round = 0; round < 2; round++) {
        const uint64_t act = __ballot(todo);
        if (!act) break;
        const int leader = __ffsll((unsigned long long)act) - 1;
        const uint64_t lpk = __shfl(pk, leader);
        const uint32_t lt = __shfl(t, leader);
        const bool mine = todo && pk == lpk && t == lt;
        if (__popcll(__ballot(mine)) < 8) break;  // (wave-uniform) not a hot row
        uint32_t o = 0;
        if ((int)lane == leader) o = probe();
        o = __shfl(o, leader);
        if (mine) {
            owner = o;
            todo = false;
        }
    }
    if (todo) owner = probe();
    return owner;
}

// Record fields and row owners in one pass: each batch record's fields are loaded from its staged
// 64-B record and the record is hashed into its bucket's row table (ovf_find_owner).
static __global__ void k_ovf_loadhash(MergeArgs a, OvfDev d) {
    OVF_LOOP(r, d.Kb) {
        const ChunkB cb = ovf_chunk_of(a, d, r);
        const uint32_t kb = cb.kb;
        const uint32_t si = cb.sbase + (r - kb);
        const Rec x = load_rec(a.stage + si);
        d.src[r] = si;
        d.cv[r] = x.cv;
        d.tc[r] = x.tcid;
        d.cl[r] = x.cl;
        d.pos[r] = x.pos;
        const uint32_t owner = ovf_find_owner(a, d, true, r, cb, x.pk, x.tcid >> 16);
        d.rowid[r] = kb + owner;  // the owner's record (scratch until the sort)
        d.recf[r] = owner == r - kb ? 1u : 0u;
        if (owner == r - kb) d.pk[r] = x.pk;  // (only a row's owner is asked for its pk)
        if (!d.reduce) d.val[r] = r;  // (the reduction's compaction writes the sort values)
    }
}

// Each row (its owner record, dense id from the scan of owner flags in epc) looked up in its region:
// prior records counted, new rows counted per bucket (the host checks the region and heap have
// room before anything is written). The removed prior records leave the live count here; the walk
// adds what it writes back.
// Row reduction (no impacts). With Mx the row's largest cl (prior records included), the records at
// cl == Mx form the row's last epoch: the first of them is its record, every later one a candidate
// or a no-op, and nothing after it starts another epoch. The walk's result depends on earlier epochs
// only through the cells they carry: none when Mx is even (a delete), and when Mx is odd only cells
// of cids without a change of their own in the last epoch -- one with col_version > 0 always beats
// a carried (zeroed) cell. So a row whose records are all inside App. A.3, with Mx even, or whose
// cids all have such a change at Mx, folds to the same clock rows from its Mx records alone (the
// row's sentinel is the epoch record's either way: App. A.1 rules 2-4). The other rows keep every
// record. Without this, a Zipf-hot row's history (88 % of its records in config 5) goes through
// the sort, scans and walk only to be dropped by its last delete or overwritten by its last epoch.
__device__ inline bool ovf_rec_bad(const MergeArgs &a, uint32_t cid, uint32_t cl, int64_t cv, uint32_t pos) {
    if (((cid == 0 || (cl & 1u) == 0) && cv != (int64_t)cl) || (!(pos & BATCH_POS) && cid != 0 && !(cl & 1u)))
        return true;
    return a.raw.conv && (pos & BATCH_POS) && a.raw.conv[batch_src(a, pos & 0x7FFFFFFFu)];
}

// device-coherent read (past the CU's L1, which does not see other CUs' atomics): a summary word is
// read before it is updated, and a hot row's lanes mostly find it set
template <typename T>
__device__ inline T ovf_ld_dev(const T *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// A row's summary is two words, each a commutative monoid, so every record's term folds in in any
// order and in one pass (no second pass once the largest cl is known):
//   w1 = Mx << 32 | F   Mx the largest cl, F the cids (bit c, c < 32) of the column changes at Mx with
//                       col_version > 0: (m, f) + (m', f') = (max, f if m is the max | f' if m' is)
//   w2 = C | bad        C the cids of all column records (bit c), bit 0 (no cid 0 term) a record
//                       outside App. A.3
// (tables with 32 or more columns keep every record: the host turns the reduction off for them)
__device__ inline uint64_t rs_comb(uint64_t x, uint64_t y) {
    const uint32_t mx = (uint32_t)(x >> 32), my = (uint32_t)(y >> 32), m = max(mx, my);
    return ((uint64_t)m << 32) | ((mx == m ? (uint32_t)x : 0u) | (my == m ? (uint32_t)y : 0u));
}

__device__ inline void rs_put(const OvfDev &d, uint32_t row, uint64_t w1, uint32_t w2, uint64_t w3 = 0) {
    OvfSum *const S = d.osum ? d.osum + row : nullptr;  // (fused form: by owner record)
    unsigned long long *p = S ? &S->w1 : (unsigned long long *)&d.rw1[row];
    uint32_t *const p2 = S ? &S->w2 : &d.rw2[row];
    unsigned long long cur = ovf_ld_dev(p);
    for (unsigned long long want = rs_comb(cur, w1); want != cur; want = rs_comb(cur, w1)) {
        const unsigned long long o = atomicCAS(p, cur, want);
        if (o == cur) break;
        cur = o;
    }
    if (w2 & ~ovf_ld_dev(p2)) atomicOr(p2, w2);
    if (S && w3 > ovf_ld_dev(&S->w3)) atomicMax(&S->w3, (unsigned long long)w3);
}

// fused form: a record's epoch term, cl << 32 | ~(compact position) (max: the largest cl, then the
// earliest position at it)
__device__ inline uint64_t rs_w3(uint32_t cl, uint32_t p) { return ((uint64_t)cl << 32) | (uint32_t)~p; }

// a record's terms
// (impact form: a batch column change with col_version <= 0 also keeps its row whole -- a carried,
// zeroed cell need not lose to it, and the reduced fold carries none)
__device__ inline void rs_terms(const MergeArgs &a, uint32_t cid, uint32_t cl, int64_t cv, uint32_t pos, uint64_t &w1,
                                uint32_t &w2) {
    const uint32_t bit = cid != 0 ? 1u << (cid & 31) : 0u;
    w1 = ((uint64_t)cl << 32) | (cv > 0 ? bit : 0u);
    const bool zero_col = a.impact && cid != 0 && cv <= 0 && (pos & BATCH_POS);
    w2 = bit | ((ovf_rec_bad(a, cid, cl, cv, pos) || zero_col) ? 1u : 0u);
}

// ---- impact form: first position of each causal length per row (F(c) of k_ovf_keep) ----------
#ifndef OVF_DIAG
#define OVF_DIAG 0
#endif
#ifndef OVF_NCL
#define OVF_NCL 8  // causal-length slots per row; a row whose causal lengths collide keeps every record
#endif
// Slot cl mod OVF_NCL holds causal length cl (a row's causal lengths are mostly a short run of
// consecutive values, which never collide), and one atomicMin both claims a free slot (~0) and keeps
// the first position. Two causal lengths that share a slot corrupt it -- the min of the two words --
// but whichever of them comes second sees the other's word come back and marks the row, which then
// keeps every record and never reads its slots (k_ovf_keep). cl 0 records are never records nor
// candidates and take no slot.
__device__ inline void rcl_put(const OvfDev &d, uint32_t row, uint32_t cl, uint32_t pos) {
    if (cl == 0) return;
    unsigned long long *sl = (unsigned long long *)d.rcl + (size_t)row * OVF_NCL + cl % OVF_NCL;
    const unsigned long long o = atomicMin(sl, ((unsigned long long)cl << 32) | pos);
    if (o != ~0ULL && (uint32_t)(o >> 32) != cl) atomicOr(&d.rw2[row], 1u);
}

// Per workgroup first (k_ovf_lookup's chunk of RS_CHUNK bucket-major records: a few buckets' rows, a
// hot row's records many times over): an LDS table keyed (row, cl) keeps the minimum position, and
// each entry goes to the row's global slots once at the end. A key without an LDS slot goes straight
// to the global slots.
#ifndef OVF_RCL_BITS
#define OVF_RCL_BITS 11
#endif
constexpr uint32_t RCL_HT = 1u << OVF_RCL_BITS;
struct RclLds {
    unsigned long long key[RCL_HT];  // row << 32 | cl, ~0: free
    uint32_t pos[RCL_HT];
};

__device__ inline void rcl_lds_clear(RclLds &L) {
    for (uint32_t i = threadIdx.x; i < RCL_HT; i += blockDim.x) {
        L.key[i] = ~0ULL;
        L.pos[i] = ~0u;
    }
}

__device__ inline bool rcl_lds_add(RclLds &L, uint32_t row, uint32_t cl, uint32_t pos) {
    const unsigned long long k = ((unsigned long long)row << 32) | cl;
    const uint32_t h = (uint32_t)((k * 0x9E3779B97F4A7C15ULL) >> (64 - OVF_RCL_BITS));
    for (uint32_t j = 0; j < 16; j++) {
        const uint32_t sl = (h + j) & (RCL_HT - 1);
        unsigned long long o = L.key[sl];
        if (o == ~0ULL) o = atomicCAS(&L.key[sl], ~0ULL, k);
        if (o != ~0ULL && o != k) continue;
        atomicMin(&L.pos[sl], pos);
        return true;
    }
    return false;
}

__device__ inline void rcl_lds_flush(const RclLds &L, const OvfDev &d) {
    for (uint32_t i = threadIdx.x; i < RCL_HT; i += blockDim.x)
        if (L.key[i] != ~0ULL) rcl_put(d, (uint32_t)(L.key[i] >> 32), (uint32_t)L.key[i], L.pos[i]);
}

// one (row, cl, position) per `todo` lane, called by every lane of the wave: lanes sharing the first
// active lane's row and causal length (a Zipf-hot row fills whole waves) take their minimum first
__device__ inline void rcl_wave_add(RclLds &L, const OvfDev &d, bool todo, uint32_t row, uint32_t cl, uint32_t pos) {
    const uint32_t lane = threadIdx.x & 63;
    for (int round = 0; round < 2; round++) {  // (two rounds, as for the summaries: the rest go to LDS)
        const uint64_t act = __ballot(todo);
        if (!act) break;
        const int leader = __ffsll((unsigned long long)act) - 1;
        const uint32_t lrow = __shfl(row, leader), lcl = __shfl(cl, leader);
        const bool mine = todo && row == lrow && cl == lcl;
        if (__popcll(__ballot(mine)) < 4) break;  // (wave-uniform) not a hot row
        uint32_t m = mine ? pos : ~0u;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) m = min(m, (uint32_t)__shfl_xor(m, o));
        if ((int)lane == leader && lcl != 0 && !rcl_lds_add(L, lrow, lcl, m)) rcl_put(d, lrow, lcl, m);
        if (mine) todo = false;
    }
    if (todo && cl != 0 && !rcl_lds_add(L, row, cl, pos)) rcl_put(d, row, cl, pos);
}

// Row summaries aggregated per workgroup first: a workgroup takes RS_CHUNK consecutive records
// (bucket-major, so a few buckets' rows, a Zipf-hot row's records many times over), folds them into
// an LDS table keyed by row, then writes each of its rows to the global words once. A record whose
// row finds no LDS slot updates the global words itself.
#ifndef OVF_RS_E
#define OVF_RS_E 16  // records per thread of a summary workgroup (4 / 8 / 16: lookup 1.57 / 1.34 / 1.15 ms at config 5)
#endif
#ifndef OVF_RS_BITS
#define OVF_RS_BITS 10
#endif
constexpr uint32_t RS_T = 256, RS_E = OVF_RS_E, RS_CHUNK = RS_T * RS_E, RS_HT = 1u << OVF_RS_BITS;
// (the fused form's w3 words only in its own table: an extra word in the others' would cost
// k_ovf_lookup<true> a workgroup per CU -- its two LDS tables sit just under a quarter of the CU's LDS)
template <bool W3>
struct RsLdsT;
template <>
struct RsLdsT<false> {
    uint32_t key[RS_HT], w2[RS_HT];  // key: row + 1 (0: free)
    unsigned long long w1[RS_HT];
};
template <>
struct RsLdsT<true> : RsLdsT<false> {
    unsigned long long w3[RS_HT];
};
using RsLds = RsLdsT<false>;

template <bool W3>
__device__ inline void rs_lds_clear(RsLdsT<W3> &L) {
    for (uint32_t i = threadIdx.x; i < RS_HT; i += blockDim.x) {
        L.key[i] = 0;
        L.w2[i] = 0;
        L.w1[i] = 0;
        if constexpr (W3) L.w3[i] = 0;
    }
}

template <bool W3>
__device__ inline bool rs_lds_add(RsLdsT<W3> &L, uint32_t row, uint64_t w1, uint32_t w2, uint64_t w3 = 0) {
    const uint32_t h = (row * 2654435761u) >> (32 - OVF_RS_BITS);
    for (uint32_t k = 0; k < 16; k++) {
        const uint32_t sl = (h + k) & (RS_HT - 1);
        const uint32_t o = atomicCAS(&L.key[sl], 0u, row + 1);
        if (o != 0 && o != row + 1) continue;
        unsigned long long cur = L.w1[sl];
        for (unsigned long long want = rs_comb(cur, w1); want != cur; want = rs_comb(cur, w1)) {
            const unsigned long long q = atomicCAS(&L.w1[sl], cur, want);
            if (q == cur) break;
            cur = q;
        }
        if (w2) atomicOr(&L.w2[sl], w2);
        if constexpr (W3) atomicMax(&L.w3[sl], (unsigned long long)w3);
        return true;
    }
    return false;
}

template <bool W3>
__device__ inline void rs_lds_flush(const RsLdsT<W3> &L, const OvfDev &d) {
    for (uint32_t i = threadIdx.x; i < RS_HT; i += blockDim.x)
        if (L.key[i]) {
            if constexpr (W3) rs_put(d, L.key[i] - 1, L.w1[i], L.w2[i], L.w3[i]);
            else rs_put(d, L.key[i] - 1, L.w1[i], L.w2[i]);
        }
}

__device__ inline uint32_t wave_or32(uint32_t x) {
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) x |= (uint32_t)__shfl_xor(x, o);
    return x;
}

__device__ inline uint32_t wave_max32(uint32_t x) {
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) x = max(x, (uint32_t)__shfl_xor(x, o));
    return x;
}

// One term per `todo` lane (called by every lane of the wave): lanes sharing the first active lane's
// row -- a Zipf-hot row fills whole waves -- are combined across the wave and added by that lane (at
// most two rounds), the rest add their own; LDS first, the global words when the table has no slot.
__device__ inline uint64_t wave_max64(uint64_t x) {
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint64_t y = __shfl_xor(x, o);
        x = y > x ? y : x;
    }
    return x;
}

template <bool W3>
__device__ inline void rs_wave_add(RsLdsT<W3> &L, const OvfDev &d, bool todo, uint32_t row, uint64_t w1, uint32_t w2,
                                   uint64_t w3 = 0) {
    const uint32_t lane = threadIdx.x & 63;
    for (int round = 0; round < 2; round++) {
        const uint64_t act = __ballot(todo);
        if (!act) break;
        const int leader = __ffsll((unsigned long long)act) - 1;
        const uint32_t lrow = __shfl(row, leader);
        const bool mine = todo && row == lrow;
        if (__popcll(__ballot(mine)) < 8) break;  // (wave-uniform) not a hot row
        const uint32_t m = wave_max32(mine ? (uint32_t)(w1 >> 32) : 0u);
        const uint32_t f = wave_or32(mine && (uint32_t)(w1 >> 32) == m ? (uint32_t)w1 : 0u);
        const uint32_t c = wave_or32(mine ? w2 : 0u);
        const uint64_t x3 = W3 ? wave_max64(mine ? w3 : 0ULL) : 0ULL;
        const uint64_t x1 = ((uint64_t)m << 32) | f;
        if ((int)lane == leader && !rs_lds_add(L, lrow, x1, c, x3)) rs_put(d, lrow, x1, c, x3);
        if (mine) todo = false;
    }
    if (todo && !rs_lds_add(L, row, w1, w2, w3)) rs_put(d, row, w1, w2, w3);
}

// Fused plain form (d.fuse): the same pass also folds every record's summary terms (rs_terms, rs_w3)
// into its row's words, keyed by the owner record -- per wave, then per workgroup in LDS, then once
// into HBM, as k_ovf_lookup does by dense row. That pass then has nothing left to do: its sort keys
// are written by k_ovf_keep<true> for the records it keeps, and the rows' owners by k_ovf_owners.
static __global__ void __launch_bounds__(RS_T) k_ovf_loadsum(MergeArgs a, OvfDev d) {
    __shared__ RsLdsT<true> L;
    const OvfDev &od = d;
    rs_lds_clear(L);
    __syncthreads();
    const uint32_t c0 = blockIdx.x * RS_CHUNK;
    for (uint32_t j = 0; j < RS_E; j++) {  // (wave-uniform: owners and summaries reduce across the wave)
        const uint32_t r = c0 + j * RS_T + threadIdx.x;
        const bool valid = r < d.Kb;
        ChunkB cb{};
        Rec x{};
        if (valid) {
            cb = ovf_chunk_of(a, d, r);
            const uint32_t si = cb.sbase + (r - cb.kb);
            x = load_rec(a.stage + si);
            d.src[r] = si;
            d.cv[r] = x.cv;
            d.tc[r] = x.tcid;
            d.cl[r] = x.cl;
            d.pos[r] = x.pos;
        }
        const uint32_t owner = ovf_find_owner(a, d, valid, r, cb, x.pk, x.tcid >> 16);
        const uint32_t o = cb.kb + owner;
        uint64_t w1 = 0, w3 = 0;
        uint32_t w2 = 0;
        if (valid) {
            d.rowid[r] = o;  // the owner's record (k_ovf_keep<true> reads its summary there)
            d.recf[r] = o == r ? 1u : 0u;
            if (o == r) d.pk[r] = x.pk;
            rs_terms(a, x.tcid & 0xFFFFu, x.cl, x.cv, x.pos, w1, w2);
            w3 = rs_w3(x.cl, d.pm + (x.pos & 0x7FFFFFFFu));
        }
        rs_wave_add(L, od, valid, o, w1, w2, w3);
    }
    __syncthreads();
    rs_lds_flush(L, od);
}

// fused form: each row's owner record and bucket (k_ovf_lookup's part for owners)
static __global__ void k_ovf_owners(MergeArgs a, OvfDev d) {
    OVF_LOOP(r, d.Kb) {
        if (!d.recf[r]) continue;
        const uint32_t row = d.epc[r] - 1u;
        uint32_t b = d.cbk[8 * (r >> 6)];
        while (d.koff[b + 1] <= r) b++;
        d.rowner[row] = r;
        d.rb[row] = b;
        d.osum[r].row = row;
    }
}


// (RIMP: the impact form's causal-length slots too; its LDS table only in that instantiation, so the
// plain form keeps its occupancy)
template <bool RIMP>
static __global__ void __launch_bounds__(RS_T) k_ovf_lookup(MergeArgs a, OvfDev d) {
    __shared__ RsLds L;
    __shared__ typename std::conditional<RIMP, RclLds, char>::type LC_;
    if (d.reduce) {
        rs_lds_clear(L);
        if constexpr (RIMP) rcl_lds_clear(LC_);
        __syncthreads();
    }
    const uint32_t c0 = blockIdx.x * RS_CHUNK;
    for (uint32_t j = 0; j < RS_E; j++) {  // (wave-uniform: the summary reduces across the wave)
        const uint32_t r = c0 + j * RS_T + threadIdx.x;
        const bool valid = r < d.Kb;
        // every record: its sort key (k_ovf_rowkey's, fused here: dense rows are known by now)
        uint32_t row = 0, pos = 0;
        bool owner = false;
        if (valid) {
            const uint32_t o = d.rowid[r];  // the row's owner record (k_ovf_loadhash)
            owner = o == r;
            row = d.epc[o] - 1u;
            pos = d.pos[r];
            d.key[r] = ((uint64_t)row << d.rshift) | ((uint64_t)d.pm + (pos & 0x7FFFFFFFu));
        }
        if (d.reduce) {
            uint64_t w1 = 0;
            uint32_t w2 = 0;
            uint32_t cl = 0;
            if (valid) {
                d.rowid[r] = row;  // (own slot: every other lane reads epc, not rowid)
                cl = d.cl[r];
                rs_terms(a, d.tc[r] & 0xFFFFu, cl, d.cv[r], pos, w1, w2);
            }
            rs_wave_add(L, d, valid, row, w1, w2);
#if !(OVF_DIAG & 1)  // (diagnostic builds only: OVF_DIAG 1 drops the causal-length slots, results not valid)
            if constexpr (RIMP) rcl_wave_add(LC_, d, valid, row, cl, d.pm + (pos & 0x7FFFFFFFu));
#endif
        }
        if (!owner) continue;  // (an owner's row: epc[r] - 1, as computed above)
        uint32_t b = d.cbk[8 * (r >> 6)];  // (its bucket: only the owners look it up)
        while (d.koff[b + 1] <= r) b++;
        const uint32_t t = d.tc[r] >> 16;
        d.rowner[row] = r;
        d.rb[row] = b;
        if (d.split) continue;
        const uint32_t e = rs_lookup(a.rs, a.ovf_list[b], d.pk[r], t);
        if (e == ROW_NONE) {
            d.rheap[row] = ROW_NONE;
            d.rprior[row] = 0;
            d.rbits[2 * row] = d.rbits[2 * row + 1] = 0;
            atomicAdd(&d.bnew[b], 1u);
            atomicAdd(&d.bnrec[b], (uint32_t)a.rs.stride[t]);
        } else {
            const RowEnt re = a.rs.ent[e];
            const uint32_t pc = row_popc(re.bits);
            d.rheap[row] = re.heap;
            d.rprior[row] = pc;
            d.rbits[2 * row] = re.bits[0];
            d.rbits[2 * row + 1] = re.bits[1];
            atomicAdd(&a.misc[MISC_LIVE], (unsigned long long)(-(long long)pc));
        }
    }
    if (d.reduce) {
        __syncthreads();
        rs_lds_flush(L, d);
#if !(OVF_DIAG & 3)  // (OVF_DIAG 2: the LDS table kept, its flush to the rows' slots dropped)
        if constexpr (RIMP) rcl_lds_flush(LC_, d);
#endif
    }
}

// Each row looked up in its region, one lane per row (k_ovf_lookup's lanes walk RS_E records each,
// so a lookup there is a chain of dependent probes per record group; here every row's probe is in
// flight at once). New rows and their heap records counted per bucket, the found rows' prior records
// leave the live count -- both summed per wave first (rows are bucket-major: a wave's rows share one
// or two buckets).
static __global__ void k_ovf_rlook(MergeArgs a, OvfDev d) {
    const uint32_t lane = threadIdx.x & 63;
    unsigned long long gone = 0;
    for (uint32_t base = blockIdx.x * blockDim.x; base < d.nrows; base += gridDim.x * blockDim.x) {  // (wave-uniform)
        const uint32_t row = base + threadIdx.x;
        const bool ok = row < d.nrows;
        uint32_t b = 0, nrec = 0;
        bool isnew = false;
        if (ok) {
            const uint32_t r = d.rowner[row], t = d.tc[r] >> 16;
            b = d.rb[row];
            const uint32_t e = rs_lookup(a.rs, a.ovf_list[b], d.pk[r], t);
            if (e == ROW_NONE) {
                d.rheap[row] = ROW_NONE;
                d.rprior[row] = 0;
                d.rbits[2 * row] = d.rbits[2 * row + 1] = 0;
                isnew = true;
                nrec = (uint32_t)a.rs.stride[t];
            } else {
                const RowEnt re = a.rs.ent[e];
                const uint32_t pc = row_popc(re.bits);
                d.rheap[row] = re.heap;
                d.rprior[row] = pc;
                d.rbits[2 * row] = re.bits[0];
                d.rbits[2 * row + 1] = re.bits[1];
                gone += pc;
            }
        }
        // per-bucket counts: the wave's new rows of the first active lane's bucket in one atomic each
        bool todo = isnew;
        while (true) {
            const uint64_t act = __ballot(todo);
            if (!act) break;
            const int leader = __ffsll((unsigned long long)act) - 1;
            const uint32_t lb = __shfl(b, leader);
            const bool mine = todo && b == lb;
            const uint32_t rows = (uint32_t)__popcll(__ballot(mine));
            const uint32_t recs = wave_sum_u32(mine ? nrec : 0u);
            if ((int)lane == leader) {
                atomicAdd(&d.bnew[lb], rows);
                atomicAdd(&d.bnrec[lb], recs);
            }
            if (mine) todo = false;
        }
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) gone += __shfl_xor(gone, o);
    if (lane == 0 && gone) atomicAdd(&a.misc[MISC_LIVE], (unsigned long long)(-(long long)gone));
}

// prior records of every found row appended at [Kb + rpoff[row] - pc, Kb + rpoff[row]) (rpoff:
// inclusive scan of the rows' prior counts)
static __global__ void k_ovf_pload(MergeArgs a, OvfDev d) {
    OVF_LOOP(row, d.nrows) {
        const uint32_t pc = d.rprior[row];
        if (!pc) continue;
        const uint32_t hb = d.rheap[row];
        uint32_t r = d.Kb + d.rpoff[row] - pc;
        for (int w = 0; w < 2; w++)
            for (uint64_t m = d.rbits[2 * row + w]; m; m &= m - 1) {
                const uint32_t c = 64 * w + (uint32_t)__ffsll((unsigned long long)m) - 1;
                const Rec pr = load_rec(a.rs.heap + hb + c);
                d.cv[r] = pr.cv;
                d.tc[r] = pr.tcid;
                d.cl[r] = pr.cl;
                d.pkey[r - d.Kb] = OvfKey{pr.cv, pr.v0, pr.v1, pr.meta, site_rank_of(a, pr.site)};
                d.pos[r] = c;  // compact position < pm: before the batch
                d.src[r] = hb + c;
                d.key[r] = ((uint64_t)row << d.rshift) | c;
                d.val[r] = r;
                if (d.reduce) {
                    // (fused form: summaries and rowid by the row's owner record, as for the batch)
                    const uint32_t sk = d.fuse ? d.rowner[row] : row;
                    d.rowid[r] = sk;
                    uint64_t w1;
                    uint32_t w2;
                    rs_terms(a, pr.tcid & 0xFFFFu, pr.cl, pr.cv, c, w1, w2);
                    rs_put(d, sk, w1, w2, rs_w3(pr.cl, c));
                    if (d.rimp) rcl_put(d, row, pr.cl, c);
                }
                r++;
            }
    }
}

// The kept records' (key, record) pairs compacted into (ckey, cval) for the sort: each workgroup
// takes a contiguous chunk, ranks its kept records by wave ballots and reserves their slots with ONE
// atomic (the order does not matter: the keys are unique and the sort orders them).
//
// Impact form (rimp; the rule is checked against the sequential oracle on the CPU in
// tests/test_ovf_reduce_rule.py::test_row_reduction_impacts_equal_full_fold): a dropped record r of a
// reduced row (cl < Mx) at compact position p, with F = its causal length's first position and H the
// first position of any larger causal length (the row's OVF_NCL slots), is
//   a record     p == F < H: flag 1, or 2 for a column change with odd cl > 1 (it resurrects); the
//                slot notes r (the epoch record a candidate group may be seeded by);
//   a candidate  F < p < H, odd cl, column change: compacted from the END of (ckey, cval) with its
//                group key (row, slot, cid) and position, for the sort and running argmax that
//                decide its flag (k_ovf_dimp);
//   a no-op      otherwise: flag 0.
__device__ inline void ovf_drop_class(const MergeArgs &a, const OvfDev &d, uint32_t r, uint32_t row, uint32_t cl,
                                      bool &cand, uint64_t &dkey) {
    cand = false;
    const uint64_t key = d.key[r];
    const uint32_t p = (uint32_t)(key & ((1ULL << d.rshift) - 1));
    const uint32_t tc = d.tc[r], cid = tc & 0xFFFFu, pos = d.pos[r];
    uint32_t F = ~0u, H = ~0u, slot = 0;
    const unsigned long long *sl = (const unsigned long long *)d.rcl + (size_t)row * OVF_NCL;
#pragma unroll
    for (uint32_t k = 0; k < OVF_NCL; k++) {
        const unsigned long long x = sl[k];
        if (x == ~0ULL) continue;
        const uint32_t c = (uint32_t)(x >> 32), fp = (uint32_t)x;
        if (c == cl) {
            F = fp;
            slot = k;
        } else if (c > cl) {
            H = min(H, fp);
        }
    }
    uint8_t flag = 0;
    if (cl != 0 && p == F && p < H) {
        flag = (cid != 0 && (cl & 1u) && cl > 1) ? 2 : 1;
        d.rclr[(size_t)row * OVF_NCL + slot] = r;
    } else if (cl != 0 && F != ~0u && F < p && p < H && (cl & 1u) && cid != 0) {
        cand = true;
        dkey = ((((uint64_t)row * OVF_NCL + slot) << d.cid_bits | cid) << d.rshift) | p;
    }
    if (!cand && (pos & BATCH_POS) && flag) a.impact[pos & 0x7FFFFFFFu] = flag;
}

#ifndef OVF_KEEP_E
#define OVF_KEEP_E 32  // records per thread (<= 32: one bit each in a lane's masks)
#endif
constexpr uint32_t KEEP_T = 256, KEEP_E = OVF_KEEP_E, KEEP_CHUNK = KEEP_T * KEEP_E;
// FUSE (the fused plain form, d.fuse): summaries are read at the owner record (rowid[r]) and the
// sort keys are made here -- a kept record of a row that is not reduced gets (row, position); a
// reduced row keeps nothing for the (row, position) sort: its epoch record (the first at Mx, rw3)
// goes to rowE and lists the row for the reduced walk, and its column records at an odd Mx are
// compacted from the END with the cell key (owner record, cid) for the cell sort (their winners:
// k_cscan_*<true>, k_ovf_rcells); a row that is not reduced is listed for the walk by its owner
// record. Only those records look up the dense row (epc): the rest read two words.
template <bool FUSE>
static __global__ void __launch_bounds__(KEEP_T) k_ovf_keep(MergeArgs a, OvfDev d, uint32_t kcap) {
    __shared__ uint32_t s_cnt[KEEP_T / 64], s_base, s_dcnt[KEEP_T / 64], s_dbase, s_ecnt[KEEP_T / 64], s_ebase,
        s_fcnt[KEEP_T / 64], s_fbase;
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6, n = d.K;
    const uint32_t c0 = blockIdx.x * KEEP_CHUNK;
    uint32_t mine = 0, cnt = 0;  // lane's kept bits per step; the wave's kept count
    uint32_t dmine = 0, dcnt = 0;  // (impact form) the same for dropped candidates
    uint32_t emine = 0, ecnt = 0;  // (fused form) the same for the reduced rows' epoch records
    uint32_t fmine = 0, fcnt = 0;  // (fused form) and for the other rows' owner records
#pragma unroll 4
    for (uint32_t j = 0; j < KEEP_E; j++) {
        const uint32_t r = c0 + j * KEEP_T + threadIdx.x;
        bool keep = false, cand = false;
        bool isE = false, isF = false;
        if (FUSE && r < n) {
            // (every load unconditional: two dependent levels, batched over the unrolled steps)
            const uint32_t o = d.rowid[r], cl = d.cl[r], pos = d.pos[r], tcr = d.tc[r];
            const uint4 *sp = reinterpret_cast<const uint4 *>(d.osum + o);
            const uint4 s0 = sp[0], s1 = sp[1];
            const uint64_t w1 = ((uint64_t)s0.y << 32) | s0.x, w3 = ((uint64_t)s0.w << 32) | s0.z;
            const uint32_t w2 = s1.x, eo = s1.y + 1u;
            const uint32_t mx = (uint32_t)(w1 >> 32);
            const bool red = !(w2 & 1u) && (!(mx & 1u) || (uint32_t)w1 == w2);
            const uint32_t p = r < d.Kb ? d.pm + (pos & 0x7FFFFFFFu) : pos;
            if (!red) {
                keep = true;
                const uint32_t row = eo - 1u;
                d.key[r] = ((uint64_t)row << d.rshift) | p;  // (its own slot, copied by the compaction)
                if (o == r) {  // the owner lists the row for the walk
                    d.rowid[r] = row;  // (its own slot: the list write below reads it back)
                    isF = true;
                }
            } else if (cl == mx) {
                if ((uint32_t)~(uint32_t)w3 == p) {
                    const uint32_t row = eo - 1u;
                    d.rowE[row] = r;
                    d.rsum[row] = ((uint64_t)mx << 32) | w2;
                    d.rowid[r] = row;  // (its own slot: the list write below reads it back)
                    isE = true;
                }
                const uint32_t cid = tcr & 0xFFFFu;
                if ((mx & 1u) && cid != 0) {
                    cand = true;
                    d.key[r] = ((uint64_t)o << d.cid_bits) | cid;
                }
            }
        } else if (r < n) {
            const uint32_t row = d.rowid[r], cl = d.cl[r], w2 = d.rw2[row];
            const uint64_t w1 = d.rw1[row];
            const uint32_t mx = (uint32_t)(w1 >> 32);
            const bool red = !(w2 & 1u) && (!(mx & 1u) || (uint32_t)w1 == w2);
            keep = !red || cl == mx;
            if (!keep && d.rimp) {
                uint64_t dk;
                ovf_drop_class(a, d, r, row, cl, cand, dk);
                if (cand) d.key[r] = dk;  // (its own slot, read by nothing else: the compaction copies it)
            }
        }
        if (FUSE) {
            emine |= isE ? 1u << j : 0u;
            ecnt += (uint32_t)__popcll(__ballot(isE));
            fmine |= isF ? 1u << j : 0u;
            fcnt += (uint32_t)__popcll(__ballot(isF));
        }
        mine |= keep ? 1u << j : 0u;
        cnt += (uint32_t)__popcll(__ballot(keep));
        dmine |= cand ? 1u << j : 0u;
        dcnt += (uint32_t)__popcll(__ballot(cand));
    }
    if (lane == 0) {
        s_cnt[w] = cnt;
        s_dcnt[w] = dcnt;
        s_ecnt[w] = ecnt;
        s_fcnt[w] = fcnt;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t t = 0, u = 0, e = 0, f = 0;
        for (uint32_t v = 0; v < KEEP_T / 64; v++) {
            t += s_cnt[v];
            u += s_dcnt[v];
            e += s_ecnt[v];
            f += s_fcnt[v];
        }
        s_base = t ? atomicAdd(d.nkeep, t) : 0u;
        s_dbase = u ? atomicAdd(d.nkeep + 1, u) : 0u;
        if (FUSE) {
            s_ebase = e ? atomicAdd(d.nkeep + 2, e) : 0u;
            s_fbase = f ? atomicAdd(d.nkeep + 3, f) : 0u;
        }
    }
    __syncthreads();
    uint32_t o = s_base, od = s_dbase, oe = FUSE ? s_ebase : 0u, of = FUSE ? s_fbase : 0u;
    for (uint32_t v = 0; v < w; v++) {
        o += s_cnt[v];
        od += s_dcnt[v];
        oe += s_ecnt[v];
        of += s_fcnt[v];
    }
    if (FUSE && (ecnt | fcnt))  // the rows' lists (k_ovf_walk modes 1 and 2)
        for (uint32_t j = 0; j < KEEP_E; j++) {
            const bool e = (emine >> j) & 1u, f = (fmine >> j) & 1u;
            const uint64_t m = __ballot(e), mf = __ballot(f);
            if (e || f) {
                const uint32_t row = d.rowid[c0 + j * KEEP_T + threadIdx.x];
                if (e) d.rlist[oe + (uint32_t)__popcll(m & ((1ULL << lane) - 1))] = row;
                else d.flist[of + (uint32_t)__popcll(mf & ((1ULL << lane) - 1))] = row;
            }
            oe += (uint32_t)__popcll(m);
            of += (uint32_t)__popcll(mf);
        }
    for (uint32_t j = 0; j < KEEP_E; j++) {
        const bool keep = (mine >> j) & 1u;
        const uint64_t m = __ballot(keep);
        const uint32_t r = c0 + j * KEEP_T + threadIdx.x;
        if (keep) {
            const uint32_t q = o + (uint32_t)__popcll(m & ((1ULL << lane) - 1));
            d.ckey[q] = d.key[r];
            d.cval[q] = r;
        }
        o += (uint32_t)__popcll(m);
        if (!dcnt) continue;  // (wave-uniform)
        const bool cand = (dmine >> j) & 1u;
        const uint64_t dm = __ballot(cand);
        if (cand) {  // dropped candidates fill (ckey, cval) from the end: kept + dropped <= kcap
            const uint32_t q = kcap - 1 - (od + (uint32_t)__popcll(dm & ((1ULL << lane) - 1)));
            d.ckey[q] = d.key[r];  // (the group key the first pass left there)
            d.cval[q] = r;
        }
        od += (uint32_t)__popcll(dm);
    }
}

// the cell key of record x (a batch record's staged copy, a prior record's key read before the walk)
__device__ inline OvfKey ovf_key_x(const MergeArgs &a, const OvfDev &d, uint32_t x) {
    if (x >= d.Kb) return d.pkey[x - d.Kb];
    const Rec r = load_rec(ovf_rec(a, d, x));
    return OvfKey{r.cv, r.v0, r.v1, r.meta, site_rank_of(a, r.site)};
}

// dropped candidates sorted by (group, position): their group keys (for the running argmax's group
// starts) and cell keys in sorted order
static __global__ void k_ovf_dgather(MergeArgs a, OvfDev d, uint32_t ndc, const uint64_t *__restrict__ dkey_s,
                                     const uint32_t *__restrict__ dval_s, uint64_t *__restrict__ dgroup,
                                     OvfKey *__restrict__ dq) {
    OVF_LOOP(q, ndc) {
        dgroup[q] = dkey_s[q] >> d.rshift;
        dq[q] = ovf_key_x(a, d, dval_s[q]);
    }
}

// a dropped candidate's flag: strictly greater than every earlier candidate of its (row, causal
// length, cid) group (dbest[q - 1]: the running argmax) and than its epoch record's own cell when
// that record is a column change of the same cid (a carried, zeroed cell loses to col_version > 0)
static __global__ void k_ovf_dimp(MergeArgs a, OvfDev d, uint32_t ndc, const uint64_t *__restrict__ dgroup,
                                  const uint32_t *__restrict__ dval_s, const OvfKey *__restrict__ dq,
                                  const uint32_t *__restrict__ dbest) {
    OVF_LOOP(q, ndc) {
        const uint32_t x = dval_s[q];
        const uint32_t pos = d.pos[x];
        if (!(pos & BATCH_POS)) continue;
        const uint64_t g = dgroup[q];
        const OvfKey k = dq[q];
        bool imp = q == 0 || dgroup[q - 1] != g || ovf_kcmp(k, dq[dbest[q - 1]], d.arena) > 0;
        if (imp) {
            const uint32_t cid = (uint32_t)(g & ((1ULL << d.cid_bits) - 1));
            const uint64_t rs = g >> d.cid_bits;  // row * OVF_NCL + slot
            const uint32_t R = d.rclr[rs];
            if ((d.tc[R] & 0xFFFFu) == cid) imp = ovf_kcmp(k, ovf_key_x(a, d, R), d.arena) > 0;
        }
        if (imp) a.impact[pos & 0x7FFFFFFFu] = 1;
    }
}

static __global__ void k_ovf_gather(OvfDev d) {
    OVF_LOOP(p, d.K) {
        const uint32_t row = (uint32_t)(d.key_s[p] >> d.rshift);
        d.rowid[p] = row;
        d.cl_s[p] = d.cl[d.val_s[p]];
        d.head[p] = 0;
        if (!d.reduce || d.rimp) d.fstg[p] = 0;  // (impacts only)
        if (p == 0 || (uint32_t)(d.key_s[p - 1] >> d.rshift) != row) {
            d.rstart[row] = p;
            d.rbad[row] = 0;
            d.rnrec[row] = 0;
        }
    }
}

static __global__ void k_ovf_classify(MergeArgs a, OvfDev d) {
    OVF_LOOP(p, d.K) {
        const uint32_t x = d.val_s[p];
        const uint32_t cl = d.cl_s[p], L = d.lx[p], cid = d.tc[x] & 0xFFFFu, pos = d.pos[x];
        const uint32_t kd = cl > L ? 1u : ((cl == L && cid != 0 && (cl & 1u)) ? 2u : 0u);
        d.kind[p] = kd;
        d.recf[p] = kd == 1 ? 1u : 0u;
        // outside App. A.3 (see rowfold.h): the sequential fold takes the row
        if (((cid == 0 || (cl & 1u) == 0) && d.cv[x] != (int64_t)cl) || (!(pos & BATCH_POS) && cid != 0 && !(cl & 1u)))
            atomicOr(&d.rbad[d.rowid[p]], 1u);
        // a converted value compares raw-vs-stored, an order the candidate argmax cannot keep
        if (a.raw.conv && (pos & BATCH_POS) && a.raw.conv[batch_src(a, pos & 0x7FFFFFFFu)])
            atomicOr(&d.rbad[d.rowid[p]], 1u);
        if (a.impact && (pos & BATCH_POS) && kd == 1)
            a.impact[pos & 0x7FFFFFFFu] = (cid != 0 && (cl & 1u) && (L > 0 || cl > 1)) ? 2 : 1;
    }
}

static __global__ void k_ovf_epochs(OvfDev d) {
    OVF_LOOP(p, d.K) {
        if (d.kind[p] != 1) continue;
        const uint32_t row = d.rowid[p], c = d.epc[p];
        d.recs[d.rstart[row] + c - 1] = p;
        atomicMax(&d.rnrec[row], c);
    }
}

// candidate keys: (position of the epoch's record, cid), ~0 for the rest (sorts last). The record
// position names (row, epoch) in log2(K) bits, so the sort has few digits to go through.
static __global__ void k_ovf_ckeys(OvfDev d) {
    const uint32_t cmask = (1u << d.cid_bits) - 1;
    OVF_LOOP(p, d.K) {
        uint64_t k = ~0ULL;
        if (d.kind[p] == 2) {  // a candidate always follows its row's first record
            const uint32_t R = d.recs[d.rstart[d.rowid[p]] + d.epc[p] - 1];
            const uint32_t cid = d.tc[d.val_s[p]] & cmask;
            k = ((uint64_t)R << d.cid_bits) | cid;
        }
        d.ckey[p] = k;
        d.slots[p] = k != ~0ULL ? 1u : 0u;  // (the row-hash slots are free by now)
    }
}

// candidates only, in order (inclusive scan of the flags at slots + K), for the candidate sort
static __global__ void k_ovf_ccompact(OvfDev d) {
    OVF_LOOP(p, d.K) {
        if (!d.slots[p]) continue;
        const uint32_t j = d.slots[d.K + p] - 1;
        d.key[j] = d.ckey[p];
        d.val[j] = p;
    }
}

static __global__ void k_ovf_cgather(MergeArgs a, OvfDev d) {
    OVF_LOOP(q, d.ncand) {
        d.qkey[q] = ovf_key_rec(a, d, d.cval_s[q], false);
    }
}

static __global__ void k_ovf_link(OvfDev d) {
    OVF_LOOP(q, d.ncand) {
        const uint64_t k = d.ckey_s[q];
        if (q + 1 < d.ncand && d.ckey_s[q + 1] == k) continue;
        d.nxt[q] = atomicExch(&d.head[(uint32_t)(k >> d.cid_bits)], q + 1);
    }
}

// The walk's carried cells (cid, source position, zeroed flag) for one row, in insertion order:
// in registers when every table has fewer than WALK_MAXC columns (dynamic indices resolved by
// unrolled compares, so nothing goes to scratch), else in the global scratch at the row's start.
constexpr uint32_t WALK_MAXC = 8;

template <bool REG>
struct WalkCells;

template <>
struct WalkCells<true> {
    uint32_t cid_[WALK_MAXC], pos_[WALK_MAXC], z_[WALK_MAXC];
    __device__ inline WalkCells(const OvfDev &, uint32_t) {}
    __device__ inline uint32_t pos(uint32_t c) const {
        uint32_t r = 0;
#pragma unroll
        for (uint32_t i = 0; i < WALK_MAXC; i++) r = i == c ? pos_[i] : r;
        return r;
    }
    __device__ inline uint32_t z(uint32_t c) const {
        uint32_t r = 0;
#pragma unroll
        for (uint32_t i = 0; i < WALK_MAXC; i++) r = i == c ? z_[i] : r;
        return r;
    }
    __device__ inline void zero_all() {
#pragma unroll
        for (uint32_t i = 0; i < WALK_MAXC; i++) z_[i] = 1;
    }
    __device__ inline int find(uint32_t cid, uint32_t n) const {
        int f = -1;
#pragma unroll
        for (uint32_t i = 0; i < WALK_MAXC; i++)
            if (f < 0 && i < n && cid_[i] == cid) f = (int)i;
        return f;
    }
    __device__ inline void put(uint32_t c, uint32_t cid, uint32_t p, uint32_t zz) {
#pragma unroll
        for (uint32_t i = 0; i < WALK_MAXC; i++)
            if (i == c) {
                cid_[i] = cid;
                pos_[i] = p;
                z_[i] = zz;
            }
    }
};

template <>
struct WalkCells<false> {
    uint32_t *cid_, *pos_, *z_;
    __device__ inline WalkCells(const OvfDev &d, uint32_t j0) : cid_(d.scid + j0), pos_(d.spos + j0), z_(d.sz + j0) {}
    __device__ inline uint32_t pos(uint32_t c) const { return pos_[c]; }
    __device__ inline uint32_t z(uint32_t c) const { return z_[c]; }
    uint32_t n_ = 0;
    __device__ inline void zero_all() {
        for (uint32_t c = 0; c < n_; c++) z_[c] = 1;
    }
    __device__ inline int find(uint32_t cid, uint32_t n) {
        n_ = n;
        for (uint32_t c = 0; c < n; c++)
            if (cid_[c] == cid) return (int)c;
        return -1;
    }
    __device__ inline void put(uint32_t c, uint32_t cid, uint32_t p, uint32_t zz) {
        cid_[c] = cid;
        pos_[c] = p;
        z_[c] = zz;
        if (c + 1 > n_) n_ = c + 1;
    }
};

// The row's heap slot: its prior one, or a fresh one for a new row (the host made room), and its
// region entry: looked up for a row that existed before the apply, inserted for a new one
// (k_ovf_lookup told them apart; rowstore.h says why the two never interfere). Returns the entry.
// (rprior, the rows' prior counts until k_ovf_pload, holds a new row's heap slot in the walk.)
__device__ inline uint32_t ovf_row_slot(const MergeArgs &a, const OvfDev &d, uint32_t row, uint32_t &hb) {
    const uint32_t bb = a.ovf_list[d.rb[row]], own = d.rowner[row], t = d.tc[own] >> 16;
    hb = d.rheap[row];
    if (hb != ROW_NONE) return rs_lookup(a.rs, bb, d.pk[own], t);
    hb = d.rprior[row];  // (k_ovf_walk allocated it, one heap request per wave)
    if (hb == ROW_NONE)  // a new row of the sequential fold: its records now that it emits (the host made room)
        hb = (uint32_t)atomicAdd(a.rs.heap_top, (unsigned long long)a.rs.stride[t]);
    const uint64_t z[2] = {0, 0};
    return rs_insert(a.rs, bb, d.pk[own], t, hb, z);
}

// general: the row holds a sentinel clock or a long value (fast bodies stay out of its region)
__device__ inline void ovf_publish(const MergeArgs &a, const OvfDev &d, uint32_t row, uint32_t e,
                                   const uint64_t bits[2], uint32_t cnt, bool general) {
    a.rs.ent[e].bits[0] = bits[0];
    a.rs.ent[e].bits[1] = bits[1];
    if (a.touch) {
        const uint32_t own = d.rowner[row];
        touch_append(a, d.pk[own], d.tc[own] >> 16);
    }
    if (general) a.rs.gen[a.ovf_list[d.rb[row]]] = 1;
}

// emitter of the sequential fold when it runs here (rows outside App. A.3)
struct OvfEmit {
    const OvfDev *d;
    __device__ inline void emit(const MergeArgs &a, const OvfView &v, const GenArrays &g, uint32_t s, uint32_t row,
                                uint32_t ncell, bool hs, int64_t scv, uint32_t ssrc) {
        if (d->rheap[row] == ROW_NONE && !hs && ncell == 0) return;
        uint32_t hb;
        const uint32_t e = ovf_row_slot(a, *d, row, hb);
        uint64_t bits[2];
        bool gen;
        const uint32_t cnt = heap_write_row(a, v, g, s, ncell, hs, scv, ssrc, hb, bits, gen);
        ovf_publish(a, *d, row, e, bits, cnt, gen);
        atomicAdd(&a.misc[MISC_LIVE], (unsigned long long)cnt);
    }
};

// clock rows of one walked row (rf_emit on the carried cells) into its heap slot; returns them.
// xr: the row's last epoch record, L: the running max of cl before it; cell c's record is
// cx(c, z) (z: the cell was carried through a resurrection, col_version zeroed)
template <class CellX>
__device__ inline uint32_t ovf_emit_x(const MergeArgs &a, const OvfDev &d, uint32_t row, uint32_t xr, uint32_t L,
                                      uint32_t ncell, const CellX &cx) {
    const uint32_t clr = d.cl[xr], cidr = d.tc[xr] & 0xFFFFu;
    const bool hs = !(cidr != 0 && clr == 1 && L == 0);
    const int64_t scv = cidr == 0 ? d.cv[xr] : (int64_t)clr;
    const int64_t rowcl = hs ? scv : 1;
    const bool cells = (clr & 1u) != 0;
    const uint32_t cnt = (hs ? 1u : 0u) + (cells ? ncell : 0u);
    if (cnt == 0) return 0;
    uint32_t hb;
    const uint32_t e = ovf_row_slot(a, d, row, hb);
    const OvfView v{&a, &d};
    uint64_t bits[2] = {0, 0};
    bool general = hs;
    if (hs) {
        Rec r = load_rec(ovf_rec(a, d, xr));
        const uint64_t ts = a.track_ts ? rec_ts(a, v, r) : 0ULL;
        r.tcid &= 0xFFFF0000u;
        r.cv = scv;
        r.cl = (uint32_t)rowcl;
        r.v0 = 0;
        r.v1 = 0;
        r.meta = CORRO_NULL;
        r.pos = hb;
        store_rec(a.rs.heap + hb, r);
        if (a.track_ts) a.rs.heap_ts[hb] = ts;
        bits[0] |= 1ULL;
    }
    if (cells) {
        for (uint32_t c = 0; c < ncell; c++) {
            uint32_t z = 0;
            const uint32_t x = cx(c, z);
            Rec r = load_rec(ovf_rec(a, d, x));
            const uint64_t ts = a.track_ts ? rec_ts(a, v, r) : 0ULL;
            rec_clear_ts(a, r);
            const uint32_t cid = r.tcid & 0xFFFFu;
            if (z) r.cv = 0;
            r.cl = (uint32_t)rowcl;
            r.pos = hb + cid;
            store_rec(a.rs.heap + hb + cid, r);
            if (a.track_ts) a.rs.heap_ts[hb + cid] = ts;
            bits[cid >> 6] |= 1ULL << (cid & 63);
            if (is_long(r.meta)) general = true;
        }
    }
    ovf_publish(a, d, row, e, bits, cnt, general);
    return cnt;
}

template <bool REG>
__device__ inline uint32_t ovf_emit(const MergeArgs &a, const OvfDev &d, uint32_t row, const WalkCells<REG> &cells_,
                                    uint32_t ncell, uint32_t rpos) {
    return ovf_emit_x(a, d, row, d.val_s[rpos], d.lx[rpos], ncell, [&](uint32_t c, uint32_t &z) {
        z = cells_.z(c);
        return d.val_s[cells_.pos(c)];
    });
}

// fused form, a reduced row: its epoch record (rowE; nothing before it at a causal length > 0, so
// L = 0) gives the sentinel and the row's causal length, and at an odd Mx the row holds one cell per
// cid of C (all changed at Mx: C == F). Here: the row's heap slot and region entry, the sentinel and
// the presence bits; the cells themselves are written by k_ovf_rcells, one lane per cell, from the
// slot and cl left in rhb / rclw (a row's cells are independent stores: no per-row chain of loads).
__device__ inline uint32_t ovf_emit_redhead(const MergeArgs &a, const OvfDev &d, uint32_t row, uint32_t C) {
    const uint32_t xr = d.rowE[row];
    const uint32_t clr = d.cl[xr], cidr = d.tc[xr] & 0xFFFFu;
    const bool hs = !(cidr != 0 && clr == 1);
    const int64_t scv = cidr == 0 ? d.cv[xr] : (int64_t)clr;
    const int64_t rowcl = hs ? scv : 1;
    const uint32_t cids = (clr & 1u) ? (C & ~1u) : 0u;  // (cids < 32: reduction only runs below 32 columns)
    const uint32_t cnt = (hs ? 1u : 0u) + (uint32_t)__popc(cids);
    if (cnt == 0) return 0;
    uint32_t hb;
    const uint32_t e = ovf_row_slot(a, d, row, hb);
    uint64_t bits[2] = {(uint64_t)cids | (hs ? 1ULL : 0ULL), 0ULL};
    if (hs) {
        const OvfView v{&a, &d};
        Rec r = load_rec(ovf_rec(a, d, xr));
        const uint64_t ts = a.track_ts ? rec_ts(a, v, r) : 0ULL;
        r.tcid &= 0xFFFF0000u;
        r.cv = scv;
        r.cl = (uint32_t)rowcl;
        r.v0 = 0;
        r.v1 = 0;
        r.meta = CORRO_NULL;
        r.pos = hb;
        store_rec(a.rs.heap + hb, r);
        if (a.track_ts) a.rs.heap_ts[hb] = ts;
    }
    d.rhb[row] = hb;
    d.rclw[row] = (uint32_t)rowcl;
    ovf_publish(a, d, row, e, bits, cnt, hs);  // (a long winner value marks the region in k_ovf_rcells)
    return cnt;
}

#ifndef OVF_WALK_WAVES
#define OVF_WALK_WAVES 4  // 6 or 8 (spilling) measured no faster on config 5
#endif
// mode 0: every row (dense ids); fused form: 1 the reduced rows (rlist), 2 the others (flist) -- in
// separate launches, so no wave runs both the reduced emission and the walk
template <bool REG, int mode>
static __global__ void __launch_bounds__(256, OVF_WALK_WAVES) k_ovf_walk(MergeArgs a, OvfDev d) {
    const uint32_t lane = threadIdx.x & 63, stride = gridDim.x * blockDim.x;
    const uint32_t nr = mode == 0 ? d.nrows : d.nkeep[mode + 1];
    const uint32_t *const list = mode == 1 ? d.rlist : d.flist;
    uint32_t live = 0;  // clock rows written (one atomic per wave at the end)
    // one thread per row, every lane busy; wave-uniform loop for the heap requests
    for (uint32_t r0 = blockIdx.x * blockDim.x + threadIdx.x - lane; r0 < nr; r0 += stride) {
        const bool inr = r0 + lane < nr;
        const uint32_t row = !inr ? d.nrows : (mode == 0 ? r0 + lane : list[r0 + lane]);
        // fused form: a reduced row's summary (k_ovf_keep<true>); the owner record's words cleared for
        // the next apply (this row's last use of them)
        const bool red = mode == 1 && inr;
        uint32_t rmx = 0, rC = 0;
        if (red) {
            const uint64_t w = d.rsum[row];
            rmx = (uint32_t)(w >> 32);
            rC = (uint32_t)w;
        }
        if (mode != 0 && inr) {
            const uint32_t o = d.rowner[row];
            uint4 *sp = reinterpret_cast<uint4 *>(d.osum + o);
            sp[0] = make_uint4(0u, 0u, 0u, 0u);
            sp[1] = make_uint4(0u, 0u, 0u, 0u);
        }
        {  // the wave's new rows take their heap records in one request (the host made room). Rows of
           // the sequential fold (rbad) may emit nothing: they allocate only when they emit.
            uint32_t need = 0;
            const bool fresh = row < d.nrows && d.rheap[row] == ROW_NONE;
            if (fresh && (red || !d.rbad[row])) need = a.rs.stride[d.tc[d.rowner[row]] >> 16];
            else if (fresh) d.rprior[row] = ROW_NONE;
            uint32_t incl = need;
#pragma unroll
            for (int off = 1; off < 64; off <<= 1) {
                const uint32_t u = __shfl_up(incl, off);
                if ((int)lane >= off) incl += u;
            }
            const uint32_t tot = __shfl(incl, 63);
            unsigned long long base = 0;
            if (lane == 63 && tot) base = atomicAdd(a.rs.heap_top, (unsigned long long)tot);
            base = __shfl(base, 63);
            if (need) d.rprior[row] = (uint32_t)base + incl - need;
        }
        if (row >= d.nrows) continue;
        if constexpr (mode == 1) {  // (a row whose every record has cl 0 has no record and emits nothing, as below)
            if (rmx) live += ovf_emit_redhead(a, d, row, rC);
            continue;
        }
        const uint32_t j0 = d.rstart[row];
        if (d.rbad[row]) {  // outside App. A.3: the sequential fold over the row's sorted records
            if (a.impact)  // (k_ovf_classify flagged its records before the row was known to be bad;
                           // the fold stores only nonzero flags)
                for (uint32_t p = j0; p < d.K && (uint32_t)(d.key_s[p] >> d.rshift) == row; p++) {
                    const uint32_t pos = d.pos[d.val_s[p]];
                    if (pos & BATCH_POS) a.impact[pos & 0x7FFFFFFFu] = 0;
                }
            GenArrays g{};
            g.key = d.key_s;
            g.val = d.val_s;
            g.pk = d.pk;
            g.cv = d.cv;
            g.tc = d.tc;
            g.cl = d.cl;
            g.pos = d.pos;
            g.ccid = d.ccid;
            g.csrc = d.csrc;
            g.ccv = d.ccv;
            g.own = nullptr;
            g.slots = 0;
            g.rshift = d.rshift;
            g.P = d.K;
            OvfEmit em{&d};
            gen_fold_row(a, OvfView{&a, &d}, em, g, j0, d.K);
            continue;
        }
        const uint32_t nrec = d.rnrec[row];
        uint32_t ncell = 0;
        WalkCells<REG> cs(d, j0);
        // A delete record (even cl) drops every cell, so without impacts (which need every epoch's
        // carried cells, fstg) the walk starts at the row's last delete: hot rows skip their history.
        uint32_t k0 = 0;
        if (!a.impact)
            for (uint32_t k = nrec; k-- > 0;)
                if ((d.cl[d.val_s[d.recs[j0 + k]]] & 1u) == 0) {
                    k0 = k;
                    break;
                }
        for (uint32_t k = k0; k < nrec; k++) {
            const uint32_t R = d.recs[j0 + k];
            const uint32_t xR = d.val_s[R];
            if ((d.cl[xR] & 1u) == 0) {
                ncell = 0;
                continue;
            }
            cs.find(0xFFFFFFFFu, ncell);  // (sizes the global store's zeroing)
            cs.zero_all();
            auto set = [&](uint32_t cid, uint32_t p, uint32_t z) {
                const int f = cs.find(cid, ncell);
                if (f >= 0) {
                    cs.put((uint32_t)f, cid, p, z);
                    return;
                }
                cs.put(ncell, cid, p, z);
                ncell++;
            };
            const uint32_t cidR = d.tc[xR] & 0xFFFFu;
            if (cidR != 0) set(cidR, R, 0);
            for (uint32_t h = d.head[R]; h; h = d.nxt[h - 1]) {
                const uint32_t qe = h - 1;  // the group's last candidate
                const uint32_t cid = (uint32_t)d.ckey_s[qe] & ((1u << d.cid_bits) - 1);
                const int found = cs.find(cid, ncell);
                const uint32_t fp = found < 0 ? 0u : cs.pos((uint32_t)found), fz = found < 0 ? 0u : cs.z((uint32_t)found);
                if (a.impact) d.fstg[d.cgs[qe]] = found < 0 ? 0u : ((fp + 1) | (fz << 31));
                const uint32_t wq = d.cbest[qe];
                if (found < 0 || ovf_kcmp(ovf_key_q(d, wq), ovf_key_p(a, d, fp, fz != 0), d.arena) > 0) set(cid, d.cval_s[wq], 0);
            }
        }
        if (nrec) live += ovf_emit<REG>(a, d, row, cs, ncell, d.recs[j0 + nrec - 1]);
    }
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) live += __shfl_xor(live, off);
    if (lane == 0 && live) atomicAdd(&a.misc[MISC_LIVE], (unsigned long long)live);
}

static __global__ void k_ovf_impacts(MergeArgs a, OvfDev d) {
    OVF_LOOP(q, d.ncand) {
        const uint64_t k = d.ckey_s[q];
        if (d.rbad[d.rowid[(uint32_t)(k >> d.cid_bits)]]) continue;
        const uint32_t p = d.cval_s[q];
        const uint32_t pos = d.pos[d.val_s[p]];
        if (!(pos & BATCH_POS)) continue;
        const bool first = q == 0 || d.ckey_s[q - 1] != k;
        const OvfKey kq = ovf_key_q(d, q);
        bool imp = first || ovf_kcmp(kq, ovf_key_q(d, d.cbest[q - 1]), d.arena) > 0;
        const uint32_t fs = d.fstg[d.cgs[q]];
        if (imp && fs) imp = ovf_kcmp(kq, ovf_key_p(a, d, (fs & 0x7FFFFFFFu) - 1, (fs >> 31) != 0), d.arena) > 0;
        if (imp) a.impact[pos & 0x7FFFFFFFu] = 1;
    }
}

static __global__ void k_ovf_finish(MergeArgs a, OvfDev d) {
    OVF_LOOP(b, d.G) a.rs.used[a.ovf_list[b]] += d.bnew[b];
}

// Running argmax of the candidates by group (cbest): a segmented scan with the 32-B keys compared
// in registers. k_cscan_tile: each wave scans 8 chunks of 64 consecutive candidates (coalesced
// loads, shuffle scan, carry from chunk to chunk), the workgroup combines its 4 waves; every
// element after the tile's first group head is final. The tile aggregates are scanned by rocPRIM
// (prims.hip, a few thousand entries), then k_cscan_fix gives each tile's leading open group its
// carry.
constexpr uint32_t CS_T = 256, CS_W = CS_T / 64, CS_C = 8, CS_TILE = CS_T * CS_C;

struct CsAgg {
    uint32_t head;  // a group starts inside
    uint32_t best;  // running argmax of the last group (~0u: none)
};

// a beats b: strictly greater, or (pos: the fused form's cells, whose sort order is not the
// application order) equal and earlier
__device__ inline bool cs_beats(const OvfKey &a, uint32_t ap, const OvfKey &b, uint32_t bp, const uint8_t *arena, bool pos) {
    const int c = ovf_kcmp(a, b, arena);
    return c > 0 || (pos && c == 0 && ap < bp);
}

// x precedes y; ~0u = none. The later one only when it beats the earlier (earliest on ties).
__device__ inline uint32_t cs_pick(const OvfKey *qk, const uint32_t *qp, uint32_t x, uint32_t y, const uint8_t *arena) {
    if (x == ~0u) return y;
    if (y == ~0u) return x;
    return cs_beats(qk[y], qp ? qp[y] : 0u, qk[x], qp ? qp[x] : 0u, arena, qp != nullptr) ? y : x;
}

struct CsComb {
    const OvfKey *qk;
    const uint8_t *arena;
    const uint32_t *qp;  // (nullptr: order decides ties)
    __device__ inline CsAgg operator()(const CsAgg &a, const CsAgg &b) const {
        return b.head ? b : CsAgg{a.head, cs_pick(qk, qp, a.best, b.best, arena)};
    }
};

__device__ inline OvfKey shfl_up_key(const OvfKey &k, int off) {
    OvfKey r;
    r.cv = __shfl_up(k.cv, off);
    r.k0 = __shfl_up(k.k0, off);
    r.k1 = __shfl_up(k.k1, off);
    r.m = __shfl_up(k.m, off);
    r.sr = __shfl_up(k.sr, off);
    return r;
}

__device__ inline OvfKey shfl_key(const OvfKey &k, int src) {
    OvfKey r;
    r.cv = __shfl(k.cv, src);
    r.k0 = __shfl(k.k0, src);
    r.k1 = __shfl(k.k1, src);
    r.m = __shfl(k.m, src);
    r.sr = __shfl(k.sr, src);
    return r;
}

template <bool POS>
static __global__ void __launch_bounds__(CS_T) k_cscan_tile(OvfDev d, CsAgg *tagg, uint32_t *tfirst) {
    __shared__ uint32_t s_head[CS_W], s_best[CS_W], s_first[CS_W], s_pos[CS_W];
    __shared__ OvfKey s_key[CS_W];
    const uint32_t *const qp = POS ? d.qpos : nullptr;
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint32_t t0 = blockIdx.x * CS_TILE, base = t0 + w * (CS_C * 64);
    if (d.ckey_s[t0] == ~0ULL) {  // the non-candidates' key sorts last: no cbest is read there
        if (threadIdx.x == 0) {
            tagg[blockIdx.x] = CsAgg{1u, ~0u};
            tfirst[blockIdx.x] = 0;
        }
        return;
    }
    uint32_t res[CS_C];
    bool open[CS_C];
    uint32_t ch = 0, cb = ~0u, cp = 0, first = CS_C * 64;  // wave carry: head seen, best (+ its position); first head offset
    OvfKey ck{};
#pragma unroll
    for (uint32_t c = 0; c < CS_C; c++) {
        const uint32_t q = base + c * 64 + lane;
        const bool valid = q < d.K;
        uint32_t h = 0, b = ~0u, kp = 0;
        OvfKey k{};
        if (valid) {
            const uint64_t kk = d.ckey_s[q];
            h = (q == 0 || d.ckey_s[q - 1] != kk) ? 1u : 0u;
            b = q;
            k = d.qkey[q];
            if (POS) kp = qp[q];
        }
        const uint64_t hb = __ballot(h != 0);
        if (hb && first == CS_C * 64) first = c * 64 + (uint32_t)(__ffsll((unsigned long long)hb) - 1);
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const uint32_t lh = __shfl_up(h, off), lb = __shfl_up(b, off);
            const uint32_t lp = POS ? (uint32_t)__shfl_up(kp, off) : 0u;
            const OvfKey lk = shfl_up_key(k, off);
            if ((int)lane >= off && !h) {
                h = lh;
                if (lb != ~0u && (b == ~0u || !cs_beats(k, kp, lk, lp, d.arena, POS))) {
                    b = lb;
                    k = lk;
                    kp = lp;
                }
            }
        }
        if (!h && cb != ~0u && (b == ~0u || !cs_beats(k, kp, ck, cp, d.arena, POS))) {
            b = cb;
            k = ck;
            kp = cp;
        }
        res[c] = b;
        open[c] = !h && !ch;
        ch |= __shfl(h, 63);
        cb = __shfl(b, 63);
        if (POS) cp = __shfl(kp, 63);
        ck = shfl_key(k, 63);
    }
    if (lane == 0) {
        s_head[w] = ch;
        s_best[w] = cb;
        s_key[w] = ck;
        s_pos[w] = cp;
        s_first[w] = w * (CS_C * 64) + first;
    }
    __syncthreads();
    // carry from the earlier waves of the tile
    uint32_t pb = ~0u;
    for (uint32_t v = 0; v < w; v++) {
        if (s_head[v]) pb = s_best[v];
        else if (s_best[v] != ~0u &&
                 (pb == ~0u || cs_beats(s_key[v], s_pos[v], d.qkey[pb], POS ? qp[pb] : 0u, d.arena, POS)))
            pb = s_best[v];
    }
#pragma unroll
    for (uint32_t c = 0; c < CS_C; c++) {
        const uint32_t q = base + c * 64 + lane;
        if (q >= d.K) continue;
        d.cbest[q] = open[c] ? cs_pick(d.qkey, qp, pb, res[c], d.arena) : res[c];
    }
    if (threadIdx.x == 0) {
        CsAgg agg{0u, ~0u};
        uint32_t f = CS_TILE;
        for (uint32_t v = 0; v < CS_W; v++) {
            if (s_head[v]) {
                agg.head = 1;
                agg.best = s_best[v];
                if (f == CS_TILE) f = s_first[v];
            } else {
                agg.best = cs_pick(d.qkey, qp, agg.best, s_best[v], d.arena);
            }
        }
        tagg[blockIdx.x] = agg;
        tfirst[blockIdx.x] = f;
    }
}

// tincl: inclusive scan of the tile aggregates; tile t's leading open group takes tincl[t - 1]
template <bool POS>
static __global__ void __launch_bounds__(CS_T) k_cscan_fix(OvfDev d, const CsAgg *tincl, const uint32_t *tfirst) {
    const uint32_t t = blockIdx.x;
    if (t == 0) return;
    const uint32_t c = tincl[t - 1].best;
    const uint32_t t0 = t * CS_TILE;
    if (c == ~0u || d.ckey_s[t0] == ~0ULL) return;
    const uint32_t e = min(d.K, t0 + tfirst[t]);
    for (uint32_t q = t0 + threadIdx.x; q < e; q += CS_T) d.cbest[q] = cs_pick(d.qkey, POS ? d.qpos : nullptr, c, d.cbest[q], d.arena);
}

// fused form: the reduced rows' column records at Mx sorted by cell key (owner << cid_bits | cid) in
// (key_s, val_s): their cell keys and positions in sorted order for the argmax
static __global__ void k_ovf_rgather(MergeArgs a, OvfDev d, uint32_t nc, uint32_t *qpos) {
    OVF_LOOP(q, nc) {
        const uint32_t x = d.val_s[q];
        d.qkey[q] = ovf_key_x(a, d, x);
        qpos[q] = d.pos[x];  // (prior records' slots < BATCH_POS | batch index: application order)
    }
}

// each reduced cell's winner (the running argmax at its last sorted record) written to its heap slot
// (after k_ovf_walk mode 1 gave the row its slot and cl; one lane per cell)
static __global__ void k_ovf_rcells(MergeArgs a, OvfDev d, uint32_t nc) {
    OVF_LOOP(q, nc) {
        const uint64_t k = d.key_s[q];
        if (q + 1 < nc && d.key_s[q + 1] == k) continue;
        const uint32_t o = (uint32_t)(k >> d.cid_bits), row = d.epc[o] - 1u;
        const uint32_t hb = d.rhb[row];
        Rec r = load_rec(ovf_rec(a, d, d.val_s[d.cbest[q]]));
        const OvfView v{&a, &d};
        const uint64_t ts = a.track_ts ? rec_ts(a, v, r) : 0ULL;
        rec_clear_ts(a, r);
        const uint32_t cid = r.tcid & 0xFFFFu;
        r.cl = d.rclw[row];
        r.pos = hb + cid;
        store_rec(a.rs.heap + hb + cid, r);
        if (a.track_ts) a.rs.heap_ts[hb + cid] = ts;
        if (is_long(r.meta)) a.rs.gen[a.ovf_list[d.rb[row]]] = 1;
    }
}

#undef OVF_LOOP

}  // namespace corro
