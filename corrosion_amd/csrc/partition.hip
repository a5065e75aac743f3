// pk-hash partition of a change batch across the ranks of one node.
//
// Each row (table, pk) is owned by exactly one rank, so after one all-to-all exchange every rank
// merges its rows independently. The partition is STABLE: a rank receives its changes in the
// sender's order, and with senders concatenated by rank the application order of the global batch
// (actors by id, then arrival) is preserved for every row.
//
// rank_of(table, pk) uses the LOW 32 bits of the same 64-bit mix whose top bits pick the merge
// bucket (merge_kernels.h bucket_of), so a rank's rows still spread over all of its buckets.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <vector>

#include "internal.h"
#include "rowhash.h"

#define TRY_PART(x)                      \
    do {                                 \
        int rc_ = (x);                   \
        if (rc_ != CORRO_OK) return rc_; \
    } while (0)

namespace corro {
int prim_inclusive_scan_u32(void *temp, size_t *temp_bytes, const uint32_t *in, uint32_t *out, uint32_t n,
                            hipStream_t s);

constexpr int PART_THREADS = 256;
constexpr int PART_MAX_RANKS = 64;

__host__ __device__ inline uint32_t rank_of(uint32_t table, uint64_t pk, uint32_t nranks) {
    const uint64_t h = mix64(pk + 0x9E3779B97F4A7C15ULL * (uint64_t)(table + 1));
    return (uint32_t)(h & 0xFFFFFFFFULL) % nranks;
}

// per tile: count of changes per destination rank
__global__ void __launch_bounds__(PART_THREADS)
k_part_count(BatchDev in, uint32_t tile, uint32_t nranks, uint32_t *__restrict__ counts) {
    __shared__ uint32_t c[PART_MAX_RANKS];
    for (uint32_t r = threadIdx.x; r < nranks; r += blockDim.x) c[r] = 0;
    __syncthreads();
    const uint32_t begin = blockIdx.x * tile, end = min(in.n, begin + tile);
    for (uint32_t i = begin + threadIdx.x; i < end; i += blockDim.x)
        atomicAdd(&c[rank_of(in.tcid[i] >> 16, in.pk[i], nranks)], 1u);
    __syncthreads();
    for (uint32_t r = threadIdx.x; r < nranks; r += blockDim.x) counts[(size_t)blockIdx.x * nranks + r] = c[r];
}

// one workgroup: counts[t][r] -> absolute output position of tile t's first change for rank r;
// totals[r] = changes for rank r. cap > 0: rank r's group starts at r * cap (the slot layout)
__global__ void k_part_scan(uint32_t *__restrict__ counts, uint32_t ntiles, uint32_t nranks,
                            uint64_t *__restrict__ totals, uint64_t cap = 0, unsigned long long *err = nullptr) {
    __shared__ uint64_t base[PART_MAX_RANKS];
    if (err && threadIdx.x == 0) *err = 0;  // (the slot partition's validation word, set by k_part_pack)
    if (threadIdx.x < nranks) {
        const uint32_t r = threadIdx.x;
        uint64_t run = 0;
        for (uint32_t t = 0; t < ntiles; t++) {
            const uint32_t x = counts[(size_t)t * nranks + r];
            counts[(size_t)t * nranks + r] = (uint32_t)run;
            run += x;
        }
        totals[r] = run;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        uint64_t run = 0;
        for (uint32_t r = 0; r < nranks; r++) {
            base[r] = cap ? (uint64_t)r * cap : run;
            run += totals[r];
        }
    }
    __syncthreads();
    if (threadIdx.x < nranks)
        for (uint32_t t = 0; t < ntiles; t++) counts[(size_t)t * nranks + threadIdx.x] += (uint32_t)base[threadIdx.x];
}

struct BatchOut {
    uint64_t *pk;
    uint32_t *tcid;
    int64_t *cv;
    int64_t *dbv;
    uint32_t *cl;
    uint32_t *seq;
    uint32_t *site;
    uint64_t *v0;
    uint64_t *v1;
    uint8_t *vt;
    uint8_t *vl;
    uint64_t *ts;
};

// stable scatter: chunks of PART_THREADS changes in order; wave ballots rank lanes per destination
__global__ void __launch_bounds__(PART_THREADS)
k_part_scatter(BatchDev in, uint32_t tile, uint32_t nranks, const uint32_t *__restrict__ offs, BatchOut o) {
    __shared__ uint32_t run[PART_MAX_RANKS];
    __shared__ uint32_t wcnt[PART_THREADS / 64][PART_MAX_RANKS];
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (uint32_t r = threadIdx.x; r < nranks; r += blockDim.x) run[r] = offs[(size_t)blockIdx.x * nranks + r];
    __syncthreads();
    const uint32_t begin = blockIdx.x * tile, end = min(in.n, begin + tile);
    const uint64_t lt = (lane == 0) ? 0ULL : (~0ULL >> (64 - lane));
    for (uint32_t base = begin; base < end; base += blockDim.x) {
        const uint32_t i = base + threadIdx.x;
        const bool act = i < end;
        const uint32_t d = act ? rank_of(in.tcid[i] >> 16, in.pk[i], nranks) : 0xFFFFFFFFu;
        uint32_t my_rank = 0;
        for (uint32_t r = 0; r < nranks; r++) {
            const uint64_t m = __ballot(d == r);
            if (d == r) my_rank = __popcll(m & lt);
            if (lane == 0) wcnt[w][r] = __popcll(m);
        }
        __syncthreads();
        uint32_t pos = 0;
        if (act) {
            pos = run[d] + my_rank;
            for (uint32_t ww = 0; ww < w; ww++) pos += wcnt[ww][d];
            o.pk[pos] = in.pk[i];
            o.tcid[pos] = in.tcid[i];
            o.cv[pos] = in.cv[i];
            o.dbv[pos] = in.dbv[i];
            o.cl[pos] = in.cl[i];
            o.seq[pos] = in.seq[i];
            o.site[pos] = in.site[i];
            o.v0[pos] = in.v0[i];
            if (o.v1) o.v1[pos] = in.v1 ? in.v1[i] : 0ULL;
            if (o.vt) o.vt[pos] = in.vt ? in.vt[i] : (uint8_t)CORRO_INTEGER;
            if (o.vl) o.vl[pos] = in.vl ? in.vl[i] : 0;
            if (o.ts) o.ts[pos] = in.ts ? in.ts[i] : 0ULL;
        }
        __syncthreads();
        if (threadIdx.x < nranks) {
            uint32_t add = 0;
            for (uint32_t ww = 0; ww < PART_THREADS / 64; ww++) add += wcnt[ww][threadIdx.x];
            run[threadIdx.x] += add;
        }
        __syncthreads();
    }
}

// Packed-record exchange format (one all-to-all of whole records instead of one per SoA field):
// PLAIN batches (INTEGER values, no val1/val_type/val_len/ts arrays) use the 48-B record of
// SURVEY §8(d); others a 80-B record that carries every optional field.
using PackedRec48 = SlotRec;  // (rowhash.h: the receiver's apply reads it in slot mode)
struct __attribute__((aligned(16))) PackedRec80 {
    uint64_t pk;
    int64_t cv, dbv;
    uint64_t v0, v1, ts;
    uint32_t tcid, cl, seq, site, meta, pad[3];
};
static_assert(sizeof(PackedRec48) == 48 && sizeof(PackedRec80) == 80, "packed record sizes");

// The slot partition validates what it packs (the checks corro_apply_batch makes before its first
// write: names, site ordinal, causal-length ranges, db_version), so the receiver can apply the slots
// in several chunks without a whole-layout validation pass first; err != null turns it on.
struct PartCheck {
    const uint16_t *ncols;
    uint32_t ntables, nsites;
    unsigned long long *err;
};

// stable scatter of whole records (same ranking as k_part_scatter); perm[pos] = source index
template <bool PLAIN>
__global__ void __launch_bounds__(PART_THREADS)
k_part_pack(BatchDev in, uint32_t tile, uint32_t nranks, const uint32_t *__restrict__ offs, void *__restrict__ out,
            uint32_t *__restrict__ perm, uint64_t cap = 0, PartCheck chk = PartCheck{}) {
    __shared__ uint32_t run[PART_MAX_RANKS];
    __shared__ uint32_t wcnt[PART_THREADS / 64][PART_MAX_RANKS];
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (uint32_t r = threadIdx.x; r < nranks; r += blockDim.x) run[r] = offs[(size_t)blockIdx.x * nranks + r];
    __syncthreads();
    const uint32_t begin = blockIdx.x * tile, end = min(in.n, begin + tile);
    const uint64_t lt = (lane == 0) ? 0ULL : (~0ULL >> (64 - lane));
    for (uint32_t base = begin; base < end; base += blockDim.x) {
        const uint32_t i = base + threadIdx.x;
        const bool act = i < end;
        const uint32_t ic = act ? i : begin;
        const uint64_t pk = in.pk[ic];
        const uint32_t tc = in.tcid[ic];
        const uint32_t d = act ? rank_of(tc >> 16, pk, nranks) : 0xFFFFFFFFu;
        uint32_t my_rank = 0;
        for (uint32_t r = 0; r < nranks; r++) {
            const uint64_t m = __ballot(d == r);
            if (d == r) my_rank = __popcll(m & lt);
            if (lane == 0) wcnt[w][r] = __popcll(m);
        }
        if (PLAIN && chk.err) {
            bool bad = false;
            if (act) {
                const uint32_t t = tc >> 16, cid = tc & 0xFFFFu, cl = in.cl[i];
                const int64_t cv = in.cv[i];
                bad = t >= chk.ntables || cid > chk.ncols[t] || in.site[i] >= chk.nsites ||
                      ((cid == 0 || (cl & 1u) == 0) && (cv < 0 || cv > 0xFFFFFFFFLL)) || in.dbv[i] < 0;
            }
            if (__ballot(bad) && lane == 0) atomicOr(chk.err, 1ULL);
        }
        __syncthreads();
        if (act) {
            uint32_t pos = run[d] + my_rank;
            for (uint32_t ww = 0; ww < w; ww++) pos += wcnt[ww][d];
            // (slot layout: a record past rank d's slot is counted, not written -- the receiver sees
            // the count and the caller repeats the exchange with exact sizes)
            if (cap && pos >= (uint64_t)(d + 1) * cap) goto next;
            if (PLAIN) {
                PackedRec48 r{pk, in.cv[i], in.dbv[i], in.v0[i], tc, in.cl[i], in.seq[i], in.site[i]};
                static_cast<PackedRec48 *>(out)[pos] = r;
            } else {
                PackedRec80 r{};
                r.pk = pk;
                r.cv = in.cv[i];
                r.dbv = in.dbv[i];
                r.v0 = in.v0[i];
                r.v1 = in.v1 ? in.v1[i] : 0ULL;
                r.ts = in.ts ? in.ts[i] : 0ULL;
                r.tcid = tc;
                r.cl = in.cl[i];
                r.seq = in.seq[i];
                r.site = in.site[i];
                r.meta = (in.vt ? (uint32_t)in.vt[i] : (uint32_t)CORRO_INTEGER) | ((in.vl ? (uint32_t)in.vl[i] : 0u) << 8);
                static_cast<PackedRec80 *>(out)[pos] = r;
            }
            if (perm) perm[pos] = i;
        }
    next:
        __syncthreads();
        if (threadIdx.x < nranks) {
            uint32_t add = 0;
            for (uint32_t ww = 0; ww < PART_THREADS / 64; ww++) add += wcnt[ww][threadIdx.x];
            run[threadIdx.x] += add;
        }
        __syncthreads();
    }
}

// received slots -> SoA at the same indices, ap[i] = i (received) / AP_SKIP (padding, or every slot
// when a source overflowed its slot: the apply is then a no-op and the caller repeats the exchange)
__global__ void k_unpack_slots(const PackedRec48 *__restrict__ recs, uint32_t nsrc, uint64_t cap,
                               const uint64_t *__restrict__ cnt, BatchOut o, uint32_t *__restrict__ ap,
                               uint32_t *__restrict__ overflow) {
    bool over = false;
    for (uint32_t s = 0; s < nsrc; s++) over |= cnt[s] > cap;
    const uint64_t n = (uint64_t)nsrc * cap;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t s = (uint32_t)(i / cap);
        const bool valid = !over && i - (uint64_t)s * cap < cnt[s];
        if (valid) {
            const PackedRec48 r = recs[i];
            o.pk[i] = r.pk; o.cv[i] = r.cv; o.dbv[i] = r.dbv; o.v0[i] = r.v0;
            o.tcid[i] = r.tcid; o.cl[i] = r.cl; o.seq[i] = r.seq; o.site[i] = r.site;
        } else {  // padding: fields no check trips over (never merged: ap = skip)
            o.pk[i] = 0; o.cv[i] = 1; o.dbv[i] = 0; o.v0[i] = 0;
            o.tcid[i] = 0xFFFFFFFFu; o.cl[i] = 1; o.seq[i] = 0; o.site[i] = 0xFFFFFFFFu;
        }
        ap[i] = valid ? (uint32_t)i : AP_SKIP;
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) *overflow = over ? 1u : 0u;
}

// received records (source-rank order) -> the SoA batch corro_apply_batch takes
template <bool PLAIN>
__global__ void k_unpack(const void *__restrict__ recs, uint32_t n, BatchOut o) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        if (PLAIN) {
            const PackedRec48 r = static_cast<const PackedRec48 *>(recs)[i];
            o.pk[i] = r.pk; o.cv[i] = r.cv; o.dbv[i] = r.dbv; o.v0[i] = r.v0;
            o.tcid[i] = r.tcid; o.cl[i] = r.cl; o.seq[i] = r.seq; o.site[i] = r.site;
        } else {
            const PackedRec80 r = static_cast<const PackedRec80 *>(recs)[i];
            o.pk[i] = r.pk; o.cv[i] = r.cv; o.dbv[i] = r.dbv; o.v0[i] = r.v0;
            o.tcid[i] = r.tcid; o.cl[i] = r.cl; o.seq[i] = r.seq; o.site[i] = r.site;
            if (o.v1) o.v1[i] = r.v1;
            if (o.ts) o.ts[i] = r.ts;
            if (o.vt) o.vt[i] = (uint8_t)(r.meta & 0xFFu);
            if (o.vl) o.vl[i] = (uint8_t)(r.meta >> 8);
        }
    }
}

// ---- every table: interned pks routed by their canonical bytes, variable-length bytes shipped ----
// Owner of a change: INTEGER-pk rows by rank_of (the pk is the row key on every engine); rows of an
// interned table by the route hash of their canonical packed pk (the dense row key is per engine).
// A table id at or past ntables (not registered: the receiving merge rejects it) is routed like an
// INTEGER pk and never dereferences the directory.
__device__ inline uint32_t route_of(const PkDir *dir, uint32_t ntables, uint32_t table, uint64_t key, uint32_t nranks) {
    if (dir && table < ntables && dir[table].interned) {
        const uint64_t h = key < dir[table].n ? dir[table].hash[key] : 0ULL;
        return (uint32_t)(mix64(h ^ (0x9E3779B97F4A7C15ULL * (uint64_t)(table + 1))) & 0xFFFFFFFFULL) % nranks;
    }
    return rank_of(table, key, nranks);
}

__global__ void __launch_bounds__(PART_THREADS)
k_partv_count(BatchDev in, const PkDir *dir, uint32_t ntables, uint32_t tile, uint32_t nranks, uint32_t *__restrict__ counts) {
    __shared__ uint32_t c[PART_MAX_RANKS];
    for (uint32_t r = threadIdx.x; r < nranks; r += blockDim.x) c[r] = 0;
    __syncthreads();
    const uint32_t begin = blockIdx.x * tile, end = min(in.n, begin + tile);
    for (uint32_t i = begin + threadIdx.x; i < end; i += blockDim.x)
        atomicAdd(&c[route_of(dir, ntables, in.tcid[i] >> 16, in.pk[i], nranks)], 1u);
    __syncthreads();
    for (uint32_t r = threadIdx.x; r < nranks; r += blockDim.x) counts[(size_t)blockIdx.x * nranks + r] = c[r];
}

// bytes change i ships: its canonical pk (interned table) then its long value's bytes
__device__ inline void var_parts(const BatchDev &in, const PkDir *dir, uint32_t ntables, uint32_t i, uint32_t &pk_len,
                                 uint32_t &vsz) {
    const uint32_t t = in.tcid[i] >> 16;
    pk_len = 0;
    if (t < ntables && dir[t].interned && in.pk[i] < dir[t].n) pk_len = (uint32_t)(dir[t].off[in.pk[i] + 1] - dir[t].off[in.pk[i]]);
    vsz = 0;
    if (in.voff && in.vsz && in.vt && in.vl && in.vl[i] == CORRO_VAL_LONG && (in.vt[i] == CORRO_TEXT || in.vt[i] == CORRO_BLOB)) {
        const uint64_t off = in.voff[i];
        const uint32_t sz = in.vsz[i];
        if (sz > 16 && sz < (1u << 24) && off <= in.ldata && sz <= in.ldata - off) vsz = sz;
    }
}

// stable scatter of 80-B records (route_of), perm[pos] = source, vlen[pos] = bytes it ships
__global__ void __launch_bounds__(PART_THREADS)
k_partv_pack(BatchDev in, const PkDir *dir, uint32_t ntables, uint32_t tile, uint32_t nranks, const uint32_t *__restrict__ offs,
             PackedRec80 *__restrict__ out, uint32_t *__restrict__ perm, uint32_t *__restrict__ vlen) {
    __shared__ uint32_t run[PART_MAX_RANKS];
    __shared__ uint32_t wcnt[PART_THREADS / 64][PART_MAX_RANKS];
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (uint32_t r = threadIdx.x; r < nranks; r += blockDim.x) run[r] = offs[(size_t)blockIdx.x * nranks + r];
    __syncthreads();
    const uint32_t begin = blockIdx.x * tile, end = min(in.n, begin + tile);
    const uint64_t lt = (lane == 0) ? 0ULL : (~0ULL >> (64 - lane));
    for (uint32_t base = begin; base < end; base += blockDim.x) {
        const uint32_t i = base + threadIdx.x;
        const bool act = i < end;
        const uint32_t ic = act ? i : begin;
        const uint64_t pk = in.pk[ic];
        const uint32_t tc = in.tcid[ic];
        const uint32_t d = act ? route_of(dir, ntables, tc >> 16, pk, nranks) : 0xFFFFFFFFu;
        uint32_t my_rank = 0;
        for (uint32_t r = 0; r < nranks; r++) {
            const uint64_t m = __ballot(d == r);
            if (d == r) my_rank = __popcll(m & lt);
            if (lane == 0) wcnt[w][r] = __popcll(m);
        }
        __syncthreads();
        if (act) {
            uint32_t pos = run[d] + my_rank;
            for (uint32_t ww = 0; ww < w; ww++) pos += wcnt[ww][d];
            PackedRec80 r{};
            r.pk = pk;
            r.cv = in.cv[i];
            r.dbv = in.dbv[i];
            r.v0 = in.v0[i];
            r.v1 = in.v1 ? in.v1[i] : 0ULL;
            r.ts = in.ts ? in.ts[i] : 0ULL;
            r.tcid = tc;
            r.cl = in.cl[i];
            r.seq = in.seq[i];
            r.site = in.site[i];
            r.meta = (in.vt ? (uint32_t)in.vt[i] : (uint32_t)CORRO_INTEGER) | ((in.vl ? (uint32_t)in.vl[i] : 0u) << 8);
            uint32_t pl, vs;
            var_parts(in, dir, ntables, i, pl, vs);
            r.pad[1] = pl;
            r.pad[2] = vs;
            out[pos] = r;
            perm[pos] = i;
            vlen[pos] = pl + vs;
        }
        __syncthreads();
        if (threadIdx.x < nranks) {
            uint32_t add = 0;
            for (uint32_t ww = 0; ww < PART_THREADS / 64; ww++) add += wcnt[ww][threadIdx.x];
            run[threadIdx.x] += add;
        }
        __syncthreads();
    }
}

// record pos: its bytes at var[vincl[pos] - vlen[pos]], its offset inside its rank's segment in
// pad[0] (the receiver adds the segment's base); one wave per record copies the bytes
__global__ void __launch_bounds__(PART_THREADS)
k_partv_fill(BatchDev in, const PkDir *dir, uint32_t n, const uint32_t *__restrict__ perm, const uint32_t *__restrict__ vlen,
             const uint32_t *__restrict__ vincl, const uint64_t *__restrict__ seg_base, const uint64_t *__restrict__ rec_base,
             uint32_t nranks, PackedRec80 *__restrict__ out, uint8_t *__restrict__ var) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t w0 = (blockIdx.x * blockDim.x + threadIdx.x) >> 6, nw = gridDim.x * blockDim.x / 64;
    for (uint32_t pos = w0; pos < n; pos += nw) {
        const uint32_t L = vlen[pos];
        const uint64_t at = (uint64_t)vincl[pos] - L;
        uint32_t r = 0;  // destination rank: the last whose first record is at or before pos
        while (r + 1 < nranks && rec_base[r + 1] <= pos) r++;
        if (lane == 0) out[pos].pad[0] = (uint32_t)(at - seg_base[r]);
        if (!L) continue;
        const uint32_t i = perm[pos];
        const uint32_t pl = out[pos].pad[1], vs = out[pos].pad[2];
        if (pl) {
            const uint8_t *src = dir[in.tcid[i] >> 16].bytes + dir[in.tcid[i] >> 16].off[in.pk[i]];
            for (uint32_t k = lane; k < pl; k += 64) var[at + k] = src[k];
        }
        if (vs) {
            const uint8_t *src = in.arena + in.voff[i];
            for (uint32_t k = lane; k < vs; k += 64) var[at + pl + k] = src[k];
        }
    }
}

// received records (source-rank order, var segments concatenated the same way) -> SoA; long
// values' val_off point into the received var bytes (the batch's val_data); interned records'
// (pk bytes offset, length) listed in pkref for the host's interning
__global__ void k_unpackv(const PackedRec80 *__restrict__ recs, uint32_t n, const uint64_t *__restrict__ src_rec,
                          const uint64_t *__restrict__ src_var, uint32_t nsrc, BatchOut o, uint64_t *__restrict__ voff,
                          uint32_t *__restrict__ vsz, uint64_t *__restrict__ pkref, uint64_t var_len,
                          unsigned long long *__restrict__ nbad) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const PackedRec80 r = recs[i];
        uint32_t s = 0;
        while (s + 1 < nsrc && src_rec[s + 1] <= i) s++;
        const uint64_t at = src_var[s] + r.pad[0];
        //  the shipped pk and value bytes must lie inside the received bytes, and a pk length
        // must fit the 24-bit reference: a corrupt or mis-sized exchange is refused, not read past
        if (r.pad[1] >= (1u << 24) || at + (uint64_t)r.pad[1] + r.pad[2] > var_len) {
            atomicAdd(nbad, 1ULL);
            pkref[i] = ~0ULL;
            voff[i] = 0;
            vsz[i] = 0;
            continue;
        }
        o.pk[i] = r.pk; o.cv[i] = r.cv; o.dbv[i] = r.dbv; o.v0[i] = r.v0;
        o.tcid[i] = r.tcid; o.cl[i] = r.cl; o.seq[i] = r.seq; o.site[i] = r.site;
        if (o.v1) o.v1[i] = r.v1;
        if (o.ts) o.ts[i] = r.ts;
        if (o.vt) o.vt[i] = (uint8_t)(r.meta & 0xFFu);
        if (o.vl) o.vl[i] = (uint8_t)(r.meta >> 8);
        voff[i] = at + r.pad[1];
        vsz[i] = r.pad[2];
        pkref[i] = r.pad[1] ? ((at << 24) | r.pad[1]) : ~0ULL;
    }
}

}  // namespace corro

using namespace corro;

static BatchDev batch_dev(const corro_changes *in, uint32_t n) {
    BatchDev bd{};
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
    bd.n = n;
    return bd;
}

extern "C" int corro_partition_ranks(corro_ctx *ctx, const corro_changes *in, uint32_t nranks, corro_changes *out,
                                     uint64_t *counts) {
    if (!ctx || !in || !out || !counts) return fail(CORRO_E_INVALID, "NULL argument");
    if (nranks == 0 || nranks > (uint32_t)PART_MAX_RANKS) return fail(CORRO_E_RANGE, "1..64 ranks");
    if (in->n >= (1ULL << 31)) return fail(CORRO_E_RANGE, "at most 2^31-1 changes per batch");
    if (!in->pk || !in->table_cid || !in->col_version || !in->db_version || !in->cl || !in->seq || !in->site ||
        !in->val0 || !out->pk || !out->table_cid || !out->col_version || !out->db_version || !out->cl ||
        !out->seq || !out->site || !out->val0)
        return fail(CORRO_E_INVALID, "a required batch array is NULL");
    if (in->val_off)
        return fail(CORRO_E_RANGE, "long values are not exchanged between ranks (apply them on their owner)");
    for (uint32_t r = 0; r < nranks; r++) counts[r] = 0;
    const uint32_t n = (uint32_t)in->n;
    if (n == 0) return CORRO_OK;
    CORRO_HIP_TRY(hipSetDevice(ctx->device));
    hipStream_t s = ctx->stream;
    const BatchDev bd = batch_dev(in, n);
    BatchOut bo{const_cast<uint64_t *>(out->pk),     const_cast<uint32_t *>(out->table_cid),
                const_cast<int64_t *>(out->col_version), const_cast<int64_t *>(out->db_version),
                const_cast<uint32_t *>(out->cl),     const_cast<uint32_t *>(out->seq),
                const_cast<uint32_t *>(out->site),   const_cast<uint64_t *>(out->val0),
                const_cast<uint64_t *>(out->val1),   const_cast<uint8_t *>(out->val_type),
                const_cast<uint8_t *>(out->val_len), const_cast<uint64_t *>(out->ts)};
    uint32_t ntiles = std::max<uint32_t>(1, std::min<uint32_t>(2048, (n + 8191) / 8192));
    uint32_t tile = (n + ntiles - 1) / ntiles;
    tile = (tile + PART_THREADS - 1) / PART_THREADS * PART_THREADS;
    ntiles = (n + tile - 1) / tile;
    if (int rc = ctx->d_part.ensure((size_t)ntiles * nranks * 4 + (PART_MAX_RANKS + 1) * 8 + 512)) return rc;
    uint32_t *d_counts = ctx->d_part.as<uint32_t>();
    uint64_t *d_tot = reinterpret_cast<uint64_t *>(ctx->d_part.as<uint8_t>() + (((size_t)ntiles * nranks * 4 + 255) / 256) * 256);
    hipLaunchKernelGGL(k_part_count, dim3(ntiles), dim3(PART_THREADS), 0, s, bd, tile, nranks, d_counts);
    hipLaunchKernelGGL(k_part_scan, dim3(1), dim3(64), 0, s, d_counts, ntiles, nranks, d_tot);
    hipLaunchKernelGGL(k_part_scatter, dim3(ntiles), dim3(PART_THREADS), 0, s, bd, tile, nranks, d_counts, bo);
    CORRO_HIP_TRY(hipGetLastError());
    CORRO_HIP_TRY(hipMemcpyAsync(counts, d_tot, nranks * 8ULL, hipMemcpyDeviceToHost, s));
    CORRO_HIP_TRY(hipStreamSynchronize(s));
    return CORRO_OK;
}

static int part_tiles(corro_ctx *ctx, uint32_t n, uint32_t nranks, uint32_t &ntiles, uint32_t &tile, uint32_t *&d_counts,
                      uint64_t *&d_tot) {
    ntiles = std::max<uint32_t>(1, std::min<uint32_t>(2048, (n + 8191) / 8192));
    tile = (n + ntiles - 1) / ntiles;
    tile = (tile + PART_THREADS - 1) / PART_THREADS * PART_THREADS;
    ntiles = (n + tile - 1) / tile;
    if (int rc = ctx->d_part.ensure((size_t)ntiles * nranks * 4 + (PART_MAX_RANKS + 1) * 8 + 512)) return rc;
    d_counts = ctx->d_part.as<uint32_t>();
    d_tot = reinterpret_cast<uint64_t *>(ctx->d_part.as<uint8_t>() + (((size_t)ntiles * nranks * 4 + 255) / 256) * 256);
    return CORRO_OK;
}

extern "C" int corro_packed_record_bytes(const corro_changes *in, uint32_t *bytes) {
    if (!in || !bytes) return fail(CORRO_E_INVALID, "NULL argument");
    *bytes = (!in->val1 && !in->val_type && !in->val_len && !in->ts) ? 48u : 80u;
    return CORRO_OK;
}

extern "C" int corro_partition_packed(corro_ctx *ctx, const corro_changes *in, uint32_t nranks, void *out,
                                      uint32_t *perm, uint64_t *counts) {
    if (!ctx || !in || !out || !counts) return fail(CORRO_E_INVALID, "NULL argument");
    if (nranks == 0 || nranks > (uint32_t)PART_MAX_RANKS) return fail(CORRO_E_RANGE, "1..64 ranks");
    if (in->n >= (1ULL << 31)) return fail(CORRO_E_RANGE, "at most 2^31-1 changes per batch");
    if (!in->pk || !in->table_cid || !in->col_version || !in->db_version || !in->cl || !in->seq || !in->site ||
        !in->val0)
        return fail(CORRO_E_INVALID, "a required batch array is NULL");
    if (in->val_off)
        return fail(CORRO_E_RANGE, "long values are not exchanged between ranks (apply them on their owner)");
    if ((uintptr_t)out % 16) return fail(CORRO_E_INVALID, "packed records must be 16-byte aligned");
    for (uint32_t r = 0; r < nranks; r++) counts[r] = 0;
    const uint32_t n = (uint32_t)in->n;
    if (n == 0) return CORRO_OK;
    CORRO_HIP_TRY(hipSetDevice(ctx->device));
    hipStream_t s = ctx->stream;
    const BatchDev bd = batch_dev(in, n);
    uint32_t ntiles, tile, *d_counts;
    uint64_t *d_tot;
    if (int rc = part_tiles(ctx, n, nranks, ntiles, tile, d_counts, d_tot)) return rc;
    const bool plain = !in->val1 && !in->val_type && !in->val_len && !in->ts;
    hipLaunchKernelGGL(k_part_count, dim3(ntiles), dim3(PART_THREADS), 0, s, bd, tile, nranks, d_counts);
    hipLaunchKernelGGL(k_part_scan, dim3(1), dim3(64), 0, s, d_counts, ntiles, nranks, d_tot);
    if (plain)
        hipLaunchKernelGGL(k_part_pack<true>, dim3(ntiles), dim3(PART_THREADS), 0, s, bd, tile, nranks, d_counts, out, perm);
    else
        hipLaunchKernelGGL(k_part_pack<false>, dim3(ntiles), dim3(PART_THREADS), 0, s, bd, tile, nranks, d_counts, out, perm);
    CORRO_HIP_TRY(hipGetLastError());
    CORRO_HIP_TRY(hipMemcpyAsync(counts, d_tot, nranks * 8ULL, hipMemcpyDeviceToHost, s));
    CORRO_HIP_TRY(hipStreamSynchronize(s));
    return CORRO_OK;
}

extern "C" int corro_unpack_records(corro_ctx *ctx, const void *recs, uint64_t n, uint32_t rec_bytes,
                                    corro_changes *out) {
    if (!ctx || (!recs && n) || !out) return fail(CORRO_E_INVALID, "NULL argument");
    if (rec_bytes != 48 && rec_bytes != 80) return fail(CORRO_E_INVALID, "record size must be 48 or 80 bytes");
    if (n >= (1ULL << 31)) return fail(CORRO_E_RANGE, "at most 2^31-1 changes per batch");
    if (n == 0) return CORRO_OK;
    if (!out->pk || !out->table_cid || !out->col_version || !out->db_version || !out->cl || !out->seq ||
        !out->site || !out->val0)
        return fail(CORRO_E_INVALID, "a required batch array is NULL");
    CORRO_HIP_TRY(hipSetDevice(ctx->device));
    hipStream_t s = ctx->stream;
    BatchOut bo{const_cast<uint64_t *>(out->pk),     const_cast<uint32_t *>(out->table_cid),
                const_cast<int64_t *>(out->col_version), const_cast<int64_t *>(out->db_version),
                const_cast<uint32_t *>(out->cl),     const_cast<uint32_t *>(out->seq),
                const_cast<uint32_t *>(out->site),   const_cast<uint64_t *>(out->val0),
                const_cast<uint64_t *>(out->val1),   const_cast<uint8_t *>(out->val_type),
                const_cast<uint8_t *>(out->val_len), const_cast<uint64_t *>(out->ts)};
    const uint32_t grid = (uint32_t)std::min<uint64_t>((n + 255) / 256, 8192);
    if (rec_bytes == 48)
        hipLaunchKernelGGL(k_unpack<true>, dim3(grid), dim3(256), 0, s, recs, (uint32_t)n, bo);
    else
        hipLaunchKernelGGL(k_unpack<false>, dim3(grid), dim3(256), 0, s, recs, (uint32_t)n, bo);
    CORRO_HIP_TRY(hipGetLastError());
    CORRO_HIP_TRY(hipStreamSynchronize(s));
    return CORRO_OK;
}

// ---------------------------------------------------------------------- stream-ordered slots
extern "C" void *corro_ctx_stream(corro_ctx *ctx) { return ctx ? (void *)ctx->stream : nullptr; }

// a batch that failed the partition's validation marks every destination's count (bit 63): each
// receiver then sees an overflowed slot, applies nothing from the slot pass, and the exchange repeats
// with exact sizes through the validating apply, which reports the error
__global__ void k_part_mark(uint64_t *__restrict__ counts, uint32_t nranks, const unsigned long long *__restrict__ err) {
    if (*err && threadIdx.x < nranks) counts[threadIdx.x] |= 1ULL << 63;
}

extern "C" int corro_partition_slots(corro_ctx *ctx, const corro_changes *in, uint32_t nranks, uint64_t cap, void *out,
                                     uint64_t *counts_dev, uint32_t *perm_dev) {
    if (!ctx || !in || !out || !counts_dev) return fail(CORRO_E_INVALID, "NULL argument");
    if (nranks == 0 || nranks > (uint32_t)PART_MAX_RANKS) return fail(CORRO_E_RANGE, "1..64 ranks");
    if (in->n >= (1ULL << 31) || cap == 0 || (uint64_t)nranks * cap >= (1ULL << 31))
        return fail(CORRO_E_RANGE, "slots: 1 <= cap, nranks * cap < 2^31 records");
    if (!in->pk || !in->table_cid || !in->col_version || !in->db_version || !in->cl || !in->seq || !in->site ||
        !in->val0)
        return fail(CORRO_E_INVALID, "a required batch array is NULL");
    if (fault_armed("partition_slots")) return fail(CORRO_E_NOMEM, "injected fault (CORRO_FAULT): partition_slots");
    if (in->val1 || in->val_type || in->val_len || in->ts || in->val_off)
        return fail(CORRO_E_RANGE, "slots carry 48-B records: INTEGER batches without val1/val_type/val_len/ts");
    if ((uintptr_t)out % 16) return fail(CORRO_E_INVALID, "packed records must be 16-byte aligned");
    CORRO_HIP_TRY(hipSetDevice(ctx->device));
    hipStream_t s = ctx->stream;
    const uint32_t n = (uint32_t)in->n;
    if (n == 0) {
        CORRO_HIP_TRY(hipMemsetAsync(counts_dev, 0, nranks * 8ULL, s));
        return CORRO_OK;
    }
    const BatchDev bd = batch_dev(in, n);
    uint32_t ntiles, tile, *d_counts;
    uint64_t *d_tot;
    if (int rc = part_tiles(ctx, n, nranks, ntiles, tile, d_counts, d_tot)) return rc;
    hipLaunchKernelGGL(k_part_count, dim3(ntiles), dim3(PART_THREADS), 0, s, bd, tile, nranks, d_counts);
    unsigned long long *err = reinterpret_cast<unsigned long long *>(d_tot + PART_MAX_RANKS);
    const PartCheck chk{ctx->d_ncols.as<uint16_t>(), (uint32_t)ctx->tables.size(), (uint32_t)ctx->sites.size(), err};
    hipLaunchKernelGGL(k_part_scan, dim3(1), dim3(64), 0, s, d_counts, ntiles, nranks, counts_dev, cap, err);
    hipLaunchKernelGGL(k_part_pack<true>, dim3(ntiles), dim3(PART_THREADS), 0, s, bd, tile, nranks, d_counts, out,
                       perm_dev, cap, chk);
    hipLaunchKernelGGL(k_part_mark, dim3(1), dim3(64), 0, s, counts_dev, nranks, (const unsigned long long *)err);
    CORRO_HIP_TRY(hipGetLastError());
    return CORRO_OK;  // (no host wait: everything is queued on ctx->stream)
}

// received impact flags -> the sender's input order: slot position p of destination d (p - d * cap <
// counts[d]) held input change perm[p]
__global__ void k_slots_back(const uint8_t *__restrict__ back, uint32_t nranks, uint64_t cap,
                             const uint64_t *__restrict__ cnt, const uint32_t *__restrict__ perm, uint8_t *__restrict__ flags,
                             uint64_t n) {
    const uint64_t m = (uint64_t)nranks * cap;
    for (uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; p < m; p += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t d = p / cap;
        if (p - d * cap >= (cnt[d] & ~(1ULL << 63))) continue;  // (bit 63: the partition's validation mark)
        const uint32_t i = perm[p];
        if (i < n) flags[i] = back[p];
    }
}

extern "C" int corro_slots_flags_back(corro_ctx *ctx, const uint8_t *back, uint32_t nranks, uint64_t cap,
                                      const uint64_t *counts_dev, const uint32_t *perm_dev, uint8_t *flags, uint64_t n) {
    if (!ctx || !back || !counts_dev || !perm_dev || (!flags && n)) return fail(CORRO_E_INVALID, "NULL argument");
    if (nranks == 0 || nranks > (uint32_t)PART_MAX_RANKS || cap == 0) return fail(CORRO_E_RANGE, "1..64 ranks, cap >= 1");
    CORRO_HIP_TRY(hipSetDevice(ctx->device));
    const uint64_t m = (uint64_t)nranks * cap;
    hipLaunchKernelGGL(k_slots_back, dim3((uint32_t)std::min<uint64_t>((m + 255) / 256, 8192)), dim3(256), 0, ctx->stream,
                       back, nranks, cap, counts_dev, perm_dev, flags, n);
    CORRO_HIP_TRY(hipGetLastError());
    return CORRO_OK;  // (queued on ctx->stream)
}

extern "C" int corro_unpack_slots(corro_ctx *ctx, const void *recs, uint32_t nsrc, uint64_t cap,
                                  const uint64_t *src_counts_dev, corro_changes *out, uint32_t *ap, uint32_t *overflow_dev) {
    if (!ctx || !recs || !src_counts_dev || !out || !ap || !overflow_dev) return fail(CORRO_E_INVALID, "NULL argument");
    if (nsrc == 0 || nsrc > (uint32_t)PART_MAX_RANKS) return fail(CORRO_E_RANGE, "1..64 source ranks");
    if (cap == 0 || (uint64_t)nsrc * cap >= (1ULL << 31)) return fail(CORRO_E_RANGE, "slots: nsrc * cap < 2^31 records");
    if (!out->pk || !out->table_cid || !out->col_version || !out->db_version || !out->cl || !out->seq ||
        !out->site || !out->val0)
        return fail(CORRO_E_INVALID, "a required batch array is NULL");
    CORRO_HIP_TRY(hipSetDevice(ctx->device));
    hipStream_t s = ctx->stream;
    BatchOut bo{const_cast<uint64_t *>(out->pk),     const_cast<uint32_t *>(out->table_cid),
                const_cast<int64_t *>(out->col_version), const_cast<int64_t *>(out->db_version),
                const_cast<uint32_t *>(out->cl),     const_cast<uint32_t *>(out->seq),
                const_cast<uint32_t *>(out->site),   const_cast<uint64_t *>(out->val0),
                nullptr, nullptr, nullptr, nullptr};
    const uint64_t n = (uint64_t)nsrc * cap;
    hipLaunchKernelGGL(k_unpack_slots, dim3((uint32_t)std::min<uint64_t>((n + 255) / 256, 8192)), dim3(256), 0, s,
                       static_cast<const PackedRec48 *>(recs), nsrc, cap, src_counts_dev, bo, ap, overflow_dev);
    CORRO_HIP_TRY(hipGetLastError());
    return CORRO_OK;
}

// ---------------------------------------------------------------------- exchange for every table

extern "C" int corro_partition_var(corro_ctx *ctx, const corro_changes *in, uint32_t nranks, void *out, uint32_t *perm,
                                   uint64_t *counts, uint8_t *var, uint64_t var_cap, uint64_t *var_counts) {
    if (!ctx || !in || !out || !counts || !var_counts) return fail(CORRO_E_INVALID, "NULL argument");
    if (nranks == 0 || nranks > (uint32_t)PART_MAX_RANKS) return fail(CORRO_E_RANGE, "1..64 ranks");
    if (in->n >= (1ULL << 31)) return fail(CORRO_E_RANGE, "at most 2^31-1 changes per batch");
    if (!in->pk || !in->table_cid || !in->col_version || !in->db_version || !in->cl || !in->seq || !in->site ||
        !in->val0)
        return fail(CORRO_E_INVALID, "a required batch array is NULL");
    if ((uintptr_t)out % 16) return fail(CORRO_E_INVALID, "packed records must be 16-byte aligned");
    for (uint32_t r = 0; r < nranks; r++) counts[r] = var_counts[r] = 0;
    const uint32_t n = (uint32_t)in->n;
    if (n == 0) return CORRO_OK;
    CORRO_HIP_TRY(hipSetDevice(ctx->device));
    hipStream_t s = ctx->stream;
    TRY_PART(pk_mirror_sync(ctx));
    uint64_t max_pk = 0;
    for (const PkTable &t : ctx->pk) max_pk = std::max<uint64_t>(max_pk, t.interned ? t.max_len : 0);
    if (in->val_data_len + (uint64_t)n * max_pk >= (1ULL << 32))
        return fail(CORRO_E_RANGE, "one exchange ships at most 4 GiB of pk / value bytes: split the batch");
    BatchDev bd = batch_dev(in, n);
    bd.voff = in->val_off;
    bd.vsz = in->val_size;
    bd.arena = in->val_data;  // (device bytes; lbase 0)
    bd.lbase = 0;
    bd.ldata = in->val_data_len;
    const PkDir *dir = ctx->d_pkdir.as<PkDir>();
    const uint32_t ntables = (uint32_t)ctx->tables.size();
    uint32_t ntiles, tile, *d_counts;
    uint64_t *d_tot;
    if (int rc = part_tiles(ctx, n, nranks, ntiles, tile, d_counts, d_tot)) return rc;
    hipLaunchKernelGGL(k_partv_count, dim3(ntiles), dim3(PART_THREADS), 0, s, bd, dir, ntables, tile, nranks, d_counts);
    hipLaunchKernelGGL(k_part_scan, dim3(1), dim3(64), 0, s, d_counts, ntiles, nranks, d_tot);
    // scratch: perm (caller's or ours), vlen, vincl, rocPRIM temp, segment / record bases
    size_t temp = 0;
    TRY_PART(prim_inclusive_scan_u32(nullptr, &temp, nullptr, nullptr, n, s));
    const size_t col = ((size_t)n * 4 + 255) & ~(size_t)255;
    if (int rc = ctx->d_part_var.ensure(3 * col + temp + 2 * 64 * 8 + 256)) return rc;
    uint8_t *sp = ctx->d_part_var.as<uint8_t>();
    uint32_t *d_perm = perm ? perm : reinterpret_cast<uint32_t *>(sp);
    uint32_t *vlen = reinterpret_cast<uint32_t *>(sp + col), *vincl = reinterpret_cast<uint32_t *>(sp + 2 * col);
    void *tmp = sp + 3 * col;
    uint64_t *d_seg = reinterpret_cast<uint64_t *>(sp + 3 * col + ((temp + 255) & ~(size_t)255));
    uint64_t *d_recb = d_seg + 64;
    hipLaunchKernelGGL(k_partv_pack, dim3(ntiles), dim3(PART_THREADS), 0, s, bd, dir, ntables, tile, nranks, d_counts,
                       static_cast<PackedRec80 *>(out), d_perm, vlen);
    CORRO_HIP_TRY(hipGetLastError());
    TRY_PART(prim_inclusive_scan_u32(tmp, &temp, vlen, vincl, n, s));
    CORRO_HIP_TRY(hipMemcpyAsync(counts, d_tot, nranks * 8ULL, hipMemcpyDeviceToHost, s));
    CORRO_HIP_TRY(hipStreamSynchronize(s));
    // per-rank record and byte bases: B(x) = bytes of records [0, x) = vincl[x - 1]
    std::vector<uint64_t> recb(nranks + 1, 0), seg(nranks + 1, 0);
    for (uint32_t r = 0; r < nranks; r++) recb[r + 1] = recb[r] + counts[r];
    for (uint32_t r = 1; r <= nranks; r++) {
        uint32_t b = 0;
        if (recb[r]) CORRO_HIP_TRY(hipMemcpy(&b, vincl + (recb[r] - 1), 4, hipMemcpyDeviceToHost));
        seg[r] = b;
    }
    for (uint32_t r = 0; r < nranks; r++) var_counts[r] = seg[r + 1] - seg[r];
    const uint64_t total = seg[nranks];
    if (total > var_cap || (total && !var)) return fail(CORRO_E_RANGE, "var bytes exceed var_cap (var_counts = the sizes)");
    CORRO_HIP_TRY(hipMemcpyAsync(d_seg, seg.data(), nranks * 8ULL, hipMemcpyHostToDevice, s));
    CORRO_HIP_TRY(hipMemcpyAsync(d_recb, recb.data(), nranks * 8ULL, hipMemcpyHostToDevice, s));
    hipLaunchKernelGGL(k_partv_fill, dim3(std::min<uint32_t>((n + 3) / 4, 8192)), dim3(PART_THREADS), 0, s, bd, dir, n,
                       d_perm, vlen, vincl, d_seg, d_recb, nranks, static_cast<PackedRec80 *>(out), var);
    CORRO_HIP_TRY(hipGetLastError());
    CORRO_HIP_TRY(hipStreamSynchronize(s));
    return CORRO_OK;
}

extern "C" int corro_unpack_var(corro_ctx *ctx, const void *recs, uint64_t n, const uint8_t *var, uint64_t var_len,
                                const uint64_t *src_counts, const uint64_t *src_var, uint32_t nsrc, corro_changes *out) {
    if (!ctx || (!recs && n) || !out || !src_counts || !src_var) return fail(CORRO_E_INVALID, "NULL argument");
    if (nsrc == 0 || nsrc > (uint32_t)PART_MAX_RANKS) return fail(CORRO_E_RANGE, "1..64 source ranks");
    if (n >= (1ULL << 31)) return fail(CORRO_E_RANGE, "at most 2^31-1 changes per batch");
    if (n == 0) return CORRO_OK;
    if (!out->pk || !out->table_cid || !out->col_version || !out->db_version || !out->cl || !out->seq ||
        !out->site || !out->val0 || !out->val1 || !out->val_type || !out->val_len || !out->ts || !out->val_off ||
        !out->val_size)
        return fail(CORRO_E_INVALID, "every batch array is needed (80-B records carry every field)");
    uint64_t tot = 0, totv = 0;
    for (uint32_t r = 0; r < nsrc; r++) {
        tot += src_counts[r];
        totv += src_var[r];
    }
    if (tot != n || totv > var_len) return fail(CORRO_E_INVALID, "source counts do not add up to the records / bytes");
    CORRO_HIP_TRY(hipSetDevice(ctx->device));
    hipStream_t s = ctx->stream;
    std::vector<uint64_t> rb(nsrc), vb(nsrc);
    uint64_t a = 0, v = 0;
    for (uint32_t r = 0; r < nsrc; r++) {
        rb[r] = a;
        vb[r] = v;
        a += src_counts[r];
        v += src_var[r];
    }
    const size_t col8 = ((size_t)n * 8 + 255) & ~(size_t)255;
    if (int rc = ctx->d_part_var.ensure(col8 + 2 * 64 * 8 + 256)) return rc;
    uint64_t *pkref = ctx->d_part_var.as<uint64_t>();
    uint64_t *d_rb = reinterpret_cast<uint64_t *>(ctx->d_part_var.as<uint8_t>() + col8), *d_vb = d_rb + 64;
    CORRO_HIP_TRY(hipMemcpyAsync(d_rb, rb.data(), nsrc * 8ULL, hipMemcpyHostToDevice, s));
    CORRO_HIP_TRY(hipMemcpyAsync(d_vb, vb.data(), nsrc * 8ULL, hipMemcpyHostToDevice, s));
    BatchOut bo{const_cast<uint64_t *>(out->pk),     const_cast<uint32_t *>(out->table_cid),
                const_cast<int64_t *>(out->col_version), const_cast<int64_t *>(out->db_version),
                const_cast<uint32_t *>(out->cl),     const_cast<uint32_t *>(out->seq),
                const_cast<uint32_t *>(out->site),   const_cast<uint64_t *>(out->val0),
                const_cast<uint64_t *>(out->val1),   const_cast<uint8_t *>(out->val_type),
                const_cast<uint8_t *>(out->val_len), const_cast<uint64_t *>(out->ts)};
    unsigned long long *d_nbad = reinterpret_cast<unsigned long long *>(d_vb + 64);
    CORRO_HIP_TRY(hipMemsetAsync(d_nbad, 0, 8, s));
    hipLaunchKernelGGL(k_unpackv, dim3((uint32_t)std::min<uint64_t>((n + 255) / 256, 8192)), dim3(256), 0, s,
                       static_cast<const PackedRec80 *>(recs), (uint32_t)n, d_rb, d_vb, nsrc, bo,
                       const_cast<uint64_t *>(out->val_off), const_cast<uint32_t *>(out->val_size), pkref, var_len,
                       d_nbad);
    CORRO_HIP_TRY(hipGetLastError());
    unsigned long long h_nbad = 0;
    CORRO_HIP_TRY(hipMemcpyAsync(&h_nbad, d_nbad, 8, hipMemcpyDeviceToHost, s));
    CORRO_HIP_TRY(hipStreamSynchronize(s));
    if (h_nbad)
        return fail(CORRO_E_INVALID, "shipped pk / value bytes outside the received var buffer (" +
                                         std::to_string(h_nbad) + " records)");
    // interned pks: this engine's row keys for the shipped canonical bytes, interned on the device
    // (pkref: var offset << 24 | length, ~0 for a change of a table that is not interned)
    for (uint32_t t = 0; t < (uint32_t)ctx->pk.size(); t++) {
        if (!ctx->pk[t].interned) continue;
        PkRefs pr;
        pr.base = static_cast<const uint8_t *>(var);
        pr.ref = pkref;
        pr.none = ~0ULL;
        pr.len_bits = 24;
        pr.tcid = out->table_cid;
        pr.limit = var_len;
        if (int rc = pk_keys_device(ctx, t, pr, n, const_cast<uint64_t *>(out->pk), nullptr, nullptr)) return rc;
    }
    CORRO_HIP_TRY(hipStreamSynchronize(s));
    return CORRO_OK;
}
