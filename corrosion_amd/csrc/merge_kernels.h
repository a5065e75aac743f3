// Device code of the batched causal-length + LWW merge (the crsql_changes INSERT loop of
// process_complete_version, /root/reference/crates/corro-agent/src/agent/util.rs:1222-1262).
//
// Pipeline for one batch of N column changes:
//   k_hist     tile-local LDS histogram of the (table, pk) bucket of every change (reads pk and
//              table_cid only); one coalesced row of counts per tile (no global atomics).
//   k_colscan  per bucket, exclusive prefix over tiles -> each tile owns a disjoint slice of the
//              bucket (deterministic slices, no atomics).
//   k_plan     one workgroup: bucket slice offsets for the staged batch and the next state.
//   k_scatter  re-read the SoA batch, stage each change as one 64-B record in its bucket slice;
//              per-bucket "general" bits, per-site crsql_db_versions maxima, input validation
//              (unknown cid / site, out-of-range encodings).
//   k_merge_fast_int (one workgroup per bucket) triages buckets and runs the INTEGER fast body;
//   k_merge_fast_wide / k_merge_gen work through the queues it fills. Per bucket: prior clock rows
//              of the bucket (as a prefix of the application order) + its staged changes ->
//                fast  (all rows cl = 1, no sentinels): per-cell argmax of
//                      (col_version, value, site_id rank, -position) by LDS 64-bit atomic-max
//                      stages; order independent (SURVEY App. A.2 reduction). 2 WGs/CU.
//                gen   sort by (row, position) in LDS, then one lane per row folds the
//                      cr-sqlite rules in application order (App. A.1), exactly.
//              Buckets larger than LDS, or holding a long row, go to the overflow path
//              (ovf_kernels.h: a parallel row fold over all of them at once, device-wide).
#pragma once
#include "internal.h"
#include "rowhash.h"
#include "rowstore.h"

namespace corro {

#ifndef CORRO_DIAG
#define CORRO_DIAG 0
#endif
constexpr int HIST_THREADS = 512;
// INTEGER fast body, two-stage argmax: every col_version of the batch in [0, CV_PACKED_LIMIT) and
// at most 2^16 sites (k_scatter flags MISC_CVBIG otherwise)
constexpr uint64_t CV_PACKED_LIMIT = 1ULL << 15;
constexpr uint32_t TILES_MAX = 256;                    // hist/scatter tiles: one per CU
constexpr int MERGE_THREADS = 512;
#ifndef CORRO_FAST_T
#define CORRO_FAST_T 512
#endif
constexpr int FAST_T = CORRO_FAST_T;                   // threads of a fast-body workgroup
constexpr int CAP_FAST = 3072;                         // records a fast body holds
constexpr int FAST_R = CAP_FAST / FAST_T;              // records per thread
static_assert(FAST_R * FAST_T == CAP_FAST, "FAST_T must divide CAP_FAST");
constexpr int FAST_WAVES_EU = 2 * (FAST_T / 64) / 4;  // two workgroups per CU (LDS)
constexpr int FAST_SLOTS = 4096;                       // cell table (distinct cells <= records)
#ifndef IMPACT_LISTS
#define IMPACT_LISTS 0  // packed impact body: counting sort by cell (0) or per-cell member lists (1: measured the same, 4.85 vs 4.83 ms)
#endif
constexpr int CAP_GEN = 2048;                          // records, general body in LDS
constexpr int GEN_SLOTS = 4096;
constexpr uint32_t LONG_ROW = 128;                     // rows this long leave the LDS body

struct MergeArgs {
    const Rec *stage;
    const uint32_t *stage_off;
    const uint32_t *new_cnt;
    const uint32_t *bflags;   // bit per bucket: batch has a non-(cl=1 column) change there
    const uint64_t *batch_ts;
    RowStore rs;              // the state (rowstore.h), updated in place
    const uint32_t *site_rank;
    uint32_t nsites;
    uint8_t *impact;
    unsigned long long *misc;  // see MISC_* below
    uint32_t *ovf_list;
    uint32_t *gen_list;        // [B] buckets for k_merge_gen, then k_merge_gen_small, k_merge_gen_mid
    uint32_t *wide_list;       // buckets for k_merge_fast_wide
    const uint8_t *fast_of;    // k_triage ran: per launched block, 1 = INTEGER fast body (null: fast_int triages)
    uint32_t *defer_list;      // buckets that could not take their new rows (re-merged after growth)
    const uint32_t *bucket_list;  // a re-merge: workgroup k takes bucket bucket_list[k] (null: k itself)
    uint32_t B;
    uint32_t force_general;    // route every non-empty bucket through the sequential general body
    uint32_t gen_ovf_min;      // general buckets of more records than this go to the device-wide fold
    uint32_t track_ts;
    uint32_t state_wide;       // the state holds non-INTEGER values
    const uint8_t *arena;      // bytes of long TEXT/BLOB values (value handles point into it)
    uint4 *touch;              // rows the apply addressed, (pk lo, pk hi, table, 0) each (null: not tracked)
    unsigned long long *touch_n;
    // column affinity: the batch's raw values (raw.conv[i] = 1: change i was staged with its
    // converted value; an incoming change still compares by its raw one, App. A.4). conv null: none.
    BatchDev raw;
    // position mode: input index of application position p (null: p itself)
    const uint32_t *pos_src;
    // batch records carry their ts in v1 (BatchDev::ts_v1); their value's v1 word is 0
    uint32_t ts_v1;
};

// input index of batch position p (position mode maps it, MergeArgs::pos_src)
// (bit 31 of a position-mode entry marks the first position of its span, agent_dev.hip k_span_pos)
__device__ inline uint32_t batch_src(const MergeArgs &a, uint32_t p) { return a.pos_src ? a.pos_src[p] & 0x7FFFFFFFu : p; }

// misc words
constexpr int MISC_ERR = 0, MISC_OVF = 1, MISC_LIVE = 2, MISC_WIDE = 3, MISC_GEN = 4, MISC_WIDEQ = 5,
              MISC_GEN_SMALL = 6, MISC_GEN_MID = 7, MISC_DEFER = 8, MISC_DEFER_WHY = 9, MISC_CVBIG = 10,
              MISC_ROWS = 11, MISC_DIAG = 16, MISC_WORDS = 24;
constexpr unsigned long long DEFER_REGION = 1, DEFER_HEAP = 2;

// misc[0] error bits
constexpr uint32_t ERR_NAME = 1u, ERR_SITE = 2u, ERR_RANGE = 4u, ERR_VALUE = 8u;

__device__ inline uint32_t cell_hash(uint64_t pk, uint32_t tcid) {
    return (uint32_t)mix64(pk * 0xD6E8FEB86659FD93ULL + tcid);
}

__device__ inline uint32_t row_hash(uint64_t pk, uint32_t table) {
    return (uint32_t)mix64(pk * 0xA0761D6478BD642FULL + table + 0x51);
}

// --- value order: type rank INTEGER > REAL > TEXT > BLOB > NULL ---------------
__device__ inline uint32_t vtype(uint32_t meta) { return meta & 0xFFu; }
__device__ inline uint32_t vlen(uint32_t meta) { return (meta >> 8) & 0xFFu; }

// order-preserving unsigned key of value word 0 within one storage class
__device__ inline uint64_t vkey0(uint32_t type, uint64_t v0) {
    switch (type) {
    case CORRO_INTEGER: return v0 ^ 0x8000000000000000ULL;
    case CORRO_REAL:
        if (v0 == 0x8000000000000000ULL) v0 = 0;  // -0.0 == 0.0
        return (v0 >> 63) ? ~v0 : (v0 | 0x8000000000000000ULL);
    case CORRO_TEXT:
    case CORRO_BLOB: return v0;
    default: return 0;
    }
}

// A TEXT/BLOB value longer than 16 bytes (length field CORRO_VAL_LONG) keeps bytes 0..7 big-endian
// in word 0 and a handle in word 1: (arena offset << 24) | byte length; its bytes live in the
// value arena. Values of up to 16 bytes stay inline (words 0/1), so a long value is never equal to
// an inline one.
constexpr uint32_t VLEN_LONG = 255;
__device__ inline bool is_long(uint32_t meta) { return vlen(meta) == VLEN_LONG; }
__device__ inline uint64_t text_len(uint32_t meta, uint64_t w1) { return is_long(meta) ? (w1 & 0xFFFFFFu) : vlen(meta); }
// byte k >= 8 of a TEXT/BLOB value (k < its length)
__device__ inline uint32_t text_byte(uint32_t meta, uint64_t w1, const uint8_t *arena, uint64_t k) {
    return is_long(meta) ? (uint32_t)arena[(w1 >> 24) + k] : (uint32_t)(w1 >> (8 * (15 - k))) & 0xFFu;
}
// TEXT/BLOB order past equal first words when either value is long: memcmp of bytes 8.. over the
// common length, then the longer is greater (SQLite's BINARY collation / blob compare)
__device__ __noinline__ int long_tail_cmp(uint32_t ma, uint64_t a1, uint32_t mb, uint64_t b1, const uint8_t *arena) {
    const uint64_t la = text_len(ma, a1), lb = text_len(mb, b1), n = la < lb ? la : lb;
    for (uint64_t k = 8; k < n; k++) {
        const uint32_t x = text_byte(ma, a1, arena, k), y = text_byte(mb, b1, arena, k);
        if (x != y) return x > y ? 1 : -1;
    }
    return la > lb ? 1 : (la < lb ? -1 : 0);
}

// value order on loose fields (type|len meta, word 0, word 1): >0: a greater, <0: b greater, 0: equal
__device__ inline int value_cmp_f(uint32_t ma, uint64_t a0, uint64_t a1, uint32_t mb, uint64_t b0, uint64_t b1,
                                  const uint8_t *arena) {
    const uint32_t ta = vtype(ma), tb = vtype(mb);
    if (ta != tb) return (5 - (int)ta) > (5 - (int)tb) ? 1 : -1;
    if (ta == CORRO_NULL) return 0;
    const uint64_t ka = vkey0(ta, a0), kb = vkey0(tb, b0);
    if (ka != kb) return ka > kb ? 1 : -1;
    if (ta == CORRO_TEXT || ta == CORRO_BLOB) {
        if (is_long(ma) || is_long(mb)) return long_tail_cmp(ma, a1, mb, b1, arena);
        if (a1 != b1) return a1 > b1 ? 1 : -1;
        const uint32_t la = vlen(ma), lb = vlen(mb);
        if (la != lb) return la > lb ? 1 : -1;
    }
    return 0;
}

__device__ inline int value_cmp(const Rec &a, const Rec &b, const uint8_t *arena) {
    return value_cmp_f(a.meta, a.v0, a.v1, b.meta, b.v0, b.v1, arena);
}

// A long value of change i (length field VLEN_LONG): validates its span and returns word 0 (bytes
// 0..7 big-endian) and word 1 (the handle of its bytes in the arena). False = malformed.
__device__ inline bool long_value(const BatchDev &in, uint32_t i, uint64_t &w0, uint64_t &w1) {
    if (!in.voff || !in.vsz || !in.arena) return false;
    const uint64_t off = in.voff[i];
    const uint32_t sz = in.vsz[i];
    if (sz <= 16 || sz >= (1u << 24) || off > in.ldata || sz > in.ldata - off) return false;
    const uint8_t *p = in.arena + in.lbase + off;
    uint64_t w = 0;
#pragma unroll
    for (int k = 0; k < 8; k++) w = (w << 8) | p[k];
    w0 = w;
    w1 = ((in.lbase + off) << 24) | sz;
    return true;
}

// Append the calling lanes' rows to the touched-row list (corro_state_export_touched): one atomic per
// wave over its active lanes, so it may be called from divergent code.
__device__ inline void touch_append(const MergeArgs &a, uint64_t pk, uint32_t table) {
    const unsigned long long act = __ballot(1);
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t leader = (uint32_t)__ffsll(act) - 1;
    const uint32_t rank = (uint32_t)__popcll(act & ((1ULL << lane) - 1ULL));
    unsigned long long base = 0;
    if (lane == leader) base = atomicAdd(a.touch_n, (unsigned long long)__popcll(act));
    base = __shfl(base, leader);
    a.touch[base + rank] = make_uint4((uint32_t)pk, (uint32_t)(pk >> 32), table, 0u);
}

__device__ inline uint32_t site_rank_of(const MergeArgs &a, uint32_t site) {
    return site < a.nsites ? a.site_rank[site] : 0u;
}

// ---------------------------------------------------------------------------------------------
// Tile histogram of row buckets. Reads only pk + table_cid (12 B per change), or only pk when the
// schema has one table (every change's bucket then uses table 0; k_scatter does the same and
// reports a bad table id as an error).
// The per-apply words the scatter and merge accumulate into (bucket general bits, misc counters,
// per-site db_version maxima) are zeroed here too: three fills fewer per apply.
struct ApplyZero {
    uint32_t *bflags;
    unsigned long long *misc, *dbv_batch;
    uint32_t nbflags, nmisc, nsites;
};
// SLOT: slot mode (corro_apply_slots) -- its own instantiation, so the SoA form keeps every load of a
// lane's HIST_U changes issued before the first use (a slot-mode branch inside that loop cost the
// config-2 histogram 0.145 -> 0.32 ms)
// MT: the schema has several tables (tables read with the pks) -- a compile-time choice, so the lane's
// table loads are issued with its pk loads (a runtime `one_table` test between them kept the compiler
// from batching the loads: config 5's histogram ran 0.36 ms against config 2's 0.15)
template <int HIST_U, bool SLOT = false, bool MT = false>
static __global__ void __launch_bounds__(HIST_THREADS)
k_hist(BatchDev in, uint32_t tile, uint32_t log2B, uint32_t one_table, uint32_t *__restrict__ hist_out, ApplyZero z) {
    extern __shared__ uint32_t hist[];
    const uint32_t B = 1u << log2B;
    {
        const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x, nt = gridDim.x * blockDim.x;
        for (uint32_t i = t; i < z.nbflags; i += nt) z.bflags[i] = 0;
        for (uint32_t i = t; i < z.nmisc; i += nt) z.misc[i] = 0;
        for (uint32_t i = t; i < z.nsites; i += nt) z.dbv_batch[i] = 0;
    }
    for (uint32_t i = threadIdx.x; i < B; i += blockDim.x) hist[i] = 0;
    bool sover = false;
    if constexpr (SLOT) {
        sover = slot_overflowed(in);
        if (in.slot_over && blockIdx.x == 0 && threadIdx.x == 0) *in.slot_over = sover ? 1u : 0u;
    }
    __syncthreads();
    const uint32_t begin = blockIdx.x * tile;
    const uint32_t end = min(in.n, begin + tile);
    // HIST_U changes per lane in flight: one CU holds a single 128-KB-LDS workgroup (8 waves), so
    // memory level parallelism has to come from each lane. Loads are unconditional (clamped index)
    // so that all of them are issued before the first wait.
    for (uint32_t base = begin; base < end; base += blockDim.x * HIST_U) {
        uint64_t pk[HIST_U];
        uint32_t tc[HIST_U], ap[HIST_U];
#pragma unroll
        for (int k = 0; k < HIST_U; k++) {
            const uint32_t i = min(base + k * blockDim.x + threadIdx.x, end - 1);
            if constexpr (SLOT) {  // (slot mode: the received record itself)
                pk[k] = in.slot_rec[i].pk;
                tc[k] = one_table ? 0u : in.slot_rec[i].tcid;
                ap[k] = slot_valid(in, i, sover) ? 0u : AP_SKIP;
            } else {
                pk[k] = in.pk[i];
                tc[k] = MT ? in.tcid[i] : 0u;
                ap[k] = in.ap && !in.ap_all ? in.ap[i] : 0u;
            }
        }
#pragma unroll
        for (int k = 0; k < HIST_U; k++) {
            const uint32_t i = base + k * blockDim.x + threadIdx.x;
            if (i < end && ap[k] != AP_SKIP) atomicAdd(&hist[bucket_of(tc[k] >> 16, pk[k], log2B)], 1u);
        }
    }
    __syncthreads();
    uint32_t *row = hist_out + (size_t)blockIdx.x * B;
    for (uint32_t b = threadIdx.x; b < B; b += blockDim.x) row[b] = hist[b];
}

// per bucket: exclusive prefix of the tile counts (in place) and the bucket total
static __global__ void k_colscan(uint32_t *__restrict__ hist, uint32_t ntiles, uint32_t B,
                          uint32_t *__restrict__ new_cnt) {
    const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= B) return;
    uint32_t run = 0;
    uint32_t t = 0;
    for (; t + 4 <= ntiles; t += 4) {
        uint32_t c[4];
#pragma unroll
        for (int k = 0; k < 4; k++) c[k] = hist[(size_t)(t + k) * B + b];
#pragma unroll
        for (int k = 0; k < 4; k++) {
            hist[(size_t)(t + k) * B + b] = run;
            run += c[k];
        }
    }
    for (; t < ntiles; t++) {
        const size_t k = (size_t)t * B + b;
        const uint32_t c = hist[k];
        hist[k] = run;
        run += c;
    }
    new_cnt[b] = run;
}

// one 1024-thread workgroup: stage_off = excl-scan(new_cnt). Every lane sums its run of `per`
// consecutive buckets with all loads issued at once (one memory latency for the whole scan), the
// lane sums are scanned by wave shuffles + one LDS round, and the lane re-reads its run (L2-resident
// now) to write the offsets.
constexpr uint32_t PLAN_PER = 32;  // B <= 1024 * PLAN_PER = 2^15 (B is a power of two)
static __global__ void __launch_bounds__(1024)
k_plan(const uint32_t *__restrict__ new_cnt, uint32_t B, uint32_t *__restrict__ stage_off) {
    __shared__ uint64_t w_a[16];
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint32_t per = B >= 1024 ? B / 1024 : 1u;  // <= PLAN_PER
    const uint32_t b0 = threadIdx.x * per;
    const uint32_t cnt = b0 < B ? per : 0u;
    uint64_t sa = 0;
    if (per >= 4) {
        uint4 x[PLAN_PER / 4];
#pragma unroll
        for (uint32_t k = 0; k < PLAN_PER / 4; k++) x[k] = reinterpret_cast<const uint4 *>(new_cnt + b0)[min(k, per / 4 - 1)];
#pragma unroll
        for (uint32_t k = 0; k < PLAN_PER / 4; k++)
            if (4 * k < per) sa += (uint64_t)x[k].x + x[k].y + x[k].z + x[k].w;
    } else {
        for (uint32_t k = 0; k < cnt; k++) sa += new_cnt[b0 + k];
    }
    uint64_t ia = sa;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint64_t xa = __shfl_up(ia, d);
        if (lane >= (uint32_t)d) ia += xa;
    }
    if (lane == 63) w_a[w] = ia;
    __syncthreads();
    uint64_t ra = ia - sa;
    for (uint32_t ww = 0; ww < w; ww++) ra += w_a[ww];
    if (per >= 4) {
#pragma unroll
        for (uint32_t k = 0; k < PLAN_PER / 4; k++) {
            if (4 * k >= per) break;
            const uint4 xk = reinterpret_cast<const uint4 *>(new_cnt + b0)[k];
            const uint32_t xs[4] = {xk.x, xk.y, xk.z, xk.w};
            uint32_t so[4];
#pragma unroll
            for (int e = 0; e < 4; e++) {
                so[e] = (uint32_t)ra;
                ra += xs[e];
            }
            reinterpret_cast<uint4 *>(stage_off + b0)[k] = make_uint4(so[0], so[1], so[2], so[3]);
        }
    } else {
        for (uint32_t k = 0; k < cnt; k++) {
            stage_off[b0 + k] = (uint32_t)ra;
            ra += new_cnt[b0 + k];
        }
    }
}

__device__ inline void store_rec(Rec *dst, const Rec &r) {
    const uint4 *s = reinterpret_cast<const uint4 *>(&r);
    uint4 *d = reinterpret_cast<uint4 *>(dst);
    d[0] = s[0];
    d[1] = s[1];
    d[2] = s[2];
    d[3] = s[3];
}

__device__ inline Rec load_rec(const Rec *src) {
    Rec r;
    const uint4 *s = reinterpret_cast<const uint4 *>(src);
    uint4 *d = reinterpret_cast<uint4 *>(&r);
    d[0] = s[0];
    d[1] = s[1];
    d[2] = s[2];
    d[3] = s[3];
    return r;
}

// Wave-cooperative store of one 64-B record per lane to base[idx] (all 64 lanes must call it).
// A 4x4 transpose across lanes {l, l+16, l+32, l+48} (v_permlane32_swap + v_permlane16_swap) lets
// store instruction k write the four 16-B quads of the records of lanes l+16k from four lanes, so
// every instruction writes 16 whole 64-B records instead of 64 scattered 16-B pieces.
__device__ inline void swap32(uint32_t &a, uint32_t &b) {
    auto r = __builtin_amdgcn_permlane32_swap(a, b, false, false);
    a = r[0];
    b = r[1];
}
__device__ inline void swap16(uint32_t &a, uint32_t &b) {
    auto r = __builtin_amdgcn_permlane16_swap(a, b, false, false);
    a = r[0];
    b = r[1];
}
template <bool NT = false>
__device__ inline void store_rec_wave(Rec *base, uint32_t idx, const Rec &r, bool valid) {
    uint4 q[4];
    const uint4 *src = reinterpret_cast<const uint4 *>(&r);
    q[0] = src[0];
    q[1] = src[1];
    q[2] = src[2];
    q[3] = src[3];
    swap32(q[0].x, q[2].x); swap32(q[0].y, q[2].y); swap32(q[0].z, q[2].z); swap32(q[0].w, q[2].w);
    swap32(q[1].x, q[3].x); swap32(q[1].y, q[3].y); swap32(q[1].z, q[3].z); swap32(q[1].w, q[3].w);
    swap16(q[0].x, q[1].x); swap16(q[0].y, q[1].y); swap16(q[0].z, q[1].z); swap16(q[0].w, q[1].w);
    swap16(q[2].x, q[3].x); swap16(q[2].y, q[3].y); swap16(q[2].z, q[3].z); swap16(q[2].w, q[3].w);
    // the destination indices ride the same transpose (no LDS permutes): after it, lane l + 16j
    // holds in ix[k] the index of lane l + 16k's record (~0u: that lane stores nothing)
    uint32_t ix[4];
    ix[0] = ix[1] = ix[2] = ix[3] = valid ? idx : ~0u;
    swap32(ix[0], ix[2]);
    swap32(ix[1], ix[3]);
    swap16(ix[0], ix[1]);
    swap16(ix[2], ix[3]);
    const uint32_t j = (threadIdx.x & 63) >> 4;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const uint32_t sidx = ix[k];
        if (sidx != ~0u) {
            uint4 *dst = reinterpret_cast<uint4 *>(base + sidx) + j;
            if (NT) {
                typedef uint32_t v4u __attribute__((ext_vector_type(4)));
                const v4u t = {q[k].x, q[k].y, q[k].z, q[k].w};
                __builtin_nontemporal_store(t, reinterpret_cast<v4u *>(dst));
            } else {
                *dst = q[k];
            }
        }
    }
}

__device__ inline unsigned long long wave_max_u64(unsigned long long x) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        const unsigned long long y = __shfl_xor(x, d);
        x = y > x ? y : x;
    }
    return x;
}

// Stage every change of the tile as one 64-B record in its bucket slice. Also: per-bucket
// "general" bits (a change with cl != 1 or a sentinel), crsql_db_versions maxima and validation.
// PLAIN: the batch has no val1/val_type/val_len arrays (INTEGER values) -- loads are unconditional
// (clamped) so all of an iteration's loads are in flight together. NT: non-temporal record stores.
template <bool PLAIN, bool NT, int SCAT_U = 4>
static __global__ void __launch_bounds__(HIST_THREADS)
k_scatter(BatchDev in, uint32_t tile, uint32_t log2B, uint32_t one_table, const uint32_t *__restrict__ hist_off,
          const uint32_t *__restrict__ stage_off, Rec *__restrict__ stage, uint32_t *__restrict__ bflags,
          unsigned long long *__restrict__ dbv_batch, uint32_t nsites, const uint16_t *__restrict__ ncols,
          uint32_t ntables, unsigned long long *misc) {
    extern __shared__ uint32_t cur[];
    const uint32_t B = 1u << log2B;
    const uint32_t nfl = (B + 31) / 32;
    uint32_t *fl = cur + B;
    const uint32_t *row = hist_off + (size_t)blockIdx.x * B;
    for (uint32_t b = threadIdx.x; b < B; b += blockDim.x) cur[b] = stage_off[b] + row[b];
    for (uint32_t w = threadIdx.x; w < nfl; w += blockDim.x) fl[w] = 0;
    __syncthreads();
    const uint32_t begin = blockIdx.x * tile;
    const uint32_t end = min(in.n, begin + tile);
    const uint32_t lane = threadIdx.x & 63;
    uint32_t err = 0, wide = 0, cvbig = 0;
    // crsql_db_versions: per-wave run of one site (a tile is a contiguous slice of the application
    // order, so a wave sees one actor's changesets for long stretches)
    uint32_t run_site = 0xFFFFFFFFu;
    unsigned long long run_max = 0;
    // SCAT_U changes per lane: all their loads are issued before any is consumed (one 132-KB-LDS
    // workgroup per CU, so memory-level parallelism must come from each lane)
    // (tiles start at multiples of 2 * blockDim.x, so pairs (2t, 2t+1) are 16-B aligned)
    // the PLAIN path needs an even tile length (pairs never straddle the tile end)
    const bool plain = PLAIN && ((end - begin) & 1u) == 0;
    const bool sover = in.slot_rec && slot_overflowed(in);
    for (uint32_t base = begin; base < end; base += blockDim.x * SCAT_U) {
        Rec rr[SCAT_U];
        if (in.slot_rec) {  // slot mode: each lane's records straight from the received slots (3 x 16 B)
#pragma unroll
            for (int u = 0; u < SCAT_U; u++) {
                const uint32_t i = base + (u / 2) * 2 * blockDim.x + 2 * threadIdx.x + (u & 1);
                Rec &r = rr[u];
                const uint32_t ic = min(i, end - 1);
                const uint4 *q = reinterpret_cast<const uint4 *>(in.slot_rec + ic);
                const uint4 x0 = q[0], x1 = q[1], x2 = q[2];
                const bool ok = i < end && slot_valid(in, i, sover);
                r.pk = ((uint64_t)x0.y << 32) | x0.x;
                r.cv = (int64_t)(((uint64_t)x0.w << 32) | x0.z);
                r.dbv = ok ? (int64_t)(((uint64_t)x1.y << 32) | x1.x) : 0;
                r.v0 = ((uint64_t)x1.w << 32) | x1.z;
                r.v1 = 0;
                r.tcid = x2.x;
                r.cl = x2.y;
                r.seq = x2.z;
                r.site = ok ? x2.w : 0xFFFFFFFFu;
                r.meta = (uint32_t)CORRO_INTEGER;
                r.pos = BATCH_POS | (ok ? i : AP_SKIP);
            }
        } else if (plain) {
#pragma unroll
            for (int p = 0; p < SCAT_U / 2; p++) {
                const uint32_t i = base + p * 2 * blockDim.x + 2 * threadIdx.x;
                const uint32_t ic = min(i, end - 2);
                Rec &a = rr[2 * p], &b = rr[2 * p + 1];
                const ulonglong2 pk = *reinterpret_cast<const ulonglong2 *>(in.pk + ic);
                const longlong2 cv = *reinterpret_cast<const longlong2 *>(in.cv + ic);
                const longlong2 dbv = *reinterpret_cast<const longlong2 *>(in.dbv + ic);
                const ulonglong2 v0 = *reinterpret_cast<const ulonglong2 *>(in.v0 + ic);
                const uint2 tc = *reinterpret_cast<const uint2 *>(in.tcid + ic);
                const uint2 cl = *reinterpret_cast<const uint2 *>(in.cl + ic);
                const uint2 sq = *reinterpret_cast<const uint2 *>(in.seq + ic);
                const uint2 st = *reinterpret_cast<const uint2 *>(in.site + ic);
                const uint2 ap2 = in.ap ? *reinterpret_cast<const uint2 *>(in.ap + ic) : make_uint2(i, i + 1);
                const bool ok = i < end;
                a.pk = pk.x; b.pk = pk.y;
                a.cv = cv.x; b.cv = cv.y;
                a.dbv = ok ? dbv.x : 0; b.dbv = ok ? dbv.y : 0;
                a.v0 = v0.x; b.v0 = v0.y;
                a.v1 = b.v1 = 0;
                a.tcid = tc.x; b.tcid = tc.y;
                a.cl = cl.x; b.cl = cl.y;
                a.seq = sq.x; b.seq = sq.y;
                a.site = ok ? st.x : 0xFFFFFFFFu; b.site = ok ? st.y : 0xFFFFFFFFu;
                a.meta = b.meta = (uint32_t)CORRO_INTEGER;
                a.pos = BATCH_POS | ap2.x;  // (AP_SKIP: not applied, see act below)
                b.pos = BATCH_POS | ap2.y;
                if (ap2.x == AP_SKIP) a.site = 0xFFFFFFFFu;
                if (ap2.y == AP_SKIP) b.site = 0xFFFFFFFFu;
                if (in.ts_v1) {  // (loads issued with the others: consumed at the store)
                    if (in.ts_pos) {
                        a.v1 = ap2.x != AP_SKIP ? in.ts[ap2.x] : 0ULL;
                        b.v1 = ap2.y != AP_SKIP ? in.ts[ap2.y] : 0ULL;
                    } else if (in.ts_v1 & 2u) {  // (16-B aligned ts array: one paired load)
                        const ulonglong2 t2 = *reinterpret_cast<const ulonglong2 *>(in.ts + ic);
                        a.v1 = t2.x;
                        b.v1 = t2.y;
                    } else {
                        a.v1 = in.ts[ic];
                        b.v1 = in.ts[ic + 1];
                    }
                }
            }
        } else {
#pragma unroll
        for (int p = 0; p < SCAT_U / 2; p++) {
            // each lane loads two consecutive changes with 16-B (8-B for 32-bit fields) accesses
            const uint32_t i = base + p * 2 * blockDim.x + 2 * threadIdx.x;
            Rec &a = rr[2 * p], &b = rr[2 * p + 1];
            a.site = b.site = 0xFFFFFFFFu;
            a.dbv = b.dbv = 0;
            if (i + 1 < end) {
                const ulonglong2 pk = *reinterpret_cast<const ulonglong2 *>(in.pk + i);
                const longlong2 cv = *reinterpret_cast<const longlong2 *>(in.cv + i);
                const longlong2 dbv = *reinterpret_cast<const longlong2 *>(in.dbv + i);
                const ulonglong2 v0 = *reinterpret_cast<const ulonglong2 *>(in.v0 + i);
                const uint2 tc = *reinterpret_cast<const uint2 *>(in.tcid + i);
                const uint2 cl = *reinterpret_cast<const uint2 *>(in.cl + i);
                const uint2 sq = *reinterpret_cast<const uint2 *>(in.seq + i);
                const uint2 st = *reinterpret_cast<const uint2 *>(in.site + i);
                a.pk = pk.x; b.pk = pk.y;
                a.cv = cv.x; b.cv = cv.y;
                a.dbv = dbv.x; b.dbv = dbv.y;
                a.v0 = v0.x; b.v0 = v0.y;
                a.tcid = tc.x; b.tcid = tc.y;
                a.cl = cl.x; b.cl = cl.y;
                a.seq = sq.x; b.seq = sq.y;
                a.site = st.x; b.site = st.y;
                if (in.v1) {
                    const ulonglong2 v1 = *reinterpret_cast<const ulonglong2 *>(in.v1 + i);
                    a.v1 = v1.x; b.v1 = v1.y;
                } else {
                    a.v1 = b.v1 = 0;
                }
                a.meta = in.vt ? ((uint32_t)in.vt[i] | ((in.vl ? (uint32_t)in.vl[i] : 0u) << 8)) : (uint32_t)CORRO_INTEGER;
                b.meta = in.vt ? ((uint32_t)in.vt[i + 1] | ((in.vl ? (uint32_t)in.vl[i + 1] : 0u) << 8))
                               : (uint32_t)CORRO_INTEGER;
                const uint32_t pa = in.ap ? in.ap[i] : i, pb = in.ap ? in.ap[i + 1] : i + 1;
                a.pos = BATCH_POS | pa;
                b.pos = BATCH_POS | pb;
                if (pa == AP_SKIP) a.site = 0xFFFFFFFFu;
                if (pb == AP_SKIP) b.site = 0xFFFFFFFFu;
            } else if (i < end) {
                a.pk = in.pk[i];
                a.cv = in.cv[i];
                a.dbv = in.dbv[i];
                a.v0 = in.v0[i];
                a.v1 = in.v1 ? in.v1[i] : 0ULL;
                a.tcid = in.tcid[i];
                a.cl = in.cl[i];
                a.seq = in.seq[i];
                a.site = in.site[i];
                const uint32_t pa = in.ap ? in.ap[i] : i;
                a.pos = BATCH_POS | pa;
                if (pa == AP_SKIP) a.site = 0xFFFFFFFFu;
                a.meta = in.vt ? ((uint32_t)in.vt[i] | ((in.vl ? (uint32_t)in.vl[i] : 0u) << 8)) : (uint32_t)CORRO_INTEGER;
            }
        }
        }
#pragma unroll
        for (int u = 0; u < SCAT_U; u++) {
            const uint32_t i = base + (u / 2) * 2 * blockDim.x + 2 * threadIdx.x + (u & 1);
            Rec &r = rr[u];
            const bool act = i < end && (!(in.ap || in.slot_rec) || (r.pos & 0x7FFFFFFFu) != (AP_SKIP & 0x7FFFFFFFu));
            uint32_t idx = 0;
            if (act) {
                // (the unpaired path of an INTEGER batch: its ts into v1 here)
                if (PLAIN && !plain && in.ts_v1) r.v1 = in.ts[in.ts_pos ? (r.pos & 0x7FFFFFFFu) : i];
                // a value its column's affinity converts is staged converted (affinity.hip); its
                // bucket takes the general body, which compares it raw as the incoming change
                const bool cvt = !PLAIN && in.conv && in.conv[i];
                if (cvt) {
                    r.v0 = in.cv0[i];
                    r.v1 = in.cv1[i];
                    r.meta = in.cmeta[i];
                }
                const uint32_t ty = vtype(r.meta), ln = vlen(r.meta);
                const uint32_t t = r.tcid >> 16, cid = r.tcid & 0xFFFFu;
                const uint32_t b = bucket_of(one_table ? 0u : t, r.pk, log2B);
                idx = atomicAdd(&cur[b], 1u);
                // long values: words from the arena; their buckets take the general body
                const bool lv = !PLAIN && !cvt && (ty == CORRO_TEXT || ty == CORRO_BLOB) && ln == VLEN_LONG;
                if (lv && !long_value(in, i, r.v0, r.v1)) err |= ERR_VALUE;
                // (the fast bodies keep a row's presence bits in one word: cids 1..63)
                if (r.cl != 1u || cid == 0 || cid >= 64 || lv || cvt) atomicOr(&fl[b >> 5], 1u << (b & 31));
                if (t >= ntables || cid > ncols[t]) err |= ERR_NAME;
                if (r.site >= nsites) err |= ERR_SITE;
                if ((cid == 0 || (r.cl & 1u) == 0) && (r.cv < 0 || r.cv > 0xFFFFFFFFLL)) err |= ERR_RANGE;
                if (r.dbv < 0) err |= ERR_RANGE;
                if ((uint64_t)r.cv >= CV_PACKED_LIMIT) cvbig = 1;
                if (ty != CORRO_INTEGER) {
                    wide = 1;
                    if (ty < 1 || ty > 5) err |= ERR_VALUE;
                    if (ty == CORRO_REAL && ((r.v0 >> 52) & 0x7FF) == 0x7FF && (r.v0 & 0xFFFFFFFFFFFFFULL)) err |= ERR_VALUE;
                    if ((ty == CORRO_TEXT || ty == CORRO_BLOB) && ln > 16 && ln != VLEN_LONG) err |= ERR_VALUE;
                }
            }
            store_rec_wave<NT>(stage, idx, r, act);
            // db_versions
            const uint32_t site0 = __shfl(r.site, 0);
            const unsigned long long dv = act ? (unsigned long long)r.dbv + 1ULL : 0ULL;
            if (__all(!act || r.site == site0)) {
                const unsigned long long m = wave_max_u64(dv);
                if (site0 == run_site) {
                    run_max = m > run_max ? m : run_max;
                } else {
                    if (lane == 0 && run_site < nsites) atomicMax(&dbv_batch[run_site], run_max);
                    run_site = site0;
                    run_max = m;
                }
            } else {
                const uint32_t psite = __shfl_up(r.site, 1);
                const unsigned long long pdv = __shfl_up(dv, 1);
                if (act && r.site < nsites && (lane == 0 || psite != r.site || pdv != dv))
                    atomicMax(&dbv_batch[r.site], dv);
            }
        }
    }
    if (lane == 0 && run_site < nsites) atomicMax(&dbv_batch[run_site], run_max);
    if (err) atomicOr(&misc[0], (unsigned long long)err);
    if (wide) atomicOr(&misc[3], 1ULL);
    if (__any(cvbig) && lane == 0) atomicOr(&misc[MISC_CVBIG], 1ULL);
    __syncthreads();
    for (uint32_t w = threadIdx.x; w < nfl; w += blockDim.x)
        if (fl[w]) atomicOr(&bflags[w], fl[w]);
}

// ------------------------------------------------------------------------ merge bodies
// A bucket's records: its staged batch changes [0, nn) and, in the general body, the prior clock
// records of the rows they touch [nn, nn + np) (heap records, named by hix[x - nn]).
struct BucketView {
    const Rec *fresh;
    uint32_t nn, np;
    const Rec *heap;
    const uint32_t *hix;
    const uint64_t *heap_ts;
    __device__ inline const Rec *at(uint32_t i) const { return i < nn ? fresh + i : heap + hix[i - nn]; }
    __device__ inline uint64_t prior_ts(const Rec &r) const { return heap_ts ? heap_ts[r.pos] : 0ULL; }
};

// Issue-only half of a wave-cooperative record load: the four coalesced 16-B loads of lane L for
// staged records [wave_base, wave_base + 64), the record index clamped to n - 1 (no branch, so a
// caller can issue the loads of several groups before the first wait). Load instruction k reads
// the 1 KB of records wave_base + 16k .. +15 with one 16-B quad per lane; rec_from_wave_quads (the
// 4x4 lane transpose of store_rec_wave, an involution) gives every lane its own record.
__device__ inline void load_rec_wave_raw(const Rec *fresh, uint32_t wave_base, uint32_t n, uint4 q[4]) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t j = lane >> 4, l = lane & 15;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const uint32_t ri = min(wave_base + l + 16 * k, n - 1);
        q[k] = reinterpret_cast<const uint4 *>(fresh + ri)[j];
    }
}

__device__ inline Rec rec_from_wave_quads(uint4 q[4]) {
    swap32(q[0].x, q[2].x); swap32(q[0].y, q[2].y); swap32(q[0].z, q[2].z); swap32(q[0].w, q[2].w);
    swap32(q[1].x, q[3].x); swap32(q[1].y, q[3].y); swap32(q[1].z, q[3].z); swap32(q[1].w, q[3].w);
    swap16(q[0].x, q[1].x); swap16(q[0].y, q[1].y); swap16(q[0].z, q[1].z); swap16(q[0].w, q[1].w);
    swap16(q[2].x, q[3].x); swap16(q[2].y, q[3].y); swap16(q[2].z, q[3].z); swap16(q[2].w, q[3].w);
    Rec r;
    uint4 *d = reinterpret_cast<uint4 *>(&r);
    d[0] = q[0];
    d[1] = q[1];
    d[2] = q[2];
    d[3] = q[3];
    return r;
}

template <class V>
__device__ inline uint64_t rec_ts(const MergeArgs &a, const V &v, const Rec &r) {
    if (r.pos & BATCH_POS) return a.ts_v1 ? r.v1 : (a.batch_ts ? a.batch_ts[r.pos & 0x7FFFFFFFu] : 0ULL);
    return v.prior_ts(r);
}
// a batch record about to be stored as a clock row: its value's v1 word back to 0 under ts_v1 (call
// after rec_ts, before pos is rewritten)
__device__ inline void rec_clear_ts(const MergeArgs &a, Rec &r) {
    if (a.ts_v1 && (r.pos & BATCH_POS)) r.v1 = 0;
}
// ts of the fast bodies' winner x (built in registers without v1), staged at stage index i
template <class V>
__device__ inline uint64_t win_ts(const MergeArgs &a, const V &v, const Rec &x, uint32_t i) {
    if (a.ts_v1 && (x.pos & BATCH_POS)) return v.fresh[i].v1;
    return rec_ts(a, v, x);
}

__device__ inline void push_overflow(const MergeArgs &a, uint32_t b) {
    const unsigned long long k = atomicAdd(&a.misc[MISC_OVF], 1ULL);
    a.ovf_list[k] = b;
}

__device__ inline void push_defer(const MergeArgs &a, uint32_t b, unsigned long long why) {
    const unsigned long long k = atomicAdd(&a.misc[MISC_DEFER], 1ULL);
    a.defer_list[k] = b;
    atomicOr(&a.misc[MISC_DEFER_WHY], why);
}

// Arrays used by the general (sequential-rule) body. They point into LDS (gen_bucket) or into a
// global scratch (overflow path); the code is the same.
struct GenArrays {
    uint64_t *pk;
    int64_t *cv;
    uint32_t *tc;
    uint32_t *cl;
    uint32_t *pos;
    uint32_t *own;   // row hash slots: owner record + 1
    uint64_t *key;   // sort keys: row << rshift | position
    uint32_t *val;   // sort payload: record index
    uint32_t *ccid;  // per-run cell scratch
    uint32_t *csrc;
    int64_t *ccv;
    uint32_t *rheap; // LDS body, per row owner: heap index of the row's slot 0
    uint32_t *rent;  // LDS body, per row owner: region entry (ROW_NONE: a new row)
    uint32_t *hix;   // LDS body: heap index of prior record x (x >= nn)
    uint32_t slots;  // pow2
    uint32_t P;      // records
    uint32_t rshift; // row = key >> rshift (32 in LDS; the overflow path's compact keys use fewer)
};

// Write a folded row into its heap slots: the sentinel clock (slot 0) and the cells (slot cid),
// every one with the row's causal length; `bits` receives the presence bits. Each written slot's
// source is the batch change that set it or the slot's own prior record, loaded before the store.
// `general` is set when the row must keep fast bodies out of its region (it holds a sentinel clock
// or a long value).
template <class V>
__device__ inline uint32_t heap_write_row(const MergeArgs &a, const V &v, const GenArrays &g, uint32_t s,
                                          uint32_t ncell, bool hs, int64_t scv, uint32_t ssrc, uint32_t hb,
                                          uint64_t bits[2], bool &general) {
    general = hs;
    const int64_t L = hs ? scv : (ncell ? 1 : 0);
    bits[0] = bits[1] = 0;
    uint32_t cnt = 0;
    if (hs) {
        Rec r = load_rec(v.at(ssrc));
        const uint64_t ts = a.track_ts ? rec_ts(a, v, r) : 0ULL;
        r.tcid &= 0xFFFF0000u;
        r.cv = scv;
        r.cl = (uint32_t)L;
        r.v0 = 0;
        r.v1 = 0;
        r.meta = CORRO_NULL;
        r.pos = hb;
        store_rec(a.rs.heap + hb, r);
        if (a.track_ts) a.rs.heap_ts[hb] = ts;
        bits[0] |= 1ULL;
        cnt++;
    }
    // four cells at a time, their loads issued together (clamped, so no branch splits them)
    constexpr uint32_t EU = 4;
    for (uint32_t c0 = 0; c0 < ncell; c0 += EU) {
        Rec r[EU];
#pragma unroll
        for (uint32_t u = 0; u < EU; u++) r[u] = load_rec(v.at(g.csrc[s + min(c0 + u, ncell - 1)]));
#pragma unroll
        for (uint32_t u = 0; u < EU; u++) {
            if (c0 + u >= ncell) break;
            const uint64_t ts = a.track_ts ? rec_ts(a, v, r[u]) : 0ULL;
            rec_clear_ts(a, r[u]);
            const uint32_t cid = r[u].tcid & 0xFFFFu;
            r[u].cv = g.ccv[s + c0 + u];
            r[u].cl = (uint32_t)L;
            r[u].pos = hb + cid;
            store_rec(a.rs.heap + hb + cid, r[u]);
            if (a.track_ts) a.rs.heap_ts[hb + cid] = ts;
            bits[cid >> 6] |= 1ULL << (cid & 63);
            if (is_long(r[u].meta)) general = true;
            cnt++;
        }
    }
    return cnt;
}

__device__ inline void gen_set_cell(const GenArrays &g, uint32_t s, uint32_t &ncell, uint32_t cid,
                                    uint32_t x, int64_t cv) {
    for (uint32_t c = 0; c < ncell; c++) {
        if (g.ccid[s + c] == cid) {
            g.csrc[s + c] = x;
            g.ccv[s + c] = cv;
            return;
        }
    }
    g.ccid[s + ncell] = cid;
    g.csrc[s + ncell] = x;
    g.ccv[s + ncell] = cv;
    ncell++;
}

// the raw (unconverted) value of batch change i into r's value fields
__device__ inline void raw_value(const BatchDev &in, uint32_t i, Rec &r) {
    const uint32_t ty = in.vt ? in.vt[i] : (uint32_t)CORRO_INTEGER, ln = in.vl ? in.vl[i] : 0u;
    r.meta = ty | (ln << 8);
    r.v0 = in.v0[i];
    r.v1 = in.v1 ? in.v1[i] : 0ULL;
    if ((ty == CORRO_TEXT || ty == CORRO_BLOB) && ln == VLEN_LONG) (void)long_value(in, i, r.v0, r.v1);
}

// Fold one row's records (sorted positions [s, e)) through the cr-sqlite rules,
// then hand the result to the emitter.
template <class V, class E>
__device__ inline void gen_fold_row(const MergeArgs &a, const V &v, E &em, const GenArrays &g, uint32_t s,
                                    uint32_t n) {
    const uint32_t row = (uint32_t)(g.key[s] >> g.rshift);
    uint32_t ncell = 0;
    bool hs = false;
    int64_t scv = 0;
    uint32_t ssrc = 0;
    for (uint32_t j = s; j < n && (uint32_t)(g.key[j] >> g.rshift) == row; j++) {
        const uint32_t x = g.val[j];
        const uint32_t cl = g.cl[x];
        const uint32_t cid = g.tc[x] & 0xFFFFu;
        const int64_t cv = g.cv[x];
        const uint32_t pos = g.pos[x];
        if (!(pos & BATCH_POS)) {
            // a prior clock row is initial state, not a change: replaying it through the rules
            // would drop the cells of a row whose (malformed) history left them under an even L
            if (cid == 0) {
                hs = true;
                scv = cv;
                ssrc = x;
            } else {
                gen_set_cell(g, s, ncell, cid, x, cv);
            }
            continue;
        }
        const int64_t L = hs ? scv : (ncell ? 1 : 0);
        const int64_t lcl = (int64_t)cl;
        uint32_t imp = 0;
        if (lcl < L) {
            // rule 1: stale causal length
        } else if ((cl & 1u) == 0) {  // rule 2: delete
            if (lcl != L) {
                ncell = 0;
                hs = true;
                scv = cv;
                ssrc = x;
                imp = 1;
            }
        } else if (cid == 0) {  // rule 3: pk-only insert / resurrect
            if (lcl > L) {
                for (uint32_t c = 0; c < ncell; c++) g.ccv[s + c] = 0;
                hs = true;
                scv = cv;
                ssrc = x;
                imp = 1;
            }
        } else if (lcl > L) {  // rule 4: column change that needs a resurrect
            if (L > 0 || cl > 1) {
                for (uint32_t c = 0; c < ncell; c++) g.ccv[s + c] = 0;
                hs = true;
                scv = lcl;
                ssrc = x;
                imp = 1;
            }
            gen_set_cell(g, s, ncell, cid, x, cv);
            imp += 1;
        } else {  // cl == L: last-writer-wins
            int found = -1;
            for (uint32_t c = 0; c < ncell; c++)
                if (g.ccid[s + c] == cid) {
                    found = (int)c;
                    break;
                }
            bool win = true;
            if (found >= 0) {
                const int64_t lcv = g.ccv[s + found];
                if (cv != lcv) {
                    win = cv > lcv;
                } else {
                    Rec xr = load_rec(v.at(x));
                    if (a.raw.conv) {
                        const uint32_t bi = batch_src(a, pos & 0x7FFFFFFFu);
                        if (a.raw.conv[bi]) raw_value(a.raw, bi, xr);
                    }
                    const Rec lr = load_rec(v.at(g.csrc[s + found]));
                    const int vc = value_cmp(xr, lr, a.arena);
                    if (vc != 0) win = vc > 0;
                    else win = site_rank_of(a, xr.site) > site_rank_of(a, lr.site);
                }
            }
            if (win) {
                gen_set_cell(g, s, ncell, cid, x, cv);
                imp = 1;
            }
        }
        if (a.impact && (pos & BATCH_POS) && imp) a.impact[pos & 0x7FFFFFFFu] = (uint8_t)imp;
    }
    em.emit(a, v, g, s, row, ncell, hs, scv, ssrc);
}

// Group the records [0, n) by row with an LDS open-addressing table (owner = first claimer):
// afterwards g.key[i] = owner << 32 | pos and g.val[i] = i.
__device__ inline void gen_rowkeys(const GenArrays &g, uint32_t n) {
    const uint32_t tid = threadIdx.x, nth = blockDim.x;
    for (uint32_t i = tid; i < g.slots; i += nth) g.own[i] = 0;
    __syncthreads();
    const uint32_t mask = g.slots - 1;
    for (uint32_t i = tid; i < n; i += nth) {
        const uint64_t pk = g.pk[i];
        const uint32_t t = g.tc[i] >> 16;
        uint32_t slot = row_hash(pk, t) & mask;
        uint32_t row;
        while (true) {
            // a plain read first: a hot row's slot is claimed once, then only read (thousands of
            // CAS on one word would serialise)
            uint32_t o = __hip_atomic_load(&g.own[slot], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            if (o == 0) o = atomicCAS(&g.own[slot], 0u, i + 1);
            if (o == 0) {
                row = i;
                break;
            }
            if (g.pk[o - 1] == pk && (g.tc[o - 1] >> 16) == t) {
                row = o - 1;
                break;
            }
            slot = (slot + 1) & mask;
        }
        g.key[i] = ((uint64_t)row << 32) | g.pos[i];
        g.val[i] = i;
    }
}

// Counting sort of the records [0, n) by row owner (counts already in g.ccid[owner], zero for
// non-owners), then every record moves to its rank by position within its row: a handful of
// barriers instead of a bitonic network. Afterwards g.key[j] / g.val[j] for sorted j, a row's
// records contiguous in application order; g.ccid / g.csrc are free again (the fold's cell
// scratch). C = ceil(n / blockDim.x) <= GEN_C.
template <uint32_t GEN_C>
__device__ inline void gen_sort_rows(const GenArrays &g, uint32_t n, uint32_t *s_wsum) {
    const uint32_t tid = threadIdx.x, nth = blockDim.x;
    // exclusive scan of the counts over owner index: GEN_C consecutive per thread
    {
        const uint32_t i0 = tid * GEN_C;
        uint32_t c[GEN_C], loc = 0;
#pragma unroll
        for (uint32_t k = 0; k < GEN_C; k++) {
            c[k] = i0 + k < n ? g.ccid[i0 + k] : 0u;
            loc += c[k];
        }
        const uint32_t lane = tid & 63, w = tid >> 6;
        uint32_t inc = loc;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t y = __shfl_up(inc, d);
            if (lane >= (uint32_t)d) inc += y;
        }
        if (lane == 63) s_wsum[w] = inc;
        __syncthreads();
        uint32_t run = inc - loc;
        for (uint32_t ww = 0; ww < w; ww++) run += s_wsum[ww];
#pragma unroll
        for (uint32_t k = 0; k < GEN_C; k++)
            if (i0 + k < n) {
                g.csrc[i0 + k] = run;
                run += c[k];
            }
    }
    __syncthreads();
    // scatter record indices by row (g.own: the row table is dead; SLOTS >= CAP)
    for (uint32_t i = tid; i < n; i += nth) g.own[atomicAdd(&g.csrc[(uint32_t)(g.key[i] >> 32)], 1u)] = i;
    __syncthreads();
    uint64_t kk[GEN_C];
#pragma unroll
    for (uint32_t k = 0; k < GEN_C; k++) {
        const uint32_t j = k * nth + tid;
        if (j < n) kk[k] = g.key[g.own[j]];
    }
    __syncthreads();
#pragma unroll
    for (uint32_t k = 0; k < GEN_C; k++) {
        const uint32_t j = k * nth + tid;
        if (j < n) {
            g.key[j] = kk[k];
            g.val[j] = g.own[j];
        }
    }
    __syncthreads();
    // each row's records by position: a record's rank in its row is the number of the row's
    // records with a smaller key (positions are distinct), counted by every lane at once (csrc[r]
    // is now the row's end, ccid[r] its length)
    uint32_t dst[GEN_C], vv[GEN_C];
#pragma unroll
    for (uint32_t k = 0; k < GEN_C; k++) {
        const uint32_t j = k * nth + tid;
        dst[k] = 0xFFFFFFFFu;
        if (j < n) {
            const uint64_t key = g.key[j];
            const uint32_t r = (uint32_t)(key >> 32), c = g.ccid[r];
            const uint32_t s = g.csrc[r] - c;
            uint32_t rank = 0;
            for (uint32_t t = s; t < s + c; t++) rank += g.key[t] < key ? 1u : 0u;
            kk[k] = key;
            vv[k] = g.val[j];
            dst[k] = s + rank;
        }
    }
    __syncthreads();
#pragma unroll
    for (uint32_t k = 0; k < GEN_C; k++)
        if (dst[k] != 0xFFFFFFFFu) {
            g.key[dst[k]] = kk[k];
            g.val[dst[k]] = vv[k];
        }
    __syncthreads();
}

// The general body comes in three sizes: CAP_GEN records (one 155 KB workgroup per CU), CAP_GEN_MID
// (78 KB, two per CU) and CAP_GEN_SMALL (39 KB, 256 threads, four per CU) for the many small general
// buckets, so that their barrier- and latency-bound phases overlap across workgroups.
constexpr uint32_t CAP_GEN_SMALL = 512, CAP_GEN_MID = 1024;
constexpr uint32_t GEN_SMALL_THREADS = 256;

template <uint32_t CAP, uint32_t THREADS = MERGE_THREADS>
struct GenCfg {
    static constexpr uint32_t C = (CAP + THREADS - 1) / THREADS;  // records per thread
    static constexpr uint32_t SLOTS = 2 * CAP;                    // row table (pow2 >= CAP)
    static constexpr size_t LDS = (size_t)CAP * (8 + 8 + 4 + 4 + 4) + (size_t)SLOTS * 4 + (size_t)CAP * (8 + 4) +
                                  (size_t)CAP * (4 + 4 + 8) + (size_t)CAP * (4 + 4 + 4);
};
static_assert(GenCfg<CAP_GEN>::LDS + 256 <= 160 * 1024, "large general body must fit the CU's LDS");

// Emission of the LDS general body: the row's heap slot (allocated before the fold for a new row),
// its region entry inserted (new row) or its presence bits replaced.
struct LdsEmit {
    uint32_t b;
    uint32_t *emitted, *general;
    __device__ inline void emit(const MergeArgs &a, const BucketView &v, const GenArrays &g, uint32_t s, uint32_t row,
                                uint32_t ncell, bool hs, int64_t scv, uint32_t ssrc) {
        const uint32_t hb = g.rheap[row], e = g.rent[row];
        if (e == ROW_NONE && !hs && ncell == 0) return;  // a new row the batch left empty (cl 0)
        uint64_t bits[2];
        bool gen;
        const uint32_t cnt = heap_write_row(a, v, g, s, ncell, hs, scv, ssrc, hb, bits, gen);
        if (e == ROW_NONE) {
            rs_insert(a.rs, b, g.pk[row], g.tc[row] >> 16, hb, bits);
        } else {
            a.rs.ent[e].bits[0] = bits[0];
            a.rs.ent[e].bits[1] = bits[1];
        }
        if (a.touch) touch_append(a, g.pk[row], g.tc[row] >> 16);
        atomicAdd(emitted, cnt);
        if (gen) *general = 1;
    }
};

__device__ inline void bucket_view(const MergeArgs &a, uint32_t b, BucketView &v) {
    v.fresh = a.stage + a.stage_off[b];
    v.nn = a.new_cnt[b];
    v.np = 0;
    v.heap = a.rs.heap;
    v.hix = nullptr;
    v.heap_ts = a.rs.heap_ts;
}

// General body in LDS for one queued bucket. Its rows' prior clock records are looked up in the
// region and gathered into LDS as the prefix of each row, the records sorted by (row, position),
// one lane per row folds the cr-sqlite rules, and each row is written back to its heap slot.
// A bucket whose batch + prior records exceed CAP moves on to the next size (NEXT_Q: the queue of
// the mid / large body, or the device-wide overflow path from the large one), as does one that
// holds a row longer than LONG_ROW (straight to the overflow path). All of these decisions, and a
// region or heap that cannot take the bucket's new rows (deferred), come before any write.
template <uint32_t CAP, uint32_t THREADS, int NEXT_Q>
__device__ inline void gen_bucket(const MergeArgs &a, uint32_t b) {
    using Cfg = GenCfg<CAP, THREADS>;
    __shared__ __attribute__((aligned(16))) uint8_t smem[Cfg::LDS];
    __shared__ uint32_t s_np, s_nrow, s_nrec, s_fail, s_emit, s_gen, s_wsum[THREADS / 64];
    __shared__ unsigned long long s_hbase;
    const uint32_t tid = threadIdx.x;
    BucketView v;
    bucket_view(a, b, v);
    const uint32_t nn = v.nn;
    auto pass_on = [&](int q) {
        if (q == 0) push_overflow(a, b);
        else if (q == 1) a.gen_list[2 * a.B + atomicAdd(&a.misc[MISC_GEN_MID], 1ULL)] = b;
        else a.gen_list[atomicAdd(&a.misc[MISC_GEN], 1ULL)] = b;
    };
    if (nn > CAP) {
        if (tid == 0) pass_on(NEXT_Q);
        return;
    }
    if (tid == 0) {
        s_np = s_nrow = s_nrec = s_fail = s_emit = s_gen = 0;
    }
    GenArrays g;
    uint8_t *p = smem;
    g.pk = reinterpret_cast<uint64_t *>(p); p += CAP * 8;
    g.cv = reinterpret_cast<int64_t *>(p); p += CAP * 8;
    g.key = reinterpret_cast<uint64_t *>(p); p += CAP * 8;
    g.ccv = reinterpret_cast<int64_t *>(p); p += CAP * 8;
    g.tc = reinterpret_cast<uint32_t *>(p); p += CAP * 4;
    g.cl = reinterpret_cast<uint32_t *>(p); p += CAP * 4;
    g.pos = reinterpret_cast<uint32_t *>(p); p += CAP * 4;
    g.val = reinterpret_cast<uint32_t *>(p); p += CAP * 4;
    g.ccid = reinterpret_cast<uint32_t *>(p); p += CAP * 4;
    g.csrc = reinterpret_cast<uint32_t *>(p); p += CAP * 4;
    g.rheap = reinterpret_cast<uint32_t *>(p); p += CAP * 4;
    g.rent = reinterpret_cast<uint32_t *>(p); p += CAP * 4;
    g.hix = reinterpret_cast<uint32_t *>(p); p += CAP * 4;
    g.own = reinterpret_cast<uint32_t *>(p);
    g.slots = Cfg::SLOTS;
    g.rshift = 32;
    v.hix = g.hix;
    // 1. the batch records' fields; counts per row start at zero
    for (uint32_t i = tid; i < nn; i += THREADS) {
        const Rec *r = v.fresh + i;
        g.pk[i] = r->pk;
        g.cv[i] = r->cv;
        g.tc[i] = r->tcid;
        g.cl[i] = r->cl;
        g.pos[i] = r->pos;
    }
    for (uint32_t i = tid; i < CAP; i += THREADS) g.ccid[i] = 0;
    // 2. rows (its barrier orders the loads above)
    gen_rowkeys(g, nn);
    __syncthreads();
    for (uint32_t i = tid; i < nn; i += THREADS) atomicAdd(&g.ccid[(uint32_t)(g.key[i] >> 32)], 1u);
    __syncthreads();
    // 3. each row owner looks its row up (read-only) and gathers its prior clock records
    for (uint32_t i = tid; i < nn; i += THREADS) {
        if ((uint32_t)(g.key[i] >> 32) != i) continue;
        const uint32_t t = g.tc[i] >> 16;
        const uint32_t e = rs_lookup(a.rs, b, g.pk[i], t);
        g.rent[i] = e;
        if (e == ROW_NONE) {
            g.rheap[i] = atomicAdd(&s_nrec, (uint32_t)a.rs.stride[t]);  // offset until the allocation
            atomicAdd(&s_nrow, 1u);
            if (g.ccid[i] > LONG_ROW) s_fail = 3;
            continue;
        }
        const RowEnt re = a.rs.ent[e];
        g.rheap[i] = re.heap;
        const uint32_t pc = row_popc(re.bits);
        if (g.ccid[i] + pc > LONG_ROW) s_fail = 3;
        const uint32_t off = atomicAdd(&s_np, pc);
        if (nn + off + pc > CAP) continue;  // the bucket moves on (step 4)
        g.ccid[i] += pc;
        uint32_t k = nn + off;
        for (int w = 0; w < 2; w++)
            for (uint64_t m = re.bits[w]; m; m &= m - 1) {
                const uint32_t c = 64 * w + (uint32_t)__ffsll((unsigned long long)m) - 1;
                const Rec *pr = a.rs.heap + re.heap + c;
                g.pk[k] = g.pk[i];
                g.cv[k] = pr->cv;
                g.tc[k] = pr->tcid;
                g.cl[k] = pr->cl;
                g.pos[k] = c;  // prior records sort first in their row (sentinel, then cells)
                g.hix[k - nn] = re.heap + c;
                g.key[k] = ((uint64_t)i << 32) | c;
                g.val[k] = k;
                k++;
            }
    }
    __syncthreads();
    // 4. decisions before any write: long row -> overflow; too many records -> the next size;
    //    region or heap without room for the new rows -> deferred
    if (tid == 0) {
        if (s_fail == 3) {
            push_overflow(a, b);
        } else if (nn + s_np > CAP) {
            pass_on(NEXT_Q);
            s_fail = 2;
        } else {
            bool ok = a.rs.used[b] + s_nrow <= a.rs.fill;
            unsigned long long h = 0;
            if (ok && s_nrec) {
                h = rs_heap_alloc(a.rs, s_nrec);
                ok = h != ~0ULL;
            }
            if (!ok) {
                push_defer(a, b, a.rs.used[b] + s_nrow <= a.rs.fill ? DEFER_HEAP : DEFER_REGION);
                s_fail = 1;
            } else {
                a.rs.used[b] += s_nrow;
                s_hbase = h;
            }
        }
    }
    __syncthreads();
    if (s_fail) return;
    const uint32_t n = nn + s_np;
    for (uint32_t i = tid; i < nn; i += THREADS)
        if ((uint32_t)(g.key[i] >> 32) == i && g.rent[i] == ROW_NONE) g.rheap[i] += (uint32_t)s_hbase;
    // 5. records by row, in application order (prior first)
    gen_sort_rows<Cfg::C>(g, n, s_wsum);
    // 6. fold + write back
    LdsEmit em{b, &s_emit, &s_gen};
    for (uint32_t i = tid; i < n; i += THREADS)
        if (i == 0 || (g.key[i] >> 32) != (g.key[i - 1] >> 32)) gen_fold_row(a, v, em, g, i, n);
    __syncthreads();
    if (tid == 0) {
        atomicAdd(&a.misc[MISC_LIVE], (unsigned long long)((long long)s_emit - (long long)s_np));
        if (s_gen) a.rs.gen[b] = 1;
    }
}

// ---------------------------------------------------------------------------------------------
// Fast bodies: every row of the bucket has causal length 1 and no sentinel, in the batch and in
// the region, so the merge is a per-cell argmax of (col_version, value order, site-id rank,
// -position) over the batch, then one comparison with the cell's prior clock in the heap (the
// prior is earlier in application order: it keeps ties). Rows of the winners are resolved in the
// region (lookups, then inserts of new rows once the region and heap are known to have room).

// Rows, then cells, in two short probes. Phase 1 (row_claim, every record): open addressing on the
// row key (pk, table) in `s_rt` (FAST_SLOTS words that are free until phase 2 has run), entries =
// claiming record + 1, an empty slot read plainly before it is claimed by CAS (lanes of one row mostly
// meet its occupied home slot: broadcast reads, no serialised atomics); row = the row's first
// claimant. Phase 2 (cell_claim, after a barrier): open addressing on the cell key (row claimant + 1,
// cid) packed into one word with the claimant, so a probe compares words without reading s_pk/s_tc
// (cid < 128: MAX_COLS; records < 4096). s_rt and s_own must be zero before phase 1.
__device__ inline uint32_t row_claim(uint32_t *s_rt, const uint64_t *s_pk, const uint32_t *s_tc, uint32_t i, uint64_t pk,
                                     uint32_t t) {
    uint32_t slot = row_hash(pk, t) & (FAST_SLOTS - 1);
    while (true) {
        uint32_t o = __hip_atomic_load(&s_rt[slot], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (o == 0) {
            o = atomicCAS(&s_rt[slot], 0u, i + 1);
            if (o == 0) return i;
        }
        const uint32_t x = o - 1;
        if (s_pk[x] == pk && (s_tc[x] >> 16) == t) return x;
        slot = (slot + 1) & (FAST_SLOTS - 1);
    }
}

__device__ inline uint32_t cell_claim(uint32_t *s_own, uint32_t i, uint32_t row, uint32_t cid) {
    static_assert(CAP_FAST <= 4096 && MAX_COLS < 128, "cell words: claimant in 12 bits, cid in 7");
    const uint32_t key = ((row + 1) << 7) | (cid & 127u);
    const uint32_t mine = (key << 12) | i;
    uint32_t slot = (key * 0x9E3779B1u) >> (32 - 12);
    while (true) {
        uint32_t o = __hip_atomic_load(&s_own[slot], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (o == 0) {
            o = atomicCAS(&s_own[slot], 0u, mine);
            if (o == 0) return i;
        }
        if ((o >> 12) == key) return o & 0xFFFu;
        slot = (slot + 1) & (FAST_SLOTS - 1);
    }
}

// Row resolution shared by the fast bodies, run by the whole workgroup once the cell table is no
// longer probed (s_heap aliases its first CAP_FAST words, the claim bitmap the rest). row[k]: the
// row's record (row_claim); the lane holding it (valid, row[k] == i) looks the row up and keeps
// its region entry in ent[k]; the row's heap word goes to s_heap[row] (row_heap() gives the heap
// index) and its prior presence word to s_bits[row]. The workgroup owns region b during the fast
// bodies, so the region is probed with plain loads -- not at all while it is empty (used0 = its fill
// at apply start) -- and a new row takes the first empty slot its probe met unless another new row
// of the workgroup took it first, decided by an LDS bitmap of the region's slots: no global atomic,
// the entry written with plain stores (regions larger than the bitmap claim by CAS). `counted`: the
// region was empty and fast_rows_count / fast_rows_alloc already ran. Returns false when the bucket
// was deferred (nothing written). s_ctl[0..2] must be zero on entry unless counted.
// Wave-aggregated LDS counters: many lanes adding to one LDS word serialise (same-address atomics),
// so a wave scans its lanes' amounts and one lane adds the total. Called by every lane of the wave.
__device__ inline uint32_t wave_incl_scan(uint32_t x) {
    const uint32_t lane = threadIdx.x & 63;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(x, d);
        if (lane >= (uint32_t)d) x += y;
    }
    return x;
}
// ctr += sum of x over the wave; returns this lane's exclusive offset (old ctr + earlier lanes' x).
__device__ inline uint32_t wave_lds_add(uint32_t *ctr, uint32_t x) {
    const uint32_t inc = wave_incl_scan(x);
    const uint32_t total = __shfl(inc, 63);
    uint32_t base = 0;
    if ((threadIdx.x & 63) == 0 && total) base = atomicAdd(ctr, total);
    return __shfl(base, 0) + inc - x;
}
__device__ inline uint32_t wave_sum_u32(uint32_t x) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) x += __shfl_xor(x, d);
    return x;
}

constexpr uint32_t RS_BM_WORDS = FAST_SLOTS - CAP_FAST;  // claim bitmap: regions of up to 32768 slots

__device__ inline uint32_t row_heap(uint32_t w, unsigned long long hbase) {
    return (w & 0x80000000u) ? (uint32_t)hbase + (w & 0x7FFFFFFFu) : w;
}

// Empty region: every row of the bucket is new, so rows and heap records are counted (and each row's
// heap offset noted) right after the cell hashing; thread 0 allocates after the next barrier, its
// latency hidden behind the argmax.
// (one wave scan of each lane's total over its R records and one LDS atomic per wave: the lane's
// records take consecutive offsets inside its share -- any disjoint assignment of heap offsets does)
template <int R>
__device__ inline void fast_rows_count(uint32_t n, const uint32_t (&row)[R], const uint32_t (&strd)[R], uint32_t *s_heap,
                                       uint32_t *s_ctl) {
    const uint32_t tid = threadIdx.x;
    uint32_t rows = 0, tot = 0;
#pragma unroll
    for (int k = 0; k < R; k++) {
        const uint32_t i = k * FAST_T + tid;
        const bool own = i < n && row[k] == i;
        tot += own ? strd[k] : 0u;
        rows += own;
    }
    uint32_t off = wave_lds_add(&s_ctl[1], tot);
#pragma unroll
    for (int k = 0; k < R; k++) {
        const uint32_t i = k * FAST_T + tid;
        if (i < n && row[k] == i) {
            s_heap[i] = 0x80000000u | off;
            off += strd[k];
        }
    }
    rows = wave_sum_u32(rows);
    if ((tid & 63) == 0 && rows) atomicAdd(&s_ctl[0], rows);
}

// thread 0: the region fill check and the heap allocation of the bucket's new rows (s_ctl[0] rows,
// s_ctl[1] records); s_ctl[2] = 1 when the bucket defers.
__device__ inline void fast_rows_alloc(const MergeArgs &a, uint32_t b, uint32_t used0, uint32_t *s_ctl,
                                       unsigned long long *s_hbase) {
    bool ok = used0 + s_ctl[0] <= a.rs.fill;
    unsigned long long h = 0;
    if (ok && s_ctl[1]) {
#if CORRO_DIAG & 8
        h = (unsigned long long)b * 640u;
#else
        h = rs_heap_alloc(a.rs, s_ctl[1]);
#endif
        ok = h != ~0ULL;
    }
    if (!ok) {
        push_defer(a, b, used0 + s_ctl[0] <= a.rs.fill ? DEFER_HEAP : DEFER_REGION);
        s_ctl[2] = 1;
    } else {
        a.rs.used[b] = used0 + s_ctl[0];
        *s_hbase = h;
    }
}

template <int R>
__device__ inline bool fast_rows(const MergeArgs &a, uint32_t b, uint32_t used0, uint32_t n, const uint32_t (&row)[R],
                                 uint32_t (&ent)[R], const uint64_t *s_pk, const uint32_t *s_tc, uint32_t *s_heap,
                                 uint64_t *s_bits, uint32_t *s_ctl, unsigned long long *s_hbase, bool counted) {
    const uint32_t tid = threadIdx.x;
    const uint32_t S = 1u << a.rs.log2S;
    uint32_t *s_bm = s_heap + CAP_FAST;
    const bool lds_claim = S <= 32 * RS_BM_WORDS;
    if (lds_claim)
        for (uint32_t w = tid; w < (S + 31) / 32; w += FAST_T) s_bm[w] = 0;
    uint32_t e0[R], hw[R];
#pragma unroll
    for (int k = 0; k < R; k++) {
        const uint32_t i = k * FAST_T + tid;
        ent[k] = ROW_NONE;
        e0[k] = 0;
        hw[k] = 0;
        if (i >= n || row[k] != i) continue;
        const uint64_t pk = s_pk[i];
        const uint32_t t = s_tc[i] >> 16;
        if (counted) {  // an empty region: new, heap word noted by fast_rows_count
            hw[k] = s_heap[i];
            s_bits[i] = 0;
            e0[k] = region_slot(pk, t, a.rs.log2S);
            ent[k] = ROW_NONE - 1;
            continue;
        }
        const uint32_t e = used0 ? rs_probe(a.rs, b, pk, t, e0[k]) : ROW_NONE;
        if (!used0) e0[k] = region_slot(pk, t, a.rs.log2S);
        if (e != ROW_NONE) {
            hw[k] = a.rs.ent[e].heap;
            s_bits[i] = a.rs.ent[e].bits[0];
            ent[k] = e;
        } else {
            hw[k] = (uint32_t)a.rs.stride[t];  // (its heap offset below)
            s_bits[i] = 0;
            ent[k] = ROW_NONE - 1;  // marks "owner of a new row"
        }
    }
    if (!counted) {  // heap offsets of the new rows: one wave scan of the lanes' totals, one LDS atomic per wave
        uint32_t rows = 0, tot = 0;
#pragma unroll
        for (int k = 0; k < R; k++) {
            const bool nw = ent[k] == ROW_NONE - 1;
            tot += nw ? hw[k] : 0u;
            rows += nw;
        }
        uint32_t off = wave_lds_add(&s_ctl[1], tot);
#pragma unroll
        for (int k = 0; k < R; k++)
            if (ent[k] == ROW_NONE - 1) {
                const uint32_t st = hw[k];
                hw[k] = 0x80000000u | off;
                off += st;
            }
        rows = wave_sum_u32(rows);
        if ((tid & 63) == 0 && rows) atomicAdd(&s_ctl[0], rows);
    }
    __syncthreads();
    if (!counted) {
#pragma unroll
        for (int k = 0; k < R; k++)
            if (ent[k] != ROW_NONE) s_heap[k * FAST_T + tid] = hw[k];
        if (tid == 0) fast_rows_alloc(a, b, used0, s_ctl, s_hbase);
        __syncthreads();
    }
    if (s_ctl[2]) return false;
    // new rows: their region entries (presence bits published by the caller at the end)
#pragma unroll
    for (int k = 0; k < R; k++) {
        const uint32_t i = k * FAST_T + tid;
        if (ent[k] != ROW_NONE - 1) continue;
#if CORRO_DIAG & 2
        ent[k] = ROW_NONE;
        continue;
#endif
        const uint32_t t = s_tc[i] >> 16, hb = row_heap(hw[k], *s_hbase);
        if (!lds_claim) {
            ent[k] = rs_claim(a.rs, b, e0[k], s_pk[i], t, hb);
            continue;
        }
        uint32_t sl = e0[k];
        while (true) {
            const uint32_t bit = 1u << (sl & 31);
            // slot e0 was empty at the probe; a later one only if its tag says so (no other
            // workgroup writes the region, and this one's claims all go through the bitmap)
            if (!(atomicOr(&s_bm[sl >> 5], bit) & bit) &&
                (sl == e0[k] || !used0 || a.rs.ent[((size_t)b << a.rs.log2S) + sl].tag == 0))
                break;
            sl = (sl + 1) & (S - 1);
        }
        const uint32_t e = (b << a.rs.log2S) | sl;
        RowEnt &re = a.rs.ent[e];
        re.pk = s_pk[i];
        re.tag = t + 1;
        re.heap = hb;
        re.bits[1] = 0;
        ent[k] = e;
    }
    return true;
}

// prior clock of a cell vs the batch winner's key: > 0 when the winner is greater
__device__ inline int prior_cmp_int(const MergeArgs &a, const Rec &pr, uint64_t cvb, uint64_t v0b, uint32_t rank) {
    const uint64_t pcv = (uint64_t)pr.cv ^ 0x8000000000000000ULL, pv = pr.v0 ^ 0x8000000000000000ULL;
    if (cvb != pcv) return cvb > pcv ? 1 : -1;
    if (v0b != pv) return v0b > pv ? 1 : -1;
    const uint32_t pr_rank = site_rank_of(a, pr.site);
    return rank != pr_rank ? (rank > pr_rank ? 1 : -1) : 0;
}

// Fast body without impact output. Registers keep only the stage keys of FAST_R records per thread;
// the full 64-B record of a winner is re-read (L2) for the wide form. LDS: cell keys + one stage
// array + the open-addressing cell table (76 KB, two workgroups per CU).
template <bool WIDE>
__device__ inline void fast_body(const MergeArgs &a, uint32_t b, const BucketView &v, bool packed = false) {
    __shared__ uint64_t s_pk[CAP_FAST];
    __shared__ uint64_t s_k[CAP_FAST];
    __shared__ uint32_t s_tc[CAP_FAST];
    __shared__ uint32_t s_own[FAST_SLOTS];
    __shared__ uint32_t s_ctl[4];
    __shared__ unsigned long long s_hbase, s_live;
    const uint32_t tid = threadIdx.x;
    const uint32_t n = v.nn;
    uint64_t cv[FAST_R], v0[FAST_R], v1[FAST_R], rp[FAST_R], dbv[FAST_R];
    uint32_t meta[FAST_R], cell[FAST_R], seq[FAST_R], site[FAST_R], row[FAST_R];
    bool alive[FAST_R];
    // every record load of this lane is issued before the first wait (one memory latency per
    // bucket instead of one per record group), then the site-rank lookups as one more batch
    uint4 q[FAST_R][4];
#if CORRO_DIAG & 64
    unsigned long long diag_t = wall_clock64();
#define DIAG_MARK(k) do { if (tid == 0) { const unsigned long long t_ = wall_clock64(); atomicAdd(&a.misc[MISC_DIAG + (k)], t_ - diag_t); diag_t = t_; } } while (0)
#else
#define DIAG_MARK(k) do { } while (0)
#endif
#pragma unroll
    for (int k = 0; k < FAST_R; k++) load_rec_wave_raw(v.fresh, k * FAST_T + (tid & ~63u), n, q[k]);
    const uint32_t used0 = a.rs.used[b];  // (issued with the record loads)
    if (tid == 0) {
        s_live = 0;
        s_ctl[0] = s_ctl[1] = s_ctl[2] = s_ctl[3] = 0;
    }
    for (uint32_t i = tid; i < FAST_SLOTS; i += FAST_T) {
        s_own[i] = 0;
        reinterpret_cast<uint32_t *>(s_k)[i] = 0;  // the row table of row_claim
    }
    uint32_t srank[FAST_R];
#pragma unroll
    for (int k = 0; k < FAST_R; k++) {
        const uint32_t i = k * FAST_T + tid;  // < CAP_FAST: stores of dead lanes are harmless
        alive[k] = i < n;
        cell[k] = 0;
        const Rec r = rec_from_wave_quads(q[k]);
        s_pk[i] = r.pk;
        s_tc[i] = r.tcid;
        cv[k] = (uint64_t)r.cv ^ 0x8000000000000000ULL;
        v0[k] = r.v0;
        v1[k] = WIDE ? r.v1 : 0;
        meta[k] = WIDE ? r.meta : (uint32_t)CORRO_INTEGER;
        rp[k] = (uint64_t)(~r.pos);
        site[k] = r.site;
        if (!WIDE) {  // INTEGER-only: keep the whole clock row in registers (no re-read)
            dbv[k] = (uint64_t)r.dbv;
            seq[k] = r.seq;
        }
    }
    // site ranks (first needed by the last argmax stage) and, for the rows an empty region gets, row
    // strides (needed after the claims): one more batch of loads, in flight during the claims
    uint32_t strd[FAST_R];
#pragma unroll
    for (int k = 0; k < FAST_R; k++) {
        srank[k] = a.site_rank[site[k] < a.nsites ? site[k] : 0u];
        strd[k] = used0 ? 0u : (uint32_t)a.rs.stride[alive[k] ? s_tc[k * FAST_T + tid] >> 16 : 0u];
    }
    __syncthreads();
    DIAG_MARK(0);
#pragma unroll
    for (int k = 0; k < FAST_R; k++) {
        const uint32_t i = k * FAST_T + tid;
        row[k] = 0;
        if (!alive[k]) continue;
        row[k] = row_claim(reinterpret_cast<uint32_t *>(s_k), s_pk, s_tc, i, s_pk[i], s_tc[i] >> 16);
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < FAST_R; k++) {
        const uint32_t i = k * FAST_T + tid;
        if (!alive[k]) continue;
        cell[k] = cell_claim(s_own, i, row[k], s_tc[i]);
        if (cell[k] == i) s_k[i] = 0;
    }
#pragma unroll
    for (int k = 0; k < FAST_R; k++) rp[k] |= (uint64_t)(site[k] < a.nsites ? srank[k] : 0u) << 32;
    __syncthreads();
    DIAG_MARK(1);
    // an empty region: all rows new -- counted now, allocated behind the argmax
    if (!used0) fast_rows_count<FAST_R>(n, row, strd, s_own, s_ctl);
    DIAG_MARK(6);
    // argmax stages: INTEGER-only: col_version, value, site|pos. Mixed: + rank, word 1, length.
    // Packed INTEGER form (`packed`: col_versions < 2^15, sites <= 2^16): two stages, (cv 15 | value
    // bits 63..16) then (1 | value bits 15..0 | site rank 16 | ~position 31): the second stage's keys
    // all exceed the first's, so the cell words need no zeroing (and no barrier) in between.
    if (!WIDE && packed) {
        uint64_t w[FAST_R];
        unsigned long long hraw = 0;
#pragma unroll
        for (int k = 0; k < FAST_R; k++) {
            w[k] = ((cv[k] ^ 0x8000000000000000ULL) << 48) | (v0[k] ^ 0x8000000000000000ULL) >> 16;
            if (alive[k]) atomicMax(reinterpret_cast<unsigned long long *>(&s_k[cell[k]]), (unsigned long long)w[k]);
        }
        __syncthreads();
        DIAG_MARK(7);
        // the bucket's heap allocation: issued now, its result consumed after the second stage
#if CORRO_DIAG & 8  // (diagnostics: no global heap atomic -- a fixed offset per bucket, results not valid)
        if (!used0 && tid == 0 && s_ctl[1] && used0 + s_ctl[0] <= a.rs.fill) hraw = (unsigned long long)b * 640u;
#else
        if (!used0 && tid == 0 && s_ctl[1] && used0 + s_ctl[0] <= a.rs.fill) hraw = atomicAdd(a.rs.heap_top, (unsigned long long)s_ctl[1]);
#endif
#pragma unroll
        for (int k = 0; k < FAST_R; k++)
            if (alive[k]) alive[k] = s_k[cell[k]] == w[k];
        __syncthreads();
#pragma unroll
        for (int k = 0; k < FAST_R; k++) {
            w[k] = (1ULL << 63) | (((v0[k] ^ 0x8000000000000000ULL) & 0xFFFFULL) << 47) | ((rp[k] >> 32) << 31) |
                   ((uint64_t)(uint32_t)rp[k] & 0x7FFFFFFFULL);
            if (alive[k]) atomicMax(reinterpret_cast<unsigned long long *>(&s_k[cell[k]]), (unsigned long long)w[k]);
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < FAST_R; k++)
            if (alive[k]) alive[k] = s_k[cell[k]] == w[k];
        __syncthreads();
        if (!used0 && tid == 0) {  // (published to the workgroup by fast_rows' first barrier)
            const unsigned long long need = s_ctl[1];
            const bool room = used0 + s_ctl[0] <= a.rs.fill;
            if (!room || (need && hraw + need > a.rs.heap_cap)) {
                if (room && need) atomicSub(a.rs.heap_top, need);  // (give the failed request back)
                push_defer(a, b, room ? DEFER_HEAP : DEFER_REGION);
                s_ctl[2] = 1;
            } else {
                a.rs.used[b] = used0 + s_ctl[0];
                s_hbase = need ? hraw : 0;
            }
        }
    }
    constexpr int nstages = WIDE ? 6 : 3;
#pragma unroll
    for (int st = 0; st < nstages; st++) {
        if (!WIDE && packed) break;
        const int which = WIDE ? st : (st == 0 ? 0 : (st == 1 ? 2 : 5));
        uint64_t w[FAST_R];
#pragma unroll
        for (int k = 0; k < FAST_R; k++) {
            w[k] = 0;
            if (!alive[k]) continue;
            const uint32_t ty = WIDE ? vtype(meta[k]) : (uint32_t)CORRO_INTEGER;
            const bool tb = ty == CORRO_TEXT || ty == CORRO_BLOB;
            switch (which) {
            case 0: w[k] = cv[k]; break;
            case 1: w[k] = 5u - ty; break;
            case 2: w[k] = vkey0(ty, v0[k]); break;
            case 3: w[k] = tb ? v1[k] : 0; break;
            case 4: w[k] = tb ? vlen(meta[k]) : 0; break;
            default: w[k] = rp[k]; break;
            }
            atomicMax(reinterpret_cast<unsigned long long *>(&s_k[cell[k]]), (unsigned long long)w[k]);
        }
        __syncthreads();
        if (st == 0 && !used0 && tid == 0) fast_rows_alloc(a, b, used0, s_ctl, &s_hbase);
#pragma unroll
        for (int k = 0; k < FAST_R; k++)
            if (alive[k]) alive[k] = s_k[cell[k]] == w[k];
        __syncthreads();
        if (st + 1 < nstages) {
#pragma unroll
            for (int k = 0; k < FAST_R; k++) {
                const uint32_t i = k * FAST_T + tid;
                if (i < n && cell[k] == i) s_k[i] = 0;
            }
            __syncthreads();
        }
    }
    // rows (s_own: heap words by row record; s_k: presence words)
    DIAG_MARK(2);
    uint32_t ent[FAST_R];
    if (!fast_rows<FAST_R>(a, b, used0, n, row, ent, s_pk, s_tc, s_own, s_k, s_ctl, &s_hbase, used0 == 0)) return;
    DIAG_MARK(3);
    // winners vs the prior clock of their cell; new cells set their presence bit
    uint32_t hb[FAST_R];
    uint32_t nlive = 0;
#pragma unroll
    for (int k = 0; k < FAST_R; k++) {
        hb[k] = 0;
        if (!alive[k]) continue;
        const uint32_t i = k * FAST_T + tid;
        const uint32_t c = s_tc[i] & 0xFFFFu;
        hb[k] = row_heap(s_own[row[k]], s_hbase) + c;
        if ((s_k[row[k]] >> c) & 1ULL) {
            const Rec pr = load_rec(a.rs.heap + hb[k]);
            int cmp;
            if (WIDE) {
                Rec x = load_rec(v.fresh + i);
                cmp = (int64_t)(cv[k] ^ 0x8000000000000000ULL) != pr.cv
                          ? ((int64_t)(cv[k] ^ 0x8000000000000000ULL) > pr.cv ? 1 : -1)
                          : value_cmp(x, pr, a.arena);
                if (cmp == 0) {
                    const uint32_t rk = (uint32_t)(rp[k] >> 32), prk = site_rank_of(a, pr.site);
                    cmp = rk != prk ? (rk > prk ? 1 : -1) : 0;
                }
            } else {
                cmp = prior_cmp_int(a, pr, cv[k], v0[k] ^ 0x8000000000000000ULL, (uint32_t)(rp[k] >> 32));
            }
            if (cmp <= 0) alive[k] = false;  // the prior clock is earlier: it keeps ties
        } else {
            atomicOr(reinterpret_cast<unsigned long long *>(&s_k[row[k]]), 1ULL << c);
            nlive++;
        }
    }
    // winners: the clock row into its heap slot (wave-cooperative 64-B stores)
#pragma unroll
    for (int k = 0; k < FAST_R; k++) {
        const uint32_t i = k * FAST_T + tid;
        Rec x;
        if (alive[k]) {
            if (WIDE) {
                x = load_rec(v.fresh + i);
            } else {
                x.pk = s_pk[i];
                x.cv = (int64_t)(cv[k] ^ 0x8000000000000000ULL);
                x.dbv = (int64_t)dbv[k];
                x.v0 = v0[k];
                x.v1 = 0;
                x.tcid = s_tc[i];
                x.seq = seq[k];
                x.site = site[k];
                x.pos = ~(uint32_t)rp[k];
                x.meta = CORRO_INTEGER;
            }
            if (a.track_ts) a.rs.heap_ts[hb[k]] = win_ts(a, v, x, i);
            rec_clear_ts(a, x);
            x.cl = 1;
            x.pos = hb[k];
        }
#if CORRO_DIAG & 1
        {   // DIAG: winners written compactly behind the bucket's heap base (timing only)
            uint32_t o = 0;
            if (alive[k]) o = atomicAdd(&s_ctl[3], 1u);
            store_rec_wave(a.rs.heap, (uint32_t)s_hbase + o, x, alive[k]);
        }
#elif CORRO_DIAG & 4
        (void)x;
#else
        store_rec_wave(a.rs.heap, hb[k], x, alive[k]);
#endif
    }
    nlive = wave_sum_u32(nlive);
    if ((tid & 63) == 0 && nlive) atomicAdd(&s_live, (unsigned long long)nlive);
    __syncthreads();
    DIAG_MARK(4);
    // owners publish the rows' presence bits
#pragma unroll
    for (int k = 0; k < FAST_R; k++) {
        const uint32_t i = k * FAST_T + tid;
        if (ent[k] != ROW_NONE && row[k] == i) {
            a.rs.ent[ent[k]].bits[0] = s_k[i];
            if (a.touch) touch_append(a, s_pk[i], s_tc[i] >> 16);
        }
    }
    if (tid == 0 && s_live) atomicAdd(&a.misc[MISC_LIVE], s_live);
    DIAG_MARK(5);
}

// Same per-cell merge with per-change crsql_rows_impacted() growth (impact output requested: the
// agent path, util.rs:1246-1262). With every cl = 1 and no sentinel (App. A.1 rule 4 with L <= 1)
// change i grows the counter by exactly 1 iff its key (col_version, value, site id) is strictly
// greater than the cell's prior clock (if any) and than every earlier change of the cell in the
// batch: a strict prefix maximum. The cell's new clock is the batch maximum (earliest among equals)
// when it beats the prior. Decided per change by one walk over the cell's member list (counting
// sort of the bucket's records by cell in LDS). Mixed value classes; one workgroup per CU (LDS).
__device__ inline void fast_body_impact_wide(const MergeArgs &a, uint32_t b, const BucketView &v) {
    __shared__ uint64_t s_pk[CAP_FAST];      // cell hashing: pk; then the biased col_version keys
    __shared__ uint32_t s_tc[CAP_FAST];      // cell hashing: table_cid; then site ranks
    __shared__ uint32_t s_own[FAST_SLOTS];   // cell / row hashing; heap indices; member counts/offsets
    __shared__ uint64_t s_v0[CAP_FAST];      // row presence words; then values
    __shared__ uint32_t s_pos[CAP_FAST];
    __shared__ uint16_t s_list[CAP_FAST];
    __shared__ uint64_t s_v1[CAP_FAST];
    __shared__ uint32_t s_meta[CAP_FAST];
    __shared__ uint32_t s_wsum[FAST_T / 64];
    __shared__ uint32_t s_ctl[4];
    __shared__ unsigned long long s_hbase, s_live;
    const uint32_t tid = threadIdx.x;
    const uint32_t n = v.nn;
    uint64_t cv[FAST_R], v0[FAST_R], v1[FAST_R], pk[FAST_R], dbv[FAST_R];
    uint32_t meta[FAST_R], cell[FAST_R], seq[FAST_R], site[FAST_R], pos[FAST_R], rank[FAST_R], tc[FAST_R];
    uint32_t row[FAST_R], ent[FAST_R], hb[FAST_R];
    bool alive[FAST_R];
    uint32_t flags = 0;  // bit 2k: beats the prior clock; bit 2k+1: the cell had no prior clock
    uint4 q[FAST_R][4];
#pragma unroll
    for (int k = 0; k < FAST_R; k++) load_rec_wave_raw(v.fresh, k * FAST_T + (tid & ~63u), n, q[k]);
    const uint32_t used0 = a.rs.used[b];  // (issued with the record loads)
    if (tid == 0) {
        s_live = 0;
        s_ctl[0] = s_ctl[1] = s_ctl[2] = 0;
    }
    for (uint32_t i = tid; i < FAST_SLOTS; i += FAST_T) {
        s_own[i] = 0;
        reinterpret_cast<uint32_t *>(s_v0)[i] = 0;  // the row table of row_claim
    }
#pragma unroll
    for (int k = 0; k < FAST_R; k++) {
        const uint32_t i = k * FAST_T + tid;
        alive[k] = i < n;
        cell[k] = 0;
        const Rec r = rec_from_wave_quads(q[k]);
        pk[k] = r.pk;
        tc[k] = r.tcid;
        s_pk[i] = r.pk;
        s_tc[i] = r.tcid;
        cv[k] = (uint64_t)r.cv ^ 0x8000000000000000ULL;
        v0[k] = r.v0;
        v1[k] = r.v1;
        meta[k] = r.meta;
        pos[k] = r.pos;
        site[k] = r.site;
        dbv[k] = (uint64_t)r.dbv;
        seq[k] = r.seq;
    }
#pragma unroll
    for (int k = 0; k < FAST_R; k++) rank[k] = a.site_rank[site[k] < a.nsites ? site[k] : 0u];
#pragma unroll
    for (int k = 0; k < FAST_R; k++) rank[k] = site[k] < a.nsites ? rank[k] : 0u;
    __syncthreads();
    // 1. rows, then cells (row_claim / cell_claim)
#pragma unroll
    for (int k = 0; k < FAST_R; k++) {
        const uint32_t i = k * FAST_T + tid;
        row[k] = 0;
        if (!alive[k]) continue;
        row[k] = row_claim(reinterpret_cast<uint32_t *>(s_v0), s_pk, s_tc, i, pk[k], tc[k] >> 16);
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < FAST_R; k++)
        if (alive[k]) cell[k] = cell_claim(s_own, k * FAST_T + tid, row[k], tc[k]);
    __syncthreads();
    // 1b. row lookups, prior clocks: does the change beat its cell's prior?
    if (!fast_rows<FAST_R>(a, b, used0, n, row, ent, s_pk, s_tc, s_own, s_v0, s_ctl, &s_hbase, false)) return;
#pragma unroll
    for (int k = 0; k < FAST_R; k++) {
        hb[k] = 0;
        if (!alive[k]) continue;
        const uint32_t c = tc[k] & 0xFFFFu;
        hb[k] = row_heap(s_own[row[k]], s_hbase) + c;
        if ((s_v0[row[k]] >> c) & 1ULL) {
            const Rec pr = load_rec(a.rs.heap + hb[k]);
            const int64_t bcv = (int64_t)(cv[k] ^ 0x8000000000000000ULL);
            int cmp = bcv != pr.cv ? (bcv > pr.cv ? 1 : -1) : value_cmp_f(meta[k], v0[k], v1[k], pr.meta, pr.v0, pr.v1, a.arena);
            if (cmp == 0) {
                const uint32_t prk = site_rank_of(a, pr.site);
                cmp = rank[k] != prk ? (rank[k] > prk ? 1 : -1) : 0;
            }
            if (cmp > 0) flags |= 1u << (2 * k);
        } else {
            flags |= 3u << (2 * k);
        }
    }
    __syncthreads();
    // 2. member counts per owner (s_own reused), keys into LDS
    for (uint32_t i = tid; i < FAST_SLOTS; i += FAST_T) s_own[i] = 0;
    __syncthreads();
#pragma unroll
    for (int k = 0; k < FAST_R; k++) {
        const uint32_t i = k * FAST_T + tid;
        if (!alive[k]) continue;
        s_pk[i] = cv[k];
        s_tc[i] = rank[k];
        s_v0[i] = v0[k];
        s_pos[i] = pos[k];
        s_v1[i] = v1[k];
        s_meta[i] = meta[k];
        atomicAdd(&s_own[cell[k]], 1u);
    }
    __syncthreads();
    // 3. exclusive scan of the counts over owner index [0, n): FAST_R consecutive per thread
    {
        const uint32_t i0 = tid * FAST_R;
        uint32_t c[FAST_R], loc = 0;
#pragma unroll
        for (int k = 0; k < FAST_R; k++) {
            c[k] = i0 + k < n ? s_own[i0 + k] : 0u;
            loc += c[k];
        }
        const uint32_t lane = tid & 63, w = tid >> 6;
        uint32_t inc = loc;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t y = __shfl_up(inc, d);
            if (lane >= (uint32_t)d) inc += y;
        }
        if (lane == 63) s_wsum[w] = inc;
        __syncthreads();
        uint32_t run = inc - loc;
        for (uint32_t ww = 0; ww < w; ww++) run += s_wsum[ww];
#pragma unroll
        for (int k = 0; k < FAST_R; k++)
            if (i0 + k < n) {
                s_own[i0 + k] = run;
                run += c[k];
            }
    }
    __syncthreads();
    uint32_t mbeg[FAST_R];
#pragma unroll
    for (int k = 0; k < FAST_R; k++) mbeg[k] = alive[k] ? s_own[cell[k]] : 0u;
    __syncthreads();
#pragma unroll
    for (int k = 0; k < FAST_R; k++) {
        const uint32_t i = k * FAST_T + tid;
        if (alive[k]) s_list[atomicAdd(&s_own[cell[k]], 1u)] = (uint16_t)i;
    }
    __syncthreads();
    // 4. one walk over the cell's members per change: impact (strict prefix max) and winner
#pragma unroll
    for (int k = 0; k < FAST_R; k++) {
        const uint32_t i = k * FAST_T + tid;
        if (!alive[k]) continue;
        const uint32_t mend = s_own[cell[k]];
        bool imp = (flags >> (2 * k)) & 1u, win = imp;
        for (uint32_t m = mbeg[k]; m < mend; m++) {
            const uint32_t j = s_list[m];
            if (j == i) continue;
            int c;
            const uint64_t cj = s_pk[j];
            if (cj != cv[k]) {
                c = cj > cv[k] ? 1 : -1;
            } else {
                c = value_cmp_f(s_meta[j], s_v0[j], s_v1[j], meta[k], v0[k], v1[k], a.arena);
                if (c == 0) {
                    const uint32_t rj = s_tc[j];
                    c = rj != rank[k] ? (rj > rank[k] ? 1 : -1) : 0;
                }
            }
            const bool earlier = s_pos[j] < pos[k];
            if (earlier && c >= 0) imp = false;             // an earlier change already holds >= key
            if (c > 0 || (c == 0 && earlier)) win = false;  // a greater key, or an equal earlier one
        }
        if (a.impact && (pos[k] & BATCH_POS) && imp) a.impact[pos[k] & 0x7FFFFFFFu] = 1;
        alive[k] = win;
    }
    __syncthreads();
    // 5. winners: the clock row into its heap slot; presence bits of new cells (s_v0 per owner)
#pragma unroll
    for (int k = 0; k < FAST_R; k++) {
        const uint32_t i = k * FAST_T + tid;
        if (ent[k] != ROW_NONE && row[k] == i) s_v0[i] = a.rs.ent[ent[k]].bits[0];
    }
    __syncthreads();
    uint32_t nlive = 0;
#pragma unroll
    for (int k = 0; k < FAST_R; k++) {
        Rec x;
        if (alive[k]) {
            x.pk = pk[k];
            x.cv = (int64_t)(cv[k] ^ 0x8000000000000000ULL);
            x.dbv = (int64_t)dbv[k];
            x.v0 = v0[k];
            x.v1 = v1[k];
            x.tcid = tc[k];
            x.seq = seq[k];
            x.site = site[k];
            x.pos = pos[k];
            x.meta = meta[k];
            if (a.track_ts) a.rs.heap_ts[hb[k]] = rec_ts(a, v, x);
            rec_clear_ts(a, x);
            x.cl = 1;
            x.pos = hb[k];
            if ((flags >> (2 * k + 1)) & 1u) {
                atomicOr(reinterpret_cast<unsigned long long *>(&s_v0[row[k]]), 1ULL << (tc[k] & 0xFFFFu));
                nlive++;
            }
        }
        store_rec_wave(a.rs.heap, hb[k], x, alive[k]);
    }
    nlive = wave_sum_u32(nlive);
    if ((tid & 63) == 0 && nlive) atomicAdd(&s_live, (unsigned long long)nlive);
    __syncthreads();
#pragma unroll
    for (int k = 0; k < FAST_R; k++) {
        const uint32_t i = k * FAST_T + tid;
        if (ent[k] != ROW_NONE && row[k] == i) {
            a.rs.ent[ent[k]].bits[0] = s_v0[i];
            if (a.touch) touch_append(a, pk[k], tc[k] >> 16);
        }
    }
    if (tid == 0 && s_live) atomicAdd(&a.misc[MISC_LIVE], s_live);
}

// The INTEGER form of the impact body in 76 KB of LDS (two workgroups per CU instead of one).
// PACKED (every col_version < 2^15, at most 2^16 sites: the no-impact body's two-stage condition):
// a member's key is two words, (col_version | value bits 63..16) and (value bits 15..0 | site rank),
// so a member slot holds both words and the position in the LDS the unpacked form needs for its
// three key words -- members are placed once and the walk compares positions directly. Unpacked: a
// cell's members are placed in application order (each member's rank among its cell's positions),
// so "earlier" is the member index and no position array is kept for the walk.
// Only zero impacts are stored: the apply initialises the flags to 1 (every other body stores each
// change's flag), which halves the byte scatter into batch order.
// (three-word keys: col_versions of 2^15 or more, or more than 2^16 sites; fast_body_impact_packed
// below takes the common case)
__device__ inline void fast_body_impact_int(const MergeArgs &a, uint32_t b, const BucketView &v) {
    __shared__ uint64_t s_a[CAP_FAST];      // hashing: pk; then the cell-ordered biased col_versions
    __shared__ uint32_t s_b[CAP_FAST];      // hashing: table_cid; then positions by member slot; then site ranks
    __shared__ uint64_t s_c[CAP_FAST];      // row presence words; then cell-ordered values; then presence words
    __shared__ uint32_t s_own[FAST_SLOTS];  // cell / row hashing; heap indices; member counts / offsets / ends
    __shared__ uint32_t s_wsum[FAST_T / 64];
    __shared__ uint32_t s_ctl[4];
    __shared__ unsigned long long s_hbase, s_live;
    const uint32_t tid = threadIdx.x;
    const uint32_t n = v.nn;
    uint64_t cv[FAST_R], v0[FAST_R], pk[FAST_R], dbv[FAST_R];
    uint32_t cell[FAST_R], seq[FAST_R], site[FAST_R], pos[FAST_R], rank[FAST_R], tc[FAST_R];
    uint32_t md[FAST_R];  // member range begin | own member slot << 16 (both < CAP_FAST); end = s_own[cell]
    uint32_t row[FAST_R], ent[FAST_R], hb[FAST_R];
    uint32_t flags = 0;   // bit 2k: beats the prior clock; bit 2k+1: the cell had no prior clock
    bool alive[FAST_R];
    uint4 q[FAST_R][4];
#if CORRO_DIAG & 256
    unsigned long long diag_t2 = wall_clock64();
#define DIAG_MARK2(k) do { if (tid == 0) { const unsigned long long t_ = wall_clock64(); atomicAdd(&a.misc[MISC_DIAG + (k)], t_ - diag_t2); diag_t2 = t_; } } while (0)
#else
#define DIAG_MARK2(k) do { } while (0)
#endif
#pragma unroll
    for (int k = 0; k < FAST_R; k++) load_rec_wave_raw(v.fresh, k * FAST_T + (tid & ~63u), n, q[k]);
    const uint32_t used0 = a.rs.used[b];  // (issued with the record loads)
    if (tid == 0) {
        s_live = 0;
        s_ctl[0] = s_ctl[1] = s_ctl[2] = 0;
    }
    for (uint32_t i = tid; i < FAST_SLOTS; i += FAST_T) {
        s_own[i] = 0;
        reinterpret_cast<uint32_t *>(s_c)[i] = 0;  // the row table of row_claim
    }
#pragma unroll
    for (int k = 0; k < FAST_R; k++) {
        const uint32_t i = k * FAST_T + tid;
        alive[k] = i < n;
        cell[k] = 0;
        const Rec r = rec_from_wave_quads(q[k]);
        pk[k] = r.pk;
        tc[k] = r.tcid;
        s_a[i] = r.pk;
        s_b[i] = r.tcid;
        cv[k] = (uint64_t)r.cv ^ 0x8000000000000000ULL;
        v0[k] = r.v0 ^ 0x8000000000000000ULL;  // INTEGER order as unsigned
        pos[k] = r.pos;
        site[k] = r.site;
        dbv[k] = (uint64_t)r.dbv;
        seq[k] = r.seq;
    }
#pragma unroll
    for (int k = 0; k < FAST_R; k++) rank[k] = a.site_rank[site[k] < a.nsites ? site[k] : 0u];
#pragma unroll
    for (int k = 0; k < FAST_R; k++) rank[k] = site[k] < a.nsites ? rank[k] : 0u;
    __syncthreads();
    DIAG_MARK2(0);
    // 1. rows, then cells (row_claim / cell_claim)
#pragma unroll
    for (int k = 0; k < FAST_R; k++) {
        const uint32_t i = k * FAST_T + tid;
        row[k] = 0;
        if (!alive[k]) continue;
        row[k] = row_claim(reinterpret_cast<uint32_t *>(s_c), s_a, s_b, i, pk[k], tc[k] >> 16);
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < FAST_R; k++)
        if (alive[k]) cell[k] = cell_claim(s_own, k * FAST_T + tid, row[k], tc[k]);
    __syncthreads();
    DIAG_MARK2(1);
    // 1b. row lookups, prior clocks: does the change beat its cell's prior?
    if (!fast_rows<FAST_R>(a, b, used0, n, row, ent, s_a, s_b, s_own, s_c, s_ctl, &s_hbase, false)) return;
    DIAG_MARK2(2);
#pragma unroll
    for (int k = 0; k < FAST_R; k++) {
        hb[k] = 0;
        if (!alive[k]) continue;
        const uint32_t c = tc[k] & 0xFFFFu;
        hb[k] = row_heap(s_own[row[k]], s_hbase) + c;
        if ((s_c[row[k]] >> c) & 1ULL) {
            const Rec pr = load_rec(a.rs.heap + hb[k]);
            if (prior_cmp_int(a, pr, cv[k], v0[k], rank[k]) > 0) flags |= 1u << (2 * k);
        } else {
            flags |= 3u << (2 * k);
        }
    }
    __syncthreads();
    DIAG_MARK2(3);
    // 2. member counts per owner, exclusive scan -> offsets
    for (uint32_t i = tid; i < FAST_SLOTS; i += FAST_T) s_own[i] = 0;
    __syncthreads();
#pragma unroll
    for (int k = 0; k < FAST_R; k++)
        if (alive[k]) atomicAdd(&s_own[cell[k]], 1u);
    __syncthreads();
    {
        const uint32_t i0 = tid * FAST_R;
        uint32_t c[FAST_R], loc = 0;
#pragma unroll
        for (int k = 0; k < FAST_R; k++) {
            c[k] = i0 + k < n ? s_own[i0 + k] : 0u;
            loc += c[k];
        }
        const uint32_t lane = tid & 63, w = tid >> 6;
        uint32_t inc = loc;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t y = __shfl_up(inc, d);
            if (lane >= (uint32_t)d) inc += y;
        }
        if (lane == 63) s_wsum[w] = inc;
        __syncthreads();
        uint32_t run = inc - loc;
        for (uint32_t ww = 0; ww < w; ww++) run += s_wsum[ww];
#pragma unroll
        for (int k = 0; k < FAST_R; k++)
            if (i0 + k < n) {
                s_own[i0 + k] = run;
                run += c[k];
            }
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < FAST_R; k++) md[k] = alive[k] ? s_own[cell[k]] : 0u;
    __syncthreads();
    DIAG_MARK2(4);
    // 3. positions by member slot, then each member's rank among its cell's positions
#pragma unroll
    for (int k = 0; k < FAST_R; k++)
        if (alive[k]) s_b[atomicAdd(&s_own[cell[k]], 1u)] = pos[k];
    __syncthreads();
#pragma unroll
    for (int k = 0; k < FAST_R; k++) {
        if (!alive[k]) continue;
        const uint32_t mb = md[k], me = s_own[cell[k]];
        uint32_t r = 0;
        for (uint32_t m = mb; m < me; m++) r += s_b[m] < pos[k] ? 1u : 0u;  // positions are distinct
        md[k] = mb | ((mb + r) << 16);
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < FAST_R; k++)
        if (alive[k]) {
            const uint32_t d = md[k] >> 16;
            s_a[d] = cv[k];
            s_c[d] = v0[k];
            s_b[d] = rank[k];
        }
    __syncthreads();
    DIAG_MARK2(5);
    // 4. one walk over the cell's members (application order) per change: impact (strict prefix
    // maximum, above the prior clock) and winner (maximum, earliest among equals, above the prior)
#pragma unroll
    for (int k = 0; k < FAST_R; k++) {
        if (!alive[k]) continue;
        bool imp = (flags >> (2 * k)) & 1u, win = imp;
        const uint32_t mb = md[k] & 0xFFFFu, d = md[k] >> 16, me = s_own[cell[k]];
        for (uint32_t m = mb; m < me; m++) {
            if (m == d) continue;
            const uint64_t cj = s_a[m], vj = s_c[m];
            const uint32_t rj = s_b[m];
            const int c = cj != cv[k] ? (cj > cv[k] ? 1 : -1)
                                      : (vj != v0[k] ? (vj > v0[k] ? 1 : -1) : (rj != rank[k] ? (rj > rank[k] ? 1 : -1) : 0));
            const bool earlier = m < d;
            if (earlier && c >= 0) imp = false;             // an earlier change already holds >= key
            if (c > 0 || (c == 0 && earlier)) win = false;  // a greater key, or an equal earlier one
        }
        if (a.impact && (pos[k] & BATCH_POS) && imp) a.impact[pos[k] & 0x7FFFFFFFu] = 1;
        alive[k] = win;
    }
    __syncthreads();
    DIAG_MARK2(6);
    // 5. winners: the clock row into its heap slot; presence bits of new cells (s_c per owner)
#pragma unroll
    for (int k = 0; k < FAST_R; k++) {
        const uint32_t i = k * FAST_T + tid;
        if (ent[k] != ROW_NONE && row[k] == i) s_c[i] = a.rs.ent[ent[k]].bits[0];
    }
    __syncthreads();
    uint32_t nlive = 0;
#pragma unroll
    for (int k = 0; k < FAST_R; k++) {
        Rec x;
        if (alive[k]) {
            x.pk = pk[k];
            x.cv = (int64_t)(cv[k] ^ 0x8000000000000000ULL);
            x.dbv = (int64_t)dbv[k];
            x.v0 = v0[k] ^ 0x8000000000000000ULL;
            x.v1 = 0;
            x.tcid = tc[k];
            x.seq = seq[k];
            x.site = site[k];
            x.pos = pos[k];
            x.meta = CORRO_INTEGER;
            if (a.track_ts) a.rs.heap_ts[hb[k]] = win_ts(a, v, x, k * FAST_T + tid);
            x.cl = 1;
            x.pos = hb[k];
            if ((flags >> (2 * k + 1)) & 1u) {
                atomicOr(reinterpret_cast<unsigned long long *>(&s_c[row[k]]), 1ULL << (tc[k] & 0xFFFFu));
                nlive++;
            }
        }
        store_rec_wave(a.rs.heap, hb[k], x, alive[k]);
    }
    nlive = wave_sum_u32(nlive);
    if ((tid & 63) == 0 && nlive) atomicAdd(&s_live, (unsigned long long)nlive);
    __syncthreads();
#pragma unroll
    for (int k = 0; k < FAST_R; k++) {
        const uint32_t i = k * FAST_T + tid;
        if (ent[k] != ROW_NONE && row[k] == i) {
            a.rs.ent[ent[k]].bits[0] = s_c[i];
            if (a.touch) touch_append(a, pk[k], tc[k] >> 16);
        }
    }
    if (tid == 0 && s_live) atomicAdd(&a.misc[MISC_LIVE], s_live);
    DIAG_MARK2(7);
}

// Packed INTEGER impact body (col_versions < 2^15, <= 2^16 sites): each change's key is two words,
// k1 = cv 15 | value bits 63..16 and k2 = value bits 15..0 | site rank 16, kept in registers with
// the change's position, cell, row and heap slot only -- the rest of a winner's clock row (db_version,
// seq, site) is re-read from its staged record at the end (the register budget of two workgroups per
// CU, no spills). An empty region (the common case of a fresh state) has no prior clocks, so its rows
// are counted right after the hashing, the heap allocation is issued before the member walk and
// consumed after it, and the region entries are written at the end; a populated region resolves its
// rows and prior clocks first (impacts depend on them).
__device__ inline int prior_cmp_packed(const MergeArgs &a, const Rec &pr, uint64_t k1, uint32_t k2) {
    const uint64_t cv = k1 >> 48, pcv = (uint64_t)pr.cv ^ 0x8000000000000000ULL;
    const uint64_t cvb = cv ^ 0x8000000000000000ULL;  // (cv >= 0: biased like pcv)
    if (cvb != pcv) return cvb > pcv ? 1 : -1;
    const uint64_t v0b = ((k1 & 0xFFFFFFFFFFFFULL) << 16) | (k2 >> 16), pv = pr.v0 ^ 0x8000000000000000ULL;
    if (v0b != pv) return v0b > pv ? 1 : -1;
    const uint32_t rank = k2 & 0xFFFFu, pr_rank = site_rank_of(a, pr.site);
    return rank != pr_rank ? (rank > pr_rank ? 1 : -1) : 0;
}

__device__ inline void fast_body_impact_packed(const MergeArgs &a, uint32_t b, const BucketView &v) {
    __shared__ uint64_t s_a[CAP_FAST];      // hashing: pk; then k1 by member slot
    __shared__ uint32_t s_b[CAP_FAST];      // hashing: table_cid; then k2 by member slot
    __shared__ uint64_t s_c[CAP_FAST];      // row table; presence words (populated region); positions by member slot; presence words
    __shared__ uint32_t s_own[FAST_SLOTS];  // cell table; heap words; member counts / offsets / ends
    __shared__ uint32_t s_wsum[FAST_T / 64];
    __shared__ uint32_t s_ctl[4];
    __shared__ unsigned long long s_hbase, s_live;
    const uint32_t tid = threadIdx.x;
    const uint32_t n = v.nn;
    uint64_t k1[FAST_R];
    uint32_t k2[FAST_R], cell[FAST_R], pos[FAST_R], tc[FAST_R], md[FAST_R], row[FAST_R], ent[FAST_R], hb[FAST_R];
    uint32_t flags = 0;   // bit 2k: beats the prior clock; bit 2k+1: the cell had no prior clock
    bool alive[FAST_R];
    uint4 q[FAST_R][4];
#if CORRO_DIAG & 256
    unsigned long long diag_t2 = wall_clock64();
#endif
#pragma unroll
    for (int k = 0; k < FAST_R; k++) load_rec_wave_raw(v.fresh, k * FAST_T + (tid & ~63u), n, q[k]);
    const uint32_t used0 = a.rs.used[b];  // (issued with the record loads)
    if (tid == 0) {
        s_live = 0;
        s_ctl[0] = s_ctl[1] = s_ctl[2] = s_ctl[3] = 0;
    }
    for (uint32_t i = tid; i < FAST_SLOTS; i += FAST_T) {
        s_own[i] = 0;
        reinterpret_cast<uint32_t *>(s_c)[i] = 0;  // the row table of row_claim
    }
    uint32_t site[FAST_R];
#pragma unroll
    for (int k = 0; k < FAST_R; k++) {
        const uint32_t i = k * FAST_T + tid;
        alive[k] = i < n;
        cell[k] = 0;
        const Rec r = rec_from_wave_quads(q[k]);
        tc[k] = r.tcid;
        s_a[i] = r.pk;
        s_b[i] = r.tcid;
        const uint64_t v0b = r.v0 ^ 0x8000000000000000ULL;  // INTEGER order as unsigned
        k1[k] = ((uint64_t)r.cv << 48) | (v0b >> 16);
        k2[k] = (uint32_t)(v0b & 0xFFFFu) << 16;
        pos[k] = r.pos;
        site[k] = r.site;
    }
    // site ranks and, for an empty region, row strides: one more batch of loads during the claims
    uint32_t strd[FAST_R];
#pragma unroll
    for (int k = 0; k < FAST_R; k++) {
        strd[k] = used0 ? 0u : (uint32_t)a.rs.stride[alive[k] ? tc[k] >> 16 : 0u];
        k2[k] |= a.site_rank[site[k] < a.nsites ? site[k] : 0u];
    }
#pragma unroll
    for (int k = 0; k < FAST_R; k++)
        if (site[k] >= a.nsites) k2[k] &= 0xFFFF0000u;
    __syncthreads();
    DIAG_MARK2(0);
    // 1. rows, then cells
#pragma unroll
    for (int k = 0; k < FAST_R; k++) {
        const uint32_t i = k * FAST_T + tid;
        row[k] = 0;
        if (!alive[k]) continue;
        row[k] = row_claim(reinterpret_cast<uint32_t *>(s_c), s_a, s_b, i, s_a[i], tc[k] >> 16);
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < FAST_R; k++)
        if (alive[k]) cell[k] = cell_claim(s_own, k * FAST_T + tid, row[k], tc[k]);
    __syncthreads();
    DIAG_MARK2(1);
    unsigned long long hraw = 0;
    if (!used0) {
        // 1b (empty region). every row new: heap offsets counted now (s_own: heap words by owner),
        // the allocation issued now and checked after the walk; no prior clocks
        fast_rows_count<FAST_R>(n, row, strd, s_own, s_ctl);
        __syncthreads();
#pragma unroll
        for (int k = 0; k < FAST_R; k++) {
            hb[k] = alive[k] ? (s_own[row[k]] & 0x7FFFFFFFu) + (tc[k] & 0xFFFFu) : 0u;  // (+ heap base below)
            ent[k] = ROW_NONE;
            if (alive[k]) flags |= 3u << (2 * k);
        }
        if (tid == 0 && s_ctl[1] && s_ctl[0] <= a.rs.fill) hraw = atomicAdd(a.rs.heap_top, (unsigned long long)s_ctl[1]);
    } else {
        // 1b (populated region). row lookups, prior clocks: does the change beat its cell's prior?
        if (!fast_rows<FAST_R>(a, b, used0, n, row, ent, s_a, s_b, s_own, s_c, s_ctl, &s_hbase, false)) return;
#pragma unroll
        for (int k = 0; k < FAST_R; k++) {
            hb[k] = 0;
            if (!alive[k]) continue;
            const uint32_t c = tc[k] & 0xFFFFu;
            hb[k] = row_heap(s_own[row[k]], s_hbase) + c;
            if ((s_c[row[k]] >> c) & 1ULL) {
                const Rec pr = load_rec(a.rs.heap + hb[k]);
                if (prior_cmp_packed(a, pr, k1[k], k2[k]) > 0) flags |= 1u << (2 * k);
            } else {
                flags |= 3u << (2 * k);
            }
        }
    }
    __syncthreads();
    DIAG_MARK2(2);
#if IMPACT_LISTS
    // 2. each cell's members as a list: its claimant heads it, the other members chain in (one LDS
    // exchange each); keys and positions stay at the members' record indices (no counting sort)
    uint32_t *s_p = reinterpret_cast<uint32_t *>(s_c), *s_nx = s_p + CAP_FAST;
    for (uint32_t i = tid; i < CAP_FAST; i += FAST_T) s_own[i] = 0;
#pragma unroll
    for (int k = 0; k < FAST_R; k++)
        if (alive[k]) {
            const uint32_t i = k * FAST_T + tid;
            s_a[i] = k1[k];
            s_b[i] = k2[k];
            s_p[i] = pos[k];
        }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < FAST_R; k++) {
        const uint32_t i = k * FAST_T + tid;
        if (alive[k] && cell[k] != i) s_nx[i] = atomicExch(&s_own[cell[k]], i + 1);
    }
    __syncthreads();
    // 4. one walk over the cell's members per change: impact (strict prefix maximum in application
    // order, above the prior clock) and winner (maximum, earliest among equals, above the prior)
#pragma unroll
    for (int k = 0; k < FAST_R; k++) {
        if (!alive[k]) continue;
        bool imp = (flags >> (2 * k)) & 1u, win = imp;
        const uint32_t i = k * FAST_T + tid;
        uint32_t m = cell[k], nxt = s_own[cell[k]];
        while (true) {
            if (m != i) {
                const uint64_t j1 = s_a[m];
                const uint32_t j2 = s_b[m];
                const int c = j1 != k1[k] ? (j1 > k1[k] ? 1 : -1) : (j2 != k2[k] ? (j2 > k2[k] ? 1 : -1) : 0);
                const bool earlier = s_p[m] < pos[k];
                if (earlier && c >= 0) imp = false;             // an earlier change already holds >= key
                if (c > 0 || (c == 0 && earlier)) win = false;  // a greater key, or an equal earlier one
            }
            if (nxt == 0) break;
            m = nxt - 1;
            nxt = s_nx[m];
        }
#if !(CORRO_DIAG & 1024)  // (1024: diagnostics only -- no flag stores, results not valid)
        if (a.impact && (pos[k] & BATCH_POS) && imp) a.impact[pos[k] & 0x7FFFFFFFu] = 1;
#endif
        alive[k] = win;
    }
#else
    // 2. member counts per cell, exclusive scan -> offsets
    for (uint32_t i = tid; i < CAP_FAST; i += FAST_T) s_own[i] = 0;
    __syncthreads();
#pragma unroll
    for (int k = 0; k < FAST_R; k++)
        if (alive[k]) atomicAdd(&s_own[cell[k]], 1u);
    __syncthreads();
    {
        const uint32_t i0 = tid * FAST_R;
        uint32_t c[FAST_R], loc = 0;
#pragma unroll
        for (int k = 0; k < FAST_R; k++) {
            c[k] = i0 + k < n ? s_own[i0 + k] : 0u;
            loc += c[k];
        }
        const uint32_t lane = tid & 63, w = tid >> 6;
        const uint32_t inc = wave_incl_scan(loc);
        if (lane == 63) s_wsum[w] = inc;
        __syncthreads();
        uint32_t run = inc - loc;
        for (uint32_t ww = 0; ww < w; ww++) run += s_wsum[ww];
#pragma unroll
        for (int k = 0; k < FAST_R; k++)
            if (i0 + k < n) {
                s_own[i0 + k] = run;
                run += c[k];
            }
    }
    __syncthreads();
    DIAG_MARK2(3);
#pragma unroll
    for (int k = 0; k < FAST_R; k++) md[k] = alive[k] ? s_own[cell[k]] : 0u;
    __syncthreads();
    // 3. keys and positions by member slot
    uint32_t *s_p = reinterpret_cast<uint32_t *>(s_c);
#pragma unroll
    for (int k = 0; k < FAST_R; k++)
        if (alive[k]) {
            const uint32_t d = atomicAdd(&s_own[cell[k]], 1u);
            s_a[d] = k1[k];
            s_b[d] = k2[k];
            s_p[d] = pos[k];
            md[k] |= d << 16;
        }
    __syncthreads();
    DIAG_MARK2(4);
    // 4. one walk over the cell's members per change: impact (strict prefix maximum in application
    // order, above the prior clock) and winner (maximum, earliest among equals, above the prior)
#pragma unroll
    for (int k = 0; k < FAST_R; k++) {
        if (!alive[k]) continue;
        bool imp = (flags >> (2 * k)) & 1u, win = imp;
        const uint32_t mb = md[k] & 0xFFFFu, d = md[k] >> 16, me = s_own[cell[k]];
#if CORRO_DIAG & 2048  // (diagnostics only: no member walk -- the cell's claimant wins, results not valid)
        win = cell[k] == k * FAST_T + tid;
        if (a.impact && (pos[k] & BATCH_POS) && imp) a.impact[pos[k] & 0x7FFFFFFFu] = 1;
        alive[k] = win;
        continue;
#endif
        for (uint32_t m = mb; m < me; m++) {
            if (m == d) continue;
            const uint64_t j1 = s_a[m];
            const uint32_t j2 = s_b[m];
            const int c = j1 != k1[k] ? (j1 > k1[k] ? 1 : -1) : (j2 != k2[k] ? (j2 > k2[k] ? 1 : -1) : 0);
            const bool earlier = s_p[m] < pos[k];
            if (earlier && c >= 0) imp = false;             // an earlier change already holds >= key
            if (c > 0 || (c == 0 && earlier)) win = false;  // a greater key, or an equal earlier one
        }
#if !(CORRO_DIAG & 1024)  // (1024: diagnostics only -- no flag stores, results not valid)
        if (a.impact && (pos[k] & BATCH_POS) && imp) a.impact[pos[k] & 0x7FFFFFFFu] = 1;
#endif
        alive[k] = win;
    }
#endif
    DIAG_MARK2(5);
    if (!used0) {
        // 4b (empty region). the heap allocation issued before the walk: room, or defer (nothing of
        // the bucket's state written yet; its impact flags depend on the batch only)
        if (tid == 0) {
            const unsigned long long need = s_ctl[1];
            const bool room = s_ctl[0] <= a.rs.fill;
            if (!room || (need && hraw + need > a.rs.heap_cap)) {
                if (room && need) atomicSub(a.rs.heap_top, need);
                push_defer(a, b, room ? DEFER_HEAP : DEFER_REGION);
                s_ctl[2] = 1;
            } else {
                a.rs.used[b] = s_ctl[0];
                s_hbase = need ? hraw : 0;
            }
        }
        __syncthreads();
        if (s_ctl[2]) return;
        // the owners' row keys and heap words again (s_a / s_b / s_own held the member lists),
        // then the region entries
#pragma unroll
        for (int k = 0; k < FAST_R; k++) {
            const uint32_t i = k * FAST_T + tid;
            if (i < n && row[k] == i) {
                s_a[i] = v.fresh[i].pk;
                s_b[i] = tc[k];
                s_own[i] = 0x80000000u | (hb[k] - (tc[k] & 0xFFFFu));
            }
        }
        if (!fast_rows<FAST_R>(a, b, 0u, n, row, ent, s_a, s_b, s_own, s_c, s_ctl, &s_hbase, true)) return;
#pragma unroll
        for (int k = 0; k < FAST_R; k++) hb[k] += (uint32_t)s_hbase;
    } else {
        __syncthreads();
        // presence words of the populated rows again (s_c held the positions)
#pragma unroll
        for (int k = 0; k < FAST_R; k++) {
            const uint32_t i = k * FAST_T + tid;
            if (ent[k] != ROW_NONE && row[k] == i) s_c[i] = a.rs.ent[ent[k]].bits[0];
        }
    }
    __syncthreads();
    DIAG_MARK2(6);
    // 5. winners: the rest of the clock row from the staged record, into its heap slot; presence bits
    uint32_t nlive = 0;
    constexpr int WH = (FAST_R + 1) / 2;  // two halves: the reloads of one half in flight at once
#pragma unroll
    for (int h = 0; h < FAST_R; h += WH) {
        uint2 w0[WH], w16[WH], w48[WH], w32[WH];  // pk | db_version | seq, site | ts (ts_v1)
        const bool tsv = a.track_ts && a.ts_v1;
#pragma unroll
        for (int u = 0; u < WH && h + u < FAST_R; u++) {
            const int k = h + u;
            const uint32_t i = k * FAST_T + tid;
            const uint2 *src = reinterpret_cast<const uint2 *>(v.fresh + i);
            if (alive[k]) {
                w0[u] = src[0];
                w16[u] = src[2];
                w48[u] = src[6];
                if (tsv) w32[u] = src[4];
            }
        }
#pragma unroll
        for (int u = 0; u < WH && h + u < FAST_R; u++) {
            const int k = h + u;
            Rec x;
            if (alive[k]) {
                x.pk = ((uint64_t)w0[u].y << 32) | w0[u].x;
                x.cv = (int64_t)(k1[k] >> 48);
                x.dbv = (int64_t)(((uint64_t)w16[u].y << 32) | w16[u].x);
                x.v0 = (((k1[k] & 0xFFFFFFFFFFFFULL) << 16) | (k2[k] >> 16)) ^ 0x8000000000000000ULL;
                x.v1 = 0;
                x.tcid = tc[k];
                x.seq = w48[u].x;
                x.site = w48[u].y;
                x.pos = pos[k];
                x.meta = CORRO_INTEGER;
                if (a.track_ts)
                    a.rs.heap_ts[hb[k]] = tsv && (x.pos & BATCH_POS) ? ((uint64_t)w32[u].y << 32) | w32[u].x : rec_ts(a, v, x);
                x.cl = 1;
                x.pos = hb[k];
                if ((flags >> (2 * k + 1)) & 1u) {
                    atomicOr(reinterpret_cast<unsigned long long *>(&s_c[row[k]]), 1ULL << (tc[k] & 0xFFFFu));
                    nlive++;
                }
            }
            store_rec_wave(a.rs.heap, hb[k], x, alive[k]);
        }
    }
    nlive = wave_sum_u32(nlive);
    if ((tid & 63) == 0 && nlive) atomicAdd(&s_live, (unsigned long long)nlive);
    __syncthreads();
    DIAG_MARK2(7);
#pragma unroll
    for (int k = 0; k < FAST_R; k++) {
        const uint32_t i = k * FAST_T + tid;
        if (ent[k] != ROW_NONE && row[k] == i) {
            a.rs.ent[ent[k]].bits[0] = s_c[i];
            if (a.touch) touch_append(a, v.fresh[i].pk, tc[k] >> 16);
        }
    }
    if (tid == 0 && s_live) atomicAdd(&a.misc[MISC_LIVE], s_live);
}

__device__ inline uint32_t bucket_of_block(const MergeArgs &a) {
    return a.bucket_list ? a.bucket_list[blockIdx.x] : blockIdx.x;
}

// Bucket triage + the INTEGER fast body (one workgroup per bucket). General buckets and, for a
// batch or state with non-INTEGER values, every fast bucket are queued for the list-driven kernels
// below, so those launch a few hundred workgroups instead of one per bucket.
// IMPACT bodies come as two kernels, PACKED chosen by the host from k_scatter's MISC_CVBIG (one
// kernel holding both forms would size its registers for the larger and halve the occupancy)
// The triage as its own pass (k_triage: one lane per bucket, each queue append aggregated per wave)
// when a batch is mostly general (config 5: 32 K one-workgroup triages of k_merge_fast_int, each one
// same-address queue atomic, cost 0.4 ms): a_fast[b] = 1 for the buckets left to the INTEGER fast
// body, whose workgroups then skip the triage. Queue q: 0 ovf, 1 gen_small, 2 gen_mid, 3 gen, 4 wide.
__device__ inline void queue_append_wave(const MergeArgs &a, int q, bool mine, uint32_t b) {
    const uint64_t m = __ballot(mine);
    if (!m) return;
    const uint32_t lane = threadIdx.x & 63;
    const int leader = __ffsll((unsigned long long)m) - 1;
    const int word = q == 0 ? MISC_OVF : q == 1 ? MISC_GEN_SMALL : q == 2 ? MISC_GEN_MID : q == 3 ? MISC_GEN : MISC_WIDEQ;
    unsigned long long base = 0;
    if ((int)lane == leader) base = atomicAdd(&a.misc[word], (unsigned long long)__popcll(m));
    base = __shfl(base, leader);
    if (!mine) return;
    const uint32_t k = (uint32_t)base + (uint32_t)__popcll(m & ((1ULL << lane) - 1));
    if (q == 0) a.ovf_list[k] = b;
    else if (q == 1) a.gen_list[a.B + k] = b;
    else if (q == 2) a.gen_list[2 * a.B + k] = b;
    else if (q == 3) a.gen_list[k] = b;
    else a.wide_list[k] = b;
}

static __global__ void __launch_bounds__(256) k_triage(MergeArgs a, uint32_t nb, uint8_t *__restrict__ fast) {
    if (a.misc[0]) return;
    const unsigned long long wide = a.misc[MISC_WIDE];
    for (uint32_t base = blockIdx.x * blockDim.x; base < nb; base += gridDim.x * blockDim.x) {  // (wave-uniform)
        const uint32_t j = base + threadIdx.x;
        int q = -1;  // -1: nothing (empty / past the end), 5: fast body
        uint32_t b = 0;
        if (j < nb) {
            b = a.bucket_list ? a.bucket_list[j] : j;
            const uint32_t n = a.new_cnt[b];
            if (n) {
                if (a.force_general || a.rs.gen[b] || ((a.bflags[b >> 5] >> (b & 31)) & 1u))
                    q = n > a.gen_ovf_min ? 0 : n <= CAP_GEN_SMALL ? 1 : n <= CAP_GEN_MID ? 2 : 3;
                else if (n > (uint32_t)CAP_FAST) q = 0;
                else if (a.state_wide || wide != 0) q = 4;
                else q = 5;
            }
            fast[j] = q == 5 ? 1 : 0;
        }
        for (int k = 0; k < 5; k++) queue_append_wave(a, k, q == k, b);
    }
}

template <bool IMPACT, bool PACKED = false>
static __global__ void __launch_bounds__(FAST_T, FAST_WAVES_EU)
k_merge_fast_int(MergeArgs a) {
    if (a.fast_of && !a.fast_of[blockIdx.x]) return;  // (k_triage queued it, or it is empty)
    if (a.misc[0]) return;  // the batch failed k_scatter's validation: nothing is merged
    const uint32_t b = bucket_of_block(a);
    // every per-bucket word is loaded up front (independent scalar loads, one latency)
    BucketView v;
    bucket_view(a, b, v);
    const uint32_t rgen = a.rs.gen[b];
    const uint32_t bword = a.bflags[b >> 5];
    const unsigned long long wide = a.misc[MISC_WIDE], cvbig = a.misc[MISC_CVBIG];
    const uint32_t n = v.nn;
    if (n == 0) return;
    if (!a.fast_of && (a.force_general || rgen || ((bword >> (b & 31)) & 1u))) {
        if (threadIdx.x == 0) {
            if (n > a.gen_ovf_min)
                push_overflow(a, b);
            else if (n <= CAP_GEN_SMALL)
                a.gen_list[a.B + atomicAdd(&a.misc[MISC_GEN_SMALL], 1ULL)] = b;
            else if (n <= CAP_GEN_MID)
                a.gen_list[2 * a.B + atomicAdd(&a.misc[MISC_GEN_MID], 1ULL)] = b;
            else
                a.gen_list[atomicAdd(&a.misc[MISC_GEN], 1ULL)] = b;
        }
        return;
    }
    if (!a.fast_of && n > (uint32_t)CAP_FAST) {
        if (threadIdx.x == 0) push_overflow(a, b);
        return;
    }
    if (!a.fast_of && (a.state_wide || wide != 0)) {
        if (threadIdx.x == 0) a.wide_list[atomicAdd(&a.misc[MISC_WIDEQ], 1ULL)] = b;
        return;
    }
    if constexpr (IMPACT) {
        (void)cvbig;
        if constexpr (PACKED) fast_body_impact_packed(a, b, v);
        else fast_body_impact_int(a, b, v);
    } else {
        fast_body<false>(a, b, v, cvbig == 0 && a.nsites <= 65536);
    }
}

constexpr uint32_t LIST_GRID = 512;

template <bool IMPACT>
static __global__ void __launch_bounds__(FAST_T, IMPACT ? FAST_WAVES_EU / 2 : FAST_WAVES_EU)
k_merge_fast_wide(MergeArgs a) {
    const uint32_t cnt = (uint32_t)a.misc[MISC_WIDEQ];
    for (uint32_t k = blockIdx.x; k < cnt; k += gridDim.x) {
        const uint32_t b = a.wide_list[k];
        BucketView v;
        bucket_view(a, b, v);
        if (IMPACT)
            fast_body_impact_wide(a, b, v);
        else
            fast_body<true>(a, b, v);
        __syncthreads();
    }
}

static __global__ void __launch_bounds__(MERGE_THREADS)
k_merge_gen(MergeArgs a) {
    const uint32_t cnt = (uint32_t)a.misc[MISC_GEN];
    for (uint32_t k = blockIdx.x; k < cnt; k += gridDim.x) {
        gen_bucket<CAP_GEN, MERGE_THREADS, 0>(a, a.gen_list[k]);
        __syncthreads();
    }
}

// general buckets of at most CAP_GEN_MID records (queued at gen_list + 2B)
static __global__ void __launch_bounds__(MERGE_THREADS, 4)
k_merge_gen_mid(MergeArgs a) {
    const uint32_t cnt = (uint32_t)a.misc[MISC_GEN_MID];
    for (uint32_t k = blockIdx.x; k < cnt; k += gridDim.x) {
        gen_bucket<CAP_GEN_MID, MERGE_THREADS, 2>(a, a.gen_list[2 * a.B + k]);
        __syncthreads();
    }
}

// general buckets of at most CAP_GEN_SMALL records (queued at gen_list + B)
static __global__ void __launch_bounds__(GEN_SMALL_THREADS, 4)
k_merge_gen_small(MergeArgs a) {
    const uint32_t cnt = (uint32_t)a.misc[MISC_GEN_SMALL];
    for (uint32_t k = blockIdx.x; k < cnt; k += gridDim.x) {
        gen_bucket<CAP_GEN_SMALL, GEN_SMALL_THREADS, 1>(a, a.gen_list[a.B + k]);
        __syncthreads();
    }
}

// Validation of a whole batch before a chunked apply commits its first chunk (the checks k_scatter
// makes per chunk; a batch is applied all or nothing).
// Rows in the state after an apply: the sum of the regions' entry counts (sizes the regions).
static __global__ void __launch_bounds__(1024) k_sum_used(const uint32_t *__restrict__ used, uint32_t B,
                                                          unsigned long long *misc) {
    unsigned long long t = 0;
    for (uint32_t b = threadIdx.x; b < B; b += 1024) t += used[b];
    for (int d = 32; d >= 1; d >>= 1) t += __shfl_xor(t, d);
    if ((threadIdx.x & 63) == 0 && t) atomicAdd(&misc[MISC_ROWS], t);
}

static __global__ void k_validate(BatchDev in, uint32_t nsites, const uint16_t *__restrict__ ncols, uint32_t ntables,
                                  unsigned long long *misc) {
    uint32_t err = 0, wide = 0;
    const bool sover = in.slot_rec && slot_overflowed(in);
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < in.n; i += gridDim.x * blockDim.x) {
        if (in.slot_rec) {  // slot mode: the received records that will be applied (INTEGER values)
            if (!slot_valid(in, i, sover)) continue;
            const SlotRec &r = in.slot_rec[i];
            const uint32_t t = r.tcid >> 16, cid = r.tcid & 0xFFFFu;
            if (t >= ntables || cid > ncols[t]) err |= ERR_NAME;
            if (r.site >= nsites) err |= ERR_SITE;
            if ((cid == 0 || (r.cl & 1u) == 0) && (r.cv < 0 || r.cv > 0xFFFFFFFFLL)) err |= ERR_RANGE;
            if (r.dbv < 0) err |= ERR_RANGE;
            continue;
        }
        const uint32_t tc = in.tcid[i], t = tc >> 16, cid = tc & 0xFFFFu, cl = in.cl[i];
        const int64_t cv = in.cv[i];
        if (t >= ntables || cid > ncols[t]) err |= ERR_NAME;
        if (in.site[i] >= nsites) err |= ERR_SITE;
        if ((cid == 0 || (cl & 1u) == 0) && (cv < 0 || cv > 0xFFFFFFFFLL)) err |= ERR_RANGE;
        if (in.dbv[i] < 0) err |= ERR_RANGE;
        if (in.vt) {
            const uint32_t ty = in.vt[i], ln = in.vl ? in.vl[i] : 0u;
            if (ty != CORRO_INTEGER) {
                wide = 1;
                const uint64_t v0 = in.v0[i];
                if (ty < 1 || ty > 5) err |= ERR_VALUE;
                if (ty == CORRO_REAL && ((v0 >> 52) & 0x7FF) == 0x7FF && (v0 & 0xFFFFFFFFFFFFFULL)) err |= ERR_VALUE;
                if ((ty == CORRO_TEXT || ty == CORRO_BLOB) && ln > 16) {
                    uint64_t w0, w1;
                    if (ln != VLEN_LONG || !long_value(in, i, w0, w1)) err |= ERR_VALUE;
                }
            }
        }
    }
    if (__any(err != 0)) {
        for (int d = 32; d >= 1; d >>= 1) err |= __shfl_xor(err, d);
        if ((threadIdx.x & 63) == 0) atomicOr(&misc[0], (unsigned long long)err);
    }
    if (__any(wide != 0) && (threadIdx.x & 63) == 0) atomicOr(&misc[3], 1ULL);
}

// crsql_db_versions fold after a batch that passed validation (misc[0]: k_scatter's error bits; a
// batch that fails them is never merged)
static __global__ void k_dbv_fold(unsigned long long *__restrict__ dbv, const unsigned long long *__restrict__ batch,
                           uint32_t nsites, const unsigned long long *__restrict__ misc) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (misc[0]) return;
    if (i < nsites && batch[i] > dbv[i]) dbv[i] = batch[i];
}

// Export / materialisation: every present clock record of the row store, row by row (rows in slot
// order; a row's records sentinel first, then by cid), each with the row's causal length. Output
// slots come from one atomic per wave (a wave-level prefix sum of the rows' record counts).
template <class F>
__device__ inline void for_each_state_record(const RowStore &rs, uint64_t nent, unsigned long long *count, F &&f) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t base = (uint64_t)blockIdx.x * blockDim.x + (threadIdx.x & ~63u); base < nent; base += stride) {
        const uint64_t e = base + lane;
        RowEnt re{};
        if (e < nent) re = rs.ent[e];
        const bool ok = re.tag != 0;
        const uint32_t cnt = ok ? row_popc(re.bits) : 0u;
        uint32_t inc = cnt;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t y = __shfl_up(inc, d);
            if (lane >= (uint32_t)d) inc += y;
        }
        const uint32_t tot = __shfl(inc, 63);
        unsigned long long w0 = 0;
        if (lane == 63 && tot) w0 = atomicAdd(count, (unsigned long long)tot);
        w0 = __shfl(w0, 63);
        if (!cnt) continue;
        unsigned long long k = w0 + inc - cnt;
        const int64_t L = (re.bits[0] & 1ULL) ? rs.heap[re.heap].cv : 1;
        for (int w = 0; w < 2; w++)
            for (uint64_t m = re.bits[w]; m; m &= m - 1) {
                const uint32_t c = 64 * w + (uint32_t)__ffsll((unsigned long long)m) - 1;
                f(k++, re.heap + c, L);
            }
    }
}

// one clock record (heap index h, row causal length L) as crsql_changes row k
__device__ inline void export_rec(const RowStore &rs, const corro_rows &o, unsigned long long k, uint32_t h, int64_t L) {
    const Rec r = load_rec(rs.heap + h);
    o.pk[k] = r.pk;
    o.table_cid[k] = r.tcid;
    o.col_version[k] = r.cv;
    o.db_version[k] = r.dbv;
    o.cl[k] = L;
    o.seq[k] = r.seq;
    o.site[k] = r.site;
    o.ts[k] = rs.heap_ts ? rs.heap_ts[h] : 0ULL;
    o.val0[k] = r.v0;
    o.val1[k] = r.v1;
    o.val_type[k] = (uint8_t)vtype(r.meta);
    o.val_len[k] = (uint8_t)vlen(r.meta);
}

static __global__ void k_export(RowStore rs, uint64_t nent, unsigned long long *count, corro_rows o) {
    for_each_state_record(rs, nent, count,
                          [&](unsigned long long k, uint32_t h, int64_t L) { export_rec(rs, o, k, h, L); });
}

// corro_state_export_touched, pass 1: each listed row's region entry (looked up in its bucket's
// region) and, for the first listing of the row in this export (stamp), its clock record count
static __global__ void k_touch_count(RowStore rs, uint32_t log2B, const uint4 *__restrict__ touch, uint64_t m,
                                     uint32_t *__restrict__ stamp, uint32_t epoch, uint32_t *__restrict__ ent,
                                     uint32_t *__restrict__ cnt) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint4 t = touch[i];
        const uint64_t pk = (uint64_t)t.x | ((uint64_t)t.y << 32);
        const uint32_t e = rs_lookup(rs, bucket_of(t.z, pk, log2B), pk, t.z);
        uint32_t c = 0;
        if (e != ROW_NONE && atomicExch(&stamp[e], epoch) != epoch) c = row_popc(rs.ent[e].bits);
        ent[i] = e;
        cnt[i] = c;
    }
}

// pass 2: the row's records at [incl - cnt, incl), sentinel first then by cid
static __global__ void k_touch_rows(RowStore rs, const uint32_t *__restrict__ ent, const uint32_t *__restrict__ cnt,
                                    const uint32_t *__restrict__ incl, uint64_t m, corro_rows o) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += (uint64_t)gridDim.x * blockDim.x) {
        if (!cnt[i]) continue;
        const RowEnt re = rs.ent[ent[i]];
        unsigned long long k = incl[i] - cnt[i];
        const int64_t L = (re.bits[0] & 1ULL) ? rs.heap[re.heap].cv : 1;
        for (int w = 0; w < 2; w++)
            for (uint64_t b = re.bits[w]; b; b &= b - 1) {
                const uint32_t c = 64 * w + (uint32_t)__ffsll((unsigned long long)b) - 1;
                export_rec(rs, o, k++, re.heap + c, L);
            }
    }
}

// dense copy of the state's clock records (64-B Recs with cl = the row's causal length, pos = the
// dense index) + their ts, for the extraction index
static __global__ void k_materialize(RowStore rs, uint64_t nent, unsigned long long *count, Rec *out,
                                     uint64_t *out_ts) {
    for_each_state_record(rs, nent, count, [&](unsigned long long k, uint32_t h, int64_t L) {
        Rec r = load_rec(rs.heap + h);
        r.cl = (uint32_t)L;
        r.pos = (uint32_t)k;
        store_rec(out + k, r);
        if (out_ts) out_ts[k] = rs.heap_ts ? rs.heap_ts[h] : 0ULL;
    });
}

// Growth: every entry of the old regions re-inserted into regions of twice the slots (a row keeps
// its region: the region is its bucket). One workgroup per old region.
static __global__ void k_rehash(const RowEnt *__restrict__ old_ent, uint32_t old_log2S, RowStore rs) {
    const uint32_t b = blockIdx.x;
    const uint32_t S = 1u << old_log2S;
    for (uint32_t s = threadIdx.x; s < S; s += blockDim.x) {
        const RowEnt re = old_ent[((size_t)b << old_log2S) + s];
        if (re.tag == 0) continue;
        rs_insert(rs, b, re.pk, re.tag - 1, re.heap, re.bits);
    }
}

}  // namespace corro

#include "ovf_kernels.h"
