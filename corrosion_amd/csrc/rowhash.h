// Shared device-side definitions: the SoA batch view and the row hash that places a row
// (table, pk) in a merge bucket (top bits) and on an owner rank (low bits).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace corro {

// One change as the multi-GPU exchange ships it (SURVEY §8(d)'s 48 B; partition.hip PackedRec48).
struct alignas(16) SlotRec {
    uint64_t pk;
    int64_t cv, dbv;
    uint64_t v0;
    uint32_t tcid, cl, seq, site;
};

struct BatchDev {
    const uint64_t *pk;
    const uint32_t *tcid;
    const int64_t *cv;
    const int64_t *dbv;
    const uint32_t *cl;
    const uint32_t *seq;
    const uint32_t *site;
    const uint64_t *v0;
    const uint64_t *v1;
    const uint8_t *vt;
    const uint8_t *vl;
    const uint64_t *ts;
    // long TEXT/BLOB values: val_off / val_size per change; the batch's val_data was copied to
    // arena + lbase (ldata bytes) before the apply
    const uint64_t *voff;
    const uint32_t *vsz;
    const uint8_t *arena;
    uint64_t lbase, ldata;
    // column affinity (affinity.hip): conv[i] = 1 when change i's stored value is its converted
    // value (cv0[i], cv1[i], cmeta[i] = type | len << 8); null when no value of the batch converts
    const uint8_t *conv;
    const uint64_t *cv0, *cv1;
    const uint32_t *cmeta;
    // position mode (the agent's batch in arrival order): ap[i] = change i's application position,
    // AP_SKIP for a change that is not applied; null: position i
    const uint32_t *ap;
    uint32_t n;
    uint32_t ap_all;  // position mode with every change applied: the histogram need not read ap
    // ts_v1 (INTEGER-only batches, k_scatter<PLAIN>): every staged record carries its change's ts in
    // its v1 word (unused by INTEGER values), so the merge reads a winner's ts from the record it
    // already holds instead of a random load from a per-position array. ts_pos: ts is indexed by
    // application position (ap), else by input index. (ts_v1 bit 1: ts is 16-B aligned, paired loads)
    uint32_t ts_v1, ts_pos;
    // slot mode (corro_apply_slots: the receiver of the stream-ordered exchange merges the received
    // 48-B records where they lie): change i is slot_rec[i], applied at position i when its source's
    // slot holds it (i % cap < slot_cnt[i / cap]) and no source overflowed its slot; the SoA arrays
    // above are not read. k_hist reports an overflow in *slot_over. A batch larger than one apply
    // chunk is applied as consecutive index ranges of the slot layout: slot_rec then points at the
    // chunk's first record, whose index in the whole layout is slot_base.
    const SlotRec *slot_rec;
    const uint64_t *slot_cnt;
    uint32_t slot_cap, slot_nsrc;
    uint32_t *slot_over;
    uint32_t slot_base;
};

// slot mode: does any source's count pass the slot (every record is then skipped)?
__device__ inline bool slot_overflowed(const BatchDev &in) {
    bool over = false;
    for (uint32_t s = 0; s < in.slot_nsrc; s++) over |= in.slot_cnt[s] > in.slot_cap;
    return over;
}
__device__ inline bool slot_valid(const BatchDev &in, uint32_t i, bool over) {  // (i: index in the chunk)
    const uint32_t g = in.slot_base + i, s = g / in.slot_cap;
    return !over && s < in.slot_nsrc && (uint64_t)(g - s * in.slot_cap) < in.slot_cnt[s];
}
constexpr uint32_t AP_SKIP = 0xFFFFFFFFu;

__host__ __device__ inline uint64_t mix64(uint64_t x) {
    x ^= x >> 33;
    x *= 0xff51afd7ed558ccdULL;
    x ^= x >> 33;
    x *= 0xc4ceb9fe1a85ec53ULL;
    x ^= x >> 33;
    return x;
}

// Bucket of a row (table, pk): the top log2B bits of a 64-bit mix. Rows never straddle buckets, so
// every causal-length interaction of a row (delete/resurrect zeroing) stays inside one workgroup.
__host__ __device__ inline uint32_t bucket_of(uint32_t table, uint64_t pk, uint32_t log2B) {
    if (log2B == 0) return 0;
    uint64_t h = mix64(pk + 0x9E3779B97F4A7C15ULL * (uint64_t)(table + 1));
    return (uint32_t)(h >> (64 - log2B));
}

}  // namespace corro
