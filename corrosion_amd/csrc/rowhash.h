// Shared device-side definitions: the SoA batch view and the row hash that places a row
// (table, pk) in a merge bucket (top bits) and on an owner rank (low bits).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace corro {

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
};
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
