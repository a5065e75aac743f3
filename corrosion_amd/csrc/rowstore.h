// The merged state: cr-sqlite's per-table clock tables (`<t>__crsql_clock(key, col_name, col_version,
// db_version, site_id, seq, ts)`) as a device row store that an apply updates IN PLACE,
// so an apply costs what its batch touches, not what the state holds (cr-sqlite's per-change INSERT
// touches only the batch's rows: /root/reference/crates/corro-agent/src/agent/util.rs:1222-1262).
//
//   rows    B regions (one per merge bucket: a row's region is its bucket, so the workgroup that
//           merges a bucket owns its region outright) of S RowEnt slots, open addressing with
//           linear probing inside the region; rows are never removed (a deleted row keeps its
//           sentinel clock), so a row is always found before the first empty slot of its probe.
//   heap    one fixed-width slot per row: (ncols + 1) 64-B clock records, the sentinel clock at
//           slot 0 and the cell of cid c at slot c; `bits` says which are present. A record's
//           `pos` field holds its own heap index (the key of its ts in heap_ts).
//
// Growth never runs inside an apply's writes: a bucket whose region or the heap cannot take its new
// rows is DEFERRED before it writes anything; the host then grows the store (regions rehashed to
// twice the slots / heap doubled) and merges the deferred buckets again.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "internal.h"
#include "rowhash.h"

namespace corro {

struct __attribute__((aligned(16))) RowEnt {
    uint64_t pk;
    uint32_t tag;      // 0 empty, else table + 1
    uint32_t heap;     // heap record index of the row's slot 0
    uint64_t bits[2];  // bit 0: sentinel clock present; bit c: clock of cid c present (c < 128)
};
static_assert(sizeof(RowEnt) == 32, "RowEnt must be 32 bytes");
constexpr uint32_t ROW_NONE = 0xFFFFFFFFu;
constexpr uint32_t MAX_COLS = 127;  // cids 1..127 fit the presence bits

struct RowStore {
    RowEnt *ent;                    // B * S
    uint32_t *used;                 // B: entries in use per region
    uint32_t *gen;                  // B: 1 once a row of the region holds a sentinel clock
    Rec *heap;
    uint64_t *heap_ts;              // null until the state tracks ts
    unsigned long long *heap_top;   // records handed out
    unsigned long long heap_cap;    // records
    uint32_t log2S;
    uint32_t fill;                  // max entries per region (S * 7 / 8)
    const uint16_t *stride;         // per table: ncols + 1
};

__host__ __device__ inline uint32_t region_slot(uint64_t pk, uint32_t table, uint32_t log2S) {
    // a different mix than bucket_of's (whose top bits pick the region) and rank_of's (low bits)
    const uint64_t h = mix64(pk * 0xA0761D6478BD642FULL + table + 0x51);
    return (uint32_t)(h >> 40) & ((1u << log2S) - 1u);
}

__device__ inline uint32_t row_popc(const uint64_t bits[2]) { return __popcll(bits[0]) + __popcll(bits[1]); }

// Read-only probe of region b (no insert may run concurrently in this region). Returns the entry's
// global index or ROW_NONE.
__device__ inline uint32_t rs_lookup(const RowStore &rs, uint32_t b, uint64_t pk, uint32_t table) {
    const uint32_t S = 1u << rs.log2S, m = S - 1;
    const RowEnt *reg = rs.ent + ((size_t)b << rs.log2S);
    uint32_t s = region_slot(pk, table, rs.log2S);
    for (uint32_t k = 0; k < S; k++, s = (s + 1) & m) {
        const uint32_t tag = reg[s].tag;
        if (tag == 0) return ROW_NONE;
        if (tag == table + 1 && reg[s].pk == pk) return (b << rs.log2S) | s;
    }
    return ROW_NONE;
}

// rs_lookup that also reports the first empty slot its probe met (the slot a new row of this key
// claims first), as a local slot index.
__device__ inline uint32_t rs_probe(const RowStore &rs, uint32_t b, uint64_t pk, uint32_t table, uint32_t &empty) {
    const uint32_t S = 1u << rs.log2S, m = S - 1;
    const RowEnt *reg = rs.ent + ((size_t)b << rs.log2S);
    uint32_t s = region_slot(pk, table, rs.log2S);
    for (uint32_t k = 0; k < S; k++, s = (s + 1) & m) {
        const uint32_t tag = reg[s].tag;
        if (tag == 0) {
            empty = s;
            return ROW_NONE;
        }
        if (tag == table + 1 && reg[s].pk == pk) return (b << rs.log2S) | s;
    }
    empty = region_slot(pk, table, rs.log2S);
    return ROW_NONE;
}

// rs_insert from a slot known to have been empty at the probe (one CAS when no other new row of
// the workgroup took it); the entry's presence bits start at zero.
__device__ inline uint32_t rs_claim(const RowStore &rs, uint32_t b, uint32_t s, uint64_t pk, uint32_t table,
                                    uint32_t heap) {
    const uint32_t m = (1u << rs.log2S) - 1;
    RowEnt *reg = rs.ent + ((size_t)b << rs.log2S);
    while (atomicCAS(&reg[s].tag, 0u, table + 1) != 0u) s = (s + 1) & m;
    reg[s].pk = pk;
    reg[s].heap = heap;
    reg[s].bits[0] = 0;
    reg[s].bits[1] = 0;
    return (b << rs.log2S) | s;
}

// Claim an empty slot of region b for a row known to be absent. Inserters race each other only for
// empty slots (one CAS on the tag); nothing looks a new row's slot up while it is written: a lookup
// runs only for rows that existed when the apply began, and such a row's probe path (its home slot up
// to its own) held no empty slot then (rows are never removed), so it never meets a slot claimed
// now. Hence plain stores, and no fences: the entry is read by later kernels. The caller has checked
// the region's fill, so an empty slot exists.
__device__ inline uint32_t rs_insert(const RowStore &rs, uint32_t b, uint64_t pk, uint32_t table, uint32_t heap,
                                     const uint64_t bits[2]) {
    const uint32_t m = (1u << rs.log2S) - 1;
    RowEnt *reg = rs.ent + ((size_t)b << rs.log2S);
    uint32_t s = region_slot(pk, table, rs.log2S);
    while (true) {
        if (__hip_atomic_load(&reg[s].tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0 &&
            atomicCAS(&reg[s].tag, 0u, table + 1) == 0u)
            break;
        s = (s + 1) & m;
    }
    reg[s].pk = pk;
    reg[s].heap = heap;
    reg[s].bits[0] = bits[0];
    reg[s].bits[1] = bits[1];
    return (b << rs.log2S) | s;
}

// Heap records for a workgroup's new rows, or ~0 when the heap cannot hold them (the bucket defers).
// One atomicAdd per workgroup, never undone: the records a failed request counted stay unused, so
// every successful range is disjoint and below the capacity; the host grows the heap past the top.
__device__ inline unsigned long long rs_heap_alloc(const RowStore &rs, unsigned long long need) {
    const unsigned long long old = atomicAdd(rs.heap_top, need);
    if (old + need <= rs.heap_cap) return old;
    // a failed request gives its records back, so the top the host grows from (and later requests
    // of this round) do not carry it (a concurrent request may still see the transient excess and
    // defer: harmless, it merges after the growth)
    atomicSub(rs.heap_top, need);
    return ~0ULL;
}

}  // namespace corro
