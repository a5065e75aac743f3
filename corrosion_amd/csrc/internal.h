// Internal declarations shared by the libcorro_hip.so translation units.
#pragma once
#include <hip/hip_runtime.h>

#include <array>
#include <cstdint>
#include <cstdlib>
#include <map>
#include <string>
#include <unordered_map>
#include <vector>

#include "corro_hip.h"

namespace corro {

// Failure injection for the atomicity / multi-rank failure tests: CORRO_FAULT names the steps that fail
// (comma-separated; read on every call, so a test arms and disarms it around one call).
inline bool fault_armed(const char *name) {
    const char *e = std::getenv("CORRO_FAULT");
    if (!e || !*e) return false;
    const std::string s = std::string(",") + e + ",";
    return s.find(std::string(",") + name + ",") != std::string::npos;
}

// Thread-local last error (corro_last_error).
void set_error(const std::string &msg);
int fail(int code, const std::string &msg);

#define CORRO_HIP_TRY(expr)                                                              \
    do {                                                                                 \
        hipError_t e_ = (expr);                                                          \
        if (e_ != hipSuccess)                                                            \
            return ::corro::fail(CORRO_E_DEVICE, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)

// One staged / state record: a column change or a clock row (64 B, 16-B aligned so a lane moves
// it with four dwordx4 accesses). `pos` orders records of one row: prior-state rows use their
// index inside the bucket's state slice (< 2^31), batch changes use BATCH_POS | batch index.
struct __attribute__((aligned(16))) Rec {
    uint64_t pk;
    int64_t cv;    // col_version (sentinel: causal length)
    int64_t dbv;   // db_version
    uint64_t v0;   // value word 0
    uint64_t v1;   // value word 1 (TEXT/BLOB bytes 8..15)
    uint32_t tcid; // table << 16 | cid
    uint32_t cl;   // change: causal length; state row: row causal length
    uint32_t seq;
    uint32_t site; // site ordinal
    uint32_t pos;
    uint32_t meta; // type | len << 8
};
static_assert(sizeof(Rec) == 64, "Rec must be 64 bytes");

constexpr uint32_t BATCH_POS = 0x80000000u;

// Growable device buffer.
struct DevBuf {
    void *p = nullptr;
    size_t bytes = 0;
    int ensure(size_t want);
    void release();
    template <class T> T *as() const { return static_cast<T *>(p); }
};

// Pointers into corro_ctx::d_xidx (extract.hip): the (site, db_version, seq) index of the state.
struct XIdxPtrs {
    uint64_t *hkey = nullptr;
    uint32_t *seq = nullptr, *ref = nullptr, *gid = nullptr, *gstart = nullptr, *glast = nullptr;
    uint64_t *gts = nullptr;
    Rec *crec = nullptr;         // clock rows in index order (clustered copy)
    uint64_t *cts = nullptr;     // their ts (when the state tracks ts)
};

// The state as dense clock records in pseudo-buckets (engine.hip state_dense_view).
struct DenseView {
    const Rec *st;
    const uint64_t *ts;
    const uint64_t *off;
    const uint32_t *cnt;
    uint32_t nb;
};

struct Table {
    std::string name;
    std::vector<std::string> cols;
};

// Row keys of one table's primary keys (pkeys.hip): interned tables key rows by a dense id of the
// canonical packed pk (cr-sqlite's __crsql_key / <t>__crsql_pks), others by the INTEGER pk itself.
// The intern table lives on the device (authoritative since round 5): canonical bytes of ids [0, n)
// at d_bytes[d_off[id], d_off[id + 1]), their route hashes, and open-addressing slots
// (tag << 32 | id; 0 = empty) that k_pk_probe claims with one 64-bit CAS.
struct PkTable {
    bool interned = false;
    DevBuf d_off, d_bytes, d_hash, d_slots;
    uint64_t n = 0, nbytes = 0;             // keys, arena bytes
    uint64_t cap_off = 0, cap_bytes = 0;    // capacities of d_off / d_hash (keys) and d_bytes
    uint64_t nslots = 0;                    // a multiple of 8 (0: no table yet)
    uint64_t max_len = 0;                   // bound on the longest canonical key
};
// Device view of one table's interned keys (partition.hip routes and ships interned pks by them).
struct PkDir {
    const uint64_t *off;
    const uint8_t *bytes;
    const uint64_t *hash;
    uint64_t n;
    uint32_t interned;
    uint32_t pad;
};
uint64_t pk_route_hash(const std::string &canon);
// Upload the directory of every table's intern arrays (ctx->d_pkdir).
int pk_mirror_sync(corro_ctx *ctx);
// Row keys of packed pks on the device (pkeys.hip): for every change i with (tcid[i] >> 16) == table and
// a reference (ref[i] != none: bytes at base + (ref >> len_bits), length ref & (2^len_bits - 1); or with
// off != null: bytes [off[i], off[i + 1]) of base), keys[i] = the row key -- the INTEGER pk of a table
// not interned, else the interned id (new canonical keys get the next ids in first-seen order: by the
// index of the first change of each new key, as cr-sqlite numbers __crsql_key rows in insertion order).
// bad (optional, n bytes): 1 for a malformed encoding, a reference past `limit` bytes of base, or a
// non-INTEGER pk of a table not interned (keys[i] untouched); *nbad = their count. All pointers device
// memory; synchronous. A failed call leaves the table as it was (its claims are dropped).
struct PkRefs {
    const uint8_t *base = nullptr;
    const uint64_t *ref = nullptr;
    const uint64_t *off = nullptr;
    uint64_t none = 0;
    uint32_t len_bits = 32;
    const uint32_t *tcid = nullptr;  // null: every change is of `table`
    uint64_t limit = ~0ULL;          // bytes readable from base: a reference past it is a bad pk
};
int pk_keys_device(corro_ctx *ctx, uint32_t table, const PkRefs &r, uint64_t n, uint64_t *keys, uint8_t *bad,
                   uint64_t *nbad);
bool pk_canonical(const uint8_t *p, uint64_t len, std::string &out, bool *single_int, int64_t *ival);
std::string pack_int_pk(int64_t v);

// the rocPRIM kernels' first-use cost paid once per process and device (prims.hip)
int prims_warm(corro_ctx *ctx);
// the agent's pinned host areas for a call of `ncs` changesets (agent_dev.hip), ahead of the first call
int agent_dev_reserve(corro_ctx *ctx, uint64_t ncs);

}  // namespace corro

struct corro_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    std::vector<corro::Table> tables;
    std::vector<corro::PkTable> pk;  // per table
    std::map<std::string, uint32_t> table_index;

    // sites (crsql_site_id analogue): ordinal -> 16 bytes; rank = memcmp order
    std::vector<std::array<uint8_t, 16>> sites;
    std::map<std::array<uint8_t, 16>, uint32_t> site_ordinal;
    corro::DevBuf d_site_rank;   // u32 per ordinal
    corro::DevBuf d_dbv;         // u64 per ordinal: max db_version + 1 (0 = never seen)
    corro::DevBuf d_dbv_batch;   // per-batch staging of the above
    size_t dbv_cap = 0;

    // bucket layout
    uint32_t log2B = 0;
    uint32_t B = 0;
    // state: the row store (rowstore.h), updated in place by every apply
    corro::DevBuf d_ent;          // RowEnt[B << log2S]
    corro::DevBuf d_used, d_gen;  // u32[B]: region fill, region holds a sentinel row
    corro::DevBuf d_heap, d_heap_ts;
    corro::DevBuf d_heap_top;     // u64 records handed out
    corro::DevBuf d_stride;       // u16 per table: ncols + 1
    uint32_t log2S = 0;
    uint64_t heap_cap = 0;        // records
    uint32_t max_stride = 1;
    uint64_t state_total = 0;     // clock records in the state
    uint64_t state_rows = 0;      // rows (region entries) in the state
    corro_metrics metrics{};      // cumulative counters (corro_ctx_metrics)
    std::vector<uint64_t> committed;  // per table: changes committed by corro_process_multiple_changes
    bool track_ts = false;
    // rows addressed by the applies since the last corro_state_export_touched (or reset): an
    // append-only list of (pk, table) written by the merge bodies, deduplicated at export
    bool track_touched = false;
    corro::DevBuf d_touch, d_touch_n, d_touch_stamp, d_touch_tmp;
    uint64_t touch_cap = 0;       // entries d_touch holds
    uint64_t touch_bound = 0;     // upper bound of the entries written so far (changes applied)
    uint32_t touch_epoch = 0;     // stamp of the current export (dedup per region entry)
    uint64_t touch_stamp_n = 0;   // entries d_touch_stamp covers
    // a failure after an apply's first merge write leaves the state part-merged: every later
    // call on the context fails until corro_state_reset (corro_hip.h "Failure atomicity")
    bool poisoned = false;
    uint64_t dbv_writes = 0;      // crsql_set_db_version passes run (a late agent failure after one poisons)
    // position mode of the next apply (set by the agent around one corro_apply_batch call on its
    // arrival-order input, agent_dev.hip): application position per input change, input index per
    // position, per-position ts, applied count
    const uint32_t *pm_ap = nullptr, *pm_src = nullptr;
    const uint64_t *pm_ts = nullptr;
    uint64_t pm_n = 0;
    bool pm_slack = false;  // corro_apply_mapped: a slot layout's padding may pass the chunk size
    // slot mode of the next apply (corro_apply_slots): the received slots merged where they lie
    const void *slot_rec = nullptr;
    const uint64_t *slot_cnt = nullptr;
    uint32_t slot_cap = 0, slot_nsrc = 0;
    uint32_t *slot_over = nullptr;
    bool apply_wrote = false;     // the current apply has launched its first merge kernel
    uint64_t heap_limit = 0;      // corro_ctx_set_store_limit (0: none)
    bool state_wide = false;      // some clock row holds a non-INTEGER value
    corro::DevBuf d_defer, d_relist;  // deferred buckets of a merge round, the re-merge list
    corro::DevBuf d_dense, d_dense_ts, d_dense_view;  // materialised state (extraction), its pseudo-buckets
    corro::DevBuf d_arena;        // long TEXT/BLOB value bytes (append-only; handles point into it)
    uint64_t arena_top = 0;       // bytes in use
    uint64_t dense_epoch = ~0ULL;

    // per-batch scratch
    corro::DevBuf d_in;           // staged device copy of a host batch
    corro::DevBuf d_hist;         // ntiles x B
    corro::DevBuf d_new_cnt, d_stage_off, d_bflags;
    corro::DevBuf d_stage;        // staged Recs
    corro::DevBuf d_misc;         // counters (merge_kernels.h MISC_*)
    corro::DevBuf d_ovf_list;     // overflow buckets
    corro::DevBuf d_gen_list;     // buckets queued for the general body
    corro::DevBuf d_wide_list;    // buckets queued for the mixed-type fast body
    corro::DevBuf d_fast_of;      // k_triage: per merged bucket, 1 = INTEGER fast body
    corro::DevBuf d_ovf_sort;     // overflow path: its device-wide arrays, offsets, rocPRIM temp
    corro::DevBuf d_ovf_rcl;      // overflow path, impact form of the row reduction: per-row cl slots
    corro::DevBuf d_ovf_sum;      // overflow path, fused plain form: row summaries by owner record (zero between applies)
    bool ovf_sum_dirty = false;   // d_ovf_sum may hold words of an apply that failed before its walk cleared them
    corro::DevBuf d_ovf_plan;     // overflow path: bucket offsets, row-table slices, totals (k_ovf_plan)
    uint64_t ovf_temp_k = 0;      // overflow path: the record count its cached rocPRIM temp size was queried for
    size_t ovf_temp = 0;
    corro::DevBuf d_setdbv;       // set_db_versions: (site, version + 1) pairs
    corro::DevBuf d_scan_tmp;     // corro_scan_offsets: rocPRIM temp
    corro::DevBuf d_impact;
    corro::DevBuf d_pm_ts;        // position mode: the input's per-change ts in application order (k_ts_by_pos)
    corro::DevBuf d_export;
    corro::DevBuf d_needs;        // sync-need scratch
    corro::DevBuf d_needs1;       // one-pass need diff: look-back status words + ticket
    corro::DevBuf d_xidx;         // changeset extraction: state index + its build scratch
    corro::DevBuf d_xout;         // changeset extraction: staged needs / outputs
    corro::XIdxPtrs x;
    uint64_t state_epoch = 0;     // bumped by every state change (apply, reset)
    uint64_t xidx_epoch = ~0ULL;  // epoch the extraction index was built for
    uint32_t x_db = 1, x_groups = 0;
    uint64_t x_max_dbv = 0;
    corro::DevBuf d_wire;         // wire decode: frame bytes, headers, staged outputs
    corro::DevBuf d_wire_schema;  // wire decode: table / column names
    corro::DevBuf d_wire_sites;   // wire decode: hash of the registered site ids
    corro::DevBuf d_wire_map;     // wire decode: kept-frame index map (cs_dev output)
    bool wire_schema_ready = false;
    const uint8_t *wire_names = nullptr;
    const uint32_t *wire_toff = nullptr, *wire_tlen = nullptr, *wire_tbase = nullptr, *wire_tn = nullptr,
                   *wire_coff = nullptr, *wire_clen = nullptr;
    size_t wire_sites_n = 0;
    uint32_t wire_hmask = 0;
    corro::DevBuf d_ncols;        // u16 column count per table
    std::vector<uint8_t> aff;     // column affinity per (table, cid), (MAX_COLS + 1) per table
    corro::DevBuf d_aff, d_affflag;
    corro::DevBuf d_aff_conv, d_aff_vals;
    corro::DevBuf d_gaps_big;              // corro_booked_insert_db_batch: counter + long-actor list  // per change of a batch: converted flag; cv0 | cv1 | cmeta
    bool aff_any = false;         // some column has an affinity other than BLOB
    int aff_policy = CORRO_AFF_POLICY_SQLITE_3_37_2;  // corro_set_affinity_policy (never refuse by default)
    corro::DevBuf d_part;         // partition counts
    corro::DevBuf d_pkdir;        // PkDir per table (pk_mirror_sync)
    corro::DevBuf d_pk_scratch;   // pk_keys_device: per-change columns, staged host inputs, rocPRIM temp
    corro::DevBuf d_pk_bad;       // wire decode: per change, a malformed interned pk
    corro::DevBuf d_part_var;     // partition_var scratch: per-record var lengths / offsets, perm
    // process_multiple_changes on the device (agent_dev.hip): staged host input, gathered batch,
    // span tables, impact flags, impactful output, and a pinned host staging area
    corro::DevBuf d_agent_in, d_agent_batch, d_agent_spans, d_agent_imp, d_agent_out, d_agent_aux;
    corro::DevBuf d_agent_fetch, d_agent_aux2;
    corro::DevBuf d_agent_hdr;    // device-header mode: per-changeset / per-site / run columns
    bool agent_sorted_mode = false;  // spans compacted from the site-rank sort (s_cs in the val column)
    // position mode: input index of every application position, bit 31 = the first position of its
    // span (k_span_pos; null when the call's batch is not in position mode)
    const uint32_t *agent_src_of = nullptr;
    void *h_agent = nullptr;
    size_t h_agent_bytes = 0;
    void *h_hdr = nullptr;           // host ChangeV1 headers staged for the device header passes (pinned)
    size_t h_hdr_bytes = 0;
    void *h_hfetch = nullptr;        // the host changesets' headers read back (pinned, agent_dev_headers)
    size_t h_hfetch_bytes = 0;
    void *h_pool = nullptr;          // the buffered-row pool's copy jobs on their way up (pinned, bufpool_append)
    size_t h_pool_bytes = 0;
    corro::DevBuf d_hdr_stage;       // their device copy + the device known outcomes
    uint64_t agent_ncs = 0;       // changesets of the current call (d_agent_spans column length)
    uint64_t agent_nbatch_max = 0;  // input changes of the current call (bound on the applied batch)
    uint64_t *h_misc = nullptr;   // pinned, 16 words
    uint32_t *h_ovf = nullptr;    // pinned, 3 B + 16 words: the overflow fold's readbacks (run_overflow)
    // stage timing
    bool profiling = false;
    hipEvent_t ev[8] = {};
    float last_ms[9] = {};        // apply stages [0..5], k_needs / extract count [6], fill [7], extract index build [8]
};
