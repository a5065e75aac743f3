/*
 * corro_hip.h — C ABI of the MI355X batched CRDT merge engine (libcorro_hip.so).
 *
 * This is the boundary a `corro-hip` Rust crate binds (see INTEGRATION.md for the `extern "C"`
 * block). It replaces, for corrosion's apply hot path, the per-change SQL loop
 *     for change in changes { INSERT INTO crsql_changes (...); SELECT crsql_rows_impacted(); }
 * in process_complete_version (/root/reference/crates/corro-agent/src/agent/util.rs:1222-1262),
 * i.e. cr-sqlite's `crsql_changes` xUpdate merge (prebuilt crsqlite-linux-x86_64.so, entry
 * `sqlite3_crsqlite_init`, loaded at corro-types/src/sqlite.rs:121-139), plus the sync
 * bookkeeping arithmetic of corro-types (SyncStateV1::compute_available_needs, sync.rs:127-249;
 * VersionsSnapshot::compute_gaps_change/insert_db, agent.rs:1108-1235).
 *
 * Conventions
 *   - Every function returns an int status: CORRO_OK (0) or a negative corro_status.
 *     corro_last_error() returns a NUL-terminated description of the last failure on the
 *     calling thread.
 *   - All pointers are plain host (or, where `mem` says so, device) pointers; sizes are counts of
 *     elements. No callbacks; no ownership transfer: the caller owns every buffer it passes.
 *   - A context is thread-compatible, not thread-safe: one context per writer, mirroring the
 *     single SQLite writer of the reference (corro-types/src/agent.rs:480-482, setup.rs:97).
 *   - The library never falls back to a CPU path: without a usable gfx950 device every compute
 *     entry point fails with CORRO_E_NO_DEVICE.
 */
#ifndef CORRO_HIP_H
#define CORRO_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CORRO_HIP_ABI_VERSION 3

typedef enum {
    CORRO_OK = 0,
    CORRO_E_INVALID = -1,        /* bad argument / malformed input */
    CORRO_E_NOMEM = -2,          /* host or device allocation failed */
    CORRO_E_DEVICE = -3,         /* HIP runtime error */
    CORRO_E_UNKNOWN_TABLE = -4,  /* "no such table" (the INSERT would fail: util.rs:839-860) */
    CORRO_E_UNKNOWN_COLUMN = -5, /* unknown cid: cr-sqlite raises "SQL logic error" */
    CORRO_E_RANGE = -6,          /* value outside the engine's fixed-width encoding */
    CORRO_E_NO_DEVICE = -7       /* no HIP device visible */
} corro_status;

/* SQLite storage classes, numbered like corro-api-types ColumnType (lib.rs:300-307) */
enum { CORRO_INTEGER = 1, CORRO_REAL = 2, CORRO_TEXT = 3, CORRO_BLOB = 4, CORRO_NULL = 5 };

/* Where a batch's arrays live */
enum { CORRO_MEM_HOST = 0, CORRO_MEM_DEVICE = 1 };
/* corro_process_multiple_changes only: like CORRO_MEM_DEVICE, and the changeset headers and
 * out->known live on the device too (a decoder's device output); cs[i].actor_id is not read. */
enum { CORRO_MEM_DEVICE_HEADERS = 2 };

typedef struct corro_ctx corro_ctx;

/* One CRR table: its name and non-pk column names. cid k (1-based) = col_names[k-1];
 * cid 0 is cr-sqlite's row sentinel "-1" (corro-api-types/src/lib.rs:748-751). */
typedef struct {
    const char *name;
    uint32_t ncols;
    const char *const *col_names;
} corro_table_desc;

/*
 * A batch of column changes (corro-types/src/change.rs:19-30 `Change`), struct-of-arrays,
 * application order = index order: actors ascending by 16-byte id, changesets in arrival
 * order, changes in vector order (util.rs:705,765,782,1222). Required arrays: pk, table_cid,
 * col_version, db_version, cl, seq, site, val0. Optional (NULL): val1, val_type, val_len, ts.
 *
 *   pk          row key: the table's single INTEGER pk value, or for an interned table the key
 *               corro_pk_keys gives its packed pk bytes (pubsub.rs:2304-2358), like cr-sqlite's
 *               `__crsql_key`
 *   table_cid   (table_index << 16) | cid, cid 0 = sentinel "-1"
 *   cl          causal length (< 2^32); sentinel changes and even-cl changes need
 *               0 <= col_version < 2^32 (their col_version becomes the row's causal length)
 *   seq         CrsqlSeq (< 2^32)
 *   site        site ordinal from corro_site_register (crsql_site_id.ordinal analogue)
 *   val0/val1   INTEGER: i64 bits in val0. REAL: f64 bits in val0 (NaN not allowed).
 *               TEXT/BLOB (<= 16 bytes): bytes 0..7 / 8..15 big-endian, zero padded.
 *   val_type    CORRO_* storage class (NULL array = all INTEGER)
 *   val_len     TEXT/BLOB byte length, or CORRO_VAL_LONG for a value longer than 16 bytes
 *   ts          changeset timestamp (NTP64), bound per change as in util.rs:1244
 *   val_off / val_size / val_data / val_data_len
 *               TEXT/BLOB values of any length (SqliteValue::Text(String) / Blob(Vec<u8>),
 *               corro-api-types/src/lib.rs:419-429): a change with val_len == CORRO_VAL_LONG has its
 *               bytes at val_data[val_off[i], val_off[i] + val_size[i]), 16 < val_size < 2^24
 *               (val0/val1 are not read for it). val_data holds val_data_len bytes in the batch's
 *               memory; val_off/val_size are read only for long values (other entries are
 *               ignored). All NULL/0 when the batch has no long value. The engine keeps the bytes
 *               in a device value arena; exported rows carry val_len == CORRO_VAL_LONG, val0 = bytes
 *               0..7 big-endian and val1 = a value handle that corro_value_bytes resolves.
 */
#define CORRO_VAL_LONG 255
typedef struct {
    uint64_t n;
    const uint64_t *pk;
    const uint32_t *table_cid;
    const int64_t *col_version;
    const int64_t *db_version;
    const uint32_t *cl;
    const uint32_t *seq;
    const uint32_t *site;
    const uint64_t *val0;
    const uint64_t *val1;
    const uint8_t *val_type;
    const uint8_t *val_len;
    const uint64_t *ts;
    const uint64_t *val_off;
    const uint32_t *val_size;
    const uint8_t *val_data;
    uint64_t val_data_len;
} corro_changes;

/* Per-batch outputs (all optional, host pointers, n elements each) */
typedef struct {
    /* crsql_rows_impacted() growth caused by each change (0, 1 or 2), util.rs:1246-1260; NULL =
     * not wanted. Host memory for a CORRO_MEM_HOST batch, device memory for CORRO_MEM_DEVICE. */
    uint8_t *impact;
} corro_apply_out;

/* crsql_changes read-back rows (table, pk, cid, val, col_version, db_version, site_id, cl, seq, ts) */
typedef struct {
    uint64_t *pk;
    uint32_t *table_cid;
    int64_t *col_version;
    int64_t *db_version;
    int64_t *cl;
    uint32_t *seq;
    uint32_t *site;
    uint64_t *ts;
    uint64_t *val0;
    uint64_t *val1;
    uint8_t *val_type;
    uint8_t *val_len;
} corro_rows;

/* ------------------------------------------------------------------ context */

const char *corro_last_error(void);
int corro_abi_version(void);
/* number of visible HIP devices (0 if none); does not initialise a context */
int corro_device_count(int *count);

/* Create an engine bound to a schema. `capacity_hint` = expected clock rows + changes per
 * apply (sizes the bucket table); `device` = HIP ordinal. Mirrors CrConn::init + apply_schema. */
int corro_ctx_create(const corro_table_desc *tables, uint32_t ntables, uint64_t capacity_hint,
                     int device, corro_ctx **out);
void corro_ctx_destroy(corro_ctx *ctx);

/* Resolve Change.table / Change.cid strings. Unknown names -> CORRO_E_UNKNOWN_TABLE/_COLUMN. */
int corro_lookup_cid(corro_ctx *ctx, const char *table, const char *cid, uint32_t *table_cid);

/* Register 16-byte site ids (ActorId bytes), returning stable ordinals (existing ids keep theirs).
 * The engine orders sites by memcmp of the bytes for the merge-equal-values tie-break. */
int corro_site_register(corro_ctx *ctx, const uint8_t *site_ids, uint64_t n, uint32_t *ordinals);
int corro_site_count(corro_ctx *ctx, uint32_t *count);
/* The registered 16-byte site ids by ordinal (at most cap written; *count = all). */
int corro_site_ids(corro_ctx *ctx, uint8_t *ids, uint32_t cap, uint32_t *count);

/* ------------------------------------------------------------------ primary keys */

/* A Change's pk is pack_columns bytes (corro-types/src/pubsub.rs:2304-2358). A table whose primary
 * key is one INTEGER column keys its rows by that integer (the default). Any other table (a BLOB,
 * TEXT, REAL or composite primary key -- corro-tests' testsblob and wide, corro-tests/src/lib.rs:13-53)
 * is marked interned before its first change: its rows are keyed by a dense id per table, handed out
 * in first-seen order for the CANONICAL packed bytes (unpacked and re-packed as pack_columns packs,
 * so non-canonical encodings of one key name one row, as cr-sqlite's __crsql_key does). */
int corro_table_set_pk_interned(corro_ctx *ctx, uint32_t table, int interned);
/* The canonical form of one packed pk (no context, no device): unpack_columns then pack_columns. */
int corro_pk_canonical(const uint8_t *bytes, uint64_t len, uint8_t *out, uint64_t cap, uint64_t *out_len);
/* n packed pks of `table` -> row keys (the corro_changes.pk values): pk i = bytes[off[i], off[i+1]).
 * CORRO_E_INVALID for a malformed encoding, CORRO_E_RANGE for a non-INTEGER pk of a table not interned. */
int corro_pk_keys(corro_ctx *ctx, uint32_t table, const uint8_t *bytes, const uint64_t *off, uint64_t n,
                  uint64_t *keys);
/* The same with bytes, off (n + 1) and keys in device memory (a decoder that leaves packed pks in HBM):
 * the intern table is an open-addressing table in HBM, so no pk crosses PCIe. Ids are dense per table
 * and persist across calls (a new key's id is the table's size at the call plus its rank among the
 * call's new keys, in no particular order). Synchronous. */
int corro_pk_keys_device(corro_ctx *ctx, uint32_t table, const uint8_t *bytes, const uint64_t *off, uint64_t n,
                         uint64_t *keys);
/* Row keys of `table` -> canonical packed pk bytes (export, extraction): key i's bytes at
 * [out_off[i], out_off[i+1]); out_off holds n + 1 entries; CORRO_E_RANGE if cap < out_off[n]. */
int corro_pk_bytes(corro_ctx *ctx, uint32_t table, const uint64_t *keys, uint64_t n, uint8_t *bytes, uint64_t cap,
                   uint64_t *out_off);

/* ------------------------------------------------------------------ column affinity */

/* SQLite column affinity. cr-sqlite stores a winning value through the base table,
 * whose column affinity may convert it; the next change is then compared unconverted against the
 * converted value. The engine does the same: a change's value is stored as its column's affinity
 * converts it (SQLite 3.37.2's applyAffinity, its x87 long-double decimal scaling emulated bit for
 * bit: INTEGER -> TEXT '5', REAL -0.0 -> INTEGER 0, INTEGER 5 -> REAL 5.0, numeric TEXT -> number,
 * REAL -> "%!.15g" TEXT), exported rows carry the stored value, and an incoming change is compared
 * by its raw value against the stored one. Without a registered affinity a column is BLOB (no
 * conversion). */
enum { CORRO_AFF_BLOB = 0, CORRO_AFF_TEXT = 1, CORRO_AFF_NUMERIC = 2, CORRO_AFF_INTEGER = 3, CORRO_AFF_REAL = 4 };
/* sqlite3AffinityType of a declared column type (schema.rs's column type names): INT -> INTEGER,
 * CHAR/CLOB/TEXT -> TEXT, BLOB or none -> BLOB, REAL/FLOA/DOUB -> REAL, else NUMERIC. Host only. */
int corro_affinity_of_type(const char *decl_type);
/* aff[c - 1] = affinity of cid c, ncols = the table's column count. */
int corro_table_set_affinity(corro_ctx *ctx, uint32_t table, const uint8_t *aff, uint32_t ncols);
/* Which conversions the engine performs. The reference bundles a newer SQLite (libsqlite3-sys 0.31.0,
 * Cargo.lock:2444) than the 3.37.2 whose conversion routines the engine emulates, and newer SQLite
 * rewrote TEXT -> REAL (sqlite3AtoF) and REAL -> TEXT rounding. SQLITE_3_37_2 (the default) converts
 * every value exactly as SQLite 3.37.2 does -- like SQLite, it never refuses a change -- and counts
 * the conversions whose result may differ in another SQLite version in corro_metrics.aff_sensitive.
 * PORTABLE (opt-in, strict) converts only values every correctly rounded implementation stores
 * identically and fails a batch holding any other conversion with CORRO_E_RANGE before it writes
 * (affinity.hip states the rules). */
enum { CORRO_AFF_POLICY_PORTABLE = 0, CORRO_AFF_POLICY_SQLITE_3_37_2 = 1 };
int corro_set_affinity_policy(corro_ctx *ctx, int policy);

/* ------------------------------------------------------------------ merge */

/* Merge one batch into the device state (equivalent to one INSERT INTO crsql_changes per change,
 * in index order). `mem` says where the arrays live. Synchronous: returns after the state is
 * resident and outputs are written. */
int corro_apply_batch(corro_ctx *ctx, const corro_changes *in, int mem, corro_apply_out *out);

/* Clock rows currently in the state (sentinels included). */
int corro_state_count(corro_ctx *ctx, uint64_t *count);
/* Copy the state out in crsql_changes form, unspecified row order; `cap` = capacity of `out`. */
int corro_state_export(corro_ctx *ctx, corro_rows *out, uint64_t cap, uint64_t *written);
/* Drop all merged state (keeps schema, sites and crsql_db_versions). Also clears a poisoned context. */
int corro_state_reset(corro_ctx *ctx);

/* Failure atomicity. A failing corro_apply_batch (or corro_process_multiple_changes) that fails
 * BEFORE its first merge write -- validation, unknown names, affinity, arena or scratch allocation --
 * leaves the state exactly as it was. One that fails after the merge began writing (a resource limit
 * hit while growing the row store, a device error, a later chunk of a chunked batch) cannot be undone
 * in place: the context is then POISONED and every later apply / export / extraction call fails with
 * CORRO_E_DEVICE until corro_state_reset, after which the caller re-seeds the state from its durable
 * store (the SQLite tables it persists with corro_state_export_touched).
 * corro_process_multiple_changes adds its bookkeeping after the merge: a failure there (the buffered
 * rows' pool reserve or copy, the header commit, a host allocation) also poisons the context once the
 * call's merge or any crsql_set_db_version has run; the bookie then keeps none of the call's pending
 * buffered segments and none of its Booked versions, and the caller rebuilds it with the state
 * (CORRO_FAULT=bufpool_reserve injects such a failure in tests). */

/* Per-apply delta for persistence (the writes each reference INSERT INTO crsql_changes makes to the
 * base table and clock table inside the caller's transaction, util.rs:749-758, :1225-1245). With
 * tracking on, the merge bodies list every row an apply addresses; corro_state_export_touched returns,
 * for every row listed since the previous successful call (or reset), the row's COMPLETE current clock
 * set in crsql_changes form (sentinel first, then cells by cid; rows contiguous, each row once). A
 * host replaces each exported (table, pk)'s clock rows with these (DELETE ... WHERE key = pk, then
 * INSERT) in the transaction that commits the apply: a delete drops cells, so the replacement set is
 * authoritative, and an addressed row whose clocks did not change is rewritten unchanged. The cost
 * scales with the rows addressed, not the state. cap < rows: CORRO_E_RANGE with *written = the row
 * count, the list kept for a retry. Long values: val1 handles as in corro_state_export. */
int corro_ctx_track_touched(corro_ctx *ctx, int on);
int corro_state_export_touched(corro_ctx *ctx, corro_rows *out, uint64_t cap, uint64_t *written);

/* Upper bound of the row store's heap in clock records (0 = none, the default): growth past it fails
 * with CORRO_E_NOMEM (a device-memory budget per context). */
int corro_ctx_set_store_limit(corro_ctx *ctx, uint64_t max_heap_records);
/* crsql_db_versions: per-site max db_version over every merged change, -1 = never seen. */
int corro_db_versions(corro_ctx *ctx, int64_t *out, uint32_t nsites);
/* Bytes of long values named by value handles (the val1 of exported / extracted rows whose val_len
 * is CORRO_VAL_LONG; a handle's low 24 bits are its length). Value i's bytes go to
 * bytes[out_off[i], out_off[i+1]); out_off holds n + 1 entries (host). CORRO_E_RANGE if cap <
 * out_off[n] (out_off is still filled), CORRO_E_INVALID for a handle outside the arena. Handles stay
 * valid until corro_state_reset. */
int corro_value_bytes(corro_ctx *ctx, const uint64_t *handles, uint64_t n, uint8_t *bytes, uint64_t cap,
                      uint64_t *out_off);

/* Stage timing with HIP events recorded on the engine's stream (for roofline reporting).
 * corro_last_timings returns milliseconds of the last apply per stage:
 * [0] k_hist [1] k_colscan [2] k_plan [3] k_scatter [4] k_merge [5] k_merge_ovf (0 if not run),
 * [6] / [7] the last need-diff or extraction count / fill pass, [8] the last extraction index build. */
int corro_ctx_set_profiling(corro_ctx *ctx, int on);
int corro_last_timings(corro_ctx *ctx, float *ms, uint32_t cap, uint32_t *count);

/* ------------------------------------------------------------------ metrics */

/* Cumulative counters of a context (the hot path's share of corrosion's metrics: util.rs:534,698,
 * 1032-1034,1178 -- processing started / time / chunk size / changes committed). */
typedef struct {
    uint64_t applies;          /* corro_apply_batch calls that committed */
    uint64_t changes;          /* changes merged by them (winners and losers) */
    uint64_t overflow_rounds;  /* applies that ran the device-wide overflow fold */
    uint64_t deferred_rounds;  /* merge rounds repeated after growing the row store */
    uint64_t region_growths, heap_growths;
    uint64_t state_rows, state_records;   /* now */
    uint64_t max_batch;        /* largest batch (chunk_size) */
    double apply_seconds;      /* wall time inside corro_apply_batch */
    uint64_t arena_bytes;      /* long-value arena in use: append-only (every batch's TEXT/BLOB values
                                  longer than 16 bytes, winners or not) until corro_state_reset, at most
                                  2^40 bytes (CORRO_E_RANGE beyond) */
    uint64_t aff_sensitive;    /* changes converted by a column affinity whose stored value may differ
                                  between SQLite versions (TEXT <-> REAL rounding), under
                                  CORRO_AFF_POLICY_SQLITE_3_37_2 (the default); PORTABLE refuses them */
} corro_metrics;
int corro_ctx_metrics(corro_ctx *ctx, corro_metrics *out);
/* corro.changes.committed{table}: changes of complete and partial changesets that
 * corro_process_multiple_changes / corro_process_fully_buffered committed, per table. */
int corro_table_committed(corro_ctx *ctx, uint32_t table, uint64_t *count);

/* ------------------------------------------------------------------ multi-GPU ingest */

/* Stable partition of a DEVICE-resident batch by owner rank, rank_of(table, pk) = low 32 bits of
 * the row hash mod nranks: `out` (device arrays, in->n each; optional arrays may be
 * NULL) receives the changes grouped by destination rank, each group in input order; counts[r]
 * (host) = changes for rank r. Followed by one all-to-all exchange (RCCL), receivers concatenate
 * by source rank, which preserves the application order of every row. 1 <= nranks <= 64. */
int corro_partition_ranks(corro_ctx *ctx, const corro_changes *in, uint32_t nranks, corro_changes *out,
                          uint64_t *counts);

/* The same partition as whole packed records, for ONE all-to-all of records per exchange (instead
 * of one per SoA field): `out` (device, 16-B aligned) receives in->n records grouped by destination
 * rank, each group in input order. Records are 48 B (pk, col_version, db_version,
 * val0, table_cid, cl, seq, site) when the batch has no val1/val_type/val_len/ts arrays, else 80 B
 * (every field); corro_packed_record_bytes says which. perm (optional, device, in->n) receives the
 * source index of every packed record (to return per-change results to the sender's order). */
int corro_packed_record_bytes(const corro_changes *in, uint32_t *bytes);
int corro_partition_packed(corro_ctx *ctx, const corro_changes *in, uint32_t nranks, void *out, uint32_t *perm,
                           uint64_t *counts);
/* Received records (concatenated by source rank) -> the SoA batch corro_apply_batch takes (device
 * arrays, n each; optional arrays may be NULL). rec_bytes = 48 or 80. */
int corro_unpack_records(corro_ctx *ctx, const void *recs, uint64_t n, uint32_t rec_bytes, corro_changes *out);

/* Stream-ordered form of the packed exchange (no host round trip between partition and merge):
 * destination r's 48-B records go to the fixed slot out[r * cap, r * cap + cap) (in input order,
 * records past cap are not written), and counts_dev[r] (DEVICE u64) receives the true count. Every
 * launch is queued on the context's stream (corro_ctx_stream), so an all-to-all with EQUAL splits
 * of cap records (RCCL on that stream) needs no host-side sizes. PLAIN batches only (48-B records). */
int corro_partition_slots(corro_ctx *ctx, const corro_changes *in, uint32_t nranks, uint64_t cap, void *out,
                          uint64_t *counts_dev, uint32_t *perm_dev);
/* (perm_dev, optional DEVICE u32 of nranks * cap: perm_dev[slot position] = the input index packed there,
 * for the impact flags coming back, corro_slots_flags_back.) The partition validates the records it
 * packs as corro_apply_batch would before writing (names, site ordinals, causal-length ranges,
 * db_version); a batch that fails sets bit 63 of every count, which every receiver reads as an
 * overflowed slot: nothing is applied from the slots and the exact-size exchange reports the error. */
/* Received slots (nsrc slots of cap records, src_counts_dev[s] = DEVICE count source s sent) ->
 * the SoA batch at the same indices (device, nsrc * cap each) and ap[i] = i for a received record,
 * CORRO_AP_SKIP for a slot's padding; *overflow_dev (device u32) = 1 when a source sent more than
 * cap (its records past cap are lost: every ap is then CORRO_AP_SKIP, so the apply is a no-op and
 * the caller repeats the exchange with exact sizes). Queued on the context's stream. */
#define CORRO_AP_SKIP 0xFFFFFFFFu
int corro_unpack_slots(corro_ctx *ctx, const void *recs, uint32_t nsrc, uint64_t cap, const uint64_t *src_counts_dev,
                       corro_changes *out, uint32_t *ap, uint32_t *overflow_dev);
/* corro_apply_batch over a DEVICE batch whose changes i with ap[i] == CORRO_AP_SKIP are not applied
 * (the others apply in index order): the slot layout above, merged without compacting it. */
int corro_apply_mapped(corro_ctx *ctx, const corro_changes *in, const uint32_t *ap, corro_apply_out *out);
/* The receiver's merge without the unpack: the received slots (recs: nsrc * cap 48-B records, DEVICE) are
 * read by the apply itself (equal to corro_unpack_slots + corro_apply_mapped). out->impact (DEVICE, nsrc *
 * cap bytes) gets each received record's flag at its slot position -- padding 0 -- ready to go back to
 * the senders with one more equal-split all-to-all. *overflow_dev (DEVICE u32) = 1 when a source overflowed
 * its slot (nothing is then applied). Synchronous, like corro_apply_batch. INTEGER batches, no affinity.
 * A layout larger than one apply chunk is applied as consecutive index ranges (application order =
 * index order, so the result is that of one apply); the records must come from corro_partition_slots,
 * which validated them: a source whose batch failed marks its counts and the receiver applies nothing. */
int corro_apply_slots(corro_ctx *ctx, const void *recs, uint32_t nsrc, uint64_t cap, const uint64_t *src_counts_dev,
                      corro_apply_out *out, uint32_t *overflow_dev);
/* The senders' side of those flags: back (DEVICE, nranks * cap, the all-to-all of every receiver's
 * out->impact) -> flags[i] (DEVICE, n) of input change i, through the partition's perm_dev and counts_dev.
 * Queued on the context's stream. */
int corro_slots_flags_back(corro_ctx *ctx, const uint8_t *back, uint32_t nranks, uint64_t cap, const uint64_t *counts_dev,
                           const uint32_t *perm_dev, uint8_t *flags, uint64_t n);
/* The HIP stream every launch of the context is queued on (a hipStream_t), for callers that order
 * their own collectives (RCCL) with the engine's kernels without a host wait. */
void *corro_ctx_stream(corro_ctx *ctx);

/* The exchange for EVERY table (interned pks, long values): 80-B records like corro_partition_packed
 * plus a second stream of variable-length bytes per record -- the canonical packed pk of a change to
 * an interned table (so the receiver keys the row in ITS own row-key space) and a long TEXT/BLOB
 * value's bytes -- grouped by destination rank like the records: var_counts[r] bytes for rank r, in
 * rank order. Rows of interned tables are routed by a hash of their canonical pk bytes (the same
 * owner on every rank, whatever dense key each engine gave them); INTEGER-pk rows as in
 * corro_partition_packed. DEVICE memory (in, out, var, perm); counts / var_counts host. var == NULL
 * or var_cap too small: CORRO_E_RANGE after counts and var_counts are filled (records written), so
 * the caller can size var and call again. One call ships < 4 GiB of bytes. */
int corro_partition_var(corro_ctx *ctx, const corro_changes *in, uint32_t nranks, void *out, uint32_t *perm,
                        uint64_t *counts, uint8_t *var, uint64_t var_cap, uint64_t *var_counts);
/* Received 80-B records and var bytes (each concatenated by source rank; src_counts / src_var = what
 * each source sent, host) -> the SoA batch (device, every array set): long values' val_off / val_size
 * point into `var`, which becomes the batch's val_data; interned tables' pks are re-keyed from their
 * shipped canonical bytes (corro_pk_keys on this engine). */
int corro_unpack_var(corro_ctx *ctx, const void *recs, uint64_t n, const uint8_t *var, uint64_t var_len,
                     const uint64_t *src_counts, const uint64_t *src_var, uint32_t nsrc, corro_changes *out);

/* ------------------------------------------------------------------ sync need diff */

/* CSR over (node-pair, actor) entries of two SyncStateV1 (sync.rs:79-87). One entry = one
 * `(actor_id, head)` of other.heads that compute_available_needs does not skip (actor !=
 * self.actor_id and head != 0, sync.rs:133-140). Partials must be listed per entry in the
 * order the caller wants them emitted (ascending version = canonical HashMap order). */
typedef struct {
    uint64_t n;
    const uint64_t *their_head;
    const int64_t *our_head;  /* -1 = None */
    const uint64_t *tn_off, *tn_start, *tn_end;               /* other.need[a] */
    const uint64_t *tp_off, *tp_ver;                           /* other.partial_need[a] keys */
    const uint64_t *tps_off, *tps_start, *tps_end;             /* ... their seq ranges */
    const uint64_t *on_off, *on_start, *on_end;                /* self.need[a] */
    const uint64_t *op_off, *op_ver;                           /* self.partial_need[a] keys */
    const uint64_t *ops_off, *ops_start, *ops_end;             /* ... our seq ranges */
} corro_sync_entries;

/* Output CSR of HashMap<ActorId, Vec<SyncNeedV1>> (sync.rs:252-264). Two passes:
 * pass 0 fills need_count/seq_count per entry; the caller scans them into need_off/seq_off
 * (n+1 entries each) and allocates; pass 1 fills the rest. */
typedef struct {
    uint64_t *need_count, *seq_count;       /* pass 0, n each */
    const uint64_t *need_off, *seq_off;     /* pass 1 inputs, n+1 each */
    uint8_t *kind;                          /* 0 Full{versions: start..=end}, 1 Partial{version: start} */
    uint64_t *start, *end;
    uint64_t *sr_off, *sr_n;                /* Partial seq ranges: [sr_off, sr_off+sr_n) */
    uint64_t *s_start, *s_end;
} corro_needs_out;

/* mem = CORRO_MEM_HOST or CORRO_MEM_DEVICE for BOTH `in` arrays and `out` arrays. */
int corro_compute_needs(corro_ctx *ctx, const corro_sync_entries *in, int mem,
                        corro_needs_out *out, int pass);
/* One-pass form for DEVICE-resident entries and outputs: reads every input once (the count and
 * the fill walk share LDS-staged inputs; workgroup offsets come from a decoupled look-back).
 * Here out->need_off / out->seq_off (n+1 each) are OUTPUTS (written, like pass 0 + scan);
 * kind/start/end/sr_off/sr_n hold need_cap elements, s_start/s_end seq_cap elements.
 * totals[0] = needs, totals[1] = seq ranges (host memory). If a total exceeds its cap the call
 * returns CORRO_E_RANGE, writes no payload past the cap, and totals still hold the exact sizes to
 * re-run with. corro_needs_bound gives caps that always suffice for disjoint need ranges. */
int corro_compute_needs_onepass(corro_ctx *ctx, const corro_sync_entries *in, corro_needs_out *out,
                              uint64_t need_cap, uint64_t seq_cap, uint64_t *totals);
/* Packed one-pass form for DEVICE-resident entries and outputs: one walk per entry, no count pass,
 * no scan. Entry e's needs occupy need slots [need_off[e], need_off[e] + need_count[e]) in reference
 * order (sync.rs:164-245), starting at the slots its own output bound reserves (tn_off[e] +
 * on_off[e] + tp_off[e] + op_off[e] + e; its seq ranges at tps_off[tp_off[e]] + ops_off[op_off[e]]):
 * slots past need_count[e] up to the next entry's are left unwritten, and need_slots / seq_slots =
 * corro_needs_bound's caps. Per need slot q:
 * kind[q] 0 Full{versions: range[2q]..=range[2q+1]}, 1 Partial{version: range[2q], seqs:
 * s_start/s_end[(range[2q+1] >> 24) + j] for j < (range[2q+1] & 0xFFFFFF)}. CORRO_E_RANGE when need
 * ranges overlap (bounds exceeded: use corro_compute_needs) or a partial carries >= 2^24 seq ranges. */
typedef struct {
    uint64_t *need_off;                     /* n */
    uint32_t *need_count;                   /* n */
    uint64_t *range;                        /* 2 per need slot, 16-byte aligned */
    uint8_t *kind;                          /* per need slot */
    uint64_t *s_start, *s_end;              /* per seq slot */
} corro_needs_packed_out;
int corro_compute_needs_packed(corro_ctx *ctx, const corro_sync_entries *in, corro_needs_packed_out *out,
                               uint64_t need_slots, uint64_t seq_slots);
/* Output-size bound from the entry CSR sizes (reads 6 words): needs <= our + their need ranges +
 * their partial versions + our partial versions + entries; seq ranges <= all partial seq ranges. */
int corro_needs_bound(corro_ctx *ctx, const corro_sync_entries *in, int mem, uint64_t *need_cap, uint64_t *seq_cap);
/* Device helper between the two passes: offsets[0] = 0, offsets[k+1] = counts[0] + ... + counts[k]
 * (n + 1 outputs), for device-resident need_count / seq_count. */
int corro_scan_offsets(corro_ctx *ctx, const uint64_t *counts, uint64_t *offsets, uint64_t n);

/* ------------------------------------------------------------------ changeset extraction */

/* Server side of a sync need (handle_need, corro-agent/src/api/peer/mod.rs:371-727): for every
 * need, the state's crsql_changes rows WHERE site_id = site AND db_version BETWEEN start AND end
 * [AND seq BETWEEN seq_start AND seq_end], grouped by db_version in DESCENDING order (:385-394),
 * rows of a group by seq ASCENDING (:423-431, :603-611). A Full need is one entry; a Partial need
 * is one entry per seq range with start = end = version. Ties on seq inside a version come out in
 * an unspecified order (as the SQL leaves them). */
typedef struct {
    uint64_t n;
    const uint32_t *site;                   /* actor site ordinal */
    const uint64_t *start, *end;            /* db_version range, inclusive */
    const uint32_t *seq_start, *seq_end;    /* optional row filter: both NULL = every seq */
} corro_extract_in;

/* Two passes, like corro_compute_needs: pass 0 fills grp_count / row_count per need; the caller
 * scans them into grp_off / row_off (n+1 each) and allocates; pass 1 fills the rest. Per group:
 * db_version, last_seq = MAX(seq) and ts = MAX(ts) over ALL of that version's rows (the GROUP BY
 * query, not the seq-filtered rows), and its rows [grp_row_off, grp_row_off + grp_rows). Row
 * arrays left NULL are not written. */
typedef struct {
    uint64_t *grp_count, *row_count;        /* pass 0, n each */
    const uint64_t *grp_off, *row_off;      /* pass 1 inputs, n+1 each */
    int64_t *version;
    uint64_t *last_seq, *ts;
    uint64_t *grp_row_off, *grp_rows;
    corro_rows rows;
} corro_extract_out;

/* mem = CORRO_MEM_HOST or CORRO_MEM_DEVICE for both. The state index behind it is rebuilt on the
 * first call after the state changed (one radix sort of the clock rows). */
int corro_extract_changes(corro_ctx *ctx, const corro_extract_in *in, int mem, corro_extract_out *out, int pass);

/* ------------------------------------------------------------------ gap bookkeeping */

/* BookedVersions (agent.rs:1260-1458): needed gaps, max, partials' presence. Host-side. */
typedef struct corro_booked corro_booked;
int corro_booked_new(corro_booked **out);
void corro_booked_free(corro_booked *b);
/* VersionsSnapshot::insert_db with `n` applied version ranges. Returns the gap rows to DELETE
 * (removed) and INSERT (inserted) in __corro_bookkeeping_gaps (agent.rs:1120-1163); pass NULL
 * buffers with caps 0 to only apply. *n_removed / *n_inserted receive the full counts. */
int corro_booked_insert_db(corro_booked *b, const uint64_t *start, const uint64_t *end, uint64_t n,
                           uint64_t *rm_start, uint64_t *rm_end, uint64_t rm_cap, uint64_t *n_removed,
                           uint64_t *in_start, uint64_t *in_end, uint64_t in_cap, uint64_t *n_inserted);
int corro_booked_needed(corro_booked *b, uint64_t *start, uint64_t *end, uint64_t cap, uint64_t *count);
int corro_booked_last(corro_booked *b, int64_t *max);     /* -1 = None */
int corro_booked_contains(corro_booked *b, uint64_t version, int *result);
int corro_booked_contains_all(corro_booked *b, uint64_t start, uint64_t end, int *result);

/* Batched insert_db on the device (csrc/gaps.hip): the same gap bookkeeping for n actors in one
 * launch, one lane per actor, DEVICE memory throughout. Inputs per actor a: its BookedVersions max
 * (-1 = None), its needed gaps [gap_off[a], gap_off[a+1]) and this call's applied versions
 * [ver_off[a], ver_off[a+1]), both canonical RangeInclusiveSets (sorted, disjoint, non-touching).
 * Outputs go to windows the input sizes reserve (no count pass): the DELETE rows at
 * rm_*[gap_off[a] .. + rm_count[a]); the INSERT rows at ins_*[gap_off[a] + ver_off[a] + a .. +
 * ins_count[a]) and the new needed gaps at new_*[the same base .. + gap_count[a]) (arrays of
 * gap_off[n] and gap_off[n] + ver_off[n] + n elements). status[a]: 0 ok, -1 a non-canonical input
 * (nothing written for that actor). Partials whose version lies in a DELETE row are the caller's to
 * drop (insert_db's partials.remove, agent.rs:1148). */
typedef struct {
    uint64_t n;
    const int64_t *max;
    const uint64_t *gap_off, *gap_start, *gap_end;
    const uint64_t *ver_off, *ver_start, *ver_end;
} corro_gaps_in;
typedef struct {
    int64_t *max;
    uint64_t *rm_count, *ins_count, *gap_count;
    uint64_t *rm_start, *rm_end;
    uint64_t *ins_start, *ins_end;
    uint64_t *new_start, *new_end;
    int32_t *status;
} corro_gaps_out;
int corro_booked_insert_db_batch(corro_ctx *ctx, const corro_gaps_in *in, corro_gaps_out *out);

/* ------------------------------------------------------------------ process_multiple_changes */

/* Bookie (corro-types/src/agent.rs:1546-1598): BookedVersions per actor, plus the buffered
 * changes / seq bookkeeping of incomplete versions (__corro_buffered_changes,
 * __corro_seq_bookkeeping, agent.rs:290-322). Host-side. */
typedef struct corro_bookie corro_bookie;

enum { CORRO_CS_FULL = 0, CORRO_CS_EMPTY = 1, CORRO_CS_EMPTY_SET = 2 };
/* KnownDbVersion outcome per changeset (agent.rs:1085-1090); negative = corro_status of a
 * version that was rolled back (its SAVEPOINT, util.rs:839-860) */
enum { CORRO_KNOWN_SKIPPED = 0, CORRO_KNOWN_CURRENT = 1, CORRO_KNOWN_CLEARED = 2, CORRO_KNOWN_PARTIAL = 3 };
/* table_cid value a caller uses for a Change whose table/cid did not resolve */
#define CORRO_TCID_UNKNOWN 0xFFFFFFFFu

/* One ChangeV1 (broadcast.rs:114-148): its actor and changeset header; its changes are
 * [change_off, change_off + change_count) of the batch arrays. */
typedef struct {
    const uint8_t *actor_id;   /* 16 bytes */
    uint32_t site;             /* site ordinal of actor_id (corro_site_register) */
    uint32_t kind;             /* CORRO_CS_* */
    uint64_t version_start;    /* Full: version; Empty: versions.start */
    uint64_t version_end;      /* Empty: versions.end */
    uint64_t seq_start, seq_end, last_seq;  /* Full */
    uint64_t ts;               /* changeset timestamp, bound to each change (util.rs:1244) */
    uint64_t change_off, change_count;
} corro_changeset;

typedef struct {
    int32_t *known;       /* per changeset: CORRO_KNOWN_* or negative status */
    uint8_t *impactful;   /* optional, per change: kept in Changeset::Full(impactful) */
    uint64_t n_ready;     /* partial versions that became complete (corro_bookie_take_ready) */
} corro_process_out;

int corro_bookie_new(corro_bookie **out);
void corro_bookie_free(corro_bookie *b);

/* process_multiple_changes (corro-agent/src/agent/util.rs:691-1037) for `ncs` ChangeV1 in arrival
 * order: dedup passes against the bookie, actors in ActorId byte order, empty versions to
 * crsql_set_db_version, incomplete versions buffered, ONE corro_apply_batch for all complete
 * versions, impactful changes with the transaction-cumulative crsql_rows_impacted() semantics,
 * then per-actor gap bookkeeping and partial tracking. `cs` (headers, host memory) names each
 * changeset's changes in `in`; cs[i].site must be the registered ordinal of cs[i].actor_id.
 * `mem` says where `in`'s arrays (val_data included) and out->impactful live: with
 * CORRO_MEM_DEVICE (e.g. corro_decode_frames' device output) no change crosses PCIe -- the
 * unknown-name screen, the applied batch (zero-copy when the applied changesets are one contiguous
 * run of `in`, else one gather kernel) and the impactful flags are device passes, and the host walks
 * only the headers (actors in parallel host threads). With CORRO_MEM_HOST the arrays are copied to
 * the device once. With CORRO_MEM_DEVICE_HEADERS `cs` and out->known are device arrays as well: the
 * header passes run on the device (one pass per changeset, one stable sort by actor, one pass per
 * sorted slot decides every actor whose changesets are complete Full versions strictly ascending in
 * arrival order and above its booked max); the host walks only the other actors' headers (fetched)
 * and runs the gap bookkeeping on per-actor version runs. Unresolved names carry table_cid =
 * CORRO_TCID_UNKNOWN. out->impactful, if set, has in->n entries (0 for changes that were not
 * applied). */
int corro_process_multiple_changes(corro_ctx *ctx, corro_bookie *bk, const corro_changeset *cs, uint64_t ncs,
                                   const corro_changes *in, int mem, corro_process_out *out);
/* (actor, version) pairs whose buffered seqs are complete; cap < count = sizing call */
int corro_bookie_take_ready(corro_bookie *bk, uint8_t *actors, uint64_t *versions, uint64_t cap, uint64_t *count);
/* process_fully_buffered_changes (util.rs:541-688) */
int corro_process_fully_buffered(corro_ctx *ctx, corro_bookie *bk, const uint8_t *actor_id, uint64_t version,
                                 int *impacted);

int corro_bookie_last(corro_bookie *bk, const uint8_t *actor_id, int64_t *max);
int corro_bookie_needed(corro_bookie *bk, const uint8_t *actor_id, uint64_t *start, uint64_t *end, uint64_t cap,
                        uint64_t *count);
int corro_bookie_contains_all(corro_bookie *bk, const uint8_t *actor_id, uint64_t start, uint64_t end,
                              int has_seqs, uint64_t seq_start, uint64_t seq_end, int *result);
int corro_bookie_partial(corro_bookie *bk, const uint8_t *actor_id, uint64_t version, uint64_t *start,
                         uint64_t *end, uint64_t cap, uint64_t *count, int64_t *last_seq);
/* __corro_seq_bookkeeping rows of (actor, version) as handle_need reads them (peer/mod.rs:505-511,
 * :640-667): seq ranges (ascending), last_seq (-1 = none), ts. */
int corro_bookie_seq_bookkeeping(corro_bookie *bk, const uint8_t *actor_id, uint64_t version, uint64_t *start,
                                 uint64_t *end, uint64_t cap, uint64_t *count, int64_t *last_seq, uint64_t *ts);
/* Versions of actor in [vstart, vend] holding buffered rows, ascending (handle_need's
 * EXISTS(__corro_buffered_changes) probe, peer/mod.rs:466-492). */
int corro_bookie_buffered_versions(corro_bookie *bk, const uint8_t *actor_id, uint64_t vstart, uint64_t vend,
                                   uint64_t *versions, uint64_t cap, uint64_t *count);
/* __corro_buffered_changes rows of (actor, version) with seq in [seq_start, seq_end], seq
 * ascending (peer/mod.rs:513-531, :672-693); *count = matching rows, at most cap written. */
int corro_bookie_buffered(corro_bookie *bk, const uint8_t *actor_id, uint64_t version, uint64_t seq_start,
                          uint64_t seq_end, corro_rows *out, uint64_t cap, uint64_t *count);
/* Bytes of the buffered row (actor, version, seq) when it holds a long value (its corro_rows entry
 * has val_len == CORRO_VAL_LONG and val1 = 0): *len = the length (0 = no such value), at most cap
 * bytes copied. */
int corro_bookie_buffered_value(corro_bookie *bk, const uint8_t *actor_id, uint64_t version, uint64_t seq,
                                uint8_t *out, uint64_t cap, uint64_t *len);

/* generate_sync (corro-types/src/sync.rs:284-333) as CSR over actors with a known head:
 * heads, needed ranges, and for every non-complete partial the seq gaps over 0..=last_seq. */
typedef struct {
    uint64_t n_actors, n_need, n_partials, n_pseqs;    /* pass 0 output */
    uint8_t *actor_ids;                                /* 16 * n_actors */
    uint64_t *heads;                                   /* n_actors */
    uint64_t *need_off, *need_start, *need_end;        /* n_actors + 1, n_need, n_need */
    uint64_t *partial_off, *partial_ver;               /* n_actors + 1, n_partials */
    uint64_t *pseq_off, *pseq_start, *pseq_end;        /* n_partials + 1, n_pseqs, n_pseqs */
} corro_sync_state;
int corro_generate_sync(corro_bookie *bk, const uint8_t *self_actor, corro_sync_state *out, int pass);

/* ------------------------------------------------------------------ wire decode */

/* Decode length-delimited frames (tokio LengthDelimitedCodec: u32 big-endian length + payload,
 * api/peer/mod.rs:917-929) of speedy-encoded changeset messages on the GPU:
 * CORRO_PAYLOAD_SYNC = SyncMessage::V1(SyncMessageV1::Changeset(ChangeV1)) (sync.rs:19-30),
 * CORRO_PAYLOAD_UNI = UniPayload::V1 { Broadcast(BroadcastV1::Change(ChangeV1)), .. }
 * (broadcast.rs:41-52, uni.rs:63). `buf` is host memory. Two passes: pass 0 sets nframes /
 * nchanges / nsets; the caller allocates; pass 1 fills one corro_changeset per frame (cs[i],
 * actor_id pointing into actor_ids) and the changes as one SoA batch (arrays on `mem`, the shape
 * corro_process_multiple_changes / corro_apply_batch take; ts = the changeset's ts). EmptySet
 * ranges go to set_start/set_end at [change_off, change_off + change_count) of their frame.
 * status[i]: 0 ok, 1 not a changeset message (skipped), CORRO_E_INVALID malformed, CORRO_E_RANGE a
 * value outside the engine encoding (a pk that is not one packed INTEGER in a table not marked
 * interned, seq or cl beyond 32 bits, a TEXT/BLOB of 16 MiB or more, or one longer than 16 bytes
 * when changes.val_off / val_size are NULL); the changes of a frame with status != 0 are
 * unspecified. Unknown table/column names give table_cid = CORRO_TCID_UNKNOWN; site ids not yet
 * registered are registered (corro_site_register) so every site field is a valid ordinal. Interned
 * tables' pks are interned (corro_pk_keys). Long TEXT/BLOB values: pass 1 fills changes.val_off /
 * val_size (caller arrays of nchanges, on `mem`) with offsets into the frame buffer, which becomes
 * changes.val_data (host: `buf` itself; device: the caller's changes.val_data, len bytes, receives a
 * copy) with val_data_len = len; with no long value decoded the four fields are set to NULL / 0. */
enum { CORRO_PAYLOAD_SYNC = 0, CORRO_PAYLOAD_UNI = 1 };
typedef struct {
    uint64_t nframes, nchanges, nsets;      /* pass 0 outputs, pass 1 inputs */
    corro_changeset *cs;                    /* host, nframes (optional when cs_dev is set) */
    uint8_t *actor_ids;                     /* host, 16 * nframes (with cs) */
    int32_t *status;                        /* host, nframes (optional) */
    corro_changes changes;                  /* nchanges each (mem); val1/val_type/val_len/ts optional */
    uint64_t *set_start, *set_end;          /* nsets each (mem) */
    /* optional, pass 1: the headers of the frames with status 0, in frame order, written on the
     * device into cs_dev (device, nframes entries) for corro_process_multiple_changes with
     * CORRO_MEM_DEVICE_HEADERS; EmptySet headers carry change_count 0 there; actor_id is NULL.
     * n_dev = how many were written. */
    corro_changeset *cs_dev;
    uint64_t n_dev;
} corro_decoded;
int corro_decode_frames(corro_ctx *ctx, const uint8_t *buf, uint64_t len, int payload, int mem, corro_decoded *out,
                        int pass);

#ifdef __cplusplus
}
#endif
#endif /* CORRO_HIP_H */
