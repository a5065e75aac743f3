/* oracle/oracle.h — TEST INFRASTRUCTURE ONLY. CPU restatements used as the parity checker.
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load liboracle.so. */
#ifndef CORRO_ORACLE_H
#define CORRO_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { OF_INTEGER = 1, OF_REAL = 2, OF_TEXT = 3, OF_BLOB = 4, OF_NULL = 5 };

/* Column-change batch, SoA, application order = index order (same field order as
 * corro_changes in include/corro_hip.h). table_cid = (table << 16) | cid, cid 0 = sentinel '-1'. */
typedef struct {
    uint64_t n;
    const uint64_t *pk;
    const uint32_t *table_cid;
    const int64_t *col_version;
    const int64_t *db_version;
    const uint32_t *cl;
    const uint32_t *seq;
    const uint32_t *site;      /* site ordinal */
    const uint64_t *val0;      /* INTEGER bits / REAL bits / TEXT,BLOB bytes 0..7 big-endian */
    const uint64_t *val1;      /* optional: TEXT,BLOB bytes 8..15 big-endian */
    const uint8_t *val_type;   /* optional: OF_* (NULL = all INTEGER) */
    const uint8_t *val_len;    /* optional: TEXT/BLOB length (<= 16) */
    const uint64_t *ts;        /* optional: changeset timestamp (NTP64) */
    /* optional: TEXT/BLOB values longer than 16 bytes. A change with val_len == OF_LONG holds its
     * bytes at val_data[val_off[i], val_off[i] + val_size[i]) (17 <= val_size < 2^24). */
    const uint64_t *val_off;
    const uint32_t *val_size;
    const uint8_t *val_data;
} of_changes;

/* val_len of a long value; in exported rows its val1 is a handle of_value_bytes resolves */
#define OF_LONG 255

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
} of_rows;

typedef struct of_state of_state;

of_state *of_new(const uint8_t *site_ids, uint32_t nsites);
void of_free(of_state *s);
void of_apply(of_state *s, const of_changes *in, uint8_t *impact_out);
uint64_t of_count(const of_state *s);
uint64_t of_export(const of_state *s, of_rows *out);
void of_db_versions(const of_state *s, int64_t *out);
/* bytes of a long value exported by of_export (val_len == OF_LONG, handle = its val1); returns the
 * length, copies min(length, cap) bytes */
uint64_t of_value_bytes(const of_state *s, uint64_t handle, uint8_t *out, uint64_t cap);
/* content hash the digests use in place of a long value's handle */
uint64_t of_bytes_hash(const uint8_t *p, uint64_t len);
/* pk-sharded parallel fold: shards[s] owns the rows hashed to s (<= 256 shards) */
int of_apply_sharded(of_state **shards, uint32_t nshards, const of_changes *in, uint8_t *impact_out,
                     uint32_t nthreads);
/* order-independent digests: {rows, sum of row hashes, xor of rotated row hashes}; state digests
 * accumulate into out (so shard digests add up), row-array digests overwrite it. A long value
 * enters a row hash as of_bytes_hash of its bytes: of_rows_digest expects the caller to have put
 * that hash in val1 of every row with val_len == OF_LONG. */
void of_state_digest(const of_state *s, uint64_t out[3]);
void of_rows_digest(const of_rows *o, uint64_t n, uint64_t out[3]);

/* ---- column affinity (affinity.c; codes as CORRO_AFF_* in include/corro_hip.h) ---- */
enum { OF_AFF_BLOB = 0, OF_AFF_TEXT = 1, OF_AFF_NUMERIC = 2, OF_AFF_INTEGER = 3, OF_AFF_REAL = 4 };
/* The value a column of affinity `aff` stores for (type, v0 = INTEGER / REAL bits, txt/len = TEXT
 * bytes). Returns 1 if that differs from the input: *otype, and *ov0 (INTEGER / REAL) or otxt/olen
 * (TEXT, at most 32 bytes). */
int of_affinity(int aff, int type, uint64_t v0, const uint8_t *txt, uint64_t len, int *otype, uint64_t *ov0,
                uint8_t *otxt, uint32_t *olen);
/* the fold stores a winning value as its column's affinity converts it (the incoming change is
 * still compared unconverted, App. A.4); aff[c] = affinity of cid c + 1 */
void of_set_affinity(of_state *s, uint32_t table, const uint8_t *aff, uint32_t ncols);

/* ---- sync need diff (corro-types/src/sync.rs:127-249), CSR over (pair, actor) entries ---- */
typedef struct {
    uint64_t n;                 /* entries */
    const uint64_t *their_head; /* > 0 (entries with head 0 / self actor are skipped by the caller) */
    const int64_t *our_head;    /* -1 = we have no head for the actor */
    const uint64_t *tn_off;     /* their need ranges: [tn_off[e], tn_off[e+1]) */
    const uint64_t *tn_start, *tn_end;
    const uint64_t *tp_off;     /* their partial versions */
    const uint64_t *tp_ver;
    const uint64_t *tps_off;    /* per their partial k: seq ranges [tps_off[k], tps_off[k+1]) */
    const uint64_t *tps_start, *tps_end;
    const uint64_t *on_off;     /* our need ranges */
    const uint64_t *on_start, *on_end;
    const uint64_t *op_off;     /* our partial versions */
    const uint64_t *op_ver;
    const uint64_t *ops_off;
    const uint64_t *ops_start, *ops_end;
} of_sync_entries;

typedef struct {
    /* count pass writes per-entry totals; fill pass writes the CSR */
    uint64_t *need_count;   /* per entry: number of SyncNeedV1 */
    uint64_t *seq_count;    /* per entry: number of seq ranges over its partial needs */
    /* fill pass (offsets = exclusive scans of the counts) */
    const uint64_t *need_off, *seq_off;
    uint8_t *kind;          /* 0 = Full, 1 = Partial */
    uint64_t *start, *end;  /* Full: versions start..=end; Partial: version in start, seq ranges in [sr_off[k], sr_off[k+1]) */
    uint64_t *sr_off;       /* per need: absolute offset of its first seq range (size = total needs) */
    uint64_t *sr_n;         /* per need: number of seq ranges */
    uint64_t *s_start, *s_end;
} of_needs_out;

void of_needs(const of_sync_entries *in, of_needs_out *out, int fill);

/* ---- gap bookkeeping (corro-types/src/agent.rs:1108-1235) ---- */
typedef struct of_booked of_booked;
of_booked *of_booked_new(void);
void of_booked_free(of_booked *b);
/* insert_db of the RangeInclusiveSet built from `n` ranges; returns 0 on success */
int of_booked_insert_db(of_booked *b, const uint64_t *start, const uint64_t *end, uint64_t n);
/* needed ranges -> out (caller sized by of_booked_needed_len) */
uint64_t of_booked_needed_len(const of_booked *b);
void of_booked_needed(const of_booked *b, uint64_t *start, uint64_t *end);
int64_t of_booked_max(const of_booked *b);  /* -1 = None */
int of_booked_contains(const of_booked *b, uint64_t version);

#ifdef __cplusplus
}
#endif
#endif
