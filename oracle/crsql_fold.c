/*
 * oracle/crsql_fold.c — TEST INFRASTRUCTURE ONLY (the checker, never the product).
 *
 * A sequential CPU restatement of the cr-sqlite 0.17.0 `crsql_changes` INSERT merge that
 * corrosion drives once per column change in `process_complete_version`
 * (/root/reference/crates/corro-agent/src/agent/util.rs:1222-1262, INSERT at :1225-1245,
 * `crsql_rows_impacted()` at :1246-1248) with `merge-equal-values = 1`
 * (/root/reference/crates/corro-types/src/agent.rs:358-362).
 *
 * The merge arithmetic itself lives in the prebuilt cr-sqlite binary shipped with the reference
 * (crates/corro-types/crsqlite-linux-x86_64.so, embedded at corro-types/src/sqlite.rs:22-27).
 * That binary is NOT loaded or run here (prebuilt machine code inside the reference).
 * The rules below restate SURVEY.md Appendix A.1 (cr-sqlite 0.17 causal-length + LWW):
 *
 *   L = col_version of the row's sentinel clock ('-1') if present, else 1 if any clock row
 *       exists, else 0.
 *   1. cl <  L                     -> no-op
 *   2. cl even: cl == L -> no-op; else delete row, drop non-sentinel clocks, sentinel := x (cv=x.cv)
 *   3. sentinel, odd cl: cl > L -> zero all non-sentinel col_versions, sentinel := x (cv=x.cv)
 *   4. column, odd cl:
 *        cl > L and (L > 0 or cl > 1): zero col_versions, sentinel := x with cv = cl (+1 impact),
 *                                      then the column wins unconditionally (+1 impact)
 *        cl > L, L == 0, cl == 1     : plain first write (+1)
 *        cl == L                     : LWW on (col_version, value, site_id bytes) vs the cell's
 *                                      current writer; no local clock -> win
 *   crsql_db_versions[site] = max(.., db_version) for EVERY inserted change.
 *
 * Value order: type rank INTEGER > REAL > TEXT > BLOB > NULL; INTEGER signed,
 * REAL numeric (-0.0 == 0.0), TEXT/BLOB memcmp then length, NULL == NULL. TEXT/BLOB values have
 * no length limit (SqliteValue::Text(String) / Blob(Vec<u8>), corro-api-types/src/lib.rs:419-429):
 * values longer than 16 bytes are kept whole in a per-state byte arena and compared in full.
 *
 * Parity pinning: the KATs of SURVEY.md App. A.5 and the worked example in
 * /root/reference/doc/crdts.md:225-245 (tests/golden/merge_kats.json, tests/test_oracle.py).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

typedef struct {
    uint32_t cid;
    int64_t cv;
    int64_t dbv;
    uint32_t site, seq;
    uint64_t ts;
    uint8_t vtype, vlen;
    uint64_t v0, v1;
} of_cell;

typedef struct {
    uint64_t pk;
    uint32_t table;
    int used;
    int has_sent;
    of_cell sent;  /* sentinel clock: cv = causal length */
    of_cell *cells;
    uint32_t ncells, capcells;
} of_row;

struct of_state {
    uint8_t *site_ids;  /* 16 bytes per ordinal */
    uint32_t nsites;
    int64_t *dbv;       /* per-site max db_version, -1 = absent */
    of_row *rows;
    uint64_t cap, nrows;
    uint8_t *arena;     /* bytes of long values; a long cell's v1 = (offset << 24) | length */
    uint64_t arena_len, arena_cap;
    uint8_t *aff;       /* column affinity, 257 per table (NULL = none: every column BLOB) */
    uint32_t aff_tables;
};

static uint64_t mix64(uint64_t x) {
    x ^= x >> 33; x *= 0xff51afd7ed558ccdULL;
    x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ULL;
    x ^= x >> 33; return x;
}

of_state *of_new(const uint8_t *site_ids, uint32_t nsites) {
    of_state *s = (of_state *)calloc(1, sizeof(of_state));
    s->nsites = nsites;
    s->site_ids = (uint8_t *)malloc((size_t)nsites * 16 + 16);
    if (nsites) memcpy(s->site_ids, site_ids, (size_t)nsites * 16);
    s->dbv = (int64_t *)malloc(sizeof(int64_t) * (nsites + 1));
    for (uint32_t i = 0; i < nsites; i++) s->dbv[i] = -1;
    s->cap = 1024;
    s->rows = (of_row *)calloc(s->cap, sizeof(of_row));
    return s;
}

void of_free(of_state *s) {
    if (!s) return;
    for (uint64_t i = 0; i < s->cap; i++) free(s->rows[i].cells);
    free(s->rows); free(s->dbv); free(s->site_ids); free(s->arena); free(s->aff); free(s);
}

static of_row *find_row(of_state *s, uint32_t table, uint64_t pk, int create);

static void grow(of_state *s) {
    of_row *old = s->rows; uint64_t oldcap = s->cap;
    s->cap *= 2;
    s->rows = (of_row *)calloc(s->cap, sizeof(of_row));
    for (uint64_t i = 0; i < oldcap; i++) {
        if (!old[i].used) continue;
        uint64_t h = mix64(old[i].pk ^ ((uint64_t)old[i].table << 48) ^ old[i].table) & (s->cap - 1);
        while (s->rows[h].used) h = (h + 1) & (s->cap - 1);
        s->rows[h] = old[i];
    }
    free(old);
}

static of_row *find_row(of_state *s, uint32_t table, uint64_t pk, int create) {
    uint64_t h = mix64(pk ^ ((uint64_t)table << 48) ^ table) & (s->cap - 1);
    while (s->rows[h].used) {
        if (s->rows[h].pk == pk && s->rows[h].table == table) return &s->rows[h];
        h = (h + 1) & (s->cap - 1);
    }
    if (!create) return NULL;
    if ((s->nrows + 1) * 2 > s->cap) { grow(s); return find_row(s, table, pk, 1); }
    of_row *r = &s->rows[h];
    memset(r, 0, sizeof(*r));
    r->used = 1; r->pk = pk; r->table = table;
    s->nrows++;
    return r;
}

static int64_t row_L(const of_row *r) {
    if (r->has_sent) return r->sent.cv;
    return r->ncells ? 1 : 0;
}

static int rank_of(uint8_t t) { return 5 - (int)t; }  /* INTEGER(1)=4 ... NULL(5)=0 */

/* A value as the merge compares it: short TEXT/BLOB bytes live big-endian in v0/v1 (zero padded,
 * length vlen), a long one (vlen == OF_LONG) at lp[0, llen). */
typedef struct {
    uint8_t type, vlen;
    uint64_t v0, v1;
    const uint8_t *lp;
    uint64_t llen;
} of_val;

static const uint8_t *val_bytes(const of_val *v, uint8_t buf[16], uint64_t *len) {
    if (v->vlen == OF_LONG) { *len = v->llen; return v->lp; }
    for (int k = 0; k < 8; k++) { buf[k] = (uint8_t)(v->v0 >> (56 - 8 * k)); buf[8 + k] = (uint8_t)(v->v1 >> (56 - 8 * k)); }
    *len = v->vlen;
    return buf;
}

/* compare incoming value a against local value b: >0 a greater, <0 b greater, 0 equal */
static int value_cmp(const of_val *a, const of_val *b) {
    if (a->type != b->type) return rank_of(a->type) > rank_of(b->type) ? 1 : -1;
    switch (a->type) {
    case OF_INTEGER: {
        int64_t x = (int64_t)a->v0, y = (int64_t)b->v0;
        return x > y ? 1 : (x < y ? -1 : 0);
    }
    case OF_REAL: {
        double x, y;
        memcpy(&x, &a->v0, 8); memcpy(&y, &b->v0, 8);
        return x > y ? 1 : (x < y ? -1 : 0);
    }
    case OF_TEXT:
    case OF_BLOB: {  /* memcmp over the common length, then the longer value is greater */
        uint8_t ba[16], bb[16];
        uint64_t la, lb;
        const uint8_t *pa = val_bytes(a, ba, &la), *pb = val_bytes(b, bb, &lb);
        int c = memcmp(pa, pb, la < lb ? la : lb);
        if (c) return c > 0 ? 1 : -1;
        return la > lb ? 1 : (la < lb ? -1 : 0);
    }
    default:
        return 0;  /* NULL == NULL */
    }
}

static of_val in_val(const of_changes *in, uint64_t i) {
    of_val v;
    v.type = in->val_type ? in->val_type[i] : OF_INTEGER;
    v.vlen = in->val_len ? in->val_len[i] : 0;
    v.v0 = in->val0 ? in->val0[i] : 0;
    v.v1 = in->val1 ? in->val1[i] : 0;
    v.lp = NULL; v.llen = 0;
    if (v.vlen == OF_LONG && (v.type == OF_TEXT || v.type == OF_BLOB)) {
        v.lp = in->val_data + in->val_off[i];
        v.llen = in->val_size[i];
        v.v0 = 0;  /* bytes 0..7 big-endian (the caller's val0 is not read) */
        for (int k = 0; k < 8; k++) v.v0 = (v.v0 << 8) | v.lp[k];
        v.v1 = 0;
    }
    return v;
}

static of_val cell_val(const of_state *s, const of_cell *c) {
    of_val v;
    v.type = c->vtype; v.vlen = c->vlen; v.v0 = c->v0; v.v1 = c->v1;
    v.lp = NULL; v.llen = 0;
    if (c->vlen == OF_LONG) { v.lp = s->arena + (c->v1 >> 24); v.llen = c->v1 & 0xFFFFFFu; }
    return v;
}

static uint64_t arena_put(of_state *s, const uint8_t *p, uint64_t len) {
    if (s->arena_len + len > s->arena_cap) {
        while (s->arena_len + len > s->arena_cap) s->arena_cap = s->arena_cap ? 2 * s->arena_cap : 4096;
        s->arena = (uint8_t *)realloc(s->arena, s->arena_cap);
    }
    const uint64_t off = s->arena_len;
    memcpy(s->arena + off, p, len);
    s->arena_len += len;
    return off;
}

uint64_t of_bytes_hash(const uint8_t *p, uint64_t len) {
    uint64_t h = mix64(len + 0x2545F4914F6CDD1DULL);
    uint64_t k = 0;
    for (; k + 8 <= len; k += 8) {
        uint64_t w;
        memcpy(&w, p + k, 8);
        h = mix64(h ^ w);
    }
    if (k < len) {
        uint64_t w = 0;
        memcpy(&w, p + k, len - k);
        h = mix64(h ^ w ^ 0x9E3779B97F4A7C15ULL);
    }
    return h;
}

uint64_t of_value_bytes(const of_state *s, uint64_t handle, uint8_t *out, uint64_t cap) {
    const uint64_t off = handle >> 24, len = handle & 0xFFFFFFu;
    if (off + len > s->arena_len) return 0;
    memcpy(out, s->arena + off, len < cap ? len : cap);
    return len;
}

#define OF_AFF_W 257
void of_set_affinity(of_state *s, uint32_t table, const uint8_t *aff, uint32_t ncols) {
    if (table >= s->aff_tables) {
        s->aff = (uint8_t *)realloc(s->aff, (size_t)(table + 1) * OF_AFF_W);
        memset(s->aff + (size_t)s->aff_tables * OF_AFF_W, OF_AFF_BLOB, (size_t)(table + 1 - s->aff_tables) * OF_AFF_W);
        s->aff_tables = table + 1;
    }
    for (uint32_t c = 0; c < ncols && c + 1 < OF_AFF_W; c++) s->aff[(size_t)table * OF_AFF_W + c + 1] = aff[c];
}

/* the base table stores the value its column's affinity converts it to (affinity.c) */
static int convert_cell(of_state *s, of_cell *c, uint32_t table, const of_val *raw) {
    if (!s->aff || table >= s->aff_tables || c->cid >= OF_AFF_W) return 0;
    const int aff = s->aff[(size_t)table * OF_AFF_W + c->cid];
    uint8_t buf[16], out[32];
    uint64_t len = 0;
    const uint8_t *p = raw->type == OF_TEXT ? val_bytes(raw, buf, &len) : NULL;
    int ot;
    uint64_t ov0;
    uint32_t olen;
    if (!of_affinity(aff, raw->type, raw->v0, p, len, &ot, &ov0, out, &olen)) return 0;
    c->vtype = (uint8_t)ot;
    c->v0 = c->v1 = 0;
    c->vlen = 0;
    if (ot != OF_TEXT) {
        c->v0 = ov0;
    } else if (olen <= 16) {
        for (uint32_t k = 0; k < olen; k++) {
            if (k < 8) c->v0 |= (uint64_t)out[k] << (56 - 8 * k);
            else c->v1 |= (uint64_t)out[k] << (56 - 8 * (k - 8));
        }
        c->vlen = (uint8_t)olen;
    } else {
        for (int k = 0; k < 8; k++) c->v0 = (c->v0 << 8) | out[k];
        c->v1 = (arena_put(s, out, olen) << 24) | olen;
        c->vlen = OF_LONG;
    }
    return 1;
}

static void fill_cell(of_state *s, of_cell *c, const of_changes *in, uint64_t i) {
    c->cid = in->table_cid[i] & 0xFFFFu;
    c->cv = in->col_version[i];
    c->dbv = in->db_version[i];
    c->site = in->site[i];
    c->seq = in->seq[i];
    c->ts = in->ts ? in->ts[i] : 0;
    c->vtype = in->val_type ? in->val_type[i] : OF_INTEGER;
    c->vlen = in->val_len ? in->val_len[i] : 0;
    c->v0 = in->val0 ? in->val0[i] : 0;
    c->v1 = in->val1 ? in->val1[i] : 0;
    if (s->aff) {
        const of_val v = in_val(in, i);
        if (convert_cell(s, c, in->table_cid[i] >> 16, &v)) return;
    }
    if (c->vlen == OF_LONG && (c->vtype == OF_TEXT || c->vtype == OF_BLOB)) {
        const of_val v = in_val(in, i);
        c->v0 = v.v0;
        c->v1 = (arena_put(s, v.lp, v.llen) << 24) | v.llen;
    }
}

static of_cell *find_cell(of_row *r, uint32_t cid) {
    for (uint32_t k = 0; k < r->ncells; k++)
        if (r->cells[k].cid == cid) return &r->cells[k];
    return NULL;
}

static of_cell *add_cell(of_row *r) {
    if (r->ncells == r->capcells) {
        r->capcells = r->capcells ? r->capcells * 2 : 4;
        r->cells = (of_cell *)realloc(r->cells, sizeof(of_cell) * r->capcells);
    }
    return &r->cells[r->ncells++];
}

static void set_cell(of_state *s, of_row *r, const of_changes *in, uint64_t i) {
    uint32_t cid = in->table_cid[i] & 0xFFFFu;
    of_cell *c = find_cell(r, cid);
    if (!c) c = add_cell(r);
    fill_cell(s, c, in, i);
}

/* the sentinel clock takes change i's clock fields (never a value) */
static void fill_sentinel(of_row *r, const of_changes *in, uint64_t i) {
    of_cell *c = &r->sent;
    c->cid = 0;
    c->cv = in->col_version[i];
    c->dbv = in->db_version[i];
    c->site = in->site[i];
    c->seq = in->seq[i];
    c->ts = in->ts ? in->ts[i] : 0;
    c->vtype = OF_NULL; c->vlen = 0; c->v0 = c->v1 = 0;
}

static void zero_cells(of_row *r) {
    for (uint32_t k = 0; k < r->ncells; k++) r->cells[k].cv = 0;
}

/* One `INSERT INTO crsql_changes` (util.rs:1225-1245). Returns the crsql_rows_impacted() delta. */
static int apply_one(of_state *s, const of_changes *in, uint64_t i) {
    uint32_t site = in->site[i];
    int64_t dbv = in->db_version[i];
    if (site < s->nsites && s->dbv[site] < dbv) s->dbv[site] = dbv;

    uint32_t table = in->table_cid[i] >> 16, cid = in->table_cid[i] & 0xFFFFu;
    int64_t cl = (int64_t)in->cl[i];
    of_row *r = find_row(s, table, in->pk[i], 1);
    int64_t L = row_L(r);

    if (cl < L) return 0;                                   /* rule 1 */
    if ((cl & 1) == 0) {                                    /* rule 2: delete */
        if (cl == L) return 0;
        r->ncells = 0;
        r->has_sent = 1;
        fill_sentinel(r, in, i);                            /* sentinel cv = x.cv */
        return 1;
    }
    if (cid == 0) {                                         /* rule 3: pk-only / resurrect */
        if (cl > L) {
            zero_cells(r);
            r->has_sent = 1;
            fill_sentinel(r, in, i);
            return 1;
        }
        return 0;
    }
    if (cl > L) {                                           /* rule 4: needs resurrect */
        int imp = 0;
        if (L > 0 || cl > 1) {
            zero_cells(r);
            r->has_sent = 1;
            fill_sentinel(r, in, i);
            r->sent.cv = cl;
            imp = 1;
        }
        set_cell(s, r, in, i);
        return imp + 1;
    }
    /* cl == L : last-writer-wins */
    of_cell *c = find_cell(r, cid);
    if (c) {
        int64_t cv = in->col_version[i];
        if (cv < c->cv) return 0;
        if (cv == c->cv) {
            const of_val a = in_val(in, i), b = cell_val(s, c);
            int vc = value_cmp(&a, &b);
            if (vc < 0) return 0;
            if (vc == 0) {
                /* merge-equal-values: bigger writer site id wins (memcmp of 16 bytes) */
                const uint8_t *a = s->site_ids + 16 * (size_t)site;
                const uint8_t *b = s->site_ids + 16 * (size_t)c->site;
                if (memcmp(a, b, 16) <= 0) return 0;
            }
        }
    }
    set_cell(s, r, in, i);
    return 1;
}

void of_apply(of_state *s, const of_changes *in, uint8_t *impact_out) {
    for (uint64_t i = 0; i < in->n; i++) {
        int imp = apply_one(s, in, i);
        if (impact_out) impact_out[i] = (uint8_t)imp;
    }
}

uint64_t of_count(const of_state *s) {
    uint64_t n = 0;
    for (uint64_t i = 0; i < s->cap; i++) {
        const of_row *r = &s->rows[i];
        if (!r->used) continue;
        n += (uint64_t)r->has_sent + r->ncells;
    }
    return n;
}

typedef struct { uint32_t table; uint64_t pk; uint64_t idx; } rowref;

static int cmp_rowref(const void *a, const void *b) {
    const rowref *x = (const rowref *)a, *y = (const rowref *)b;
    if (x->table != y->table) return x->table < y->table ? -1 : 1;
    if (x->pk != y->pk) return x->pk < y->pk ? -1 : 1;
    return 0;
}

static int cmp_cell(const void *a, const void *b) {
    const of_cell *x = (const of_cell *)a, *y = (const of_cell *)b;
    return x->cid < y->cid ? -1 : (x->cid > y->cid ? 1 : 0);
}

static void emit(of_rows *o, uint64_t k, const of_row *r, const of_cell *c, uint32_t cid, int64_t cl) {
    o->pk[k] = r->pk;
    o->table_cid[k] = (r->table << 16) | cid;
    o->col_version[k] = c->cv;
    o->db_version[k] = c->dbv;
    o->cl[k] = cl;
    o->seq[k] = c->seq;
    o->site[k] = c->site;
    o->ts[k] = c->ts;
    o->val_type[k] = cid == 0 ? OF_NULL : c->vtype;
    o->val_len[k] = cid == 0 ? 0 : c->vlen;
    o->val0[k] = cid == 0 ? 0 : c->v0;
    o->val1[k] = cid == 0 ? 0 : c->v1;
}

/* crsql_changes read-back, canonical order (table, pk, cid) with the sentinel ('-1' = cid 0) first */
uint64_t of_export(const of_state *s, of_rows *o) {
    rowref *refs = (rowref *)malloc(sizeof(rowref) * (s->nrows + 1));
    uint64_t m = 0;
    for (uint64_t i = 0; i < s->cap; i++)
        if (s->rows[i].used) { refs[m].table = s->rows[i].table; refs[m].pk = s->rows[i].pk; refs[m].idx = i; m++; }
    qsort(refs, m, sizeof(rowref), cmp_rowref);
    uint64_t k = 0;
    for (uint64_t j = 0; j < m; j++) {
        of_row *r = &s->rows[refs[j].idx];
        int64_t L = row_L(r);
        if (r->has_sent) emit(o, k++, r, &r->sent, 0, L);
        if (r->ncells > 1) qsort(r->cells, r->ncells, sizeof(of_cell), cmp_cell);
        for (uint32_t c = 0; c < r->ncells; c++) emit(o, k++, r, &r->cells[c], r->cells[c].cid, L);
    }
    free(refs);
    return k;
}

/* crsql_db_versions: per-site max db_version (-1 = site never seen) */
void of_db_versions(const of_state *s, int64_t *out) {
    memcpy(out, s->dbv, sizeof(int64_t) * s->nsites);
}

/* ---- pk-sharded fold (SURVEY.md §8(d) CPU baseline (ii), and the checker at >= 512M changes) ----
 * Rows merge independently, so S shard states, each owning the rows whose
 * mix64(table, pk) falls in it, folded by S threads over their changes in application order, give
 * exactly the sequential fold's rows and impacts; crsql_db_versions is the per-site max over shards. */
#include <pthread.h>

static uint32_t shard_of(uint32_t table, uint64_t pk, uint32_t nshards) {
    return (uint32_t)(((mix64(pk ^ ((uint64_t)table << 48) ^ table) >> 32) * nshards) >> 32);
}

typedef struct {
    of_state **shards;
    uint32_t nshards, nthreads, t;
    const of_changes *in;
    uint8_t *impact;
    uint8_t *sid;        /* shard id per change */
    uint64_t *counts;    /* [nthreads][nshards] */
    uint64_t *offs;      /* [nthreads][nshards] start of this slice's run in idx */
    uint32_t *idx;       /* change indices grouped by shard, application order within a shard */
    uint64_t *shard_off; /* [nshards + 1] */
    int phase;
} sh_job;

static void *sh_worker(void *p) {
    sh_job *j = (sh_job *)p;
    uint64_t n = j->in->n;
    uint64_t lo = n * j->t / j->nthreads, hi = n * (j->t + 1) / j->nthreads;
    if (j->phase == 0) {
        uint64_t *c = j->counts + (size_t)j->t * j->nshards;
        for (uint64_t i = lo; i < hi; i++) {
            uint32_t s = shard_of(j->in->table_cid[i] >> 16, j->in->pk[i], j->nshards);
            j->sid[i] = (uint8_t)s;
            c[s]++;
        }
    } else if (j->phase == 1) {
        uint64_t *o = j->offs + (size_t)j->t * j->nshards;
        for (uint64_t i = lo; i < hi; i++) j->idx[o[j->sid[i]]++] = (uint32_t)i;
    } else {
        for (uint32_t s = j->t; s < j->nshards; s += j->nthreads) {
            of_state *st = j->shards[s];
            for (uint64_t k = j->shard_off[s]; k < j->shard_off[s + 1]; k++) {
                uint64_t i = j->idx[k];
                int imp = apply_one(st, j->in, i);
                if (j->impact) j->impact[i] = (uint8_t)imp;
            }
        }
    }
    return NULL;
}

static void sh_run(sh_job *base, uint32_t nthreads, int phase) {
    pthread_t *th = (pthread_t *)malloc(sizeof(pthread_t) * nthreads);
    sh_job *jobs = (sh_job *)malloc(sizeof(sh_job) * nthreads);
    for (uint32_t t = 0; t < nthreads; t++) {
        jobs[t] = *base; jobs[t].t = t; jobs[t].phase = phase;
        pthread_create(&th[t], NULL, sh_worker, &jobs[t]);
    }
    for (uint32_t t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
    free(jobs); free(th);
}

/* Apply one batch to `nshards` (<= 256) shard states with `nthreads` threads. Returns 0, or -1 if
 * the batch exceeds 2^32-1 changes. */
int of_apply_sharded(of_state **shards, uint32_t nshards, const of_changes *in, uint8_t *impact_out,
                     uint32_t nthreads) {
    if (in->n >= (1ULL << 32) || nshards == 0 || nshards > 256) return -1;
    if (nthreads == 0) nthreads = 1;
    sh_job b;
    memset(&b, 0, sizeof(b));
    b.shards = shards; b.nshards = nshards; b.nthreads = nthreads; b.in = in; b.impact = impact_out;
    b.sid = (uint8_t *)malloc(in->n + 1);
    b.counts = (uint64_t *)calloc((size_t)nthreads * nshards, sizeof(uint64_t));
    b.offs = (uint64_t *)malloc(sizeof(uint64_t) * (size_t)nthreads * nshards);
    b.idx = (uint32_t *)malloc(sizeof(uint32_t) * (in->n + 1));
    b.shard_off = (uint64_t *)malloc(sizeof(uint64_t) * (nshards + 1));
    sh_run(&b, nthreads, 0);
    uint64_t run = 0;  /* shard-major, slice-minor: stable in application order */
    for (uint32_t s = 0; s < nshards; s++) {
        b.shard_off[s] = run;
        for (uint32_t t = 0; t < nthreads; t++) {
            b.offs[(size_t)t * nshards + s] = run;
            run += b.counts[(size_t)t * nshards + s];
        }
    }
    b.shard_off[nshards] = run;
    sh_run(&b, nthreads, 1);
    sh_run(&b, nthreads, 2);
    free(b.sid); free(b.counts); free(b.offs); free(b.idx); free(b.shard_off);
    return 0;
}

/* ---- order-independent digest of crsql_changes rows (checksum of per-row checksums) ---- */
static uint64_t row_hash(uint64_t pk, uint32_t tcid, int64_t cv, int64_t dbv, int64_t cl, uint32_t seq,
                         uint32_t site, uint64_t ts, uint8_t vt, uint8_t vl, uint64_t v0, uint64_t v1) {
    uint64_t h = mix64(pk + 0x9E3779B97F4A7C15ULL);
    h = mix64(h ^ tcid);
    h = mix64(h ^ (uint64_t)cv);
    h = mix64(h ^ (uint64_t)dbv);
    h = mix64(h ^ (uint64_t)cl);
    h = mix64(h ^ (((uint64_t)seq << 32) | site));
    h = mix64(h ^ ts);
    h = mix64(h ^ (((uint64_t)vt << 8) | vl));
    h = mix64(h ^ v0);
    h = mix64(h ^ v1);
    return h;
}

/* out[0] = rows, out[1] = sum of row hashes, out[2] = xor of rotated row hashes */
static void digest_add(uint64_t out[3], uint64_t h) {
    out[0]++; out[1] += h; out[2] ^= (h << 17) | (h >> 47);
}

void of_rows_digest(const of_rows *o, uint64_t n, uint64_t out[3]) {
    out[0] = out[1] = out[2] = 0;
    for (uint64_t k = 0; k < n; k++)
        digest_add(out, row_hash(o->pk[k], o->table_cid[k], o->col_version[k], o->db_version[k], o->cl[k],
                                 o->seq[k], o->site[k], o->ts[k], o->val_type[k], o->val_len[k],
                                 o->val0[k], o->val1[k]));
}

/* digest of the rows of_export would emit (any order) */
void of_state_digest(const of_state *s, uint64_t out[3]) {
    for (uint64_t i = 0; i < s->cap; i++) {
        const of_row *r = &s->rows[i];
        if (!r->used) continue;
        int64_t L = row_L(r);
        if (r->has_sent)
            digest_add(out, row_hash(r->pk, r->table << 16, r->sent.cv, r->sent.dbv, L, r->sent.seq, r->sent.site,
                                     r->sent.ts, OF_NULL, 0, 0, 0));
        for (uint32_t k = 0; k < r->ncells; k++) {
            const of_cell *c = &r->cells[k];
            const uint64_t v1 = c->vlen == OF_LONG ? of_bytes_hash(s->arena + (c->v1 >> 24), c->v1 & 0xFFFFFFu) : c->v1;
            digest_add(out, row_hash(r->pk, (r->table << 16) | c->cid, c->cv, c->dbv, L, c->seq, c->site, c->ts,
                                     c->vtype, c->vlen, c->v0, v1));
        }
    }
}
