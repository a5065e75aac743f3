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
 * REAL numeric (-0.0 == 0.0), TEXT/BLOB memcmp then length, NULL == NULL.
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
    free(s->rows); free(s->dbv); free(s->site_ids); free(s);
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

/* compare incoming value a against local value b: >0 a greater, <0 b greater, 0 equal */
static int value_cmp(uint8_t ta, uint64_t a0, uint64_t a1, uint8_t la,
                     uint8_t tb, uint64_t b0, uint64_t b1, uint8_t lb) {
    if (ta != tb) return rank_of(ta) > rank_of(tb) ? 1 : -1;
    switch (ta) {
    case OF_INTEGER: {
        int64_t x = (int64_t)a0, y = (int64_t)b0;
        return x > y ? 1 : (x < y ? -1 : 0);
    }
    case OF_REAL: {
        double x, y;
        memcpy(&x, &a0, 8); memcpy(&y, &b0, 8);
        return x > y ? 1 : (x < y ? -1 : 0);
    }
    case OF_TEXT:
    case OF_BLOB:
        if (a0 != b0) return a0 > b0 ? 1 : -1;
        if (a1 != b1) return a1 > b1 ? 1 : -1;
        return la > lb ? 1 : (la < lb ? -1 : 0);
    default:
        return 0;  /* NULL == NULL */
    }
}

static void fill_cell(of_cell *c, const of_changes *in, uint64_t i) {
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

static void set_cell(of_row *r, const of_changes *in, uint64_t i) {
    uint32_t cid = in->table_cid[i] & 0xFFFFu;
    of_cell *c = find_cell(r, cid);
    if (!c) c = add_cell(r);
    fill_cell(c, in, i);
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
        fill_cell(&r->sent, in, i);                         /* sentinel cv = x.cv */
        r->sent.cid = 0; r->sent.vtype = OF_NULL; r->sent.v0 = r->sent.v1 = 0; r->sent.vlen = 0;
        return 1;
    }
    if (cid == 0) {                                         /* rule 3: pk-only / resurrect */
        if (cl > L) {
            zero_cells(r);
            r->has_sent = 1;
            fill_cell(&r->sent, in, i);
            r->sent.cid = 0; r->sent.vtype = OF_NULL; r->sent.v0 = r->sent.v1 = 0; r->sent.vlen = 0;
            return 1;
        }
        return 0;
    }
    if (cl > L) {                                           /* rule 4: needs resurrect */
        int imp = 0;
        if (L > 0 || cl > 1) {
            zero_cells(r);
            r->has_sent = 1;
            fill_cell(&r->sent, in, i);
            r->sent.cv = cl;
            r->sent.cid = 0; r->sent.vtype = OF_NULL; r->sent.v0 = r->sent.v1 = 0; r->sent.vlen = 0;
            imp = 1;
        }
        set_cell(r, in, i);
        return imp + 1;
    }
    /* cl == L : last-writer-wins */
    of_cell *c = find_cell(r, cid);
    if (c) {
        int64_t cv = in->col_version[i];
        if (cv < c->cv) return 0;
        if (cv == c->cv) {
            int vc = value_cmp(in->val_type ? in->val_type[i] : OF_INTEGER,
                               in->val0 ? in->val0[i] : 0, in->val1 ? in->val1[i] : 0,
                               in->val_len ? in->val_len[i] : 0,
                               c->vtype, c->v0, c->v1, c->vlen);
            if (vc < 0) return 0;
            if (vc == 0) {
                /* merge-equal-values: bigger writer site id wins (memcmp of 16 bytes) */
                const uint8_t *a = s->site_ids + 16 * (size_t)site;
                const uint8_t *b = s->site_ids + 16 * (size_t)c->site;
                if (memcmp(a, b, 16) <= 0) return 0;
            }
        }
    }
    set_cell(r, in, i);
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
