/*
 * oracle/ranges.c — TEST INFRASTRUCTURE ONLY (the checker, never the product).
 *
 * Straight-line CPU restatements of
 *   - rangemap 1.5.1 `RangeInclusiveSet<u64>` (Cargo.lock:3471): sorted, disjoint ranges where
 *     touching ranges coalesce ([1..=3] + [4..=5] -> [1..=5]) because CrsqlDbVersion/CrsqlSeq
 *     implement `StepLite` (corro-base-types/src/lib.rs:34-42);
 *   - `SyncStateV1::compute_available_needs` (corro-types/src/sync.rs:127-249);
 *   - `VersionsSnapshot::compute_gaps_change` + `insert_db` (corro-types/src/agent.rs:1108-1235).
 * Pinned by the reference's own unit tests: sync.rs:386-500 and agent.rs:1605-1868
 * (tests/golden/sync_kats.json, tests/golden/gaps_kats.json).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

typedef struct { uint64_t s, e; } rg;
typedef struct { rg *r; uint64_t n, cap; } rset;

static void rs_init(rset *x) { x->r = NULL; x->n = x->cap = 0; }
static void rs_free(rset *x) { free(x->r); x->r = NULL; x->n = x->cap = 0; }
static void rs_push(rset *x, uint64_t s, uint64_t e) {
    if (x->n == x->cap) { x->cap = x->cap ? 2 * x->cap : 8; x->r = (rg *)realloc(x->r, x->cap * sizeof(rg)); }
    x->r[x->n].s = s; x->r[x->n].e = e; x->n++;
}

/* insert [s,e] coalescing overlapping and touching ranges */
static void rs_insert(rset *x, uint64_t s, uint64_t e) {
    rset out; rs_init(&out);
    uint64_t i = 0;
    while (i < x->n && x->r[i].e != UINT64_MAX && x->r[i].e + 1 < s) { rs_push(&out, x->r[i].s, x->r[i].e); i++; }
    uint64_t ns = s, ne = e;
    while (i < x->n && (e == UINT64_MAX || x->r[i].s <= e + 1)) {
        if (x->r[i].s < ns) ns = x->r[i].s;
        if (x->r[i].e > ne) ne = x->r[i].e;
        i++;
    }
    rs_push(&out, ns, ne);
    while (i < x->n) { rs_push(&out, x->r[i].s, x->r[i].e); i++; }
    free(x->r); *x = out;
}

static void rs_remove(rset *x, uint64_t s, uint64_t e) {
    rset out; rs_init(&out);
    for (uint64_t i = 0; i < x->n; i++) {
        rg a = x->r[i];
        if (a.e < s || a.s > e) { rs_push(&out, a.s, a.e); continue; }
        if (a.s < s) rs_push(&out, a.s, s - 1);
        if (a.e > e) rs_push(&out, e + 1, a.e);
    }
    free(x->r); *x = out;
}

static int rs_contains(const rset *x, uint64_t v) {
    for (uint64_t i = 0; i < x->n; i++) if (x->r[i].s <= v && v <= x->r[i].e) return 1;
    return 0;
}

static const rg *rs_get(const rset *x, uint64_t v) {
    for (uint64_t i = 0; i < x->n; i++) if (x->r[i].s <= v && v <= x->r[i].e) return &x->r[i];
    return NULL;
}

/* ------------------------- compute_available_needs ------------------------- */

typedef struct { uint64_t nn, ns; } cnt;

static void emit_full(of_needs_out *o, int fill, uint64_t e, cnt *c, uint64_t s, uint64_t en) {
    if (fill) {
        uint64_t k = o->need_off[e] + c->nn;
        o->kind[k] = 0; o->start[k] = s; o->end[k] = en;
        o->sr_off[k] = o->seq_off[e] + c->ns; o->sr_n[k] = 0;
    }
    c->nn++;
}

void of_needs(const of_sync_entries *in, of_needs_out *o, int fill) {
    for (uint64_t e = 0; e < in->n; e++) {
        cnt c = {0, 0};
        uint64_t head = in->their_head[e];
        /* haves = {1..=head} - their need - their partial versions (sync.rs:141-162) */
        rset haves; rs_init(&haves);
        rs_insert(&haves, 1, head);
        for (uint64_t k = in->tn_off[e]; k < in->tn_off[e + 1]; k++) rs_remove(&haves, in->tn_start[k], in->tn_end[k]);
        for (uint64_t k = in->tp_off[e]; k < in->tp_off[e + 1]; k++) rs_remove(&haves, in->tp_ver[k], in->tp_ver[k]);

        /* Full(our_need ∩ haves) in our range order (sync.rs:164-174) */
        for (uint64_t k = in->on_off[e]; k < in->on_off[e + 1]; k++) {
            uint64_t s = in->on_start[k], t = in->on_end[k];
            for (uint64_t h = 0; h < haves.n; h++) {
                if (haves.r[h].e < s || haves.r[h].s > t) continue;
                uint64_t a = haves.r[h].s > s ? haves.r[h].s : s;
                uint64_t b = haves.r[h].e < t ? haves.r[h].e : t;
                emit_full(o, fill, e, &c, a, b);
            }
        }
        /* our partials (sync.rs:176-226) */
        for (uint64_t k = in->op_off[e]; k < in->op_off[e + 1]; k++) {
            uint64_t v = in->op_ver[k];
            if (rs_contains(&haves, v)) {
                if (fill) {
                    uint64_t q = o->need_off[e] + c.nn;
                    o->kind[q] = 1; o->start[q] = v; o->end[q] = v;
                    o->sr_off[q] = o->seq_off[e] + c.ns;
                    o->sr_n[q] = in->ops_off[k + 1] - in->ops_off[k];
                    for (uint64_t j = in->ops_off[k]; j < in->ops_off[k + 1]; j++) {
                        o->s_start[o->sr_off[q] + (j - in->ops_off[k])] = in->ops_start[j];
                        o->s_end[o->sr_off[q] + (j - in->ops_off[k])] = in->ops_end[j];
                    }
                }
                c.ns += in->ops_off[k + 1] - in->ops_off[k];
                c.nn++;
                continue;
            }
            /* does the other side have a partial at v? */
            int64_t tk = -1;
            for (uint64_t j = in->tp_off[e]; j < in->tp_off[e + 1]; j++)
                if (in->tp_ver[j] == v) { tk = (int64_t)j; break; }
            if (tk < 0) continue;
            int have_end = 0; uint64_t end = 0;
            for (uint64_t j = in->tps_off[tk]; j < in->tps_off[tk + 1]; j++)
                if (!have_end || in->tps_end[j] > end) { end = in->tps_end[j]; have_end = 1; }
            for (uint64_t j = in->ops_off[k]; j < in->ops_off[k + 1]; j++)
                if (!have_end || in->ops_end[j] > end) { end = in->ops_end[j]; have_end = 1; }
            if (!have_end) continue;
            rset sh; rs_init(&sh);
            rs_insert(&sh, 0, end);
            for (uint64_t j = in->tps_off[tk]; j < in->tps_off[tk + 1]; j++) rs_remove(&sh, in->tps_start[j], in->tps_end[j]);
            uint64_t nseq = 0, base = fill ? o->seq_off[e] + c.ns : 0;
            for (uint64_t j = in->ops_off[k]; j < in->ops_off[k + 1]; j++) {
                uint64_t s = in->ops_start[j], t = in->ops_end[j];
                for (uint64_t h = 0; h < sh.n; h++) {
                    if (sh.r[h].e < s || sh.r[h].s > t) continue;
                    if (fill) {
                        o->s_start[base + nseq] = sh.r[h].s > s ? sh.r[h].s : s;
                        o->s_end[base + nseq] = sh.r[h].e < t ? sh.r[h].e : t;
                    }
                    nseq++;
                }
            }
            rs_free(&sh);
            if (nseq) {
                if (fill) {
                    uint64_t q = o->need_off[e] + c.nn;
                    o->kind[q] = 1; o->start[q] = v; o->end[q] = v;
                    o->sr_off[q] = base; o->sr_n[q] = nseq;
                }
                c.nn++; c.ns += nseq;
            }
        }
        /* missing tail (sync.rs:229-245) */
        int64_t ours = in->our_head[e];
        if (ours < 0) emit_full(o, fill, e, &c, 1, head);
        else if (head > (uint64_t)ours) emit_full(o, fill, e, &c, (uint64_t)ours + 1, head);
        rs_free(&haves);
        if (!fill) { o->need_count[e] = c.nn; o->seq_count[e] = c.ns; }
    }
}

/* ------------------------- gap bookkeeping ------------------------- */

struct of_booked { rset needed; int has_max; uint64_t max; };

of_booked *of_booked_new(void) { of_booked *b = (of_booked *)calloc(1, sizeof(of_booked)); rs_init(&b->needed); return b; }
void of_booked_free(of_booked *b) { if (b) { rs_free(&b->needed); free(b); } }

static void ins_unique(rset *list, uint64_t s, uint64_t e) {  /* HashSet<RangeInclusive> insert */
    for (uint64_t i = 0; i < list->n; i++) if (list->r[i].s == s && list->r[i].e == e) return;
    rs_push(list, s, e);
}

int of_booked_insert_db(of_booked *b, const uint64_t *start, const uint64_t *end, uint64_t n) {
    rset versions; rs_init(&versions);
    for (uint64_t i = 0; i < n; i++) rs_insert(&versions, start[i], end[i]);
    rset insert_set; rs_init(&insert_set);
    rset remove_list; rs_init(&remove_list);
    int has_max = b->has_max; uint64_t max = b->max;
    for (uint64_t i = 0; i < versions.n; i++) {
        uint64_t s = versions.r[i].s, e = versions.r[i].e;
        if (!has_max || e > max) { max = e; has_max = 1; }
        for (uint64_t k = 0; k < b->needed.n; k++) {
            rg r = b->needed.r[k];
            if (r.e < s || r.s > e) continue;
            rs_insert(&insert_set, r.s, r.e); ins_unique(&remove_list, r.s, r.e);
        }
        const rg *p = s > 0 ? rs_get(&b->needed, s - 1) : NULL;
        if (p) { rg r = *p; rs_insert(&insert_set, r.s, r.e); ins_unique(&remove_list, r.s, r.e); }
        p = e < UINT64_MAX ? rs_get(&b->needed, e + 1) : NULL;
        if (p) { rg r = *p; rs_insert(&insert_set, r.s, r.e); ins_unique(&remove_list, r.s, r.e); }
        uint64_t current_max = b->has_max ? b->max : 0;  /* self.max, not the running max */
        uint64_t gap_start = current_max + 1;
        if (gap_start < s) {
            rs_insert(&insert_set, gap_start, s);
            for (uint64_t k = 0; k < b->needed.n; k++) {
                rg r = b->needed.r[k];
                if (r.e < gap_start || r.s > s) continue;
                rs_insert(&insert_set, r.s, r.e); ins_unique(&remove_list, r.s, r.e);
            }
        }
    }
    for (uint64_t i = 0; i < versions.n; i++) rs_remove(&insert_set, versions.r[i].s, versions.r[i].e);

    for (uint64_t i = 0; i < remove_list.n; i++) rs_remove(&b->needed, remove_list.r[i].s, remove_list.r[i].e);
    int rc = 0;
    for (uint64_t i = 0; i < insert_set.n; i++) {
        /* __corro_bookkeeping_gaps has PK (actor_id, start): a duplicate start fails the insert */
        for (uint64_t k = 0; k < b->needed.n; k++) if (b->needed.r[k].s == insert_set.r[i].s) rc = -1;
        rs_insert(&b->needed, insert_set.r[i].s, insert_set.r[i].e);
    }
    b->has_max = has_max; b->max = max;
    rs_free(&versions); rs_free(&insert_set); rs_free(&remove_list);
    return rc;
}

uint64_t of_booked_needed_len(const of_booked *b) { return b->needed.n; }
void of_booked_needed(const of_booked *b, uint64_t *start, uint64_t *end) {
    for (uint64_t i = 0; i < b->needed.n; i++) { start[i] = b->needed.r[i].s; end[i] = b->needed.r[i].e; }
}
int64_t of_booked_max(const of_booked *b) { return b->has_max ? (int64_t)b->max : -1; }
int of_booked_contains(const of_booked *b, uint64_t v) {
    /* BookedVersions::contains_version (agent.rs:1353-1362) */
    return !rs_contains(&b->needed, v) && (b->has_max ? b->max : 0) >= v;
}
