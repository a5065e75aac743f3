// process_multiple_changes and friends, host side (C++), over the device merge.
//
// Mirrors /root/reference/crates/corro-agent/src/agent/util.rs:
//   process_multiple_changes      :691-1037   (dedup passes, actor order, one apply per call,
//                                              per-actor gap snapshot, partial bookkeeping)
//   process_single_version        :488-538    (complete -> merge, incomplete -> buffer)
//   process_empty_version         :1040-1050  (crsql_set_db_version)
//   process_incomplete_version    :1053-1186  (buffer rows, merge seq ranges)
//   process_complete_version      :1189-1290  (impactful changes with the cumulative
//                                              crsql_rows_impacted() quirk)
//   process_fully_buffered_changes :541-688   (apply a version once all its seqs arrived)
// and generate_sync (corro-types/src/sync.rs:284-333). The merge itself is corro_apply_batch.
#include <array>
#include <algorithm>
#include <cstring>
#include <map>
#include <optional>
#include <set>
#include <string>
#include <tuple>
#include <vector>

#include "booked.h"
#include "corro_hip.h"

// engine.hip: adds per-table committed counts to the context (corro_table_committed)
void corro_detail_add_committed(corro_ctx *ctx, const uint64_t *counts, size_t n);

namespace corro {
int fail(int code, const std::string &msg);
int set_db_version(corro_ctx *ctx, uint32_t site, uint64_t version);
}  // namespace corro

using corro::fail;
using corro::Range;
using corro::RangeSet;
using ActorId = std::array<uint8_t, 16>;

namespace {

struct HostRow {  // one buffered change (__corro_buffered_changes row)
    uint64_t pk, v0, v1, ts;
    int64_t cv, dbv;
    uint32_t tcid, cl, seq, site;
    uint8_t vt, vl;
    std::string lv;  // a long TEXT/BLOB value's bytes (vl == CORRO_VAL_LONG)
};

bool is_long(uint8_t vt, uint8_t vl) { return vl == CORRO_VAL_LONG && (vt == CORRO_TEXT || vt == CORRO_BLOB); }

struct SeqBook {  // __corro_seq_bookkeeping rows of one (site, version)
    std::vector<Range> ranges;
    uint64_t last_seq = 0, ts = 0;
};

}  // namespace

struct corro_bookie {
    std::map<ActorId, corro::Booked> actors;                  // Bookie (agent.rs:1546-1598)
    std::map<std::pair<uint32_t, int64_t>, std::map<uint32_t, HostRow>> buffered;  // (site, dbv) -> seq -> row
    std::map<std::pair<uint32_t, uint64_t>, SeqBook> seqbook;  // (site, version)
    std::vector<std::pair<ActorId, uint64_t>> ready;           // fully buffered, to apply
    std::map<ActorId, uint32_t> site_of;                       // actor -> site ordinal
};

namespace {

ActorId actor_of(const uint8_t *p) {
    ActorId a;
    std::memcpy(a.data(), p, 16);
    return a;
}

struct Batch {  // application-order SoA assembled on the host
    std::vector<uint64_t> pk, v0, v1, ts, voff;
    std::vector<int64_t> cv, dbv;
    std::vector<uint32_t> tcid, cl, seq, site, vsz;
    std::vector<uint8_t> vt, vl;
    std::string data;  // long values' bytes
    bool any_long = false;
    void push(const HostRow &r) {
        pk.push_back(r.pk); v0.push_back(r.v0); v1.push_back(r.v1); ts.push_back(r.ts);
        cv.push_back(r.cv); dbv.push_back(r.dbv); tcid.push_back(r.tcid); cl.push_back(r.cl);
        seq.push_back(r.seq); site.push_back(r.site); vt.push_back(r.vt); vl.push_back(r.vl);
        voff.push_back(data.size());
        vsz.push_back((uint32_t)r.lv.size());
        if (is_long(r.vt, r.vl)) {
            data += r.lv;
            any_long = true;
        }
    }
    size_t size() const { return pk.size(); }
    corro_changes view() const {
        corro_changes c{};
        c.n = pk.size();
        c.pk = pk.data(); c.table_cid = tcid.data(); c.col_version = cv.data(); c.db_version = dbv.data();
        c.cl = cl.data(); c.seq = seq.data(); c.site = site.data(); c.val0 = v0.data(); c.val1 = v1.data();
        c.val_type = vt.data(); c.val_len = vl.data(); c.ts = ts.data();
        if (any_long) {
            c.val_off = voff.data();
            c.val_size = vsz.data();
            c.val_data = reinterpret_cast<const uint8_t *>(data.data());
            c.val_data_len = data.size();
        }
        return c;
    }
};

HostRow row_at(const corro_changes *in, uint64_t i, uint64_t ts) {
    HostRow r;
    r.pk = in->pk[i];
    r.tcid = in->table_cid[i];
    r.cv = in->col_version[i];
    r.dbv = in->db_version[i];
    r.cl = in->cl[i];
    r.seq = in->seq[i];
    r.site = in->site[i];
    r.v0 = in->val0[i];
    r.v1 = in->val1 ? in->val1[i] : 0;
    r.vt = in->val_type ? in->val_type[i] : (uint8_t)CORRO_INTEGER;
    r.vl = in->val_len ? in->val_len[i] : 0;
    r.ts = in->ts ? in->ts[i] : ts;
    // a long value whose span is malformed is passed on as it is (empty): the apply rejects it
    if (is_long(r.vt, r.vl) && in->val_off && in->val_size && in->val_data && in->val_size[i] > 16 &&
        in->val_off[i] <= in->val_data_len && in->val_size[i] <= in->val_data_len - in->val_off[i])
        r.lv.assign(reinterpret_cast<const char *>(in->val_data + in->val_off[i]), in->val_size[i]);
    return r;
}

// process_incomplete_version (util.rs:1053-1186): buffer the rows, merge the seq range into the
// seq bookkeeping. Returns the PartialVersion (seqs = the merged range only) or an error.
// Writes of one process_multiple_changes call that must not outlive a failed call: the reference
// makes them inside the call's single transaction (util.rs:749, :936), so they are staged here and
// applied only once the merge and the gap bookkeeping have succeeded.
struct Staged {
    std::vector<std::pair<uint32_t, uint64_t>> set_dbv;                      // crsql_set_db_version
    std::vector<HostRow> buffered;                                            // __corro_buffered_changes
    std::map<std::pair<uint32_t, uint64_t>, SeqBook> seqbook;                 // __corro_seq_bookkeeping
    SeqBook &seq(const corro_bookie *bk, uint32_t site, uint64_t version) {
        auto it = seqbook.find({site, version});
        if (it != seqbook.end()) return it->second;
        auto b = bk->seqbook.find({site, version});
        return seqbook.emplace(std::make_pair(site, version), b == bk->seqbook.end() ? SeqBook{} : b->second)
            .first->second;
    }
};

int process_incomplete(const corro_bookie *bk, Staged &st, const corro_changeset &cs, const corro_changes *in,
                       corro::PartialVersion &out) {
    for (uint64_t k = 0; k < cs.change_count; k++) st.buffered.push_back(row_at(in, cs.change_off + k, cs.ts));
    SeqBook &sb = st.seq(bk, cs.site, cs.version_start);
    const uint64_t s = cs.seq_start, e = cs.seq_end;
    RangeSet merged;
    std::vector<Range> keep;
    for (const Range &r : sb.ranges) {
        const bool hit = (r.first >= s && r.first <= e) || (r.first <= s && r.second >= e) ||
                         (r.first <= e && r.second >= e) || (r.second >= s && r.second <= e) ||
                         (r.first == e + 1 && r.second != 0) || (s > 0 && r.second == s - 1);
        if (hit) merged.insert(r.first, r.second);
        else keep.push_back(r);
    }
    merged.insert(s, e);
    if (merged.size() != 1) return fail(CORRO_E_INVALID, "deleted non-contiguous seq ranges");
    keep.push_back(*merged.ranges().begin());
    sb.ranges = keep;
    sb.last_seq = cs.last_seq;
    sb.ts = cs.ts;
    out = corro::PartialVersion();
    out.seqs = merged;
    out.last_seq = cs.last_seq;
    out.ts = cs.ts;
    return CORRO_OK;
}

void clear_buffered(corro_bookie *bk, uint32_t site, uint64_t vs, uint64_t ve) {
    for (auto it = bk->buffered.lower_bound({site, (int64_t)vs}); it != bk->buffered.end();) {
        if (it->first.first != site || (uint64_t)it->first.second > ve) break;
        it = bk->buffered.erase(it);
    }
    for (auto it = bk->seqbook.lower_bound({site, vs}); it != bk->seqbook.end();) {
        if (it->first.first != site || it->first.second > ve) break;
        it = bk->seqbook.erase(it);
    }
}

}  // namespace

extern "C" {

int corro_bookie_new(corro_bookie **out) {
    if (!out) return fail(CORRO_E_INVALID, "out is NULL");
    *out = new corro_bookie();
    return CORRO_OK;
}

void corro_bookie_free(corro_bookie *b) { delete b; }

int corro_process_multiple_changes(corro_ctx *ctx, corro_bookie *bk, const corro_changeset *cs, uint64_t ncs,
                                   const corro_changes *in, corro_process_out *out) {
    if (!ctx || !bk || (ncs && !cs) || !out) return fail(CORRO_E_INVALID, "NULL argument");
    if (ncs && (!out->known)) return fail(CORRO_E_INVALID, "out->known is required");
    const uint64_t nchanges = in ? in->n : 0;
    for (uint64_t i = 0; i < ncs; i++) {
        out->known[i] = CORRO_KNOWN_SKIPPED;
        if (cs[i].kind == CORRO_CS_FULL && cs[i].change_count &&
            (!in || cs[i].change_off + cs[i].change_count > nchanges))
            return fail(CORRO_E_INVALID, "changeset change span outside the batch");
    }
    if (out->impactful)
        for (uint64_t j = 0; j < nchanges; j++) out->impactful[j] = 0;

    auto versions_of = [](const corro_changeset &c) -> Range {
        if (c.kind == CORRO_CS_EMPTY_SET) return {0, 0};  // Changeset::versions() dummy (broadcast.rs:176-178)
        return {c.version_start, c.kind == CORRO_CS_FULL ? c.version_start : c.version_end};
    };
    auto seqs_of = [](const corro_changeset &c, Range &r) -> const Range * {
        if (c.kind != CORRO_CS_FULL) return nullptr;
        r = {c.seq_start, c.seq_end};
        return &r;
    };
    auto is_complete = [](const corro_changeset &c) {
        return c.kind != CORRO_CS_FULL || (c.seq_start == 0 && c.seq_end == c.last_seq);
    };
    auto is_empty = [](const corro_changeset &c) { return c.kind != CORRO_CS_FULL || c.change_count == 0; };

    // pass 1 (util.rs:704-739): batch-local dedup, then drop already-known versions
    std::set<std::tuple<ActorId, uint64_t, uint64_t, int, uint64_t, uint64_t>> seen;
    std::map<ActorId, std::vector<uint64_t>> unknown;  // BTreeMap<ActorId, _>: byte order
    for (uint64_t i = 0; i < ncs; i++) {
        const ActorId a = actor_of(cs[i].actor_id);
        const Range v = versions_of(cs[i]);
        Range sq;
        const Range *seqs = seqs_of(cs[i], sq);
        if (!seen.emplace(a, v.first, v.second, seqs ? 1 : 0, seqs ? sq.first : 0, seqs ? sq.second : 0).second)
            continue;
        corro::Booked &booked = bk->actors[a];  // Bookie::ensure
        bk->site_of[a] = cs[i].site;
        if (booked.contains_all(v.first, v.second, seqs)) continue;
        unknown[a].push_back(i);
    }

    // pass 2 (util.rs:765-884): per actor, in order
    Staged st;
    Batch batch;
    std::vector<std::pair<uint64_t, uint64_t>> applied;  // (changeset, first batch row)
    std::map<ActorId, std::vector<std::pair<Range, std::optional<corro::PartialVersion>>>> processed;
    for (auto &[actor, idxs] : unknown) {
        corro::Booked &booked = bk->actors[actor];
        const bool had_max = booked.has_max;
        const uint64_t max = booked.max;
        std::vector<std::pair<Range, std::optional<corro::PartialVersion>>> seen_local;  // RangeInclusiveMap
        auto seen_get = [&](uint64_t v) -> const std::optional<corro::PartialVersion> * {
            for (auto it = seen_local.rbegin(); it != seen_local.rend(); ++it)
                if (it->first.first <= v && v <= it->first.second) return &it->second;
            return nullptr;
        };
        for (uint64_t i : idxs) {
            const corro_changeset &c = cs[i];
            const Range v = versions_of(c);
            Range sq;
            const Range *seqs = seqs_of(c, sq);
            if (booked.contains_all(v.first, v.second, seqs)) continue;
            bool all_seen = true;
            for (uint64_t ver = v.first; ver <= v.second && all_seen; ver++) {
                const auto *p = seen_get(ver);
                if (!p) all_seen = false;
                else if (seqs && p->has_value()) all_seen = (*p)->seqs.contains_range(seqs->first, seqs->second);
                if (ver == UINT64_MAX) break;
            }
            if (all_seen) continue;

            std::optional<corro::PartialVersion> partial;
            if (is_complete(c) && is_empty(c)) {
                // process_empty_version only when end > booked max (util.rs:810-824)
                if (!had_max || v.second > max) st.set_dbv.emplace_back(c.site, v.second);
                out->known[i] = CORRO_KNOWN_CLEARED;
            } else {
                if (seqs && seqs->second < seqs->first) continue;  // invalid seqs (util.rs:826-831)
                bool bad = false;
                for (uint64_t k = 0; k < c.change_count; k++)
                    if (in->table_cid[c.change_off + k] == CORRO_TCID_UNKNOWN) bad = true;
                if (bad) {  // the INSERT fails, the version's SAVEPOINT rolls back (util.rs:839-860)
                    out->known[i] = CORRO_E_UNKNOWN_COLUMN;
                    continue;
                }
                if (is_complete(c)) {
                    applied.emplace_back(i, batch.size());
                    for (uint64_t k = 0; k < c.change_count; k++) batch.push(row_at(in, c.change_off + k, c.ts));
                    out->known[i] = CORRO_KNOWN_CURRENT;  // final value decided after the merge
                } else {
                    corro::PartialVersion p;
                    if (process_incomplete(bk, st, c, in, p) != CORRO_OK) {
                        out->known[i] = CORRO_E_INVALID;
                        continue;
                    }
                    partial = p;
                    out->known[i] = CORRO_KNOWN_PARTIAL;
                }
            }
            seen_local.emplace_back(v, partial);
            processed[actor].emplace_back(v, partial);
        }
    }

    // gap bookkeeping first, on copies of the actors' Booked (VersionsSnapshot, agent.rs:1108-1235): an
    // INSERT that would violate __corro_bookkeeping_gaps' key fails the whole call before the merge
    // has touched the state, as the transaction's rollback would undo it (util.rs:894-936)
    std::map<ActorId, corro::Booked> next;
    std::vector<std::pair<ActorId, uint64_t>> ready;
    for (auto &[actor, list] : processed) {
        corro::Booked nb = bk->actors[actor];
        RangeSet versions;
        for (auto &e : list) versions.insert(e.first.first, e.first.second);
        if (!nb.insert_db(versions, nullptr, nullptr))
            return fail(CORRO_E_INVALID, "UNIQUE constraint failed: __corro_bookkeeping_gaps.start");
        for (auto &e : list) {
            if (!e.second) continue;
            const uint64_t version = e.first.first;
            const corro::PartialVersion &p = nb.insert_partial(version, *e.second);
            if (p.seqs.gaps(0, p.last_seq).empty()) ready.emplace_back(actor, version);
        }
        next.emplace(actor, std::move(nb));
    }

    // the merge: one batch in application order
    std::vector<uint8_t> impact(batch.size(), 0);
    if (batch.size()) {
        corro_changes view = batch.view();
        corro_apply_out ao{};
        ao.impact = impact.data();
        int rc = corro_apply_batch(ctx, &view, CORRO_MEM_HOST, &ao);
        if (rc != CORRO_OK) {  // the transaction fails as a whole (util.rs:849-855)
            for (uint64_t i = 0; i < ncs; i++) out->known[i] = CORRO_KNOWN_SKIPPED;
            return rc;
        }
    }
    // commit: everything below only records what the successful transaction did
    for (const auto &[site, version] : st.set_dbv) {
        int rc = corro::set_db_version(ctx, site, version);
        if (rc != CORRO_OK) return rc;
    }
    // corro.changes.committed{table} (util.rs:533-535): every buffered change of an incomplete
    // version (:1101-1105), every impactful change of a complete one (:1254-1258, below)
    std::vector<uint64_t> committed;
    auto commit_count = [&](uint32_t tcid) {
        if ((tcid >> 16) >= committed.size()) committed.resize((tcid >> 16) + 1, 0);
        committed[tcid >> 16]++;
    };
    for (const HostRow &r : st.buffered) {  // ON CONFLICT (site_id, db_version, seq) DO NOTHING
        bk->buffered[{r.site, r.dbv}].emplace(r.seq, r);
        commit_count(r.tcid);
    }
    for (auto &[key, sb] : st.seqbook) bk->seqbook[key] = sb;
    // impactful changes: crsql_rows_impacted() is cumulative over the transaction, while
    // last_rows_impacted restarts at 0 for every version (util.rs:1218-1261)
    uint64_t cum = 0;
    for (size_t a = 0; a < applied.size(); a++) {
        const uint64_t ci = applied[a].first, row0 = applied[a].second;
        const corro_changeset &c = cs[ci];
        uint64_t last = 0;
        bool any = false;
        for (uint64_t k = 0; k < c.change_count; k++) {
            cum += impact[row0 + k];
            const bool hit = cum > last;
            last = cum;
            if (hit) {
                any = true;
                if (out->impactful) out->impactful[c.change_off + k] = 1;
                commit_count(in->table_cid[c.change_off + k]);
            }
        }
        out->known[ci] = any ? CORRO_KNOWN_CURRENT : CORRO_KNOWN_CLEARED;
        if (!c.change_count) out->known[ci] = CORRO_KNOWN_CLEARED;
        // check_buffered_meta_to_clear (util.rs:513-520, :1292-1303)
        clear_buffered(bk, c.site, c.version_start, c.version_start);
    }
    // per-actor gap snapshot commit, then partials (util.rs:936-1008)
    for (auto &[actor, nb] : next) bk->actors[actor] = std::move(nb);
    for (auto &r : ready) bk->ready.push_back(r);
    out->n_ready = ready.size();
    corro_detail_add_committed(ctx, committed.data(), committed.size());
    return CORRO_OK;
}

int corro_bookie_take_ready(corro_bookie *bk, uint8_t *actors, uint64_t *versions, uint64_t cap, uint64_t *count) {
    if (!bk || !count) return fail(CORRO_E_INVALID, "NULL argument");
    const uint64_t n = bk->ready.size();
    *count = n;
    if (cap < n) return CORRO_OK;  // sizing call
    for (uint64_t k = 0; k < n; k++) {
        if (actors) std::memcpy(actors + 16 * k, bk->ready[k].first.data(), 16);
        if (versions) versions[k] = bk->ready[k].second;
    }
    bk->ready.clear();
    return CORRO_OK;
}

// process_fully_buffered_changes (util.rs:541-688)
int corro_process_fully_buffered(corro_ctx *ctx, corro_bookie *bk, const uint8_t *actor_id, uint64_t version,
                                 int *impacted) {
    if (!ctx || !bk || !actor_id) return fail(CORRO_E_INVALID, "NULL argument");
    if (impacted) *impacted = 0;
    const ActorId a = actor_of(actor_id);
    auto bit = bk->actors.find(a);
    auto sit = bk->site_of.find(a);
    if (bit == bk->actors.end() || sit == bk->site_of.end()) return CORRO_OK;  // "version not found in cache"
    corro::Booked &booked = bit->second;
    auto pit = booked.partials.find(version);
    if (pit == booked.partials.end()) return CORRO_OK;
    if (!pit->second.seqs.gaps(0, pit->second.last_seq).empty()) return CORRO_OK;  // gaps: abort
    const uint32_t site = sit->second;
    Batch batch;
    auto rows = bk->buffered.find({site, (int64_t)version});
    if (rows != bk->buffered.end())
        for (auto &kv : rows->second) batch.push(kv.second);  // ORDER BY db_version, seq
    RangeSet v;
    v.insert(version, version);
    corro::Booked nb = booked;  // committed only with the merge (one transaction, util.rs:560-676)
    if (!nb.insert_db(v, nullptr, nullptr))
        return fail(CORRO_E_INVALID, "UNIQUE constraint failed: __corro_bookkeeping_gaps.start");
    std::vector<uint8_t> impact(batch.size(), 0);
    if (batch.size()) {
        corro_changes view = batch.view();
        corro_apply_out ao{};
        ao.impact = impact.data();
        int rc = corro_apply_batch(ctx, &view, CORRO_MEM_HOST, &ao);
        if (rc != CORRO_OK) return rc;
    }
    clear_buffered(bk, site, version, version);
    booked = std::move(nb);
    uint64_t total = 0;
    for (uint8_t x : impact) total += x;
    if (impacted) *impacted = total > 0;
    return CORRO_OK;
}

// ---- per-actor Booked views -------------------------------------------------------------------
int corro_bookie_last(corro_bookie *bk, const uint8_t *actor_id, int64_t *max) {
    if (!bk || !actor_id || !max) return fail(CORRO_E_INVALID, "NULL argument");
    auto it = bk->actors.find(actor_of(actor_id));
    *max = (it == bk->actors.end() || !it->second.has_max) ? -1 : (int64_t)it->second.max;
    return CORRO_OK;
}

int corro_bookie_needed(corro_bookie *bk, const uint8_t *actor_id, uint64_t *start, uint64_t *end, uint64_t cap,
                        uint64_t *count) {
    if (!bk || !actor_id || !count) return fail(CORRO_E_INVALID, "NULL argument");
    auto it = bk->actors.find(actor_of(actor_id));
    uint64_t k = 0;
    if (it != bk->actors.end())
        for (const auto &r : it->second.needed.ranges()) {
            if (k < cap && start && end) {
                start[k] = r.first;
                end[k] = r.second;
            }
            k++;
        }
    *count = k;
    return CORRO_OK;
}

int corro_bookie_contains_all(corro_bookie *bk, const uint8_t *actor_id, uint64_t start, uint64_t end,
                              int has_seqs, uint64_t seq_start, uint64_t seq_end, int *result) {
    if (!bk || !actor_id || !result) return fail(CORRO_E_INVALID, "NULL argument");
    auto it = bk->actors.find(actor_of(actor_id));
    if (it == bk->actors.end()) {
        corro::Booked empty;
        Range sq{seq_start, seq_end};
        *result = empty.contains_all(start, end, has_seqs ? &sq : nullptr);
        return CORRO_OK;
    }
    Range sq{seq_start, seq_end};
    *result = it->second.contains_all(start, end, has_seqs ? &sq : nullptr);
    return CORRO_OK;
}

// __corro_seq_bookkeeping rows of one (actor, version) as handle_need reads them
// (corro-agent/src/api/peer/mod.rs:505-511, :640-667): seq ranges, last_seq (-1 = no rows), ts.
int corro_bookie_seq_bookkeeping(corro_bookie *bk, const uint8_t *actor_id, uint64_t version, uint64_t *start,
                                 uint64_t *end, uint64_t cap, uint64_t *count, int64_t *last_seq, uint64_t *ts) {
    if (!bk || !actor_id || !count || !last_seq || !ts) return fail(CORRO_E_INVALID, "NULL argument");
    *count = 0;
    *last_seq = -1;
    *ts = 0;
    auto so = bk->site_of.find(actor_of(actor_id));
    if (so == bk->site_of.end()) return CORRO_OK;
    auto it = bk->seqbook.find({so->second, version});
    if (it == bk->seqbook.end()) return CORRO_OK;
    std::vector<Range> rs = it->second.ranges;
    std::sort(rs.begin(), rs.end());
    uint64_t k = 0;
    for (const Range &r : rs) {
        if (k < cap && start && end) {
            start[k] = r.first;
            end[k] = r.second;
        }
        k++;
    }
    *count = k;
    *last_seq = (int64_t)it->second.last_seq;
    *ts = it->second.ts;
    return CORRO_OK;
}

// versions of `actor` in [vstart, vend] with buffered rows (the EXISTS(__corro_buffered_changes)
// probe of handle_need, peer/mod.rs:466-492), ascending; *count = all of them, at most cap written.
int corro_bookie_buffered_versions(corro_bookie *bk, const uint8_t *actor_id, uint64_t vstart, uint64_t vend,
                                   uint64_t *versions, uint64_t cap, uint64_t *count) {
    if (!bk || !actor_id || !count || (cap && !versions)) return fail(CORRO_E_INVALID, "NULL argument");
    *count = 0;
    auto so = bk->site_of.find(actor_of(actor_id));
    if (so == bk->site_of.end() || vstart > vend || vstart > (uint64_t)INT64_MAX) return CORRO_OK;
    uint64_t k = 0;
    for (auto it = bk->buffered.lower_bound({so->second, (int64_t)vstart}); it != bk->buffered.end(); ++it) {
        if (it->first.first != so->second || (uint64_t)it->first.second > vend) break;
        if (it->second.empty()) continue;
        if (k < cap) versions[k] = (uint64_t)it->first.second;
        k++;
    }
    *count = k;
    return CORRO_OK;
}

// __corro_buffered_changes rows of (actor, version) with seq in [seq_start, seq_end], seq
// ascending (peer/mod.rs:513-531, :672-693). *count = all matching rows; at most cap are written.
int corro_bookie_buffered(corro_bookie *bk, const uint8_t *actor_id, uint64_t version, uint64_t seq_start,
                          uint64_t seq_end, corro_rows *o, uint64_t cap, uint64_t *count) {
    if (!bk || !actor_id || !count || (cap && !o)) return fail(CORRO_E_INVALID, "NULL argument");
    *count = 0;
    auto so = bk->site_of.find(actor_of(actor_id));
    if (so == bk->site_of.end()) return CORRO_OK;
    auto it = bk->buffered.find({so->second, (int64_t)version});
    if (it == bk->buffered.end() || seq_start > seq_end || seq_start > 0xFFFFFFFFULL) return CORRO_OK;
    const uint32_t hi = seq_end > 0xFFFFFFFFULL ? 0xFFFFFFFFu : (uint32_t)seq_end;
    uint64_t k = 0;
    for (auto r = it->second.lower_bound((uint32_t)seq_start); r != it->second.end() && r->first <= hi; ++r, ++k) {
        if (k >= cap) continue;
        const HostRow &h = r->second;
        if (o->pk) o->pk[k] = h.pk;
        if (o->table_cid) o->table_cid[k] = h.tcid;
        if (o->col_version) o->col_version[k] = h.cv;
        if (o->db_version) o->db_version[k] = h.dbv;
        if (o->cl) o->cl[k] = h.cl;
        if (o->seq) o->seq[k] = h.seq;
        if (o->site) o->site[k] = h.site;
        if (o->ts) o->ts[k] = h.ts;
        if (o->val0) o->val0[k] = h.v0;
        if (o->val1) o->val1[k] = h.v1;
        if (o->val_type) o->val_type[k] = h.vt;
        if (o->val_len) o->val_len[k] = h.vl;
    }
    *count = k;
    return CORRO_OK;
}

// bytes of a buffered long value (the row of (actor, version, seq)); *len = its length (0: none)
int corro_bookie_buffered_value(corro_bookie *bk, const uint8_t *actor_id, uint64_t version, uint64_t seq,
                                uint8_t *out, uint64_t cap, uint64_t *len) {
    if (!bk || !actor_id || !len || (cap && !out)) return fail(CORRO_E_INVALID, "NULL argument");
    *len = 0;
    auto so = bk->site_of.find(actor_of(actor_id));
    if (so == bk->site_of.end() || seq > 0xFFFFFFFFULL) return CORRO_OK;
    auto it = bk->buffered.find({so->second, (int64_t)version});
    if (it == bk->buffered.end()) return CORRO_OK;
    auto r = it->second.find((uint32_t)seq);
    if (r == it->second.end()) return CORRO_OK;
    const std::string &lv = r->second.lv;
    *len = lv.size();
    std::memcpy(out, lv.data(), std::min<uint64_t>(cap, lv.size()));
    return CORRO_OK;
}

// partial seqs of one version: ranges received so far + last_seq (-1 last_seq = no partial)
int corro_bookie_partial(corro_bookie *bk, const uint8_t *actor_id, uint64_t version, uint64_t *start,
                         uint64_t *end, uint64_t cap, uint64_t *count, int64_t *last_seq) {
    if (!bk || !actor_id || !count || !last_seq) return fail(CORRO_E_INVALID, "NULL argument");
    *count = 0;
    *last_seq = -1;
    auto it = bk->actors.find(actor_of(actor_id));
    if (it == bk->actors.end()) return CORRO_OK;
    auto p = it->second.partials.find(version);
    if (p == it->second.partials.end()) return CORRO_OK;
    uint64_t k = 0;
    for (const auto &r : p->second.seqs.ranges()) {
        if (k < cap && start && end) {
            start[k] = r.first;
            end[k] = r.second;
        }
        k++;
    }
    *count = k;
    *last_seq = (int64_t)p->second.last_seq;
    return CORRO_OK;
}

// generate_sync (sync.rs:284-333) as CSR over actors with a head. pass 0 fills the four counts;
// pass 1 fills caller-sized arrays.
int corro_generate_sync(corro_bookie *bk, const uint8_t *self_actor, corro_sync_state *o, int pass) {
    (void)self_actor;
    if (!bk || !o) return fail(CORRO_E_INVALID, "NULL argument");
    uint64_t na = 0, nn = 0, np = 0, ns = 0;
    for (const auto &[actor, booked] : bk->actors) {
        if (!booked.has_max) continue;  // last() is None: skipped
        if (pass == 1) {
            std::memcpy(o->actor_ids + 16 * na, actor.data(), 16);
            o->heads[na] = booked.max;
            o->need_off[na] = nn;
            o->partial_off[na] = np;
        }
        for (const auto &r : booked.needed.ranges()) {
            if (pass == 1) {
                o->need_start[nn] = r.first;
                o->need_end[nn] = r.second;
            }
            nn++;
        }
        for (const auto &[v, p] : booked.partials) {
            if (p.is_complete()) continue;  // "don't set partial if it is effectively complete"
            if (pass == 1) {
                o->partial_ver[np] = v;
                o->pseq_off[np] = ns;
            }
            for (const auto &g : p.seqs.gaps(0, p.last_seq)) {
                if (pass == 1) {
                    o->pseq_start[ns] = g.first;
                    o->pseq_end[ns] = g.second;
                }
                ns++;
            }
            np++;
        }
        na++;
    }
    if (pass == 1) {
        o->need_off[na] = nn;
        o->partial_off[na] = np;
        o->pseq_off[np] = ns;
    }
    o->n_actors = na;
    o->n_need = nn;
    o->n_partials = np;
    o->n_pseqs = ns;
    return CORRO_OK;
}

}  // extern "C"
