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
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <exception>
#include <functional>
#include <mutex>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <optional>
#include <set>
#include <stdexcept>
#include <string>
#include <thread>
#include <tuple>
#include <vector>

#include "agent_dev.h"
#include "booked.h"
#include "corro_hip.h"

// engine.hip: adds per-table committed counts to the context (corro_table_committed)
void corro_detail_add_committed(corro_ctx *ctx, const uint64_t *counts, size_t n);

namespace corro {
int fail(int code, const std::string &msg);
int set_db_version(corro_ctx *ctx, uint32_t site, uint64_t version);
int set_db_versions(corro_ctx *ctx, const std::vector<std::pair<uint32_t, uint64_t>> &sv);
uint64_t ctx_write_mark(const corro_ctx *ctx);   // engine.hip: committed applies + set_db_version passes
void ctx_poison(corro_ctx *ctx, const char *why);  // engine.hip
bool ctx_poisoned(const corro_ctx *ctx);            // engine.hip
}  // namespace corro

#define TRY_RC(x)                        \
    do {                                 \
        int rc_ = (x);                   \
        if (rc_ != CORRO_OK) return rc_; \
    } while (0)

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

// Failure injection for the atomicity tests: CORRO_FAULT names the steps that fail (comma-separated;
// read on every call, so a test arms and disarms it around one call). (internal.h holds the same
// helper for the HIP translation units; this one is compiled without the HIP headers.)
bool fault_armed(const char *name) {
    const char *e = std::getenv("CORRO_FAULT");
    if (!e || !*e) return false;
    const std::string s = std::string(",") + e + ",";
    return s.find(std::string(",") + name + ",") != std::string::npos;
}

struct SeqBook {  // __corro_seq_bookkeeping rows of one (site, version)
    corro::SmallVec<Range, 2> ranges;  // (one or two ranges inline: no allocation per partial version)
    uint64_t last_seq = 0, ts = 0;
};

// The __corro_buffered_changes rows of one (site, db_version): one vector sorted by seq, unique seqs
// (a node per version, not per row: a call can buffer millions of rows).
using BufRows = std::vector<HostRow>;

bool seq_less(const HostRow &a, const HostRow &b) { return a.seq < b.seq; }

// INSERT ... ON CONFLICT (site_id, db_version, seq) DO NOTHING of rows [first, last) into dst:
// the first row of each seq wins (rows already stored, then earlier rows of the batch)
void buf_insert(BufRows &dst, HostRow *first, HostRow *last) {
    std::stable_sort(first, last, seq_less);
    BufRows out;
    out.reserve(dst.size() + (size_t)(last - first));
    auto a = dst.begin();
    for (HostRow *b = first; b != last;) {
        if (a != dst.end() && a->seq <= b->seq) {
            if (a->seq == b->seq)  // the stored row wins; drop every batch row of that seq
                for (const uint32_t q = b->seq; b != last && b->seq == q;) ++b;
            out.push_back(std::move(*a++));
            continue;
        }
        out.push_back(std::move(*b));
        const uint32_t q = b->seq;
        for (++b; b != last && b->seq == q;) ++b;  // later rows of the same seq
    }
    for (; a != dst.end(); ++a) out.push_back(std::move(*a));
    dst.swap(out);
}

BufRows::const_iterator buf_lower(const BufRows &v, uint32_t seq) {
    return std::lower_bound(v.begin(), v.end(), seq, [](const HostRow &r, uint32_t q) { return r.seq < q; });
}

// Rows of one (site, db_version) in the bookie's device pool (bufpool.hip): pool rows [off, off + n)
// hold seqs seq0 .. seq0 + n - 1 in order. A key's segments are sorted by seq0 and disjoint.
struct PoolSeg {
    uint64_t off;
    uint32_t seq0, n;
};
constexpr uint64_t SEG_PENDING = 1ULL << 63;  // off = SEG_PENDING | copy job (until the copy runs)

// A key's segments: sorted by seq0; the first two inline (a version arrives in a few pieces, and a
// call buffers tens of thousands of keys: no allocation per key)
class SegList {
  public:
    SegList() = default;
    SegList(const SegList &o) : n_(o.n_), more_(o.more_) { std::copy(o.in_, o.in_ + 2, in_); }
    SegList(SegList &&o) noexcept : n_(o.n_), more_(std::move(o.more_)) {
        std::copy(o.in_, o.in_ + 2, in_);
        o.n_ = 0;
    }
    SegList &operator=(SegList o) noexcept {
        n_ = o.n_;
        std::copy(o.in_, o.in_ + 2, in_);
        more_.swap(o.more_);
        return *this;
    }
    size_t size() const { return n_; }
    bool empty() const { return n_ == 0; }
    PoolSeg *begin() { return n_ <= 2 ? in_ : more_.data(); }
    PoolSeg *end() { return begin() + n_; }
    const PoolSeg *begin() const { return n_ <= 2 ? in_ : more_.data(); }
    const PoolSeg *end() const { return begin() + n_; }
    void clear() {
        n_ = 0;
        more_.clear();
    }
    // insert keeping seq0 order
    void insert_sorted(const PoolSeg &g) {
        if (n_ < 2) {
            in_[n_++] = g;
            if (n_ == 2 && in_[1].seq0 < in_[0].seq0) std::swap(in_[0], in_[1]);
            return;
        }
        if (n_ == 2) more_.assign(in_, in_ + 2);
        more_.insert(std::lower_bound(more_.begin(), more_.end(), g,
                                      [](const PoolSeg &x, const PoolSeg &y) { return x.seq0 < y.seq0; }),
                     g);
        n_++;
    }
    // drop the segments whose copy never ran (a failed commit_staged); order is kept
    void drop_pending() {
        std::vector<PoolSeg> keep;
        for (const PoolSeg &g : *this)
            if (!(g.off & SEG_PENDING)) keep.push_back(g);
        clear();
        for (const PoolSeg &g : keep) insert_sorted(g);
    }
    bool any_pending() const {
        for (const PoolSeg &g : *this)
            if (g.off & SEG_PENDING) return true;
        return false;
    }

  private:
    size_t n_ = 0;
    PoolSeg in_[2] = {};
    std::vector<PoolSeg> more_;  // (all of them once there are more than two)
};

// __corro_buffered_changes rows of one (site, db_version): host rows, or (every row of the key came
// from canonical partial changesets of a device batch) pool segments -- never both
struct BufEntry {
    BufRows rows;
    SegList segs;
    bool empty() const { return rows.empty() && segs.empty(); }
};

// A sorted vector map for the bookie's per-(site, version) tables: a call inserts its new keys as one
// sorted batch (merge, O(n + m)) instead of one tree node each, lookups are binary searches (safe
// from the parallel actor walks), erased keys are tombstones dropped at the next merge.
template <class K, class V>
class FlatMap {
  public:
    struct Slot {
        K key;
        V val;
        bool dead;
    };
    using Entries = std::vector<Slot>;  // a batch of new keys, in the map's own slot form
    size_t lower(const K &k) const {
        return (size_t)(std::lower_bound(v_.begin(), v_.end(), k, [](const Slot &s, const K &x) { return s.key < x; }) -
                        v_.begin());
    }
    // lower(k) for a k at or past the key of slot `from` (galloping from there: a sorted run of
    // lookups walks the map once)
    size_t lower_from(size_t from, const K &k) const {
        const size_t n = v_.size();
        if (from >= n || !(v_[from].key < k)) return from;
        size_t lo = from, step = 1;
        while (lo + step < n && v_[lo + step].key < k) {
            lo += step;
            step *= 2;
        }
        const auto e = v_.begin() + (ptrdiff_t)std::min(n, lo + step + 1);
        return (size_t)(std::lower_bound(v_.begin() + (ptrdiff_t)lo + 1, e, k,
                                         [](const Slot &s, const K &x) { return s.key < x; }) - v_.begin());
    }
    V *find(const K &k) {
        const size_t i = lower(k);
        return i < v_.size() && !(k < v_[i].key) && !v_[i].dead ? &v_[i].val : nullptr;
    }
    const V *find(const K &k) const { return const_cast<FlatMap *>(this)->find(k); }
    void erase_at(size_t i) {
        if (kill_at(i)) dead_++;
    }
    // erase_at without the tombstone count (threads erasing disjoint slots; the caller adds them)
    bool kill_at(size_t i) {
        if (v_[i].dead) return false;
        v_[i].dead = true;
        v_[i].val = V{};
        return true;
    }
    void add_dead(size_t k) { dead_ += k; }
    // `add`: keys ascending, unique, none live in the map, every slot live. A map with no live key takes
    // the batch as it is (a swap: the common case of a bookie whose partial versions all completed;
    // moving a call's ~100 K new entries one by one cost 1.5 ms in the mixed agent call).
    void merge(Entries &&add) {
        if (add.empty() && dead_ * 2 <= v_.size()) return;
        if (v_.size() == dead_) {
            v_.swap(add);
            dead_ = 0;
            Entries().swap(add);  // (the old tombstones freed here)
            return;
        }
        Entries out;
        out.reserve(v_.size() - dead_ + add.size());
        size_t a = 0;
        for (Slot &x : v_) {
            for (; a < add.size() && add[a].key < x.key; a++) out.push_back(std::move(add[a]));
            if (a < add.size() && !(x.key < add[a].key)) {  // (a dead slot of the same key)
                out.push_back(std::move(add[a]));
                a++;
                continue;
            }
            if (!x.dead) out.push_back(std::move(x));
        }
        for (; a < add.size(); a++) out.push_back(std::move(add[a]));
        v_.swap(out);
        dead_ = 0;
    }
    size_t slots() const { return v_.size(); }
    size_t live() const { return v_.size() - dead_; }
    Slot &at(size_t i) { return v_[i]; }
    const Slot &at(size_t i) const { return v_[i]; }

  private:
    std::vector<Slot> v_;
    size_t dead_ = 0;
};

using BufKey = std::pair<uint32_t, int64_t>;   // (site, db_version)
using SeqKey = std::pair<uint32_t, uint64_t>;  // (site, version)

}  // namespace

struct corro_bookie {
    ~corro_bookie() { corro::bufpool_free(pool); }
    std::map<ActorId, corro::Booked> actors;                   // Bookie (agent.rs:1546-1598)
    FlatMap<BufKey, BufEntry> buffered;                         // (site, dbv) -> rows by seq
    corro::DevBufPool *pool = nullptr;                          // device rows of BufEntry::segs
    FlatMap<SeqKey, SeqBook> seqbook;                           // (site, version)
    std::vector<std::pair<ActorId, uint64_t>> ready;           // fully buffered, to apply
    std::map<ActorId, uint32_t> site_of;                       // actor -> site ordinal
    // site ordinal -> its actor's Booked (a map node: stable), checked against the ordinal's id: the
    // per-call Bookie::ensure without a tree search per actor
    std::vector<corro::Booked *> site_booked;
    std::vector<ActorId> site_booked_id;
    std::vector<uint64_t> scratch_ver;                          // process_multiple_changes scratch
};

namespace {

// Bookie::ensure (agent.rs:1546-1598) through the site cache; create = false: nullptr for an actor
// the bookie does not hold
corro::Booked *booked_of_site(corro_bookie *bk, uint32_t site, const ActorId &id, bool create) {
    if (site < bk->site_booked.size() && bk->site_booked[site] && bk->site_booked_id[site] == id)
        return bk->site_booked[site];
    corro::Booked *b = nullptr;
    if (create) {
        b = &bk->actors[id];
        bk->site_of[id] = site;
    } else {
        auto it = bk->actors.find(id);
        if (it == bk->actors.end()) return nullptr;
        b = &it->second;
    }
    if (site >= bk->site_booked.size()) {
        bk->site_booked.resize((size_t)site + 1, nullptr);
        bk->site_booked_id.resize((size_t)site + 1);
    }
    bk->site_booked[site] = b;
    bk->site_booked_id[site] = id;
    return b;
}

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
struct StagedBuf {  // one partial changeset's __corro_buffered_changes INSERTs, in walk order
    bool dev;           // canonical changeset of a device batch: its rows stay in HBM
    uint64_t a, b;      // (host) rows [a, b) of Staged::buffered
    uint64_t src, ts;   // (dev) input span start, the changeset ts
    uint32_t seq0, n, site;
    int64_t dbv;
    uint32_t tab;       // (dev) the table index of all its changes, or HDR_TAB_MIXED
};
struct Staged {
    std::vector<std::pair<uint32_t, uint64_t>> set_dbv;                      // crsql_set_db_version
    std::vector<HostRow> buffered;                                            // __corro_buffered_changes
    std::vector<StagedBuf> items;
    // __corro_seq_bookkeeping rows of the call, sorted by key: one vector (an actor's versions mostly
    // arrive ascending, so a new key is usually appended; no tree node per partial version)
    std::vector<std::pair<std::pair<uint32_t, uint64_t>, SeqBook>> seqbook;
    SeqBook &seq(const corro_bookie *bk, uint32_t site, uint64_t version) {
        const std::pair<uint32_t, uint64_t> key{site, version};
        auto it = seqbook.end();
        if (seqbook.empty() || seqbook.back().first < key) {
            it = seqbook.end();
        } else {
            it = std::lower_bound(seqbook.begin(), seqbook.end(), key,
                                  [](const auto &x, const std::pair<uint32_t, uint64_t> &k) { return x.first < k; });
            if (it != seqbook.end() && it->first == key) return it->second;
        }
        const SeqBook *b = bk->seqbook.find(key);
        return seqbook.emplace(it, key, b ? *b : SeqBook{})->second;
    }
};

// row(k) = HostRow of the changeset's k-th change
// canon: the changeset's rows are canonical in a device batch (bufpool.hip): staged as a span
// tab: (canon) the table index of all its changes, or HDR_TAB_MIXED
template <class RowFn>
int process_incomplete(const corro_bookie *bk, Staged &st, const corro_changeset &cs, bool canon, uint32_t tab,
                       RowFn row, corro::PartialVersion &out) {
    if (canon) {
        st.items.push_back(StagedBuf{true, 0, 0, cs.change_off, cs.ts, (uint32_t)cs.seq_start,
                                     (uint32_t)cs.change_count, cs.site, (int64_t)cs.version_start, tab});
    } else {
        const uint64_t a = st.buffered.size();
        for (uint64_t k = 0; k < cs.change_count; k++) st.buffered.push_back(row(k));
        st.items.push_back(StagedBuf{false, a, st.buffered.size(), 0, 0, 0, 0, 0, 0, corro::HDR_TAB_MIXED});
    }
    SeqBook &sb = st.seq(bk, cs.site, cs.version_start);
    const uint64_t s = cs.seq_start, e = cs.seq_end;
    RangeSet merged;
    corro::SmallVec<Range, 2> keep;
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
    sb.ranges = std::move(keep);
    sb.last_seq = cs.last_seq;
    sb.ts = cs.ts;
    out = corro::PartialVersion();
    out.seqs = std::move(merged);
    out.last_seq = cs.last_seq;
    out.ts = cs.ts;
    return CORRO_OK;
}

// f(0) .. f(n - 1) on the host pool (defined below)
template <class F>
void run_parallel(size_t n, F &&f, size_t per = 8);

// a device entry's segments -> host rows (seq order), the pool rows left dead
int materialize(corro_bookie *bk, BufEntry &e) {
    if (e.segs.empty()) return CORRO_OK;
    for (const PoolSeg &g : e.segs) {
        corro::HostSpanRows r;
        TRY_RC(corro::bufpool_read(bk->pool, g.off, g.n, r));
        for (uint64_t j = 0; j < g.n; j++) {
            HostRow h;
            h.pk = r.pk[j];
            h.v0 = r.v0[j];
            h.v1 = r.v1[j];
            h.ts = r.ts[j];
            h.cv = r.cv[j];
            h.dbv = r.dbv[j];
            h.tcid = r.tcid[j];
            h.cl = r.cl[j];
            h.seq = r.seq[j];
            h.site = r.site[j];
            h.vt = r.vt[j];
            h.vl = r.vl[j];
            e.rows.push_back(std::move(h));
        }
    }
    e.segs.clear();
    return CORRO_OK;
}

// [s, e] minus the (sorted, disjoint) segments: the seqs not buffered yet, ascending
void seq_pieces(const SegList &segs, uint64_t s, uint64_t e, std::vector<Range> &out) {
    out.clear();
    uint64_t x = s;
    for (const PoolSeg &g : segs) {
        const uint64_t gs = g.seq0, ge = (uint64_t)g.seq0 + g.n - 1;
        if (ge < x) continue;
        if (gs > e) break;
        if (gs > x) out.emplace_back(x, gs - 1);
        x = ge + 1;
        if (x > e) break;
    }
    if (x <= e) out.emplace_back(x, e);
}

// One key's share of one staged INSERT batch (the item's fields copied in: the commit passes walk
// the subs in key order without chasing pointers)
struct CommitSub {
    BufKey key;
    uint64_t call;
    Staged *st;
    uint64_t a, b;     // (host) rows [a, b) of st->buffered, all of this key
    uint64_t fr;       // (dev, fetched) first row in the fetched rows
    uint64_t src, ts;  // (dev) the item's input span start and ts
    uint32_t seq0, n;  // (dev) its first seq and change count
    bool dev;
    bool tc;           // (dev) its changes' tables are counted on the device (k_tab_count)
};

// What commit_prepare computes without writing the bookie (so it can run on another host thread while
// the merge runs): the subs by actor, and on the fast path the copy jobs, the new keys and, for keys
// the bookie already holds, their entries with this call's segments added (copies, swapped in by
// commit_prepared). Pending segment offsets name (block, local job) until the pool append.
struct CommitPrep {
    bool any = false;                          // some staged item
    bool fast = false;                         // the fast path below applies
    std::vector<std::vector<CommitSub>> per;   // per actor, sorted by (key, call)
    std::vector<size_t> blk;                   // actors with subs, by first key
    std::vector<uint64_t> committed;           // per table: the buffered changes counted on the host
    std::vector<corro::AgentSpan> all_dev;     // (fast) mixed-table spans, counted on the device
    std::vector<corro::PoolCopy> jobs;         // (fast) pool copy jobs, block-major
    std::vector<size_t> jbase;                 // (fast) first job of each block
    FlatMap<BufKey, BufEntry>::Entries add;        // (fast) new keys, ascending
    std::vector<std::pair<BufKey, BufEntry>> upd;  // (fast) held keys: their updated entries
    std::string prof;                          // stage marks (CORRO_AGENT_PROFILE)
};

// The call's staged __corro_buffered_changes INSERTs into the bookie; ON CONFLICT (site_id,
// db_version, seq) DO NOTHING: the first row of a key wins. Keys are independent, so the INSERTs are
// grouped by key, each key's in call order (actors in `order` = ActorId order, as util.rs:765 walks
// them, each actor's in walk order). committed[t] counts every buffered change of table t
// (util.rs:1101-1105). A key stays in the device pool while all its rows come from canonical
// changesets (segments trimmed against the key's earlier ones); a key that receives host rows is
// brought to the host first. dv: the call's device batch (null: host rows only).
// commit_prepare: the part that only READS the bookie (thread-safe against the merge).
void commit_prepare(corro_ctx *ctx, const corro_bookie *bk, bool have_dv, const std::vector<Staged *> &order,
                    size_t ntables, CommitPrep &P, const std::function<void(const char *)> &mark) {
    using Sub = CommitSub;
    P.committed.assign(ntables, 0);
    for (Staged *st : order) P.any |= !st->items.empty();
    if (!P.any) return;
    // per actor (in parallel): its subs sorted by (key, call), call = ActorId rank << 40 | walk index;
    // the actors' blocks concatenated by first key are globally sorted unless two actors share a key
    std::vector<std::vector<Sub>> &per = P.per;
    per.assign(order.size(), {});
    std::vector<std::vector<uint64_t>> ptab(order.size(), std::vector<uint64_t>(ntables, 0));
    std::vector<uint8_t> host_rows(order.size(), 0);  // the actor staged host rows
    run_parallel(order.size(), [&](size_t ai) {
        Staged *st = order[ai];
        std::vector<Sub> &v = per[ai];
        uint64_t call = (uint64_t)ai << 40;
        const std::vector<HostRow> &rows = st->buffered;
        for (const StagedBuf &it : st->items) {
            if (it.dev) {  // a single-table changeset counts here, the others on the device
                const bool tc = it.tab == corro::HDR_TAB_MIXED;
                if (!tc && it.tab < ntables) ptab[ai][it.tab] += it.n;
                v.push_back(Sub{{it.site, it.dbv}, call++, st, 0, 0, 0, it.src, it.ts, it.seq0, it.n, true, tc});
                continue;
            }
            for (uint64_t a = it.a; a < it.b;) {
                uint64_t b = a + 1;
                while (b < it.b && rows[b].site == rows[a].site && rows[b].dbv == rows[a].dbv) b++;
                v.push_back(Sub{{rows[a].site, rows[a].dbv}, call++, st, a, b, 0, 0, 0, 0, 0, false, false});
                host_rows[ai] = 1;
                for (uint64_t k = a; k < b; k++)
                    if ((rows[k].tcid >> 16) < ntables) ptab[ai][rows[k].tcid >> 16]++;
                a = b;
            }
        }
        auto less = [](const Sub &x, const Sub &y) { return x.key < y.key || (x.key == y.key && x.call < y.call); };
        if (!std::is_sorted(v.begin(), v.end(), less)) std::sort(v.begin(), v.end(), less);
    });
    mark("cb_subs");
    for (const auto &t : ptab)
        for (size_t k = 0; k < ntables; k++) P.committed[k] += t[k];
    std::vector<size_t> &blk = P.blk;
    for (size_t ai = 0; ai < per.size(); ai++)
        if (!per[ai].empty()) blk.push_back(ai);
    std::sort(blk.begin(), blk.end(), [&](size_t x, size_t y) { return per[x][0].key < per[y][0].key; });
    const bool pool_ok = have_dv && (bk->pool ? corro::bufpool_usable(ctx, bk->pool) : true);
    const bool any_buffered = bk->buffered.slots() != 0;
    // Fast path -- the common shape: every sub a canonical device changeset, the actors' key ranges
    // disjoint (each actor's keys carry its own site) and no key holding host rows. Then no group is
    // host, nothing is fetched or materialized, and each actor's groups, segment trims and copy jobs
    // are built in parallel (pending segment offsets name (actor, local job)), concatenated in key
    // order afterwards.
    bool fast = pool_ok && !blk.empty();
    for (size_t k = 0; k < blk.size() && fast; k++) {
        fast = !host_rows[blk[k]];
        if (fast && k + 1 < blk.size()) fast = per[blk[k]].back().key < per[blk[k + 1]][0].key;
    }
    if (fast && any_buffered) {  // (read-only check: a key of this call that holds host rows)
        std::vector<uint8_t> hostkey(blk.size(), 0);
        run_parallel(blk.size(), [&](size_t k) {
            const std::vector<Sub> &v = per[blk[k]];
            for (size_t q = 0; q < v.size(); q++) {
                if (q && v[q].key == v[q - 1].key) continue;
                const BufEntry *e = bk->buffered.find(v[q].key);
                if (e && !e->rows.empty()) {
                    hostkey[k] = 1;
                    return;
                }
            }
        });
        for (uint8_t h : hostkey) fast = fast && !h;
    }
    P.fast = fast;
    if (!fast) return;
    struct Out {
        std::vector<corro::AgentSpan> dev;
        std::vector<corro::PoolCopy> jobs;
        FlatMap<BufKey, BufEntry>::Entries add;
        std::vector<std::pair<BufKey, BufEntry>> upd;
    };
    std::vector<Out> outs(blk.size());
    run_parallel(blk.size(), [&](size_t k) {
        const std::vector<Sub> &v = per[blk[k]];
        Out &o = outs[k];
        o.dev.reserve(v.size());
        std::vector<Range> pieces;
        for (size_t g0 = 0; g0 < v.size();) {
            size_t g1 = g0 + 1;
            while (g1 < v.size() && v[g1].key == v[g0].key) g1++;
            // a held key works on a copy of its entry (swapped in after the merge); a new key on a fresh one
            const BufEntry *held = any_buffered ? bk->buffered.find(v[g0].key) : nullptr;  // (keys of this block only)
            BufEntry local;
            if (held) local = *held;
            for (size_t q = g0; q < g1; q++) {
                const Sub &u = v[q];
                if (u.tc) o.dev.push_back({u.src, 0, u.n, u.ts});
                seq_pieces(local.segs, u.seq0, (uint64_t)u.seq0 + u.n - 1, pieces);
                for (const Range &r : pieces) {
                    const PoolSeg g{SEG_PENDING | ((uint64_t)k << 32) | o.jobs.size(), (uint32_t)r.first,
                                    (uint32_t)(r.second - r.first + 1)};
                    o.jobs.push_back({u.src + (r.first - u.seq0), r.second - r.first + 1, u.ts, 0});
                    local.segs.insert_sorted(g);
                }
            }
            if (held) o.upd.emplace_back(v[g0].key, std::move(local));
            else if (!local.empty()) o.add.push_back({v[g0].key, std::move(local), false});
            g0 = g1;
        }
    });
    mark("cb_groups");
    size_t nd = 0, nj = 0, na = 0, nu = 0;
    for (const Out &o : outs) {
        nd += o.dev.size();
        nj += o.jobs.size();
        na += o.add.size();
        nu += o.upd.size();
    }
    P.all_dev.reserve(nd);
    P.jobs.reserve(nj);
    P.add.reserve(na);
    P.upd.reserve(nu);
    P.jbase.resize(blk.size());
    for (size_t k = 0; k < outs.size(); k++) {
        P.all_dev.insert(P.all_dev.end(), outs[k].dev.begin(), outs[k].dev.end());
        P.jbase[k] = P.jobs.size();
        P.jobs.insert(P.jobs.end(), outs[k].jobs.begin(), outs[k].jobs.end());
        for (auto &x : outs[k].add) P.add.push_back(std::move(x));
        for (auto &x : outs[k].upd) P.upd.push_back(std::move(x));
    }
    mark("cb_tables");
}

// the pool copy of the jobs and the pending offsets resolved (both paths)
int commit_pool(corro_ctx *ctx, corro_bookie *bk, const corro_changes *dv, std::vector<corro::PoolCopy> &jobs, bool fast,
                const std::vector<size_t> &jbase, const std::function<void(const char *)> &mark);

// The fast path's writes, after the merge: the device table counts of mixed-table spans, the held
// keys' updated entries swapped in, the new keys merged, then the pool copy.
int commit_prepared(corro_ctx *ctx, corro_bookie *bk, const corro_changes *dv, CommitPrep &P, std::vector<uint64_t> &committed,
                    const std::function<void(const char *)> &mark) {
    const size_t ntables = committed.size();
    for (size_t t = 0; t < ntables; t++) committed[t] += P.committed[t];
    if (!P.all_dev.empty()) {
        std::vector<uint64_t> tc;
        TRY_RC(corro::agent_dev_table_counts(ctx, dv, P.all_dev, (uint32_t)ntables, tc));
        for (size_t t = 0; t < ntables; t++) committed[t] += tc[t];
    }
    if (!bk->pool) bk->pool = corro::bufpool_new();
    for (auto &[key, e] : P.upd) {
        BufEntry *x = bk->buffered.find(key);
        if (!x) throw std::logic_error("buffered key vanished between prepare and commit");
        *x = std::move(e);
    }
    mark("cb_trim");
    bk->buffered.merge(std::move(P.add));
    mark("cb_merge");
    return commit_pool(ctx, bk, dv, P.jobs, true, P.jbase, mark);
}

int commit_staged_impl(corro_ctx *ctx, corro_bookie *bk, const corro_changes *dv, const std::vector<Staged *> &order,
                       std::vector<uint64_t> &committed, const std::function<void(const char *)> &stage,
                       CommitPrep *prepared = nullptr) {
    using Sub = CommitSub;
    auto mark = [&](const char *n) {
        if (stage) stage(n);
    };
    const size_t ntables = committed.size();
    CommitPrep own;
    CommitPrep &P = prepared ? *prepared : own;
    if (!prepared) commit_prepare(ctx, bk, dv != nullptr, order, ntables, P, mark);
    if (!P.any) return CORRO_OK;
    if (P.fast) return commit_prepared(ctx, bk, dv, P, committed, mark);
    for (size_t t = 0; t < ntables; t++) committed[t] += P.committed[t];
    std::vector<std::vector<Sub>> &per = P.per;
    const std::vector<size_t> &blk = P.blk;
    const bool pool_ok = dv && (bk->pool ? corro::bufpool_usable(ctx, bk->pool) : true);
    const bool any_buffered = bk->buffered.slots() != 0;
    std::vector<corro::PoolCopy> jobs;
    FlatMap<BufKey, BufEntry>::Entries add;
    const std::vector<size_t> jbase;
    {
    std::vector<Sub> sp;  // every sub in (key, call) order, contiguous
    size_t nsub = 0;
    for (size_t ai : blk) nsub += per[ai].size();
    if (!nsub) return CORRO_OK;
    sp.reserve(nsub);
    for (size_t ai : blk) {
        sp.insert(sp.end(), per[ai].begin(), per[ai].end());
        std::vector<Sub>().swap(per[ai]);
    }
    auto sless = [](const Sub &x, const Sub &y) { return x.key < y.key || (x.key == y.key && x.call < y.call); };
    if (!std::is_sorted(sp.begin(), sp.end(), sless)) std::sort(sp.begin(), sp.end(), sless);
    // per key group: host at the end of the call (it holds host rows, or receives some, or there is no
    // pool for it)? Its device segments come to the host first; its canonical changesets' rows are
    // fetched from the batch.
    std::vector<std::pair<size_t, size_t>> groups;
    std::vector<uint8_t> ghost;
    std::vector<BufEntry *> gent;  // the key's entry before this call (null: a new key)
    std::vector<corro::AgentSpan> fsp, all_dev;
    all_dev.reserve(sp.size());
    groups.reserve(sp.size());
    ghost.reserve(sp.size());
    gent.reserve(sp.size());
    uint64_t fr_n = 0;
    bool any_dev = false;
    for (size_t g0 = 0; g0 < sp.size();) {
        size_t g1 = g0 + 1;
        while (g1 < sp.size() && sp[g1].key == sp[g0].key) g1++;
        BufEntry *e = any_buffered ? bk->buffered.find(sp[g0].key) : nullptr;
        bool host = !pool_ok || (e && !e->rows.empty());
        for (size_t q = g0; q < g1 && !host; q++) host = !sp[q].dev;
        if (host && e) TRY_RC(materialize(bk, *e));
        for (size_t q = g0; q < g1; q++) {
            Sub &u = sp[q];
            if (!u.dev) continue;
            any_dev = true;
            if (u.tc) all_dev.push_back({u.src, 0, u.n, u.ts});
            if (host) {
                u.fr = fr_n;
                fsp.push_back({u.src, fr_n, u.n, u.ts});
                fr_n += u.n;
            }
        }
        groups.emplace_back(g0, g1);
        ghost.push_back(host);
        gent.push_back(e);
        g0 = g1;
    }
    mark("cb_groups");
    corro::HostSpanRows fr;
    if (!fsp.empty()) TRY_RC(corro::agent_dev_fetch(ctx, dv, fsp, fr));
    mark("cb_fetch");
    if (!all_dev.empty()) {
        std::vector<uint64_t> tc;
        TRY_RC(corro::agent_dev_table_counts(ctx, dv, all_dev, (uint32_t)ntables, tc));
        for (size_t t = 0; t < ntables; t++) committed[t] += tc[t];
    }
    mark("cb_tables");
    if (any_dev && pool_ok && !bk->pool) bk->pool = corro::bufpool_new();
    std::vector<Range> pieces;
    jobs.reserve(all_dev.size());
    add.reserve(groups.size());
    for (size_t gi = 0; gi < groups.size(); gi++) {
        const BufKey key = sp[groups[gi].first].key;
        BufEntry local;
        BufEntry *e = gent[gi];  // (materialize keeps the entry where it is)
        const bool fresh = !e;
        if (fresh) e = &local;
        for (size_t q = groups[gi].first; q < groups[gi].second; q++) {
            const Sub &u = sp[q];
            if (!u.dev) {
                buf_insert(e->rows, u.st->buffered.data() + u.a, u.st->buffered.data() + u.b);
            } else if (ghost[gi]) {
                std::vector<HostRow> hr(u.n);
                for (uint64_t j = 0; j < u.n; j++) {
                    const uint64_t x = u.fr + j;
                    HostRow &h = hr[j];
                    h.pk = fr.pk[x];
                    h.v0 = fr.v0[x];
                    h.v1 = fr.v1[x];
                    h.ts = dv->ts ? fr.ts[x] : u.ts;
                    h.cv = fr.cv[x];
                    h.dbv = fr.dbv[x];
                    h.tcid = fr.tcid[x];
                    h.cl = fr.cl[x];
                    h.seq = fr.seq[x];
                    h.site = fr.site[x];
                    h.vt = fr.vt[x];
                    h.vl = fr.vl[x];
                }
                buf_insert(e->rows, hr.data(), hr.data() + hr.size());
            } else {
                seq_pieces(e->segs, u.seq0, (uint64_t)u.seq0 + u.n - 1, pieces);
                for (const Range &r : pieces) {
                    const PoolSeg g{SEG_PENDING | jobs.size(), (uint32_t)r.first, (uint32_t)(r.second - r.first + 1)};
                    jobs.push_back({u.src + (r.first - u.seq0), r.second - r.first + 1, u.ts, 0});
                    e->segs.insert_sorted(g);
                }
            }
        }
        if (fresh && !local.empty()) add.push_back({key, std::move(local), false});
    }
    mark("cb_trim");
    }  // (serial path)
    bk->buffered.merge(std::move(add));
    mark("cb_merge");
    return commit_pool(ctx, bk, dv, jobs, false, jbase, mark);
}

int commit_pool(corro_ctx *ctx, corro_bookie *bk, const corro_changes *dv, std::vector<corro::PoolCopy> &jobs, bool fast,
                const std::vector<size_t> &jbase, const std::function<void(const char *)> &mark) {
    if (jobs.empty()) return CORRO_OK;
    uint64_t need = 0;
    for (const corro::PoolCopy &j : jobs) need += j.count;
    // (both passes over the buffered table in parallel chunks of slots: a mixed call leaves ~10^5 keys)
    constexpr size_t CH = 4096;
    const size_t nsl = bk->buffered.slots(), nch = (nsl + CH - 1) / CH;
    std::vector<uint64_t *> offs;
    std::vector<uint64_t> lens;
    {
        std::vector<std::vector<uint64_t *>> po(nch);
        std::vector<std::vector<uint64_t>> pl(nch);
        run_parallel(nch, [&](size_t c) {
            for (size_t i = c * CH; i < std::min(nsl, (c + 1) * CH); i++) {
                auto &x = bk->buffered.at(i);
                if (x.dead) continue;
                for (PoolSeg &g : x.val.segs)
                    if (!(g.off & SEG_PENDING)) {
                        po[c].push_back(&g.off);
                        pl[c].push_back(g.n);
                    }
            }
        }, 1);
        size_t tot = 0;
        for (const auto &v : po) tot += v.size();
        offs.reserve(tot);
        lens.reserve(tot);
        for (size_t c = 0; c < nch; c++) {  // (slot order, as one pass would list them)
            offs.insert(offs.end(), po[c].begin(), po[c].end());
            lens.insert(lens.end(), pl[c].begin(), pl[c].end());
        }
    }
    mark("cb_offs");
    if (fault_armed("bufpool_reserve")) return fail(CORRO_E_NOMEM, "injected fault (CORRO_FAULT): bufpool_reserve");
    TRY_RC(corro::bufpool_reserve(ctx, bk->pool, need, offs, lens));
    mark("cb_reserve");
    TRY_RC(corro::bufpool_append(ctx, bk->pool, dv, jobs));
    mark("cb_append");
    // (one sequential pass: no per-key searches; a pending offset names (block, job) on the fast
    // path, the global job on the serial one)
    run_parallel(nch, [&](size_t c) {
        for (size_t i = c * CH; i < std::min(nsl, (c + 1) * CH); i++)
            for (PoolSeg &g : bk->buffered.at(i).val.segs)
                if (g.off & SEG_PENDING) {
                    const uint64_t x = g.off & ~SEG_PENDING;
                    g.off = jobs[fast ? jbase[x >> 32] + (x & 0xFFFFFFFFULL) : x].dst;
                }
    }, 1);
    mark("cb_fix");
    return CORRO_OK;
}

// A failure inside commit_staged_impl (table counts, pool reserve or copy: HBM or HIP errors) can come
// after segments were inserted into the bookie with pending offsets naming this call's copy jobs.
// They are dropped again (keys left without rows are erased), so the bookie never names pool rows
// that were not copied and no seq counts as buffered that is not: a re-sent piece buffers again.
int commit_staged(corro_ctx *ctx, corro_bookie *bk, const corro_changes *dv, const std::vector<Staged *> &order,
                  std::vector<uint64_t> &committed, const std::function<void(const char *)> &stage = nullptr,
                  CommitPrep *prepared = nullptr) {
    const int rc = commit_staged_impl(ctx, bk, dv, order, committed, stage, prepared);
    if (rc == CORRO_OK) return rc;
    for (size_t i = 0; i < bk->buffered.slots(); i++) {
        auto &x = bk->buffered.at(i);
        if (x.dead || !x.val.segs.any_pending()) continue;
        x.val.segs.drop_pending();
        if (x.val.empty()) bk->buffered.erase_at(i);
    }
    return rc;
}

// The call's __corro_seq_bookkeeping rows (one per (site, version): the actors' keys are disjoint), in
// two parts: seqbook_prepare only READS the bookie (it runs alongside the merge on the commit
// preparation thread) and moves the call's books out of the staged maps into new entries and updates
// of held slots; seqbook_apply writes them after the merge.
struct SeqPrep {
    FlatMap<SeqKey, SeqBook>::Entries add;            // new keys, ascending
    std::vector<std::pair<SeqBook *, SeqBook>> upd;   // held keys: their slots and new books
};
void seqbook_prepare(corro_bookie *bk, const std::vector<Staged *> &order, SeqPrep &S) {
    std::vector<Staged *> blk;
    for (Staged *st : order)
        if (!st->seqbook.empty()) blk.push_back(st);
    if (blk.empty()) return;
    std::sort(blk.begin(), blk.end(), [](Staged *x, Staged *y) { return x->seqbook.begin()->first < y->seqbook.begin()->first; });
    std::vector<size_t> base(blk.size() + 1, 0);
    for (size_t b = 0; b < blk.size(); b++) base[b + 1] = base[b] + blk[b]->seqbook.size();
    if (bk->seqbook.live() == 0) {
        // no seq books held (every earlier partial version completed or was cleared): the call's books,
        // one actor's (sorted, disjoint) keys per task, are written in place into the map's new storage
        FlatMap<SeqKey, SeqBook>::Entries &add = S.add;
        add.resize(base.back());
        run_parallel(blk.size(), [&](size_t b) {
            size_t q = base[b];
            for (auto &[k, sb] : blk[b]->seqbook) {
                add[q].key = k;
                add[q].val = std::move(sb);
                add[q].dead = false;
                q++;
            }
        }, 16);
        bool sorted = true;
        for (size_t q = 1; q < add.size() && sorted; q++) sorted = add[q - 1].key < add[q].key;
        if (!sorted) std::sort(add.begin(), add.end(), [](const auto &x, const auto &y) { return x.key < y.key; });
        return;
    }
    // gathered in parallel (one actor's map per task), each item with the slot it updates, if any
    std::vector<std::pair<SeqKey, SeqBook>> items(base.back());
    std::vector<SeqBook *> hit(base.back());
    run_parallel(blk.size(), [&](size_t b) {
        size_t q = base[b];
        for (auto &[k, sb] : blk[b]->seqbook) {
            items[q].first = k;
            items[q].second = std::move(sb);
            hit[q] = bk->seqbook.find(k);  // (read-only lookups)
            q++;
        }
    }, 16);
    bool sorted = true;
    for (size_t q = 1; q < items.size() && sorted; q++) sorted = items[q - 1].first < items[q].first;
    if (!sorted) {  // (two actors' keys interleave: plain path)
        std::sort(items.begin(), items.end(), [](const auto &x, const auto &y) { return x.first < y.first; });
        for (auto &[k, sb] : items) {
            if (SeqBook *x = bk->seqbook.find(k)) S.upd.emplace_back(x, std::move(sb));
            else S.add.push_back({k, std::move(sb), false});
        }
    } else {
        S.add.reserve(items.size());
        for (size_t q = 0; q < items.size(); q++) {
            if (hit[q]) S.upd.emplace_back(hit[q], std::move(items[q].second));
            else S.add.push_back({items[q].first, std::move(items[q].second), false});
        }
    }
}
void seqbook_apply(corro_bookie *bk, SeqPrep &S) {
    for (auto &[x, sb] : S.upd) *x = std::move(sb);
    bk->seqbook.merge(std::move(S.add));
}
void commit_seqbook(corro_bookie *bk, const std::vector<Staged *> &order) {
    SeqPrep S;
    seqbook_prepare(bk, order, S);
    seqbook_apply(bk, S);
}

// sorted site << 40 | version keys of every (site, version) holding buffered rows or seq bookkeeping
std::vector<uint64_t> buffered_keys(const corro_bookie *bk) {
    // (each map's slots scanned in parallel chunks, the chunks' keys concatenated in order)
    auto scan = [](size_t n, auto &&key_of) {
        constexpr size_t CH = 8192;
        const size_t nch = (n + CH - 1) / CH;
        std::vector<std::vector<uint64_t>> part(nch);
        run_parallel(nch, [&](size_t c) {
            for (size_t i = c * CH; i < std::min(n, (c + 1) * CH); i++) {
                uint64_t x;
                if (key_of(i, x)) part[c].push_back(x);
            }
        }, 1);
        size_t tot = 0;
        for (const auto &p : part) tot += p.size();
        std::vector<uint64_t> out;
        out.reserve(tot);
        for (const auto &p : part) out.insert(out.end(), p.begin(), p.end());
        return out;
    };
    const std::vector<uint64_t> a = scan(bk->buffered.slots(), [&](size_t i, uint64_t &key) {
        const auto &x = bk->buffered.at(i);
        if (x.dead || x.val.empty() || x.key.second < 0 || (uint64_t)x.key.second >= (1ULL << 40)) return false;
        key = (uint64_t)x.key.first << 40 | (uint64_t)x.key.second;
        return true;
    });
    const std::vector<uint64_t> b = scan(bk->seqbook.slots(), [&](size_t i, uint64_t &key) {
        const auto &x = bk->seqbook.at(i);
        if (x.dead || x.key.second >= (1ULL << 40)) return false;
        key = (uint64_t)x.key.first << 40 | x.key.second;
        return true;
    });
    std::vector<uint64_t> k(a.size() + b.size());  // (both ascending: the maps' key order is (site, version))
    std::merge(a.begin(), a.end(), b.begin(), b.end(), k.begin());
    k.erase(std::unique(k.begin(), k.end()), k.end());
    return k;
}

// buffered_keys as it will read once the prepared commit (fast path, or nothing staged) and the prepared
// seq books are written: the bookie's keys now plus the ones those writes add (the writes only add
// keys or fill held ones), computed alongside the merge
std::vector<uint64_t> buffered_keys_after(const corro_bookie *bk, const CommitPrep &P, const SeqPrep &S) {
    // (every list ascending: the tables, the prepared new and updated keys -- actors' disjoint key
    // ranges in key order on the fast path -- and the new seq books; merged, not sorted)
    std::vector<uint64_t> a, b, c;
    a.reserve(P.add.size());
    b.reserve(P.upd.size());
    c.reserve(S.add.size());
    auto buf_key = [](std::vector<uint64_t> &v, const BufKey &key, const BufEntry &e) {
        if (!e.empty() && key.second >= 0 && (uint64_t)key.second < (1ULL << 40))
            v.push_back((uint64_t)key.first << 40 | (uint64_t)key.second);
    };
    for (const auto &x : P.add) buf_key(a, x.key, x.val);
    for (const auto &[key, e] : P.upd) buf_key(b, key, e);
    for (const auto &x : S.add)
        if (x.key.second < (1ULL << 40)) c.push_back((uint64_t)x.key.first << 40 | x.key.second);
    auto merge2 = [](const std::vector<uint64_t> &x, const std::vector<uint64_t> &y) {
        std::vector<uint64_t> o(x.size() + y.size());
        std::merge(x.begin(), x.end(), y.begin(), y.end(), o.begin());
        return o;
    };
    if (!std::is_sorted(b.begin(), b.end())) std::sort(b.begin(), b.end());
    std::vector<uint64_t> out = merge2(merge2(buffered_keys(bk), a), merge2(b, c));
    out.erase(std::unique(out.begin(), out.end()), out.end());
    return out;
}

// clear_buffered of single versions, many at once: sorted, then each map walked once per slice of the
// versions, the slices in parallel (each lookup is a few cache misses into tables the walk's threads
// just wrote: ~0.3 us each, serially 0.6 ms for a mixed call's 2 K versions)
void clear_buffered_each(corro_bookie *bk, std::vector<std::pair<uint32_t, uint64_t>> &sv) {
    std::sort(sv.begin(), sv.end());
    sv.erase(std::unique(sv.begin(), sv.end()), sv.end());
    constexpr size_t PER = 128;
    const size_t nparts = (sv.size() + PER - 1) / PER;
    std::vector<std::pair<size_t, size_t>> killed(nparts, {0, 0});
    run_parallel(nparts, [&](size_t q) {
        size_t i = 0, j = 0, kb = 0, ks = 0;
        for (size_t x = q * PER; x < std::min(sv.size(), (q + 1) * PER); x++) {
            const auto &[site, v] = sv[x];
            if (v <= (uint64_t)INT64_MAX) {
                const BufKey k{site, (int64_t)v};
                for (i = bk->buffered.lower_from(x == q * PER ? bk->buffered.lower(k) : i, k);
                     i < bk->buffered.slots() && !(k < bk->buffered.at(i).key); i++)
                    kb += bk->buffered.kill_at(i);
            }
            const SeqKey k{site, v};
            for (j = bk->seqbook.lower_from(x == q * PER ? bk->seqbook.lower(k) : j, k);
                 j < bk->seqbook.slots() && !(k < bk->seqbook.at(j).key); j++)
                ks += bk->seqbook.kill_at(j);
        }
        killed[q] = {kb, ks};
    }, 1);
    for (const auto &[kb, ks] : killed) {
        bk->buffered.add_dead(kb);
        bk->seqbook.add_dead(ks);
    }
}

void clear_buffered(corro_bookie *bk, uint32_t site, uint64_t vs, uint64_t ve) {
    if (vs <= (uint64_t)INT64_MAX)
        for (size_t i = bk->buffered.lower({site, (int64_t)vs}); i < bk->buffered.slots(); i++) {
            const auto &x = bk->buffered.at(i);
            if (x.key.first != site || (uint64_t)x.key.second > ve) break;
            bk->buffered.erase_at(i);
        }
    for (size_t i = bk->seqbook.lower({site, vs}); i < bk->seqbook.slots(); i++) {
        const auto &x = bk->seqbook.at(i);
        if (x.key.first != site || x.key.second > ve) break;
        bk->seqbook.erase_at(i);
    }
}

// tombstones of cleared keys dropped once they are half of a table
void compact_tables(corro_bookie *bk) {
    bk->buffered.merge({});
    bk->seqbook.merge({});
}

// A persistent pool of host workers for the per-call parallel passes: spawning threads per pass
// cost more than the passes themselves (four passes x 15 threads per call). Workers sleep on a
// condition variable between jobs; one job runs at a time (callers serialise on the pool).
class HostPool {
  public:
    static HostPool &get() {
        static HostPool *p = new HostPool();  // never destroyed: its workers outlive static teardown
        return *p;
    }
    unsigned threads() const { return cap_; }
    // fn(arg, k) for k in [0, n) on up to nth threads (the caller is one of them). Exception-safe:
    // an exception thrown by fn (on the caller or a worker) stops further indices from starting, the
    // call still waits for every worker that joined, then rethrows the first one on the caller.
    // A nested call (fn itself calling run) runs serially on the calling thread.
    void run(size_t n, unsigned nth, void (*fn)(void *, size_t), void *arg) {
        if (in_pool_) {
            for (size_t k = 0; k < n; k++) fn(arg, k);
            return;
        }
        std::lock_guard<std::mutex> one(job_mu_);
        {
            std::lock_guard<std::mutex> g(mu_);
            fn_ = fn;
            arg_ = arg;
            n_ = n;
            next_.store(0, std::memory_order_relaxed);
            want_ = nth - 1;
            joined_ = 0;
            done_ = 0;
            err_ = nullptr;
            gen_++;
        }
        cv_.notify_all();
        work(fn, arg, n);
        std::unique_lock<std::mutex> g(mu_);
        want_ = 0;  // no worker joins this job any more; wait for the ones that did
        done_cv_.wait(g, [&] { return done_ == joined_; });
        if (err_) {
            std::exception_ptr e = err_;
            err_ = nullptr;
            g.unlock();
            std::rethrow_exception(e);
        }
    }

  private:
    HostPool() {
        const char *e = std::getenv("CORRO_HOST_THREADS");
        const long v = e ? std::atol(e) : 0;
        const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
        cap_ = v > 0 ? (unsigned)std::min<long>(v, 256) : std::min(16u, hw);
        for (unsigned t = 1; t < cap_; t++) std::thread([this] { loop(); }).detach();
        warm_heap();  // (this thread's; each worker warms its own before its first wait)
    }
    // The first call of a process paid its host threads' first heap growth (the allocator's mmap
    // threshold starts at 128 KB, so every large per-actor vector was a fresh mmap + page faults that
    // later calls reuse from the arena: the first mixed call's walk 9.3 vs 3.2 ms,
    // profiles/history/r05_agent_cold_first_call.log). Each worker grows its arena once here: one 16-MB block
    // freed raises its mmap / trim thresholds, then a spread of smaller blocks is touched and freed so
    // the arena keeps the pages. (CORRO_HEAP_WARM=0 skips it.)
    static void warm_heap() {
        const char *e = std::getenv("CORRO_HEAP_WARM");
        if (e && std::atoi(e) == 0) return;
        const size_t big = 16u << 20;
        if (void *p = std::malloc(big)) {
            std::memset(p, 0, big);
            std::free(p);
        }
        std::vector<void *> blocks;
        for (size_t sz = 4096, tot = 0; tot < (24u << 20); sz = sz < (1u << 20) ? 2 * sz : 4096) {
            void *p = std::malloc(sz);
            if (!p) break;
            std::memset(p, 0, sz);
            blocks.push_back(p);
            tot += sz;
        }
        for (void *p : blocks) std::free(p);
    }
    void work(void (*fn)(void *, size_t), void *arg, size_t n) {
        in_pool_ = true;
        try {
            for (size_t k; (k = next_.fetch_add(1, std::memory_order_relaxed)) < n;) fn(arg, k);
        } catch (...) {
            next_.store(n, std::memory_order_relaxed);  // no further index starts
            std::lock_guard<std::mutex> g(mu_);
            if (!err_) err_ = std::current_exception();
        }
        in_pool_ = false;
    }
    void loop() {
        warm_heap();
        uint64_t seen = 0;
        std::unique_lock<std::mutex> g(mu_);
        while (true) {
            cv_.wait(g, [&] { return gen_ != seen; });
            seen = gen_;
            if (joined_ >= want_) continue;  // enough workers for this job
            joined_++;
            auto fn = fn_;
            auto arg = arg_;
            const size_t n = n_;
            g.unlock();
            work(fn, arg, n);
            g.lock();
            done_++;
            done_cv_.notify_all();
        }
    }
    unsigned cap_ = 1;
    std::mutex job_mu_, mu_;
    std::condition_variable cv_, done_cv_;
    void (*fn_)(void *, size_t) = nullptr;
    void *arg_ = nullptr;
    size_t n_ = 0;
    std::atomic<size_t> next_{0};
    unsigned want_ = 0, joined_ = 0, done_ = 0;
    uint64_t gen_ = 0;
    std::exception_ptr err_;
    static thread_local bool in_pool_;
};
thread_local bool HostPool::in_pool_ = false;

// f(0) .. f(n - 1) on up to CORRO_HOST_THREADS (default: min(16, hardware)) host threads, at least
// `per` indices per thread (serial for small n). f must only touch state of its own index.
template <class F>
void run_parallel(size_t n, F &&f, size_t per) {
    HostPool &pool = HostPool::get();
    const unsigned nth = (unsigned)std::min<size_t>(pool.threads(), n / std::max<size_t>(per, 1));
    if (nth <= 1) {
        for (size_t k = 0; k < n; k++) f(k);
        return;
    }
    using FT = typename std::remove_reference<F>::type;
    pool.run(n, nth, [](void *p, size_t k) { (*static_cast<FT *>(p))(k); }, (void *)&f);
}

}  // namespace

extern "C" {

int corro_bookie_new(corro_bookie **out) {
    if (!out) return fail(CORRO_E_INVALID, "out is NULL");
    *out = new corro_bookie();
    (void)HostPool::get();  // the walk's worker threads start now, not inside the first call
    return CORRO_OK;
}

void corro_bookie_free(corro_bookie *b) { delete b; }

}  // extern "C"

namespace {

// RangeInclusiveMap<Version, Option<PartialVersion>> of the versions one actor has seen in this
// call (util.rs:762-807): covered versions plus, per version whose latest entry is a partial, that
// PartialVersion (a later entry over the version replaces it).
// (a partial is held by index into the actor's partial list, which keeps every one in walk order: no
// copy of its seq ranges)
struct SeenMap {
    using Parts = std::vector<std::pair<uint64_t, corro::PartialVersion>>;
    explicit SeenMap(const Parts &parts) : parts_(parts) {}
    RangeSet covered;
    std::vector<std::pair<uint64_t, size_t>> partial_at;  // version -> part, sorted (no tree node per partial)
    void insert(const Range &v, size_t part = SIZE_MAX) {  // part: index in parts, SIZE_MAX = none
        covered.insert(v.first, v.second);
        auto lo = first_at(v.first);
        auto hi = lo;
        while (hi != partial_at.end() && hi->first <= v.second) ++hi;
        lo = partial_at.erase(lo, hi);
        if (part != SIZE_MAX) partial_at.insert(lo, {v.first, part});
    }
    // every version of v seen, and (with seqs) each seen partial holding the seqs
    bool all_seen(const Range &v, const Range *seqs) const {
        if (!covered.contains_range(v.first, v.second)) return false;
        if (!seqs || partial_at.empty()) return true;
        for (auto it = first_at(v.first); it != partial_at.end() && it->first <= v.second; ++it)
            if (!parts_[it->second].second.seqs.contains_range(seqs->first, seqs->second)) return false;
        return true;
    }

  private:
    std::vector<std::pair<uint64_t, size_t>>::iterator first_at(uint64_t v) {
        return std::lower_bound(partial_at.begin(), partial_at.end(), v, [](const auto &x, uint64_t k) { return x.first < k; });
    }
    std::vector<std::pair<uint64_t, size_t>>::const_iterator first_at(uint64_t v) const {
        return std::lower_bound(partial_at.begin(), partial_at.end(), v, [](const auto &x, uint64_t k) { return x.first < k; });
    }
    const Parts &parts_;
};

// One actor's share of a process_multiple_changes call. Actors are independent (util.rs:765-884
// handles them one at a time under their own booked write lock), so their header passes run in
// parallel on the host.
struct ActorWork {
    ActorId id{};
    uint32_t site = 0;
    corro::Booked *booked = nullptr;
    bool had_max = false;
    uint64_t max = 0;
    bool fast = false;                // every changeset a complete Full version, ascending (arrival order)
    const uint64_t *idx = nullptr;    // (not fast) changesets the walk takes, in arrival order
    uint64_t nidx = 0;
    // results (not fast: the per-actor passes; fast ones are counted per chunk)
    uint64_t nspans = 0, nchanges = 0;
    bool ts = false;
    std::vector<uint64_t> set_dbv;    // crsql_set_db_version(site, v)
    Staged st;                        // buffered rows / seq bookkeeping of incomplete versions
    std::vector<std::pair<uint64_t, corro::PartialVersion>> partials;
    bool has_next = false;
    corro::Booked next;               // the committed VersionsSnapshot
    std::vector<uint64_t> ready;      // versions now fully buffered
    bool defer_gaps = false;          // the call's gap bookkeeping runs batched on the device (gaps_batch)
    RangeSet versions;                // (deferred) the versions this call adds
    int rc = CORRO_OK;
    std::string err;
    double t_walk[4] = {0, 0, 0, 0};  // (CORRO_AGENT_PROFILE) runs, pass 1, pass 2, gaps + partials: ms
};

// A call's per-actor work is freed on a background thread after the call returns (a large mixed
// call's buffered rows, seq maps and snapshots are ~1 ms of frees; nothing in them refers to the
// bookie). One thread, a queue of batches; like HostPool it is never joined.
class Reaper {
  public:
    static Reaper &get() {
        static Reaper *r = new Reaper();
        return *r;
    }
    void give(std::vector<ActorWork> &&w) {
        auto *p = new std::vector<ActorWork>(std::move(w));
        {
            std::lock_guard<std::mutex> g(mu_);
            q_.push_back(p);
        }
        cv_.notify_one();
    }

  private:
    Reaper() { std::thread([this] { loop(); }).detach(); }
    void loop() {
        while (true) {
            std::vector<std::vector<ActorWork> *> batch;
            {
                std::unique_lock<std::mutex> g(mu_);
                cv_.wait(g, [&] { return !q_.empty(); });
                batch.swap(q_);
            }
            for (auto *p : batch) delete p;
        }
    }
    std::mutex mu_;
    std::condition_variable cv_;
    std::vector<std::vector<ActorWork> *> q_;
};

Range versions_of(const corro_changeset &c) {
    if (c.kind == CORRO_CS_EMPTY_SET) return {0, 0};  // Changeset::versions() dummy (broadcast.rs:176-178)
    return {c.version_start, c.kind == CORRO_CS_FULL ? c.version_start : c.version_end};
}
const Range *seqs_of(const corro_changeset &c, Range &r) {
    if (c.kind != CORRO_CS_FULL) return nullptr;
    r = {c.seq_start, c.seq_end};
    return &r;
}
bool is_complete(const corro_changeset &c) { return c.kind != CORRO_CS_FULL || (c.seq_start == 0 && c.seq_end == c.last_seq); }
bool is_empty(const corro_changeset &c) { return c.kind != CORRO_CS_FULL || c.change_count == 0; }

// Where the per-actor walk reads changeset i and records its outcome: the caller's headers and
// out->known (host headers), or host copies of the slow actors' changesets (device headers).
struct CsView {
    const corro_changeset *cs;
    const uint8_t *bad;   // unknown-name screen
    int32_t *known;
    uint8_t *flag;        // 1 = merged by this call
    const uint8_t *canon; // canonical partial changeset of a device batch (bufpool.hip; null: none)
    const uint32_t *ctab; // a canonical one's table index, or HDR_TAB_MIXED (null: all mixed)
};

// One actor's passes 1 and 2 (util.rs:704-884) over its changesets w.idx (arrival order) unless it
// is fast, plus the versions of the runs given (decided elsewhere: a fast actor's, or the device's
// isolated changesets, which share no version with w.idx), then its gap snapshot (:894-932) and
// partials.
// (the version runs an actor's changesets decided elsewhere add -- device decisions: columns of the
// header result; host fast path: Range pairs)
struct RunView {
    const uint64_t *s = nullptr, *e = nullptr;
    const Range *r = nullptr;
    size_t n = 0;
};
template <class RowOf>
void run_actor_walk(corro_bookie *bk, ActorWork &w, const CsView &v, const RunView &fast_runs, RowOf &&row_of) {
    static const bool prof = std::getenv("CORRO_AGENT_PROFILE") != nullptr;
    auto t_prev = std::chrono::steady_clock::now();
    auto lap = [&](int k) {
        if (!prof) return;
        const auto t = std::chrono::steady_clock::now();
        w.t_walk[k] += std::chrono::duration<double, std::milli>(t - t_prev).count();
        t_prev = t;
    };
    corro::Booked &booked = *w.booked;
    const bool had_max = w.had_max;
    const uint64_t max = w.max;
    RangeSet versions;
    for (size_t k = 0; k < fast_runs.n; k++) {
        if (fast_runs.r) versions.insert(fast_runs.r[k].first, fast_runs.r[k].second);
        else versions.insert(fast_runs.s[k], fast_runs.e[k]);
    }
    lap(0);
    if (!w.fast) {
        // pass 1: batch-local dedup of (versions, seqs), then versions the actor already holds
        std::vector<uint64_t> unknown;
        unknown.reserve(w.nidx);
        // the seen set of (versions, seqs) keys: the first changeset of each key in arrival order
        // (one sort of the actor's keys instead of a tree node per changeset)
        struct SeenKey {
            uint64_t vs, ve, ss, se;
            uint32_t has_seqs, k;
        };
        std::vector<SeenKey> keys(w.nidx);
        for (uint64_t k = 0; k < w.nidx; k++) {
            const corro_changeset &c = v.cs[w.idx[k]];
            const Range vr = versions_of(c);
            Range sq;
            const Range *seqs = seqs_of(c, sq);
            keys[k] = SeenKey{vr.first, vr.second, seqs ? sq.first : 0, seqs ? sq.second : 0, seqs ? 1u : 0u, (uint32_t)k};
        }
        auto kless = [](const SeenKey &x, const SeenKey &y) {
            return std::tie(x.vs, x.ve, x.has_seqs, x.ss, x.se, x.k) < std::tie(y.vs, y.ve, y.has_seqs, y.ss, y.se, y.k);
        };
        std::sort(keys.begin(), keys.end(), kless);
        std::vector<uint8_t> first_of_key(w.nidx, 0);
        for (uint64_t q = 0; q < keys.size(); q++) {
            const SeenKey &x = keys[q];
            if (q == 0 || std::tie(x.vs, x.ve, x.has_seqs, x.ss, x.se) !=
                              std::tie(keys[q - 1].vs, keys[q - 1].ve, keys[q - 1].has_seqs, keys[q - 1].ss, keys[q - 1].se))
                first_of_key[x.k] = 1;
        }
        for (uint64_t k = 0; k < w.nidx; k++) {
            if (!first_of_key[k]) continue;
            const uint64_t i = w.idx[k];
            const Range vr = versions_of(v.cs[i]);
            Range sq;
            const Range *seqs = seqs_of(v.cs[i], sq);
            if (booked.contains_all(vr.first, vr.second, seqs)) continue;
            unknown.push_back(i);
        }
        lap(1);
        // pass 2 (the bookie is not written until the call commits, so pass 1's contains_all stands)
        SeenMap seen_local(w.partials);
        // (the versions pass 2 adds are collected and merged with the runs' in one linear pass at the
        // end: inserted one by one they filled holes between the runs, a shift of the range list each)
        std::vector<Range> added;
        added.reserve(unknown.size());
        for (uint64_t i : unknown) {
            const corro_changeset &c = v.cs[i];
            const Range vr = versions_of(c);
            Range sq;
            const Range *seqs = seqs_of(c, sq);
            if (seen_local.all_seen(vr, seqs)) continue;
            std::optional<corro::PartialVersion> partial;
            if (is_complete(c) && is_empty(c)) {
                // process_empty_version only when end > booked max (util.rs:810-824)
                if (!had_max || vr.second > max) w.set_dbv.push_back(vr.second);
                v.known[i] = CORRO_KNOWN_CLEARED;
            } else {
                if (seqs && seqs->second < seqs->first) continue;  // invalid seqs (util.rs:826-831)
                if (v.bad[i]) {  // the INSERT fails, the version's SAVEPOINT rolls back (util.rs:839-860)
                    v.known[i] = CORRO_E_UNKNOWN_COLUMN;
                    continue;
                }
                if (is_complete(c)) {
                    v.flag[i] = 1;
                    w.nspans++;
                    w.nchanges += c.change_count;
                    w.ts |= c.ts != 0;
                    v.known[i] = CORRO_KNOWN_CURRENT;  // final value decided after the merge
                } else {
                    corro::PartialVersion p;
                    const bool canon = v.canon && v.canon[i];
                    const uint32_t tab = canon && v.ctab ? v.ctab[i] : corro::HDR_TAB_MIXED;
                    if (process_incomplete(bk, w.st, c, canon, tab, [&](uint64_t k) { return row_of(c, i, k); },
                                           p) != CORRO_OK) {
                        v.known[i] = CORRO_E_INVALID;
                        continue;
                    }
                    partial = std::move(p);
                    v.known[i] = CORRO_KNOWN_PARTIAL;
                }
            }
            if (partial) w.partials.emplace_back(vr.first, std::move(*partial));
            seen_local.insert(vr, partial ? w.partials.size() - 1 : SIZE_MAX);
            added.push_back(vr);
        }
        if (!added.empty()) {
            std::sort(added.begin(), added.end());
            RangeSet all;  // (ascending starts: every insert appends or extends the last range)
            const auto &fr = versions.ranges();
            size_t x = 0, y = 0;
            while (x < fr.size() || y < added.size()) {
                const Range &r = (y == added.size() || (x < fr.size() && fr[x].first <= added[y].first)) ? fr[x++] : added[y++];
                all.insert(r.first, r.second);
            }
            versions = std::move(all);
        }
        lap(2);
    }
    if (versions.empty()) return;
    if (w.defer_gaps) {  // (many actors: one device pass for all of them, gaps_batch)
        w.versions = std::move(versions);
        return;
    }
    // gap bookkeeping on a copy of the actor's Booked (VersionsSnapshot, agent.rs:1108-1235): an
    // INSERT that would violate __corro_bookkeeping_gaps' key fails the whole call before the
    // merge has touched the state, as the transaction's rollback would undo it (util.rs:894-936)
    w.next = booked;
    w.has_next = true;
    if (!w.next.insert_db(versions, nullptr, nullptr)) {
        w.rc = CORRO_E_INVALID;
        w.err = "UNIQUE constraint failed: __corro_bookkeeping_gaps.start";
        return;
    }
    for (auto &[version, pv] : w.partials) {  // (w.partials is done with: moved into the snapshot)
        const corro::PartialVersion &p = w.next.insert_partial(version, std::move(pv));
        if (!p.seqs.has_gap(0, p.last_seq)) w.ready.push_back(version);
    }
    lap(3);
}

// Whether the call's gap bookkeeping goes through the batched device form (corro_booked_insert_db_batch)
// instead of insert_db inside each actor's (parallel) walk: CORRO_AGENT_GAPS_BATCH=1, and only when
// every booked max fits its signed input. Off by default: with the Bookie on the host, the CSR
// round trip and the per-actor rebuild of the gap lists cost more than the host pass at every size
// measured (tools/bench_agent_actors.py: 100 K actors x 2 gaps 90 vs 109 ms, 20 K x 31 gaps 28 vs
// 67 ms, 4 K x 199 gaps 20 vs 48 ms for the whole call); it pays only for gap lists kept on the device.
bool want_gaps_batch(const std::vector<ActorWork> &work) {
    const char *e = std::getenv("CORRO_AGENT_GAPS_BATCH");  // (read per call: tests switch it)
    if (!e || std::atoi(e) != 1 || work.empty()) return false;
    for (const ActorWork &w : work)
        if (w.booked->has_max && w.booked->max > (uint64_t)INT64_MAX) return false;
    return true;
}

// The deferred actors' insert_db (agent.rs:1108-1235) in one device pass: new max and gap lists from
// the device, the partials inside a deleted gap dropped, the UNIQUE (actor_id, start) check on the
// host (an INSERT row starting where a gap the pass kept starts), then insert_partial as in the walk.
int gaps_batch(corro_ctx *ctx, std::vector<ActorWork> &work) {
    std::vector<size_t> A;
    for (size_t k = 0; k < work.size(); k++)
        if (work[k].defer_gaps && !work[k].versions.empty() && work[k].rc == CORRO_OK) A.push_back(k);
    if (A.empty()) return CORRO_OK;
    const size_t n = A.size();
    corro::GapsHost in;
    in.max.resize(n);
    in.gap_off.assign(n + 1, 0);
    in.ver_off.assign(n + 1, 0);
    for (size_t q = 0; q < n; q++) {
        const ActorWork &w = work[A[q]];
        in.max[q] = w.booked->has_max ? (int64_t)w.booked->max : -1;
        in.gap_off[q + 1] = in.gap_off[q] + w.booked->needed.ranges().size();
        in.ver_off[q + 1] = in.ver_off[q] + w.versions.ranges().size();
    }
    in.gap_start.resize(in.gap_off[n]);
    in.gap_end.resize(in.gap_off[n]);
    in.ver_start.resize(in.ver_off[n]);
    in.ver_end.resize(in.ver_off[n]);
    for (size_t q = 0; q < n; q++) {
        const ActorWork &w = work[A[q]];
        uint64_t o = in.gap_off[q];
        for (const Range &r : w.booked->needed.ranges()) {
            in.gap_start[o] = r.first;
            in.gap_end[o++] = r.second;
        }
        o = in.ver_off[q];
        for (const Range &r : w.versions.ranges()) {
            in.ver_start[o] = r.first;
            in.ver_end[o++] = r.second;
        }
    }
    corro::GapsHostOut out;
    TRY_RC(corro::agent_dev_gaps(ctx, in, out));
    run_parallel(n, [&](size_t q) {
        ActorWork &w = work[A[q]];
        if (out.status[q] != 0) {
            w.rc = CORRO_E_INVALID;
            w.err = "gap bookkeeping input not canonical";
            return;
        }
        const corro::Booked &old = *w.booked;
        const uint64_t rb = in.gap_off[q], ib = in.gap_off[q] + in.ver_off[q] + q;
        std::vector<uint64_t> removed(out.rm_start.begin() + rb, out.rm_start.begin() + rb + out.rm_count[q]);
        std::sort(removed.begin(), removed.end());
        for (uint64_t k = 0; k < out.ins_count[q]; k++) {
            const uint64_t st = out.ins_start[ib + k];
            uint64_t a0 = 0, b0 = 0;
            if (old.needed.get(st, a0, b0) && a0 == st && !std::binary_search(removed.begin(), removed.end(), st)) {
                w.rc = CORRO_E_INVALID;
                w.err = "UNIQUE constraint failed: __corro_bookkeeping_gaps.start";
                return;
            }
        }
        w.next.needed = RangeSet();
        for (uint64_t k = 0; k < out.gap_count[q]; k++) w.next.needed.insert(out.new_start[ib + k], out.new_end[ib + k]);
        w.next.has_max = out.max[q] >= 0;
        w.next.max = out.max[q] >= 0 ? (uint64_t)out.max[q] : 0;
        w.next.partials = old.partials;
        for (uint64_t k = 0; k < out.rm_count[q]; k++)
            w.next.partials.erase(w.next.partials.lower_bound(out.rm_start[rb + k]),
                                  w.next.partials.upper_bound(out.rm_end[rb + k]));
        w.has_next = true;
        for (auto &[version, pv] : w.partials) {
            const corro::PartialVersion &p = w.next.insert_partial(version, std::move(pv));
            if (!p.seqs.has_gap(0, p.last_seq)) w.ready.push_back(version);
        }
    }, 16);
    return CORRO_OK;
}

}  // namespace


namespace {

// corro_process_multiple_changes with CORRO_MEM_DEVICE_HEADERS: the header passes on the device
// (agent_dev_headers decides every changeset its actor's other changesets do not overlap), the host
// walks only the rest, then the same merge / impacts / commit as the host-header path.
int process_dev_headers(corro_ctx *ctx, corro_bookie *bk, const corro_changeset *dcs, uint64_t ncs,
                        const corro_changes *in, corro_process_out *out) {
    static const bool prof = std::getenv("CORRO_AGENT_PROFILE") != nullptr;
    auto t_last = std::chrono::steady_clock::now();
    std::string prof_line;
    auto stage = [&](const char *name) {
        if (!prof) return;
        const auto t = std::chrono::steady_clock::now();
        prof_line += std::string(" ") + name + "=" +
                     std::to_string(std::chrono::duration<double, std::milli>(t - t_last).count()).substr(0, 6);
        t_last = t;
    };
    const uint64_t nchanges = in ? in->n : 0;
    corro::AgentPinned P{};
    TRY_RC(corro::agent_dev_begin(ctx, ncs, nchanges, &P));
    stage("begin");
    const uint32_t nsites = corro::agent_site_count(ctx);
    std::vector<ActorId> site_id(nsites);
    std::vector<int64_t> site_max(nsites, -1);
    for (uint32_t t = 0; t < nsites; t++) {
        corro::agent_site_id(ctx, t, site_id[t].data());
        const corro::Booked *b = booked_of_site(bk, t, site_id[t], false);
        if (b && b->has_max) site_max[t] = (int64_t)b->max;
    }
    corro_changes dv{};
    if (in) dv = *in;
    corro::DevHdrResult R;
    TRY_RC(corro::agent_dev_headers(ctx, dcs, ncs, nchanges ? &dv : nullptr, site_max, out->known, R));
    if (R.err & 1) return fail(CORRO_E_INVALID, "changeset change span outside the batch");
    if (R.err & 2) return fail(CORRO_E_INVALID, "changeset site ordinal is not registered (or actor_id is NULL)");
    stage("headers");

    // A call whose every changeset the device decided (no host changesets) knows its batch now: the
    // order pass (agent_dev_batch_sorted: the applied spans in ActorId order and their positions --
    // device scratch only, neither the state nor the bookie) runs on a second thread while this one
    // walks the actors' bookkeeping. The merge still waits for the walk (a gap conflict fails the call
    // before the state is touched). This thread makes no device call until it joins the other.
    struct EarlyOrder {
        std::thread t;
        int rc = CORRO_OK;
        std::string err;
        corro_changes batch{};
        bool gathered = false;
        corro::AgentPositions pm{};
        ~EarlyOrder() {
            if (t.joinable()) t.join();
        }
    } early;
    {
        const char *gb = std::getenv("CORRO_AGENT_GAPS_BATCH");  // (the batched gap pass uses the device)
        if (R.nh == 0 && nchanges && R.nspans && !(gb && std::atoi(gb) == 1))
            early.t = std::thread([&] {
                try {
                    early.rc = corro::agent_dev_batch_sorted(ctx, &dv, ncs, R.nspans, R.nchanges, R.ts_any, &early.batch,
                                                             &early.gathered, &early.pm);
                    if (early.rc != CORRO_OK) early.err = corro_last_error();
                } catch (const std::bad_alloc &) {
                    early.rc = CORRO_E_NOMEM;
                    early.err = "host allocation failed ordering the batch";
                } catch (const std::exception &e) {
                    early.rc = CORRO_E_INVALID;
                    early.err = e.what();
                }
            });
    }

    // actors of the call, each with its host changesets (R.hcs: grouped by actor in site-rank order)
    std::vector<ActorWork> work;
    std::vector<int64_t> work_of(nsites, -1);
    {
        size_t na = 0;
        for (uint32_t t = 0; t < nsites; t++) na += R.sites[t].gstart != 0xFFFFFFFFu;
        work.reserve(na);  // (no reallocation moves of the per-actor state)
    }
    for (uint32_t t = 0; t < nsites; t++) {
        if (R.sites[t].gstart == 0xFFFFFFFFu) continue;
        work_of[t] = (int64_t)work.size();
        work.emplace_back();
        ActorWork &w = work.back();
        w.site = t;
        w.id = site_id[t];
    }
    for (ActorWork &w : work) {  // Bookie::ensure
        w.booked = booked_of_site(bk, w.site, w.id, true);
        w.had_max = w.booked->has_max;
        w.max = w.booked->max;
    }
    stage("act_setup");
    const uint64_t nh = R.nh;
    const corro_changeset *hcs = R.hcs;
    std::vector<uint8_t> hflag(nh, 0);
    std::vector<int32_t> hknown(nh, CORRO_KNOWN_SKIPPED);
    std::vector<uint64_t> local(nh);
    std::vector<uint64_t> inc_row(nh, ~0ULL);  // host changeset (local index) -> first fetched row
    // partial changesets: canonical ones keep their rows in HBM (bufpool.hip) when the bookie's pool
    // can take them, the others' rows come to the host
    const bool pool_ok = !bk->pool || corro::bufpool_usable(ctx, bk->pool);
    const uint8_t *canon = pool_ok ? R.hcanon : nullptr;
    corro::HostSpanRows inc;
    if (nh) {
        // one pass over the headers (they arrive by DMA: each pass is a DRAM read of 80 B per changeset):
        // the per-actor groups and the partial changesets whose rows come to the host
        // (in parallel chunks: a mixed call's 10^5 headers were 0.6 ms of one thread's reads)
        const auto fetched = [&](const corro_changeset &c, uint64_t k) {
            return c.kind == CORRO_CS_FULL && c.change_count && !is_complete(c) && !R.hbad[k] && !(canon && canon[k]);
        };
        constexpr uint64_t HCH = 4096;
        const uint64_t nch = (nh + HCH - 1) / HCH;
        std::vector<uint64_t> gend(work.size(), 0);
        std::vector<uint8_t> any_fetch(nch, 0);
        run_parallel(nch, [&](size_t ch) {
            const uint64_t lo = ch * HCH, hi = std::min<uint64_t>(nh, lo + HCH);
            for (uint64_t k = lo; k < hi; k++) {
                const corro_changeset &c = hcs[k];
                local[k] = k;
                const size_t wk = (size_t)work_of[c.site];
                if (k == 0 || hcs[k - 1].site != c.site) work[wk].idx = local.data() + k;  // (one group per actor)
                if (k + 1 == nh || hcs[k + 1].site != c.site) gend[wk] = k + 1;
                if (fetched(c, k)) any_fetch[ch] = 1;
            }
        }, 1);
        for (size_t q = 0; q < work.size(); q++)
            if (work[q].idx) work[q].nidx = gend[q] - (uint64_t)(work[q].idx - local.data());
        std::vector<corro::AgentSpan> sp;
        uint64_t r = 0;
        for (uint64_t ch = 0; ch < nch; ch++) {
            if (!any_fetch[ch]) continue;
            for (uint64_t k = ch * HCH; k < std::min<uint64_t>(nh, (ch + 1) * HCH); k++) {
                const corro_changeset &c = hcs[k];
                if (!fetched(c, k)) continue;
                inc_row[k] = r;
                sp.push_back({c.change_off, r, c.change_count, c.ts});
                r += c.change_count;
            }
        }
        stage("host_headers");
        if (!sp.empty()) TRY_RC(corro::agent_dev_fetch(ctx, &dv, sp, inc));
        stage("partial_rows");
    }
    auto row_of = [&](const corro_changeset &c, uint64_t ci, uint64_t k) -> HostRow {
        if (inc_row[ci] == ~0ULL) throw std::logic_error("partial changeset rows not fetched");
        const uint64_t j = inc_row[ci] + k;
        HostRow r;
        r.pk = inc.pk[j];
        r.tcid = inc.tcid[j];
        r.cv = inc.cv[j];
        r.dbv = inc.dbv[j];
        r.cl = inc.cl[j];
        r.seq = inc.seq[j];
        r.site = inc.site[j];
        r.v0 = inc.v0[j];
        r.v1 = in->val1 ? inc.v1[j] : 0;
        r.vt = inc.vt[j];
        r.vl = in->val_len ? inc.vl[j] : 0;
        r.ts = in->ts ? inc.ts[j] : c.ts;
        if (inc.lv_len[j])
            r.lv.assign(reinterpret_cast<const char *>(inc.lv_data.data() + inc.lv_off[j]), inc.lv_len[j]);
        return r;
    };
    // (R's runs are grouped by site: each actor's are one slice of the columns)
    std::vector<RunView> dev_runs(work.size());
    for (size_t r = 0; r < R.run_site.size();) {
        size_t q = r + 1;
        while (q < R.run_site.size() && R.run_site[q] == R.run_site[r]) q++;
        RunView &rv = dev_runs[(size_t)work_of[R.run_site[r]]];
        if (rv.n) throw std::logic_error("device runs not grouped by site");
        rv = RunView{R.run_start.data() + r, R.run_end.data() + r, nullptr, q - r};
        r = q;
    }
    const CsView view{hcs, R.hbad, hknown.data(), hflag.data(), canon, canon ? R.hctab : nullptr};
    if (want_gaps_batch(work))
        for (ActorWork &w : work) w.defer_gaps = true;
    stage("act_runs");
    run_parallel(work.size(), [&](size_t k) { run_actor_walk(bk, work[k], view, dev_runs[k], row_of); });
    TRY_RC(gaps_batch(ctx, work));
    for (ActorWork &w : work)
        if (w.rc != CORRO_OK) return fail(w.rc, w.err);
    stage("act_walk");
    if (prof) {  // the walk's parts summed over actors (thread-ms; the pool runs up to 16 at once)
        double tw[4] = {0, 0, 0, 0};
        for (const ActorWork &w : work)
            for (int k = 0; k < 4; k++) tw[k] += w.t_walk[k];
        char buf[160];
        snprintf(buf, sizeof buf, " [walk thread-ms: runs=%.2f pass1=%.2f pass2=%.2f gaps=%.2f]", tw[0], tw[1], tw[2], tw[3]);
        prof_line += buf;
    }
    uint64_t nspans = R.nspans, nb = R.nchanges;
    for (const ActorWork &w : work) {
        nspans += w.nspans;
        nb += w.nchanges;
    }
    if (nh) TRY_RC(corro::agent_dev_put_host(ctx, R.hidx, nh, hflag, hknown, out->known));
    stage("actors");

    const uint32_t ntables = corro::agent_table_count(ctx);
    std::vector<uint64_t> committed(ntables, 0);
    // actors in ActorId order: the device sort's site-rank order (each actor's first sorted slot)
    std::vector<size_t> order(work.size());
    for (size_t k = 0; k < order.size(); k++) order[k] = k;
    std::sort(order.begin(), order.end(),
              [&](size_t x, size_t y) { return R.sites[work[x].site].gstart < R.sites[work[y].site].gstart; });
    std::vector<Staged *> sto;
    for (size_t k : order) sto.push_back(&work[k].st);
    // The buffered-row commit's preparation only reads the bookie and the staged rows, so it runs on a
    // host thread while the merge runs on the device (its writes wait for the merge: a failed merge
    // leaves the bookie as it was).
    // (and the seq books' moves and the buffered-meta keys the commit will leave, both read-only too)
    CommitPrep prep;
    SeqPrep seqp;
    std::vector<uint64_t> pre_keys;
    bool seq_ready = false, keys_ready = false;
    std::string prep_err;
    int prep_rc = CORRO_OK;
    bool prep_started = false;
    std::thread prep_thread;
    const char *pm_env = std::getenv("CORRO_AGENT_PREP_MIN");  // (read per call: tests run small calls through it)
    const uint64_t prep_min = pm_env ? std::strtoull(pm_env, nullptr, 10) : 4096;
    if (nh >= prep_min) {
        prep_started = true;
        prep_thread = std::thread([&, have_dv = nchanges != 0] {
            auto t0 = std::chrono::steady_clock::now();
            auto markp = [&](const char *name) {
                if (!prof) return;
                const auto t = std::chrono::steady_clock::now();
                prep.prof += std::string(" ") + name + "=" +
                             std::to_string(std::chrono::duration<double, std::milli>(t - t0).count()).substr(0, 6);
                t0 = t;
            };
            try {
                // (the seq books' moves on a third thread: they read other staged data and other bookie
                // tables than the buffered-row preparation, and both have serial stretches)
                std::string seq_err;
                bool seq_ok = false, seq_oom = false;
                std::thread seq_thread([&] {
                    try {
                        seqbook_prepare(bk, sto, seqp);
                        seq_ok = true;
                    } catch (const std::bad_alloc &) {
                        seq_oom = true;
                    } catch (const std::exception &e) {
                        seq_err = e.what();
                    }
                });
                try {
                    commit_prepare(ctx, bk, have_dv, sto, ntables, prep, markp);
                } catch (...) {
                    seq_thread.join();
                    throw;
                }
                seq_thread.join();
                if (seq_oom) throw std::bad_alloc();
                if (!seq_ok) throw std::runtime_error(seq_err);
                seq_ready = true;
                markp("seq_prep");
                if (!prep.any || prep.fast) {
                    pre_keys = buffered_keys_after(bk, prep, seqp);
                    keys_ready = true;
                    markp("keys_prep");
                }
            } catch (const std::bad_alloc &) {  // (same code as the serial path's host OOM)
                prep_rc = CORRO_E_NOMEM;
                prep_err = "host allocation failed preparing the commit";
            } catch (const std::exception &e) {
                prep_rc = CORRO_E_INVALID;
                prep_err = e.what();
            } catch (...) {
                prep_rc = CORRO_E_INVALID;
                prep_err = "unknown host exception";
            }
        });
    }
    struct JoinPrep {  // (every return path waits for the preparation thread)
        std::thread &t;
        ~JoinPrep() {
            if (t.joinable()) t.join();
        }
    } join_prep{prep_thread};
    const bool early_ran = early.t.joinable();
    if (early_ran) early.t.join();  // (before this thread's next device call: one thread on ctx at a time)
    if (early_ran && early.rc != CORRO_OK) return fail(early.rc, early.err);
    if (nb || out->impactful) {
        corro_changes batch{};
        const uint8_t *imp = nullptr;
        corro::AgentPositions pm{};
        if (nb) {
            bool gathered = false;
            if (early_ran) {  // (ordered alongside the walk)
                if (nspans != R.nspans || nb != R.nchanges) throw std::logic_error("early order: the walk added spans");
                batch = early.batch;
                gathered = early.gathered;
                pm = early.pm;
                stage("order_joined");
            } else {
                TRY_RC(corro::agent_dev_batch_sorted(ctx, &dv, ncs, nspans, nb, R.ts_any, &batch, &gathered, &pm));
                stage(gathered ? "order+gather" : (pm.on ? "order+positions" : "order"));
            }
            int rc = CORRO_OK;
            uint8_t *ib = corro::agent_dev_impact_buf(ctx, nb, &rc);
            if (rc != CORRO_OK) return rc;
            corro_apply_out ao{};
            ao.impact = ib;
            corro::agent_dev_set_positions(ctx, pm.on ? &pm : nullptr);
            rc = corro_apply_batch(ctx, &batch, CORRO_MEM_DEVICE, &ao);
            corro::agent_dev_set_positions(ctx, nullptr);
            if (rc != CORRO_OK) {  // the transaction fails as a whole (util.rs:849-855)
                (void)corro::agent_dev_clear_known(ctx, out->known, ncs);
                return rc;
            }
            imp = ib;
            stage("apply");
        }
        TRY_RC(corro::agent_dev_impacts(ctx, imp, batch.table_cid, pm.on, nb, P, ncs, nspans, out->impactful, nchanges,
                                        CORRO_MEM_DEVICE, ntables));
        for (uint32_t t = 0; t < ntables; t++) committed[t] += P.committed[t];
        stage("impacts");
    }

    // commit
    {  // crsql_set_db_version of every processed empty version, one device pass
        std::vector<std::pair<uint32_t, uint64_t>> sv;
        for (ActorWork &w : work)
            for (uint64_t version : w.set_dbv) sv.emplace_back(w.site, version);
        TRY_RC(corro::set_db_versions(ctx, sv));
    }
    if (prep_started) {
        prep_thread.join();
        if (prep_rc != CORRO_OK) return fail(prep_rc, "process_multiple_changes: " + prep_err);
        if (prof) prof_line += " [prepared alongside the merge:" + prep.prof + "]";
    }
    TRY_RC(commit_staged(ctx, bk, nchanges ? &dv : nullptr, sto, committed, stage, prep_started ? &prep : nullptr));
    if (seq_ready) seqbook_apply(bk, seqp);
    else commit_seqbook(bk, sto);
    stage("seqbook");
    // check_buffered_meta_to_clear (util.rs:513-520, :1292-1303): the merged versions that hold
    // buffered rows or seq bookkeeping, found on the device against the (small) set of such keys
    std::vector<uint64_t> bkeys = keys_ready ? std::move(pre_keys) : buffered_keys(bk);
    stage("bkeys");
    std::vector<std::pair<uint32_t, uint64_t>> sv;
    TRY_RC(corro::agent_dev_commit_headers(ctx, ncs, out->known, bkeys.empty() ? nullptr : &bkeys, &sv));
    stage("commit_hdr");
    if (prof) prof_line += " [cleared_versions=" + std::to_string(sv.size()) + " meta_keys=" + std::to_string(bkeys.size()) + "]";
    clear_buffered_each(bk, sv);
    stage("clear");
    compact_tables(bk);
    stage("compact");
    uint64_t nready = 0;
    for (size_t k : order) {
        ActorWork &w = work[k];
        if (w.has_next) std::swap(*w.booked, w.next);  // (the old state is freed with the call's work)
        for (uint64_t v : w.ready) bk->ready.emplace_back(w.id, v);
        nready += w.ready.size();
    }
    out->n_ready = nready;
    corro_detail_add_committed(ctx, committed.data(), committed.size());
    stage("commit");
    if (nh >= 4096) Reaper::get().give(std::move(work));  // (freed after the call returns)
    stage("free");
    if (prof) fprintf(stderr, "[corro agent dev] ncs=%llu spans=%llu changes=%llu host=%zu ms:%s\n", (unsigned long long)ncs,
                      (unsigned long long)nspans, (unsigned long long)nb, (size_t)nh, prof_line.c_str());
    return CORRO_OK;
}

// CORRO_MEM_DEVICE with headers in host memory, for large calls: the headers are copied into a
// pinned area in parallel chunks (each checked against the registered actor ids and uploaded as soon
// as it is copied), then the device header passes run as with CORRO_MEM_DEVICE_HEADERS and the
// outcomes come back in one copy. The host header walk (the form below) costs more than the copy
// once a call carries tens of thousands of changesets.
int process_staged_headers(corro_ctx *ctx, corro_bookie *bk, const corro_changeset *cs, uint64_t ncs,
                           const corro_changes *in, corro_process_out *out) {
    corro::HdrStage st{};
    TRY_RC(corro::agent_dev_stage_begin(ctx, ncs, &st));
    const uint32_t nsites = corro::agent_site_count(ctx);
    std::vector<ActorId> site_id(nsites);
    for (uint32_t k = 0; k < nsites; k++) corro::agent_site_id(ctx, k, site_id[k].data());
    const size_t nchunk = std::max<size_t>(1, std::min<size_t>(16, ncs / 4096));
    std::vector<int> cerr(nchunk, CORRO_OK);
    run_parallel(nchunk, [&](size_t k) {
        const uint64_t lo = ncs * k / nchunk, hi = ncs * (k + 1) / nchunk;
        std::memcpy(st.pinned + lo, cs + lo, (hi - lo) * sizeof(corro_changeset));
        const uint8_t *last_ptr = nullptr;
        uint32_t last_site = 0xFFFFFFFFu;
        for (uint64_t i = lo; i < hi; i++) {
            const corro_changeset &c = st.pinned[i];
            if (c.site >= nsites || !c.actor_id) {
                cerr[k] = 2;
                return;
            }
            if (c.actor_id != last_ptr || c.site != last_site) {
                if (std::memcmp(site_id[c.site].data(), c.actor_id, 16) != 0) {
                    cerr[k] = 3;
                    return;
                }
                last_ptr = c.actor_id;
                last_site = c.site;
            }
        }
        cerr[k] = corro::agent_dev_stage_upload(ctx, st, lo, hi) == CORRO_OK ? CORRO_OK : 4;
    }, 1);
    auto skip_all = [&]() {
        for (uint64_t i = 0; i < ncs; i++) out->known[i] = CORRO_KNOWN_SKIPPED;
    };
    for (int e : cerr) {
        if (e == CORRO_OK) continue;
        skip_all();
        if (e == 2) return fail(CORRO_E_INVALID, "changeset site ordinal is not registered (or actor_id is NULL)");
        if (e == 3) return fail(CORRO_E_INVALID, "changeset site ordinal does not name its actor_id");
        return fail(CORRO_E_DEVICE, "header upload failed");
    }
    corro_process_out o2 = *out;
    o2.known = st.dknown;
    const int rc = process_dev_headers(ctx, bk, st.dev, ncs, in, &o2);
    out->n_ready = o2.n_ready;
    if (rc != CORRO_OK) {
        const std::string msg = corro_last_error();
        skip_all();
        return fail(rc, msg);
    }
    TRY_RC(corro::agent_dev_stage_known(ctx, st, out->known, ncs));
    return CORRO_OK;
}

}  // namespace

namespace {
int process_multiple_changes(corro_ctx *ctx, corro_bookie *bk, const corro_changeset *cs, uint64_t ncs,
                             const corro_changes *in, int mem, corro_process_out *out) {
    if (!ctx || !bk || (ncs && !cs) || !out) return fail(CORRO_E_INVALID, "NULL argument");
    if (ncs && (!out->known)) return fail(CORRO_E_INVALID, "out->known is required");
    if (mem != CORRO_MEM_HOST && mem != CORRO_MEM_DEVICE && mem != CORRO_MEM_DEVICE_HEADERS)
        return fail(CORRO_E_INVALID, "bad mem kind");
    const uint64_t nchanges = in ? in->n : 0;
    if (nchanges && !in->table_cid) return fail(CORRO_E_INVALID, "a required batch array is NULL");
    out->n_ready = 0;
    if (mem == CORRO_MEM_DEVICE_HEADERS) return process_dev_headers(ctx, bk, cs, ncs, in, out);
    // host headers of a device batch: staged for the device header passes when the call is large
    // (CORRO_AGENT_STAGE_HEADERS=1 always, =0 never; tests)
    const char *stage_e = std::getenv("CORRO_AGENT_STAGE_HEADERS");
    const int stage_env = stage_e ? std::atoi(stage_e) : -1;
    if (mem == CORRO_MEM_DEVICE && ncs && (stage_env == 1 || (stage_env == -1 && ncs >= 32768)))
        return process_staged_headers(ctx, bk, cs, ncs, in, out);

    // CORRO_AGENT_PROFILE=1: host-side stage times of each call on stderr (tools)
    static const bool prof = std::getenv("CORRO_AGENT_PROFILE") != nullptr;
    auto t_last = std::chrono::steady_clock::now();
    std::string prof_line;
    auto stage = [&](const char *name) {
        if (!prof) return;
        const auto t = std::chrono::steady_clock::now();
        prof_line += std::string(" ") + name + "=" +
                     std::to_string(std::chrono::duration<double, std::milli>(t - t_last).count()).substr(0, 6);
        t_last = t;
    };
    corro::AgentPinned P{};
    TRY_RC(corro::agent_dev_begin(ctx, ncs, nchanges, &P));
    stage("begin");

    // Host passes walk the headers in ARRIVAL order (sequential chunks in parallel threads): an actor's
    // changesets are interleaved with everyone else's, so a walk in actor order would miss the cache
    // on every header. Per-changeset results go to the pinned arrays; the regroup into ActorId order
    // happens on the device (agent_dev_batch).
    const uint32_t nsites = corro::agent_site_count(ctx);
    std::vector<std::array<uint8_t, 16>> site_id(nsites);
    for (uint32_t k = 0; k < nsites; k++) corro::agent_site_id(ctx, k, site_id[k].data());
    const size_t nchunk = std::max<size_t>(1, std::min<size_t>(16, ncs / 4096));
    auto chunk_of = [&](size_t k, uint64_t &lo, uint64_t &hi) {
        lo = ncs * k / nchunk;
        hi = ncs * (k + 1) / nchunk;
    };
    // per (chunk, site): changesets, first / last version, every one a complete Full ascending
    struct SiteStat {
        uint64_t count = 0, first = 0, last = 0;
        bool ok = true;
    };
    std::vector<std::vector<SiteStat>> cstat(nchunk);
    std::vector<int> cerr(nchunk, CORRO_OK);
    std::vector<uint64_t> cfull(nchunk, 0);
    std::vector<uint8_t> chunk_ts(nchunk, 0);
    const bool in_ts = in && in->ts;
    // compact per-changeset copy of what the later host pass reads (8 B instead of the 80-B header);
    // kept by the bookie between calls (no fresh pages to fault in per call)
    if (bk->scratch_ver.size() < ncs) bk->scratch_ver.resize(ncs);
    uint64_t *ver = bk->scratch_ver.data();
    // 1. headers: spans checked, staged for the device, actors checked against the registered ids
    run_parallel(nchunk, [&](size_t k) {
        uint64_t lo, hi;
        chunk_of(k, lo, hi);
        bool cts = false;
        struct Flush {
            std::vector<uint8_t> &v; size_t k; bool &b;
            ~Flush() { v[k] = b; }
        } flush{chunk_ts, k, cts};
        std::vector<SiteStat> &st = cstat[k];
        st.assign(nsites, SiteStat{});
        const uint8_t *last_ptr = nullptr;
        uint32_t last_site = 0xFFFFFFFFu;
        for (uint64_t i = lo; i < hi; i++) {
            const corro_changeset &c = cs[i];
            out->known[i] = CORRO_KNOWN_SKIPPED;
            const bool full = c.kind == CORRO_CS_FULL && c.change_count;
            if (full && (!in || c.change_off > nchanges || c.change_count > nchanges - c.change_off)) {
                cerr[k] = 1;
                return;
            }
            if (c.site >= nsites || !c.actor_id) {
                cerr[k] = 2;
                return;
            }
            if (c.actor_id != last_ptr || c.site != last_site) {  // (a run of one actor checks once)
                if (std::memcmp(site_id[c.site].data(), c.actor_id, 16) != 0) {
                    cerr[k] = 3;
                    return;
                }
                last_ptr = c.actor_id;
                last_site = c.site;
            }
            P.off[i] = full ? c.change_off : 0;
            P.cnt[i] = full ? c.change_count : 0;
            if (!in_ts) P.ts[i] = c.ts;  // (per-change ts in the input: the span ts is never read)
            P.site[i] = c.site;
            P.flag[i] = 0;
            ver[i] = c.version_start;
            cts |= c.ts != 0;
            cfull[k] += full;
            SiteStat &t = st[c.site];
            const bool fast = c.kind == CORRO_CS_FULL && is_complete(c) && (!t.count || c.version_start > t.last);
            if (!t.count) t.first = c.version_start;
            t.last = c.version_start;
            t.ok = t.ok && fast;
            t.count++;
        }
    }, 1);
    for (int e : cerr) {
        if (e == 1) return fail(CORRO_E_INVALID, "changeset change span outside the batch");
        if (e == 2) return fail(CORRO_E_INVALID, "changeset site ordinal is not registered (or actor_id is NULL)");
        if (e == 3) return fail(CORRO_E_INVALID, "changeset site ordinal does not name its actor_id");
    }
    uint64_t nfull = 0;
    for (uint64_t f : cfull) nfull += f;
    // actors; the fast ones (every changeset a complete Full version, strictly ascending in arrival
    // order) need no per-actor walk: no version repeats, so no batch-local dedup and nothing already
    // seen in this call -- pass 1's contains_all is the only check left, made per changeset below
    std::vector<ActorWork> work;
    work.reserve(std::min<uint64_t>(nsites, ncs));  // (no reallocation moves of the per-actor state)
    std::vector<int64_t> work_of(nsites, -1);
    bool any_slow = false;
    for (uint32_t t = 0; t < nsites; t++) {
        uint64_t count = 0, last = 0;
        bool ok = true;
        for (size_t k = 0; k < nchunk; k++) {
            const SiteStat &x = cstat[k][t];
            if (!x.count) continue;
            ok = ok && x.ok && (!count || x.first > last);
            last = x.last;
            count += x.count;
        }
        if (!count) continue;
        work_of[t] = (int64_t)work.size();
        work.emplace_back();
        ActorWork &w = work.back();
        w.site = t;
        w.fast = ok;
        w.nidx = count;
        std::memcpy(w.id.data(), site_id[t].data(), 16);
        any_slow |= !ok;
    }
    for (ActorWork &w : work) {  // Bookie::ensure (std::map nodes: stable pointers for the workers)
        w.booked = booked_of_site(bk, w.site, w.id, true);
        w.had_max = w.booked->has_max;
        w.max = w.booked->max;
    }
    // the changesets of the other actors, grouped (stable counting sort by site)
    std::vector<uint64_t> by_actor;
    if (any_slow) {
        std::vector<uint64_t> base(work.size() + 1, 0);
        for (size_t k = 0; k < work.size(); k++) base[k + 1] = base[k] + (work[k].fast ? 0 : work[k].nidx);
        by_actor.resize(base.back());
        std::vector<uint64_t> cur(base.begin(), base.end() - 1);
        for (uint64_t i = 0; i < ncs; i++) {
            const ActorWork &w = work[(size_t)work_of[cs[i].site]];
            if (!w.fast) by_actor[cur[(size_t)work_of[cs[i].site]]++] = i;
        }
        for (size_t k = 0; k < work.size(); k++) work[k].idx = by_actor.data() + base[k];
    }
    stage("headers");

    // 2. the device view of the input and the per-changeset unknown-name screen (one kernel)
    corro_changes dv{};
    if (nfull) {
        TRY_RC(corro::agent_dev_input(ctx, in, mem, &dv));
        TRY_RC(corro::agent_dev_bad(ctx, &dv, P, ncs));
    } else {
        for (uint64_t i = 0; i < ncs; i++) P.bad[i] = 0;
    }
    const uint8_t *bad = P.bad;
    // the changes of incomplete versions are buffered on the host: fetched once (device input)
    std::map<uint64_t, uint64_t> inc_row;  // changeset -> first fetched row
    corro::HostSpanRows inc;
    if (mem == CORRO_MEM_DEVICE && any_slow) {
        std::vector<corro::AgentSpan> sp;
        uint64_t r = 0;
        for (uint64_t i = 0; i < ncs; i++)
            if (cs[i].kind == CORRO_CS_FULL && cs[i].change_count && !is_complete(cs[i]) && !bad[i]) {
                inc_row[i] = r;
                sp.push_back({cs[i].change_off, r, cs[i].change_count, cs[i].ts});
                r += cs[i].change_count;
            }
        stage("slow_headers");
        if (!sp.empty()) TRY_RC(corro::agent_dev_fetch(ctx, &dv, sp, inc));
        stage("partial_rows");
    }
    auto row_of = [&](const corro_changeset &c, uint64_t ci, uint64_t k) -> HostRow {
        if (mem == CORRO_MEM_HOST) return row_at(in, c.change_off + k, c.ts);
        const uint64_t j = inc_row.at(ci) + k;
        HostRow r;
        r.pk = inc.pk[j];
        r.tcid = inc.tcid[j];
        r.cv = inc.cv[j];
        r.dbv = inc.dbv[j];
        r.cl = inc.cl[j];
        r.seq = inc.seq[j];
        r.site = inc.site[j];
        r.v0 = inc.v0[j];
        r.v1 = in->val1 ? inc.v1[j] : 0;
        r.vt = inc.vt[j];
        r.vl = in->val_len ? inc.vl[j] : 0;
        r.ts = in->ts ? inc.ts[j] : c.ts;
        if (inc.lv_len[j])
            r.lv.assign(reinterpret_cast<const char *>(inc.lv_data.data() + inc.lv_off[j]), inc.lv_len[j]);
        return r;
    };
    stage("screen");

    // 3a. the fast actors' changesets, in arrival order (chunks in parallel): each one new to the actor
    // (contains_all) is merged, or cleared when empty (process_empty_version, util.rs:810-824), or
    // rolled back alone when it names an unknown table / column (util.rs:839-860). Their version runs
    // per (chunk, actor) feed the gap bookkeeping.
    struct ChunkOut {
        std::vector<std::pair<uint32_t, Range>> runs;  // (work index, versions) in arrival order
        std::vector<std::pair<uint32_t, uint64_t>> set_dbv;
        uint64_t nspans = 0, nb = 0;
        bool ts = false;
    };
    std::vector<ChunkOut> cout(nchunk);
    run_parallel(nchunk, [&](size_t k) {
        uint64_t lo, hi;
        chunk_of(k, lo, hi);
        ChunkOut &o = cout[k];
        std::vector<int64_t> open(work.size(), -1);  // index into o.runs of the actor's open run
        for (uint64_t i = lo; i < hi; i++) {
            const uint32_t wi = (uint32_t)work_of[P.site[i]];
            const ActorWork &w = work[wi];
            if (!w.fast) continue;
            const uint64_t v = ver[i];
            if (w.had_max && v <= w.max) {
                Range sq{cs[i].seq_start, cs[i].seq_end};
                if (w.booked->contains_all(v, v, &sq)) continue;
            }
            if (P.cnt[i] == 0) {  // (a fast actor's changesets are all Full: cnt 0 = no changes)
                if (!w.had_max || v > w.max) o.set_dbv.emplace_back(wi, v);
                out->known[i] = CORRO_KNOWN_CLEARED;
            } else if (bad[i]) {
                out->known[i] = CORRO_E_UNKNOWN_COLUMN;
                continue;
            } else {
                P.flag[i] = 1;
                out->known[i] = CORRO_KNOWN_CURRENT;
                o.nspans++;
                o.nb += P.cnt[i];
            }
            int64_t &r = open[wi];
            if (r >= 0 && o.runs[(size_t)r].second.second + 1 == v) {
                o.runs[(size_t)r].second.second = v;
            } else {
                r = (int64_t)o.runs.size();
                o.runs.emplace_back(wi, Range{v, v});
            }
        }
    }, 1);
    // 3b. per actor: the other actors' passes 1 and 2 (util.rs:704-884), then every actor's gap
    // snapshot (:894-932)
    std::vector<std::vector<Range>> fast_runs(work.size());
    for (size_t k = 0; k < nchunk; k++)
        for (auto &[wi, r] : cout[k].runs) fast_runs[wi].push_back(r);
    const CsView view{cs, bad, out->known, P.flag, nullptr, nullptr};
    auto run_actor = [&](size_t wi) {
        run_actor_walk(bk, work[wi], view, RunView{nullptr, nullptr, fast_runs[wi].data(), fast_runs[wi].size()}, row_of);
    };
    if (want_gaps_batch(work))
        for (ActorWork &w : work) w.defer_gaps = true;
    run_parallel(work.size(), [&](size_t k) { run_actor(k); });
    TRY_RC(gaps_batch(ctx, work));
    for (ActorWork &w : work)
        if (w.rc != CORRO_OK) return fail(w.rc, w.err);
    uint64_t nspans = 0, nb = 0;
    bool need_ts = false;
    for (size_t k = 0; k < nchunk; k++) {
        nspans += cout[k].nspans;
        nb += cout[k].nb;
        need_ts |= chunk_ts[k] != 0;  // (any changeset's ts: a superset of the applied ones')
    }
    for (const ActorWork &w : work) {
        nspans += w.nspans;
        nb += w.nchanges;
        need_ts |= w.ts;
    }
    stage("actors");

    // 4. the merge: one batch of every flagged changeset, actors in ActorId byte order (the device
    // orders and gathers them)
    const uint32_t ntables = corro::agent_table_count(ctx);
    std::vector<uint64_t> committed(ntables, 0);
    if (nb || out->impactful) {
        corro_changes batch{};
        const uint8_t *imp = nullptr;
        corro::AgentPositions pm{};
        if (nb) {
            bool gathered = false;
            TRY_RC(corro::agent_dev_batch(ctx, &dv, P, ncs, nspans, nb, need_ts, &batch, &gathered, &pm));
            stage(gathered ? "order+gather" : (pm.on ? "order+positions" : "order"));
            int rc = CORRO_OK;
            uint8_t *ib = corro::agent_dev_impact_buf(ctx, nb, &rc);
            if (rc != CORRO_OK) return rc;
            corro_apply_out ao{};
            ao.impact = ib;
            // (position mode: the input where it lies, each change at its application position)
            corro::agent_dev_set_positions(ctx, pm.on ? &pm : nullptr);
            rc = corro_apply_batch(ctx, &batch, CORRO_MEM_DEVICE, &ao);
            corro::agent_dev_set_positions(ctx, nullptr);
            if (rc != CORRO_OK) {  // the transaction fails as a whole (util.rs:849-855)
                for (uint64_t i = 0; i < ncs; i++) out->known[i] = CORRO_KNOWN_SKIPPED;
                return rc;
            }
            imp = ib;
            stage("apply");
        }
        TRY_RC(corro::agent_dev_impacts(ctx, imp, batch.table_cid, pm.on, nb, P, ncs, nspans, out->impactful, nchanges,
                                        mem, ntables));
        for (uint32_t t = 0; t < ntables; t++) committed[t] += P.committed[t];
        stage("impacts");
    }

    // 5. commit: everything below only records what the successful transaction did
    {  // crsql_set_db_version of every processed empty version, one device pass
        std::vector<std::pair<uint32_t, uint64_t>> sv;
        for (const ChunkOut &o : cout)
            for (auto &[wi, version] : o.set_dbv) sv.emplace_back(work[wi].site, version);
        for (ActorWork &w : work)
            for (uint64_t version : w.set_dbv) sv.emplace_back(w.site, version);
        TRY_RC(corro::set_db_versions(ctx, sv));
    }
    // corro.changes.committed{table} (util.rs:533-535): every buffered change of an incomplete version
    // (:1101-1105), every impactful change of a complete one (:1254-1258, counted on the device)
    std::vector<size_t> order(work.size());
    for (size_t k = 0; k < order.size(); k++) order[k] = k;
    std::sort(order.begin(), order.end(), [&](size_t x, size_t y) { return work[x].id < work[y].id; });
    {
        std::vector<Staged *> sto;
        for (size_t k : order) sto.push_back(&work[k].st);
        TRY_RC(commit_staged(ctx, bk, nullptr, sto, committed));
        commit_seqbook(bk, sto);
    }
    // known: Current when the version had an impactful change, else Cleared (util.rs:1264-1287)
    const std::vector<uint64_t> bkeys = buffered_keys(bk);
    if (nspans)
        run_parallel(nchunk, [&](size_t k) {
            uint64_t lo, hi;
            chunk_of(k, lo, hi);
            for (uint64_t i = lo; i < hi; i++)
                if (P.flag[i]) out->known[i] = P.any[i] ? CORRO_KNOWN_CURRENT : CORRO_KNOWN_CLEARED;
        }, 1);
    // check_buffered_meta_to_clear (util.rs:513-520, :1292-1303)
    if (!bkeys.empty())
        for (uint64_t i = 0; i < ncs; i++)
            if (P.flag[i] && cs[i].version_start < (1ULL << 40) &&
                std::binary_search(bkeys.begin(), bkeys.end(), (uint64_t)cs[i].site << 40 | cs[i].version_start))
                clear_buffered(bk, cs[i].site, cs[i].version_start, cs[i].version_start);
    compact_tables(bk);
    // per-actor gap snapshot commit, then partials (util.rs:936-1008), actors in ActorId order
    uint64_t nready = 0;
    for (size_t k : order) {
        ActorWork &w = work[k];
        if (w.has_next) std::swap(*w.booked, w.next);  // (the old state is freed with the call's work)
        for (uint64_t v : w.ready) bk->ready.emplace_back(w.id, v);
        nready += w.ready.size();
    }
    out->n_ready = nready;
    corro_detail_add_committed(ctx, committed.data(), committed.size());
    stage("commit");
    if (prof) fprintf(stderr, "[corro agent] ncs=%llu spans=%llu changes=%llu ms:%s\n", (unsigned long long)ncs,
                      (unsigned long long)nspans, (unsigned long long)nb, prof_line.c_str());
    return CORRO_OK;
}

}  // namespace

extern "C" {

// The C ABI never lets a C++ exception out (a host allocation failing inside the header walks or the
// host pool's workers): std::bad_alloc is CORRO_E_NOMEM, anything else CORRO_E_INVALID.
// Failure atomicity of the call: a failure BEFORE the merge or any crsql_set_db_version wrote the state
// leaves the state, the bookie's Booked versions and its buffered rows as they were (the caller's
// transaction rolls back, util.rs:849-855). A failure AFTER one of them (the buffered-row commit, the
// header commit, a host exception in the bookkeeping) cannot be undone on the device: the context is
// poisoned (every later call fails until corro_state_reset, as for a mid-apply failure) and the bookie
// keeps no pending buffered segment of the failed call (commit_staged), but its Booked versions do not
// include the call either, so the caller re-seeds both from its durable store (corro_hip.h, "Failure
// atomicity").
int corro_process_multiple_changes(corro_ctx *ctx, corro_bookie *bk, const corro_changeset *cs, uint64_t ncs,
                                   const corro_changes *in, int mem, corro_process_out *out) {
    if (ctx && corro::ctx_poisoned(ctx))
        return fail(CORRO_E_DEVICE, "context poisoned: an earlier call failed after it began writing the state; "
                                    "call corro_state_reset");
    const uint64_t mark0 = ctx ? corro::ctx_write_mark(ctx) : 0;
    int rc;
    try {
        rc = process_multiple_changes(ctx, bk, cs, ncs, in, mem, out);
    } catch (const std::bad_alloc &) {
        rc = fail(CORRO_E_NOMEM, "host allocation failed in process_multiple_changes");
    } catch (const std::exception &e) {
        rc = fail(CORRO_E_INVALID, std::string("process_multiple_changes: ") + e.what());
    } catch (...) {
        rc = fail(CORRO_E_INVALID, "process_multiple_changes: unknown host exception");
    }
    if (rc != CORRO_OK && ctx && corro::ctx_write_mark(ctx) != mark0)
        corro::ctx_poison(ctx, " (after the merge: the context is poisoned until corro_state_reset)");
    return rc;
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
    if (pit->second.seqs.has_gap(0, pit->second.last_seq)) return CORRO_OK;  // gaps: abort
    const uint32_t site = sit->second;
    Batch batch;
    if (BufEntry *rows = bk->buffered.find({site, (int64_t)version})) {
        TRY_RC(materialize(bk, *rows));
        for (const HostRow &r : rows->rows) batch.push(r);  // ORDER BY db_version, seq
    }
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
    compact_tables(bk);
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
    const SeqBook *sb = bk->seqbook.find({so->second, version});
    if (!sb) return CORRO_OK;
    std::vector<Range> rs(sb->ranges.begin(), sb->ranges.end());
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
    *last_seq = (int64_t)sb->last_seq;
    *ts = sb->ts;
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
    for (size_t i = bk->buffered.lower({so->second, (int64_t)vstart}); i < bk->buffered.slots(); i++) {
        const auto &x = bk->buffered.at(i);
        if (x.key.first != so->second || (uint64_t)x.key.second > vend) break;
        if (x.dead || x.val.empty()) continue;
        if (k < cap) versions[k] = (uint64_t)x.key.second;
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
    BufEntry *it = version <= (uint64_t)INT64_MAX ? bk->buffered.find({so->second, (int64_t)version}) : nullptr;
    if (!it || seq_start > seq_end || seq_start > 0xFFFFFFFFULL) return CORRO_OK;
    TRY_RC(materialize(bk, *it));
    const BufRows &rows = it->rows;
    const uint32_t hi = seq_end > 0xFFFFFFFFULL ? 0xFFFFFFFFu : (uint32_t)seq_end;
    uint64_t k = 0;
    for (auto r = buf_lower(rows, (uint32_t)seq_start); r != rows.end() && r->seq <= hi; ++r, ++k) {
        if (k >= cap) continue;
        const HostRow &h = *r;
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
    BufEntry *it = version <= (uint64_t)INT64_MAX ? bk->buffered.find({so->second, (int64_t)version}) : nullptr;
    if (!it) return CORRO_OK;
    TRY_RC(materialize(bk, *it));
    auto r = buf_lower(it->rows, (uint32_t)seq);
    if (r == it->rows.end() || r->seq != (uint32_t)seq) return CORRO_OK;
    const std::string &lv = r->lv;
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
