// Host-side gap bookkeeping: BookedVersions / VersionsSnapshot::insert_db
// (/root/reference/crates/corro-types/src/agent.rs:1108-1235 and :1260-1458).
//
// RangeInclusiveSet<u64> (rangemap 1.5.1) is modelled as an ordered map start -> end whose
// ranges are disjoint and never touch (touching ranges coalesce, StepLite semantics).
#include <algorithm>
#include <cstdint>
#include <map>
#include <set>
#include <string>
#include <utility>
#include <vector>

#include "corro_hip.h"

namespace corro {
int fail(int code, const std::string &msg);

class RangeSet {
  public:
    using Map = std::map<uint64_t, uint64_t>;

    void insert(uint64_t s, uint64_t e) {
        if (s > e) return;
        auto it = m_.upper_bound(s);
        if (it != m_.begin()) {
            auto prev = std::prev(it);
            if (prev->second == UINT64_MAX || prev->second + 1 >= s) {  // overlaps or touches
                s = prev->first;
                e = std::max(e, prev->second);
                it = m_.erase(prev);
            }
        }
        while (it != m_.end() && (e == UINT64_MAX || it->first <= e + 1)) {
            e = std::max(e, it->second);
            it = m_.erase(it);
        }
        m_[s] = e;
    }

    void remove(uint64_t s, uint64_t e) {
        if (s > e) return;
        auto it = m_.upper_bound(s);
        if (it != m_.begin()) --it;
        while (it != m_.end() && it->first <= e) {
            const uint64_t a = it->first, b = it->second;
            if (b < s) {
                ++it;
                continue;
            }
            it = m_.erase(it);
            if (a < s) m_[a] = s - 1;
            if (b > e) {
                m_[e + 1] = b;
                break;
            }
        }
    }

    // range containing v, if any
    bool get(uint64_t v, uint64_t &s, uint64_t &e) const {
        auto it = m_.upper_bound(v);
        if (it == m_.begin()) return false;
        --it;
        if (it->second < v) return false;
        s = it->first;
        e = it->second;
        return true;
    }

    bool contains(uint64_t v) const {
        uint64_t s, e;
        return get(v, s, e);
    }

    // stored ranges intersecting [s, e], ascending
    std::vector<std::pair<uint64_t, uint64_t>> overlapping(uint64_t s, uint64_t e) const {
        std::vector<std::pair<uint64_t, uint64_t>> out;
        auto it = m_.upper_bound(s);
        if (it != m_.begin()) {
            auto prev = std::prev(it);
            if (prev->second >= s) out.emplace_back(prev->first, prev->second);
        }
        for (; it != m_.end() && it->first <= e; ++it) out.emplace_back(it->first, it->second);
        return out;
    }

    const Map &ranges() const { return m_; }

  private:
    Map m_;
};

}  // namespace corro

struct corro_booked {
    corro::RangeSet needed;
    bool has_max = false;
    uint64_t max = 0;
};

using corro::fail;

extern "C" {

int corro_booked_new(corro_booked **out) {
    if (!out) return fail(CORRO_E_INVALID, "out is NULL");
    *out = new corro_booked();
    return CORRO_OK;
}

void corro_booked_free(corro_booked *b) { delete b; }

int corro_booked_insert_db(corro_booked *b, const uint64_t *start, const uint64_t *end, uint64_t n,
                           uint64_t *rm_start, uint64_t *rm_end, uint64_t rm_cap, uint64_t *n_removed,
                           uint64_t *in_start, uint64_t *in_end, uint64_t in_cap, uint64_t *n_inserted) {
    if (!b || (n && (!start || !end))) return fail(CORRO_E_INVALID, "NULL argument");
    corro::RangeSet versions;
    for (uint64_t i = 0; i < n; i++) versions.insert(start[i], end[i]);

    // compute_gaps_change (agent.rs:1170-1235)
    corro::RangeSet insert_set;
    std::set<std::pair<uint64_t, uint64_t>> remove_ranges;  // HashSet<RangeInclusive>
    bool has_max = b->has_max;
    uint64_t max = b->max;
    auto absorb = [&](uint64_t s, uint64_t e) {
        insert_set.insert(s, e);
        remove_ranges.emplace(s, e);
    };
    for (const auto &r : versions.ranges()) {
        const uint64_t s = r.first, e = r.second;
        if (!has_max || e > max) {
            max = e;
            has_max = true;
        }
        for (const auto &o : b->needed.overlapping(s, e)) absorb(o.first, o.second);
        uint64_t gs, ge;
        if (s > 0 && b->needed.get(s - 1, gs, ge)) absorb(gs, ge);
        if (e < UINT64_MAX && b->needed.get(e + 1, gs, ge)) absorb(gs, ge);
        const uint64_t gap_start = (b->has_max ? b->max : 0) + 1;  // self.max of the snapshot
        if (gap_start < s) {
            insert_set.insert(gap_start, s);
            for (const auto &o : b->needed.overlapping(gap_start, s)) absorb(o.first, o.second);
        }
    }
    for (const auto &r : versions.ranges()) insert_set.remove(r.first, r.second);

    // insert_db (agent.rs:1108-1168): DELETE the removed rows, INSERT the new ones
    uint64_t k = 0;
    for (const auto &r : remove_ranges) {
        if (k < rm_cap && rm_start && rm_end) {
            rm_start[k] = r.first;
            rm_end[k] = r.second;
        }
        k++;
        b->needed.remove(r.first, r.second);
    }
    if (n_removed) *n_removed = k;
    k = 0;
    int rc = CORRO_OK;
    for (const auto &r : insert_set.ranges()) {
        uint64_t s0, e0;
        // __corro_bookkeeping_gaps PK (actor_id, start): an existing row at `start` fails the INSERT
        if (b->needed.get(r.first, s0, e0) && s0 == r.first)
            rc = fail(CORRO_E_INVALID, "UNIQUE constraint failed: __corro_bookkeeping_gaps.start");
        if (k < in_cap && in_start && in_end) {
            in_start[k] = r.first;
            in_end[k] = r.second;
        }
        k++;
        b->needed.insert(r.first, r.second);
    }
    if (n_inserted) *n_inserted = k;
    b->has_max = has_max;
    b->max = max;
    return rc;
}

int corro_booked_needed(corro_booked *b, uint64_t *start, uint64_t *end, uint64_t cap, uint64_t *count) {
    if (!b || !count) return fail(CORRO_E_INVALID, "NULL argument");
    uint64_t k = 0;
    for (const auto &r : b->needed.ranges()) {
        if (k < cap && start && end) {
            start[k] = r.first;
            end[k] = r.second;
        }
        k++;
    }
    *count = k;
    return CORRO_OK;
}

int corro_booked_last(corro_booked *b, int64_t *max) {
    if (!b || !max) return fail(CORRO_E_INVALID, "NULL argument");
    *max = b->has_max ? (int64_t)b->max : -1;
    return CORRO_OK;
}

// BookedVersions::contains_version (agent.rs:1353-1362)
int corro_booked_contains(corro_booked *b, uint64_t version, int *result) {
    if (!b || !result) return fail(CORRO_E_INVALID, "NULL argument");
    *result = !b->needed.contains(version) && (b->has_max ? b->max : 0) >= version;
    return CORRO_OK;
}

// BookedVersions::contains_all without seqs (agent.rs:1384-1390)
int corro_booked_contains_all(corro_booked *b, uint64_t start, uint64_t end, int *result) {
    if (!b || !result) return fail(CORRO_E_INVALID, "NULL argument");
    if (start > end) {
        *result = 1;
        return CORRO_OK;
    }
    const uint64_t m = b->has_max ? b->max : 0;
    *result = end <= m && b->needed.overlapping(start, end).empty();
    return CORRO_OK;
}

}  // extern "C"
