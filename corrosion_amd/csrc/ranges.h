// rangemap 1.5.1 RangeInclusiveSet<u64> semantics (Cargo.lock:3471) for the host-side
// bookkeeping: disjoint ranges that never touch (touching ranges coalesce because CrsqlDbVersion /
// CrsqlSeq implement StepLite, corro-base-types/src/lib.rs:34-42).
//
// Stored as one sorted vector of (start, end): lookups are binary searches, copies are one
// allocation (a call's per-actor snapshot, VersionsSnapshot, copies the needed set), and the common
// insert -- versions arriving in ascending order -- appends or extends the last range in O(1).
#pragma once
#include <algorithm>
#include <cstdint>
#include <utility>
#include <vector>

namespace corro {

class RangeSet {
  public:
    using R = std::pair<uint64_t, uint64_t>;
    using Vec = std::vector<R>;

    void insert(uint64_t s, uint64_t e) {
        if (s > e) return;
        // fast paths: past the end of the last range, or overlapping / touching only the last one
        if (v_.empty() || (v_.back().second != UINT64_MAX && v_.back().second + 1 < s)) {
            v_.emplace_back(s, e);
            return;
        }
        if (s >= v_.back().first) {
            if (e > v_.back().second) v_.back().second = e;
            return;
        }
        // ranges that overlap or touch [s, e]: end >= s - 1 and start <= e + 1
        const uint64_t lo_key = s == 0 ? 0 : s - 1;
        auto lo = std::lower_bound(v_.begin(), v_.end(), lo_key, [](const R &r, uint64_t k) { return r.second < k; });
        auto hi = e == UINT64_MAX ? v_.end()
                                  : std::upper_bound(lo, v_.end(), e + 1, [](uint64_t k, const R &r) { return k < r.first; });
        if (lo == hi) {
            v_.insert(lo, R{s, e});
            return;
        }
        const uint64_t ns = std::min(s, lo->first), ne = std::max(e, (hi - 1)->second);
        *lo = R{ns, ne};
        v_.erase(lo + 1, hi);
    }

    void remove(uint64_t s, uint64_t e) {
        if (s > e || v_.empty()) return;
        auto lo = std::lower_bound(v_.begin(), v_.end(), s, [](const R &r, uint64_t k) { return r.second < k; });
        auto hi = std::upper_bound(lo, v_.end(), e, [](uint64_t k, const R &r) { return k < r.first; });
        if (lo == hi) return;
        R left{1, 0}, right{1, 0};  // empty unless a remnant survives
        if (lo->first < s) left = R{lo->first, s - 1};
        if ((hi - 1)->second > e) right = R{e + 1, (hi - 1)->second};
        const size_t at = lo - v_.begin();
        v_.erase(lo, hi);
        if (right.first <= right.second) v_.insert(v_.begin() + at, right);
        if (left.first <= left.second) v_.insert(v_.begin() + at, left);
    }

    // range containing v, if any
    bool get(uint64_t v, uint64_t &s, uint64_t &e) const {
        auto it = std::upper_bound(v_.begin(), v_.end(), v, [](uint64_t k, const R &r) { return k < r.first; });
        if (it == v_.begin()) return false;
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
    Vec overlapping(uint64_t s, uint64_t e) const {
        Vec out;
        if (s > e) return out;
        auto it = std::lower_bound(v_.begin(), v_.end(), s, [](const R &r, uint64_t k) { return r.second < k; });
        for (; it != v_.end() && it->first <= e; ++it) out.push_back(*it);
        return out;
    }

    bool any_overlap(uint64_t s, uint64_t e) const {
        if (s > e) return false;
        auto it = std::lower_bound(v_.begin(), v_.end(), s, [](const R &r, uint64_t k) { return r.second < k; });
        return it != v_.end() && it->first <= e;
    }

    // maximal sub-ranges of [s, e] not covered by the set (RangeInclusiveSet::gaps), ascending
    Vec gaps(uint64_t s, uint64_t e) const {
        Vec out;
        if (s > e) return out;
        uint64_t x = s;
        for (const auto &r : overlapping(s, e)) {
            if (r.first > x) out.emplace_back(x, r.first - 1);
            if (r.second >= e) return out;
            x = r.second + 1;
        }
        out.emplace_back(x, e);
        return out;
    }

    bool contains_range(uint64_t s, uint64_t e) const {
        uint64_t a, b;
        return s <= e && get(s, a, b) && b >= e;
    }

    bool empty() const { return v_.empty(); }
    size_t size() const { return v_.size(); }
    const R &last() const { return v_.back(); }

    const Vec &ranges() const { return v_; }

  private:
    Vec v_;
};

}  // namespace corro
