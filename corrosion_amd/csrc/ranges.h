// rangemap 1.5.1 RangeInclusiveSet<u64> semantics (Cargo.lock:3471) for the host-side
// bookkeeping: an ordered map start -> end of disjoint ranges that never touch (touching ranges
// coalesce because CrsqlDbVersion / CrsqlSeq implement StepLite, corro-base-types/src/lib.rs:34-42).
#pragma once
#include <algorithm>
#include <cstdint>
#include <iterator>
#include <map>
#include <utility>
#include <vector>

namespace corro {

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

    // maximal sub-ranges of [s, e] not covered by the set (RangeInclusiveSet::gaps), ascending
    std::vector<std::pair<uint64_t, uint64_t>> gaps(uint64_t s, uint64_t e) const {
        std::vector<std::pair<uint64_t, uint64_t>> out;
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

    bool empty() const { return m_.empty(); }
    size_t size() const { return m_.size(); }

    const Map &ranges() const { return m_; }

  private:
    Map m_;
};


}  // namespace corro
