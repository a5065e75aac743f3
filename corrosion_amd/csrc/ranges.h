// rangemap 1.5.1 RangeInclusiveSet<u64> semantics (Cargo.lock:3471) for the host-side
// bookkeeping: disjoint ranges that never touch (touching ranges coalesce because CrsqlDbVersion /
// CrsqlSeq implement StepLite, corro-base-types/src/lib.rs:34-42).
//
// Stored as one sorted vector of (start, end): lookups are binary searches, copies are one
// allocation (a call's per-actor snapshot, VersionsSnapshot, copies the needed set), and the common
// insert -- versions arriving in ascending order -- appends or extends the last range in O(1).
// The vector keeps up to two ranges inline: a partial version's seq set or a seq book is one or two
// ranges, and a mixed gossip call builds hundreds of thousands of them (a heap allocation each was
// most of the host walk's time).
#pragma once
#include <algorithm>
#include <cstdint>
#include <utility>
#include <vector>

namespace corro {

// a vector of small copyable T with N elements inline (the subset of std::vector the range code uses)
template <class T, unsigned N>
class SmallVec {
  public:
    SmallVec() = default;
    SmallVec(const SmallVec &o) { assign(o.begin(), o.end()); }
    SmallVec(SmallVec &&o) noexcept { take(o); }
    ~SmallVec() { release(); }
    SmallVec &operator=(const SmallVec &o) {
        if (this != &o) {
            n_ = 0;
            assign(o.begin(), o.end());
        }
        return *this;
    }
    SmallVec &operator=(SmallVec &&o) noexcept {
        if (this != &o) {
            release();
            take(o);
        }
        return *this;
    }
    T *begin() { return p_; }
    T *end() { return p_ + n_; }
    const T *begin() const { return p_; }
    const T *end() const { return p_ + n_; }
    T *data() { return p_; }
    const T *data() const { return p_; }
    size_t size() const { return n_; }
    bool empty() const { return n_ == 0; }
    T &back() { return p_[n_ - 1]; }
    const T &back() const { return p_[n_ - 1]; }
    T &operator[](size_t i) { return p_[i]; }
    const T &operator[](size_t i) const { return p_[i]; }
    void clear() { n_ = 0; }
    void reserve(size_t c) {
        if (c > cap_) grow(c);
    }
    void push_back(const T &x) {
        if (n_ == cap_) grow(cap_ * 2);
        p_[n_++] = x;
    }
    template <class... A>
    void emplace_back(A &&...a) {
        push_back(T{std::forward<A>(a)...});
    }
    T *insert(T *at, const T &x) {
        const size_t k = at - p_;
        if (n_ == cap_) grow(cap_ * 2);
        std::copy_backward(p_ + k, p_ + n_, p_ + n_ + 1);
        p_[k] = x;
        n_++;
        return p_ + k;
    }
    T *erase(T *a, T *b) {
        std::copy(b, end(), a);
        n_ -= b - a;
        return a;
    }

  private:
    void assign(const T *a, const T *b) {
        reserve(b - a);
        std::copy(a, b, p_);
        n_ = b - a;
    }
    void grow(size_t c) {
        T *q = new T[c];
        std::copy(p_, p_ + n_, q);
        const size_t n = n_;
        release();
        n_ = n;
        p_ = q;
        cap_ = c;
    }
    void release() {
        if (p_ != in_) delete[] p_;
        p_ = in_;
        cap_ = N;
    }
    void take(SmallVec &o) {
        if (o.p_ == o.in_) {
            std::copy(o.in_, o.in_ + o.n_, in_);
            p_ = in_;
            cap_ = N;
        } else {
            p_ = o.p_;
            cap_ = o.cap_;
            o.p_ = o.in_;
            o.cap_ = N;
        }
        n_ = o.n_;
        o.n_ = 0;
    }
    T in_[N];
    T *p_ = in_;
    size_t n_ = 0, cap_ = N;
};

class RangeSet {
  public:
    using R = std::pair<uint64_t, uint64_t>;
    using Vec = SmallVec<R, 2>;

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

    // gaps(s, e) non-empty, without building them
    bool has_gap(uint64_t s, uint64_t e) const {
        if (s > e) return false;
        uint64_t a, b;
        return !(get(s, a, b) && b >= e);  // (touching ranges coalesce: [s, e] covered = one range holds it)
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
