// BookedVersions (/root/reference/crates/corro-types/src/agent.rs:1260-1458): per-actor known
// versions = max, needed gaps, partially received versions. Host-side, shared by booked.cpp (C ABI
// for the bare bookkeeping) and agent.cpp (process_multiple_changes).
#pragma once
#include <cstdint>
#include <map>
#include <set>
#include <utility>
#include <vector>

#include "ranges.h"

namespace corro {

using Range = std::pair<uint64_t, uint64_t>;

// PartialVersion (agent.rs:1057-1075)
struct PartialVersion {
    RangeSet seqs;
    uint64_t last_seq = 0;
    uint64_t ts = 0;
    // quirk kept from the reference: completeness is checked over 1..=last_seq, not 0..=last_seq
    bool is_complete() const { return !seqs.has_gap(1, last_seq); }
};

struct Booked {
    RangeSet needed;
    bool has_max = false;
    uint64_t max = 0;
    std::map<uint64_t, PartialVersion> partials;

    uint64_t max_or_zero() const { return has_max ? max : 0; }

    // contains_version (agent.rs:1353-1362)
    bool contains_version(uint64_t v) const { return !needed.contains(v) && max_or_zero() >= v; }

    // contains_all (agent.rs:1368-1390), without iterating every version of a large range
    bool contains_all(uint64_t s, uint64_t e, const Range *seqs) const {
        if (s > e) return true;
        if (e > max_or_zero()) return false;
        if (needed.any_overlap(s, e)) return false;
        if (!seqs || seqs->first > seqs->second) return true;
        for (auto it = partials.lower_bound(s); it != partials.end() && it->first <= e; ++it)
            if (!it->second.seqs.contains_range(seqs->first, seqs->second)) return false;
        return true;
    }

    // VersionsSnapshot::compute_gaps_change + insert_db (agent.rs:1108-1235). Fills the gap rows
    // the reference DELETEs / INSERTs in __corro_bookkeeping_gaps. Returns false when an INSERT
    // would hit an existing (actor_id, start) row.
    bool insert_db(const RangeSet &versions, std::vector<Range> *removed, std::vector<Range> *inserted) {
        RangeSet insert_set;
        std::set<Range> remove_ranges;  // HashSet<RangeInclusive>
        bool nhas = has_max;
        uint64_t nmax = max;
        auto absorb = [&](uint64_t a, uint64_t b) {
            insert_set.insert(a, b);
            remove_ranges.emplace(a, b);
        };
        for (const auto &r : versions.ranges()) {
            const uint64_t s = r.first, e = r.second;
            if (!nhas || e > nmax) {
                nmax = e;
                nhas = true;
            }
            for (const auto &o : needed.overlapping(s, e)) absorb(o.first, o.second);
            uint64_t gs, ge;
            if (s > 0 && needed.get(s - 1, gs, ge)) absorb(gs, ge);
            if (e < UINT64_MAX && needed.get(e + 1, gs, ge)) absorb(gs, ge);
            const uint64_t gap_start = max_or_zero() + 1;  // self.max of the snapshot, not the running max
            if (gap_start < s) {
                insert_set.insert(gap_start, s);
                for (const auto &o : needed.overlapping(gap_start, s)) absorb(o.first, o.second);
            }
        }
        for (const auto &r : versions.ranges()) insert_set.remove(r.first, r.second);
        for (const auto &r : remove_ranges) {
            if (removed) removed->push_back(r);
            partials.erase(partials.lower_bound(r.first), partials.upper_bound(r.second));
            needed.remove(r.first, r.second);
        }
        bool ok = true;
        for (const auto &r : insert_set.ranges()) {
            uint64_t a, b;
            if (needed.get(r.first, a, b) && a == r.first) ok = false;
            if (inserted) inserted->push_back(r);
            needed.insert(r.first, r.second);
        }
        has_max = nhas;
        max = nmax;
        return ok;
    }

    // insert_partial (agent.rs:1414-1432)
    // (by value: a caller done with its PartialVersion moves it in, no copy of its ranges)
    const PartialVersion &insert_partial(uint64_t version, PartialVersion p) {
        auto it = partials.find(version);
        if (it == partials.end()) {
            if (!has_max || version > max) {
                max = version;
                has_max = true;
            }
            return partials.emplace_hint(it, version, std::move(p))->second;
        }
        for (const auto &r : p.seqs.ranges()) it->second.seqs.insert(r.first, r.second);
        return it->second;
    }
};

}  // namespace corro
