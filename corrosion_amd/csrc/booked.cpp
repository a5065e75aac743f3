// C ABI over BookedVersions (booked.h): the gap bookkeeping of
// /root/reference/crates/corro-types/src/agent.rs:1108-1235 and :1353-1392.
#include <cstdint>
#include <string>
#include <vector>

#include "booked.h"
#include "corro_hip.h"

namespace corro {
int fail(int code, const std::string &msg);
}

struct corro_booked {
    corro::Booked b;
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
    std::vector<corro::Range> removed, inserted;
    const bool ok = b->b.insert_db(versions, &removed, &inserted);
    for (size_t k = 0; k < removed.size() && k < rm_cap && rm_start && rm_end; k++) {
        rm_start[k] = removed[k].first;
        rm_end[k] = removed[k].second;
    }
    for (size_t k = 0; k < inserted.size() && k < in_cap && in_start && in_end; k++) {
        in_start[k] = inserted[k].first;
        in_end[k] = inserted[k].second;
    }
    if (n_removed) *n_removed = removed.size();
    if (n_inserted) *n_inserted = inserted.size();
    if (!ok) return fail(CORRO_E_INVALID, "UNIQUE constraint failed: __corro_bookkeeping_gaps.start");
    return CORRO_OK;
}

int corro_booked_needed(corro_booked *b, uint64_t *start, uint64_t *end, uint64_t cap, uint64_t *count) {
    if (!b || !count) return fail(CORRO_E_INVALID, "NULL argument");
    uint64_t k = 0;
    for (const auto &r : b->b.needed.ranges()) {
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
    *max = b->b.has_max ? (int64_t)b->b.max : -1;
    return CORRO_OK;
}

int corro_booked_contains(corro_booked *b, uint64_t version, int *result) {
    if (!b || !result) return fail(CORRO_E_INVALID, "NULL argument");
    *result = b->b.contains_version(version);
    return CORRO_OK;
}

int corro_booked_contains_all(corro_booked *b, uint64_t start, uint64_t end, int *result) {
    if (!b || !result) return fail(CORRO_E_INVALID, "NULL argument");
    *result = b->b.contains_all(start, end, nullptr);
    return CORRO_OK;
}

}  // extern "C"
