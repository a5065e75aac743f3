// Device half of corro_process_multiple_changes (agent.cpp), in plain C++ types: agent.cpp is host
// C++ and never sees HIP. Implemented in agent_dev.hip.
//
// The call keeps the caller's change batch where it is (device memory, or staged once from host
// memory) and does its per-change work on the GPU: the bad-cid screen of every changeset (util.rs
// :839-860), the applied batch (zero-copy when the applied changesets are one contiguous run of the
// input, else one gather kernel), and the impactful-change flags with the transaction-cumulative
// crsql_rows_impacted() rule (util.rs:1218-1261). The host only walks changeset headers.
#pragma once
#include <cstdint>
#include <vector>

#include "corro_hip.h"

namespace corro {

// A run of input changes that goes into the applied batch: input [src, src + count) -> batch
// [dst, dst + count); ts = the changeset timestamp (bound per change when the input has no ts).
struct AgentSpan {
    uint64_t src, dst, count, ts;
};

// Pinned host arrays of one call (agent_dev_begin; valid until the next begin on the context), per
// changeset in arrival order. The host fills them in sequential parallel passes and each crosses to
// the device with one copy:
//   off / cnt  its change span (cnt 0 = not screened: not a non-empty Full)
//   ts / site  its timestamp and actor (site ordinal)
//   flag       1 = merged by this call (a complete version that passed every check)
//   bad        filled by agent_dev_bad; any: filled by agent_dev_impacts (flag set only)
struct AgentPinned {
    uint64_t *off, *cnt, *ts;
    uint32_t *site;
    uint8_t *flag, *bad, *any;
    uint64_t *committed;  // per table
};
int agent_dev_begin(corro_ctx *ctx, uint64_t ncs, uint64_t nchanges, AgentPinned *p);

// Device view of the input: `in` itself for CORRO_MEM_DEVICE, else every field copied to device
// scratch (val_data too). The view stays valid until the call ends.
int agent_dev_input(corro_ctx *ctx, const corro_changes *in, int mem, corro_changes *dv);

// p.bad[j] = 1 when changes [off[j], off[j] + cnt[j]) hold a table_cid of CORRO_TCID_UNKNOWN.
int agent_dev_bad(corro_ctx *ctx, const corro_changes *dv, const AgentPinned &p, uint64_t ncs);

// Host copies of the input changes of `spans` (dst ignored), concatenated: field arrays of
// sum(count) elements + the bytes of their long values (lv_off/lv_len index lv_data; len 0 = none).
// (Incomplete versions only: pageable copies, its own device scratch.)
struct HostSpanRows {
    std::vector<uint64_t> pk, v0, v1, ts;
    std::vector<int64_t> cv, dbv;
    std::vector<uint32_t> tcid, cl, seq, site;
    std::vector<uint8_t> vt, vl;
    std::vector<uint64_t> lv_off, lv_len;
    std::vector<uint8_t> lv_data;
};
int agent_dev_fetch(corro_ctx *ctx, const corro_changes *dv, const std::vector<AgentSpan> &spans, HostSpanRows &out);

// The applied batch (device SoA, application order) of the nspans flagged changesets: their order
// (actors by ActorId bytes = site rank, arrival order within an actor) from a stable device radix
// sort, their batch offsets from a device scan. Zero-copy (pointers into dv) when the spans are one
// contiguous, suitably aligned run of the input and every needed field is there; else a gather into
// device scratch that also fills ts from the changesets when the input has none and some changeset
// carries one. *gathered says which. The span tables stay on the device for agent_dev_impacts.
// Position mode (pm non-null, taken when the input is one apply chunk with the apply's alignment):
// no gather; *batch = the input itself and pm the application position of every input change
// (ap, AP_SKIP = not applied), the input index of every position (src) and the per-position ts.
struct AgentPositions {
    bool on;
    const uint32_t *ap, *src;
    const uint64_t *ts;
    uint64_t n;
};
int agent_dev_batch(corro_ctx *ctx, const corro_changes *dv, const AgentPinned &p, uint64_t ncs, uint64_t nspans,
                    uint64_t nbatch, bool need_ts, corro_changes *batch, bool *gathered, AgentPositions *pm);
// the next corro_apply_batch on ctx runs in position mode (null: back to normal)
void agent_dev_set_positions(corro_ctx *ctx, const AgentPositions *pm);

// Device impact buffer for a batch of n changes (valid until the next call).
uint8_t *agent_dev_impact_buf(corro_ctx *ctx, uint64_t n, int *rc);

// From the batch's per-change impact growth: impactful[span.src + k] (0/1 over all nin input
// changes, in `mem` memory; NULL = not wanted), p.any[i] = flagged changeset i had an impactful change,
// p.committed[t] = impactful changes of table t (tcid = the batch's table_cid array, device, by batch
// position -- or by input index with tcid_by_src). Rule
// (util.rs:1218-1261): a version's first change is impactful when the transaction's cumulative
// counter is > 0 after it (any impact at or before it in the batch); its later changes when their
// own growth is > 0.
int agent_dev_impacts(corro_ctx *ctx, const uint8_t *impact, const uint32_t *tcid, bool tcid_by_src, uint64_t nbatch,
                      const AgentPinned &p, uint64_t ncs, uint64_t nspans, uint8_t *impactful, uint64_t nin, int mem,
                      uint32_t ntables);

// ---- device-resident headers (CORRO_MEM_DEVICE_HEADERS) -----------------------------------------
// The changeset headers, out->known and out->impactful live on the device. One pass per changeset
// (span check, unknown-name screen, columns), one stable sort by site rank (the application order
// and the per-actor grouping at once), a second by (site rank, version start) that decides every
// changeset nothing else of its actor in the call overlaps and whose versions are all above the
// actor's booked max (a complete Full version: merged / rolled back; an empty one or an Empty range:
// cleared; later copies of its dedup key: skipped), and the decided versions' runs for the gap
// bookkeeping. The host gets per-site summaries, the runs, and the headers of the other ("host")
// changesets, which it walks with the reference's per-actor passes.
constexpr uint32_t HDR_TAB_MIXED = 0xFFFFFFFFu;  // (DevHdrResult::hctab) tables differ, or not canonical
struct DevHdrSite {
    uint32_t gstart, gend;   // sorted slots [gstart, gend] of the site's changesets (gstart ~0: none)
};
struct DevHdrResult {
    uint32_t err;            // bit 0 span outside the batch, bit 1 site ordinal not registered
    bool ts_any;             // some changeset has a non-zero ts
    uint64_t nspans, nchanges;   // changesets merged by a device decision and their changes
    std::vector<DevHdrSite> sites;             // per site ordinal
    std::vector<uint32_t> run_site;            // decided version runs, grouped by site, ascending
    std::vector<uint64_t> run_start, run_end;
    // the host's changesets in sorted order (grouped by actor, arrival order inside): header, arrival
    // index, unknown-name flag, canonical partial (bufpool.hip); pinned, valid until the next call
    uint64_t nh;
    const corro_changeset *hcs;
    const uint32_t *hidx;
    const uint8_t *hbad, *hcanon;
    const uint32_t *hctab;  // per host changeset: its table index when canonical and single-table, else HDR_TAB_MIXED
};
// site_max[s] = the actor's booked max (-1: none); dknown: device, ncs entries
int agent_dev_headers(corro_ctx *ctx, const corro_changeset *dcs, uint64_t ncs, const corro_changes *dv,
                      const std::vector<int64_t> &site_max, int32_t *dknown, DevHdrResult &res);
// the host's decisions for its changesets: flag[idx[k]] = flag[k], known[idx[k]] = known[k]
int agent_dev_put_host(corro_ctx *ctx, const uint32_t *idx, uint64_t n, const std::vector<uint8_t> &flag,
                       const std::vector<int32_t> &known, int32_t *dknown);
// the applied batch in sorted order (flagged changesets only), like agent_dev_batch
int agent_dev_batch_sorted(corro_ctx *ctx, const corro_changes *dv, uint64_t ncs, uint64_t nspans, uint64_t nbatch,
                           bool need_ts, corro_changes *batch, bool *gathered, AgentPositions *pm);
// after a successful merge: known of flagged changesets (Current / Cleared by p.any on the device),
// crsql_set_db_version of the device-decided empty versions; with `keys` (sorted site << 40 | version
// keys holding buffered meta) *hits = the (site, version) of every flagged changeset among them (a
// device binary search per changeset, for check_buffered_meta_to_clear)
int agent_dev_commit_headers(corro_ctx *ctx, uint64_t ncs, int32_t *dknown, const std::vector<uint64_t> *keys,
                             std::vector<std::pair<uint32_t, uint64_t>> *hits);

// Host headers staged for the device header passes (CORRO_MEM_DEVICE with host headers, large
// calls): a pinned area the host fills in parallel chunks, each chunk uploaded as soon as it is
// copied, and the device outcome array copied back at the end.
struct HdrStage {
    corro_changeset *pinned, *dev;
    int32_t *dknown;
};
int agent_dev_stage_begin(corro_ctx *ctx, uint64_t ncs, HdrStage *st);
// async upload of headers [lo, hi) (callable from pool threads)
int agent_dev_stage_upload(corro_ctx *ctx, const HdrStage &st, uint64_t lo, uint64_t hi);
int agent_dev_stage_known(corro_ctx *ctx, const HdrStage &st, int32_t *known, uint64_t ncs);

// ---- device-resident buffered rows (bufpool.hip) ------------------------------------------------
// A bookie's pool of __corro_buffered_changes rows in HBM (columns of corro_changes without long
// values), on the device of the first context that writes it.
struct DevBufPool;
DevBufPool *bufpool_new();
void bufpool_free(DevBufPool *p);
bool bufpool_usable(corro_ctx *ctx, const DevBufPool *p);
uint64_t bufpool_top(const DevBufPool *p);
// per-table counts of the changes of the spans (src, count)
int agent_dev_table_counts(corro_ctx *ctx, const corro_changes *dv, const std::vector<AgentSpan> &spans,
                           uint32_t ntables, std::vector<uint64_t> &counts);
// room for `need` more rows at the top: grows, or compacts the live segments (*offs[k], lens[k]),
// rewriting their offsets, when at least half of the rows below the top are dead
int bufpool_reserve(corro_ctx *ctx, DevBufPool *p, uint64_t need, std::vector<uint64_t *> &offs,
                    const std::vector<uint64_t> &lens);
// input changes [src, src + count) -> pool rows at the top (dst set per job); ts = the changeset's
// when the input has no ts
struct PoolCopy {
    uint64_t src, count, ts, dst;
};
int bufpool_append(corro_ctx *ctx, DevBufPool *p, const corro_changes *dv, std::vector<PoolCopy> &jobs);
// pool rows [off, off + n) to the host (no long values)
int bufpool_read(const DevBufPool *p, uint64_t off, uint64_t n, HostSpanRows &out);

// Batched gap bookkeeping (corro_booked_insert_db_batch, gaps.hip) for a call with many actors:
// host CSR in (per actor: booked max or -1, needed gaps, this call's versions), host arrays out
// (per actor: new max, DELETE rows, INSERT rows, new gaps, status).
struct GapsHost {
    std::vector<int64_t> max;
    std::vector<uint64_t> gap_off, gap_start, gap_end, ver_off, ver_start, ver_end;
};
struct GapsHostOut {
    std::vector<int64_t> max;
    std::vector<uint64_t> rm_count, ins_count, gap_count, rm_start, rm_end, ins_start, ins_end, new_start, new_end;
    std::vector<int32_t> status;
};
int agent_dev_gaps(corro_ctx *ctx, const GapsHost &in, GapsHostOut &out);

// every known entry back to Skipped (a failed call)
int agent_dev_clear_known(corro_ctx *ctx, int32_t *dknown, uint64_t ncs);

// The registered 16-byte id of a site ordinal (false: not registered).
bool agent_site_id(corro_ctx *ctx, uint32_t site, uint8_t out[16]);
uint32_t agent_site_count(corro_ctx *ctx);
uint32_t agent_table_count(corro_ctx *ctx);

}  // namespace corro
