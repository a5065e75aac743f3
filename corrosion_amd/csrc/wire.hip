// Wire decode: length-delimited frames of speedy-encoded changesets ->
// the SoA batch + changeset headers that corro_process_multiple_changes / corro_apply_batch take.
//
// Reference: frames are tokio LengthDelimitedCodec (u32 big-endian length + payload,
// corro-agent/src/api/peer/mod.rs:917-929, corro-types/src/sync.rs:366-376); payloads are
// SyncMessage::V1(SyncMessageV1::Changeset(ChangeV1)) (sync.rs:19-30) or
// UniPayload::V1 { Broadcast(BroadcastV1::Change(ChangeV1)), cluster_id } (broadcast.rs:41-52,
// 93-96), read with speedy's derived layout (u32 enum tags, u32 length prefixes, little endian;
// corrosion_amd/wire.py restates it); ChangeV1 / Changeset / Change: broadcast.rs:114-148,
// change.rs:19-30; SqliteValue's own encoding: corro-api-types/src/lib.rs:615-680; packed pks:
// unpack_columns (corro-types/src/pubsub.rs:2396-2451).
//
// Kernels:
//   k_wire_hdr     one lane per frame: message tags, actor, changeset variant and its fixed
//                  header (Full: version + change count; Empty: versions + optional ts; EmptySet:
//                  ranges + ts)
//   k_wire_decode  one 64-lane workgroup per Full frame: the frame is staged into LDS with
//                  coalesced loads, lane 0 walks the variable-length changes once to record each
//                  change's offset (and reads the trailing seqs / last_seq / ts), then all lanes
//                  decode changes in parallel: table / column names matched against the schema,
//                  pk unpacked, value to the engine's fixed-width encoding, site id to its ordinal
//                  through a device hash of the registered sites. A TEXT/BLOB longer than 16 bytes
//                  stays in the frame bytes: the change names it by val_off / val_size (offsets in
//                  the frame buffer, which becomes the batch's val_data). The pk of an interned table
//                  (corro_table_set_pk_interned: BLOB / TEXT / composite pks) is left as a reference
//                  to its packed bytes, which the host interns (corro_pk_keys) after the kernel.
// Unknown site ids are collected; the host registers them (corro_site_register) and re-runs the
// decode, so ordinals match the engine's site table. Unknown table / column names give
// table_cid = CORRO_TCID_UNKNOWN (the host rolls that version back, as the failing INSERT's
// SAVEPOINT does, util.rs:839-860).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "internal.h"

namespace corro {
namespace {

#ifndef CORRO_DIAG
#define CORRO_DIAG 0
#endif
#if CORRO_DIAG & 512  // phase times of a few k_wire_decode workgroups (tools/diag_wire.py)
#define WDIAG(i) const uint64_t t##i = wall_clock64();
#else
#define WDIAG(i)
#endif

constexpr uint32_t WIRE_LDS = 16384;      // at most this many frame bytes staged per workgroup
constexpr uint32_t WIRE_OFFS = 1024;      // at most this many change offsets kept in LDS
constexpr int32_t ST_NOT_CHANGESET = 1;   // a frame that is not a changeset message (skipped)

__device__ inline uint64_t wmix(uint64_t x) {
    x ^= x >> 33; x *= 0xff51afd7ed558ccdULL;
    x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ULL;
    x ^= x >> 33; return x;
}

struct WireDev {
    const uint8_t *buf;
    const uint64_t *foff;     // frame payload offsets
    const uint32_t *flen;     // frame payload lengths
    uint32_t nframes, kind;   // kind: 0 sync message, 1 uni payload
    // per frame header (out)
    int32_t *status;
    uint32_t *cs_kind, *nchg, *nset, *chg_start, *site;
    uint64_t *v0, *v1, *s0, *s1, *last, *ts;
    uint8_t *actor;           // 16 per frame
    const uint64_t *chg_off, *set_off;   // pass 1 inputs
    uint64_t *set_start, *set_end;
    // schema
    const uint8_t *names;
    const uint32_t *tname_off, *tname_len, *tcol_base, *tncols, *cname_off, *cname_len;
    uint32_t ntables;
    // sites
    const uint64_t *hlo, *hhi;
    const uint32_t *hord;
    uint32_t hmask;
    uint8_t *unknown;         // 16 per unknown site slot
    unsigned long long *nunknown;
    uint32_t unknown_cap;
    // outputs (SoA)
    corro_changes out;
    uint32_t *chg_rel;        // scratch: per change offset within its frame (frames with > WIRE_OFFS changes)
    const uint8_t *interned;  // per table: 1 = rows keyed by interned pk bytes
    uint64_t *pkref;          // per change: 0, or (buffer offset << 32 | length) of an interned pk
    unsigned long long *nref, *nlong;  // interned pk references, long values
    uint32_t lds_len, off_cap;         // k_wire_decode's dynamic LDS: frame bytes, change offsets
};

// little-endian / big-endian readers over any byte pointer, bounds-checked against end
struct Rd {
    const uint8_t *p;
    uint32_t pos, end;
    bool bad;
    __device__ inline bool need(uint32_t n) {
        if (pos + n > end || pos + n < pos) bad = true;
        return !bad;
    }
    __device__ inline uint64_t le(uint32_t n) {
        if (!need(n)) return 0;
        uint64_t v = 0;
        for (uint32_t i = 0; i < n; i++) v |= (uint64_t)p[pos + i] << (8 * i);
        pos += n;
        return v;
    }
    __device__ inline uint32_t u32() { return (uint32_t)le(4); }
    __device__ inline uint64_t u64() { return le(8); }
};

__device__ inline uint32_t site_lookup(const WireDev &d, uint64_t lo, uint64_t hi) {
    if (d.hmask == 0) return 0xFFFFFFFFu;
    uint32_t h = (uint32_t)wmix(lo ^ (hi * 0x9E3779B97F4A7C15ULL)) & d.hmask;
    while (true) {
        const uint32_t o = d.hord[h];
        if (o == 0xFFFFFFFFu) return o;
        if (d.hlo[h] == lo && d.hhi[h] == hi) return o;
        h = (h + 1) & d.hmask;
    }
}

__device__ inline void note_unknown(const WireDev &d, uint64_t lo, uint64_t hi) {
    const unsigned long long k = atomicAdd(d.nunknown, 1ULL);
    if (k < d.unknown_cap) {
        uint64_t *u = reinterpret_cast<uint64_t *>(d.unknown + 16 * k);
        u[0] = lo;
        u[1] = hi;
    }
}

__global__ void k_wire_hdr(WireDev d) {
    const uint32_t f = blockIdx.x * blockDim.x + threadIdx.x;
    if (f >= d.nframes) return;
    Rd r{d.buf + d.foff[f], 0, d.flen[f], false};
    int32_t st = 0;
    uint32_t kind = 0, nchg = 0, nset = 0, cstart = 0;
    uint64_t v0 = 0, v1 = 0, ts = 0;
    if (d.kind == 0) {
        if (r.u32() != 0 || r.u32() != 1) st = ST_NOT_CHANGESET;   // SyncMessage::V1, ::Changeset
    } else {
        if (r.u32() != 0 || r.u32() != 0 || r.u32() != 0) st = ST_NOT_CHANGESET;  // UniPayload::V1/Broadcast/Change
    }
    uint64_t alo = 0, ahi = 0;
    if (!st) {
        alo = r.u64();
        ahi = r.u64();
        kind = r.u32();
        if (kind == 0) {            // Empty { versions, ts: Option<Timestamp> (default_on_eof) }
            v0 = r.u64();
            v1 = r.u64();
            if (!r.bad && r.pos < r.end) {
                const uint32_t some = (uint32_t)r.le(1);
                if (some == 1) ts = r.u64();
                else if (some != 0) st = CORRO_E_INVALID;
            }
        } else if (kind == 1) {     // Full { version, changes, ... } (the rest follows the changes)
            v0 = v1 = r.u64();
            nchg = r.u32();
            cstart = r.pos;
            // the count is untrusted: the smallest encoded change is 61 bytes (three u32 length
            // prefixes, a value tag and 48 bytes of fixed fields), so a count the frame cannot hold
            // is malformed (and must not size the caller's allocations)
            if (!r.bad && (uint64_t)nchg * 61 > (uint64_t)(r.end - r.pos)) st = CORRO_E_INVALID;
        } else if (kind == 2) {     // EmptySet { versions: Vec<RangeInclusive>, ts }
            nset = r.u32();
            const uint64_t body = (uint64_t)nset * 16;
            if (!r.need(body > 0xFFFFFFFFULL ? 0xFFFFFFFFu : (uint32_t)body)) nset = 0;
            else r.pos += (uint32_t)body;
            ts = r.u64();
        } else {
            st = CORRO_E_INVALID;
        }
        if (r.bad) st = CORRO_E_INVALID;
    }
    d.status[f] = st;
    d.cs_kind[f] = kind;
    d.nchg[f] = st ? 0 : nchg;
    d.nset[f] = st ? 0 : nset;
    d.chg_start[f] = cstart;
    d.v0[f] = v0;
    d.v1[f] = v1;
    d.ts[f] = ts;
    d.s0[f] = d.s1[f] = d.last[f] = 0;
    uint64_t *a = reinterpret_cast<uint64_t *>(d.actor + 16 * (uint64_t)f);
    a[0] = alo;
    a[1] = ahi;
    uint32_t so = 0xFFFFFFFFu;
    if (!st) {
        so = site_lookup(d, alo, ahi);
        if (so == 0xFFFFFFFFu) note_unknown(d, alo, ahi);
    }
    d.site[f] = so;
}

// EmptySet ranges (pass 1)
__global__ void k_wire_sets(WireDev d) {
    const uint32_t f = blockIdx.x * blockDim.x + threadIdx.x;
    if (f >= d.nframes || d.status[f] || d.cs_kind[f] != 2) return;
    Rd r{d.buf + d.foff[f], 0, d.flen[f], false};
    r.pos = (d.kind == 0 ? 8 : 12) + 16 + 4 + 4;
    const uint64_t o = d.set_off[f];
    for (uint32_t k = 0; k < d.nset[f]; k++) {
        d.set_start[o + k] = r.u64();
        d.set_end[o + k] = r.u64();
    }
}

__device__ inline bool name_eq(const uint8_t *a, uint32_t alen, const uint8_t *b, uint32_t blen) {
    if (alen != blen) return false;
    for (uint32_t i = 0; i < alen; i++)
        if (a[i] != b[i]) return false;
    return true;
}

// The walk over a frame's variable-length changes, done by the whole wave with wave-uniform
// (scalar) state: lane i of the window holds the little-endian u32 at base + i, so each length
// prefix is ONE readlane and a change costs one window load (4 LDS byte reads per lane, VALU) plus
// ~40 scalar instructions. The scalar unit is shared by every wave of a CU, and a byte-at-a-time
// walk (~300 scalar instructions per change) saturated it: 90 us per 128-change frame.
struct WaveWin {
    const uint8_t *p;
    uint32_t len, base, word;
    bool padded;  // p has >= 68 readable bytes past len (the LDS copy): no per-byte bounds checks
    __device__ inline void load(uint32_t at) {
        base = at;
        const uint32_t i = at + threadIdx.x;
        uint32_t v = 0;
        if (padded) {
            v = (uint32_t)p[i] | (uint32_t)p[i + 1] << 8 | (uint32_t)p[i + 2] << 16 | (uint32_t)p[i + 3] << 24;
        } else {
#pragma unroll
            for (uint32_t b = 0; b < 4; b++) v |= (i + b < len ? (uint32_t)p[i + b] : 0u) << (8 * b);
        }
        word = v;
    }
    // the u32 at `at`; the caller has checked at + 4 <= len
    __device__ inline uint32_t u32(uint32_t at) {
        if (at - base > 63u) load(at);
        return (uint32_t)__builtin_amdgcn_readlane((int)word, (int)(at - base));
    }
};

__global__ void __launch_bounds__(64) k_wire_decode(WireDev d) {
    // dynamic LDS: change offsets (off_cap words), then the staged frame (lds_len bytes)
    extern __shared__ uint32_t s_dyn[];
    __shared__ uint64_t s_tail;
    __shared__ int32_t s_bad;
    uint32_t *s_off = s_dyn;
    uint8_t *s_buf = reinterpret_cast<uint8_t *>(s_dyn + d.off_cap);
    const uint32_t f = blockIdx.x;
    if (d.status[f] || d.cs_kind[f] != 1) return;   // uniform per workgroup
    WDIAG(0)
    const uint32_t len = d.flen[f], n = d.nchg[f];
    const uint8_t *g = d.buf + d.foff[f];
    const bool lds = len <= d.lds_len;
    if (lds) {
        // coalesced staging: 8-byte words where aligned, bytes at the ragged ends
        const uintptr_t base = reinterpret_cast<uintptr_t>(g);
        const uint32_t head = (uint32_t)std::min<uintptr_t>((8 - (base & 7)) & 7, len);
        for (uint32_t i = threadIdx.x; i < head; i += 64) s_buf[i] = g[i];
        const uint32_t nw = (len - head) / 8;
        const uint64_t *gw = reinterpret_cast<const uint64_t *>(g + head);
        for (uint32_t w = threadIdx.x; w < nw; w += 64) {
            const uint64_t x = gw[w];
            for (int b = 0; b < 8; b++) s_buf[head + 8 * w + b] = (uint8_t)(x >> (8 * b));
        }
        for (uint32_t i = head + 8 * nw + threadIdx.x; i < len; i += 64) s_buf[i] = g[i];
    }
    __syncthreads();
    WDIAG(1)
    // the rest runs on a pointer of known address space (LDS or global): through a generic pointer
    // every byte read is a flat load, several hundred cycles each on the walk's dependent chain
    auto body = [&](const uint8_t *p, const bool padded) __attribute__((always_inline)) {
    const bool off_lds = n <= d.off_cap;
    const uint64_t co = d.chg_off[f];
    bool walk_bad;
    uint64_t ts3;
    if (padded) {
        // LDS copy: lane 0 walks in vector registers (the four SIMDs' VALUs instead of the CU's
        // one scalar unit, which the wave-uniform walk saturates at ~15 waves per CU). Lengths are
        // clamped to len so positions cannot wrap and one check per change is exact: a position
        // only grows, so a read past the end makes the change's end pass len too. Reads are
        // clamped into the staged bytes (+80 padding).
        if (threadIdx.x == 0) {
            auto rd32 = [&](uint32_t a) -> uint32_t {
                a = a < len ? a : len;
                return (uint32_t)p[a] | (uint32_t)p[a + 1] << 8 | (uint32_t)p[a + 2] << 16 | (uint32_t)p[a + 3] << 24;
            };
            auto rd8 = [&](uint32_t a) -> uint32_t { return p[a < len ? a : len]; };
            // speculation: a change's table / pk / cid lengths are predicted to equal the previous
            // change's, so the four dependent reads (lt -> lp -> lc -> tag) are issued together and
            // a change costs one LDS round trip when the predictions hold (one table per changeset,
            // fixed-width pks and equal-length column names are the common case); a miss re-reads
            // from the first wrong field on, sequentially.
            uint32_t pos = d.chg_start[f];
            bool bad = false;
            uint32_t plt = 0, plp = 0, plc = 0;
            for (uint32_t k = 0; k < n; k++) {
                if (off_lds) s_off[k] = pos;
                else d.chg_rel[co + k] = pos;
                const uint32_t q1 = pos + 4 + plt, q2 = q1 + 4 + plp, q3 = q2 + 4 + plc;
                const uint32_t lt = rd32(pos), s1 = rd32(q1), s2 = rd32(q2), st = rd8(q3), sv = rd32(q3 + 1);
                uint32_t a = pos + 4 + min(lt, len);
                uint32_t lp, lc, tag, vl;
                if (lt == plt) {
                    lp = s1;
                } else {
                    lp = rd32(a);
                }
                const bool hit1 = lt == plt;
                a += 4 + min(lp, len);
                if (hit1 && lp == plp) {
                    lc = s2;
                } else {
                    lc = rd32(a);
                }
                const bool hit2 = hit1 && lp == plp;
                a += 4 + min(lc, len);
                if (hit2 && lc == plc) {
                    tag = st;
                    vl = sv;
                } else {
                    tag = rd8(a);
                    vl = rd32(a + 1);
                }
                plt = min(lt, len);
                plp = min(lp, len);
                plc = min(lc, len);
                a += 1;
                if (tag == 1 || tag == 2) a += 8;
                else if (tag == 3 || tag == 4) a += 4 + min(vl, len);
                else if (tag != 0) bad = true;
                a += 48;                             // col_version, db_version, seq, site_id, cl
                if (bad || a > len) {
                    bad = true;
                    break;
                }
                pos = a;
            }
            if (!bad && len - pos < 32) bad = true;
            uint64_t tl[4] = {0, 0, 0, 0};
            if (!bad)
                for (int i = 0; i < 4; i++) tl[i] = (uint64_t)rd32(pos + 8 * i) | (uint64_t)rd32(pos + 8 * i + 4) << 32;
            d.s0[f] = tl[0];
            d.s1[f] = tl[1];
            d.last[f] = tl[2];
            d.ts[f] = tl[3];
            s_tail = tl[3];
            s_bad = bad ? 1 : 0;
            if (!off_lds) __threadfence_block();
        }
        __syncthreads();
        walk_bad = s_bad != 0;
        ts3 = s_tail;
    } else {
        // the walk: offsets of the variable-length changes, then the Full tail (wave-uniform). Lane
        // k % 64 keeps change k's offset; every 64 changes the wave stores them at once.
        WaveWin w{p, len, 0, 0, padded};
        uint32_t pos = d.chg_start[f];
        w.load(pos);
        bool bad = false;
        uint32_t myoff = 0;
        uint32_t k = 0;
        const uint32_t lane = threadIdx.x;
        for (; k < n; k++) {
            if (lane == (k & 63)) myoff = pos;
            if ((k & 63) == 63) {
                if (off_lds) s_off[k - 63 + lane] = myoff;
                else d.chg_rel[co + k - 63 + lane] = myoff;
            }
            // table, pk, cid: u32 length + bytes each (a length must leave room for what follows)
            uint32_t a = pos;
    #pragma unroll
            for (int fld = 0; fld < 3; fld++) {
                if (a > len - 4 || len < 4) { bad = true; break; }
                const uint32_t l = w.u32(a);
                if (l > len - (a + 4)) { bad = true; break; }
                a += 4 + l;
            }
            if (bad) break;
            if (a > len - 4 || len < 4) { bad = true; break; }  // the tag is followed by >= 48 bytes
            const uint32_t tw = w.u32(a), tag = tw & 0xFF;
            a += 1;
            if (tag == 1 || tag == 2) {
                a += 8;
            } else if (tag == 3 || tag == 4) {
                if (a > len - 4) { bad = true; break; }
                const uint32_t l = w.u32(a);
                if (l > len - (a + 4)) { bad = true; break; }
                a += 4 + l;
            } else if (tag != 0) {
                bad = true;
                break;
            }
            if (a > len || len - a < 48) { bad = true; break; }  // col_version, db_version, seq, site_id, cl
            pos = a + 48;
        }
        if (!bad && (n & 63)) {  // the last partial group of offsets
            const uint32_t g0 = n & ~63u;
            if (lane < (n & 63)) {
                if (off_lds) s_off[g0 + lane] = myoff;
                else d.chg_rel[co + g0 + lane] = myoff;
            }
        }
        uint64_t tl[4] = {0, 0, 0, 0};
        if (!bad && len - pos >= 32) {
    #pragma unroll
            for (int i = 0; i < 4; i++) tl[i] = (uint64_t)w.u32(pos + 8 * i) | (uint64_t)w.u32(pos + 8 * i + 4) << 32;
        } else {
            bad = true;
        }
        ts3 = tl[3];
        if (threadIdx.x == 0) {
            d.s0[f] = tl[0];
            d.s1[f] = tl[1];
            d.last[f] = tl[2];
            d.ts[f] = tl[3];
            if (!off_lds) __threadfence_block();
        }
        walk_bad = bad;
    }
    WDIAG(2)
    __syncthreads();
    if (walk_bad) {
        if (threadIdx.x == 0) d.status[f] = CORRO_E_INVALID;
        return;
    }
    const uint64_t ts = ts3;
    int32_t err = 0;
    for (uint32_t k = threadIdx.x; k < n; k += 64) {
        Rd r{p, off_lds ? s_off[k] : d.chg_rel[co + k], len, false};
        const uint32_t lt = r.u32();
        const uint32_t pt = r.pos;
        r.pos += lt;
        const uint32_t lp = r.u32();
        const uint32_t pp = r.pos;
        r.pos += lp;
        const uint32_t lc = r.u32();
        const uint32_t pc = r.pos;
        r.pos += lc;
        // table / column names
        uint32_t tcid = CORRO_TCID_UNKNOWN;
        for (uint32_t t = 0; t < d.ntables; t++) {
            if (!name_eq(p + pt, lt, d.names + d.tname_off[t], d.tname_len[t])) continue;
            if (lc == 2 && p[pc] == '-' && p[pc + 1] == '1') {
                tcid = t << 16;
            } else {
                for (uint32_t c = 0; c < d.tncols[t]; c++) {
                    const uint32_t ci = d.tcol_base[t] + c;
                    if (name_eq(p + pc, lc, d.names + d.cname_off[ci], d.cname_len[ci])) {
                        tcid = (t << 16) | (c + 1);
                        break;
                    }
                }
            }
            break;
        }
        // pk: one packed INTEGER column (unpack_columns: get_int sign-extends big-endian bytes), or
        // for an interned table a reference to the packed bytes (the host interns them)
        uint64_t pk = 0;
        const uint64_t q = co + k;
        const bool known = tcid != CORRO_TCID_UNKNOWN;
        if (known && d.interned[tcid >> 16]) {
            d.pkref[q] = ((d.foff[f] + pp) << 32) | lp;
            atomicAdd(d.nref, 1ULL);
        } else if (lp < 2 || p[pp] != 1 || (p[pp + 1] & 7) != 1 || (uint32_t)(p[pp + 1] >> 3) + 2 != lp ||
                   (p[pp + 1] >> 3) > 8) {
            if (known) err = CORRO_E_RANGE;  // (a change of an unknown table rolls its version back anyway)
        } else {
            const uint32_t nb = p[pp + 1] >> 3;
            for (uint32_t i = 0; i < nb; i++) pk = (pk << 8) | p[pp + 2 + i];
            if (nb && nb < 8 && (pk >> (8 * nb - 1)) & 1) pk |= ~0ULL << (8 * nb);
        }
        // value -> (type, val0, val1, len)
        const uint32_t tag = (uint32_t)r.le(1);
        uint32_t vt = CORRO_NULL, vl = 0;
        uint64_t w0 = 0, w1 = 0;
        if (tag == 1) {
            vt = CORRO_INTEGER;
            w0 = r.u64();
        } else if (tag == 2) {
            w0 = r.u64();
            const bool nan = ((w0 >> 52) & 0x7FF) == 0x7FF && (w0 & 0xFFFFFFFFFFFFFULL);
            if (nan) w0 = 0;             // SQLite binds NaN as NULL
            else vt = CORRO_REAL;
        } else if (tag == 3 || tag == 4) {
            const uint32_t l = r.u32();
            vt = tag == 3 ? CORRO_TEXT : CORRO_BLOB;
            const uint32_t nb = l > 16 ? 8 : l;
            for (uint32_t i = 0; i < nb; i++) {
                const uint64_t b = p[r.pos + i];
                if (i < 8) w0 |= b << (8 * (7 - i));
                else w1 |= b << (8 * (15 - i));
            }
            vl = l;
            if (l > 16) {  // a long value: its bytes stay in the frame buffer
                vl = CORRO_VAL_LONG;
                if (!d.out.val_off || !d.out.val_size || l >= (1u << 24)) {
                    err = CORRO_E_RANGE;
                } else {
                    const_cast<uint64_t *>(d.out.val_off)[q] = d.foff[f] + r.pos;
                    const_cast<uint32_t *>(d.out.val_size)[q] = l;
                    atomicAdd(d.nlong, 1ULL);
                }
            }
            r.pos += l;
        }
        const int64_t cv = (int64_t)r.u64();
        const uint64_t dbv = r.u64();
        const uint64_t seq = r.u64();
        const uint64_t slo = r.u64(), shi = r.u64();
        const int64_t cl = (int64_t)r.u64();
        if (seq > 0xFFFFFFFFULL || cl < 0 || cl > 0xFFFFFFFFLL || dbv > (uint64_t)INT64_MAX) err = CORRO_E_RANGE;
        uint32_t so = site_lookup(d, slo, shi);
        if (so == 0xFFFFFFFFu) note_unknown(d, slo, shi);
        const corro_changes &o = d.out;
        const_cast<uint64_t *>(o.pk)[q] = pk;
        const_cast<uint32_t *>(o.table_cid)[q] = tcid;
        const_cast<int64_t *>(o.col_version)[q] = cv;
        const_cast<int64_t *>(o.db_version)[q] = (int64_t)dbv;
        const_cast<uint32_t *>(o.cl)[q] = (uint32_t)cl;
        const_cast<uint32_t *>(o.seq)[q] = (uint32_t)seq;
        const_cast<uint32_t *>(o.site)[q] = so;
        const_cast<uint64_t *>(o.val0)[q] = w0;
        if (o.val1) const_cast<uint64_t *>(o.val1)[q] = w1;
        if (o.val_type) const_cast<uint8_t *>(o.val_type)[q] = (uint8_t)vt;
        if (o.val_len) const_cast<uint8_t *>(o.val_len)[q] = (uint8_t)vl;
        if (o.ts) const_cast<uint64_t *>(o.ts)[q] = ts;
    }
    if (err) atomicMin(&d.status[f], err);
#if CORRO_DIAG & 512
    const uint64_t t3 = wall_clock64();
    if (threadIdx.x == 0 && (f % 997) == 0)
        printf("WDIAG f=%u len=%u n=%u stage=%lu walk=%lu decode=%lu (x10ns) t0=%lu\n", f, len, n,
               (unsigned long)(t1 - t0), (unsigned long)(t2 - t1), (unsigned long)(t3 - t2), (unsigned long)t0);
#endif
    };
    if (lds) body(s_buf, true);
    else body(g, false);
}

size_t al(size_t b) { return ((b + 255) / 256) * 256; }

uint64_t hmix(uint64_t x) {
    x ^= x >> 33; x *= 0xff51afd7ed558ccdULL;
    x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ULL;
    x ^= x >> 33; return x;
}

// device copies of the schema names (once) and of the site hash (whenever sites were added)
// the kept frames' headers on the device (map[f] = output index, ~0 = dropped)
__global__ void k_wire_cs(WireDev d, const uint32_t *__restrict__ map, corro_changeset *__restrict__ out) {
    const uint32_t f = blockIdx.x * blockDim.x + threadIdx.x;
    if (f >= d.nframes || map[f] == 0xFFFFFFFFu) return;
    corro_changeset c;
    const uint32_t k = d.cs_kind[f];
    c.actor_id = nullptr;
    c.site = d.site[f];
    c.kind = k == 0 ? CORRO_CS_EMPTY : (k == 1 ? CORRO_CS_FULL : CORRO_CS_EMPTY_SET);
    c.version_start = d.v0[f];
    c.version_end = d.v1[f];
    c.seq_start = d.s0[f];
    c.seq_end = d.s1[f];
    c.last_seq = d.last[f];
    c.ts = d.ts[f];
    c.change_off = k == 2 ? 0 : d.chg_off[f];
    c.change_count = k == 2 ? 0 : d.nchg[f];
    out[map[f]] = c;
}

int wire_tables(corro_ctx *ctx) {
    if (!ctx->wire_schema_ready) {
        std::vector<uint8_t> names;
        std::vector<uint32_t> toff, tlen, tbase, tn, coff, clen;
        for (const auto &t : ctx->tables) {
            toff.push_back((uint32_t)names.size());
            tlen.push_back((uint32_t)t.name.size());
            names.insert(names.end(), t.name.begin(), t.name.end());
            tbase.push_back((uint32_t)coff.size());
            tn.push_back((uint32_t)t.cols.size());
            for (const auto &c : t.cols) {
                coff.push_back((uint32_t)names.size());
                clen.push_back((uint32_t)c.size());
                names.insert(names.end(), c.begin(), c.end());
            }
        }
        const size_t nt = toff.size(), nc = coff.size();
        const size_t bytes = al(names.size() + 1) + 4 * al(nt * 4 + 4) + 2 * al(nc * 4 + 4);
        if (int rc = ctx->d_wire_schema.ensure(bytes)) return rc;
        uint8_t *q = ctx->d_wire_schema.as<uint8_t>();
        auto put = [&](const void *src, size_t b) -> uint8_t * {
            uint8_t *r = q;
            if (b && hipMemcpy(r, src, b, hipMemcpyHostToDevice) != hipSuccess) return nullptr;
            q += al(b + 4);
            return r;
        };
        ctx->wire_names = put(names.data(), names.size());
        ctx->wire_toff = (uint32_t *)put(toff.data(), nt * 4);
        ctx->wire_tlen = (uint32_t *)put(tlen.data(), nt * 4);
        ctx->wire_tbase = (uint32_t *)put(tbase.data(), nt * 4);
        ctx->wire_tn = (uint32_t *)put(tn.data(), nt * 4);
        ctx->wire_coff = (uint32_t *)put(coff.data(), nc * 4);
        ctx->wire_clen = (uint32_t *)put(clen.data(), nc * 4);
        if (!ctx->wire_names) return fail(CORRO_E_DEVICE, "upload of the schema names failed");
        ctx->wire_schema_ready = true;
    }
    if (ctx->wire_sites_n != ctx->sites.size() || !ctx->d_wire_sites.p) {
        const size_t n = ctx->sites.size();
        uint32_t H = 16;
        while (H < 2 * n) H <<= 1;
        std::vector<uint64_t> lo(H, 0), hi(H, 0);
        std::vector<uint32_t> ord(H, 0xFFFFFFFFu);
        for (size_t i = 0; i < n; i++) {
            uint64_t a, b;
            std::memcpy(&a, ctx->sites[i].data(), 8);
            std::memcpy(&b, ctx->sites[i].data() + 8, 8);
            uint32_t h = (uint32_t)hmix(a ^ (b * 0x9E3779B97F4A7C15ULL)) & (H - 1);
            while (ord[h] != 0xFFFFFFFFu) h = (h + 1) & (H - 1);
            lo[h] = a;
            hi[h] = b;
            ord[h] = (uint32_t)i;
        }
        if (int rc = ctx->d_wire_sites.ensure(al(H * 8ULL) * 2 + al(H * 4ULL))) return rc;
        uint8_t *q = ctx->d_wire_sites.as<uint8_t>();
        CORRO_HIP_TRY(hipMemcpy(q, lo.data(), H * 8ULL, hipMemcpyHostToDevice));
        CORRO_HIP_TRY(hipMemcpy(q + al(H * 8ULL), hi.data(), H * 8ULL, hipMemcpyHostToDevice));
        CORRO_HIP_TRY(hipMemcpy(q + 2 * al(H * 8ULL), ord.data(), H * 4ULL, hipMemcpyHostToDevice));
        ctx->wire_hmask = H - 1;
        ctx->wire_sites_n = n;
    }
    return CORRO_OK;
}

}  // namespace
}  // namespace corro

using namespace corro;

extern "C" int corro_decode_frames(corro_ctx *ctx, const uint8_t *buf, uint64_t len, int payload, int mem,
                                   corro_decoded *out, int pass) {
    if (!ctx || (!buf && len) || !out) return fail(CORRO_E_INVALID, "NULL argument");
    if (payload != CORRO_PAYLOAD_SYNC && payload != CORRO_PAYLOAD_UNI) return fail(CORRO_E_INVALID, "bad payload kind");
    if (mem != CORRO_MEM_HOST && mem != CORRO_MEM_DEVICE) return fail(CORRO_E_INVALID, "bad mem kind");
    if (pass != 0 && pass != 1) return fail(CORRO_E_INVALID, "pass must be 0 or 1");
    if (len >= (1ULL << 32)) return fail(CORRO_E_RANGE, "at most 4 GiB of frames per call");
    // frame scan (host: the length prefixes are a sequential chain)
    std::vector<uint64_t> foff;
    std::vector<uint32_t> flen;
    uint64_t pos = 0;
    while (pos + 4 <= len) {
        const uint32_t l = ((uint32_t)buf[pos] << 24) | ((uint32_t)buf[pos + 1] << 16) | ((uint32_t)buf[pos + 2] << 8) |
                           (uint32_t)buf[pos + 3];
        if (pos + 4 + l > len) return fail(CORRO_E_INVALID, "truncated frame");
        foff.push_back(pos + 4);
        flen.push_back(l);
        pos += 4 + (uint64_t)l;
    }
    if (pos != len) return fail(CORRO_E_INVALID, "trailing bytes after the last frame");
    const uint32_t F = (uint32_t)foff.size();
    if (pass == 0) {
        out->nframes = F;
        out->nchanges = out->nsets = 0;
    } else if (out->nframes != F) {
        return fail(CORRO_E_INVALID, "nframes differs from pass 0");
    }
    if (F == 0) return CORRO_OK;
    CORRO_HIP_TRY(hipSetDevice(ctx->device));
    hipStream_t s = ctx->stream;
    if (int rc = wire_tables(ctx)) return rc;
    const uint64_t NC = pass == 1 ? out->nchanges : 0, NS = pass == 1 ? out->nsets : 0;
    const uint32_t ucap = 4096;
    // scratch: bytes, frame index, headers, offsets, unknown sites, outputs staged for host mode
    const size_t hdr = 6 * al(F * 4ULL) + 6 * al(F * 8ULL) + al(F * 16ULL);
    const size_t outb = (mem == CORRO_MEM_HOST && pass == 1) ? (al(NC * 8) * 6 + al(NC * 4) * 4 + al(NC) * 2) : 0;
    const size_t need = al(len) + al(F * 8ULL) + al(F * 4ULL) + hdr + 2 * al((F + 1) * 8ULL) + al(NC * 4 + 4) +
                        al(ucap * 16ULL) + 256 + outb + 2 * al(NS * 8 + 8) + al(NC * 8 + 8) + al(NC * 12 + 12) +
                        al(ctx->tables.size() + 1);
    if (int rc = ctx->d_wire.ensure(need)) return rc;
    uint8_t *q = ctx->d_wire.as<uint8_t>();
    auto carve = [&](size_t b) {
        uint8_t *r = q;
        q += al(b);
        return r;
    };
    WireDev d{};
    uint8_t *dbuf = carve(len);
    uint64_t *dfoff = (uint64_t *)carve(F * 8ULL);
    uint32_t *dflen = (uint32_t *)carve(F * 4ULL);
    d.buf = dbuf;
    d.foff = dfoff;
    d.flen = dflen;
    d.nframes = F;
    d.kind = (uint32_t)payload;
    d.status = (int32_t *)carve(F * 4ULL);
    d.cs_kind = (uint32_t *)carve(F * 4ULL);
    d.nchg = (uint32_t *)carve(F * 4ULL);
    d.nset = (uint32_t *)carve(F * 4ULL);
    d.chg_start = (uint32_t *)carve(F * 4ULL);
    d.site = (uint32_t *)carve(F * 4ULL);
    d.v0 = (uint64_t *)carve(F * 8ULL);
    d.v1 = (uint64_t *)carve(F * 8ULL);
    d.s0 = (uint64_t *)carve(F * 8ULL);
    d.s1 = (uint64_t *)carve(F * 8ULL);
    d.last = (uint64_t *)carve(F * 8ULL);
    d.ts = (uint64_t *)carve(F * 8ULL);
    d.actor = carve(F * 16ULL);
    uint64_t *dchg = (uint64_t *)carve((F + 1) * 8ULL), *dset = (uint64_t *)carve((F + 1) * 8ULL);
    d.chg_off = dchg;
    d.set_off = dset;
    d.chg_rel = (uint32_t *)carve(NC * 4 + 4);
    d.unknown = carve(ucap * 16ULL);
    d.nunknown = (unsigned long long *)carve(256);
    d.nref = d.nunknown + 1;
    d.nlong = d.nunknown + 2;
    d.unknown_cap = ucap;
    d.pkref = (uint64_t *)carve(NC * 8 + 8);
    {
        std::vector<uint8_t> fl(ctx->tables.size() + 1, 0);
        for (size_t t = 0; t < ctx->tables.size() && t < ctx->pk.size(); t++) fl[t] = ctx->pk[t].interned ? 1 : 0;
        uint8_t *dfl = carve(fl.size());
        CORRO_HIP_TRY(hipMemcpyAsync(dfl, fl.data(), fl.size(), hipMemcpyHostToDevice, s));
        d.interned = dfl;
    }
    d.names = ctx->wire_names;
    d.tname_off = ctx->wire_toff;
    d.tname_len = ctx->wire_tlen;
    d.tcol_base = ctx->wire_tbase;
    d.tncols = ctx->wire_tn;
    d.cname_off = ctx->wire_coff;
    d.cname_len = ctx->wire_clen;
    d.ntables = (uint32_t)ctx->tables.size();
    CORRO_HIP_TRY(hipMemcpyAsync(dbuf, buf, len, hipMemcpyHostToDevice, s));
    CORRO_HIP_TRY(hipMemcpyAsync(dfoff, foff.data(), F * 8ULL, hipMemcpyHostToDevice, s));
    CORRO_HIP_TRY(hipMemcpyAsync(dflen, flen.data(), F * 4ULL, hipMemcpyHostToDevice, s));
    // outputs
    corro_changes o{};
    uint64_t *dss = nullptr, *dse = nullptr;
    if (pass == 1) {
        if (mem == CORRO_MEM_DEVICE) {
            o = out->changes;
            dss = out->set_start;
            dse = out->set_end;
        } else {
            o.pk = (uint64_t *)carve(NC * 8);
            o.col_version = (int64_t *)carve(NC * 8);
            o.db_version = (int64_t *)carve(NC * 8);
            o.val0 = (uint64_t *)carve(NC * 8);
            o.val1 = (uint64_t *)carve(NC * 8);
            o.ts = (uint64_t *)carve(NC * 8);
            o.table_cid = (uint32_t *)carve(NC * 4);
            o.cl = (uint32_t *)carve(NC * 4);
            o.seq = (uint32_t *)carve(NC * 4);
            o.site = (uint32_t *)carve(NC * 4);
            o.val_type = (uint8_t *)carve(NC);
            o.val_len = (uint8_t *)carve(NC);
            dss = (uint64_t *)carve(NS * 8 + 8);
            dse = (uint64_t *)carve(NS * 8 + 8);
            // long values' spans, when the caller takes them
            uint8_t *lv = carve(NC * 12 + 12);
            if (out->changes.val_off && out->changes.val_size) {
                o.val_off = (uint64_t *)lv;
                o.val_size = (uint32_t *)(lv + NC * 8 + 8);
            }
        }
        if (NC && (!o.pk || !o.table_cid || !o.col_version || !o.db_version || !o.cl || !o.seq || !o.site || !o.val0))
            return fail(CORRO_E_INVALID, "a required change output array is NULL");
        if (NS && (!dss || !dse)) return fail(CORRO_E_INVALID, "EmptySet range outputs are NULL");
    }
    d.out = o;
    d.set_start = dss;
    d.set_end = dse;
    std::vector<int32_t> st(F);
    std::vector<uint32_t> kind(F), nchg(F), nset(F), site(F);
    std::vector<uint64_t> cofs(F + 1, 0);
    uint64_t cnt3[3] = {0, 0, 0};  // unknown sites, interned pk references, long values
    for (int attempt = 0; attempt < 2; attempt++) {
        if (int rc = wire_tables(ctx)) return rc;
        uint8_t *sq = ctx->d_wire_sites.as<uint8_t>();
        const uint32_t H = ctx->wire_hmask + 1;
        d.hlo = (const uint64_t *)sq;
        d.hhi = (const uint64_t *)(sq + al(H * 8ULL));
        d.hord = (const uint32_t *)(sq + 2 * al(H * 8ULL));
        d.hmask = ctx->wire_hmask;
        CORRO_HIP_TRY(hipMemsetAsync(d.nunknown, 0, 24, s));
        if (NC) CORRO_HIP_TRY(hipMemsetAsync(d.pkref, 0, NC * 8, s));
        if (ctx->profiling) CORRO_HIP_TRY(hipEventRecord(ctx->ev[0], s));
        hipLaunchKernelGGL(k_wire_hdr, dim3((F + 255) / 256), dim3(256), 0, s, d);
        if (ctx->profiling) CORRO_HIP_TRY(hipEventRecord(ctx->ev[1], s));
        CORRO_HIP_TRY(hipGetLastError());
        CORRO_HIP_TRY(hipMemcpyAsync(st.data(), d.status, F * 4ULL, hipMemcpyDeviceToHost, s));
        CORRO_HIP_TRY(hipMemcpyAsync(kind.data(), d.cs_kind, F * 4ULL, hipMemcpyDeviceToHost, s));
        CORRO_HIP_TRY(hipMemcpyAsync(nchg.data(), d.nchg, F * 4ULL, hipMemcpyDeviceToHost, s));
        CORRO_HIP_TRY(hipMemcpyAsync(nset.data(), d.nset, F * 4ULL, hipMemcpyDeviceToHost, s));
        CORRO_HIP_TRY(hipStreamSynchronize(s));
        std::vector<uint64_t> co(F + 1, 0), so(F + 1, 0);
        for (uint32_t f = 0; f < F; f++) {
            co[f + 1] = co[f] + nchg[f];
            so[f + 1] = so[f] + nset[f];
        }
        if (pass == 0) {
            out->nchanges = co[F];
            out->nsets = so[F];
            return CORRO_OK;
        }
        if (co[F] != NC || so[F] != NS) return fail(CORRO_E_INVALID, "sizes differ from pass 0");
        cofs = co;
        CORRO_HIP_TRY(hipMemcpyAsync(dchg, co.data(), (F + 1) * 8ULL, hipMemcpyHostToDevice, s));
        CORRO_HIP_TRY(hipMemcpyAsync(dset, so.data(), (F + 1) * 8ULL, hipMemcpyHostToDevice, s));
        // (device time = header kernel + these two: the host round trip between them is not kernel time)
        if (ctx->profiling) CORRO_HIP_TRY(hipEventRecord(ctx->ev[2], s));
        hipLaunchKernelGGL(k_wire_sets, dim3((F + 255) / 256), dim3(256), 0, s, d);
        {
            // LDS sized by this call's Full frames (occupancy is LDS-bound: ~10 KB frames fit 15
            // workgroups per CU where a fixed 20 KB fits 8); longer frames are read from HBM
            uint32_t ml = 0, mn = 0;
            for (uint32_t f = 0; f < F; f++)
                if (!st[f] && kind[f] == 1) {
                    if (flen[f] <= WIRE_LDS) ml = std::max(ml, flen[f]);
                    mn = std::max(mn, std::min(nchg[f], WIRE_OFFS));
                }
            d.lds_len = (ml + 15) & ~15u;
            d.off_cap = (mn + 3) & ~3u;
        }
        // (+ 80 bytes: the walk's window reads run up to 67 bytes past a frame)
        hipLaunchKernelGGL(k_wire_decode, dim3(F), dim3(64), (size_t)d.off_cap * 4 + d.lds_len + 80, s, d);
        if (ctx->profiling) CORRO_HIP_TRY(hipEventRecord(ctx->ev[3], s));
        CORRO_HIP_TRY(hipGetLastError());
        CORRO_HIP_TRY(hipMemcpyAsync(cnt3, d.nunknown, 24, hipMemcpyDeviceToHost, s));
        CORRO_HIP_TRY(hipStreamSynchronize(s));
        const uint64_t nu = cnt3[0];
        if (ctx->profiling) {
            float a = 0.f, b = 0.f;
            CORRO_HIP_TRY(hipEventElapsedTime(&a, ctx->ev[0], ctx->ev[1]));
            CORRO_HIP_TRY(hipEventElapsedTime(&b, ctx->ev[2], ctx->ev[3]));
            ctx->last_ms[7] = a + b;
        }
        if (nu == 0) break;
        if (attempt == 1) return fail(CORRO_E_DEVICE, "internal: sites still unknown after registering them");
        // register every site id seen but not yet known, then decode again with the new table
        const uint64_t take = std::min<uint64_t>(nu, ucap);
        std::vector<uint8_t> ids(take * 16);
        CORRO_HIP_TRY(hipMemcpy(ids.data(), d.unknown, take * 16, hipMemcpyDeviceToHost));
        if (int rc = corro_site_register(ctx, ids.data(), take, nullptr)) return rc;
        if (nu > ucap) attempt = -1;  // more unknown ids than one pass collects: keep going
    }
    // interned pks: their packed bytes -> row keys on the device (pk_keys_device), patched into the
    // decoded pk column before anything is copied out; a malformed pk fails its frame
    if (cnt3[1] && NC) {
        if (int rc = ctx->d_pk_bad.ensure(NC + 256)) return rc;
        uint8_t *dbad = ctx->d_pk_bad.as<uint8_t>();
        bool any_bad = false;
        for (uint32_t t = 0; t < (uint32_t)ctx->pk.size(); t++) {
            if (!ctx->pk[t].interned) continue;
            PkRefs pr;
            pr.base = dbuf;
            pr.ref = d.pkref;
            pr.none = 0;
            pr.len_bits = 32;
            pr.tcid = o.table_cid;
            uint64_t nbad = 0;
            if (int rc = pk_keys_device(ctx, t, pr, NC, const_cast<uint64_t *>(o.pk), dbad + 0, &nbad)) return rc;
            if (nbad) {
                if (!any_bad) CORRO_HIP_TRY(hipMemcpy(st.data(), d.status, F * 4ULL, hipMemcpyDeviceToHost));
                std::vector<uint8_t> hb(NC);
                CORRO_HIP_TRY(hipMemcpy(hb.data(), dbad, NC, hipMemcpyDeviceToHost));
                uint32_t f = 0;
                for (uint64_t q = 0; q < NC; q++) {
                    if (!hb[q]) continue;
                    while (cofs[f + 1] <= q) f++;
                    st[f] = std::min(st[f], (int32_t)CORRO_E_INVALID);
                }
                any_bad = true;
            }
        }
        if (any_bad)  // (the frames' status words on the device, read back with the headers below)
            CORRO_HIP_TRY(hipMemcpy(d.status, st.data(), F * 4ULL, hipMemcpyHostToDevice));
    }
    // headers -> host
    std::vector<uint64_t> v0(F), v1(F), s0(F), s1(F), last(F), ts(F);
    std::vector<uint8_t> actor(F * 16ULL);
    CORRO_HIP_TRY(hipMemcpyAsync(st.data(), d.status, F * 4ULL, hipMemcpyDeviceToHost, s));
    CORRO_HIP_TRY(hipMemcpyAsync(site.data(), d.site, F * 4ULL, hipMemcpyDeviceToHost, s));
    struct H8 { std::vector<uint64_t> *h; uint64_t *dv; } h8[] = {{&v0, d.v0}, {&v1, d.v1}, {&s0, d.s0}, {&s1, d.s1},
                                                                  {&last, d.last}, {&ts, d.ts}};
    for (auto &x : h8) CORRO_HIP_TRY(hipMemcpyAsync(x.h->data(), x.dv, F * 8ULL, hipMemcpyDeviceToHost, s));
    CORRO_HIP_TRY(hipMemcpyAsync(actor.data(), d.actor, F * 16ULL, hipMemcpyDeviceToHost, s));
    if (mem == CORRO_MEM_HOST && NC) {
        const corro_changes &h = out->changes;
        struct Cp { const void *dst; const void *src; size_t b; } cp[] = {
            {h.pk, o.pk, NC * 8},         {h.col_version, o.col_version, NC * 8}, {h.db_version, o.db_version, NC * 8},
            {h.val0, o.val0, NC * 8},     {h.val1, o.val1, NC * 8},               {h.ts, o.ts, NC * 8},
            {h.table_cid, o.table_cid, NC * 4}, {h.cl, o.cl, NC * 4},             {h.seq, o.seq, NC * 4},
            {h.site, o.site, NC * 4},     {h.val_type, o.val_type, NC},           {h.val_len, o.val_len, NC},
            {cnt3[2] ? h.val_off : nullptr, o.val_off, NC * 8}, {cnt3[2] ? h.val_size : nullptr, o.val_size, NC * 4}};
        for (auto &c : cp)
            if (c.dst) CORRO_HIP_TRY(hipMemcpyAsync(const_cast<void *>(c.dst), c.src, c.b, hipMemcpyDeviceToHost, s));
    }
    if (mem == CORRO_MEM_HOST && NS) {
        CORRO_HIP_TRY(hipMemcpyAsync(out->set_start, dss, NS * 8, hipMemcpyDeviceToHost, s));
        CORRO_HIP_TRY(hipMemcpyAsync(out->set_end, dse, NS * 8, hipMemcpyDeviceToHost, s));
    }
    CORRO_HIP_TRY(hipStreamSynchronize(s));
    // long values: the frame bytes are the batch's val_data (host: the caller's own buffer)
    corro_changes &oc = out->changes;
    if (cnt3[2]) {
        if (mem == CORRO_MEM_HOST) {
            oc.val_data = buf;
        } else {
            if (!oc.val_data) return fail(CORRO_E_RANGE, "long values decoded: changes.val_data must hold len bytes");
            CORRO_HIP_TRY(hipMemcpyAsync(const_cast<uint8_t *>(oc.val_data), dbuf, len, hipMemcpyDeviceToDevice, s));
        }
        oc.val_data_len = len;
    } else if (pass == 1) {
        oc.val_off = nullptr;
        oc.val_size = nullptr;
        oc.val_data = nullptr;
        oc.val_data_len = 0;
    }
    if (out->cs_dev) {  // the kept headers for CORRO_MEM_DEVICE_HEADERS, built where they lie
        std::vector<uint32_t> map(F);
        uint64_t k = 0;
        for (uint32_t f = 0; f < F; f++) map[f] = st[f] == 0 ? (uint32_t)k++ : 0xFFFFFFFFu;
        if (int rc = ctx->d_wire_map.ensure(F * 4ULL + 256)) return rc;
        CORRO_HIP_TRY(hipMemcpyAsync(ctx->d_wire_map.p, map.data(), F * 4ULL, hipMemcpyHostToDevice, s));
        hipLaunchKernelGGL(k_wire_cs, dim3((F + 255) / 256), dim3(256), 0, s, d, ctx->d_wire_map.as<uint32_t>(), out->cs_dev);
        CORRO_HIP_TRY(hipGetLastError());
        CORRO_HIP_TRY(hipStreamSynchronize(s));  // (map is a host vector)
        out->n_dev = k;
    }
    if (!out->cs) {
        if (out->status)
            for (uint32_t f = 0; f < F; f++) out->status[f] = st[f];
        return CORRO_OK;
    }
    uint64_t coff = 0, soff = 0;
    for (uint32_t f = 0; f < F; f++) {
        corro_changeset &c = out->cs[f];
        std::memcpy(out->actor_ids + 16ULL * f, actor.data() + 16ULL * f, 16);
        c.actor_id = out->actor_ids + 16ULL * f;
        c.site = site[f];
        // speedy variant index (Empty 0, Full 1, EmptySet 2) -> CORRO_CS_*
        c.kind = kind[f] == 0 ? CORRO_CS_EMPTY : (kind[f] == 1 ? CORRO_CS_FULL : CORRO_CS_EMPTY_SET);
        c.version_start = v0[f];
        c.version_end = v1[f];
        c.seq_start = s0[f];
        c.seq_end = s1[f];
        c.last_seq = last[f];
        c.ts = ts[f];
        c.change_off = kind[f] == 2 ? soff : coff;
        c.change_count = kind[f] == 2 ? nset[f] : nchg[f];
        coff += nchg[f];
        soff += nset[f];
        if (out->status) out->status[f] = st[f];
    }
    return CORRO_OK;
}
