// Row keys of primary keys (host side). corrosion ships a row's primary key as pack_columns bytes
// (/root/reference/crates/corro-types/src/pubsub.rs:2304-2358; unpack_columns :2396-2451); cr-sqlite
// keys its clock rows by `__crsql_key`, the rowid of the packed pk in `<t>__crsql_pks`. Here:
//   * a table whose primary key is one INTEGER column keys a row by that integer (the default);
//   * any other table (BLOB, TEXT, REAL or composite pk -- corro-tests' testsblob and wide) is
//     "interned": a row is keyed by a dense id per table, the `__crsql_pks` analogue, held in HBM
//     next to the state (round 5: an open-addressing device table, so a wire decoder, the multi-GPU
//     receiver or a caller with pk bytes in HBM interns without a host round trip).
// pks are canonicalised before interning (unpacked and re-packed the way pack_columns packs), so
// non-canonical encodings of one key name one row, as cr-sqlite's re-packing makes them (SURVEY
// App. A.3).
//
// Device intern (pk_keys_device), per table, over the changes that reference packed bytes (round 6:
// one fused pass for the common case):
//   k_pk_find    per wave, the 64 changes' packed bytes staged in LDS with 16-B loads along the bytes;
//                per change unpack_columns + pack_columns restated without writing (canonical length,
//                route hash pk_route_hash, whether the input already is canonical, the value of a
//                one-INTEGER pk), then the probe of the table's slots (plain 32-B slot loads): a held key
//                writes its id straight into keys[] (a warm call is this one kernel); an empty slot is
//                claimed with one 64-bit CAS of (tag, NEW | change); a change that finds another's claim
//                compares against the claimant's input bytes and raises the claim's first-seen word
//   [k_pk_canon, k_pk_probe_slow]  only for inputs that are not canonical: their canonical bytes into a
//                scratch, then the same probe through the claimants' recorded bytes
//   k_pk_mark + scans  each claim's first-seen position flagged -> new ids (table size + rank) in
//                first-seen order, their bytes -> arena offsets
//   k_pk_commit  keys of the new keys; each claim's canonical bytes, offset and hash appended, its slot
//                -> the id and the key's inline words
// The slots (32 B: claim word, length, up to 23 canonical bytes inline) are sized by the keys the
// table holds (load <= 1/2 with a share of new ones), not by the changes of a call; a probe that runs
// past PK_MAX_PROBE slots marks the call for a retry with a table four times larger (rebuilt from the
// arena). Any failed call drops its claims (the slots rebuilt from the committed keys).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <string>
#include <vector>

#include "internal.h"

#define TRY_PK(x)                        \
    do {                                 \
        int rc_ = (x);                   \
        if (rc_ != CORRO_OK) return rc_; \
    } while (0)

namespace corro {

namespace {

// num_bytes_needed_i64 / _i32 of pubsub.rs:2363-2388, quirks included (1 byte iff val * 0xFF != 0
// for a value in the last byte; any set bit in a higher byte takes every byte up to it)
uint32_t nbytes_i32(int32_t v) {
    if (v & (int32_t)0xFF000000u) return 4;
    if (v & 0x00FF0000) return 3;
    if (v & 0x0000FF00) return 2;
    if ((int32_t)((uint32_t)v * 0xFFu) != 0) return 1;
    return 0;
}
uint32_t nbytes_i64(int64_t v) {
    if (v & (int64_t)0xFF00000000000000ULL) return 8;
    if (v & 0x00FF000000000000LL) return 7;
    if (v & 0x0000FF0000000000LL) return 6;
    if (v & 0x000000FF00000000LL) return 5;
    return nbytes_i32((int32_t)v);
}

void put_int(std::string &out, int64_t v, uint32_t nb) {
    for (uint32_t i = 0; i < nb; i++) out.push_back((char)(uint8_t)((uint64_t)v >> (8 * (nb - 1 - i))));
}

// bytes::Buf::get_int(n): n big-endian bytes, sign-extended
bool get_int(const uint8_t *p, uint64_t len, uint64_t &pos, uint32_t n, int64_t &v) {
    if (n > 8 || len - pos < n) return false;
    uint64_t x = 0;
    for (uint32_t i = 0; i < n; i++) x = (x << 8) | p[pos + i];
    if (n && n < 8 && ((x >> (8 * n - 1)) & 1)) x |= ~0ULL << (8 * n);
    pos += n;
    v = (int64_t)x;
    return true;
}

}  // namespace

// unpack_columns + pack_columns: the canonical bytes of a packed pk; false when malformed.
// Sets *single_int (and *ival) when the pk is exactly one INTEGER column.
bool pk_canonical(const uint8_t *p, uint64_t len, std::string &out, bool *single_int, int64_t *ival) {
    out.clear();
    if (len < 1) return false;
    uint64_t pos = 0;
    const uint32_t ncol = p[pos++];
    out.push_back((char)ncol);
    bool one_int = ncol == 1;
    for (uint32_t c = 0; c < ncol; c++) {
        if (pos >= len) return false;
        const uint8_t tb = p[pos++];
        const uint32_t type = tb & 7, intlen = tb >> 3;
        int64_t v = 0;
        switch (type) {
        case CORRO_INTEGER:
            if (!get_int(p, len, pos, intlen, v)) return false;
            out.push_back((char)(uint8_t)((nbytes_i64(v) << 3) | CORRO_INTEGER));
            put_int(out, v, nbytes_i64(v));
            if (ival) *ival = v;
            break;
        case CORRO_REAL: {
            if (len - pos < 8) return false;
            uint64_t bits = 0;
            for (int i = 0; i < 8; i++) bits = (bits << 8) | p[pos + i];
            pos += 8;
            if (bits == 0x8000000000000000ULL) bits = 0;  // -0.0 and 0.0 are one key
            out.push_back((char)CORRO_REAL);
            put_int(out, (int64_t)bits, 8);
            one_int = false;
            break;
        }
        case CORRO_TEXT:
        case CORRO_BLOB: {
            if (!get_int(p, len, pos, intlen, v) || v < 0 || (uint64_t)v > len - pos) return false;
            const uint32_t nb = nbytes_i32((int32_t)v);
            out.push_back((char)(uint8_t)((nb << 3) | type));
            put_int(out, v, nb);
            out.append(reinterpret_cast<const char *>(p + pos), (size_t)v);
            pos += (uint64_t)v;
            one_int = false;
            break;
        }
        case CORRO_NULL:
            out.push_back((char)CORRO_NULL);
            one_int = false;
            break;
        default:
            return false;
        }
    }
    if (single_int) *single_int = one_int;
    return true;
}

// Owner-routing hash of a canonical packed pk: FNV-1a over the bytes, then a 64-bit finaliser. A
// function of the bytes alone, so every engine routes a row to the same rank whatever dense id its
// own intern table gave it.
uint64_t pk_route_hash(const std::string &canon) {
    uint64_t h = 0xCBF29CE484222325ULL;
    for (unsigned char c : canon) {
        h ^= c;
        h *= 0x100000001B3ULL;
    }
    h ^= h >> 33;
    h *= 0xFF51AFD7ED558CCDULL;
    h ^= h >> 33;
    h *= 0xC4CEB9FE1A85EC53ULL;
    h ^= h >> 33;
    return h;
}

// grow a device buffer to hold `want` bytes, keeping its first `keep` bytes
static int grow_keep(DevBuf &b, size_t want, size_t keep, hipStream_t s) {
    if (want <= b.bytes && b.p) return CORRO_OK;
    DevBuf nb;
    if (int rc = nb.ensure(std::max<size_t>(want, 2 * b.bytes))) return rc;
    if (keep) CORRO_HIP_TRY(hipMemcpyAsync(nb.p, b.p, keep, hipMemcpyDeviceToDevice, s));
    CORRO_HIP_TRY(hipStreamSynchronize(s));
    b.release();
    b = nb;
    nb.p = nullptr;
    return CORRO_OK;
}

int pk_mirror_sync(corro_ctx *ctx) {
    if (ctx->pk.size() < ctx->tables.size()) ctx->pk.resize(ctx->tables.size());
    hipStream_t s = ctx->stream;
    std::vector<PkDir> dir(ctx->tables.size());
    for (size_t t = 0; t < ctx->tables.size(); t++) {
        const PkTable &pt = ctx->pk[t];
        PkDir &d = dir[t];
        d = PkDir{};
        d.interned = pt.interned ? 1u : 0u;
        if (!pt.interned) continue;
        d.off = pt.d_off.as<uint64_t>();
        d.bytes = pt.d_bytes.as<uint8_t>();
        d.hash = pt.d_hash.as<uint64_t>();
        d.n = pt.n;
    }
    if (int rc = ctx->d_pkdir.ensure(std::max<size_t>(dir.size(), 1) * sizeof(PkDir))) return rc;
    if (dir.empty()) dir.push_back(PkDir{});  // (no table: one zeroed entry, never an uninitialised one)
    CORRO_HIP_TRY(hipMemcpyAsync(ctx->d_pkdir.p, dir.data(), dir.size() * sizeof(PkDir), hipMemcpyHostToDevice, s));
    CORRO_HIP_TRY(hipStreamSynchronize(s));
    return CORRO_OK;
}

// ---- device intern ---------------------------------------------------------------------------------
int prim_inclusive_scan_u32(void *temp, size_t *temp_bytes, const uint32_t *in, uint32_t *out, uint32_t n,
                            hipStream_t s);
int prim_inclusive_scan_u32_u64(void *temp, size_t *temp_bytes, const uint32_t *in, uint64_t *out, uint64_t n,
                                hipStream_t s);
int prim_inclusive_max_u64(void *temp, size_t *temp_bytes, const uint64_t *in, uint64_t *out, uint64_t n, hipStream_t s);
int ovf_sort_pairs(void *temp, size_t *temp_bytes, const uint64_t *ki, uint64_t *ko, const uint32_t *vi, uint32_t *vo,
                   uint32_t n, uint32_t end_bit, hipStream_t s);

namespace {

constexpr uint32_t PK_NEW = 0x80000000u;   // slot / owner word: a claim by change (word & ~PK_NEW)
constexpr uint32_t PK_INLINE = 23;         // canonical keys of at most this many bytes live in their slot

// One slot, 32 B (one half of a cache line): the claim word (tag << 32 | id, or | PK_NEW | change while a
// call's new key is being interned) and, once committed, the key's length and -- for a short key -- its
// canonical bytes, so a lookup of an existing key reads one line (the arena only for longer keys).
struct alignas(32) PkSlot {
    unsigned long long w;
    uint8_t len;
    uint8_t b[PK_INLINE];
};
static_assert(sizeof(PkSlot) == 32, "pk slot size");
constexpr uint32_t PK_MAX_PROBE = 256;     // past this many slots a probe asks for a larger table
// Homes lie in the first PkTable::nslots slots; PK_PAD more follow them before a probe wraps to slot 0,
// so a table rebuilt in home order (pk_place_ordered) holds every key between its home and the end.
constexpr uint64_t PK_PAD = 1024;
constexpr uint64_t PK_SCRATCH = 1ULL << 63;  // cref: canonical bytes in the scratch, not the input

__device__ inline uint32_t pk_wave_sum(uint32_t x) {
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) x += (uint32_t)__shfl_xor(x, o);
    return x;
}
__device__ inline uint32_t pk_wave_max(uint32_t x) {
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) x = max(x, (uint32_t)__shfl_xor(x, o));
    return x;
}

__device__ inline uint32_t dnb32(int32_t v) {
    if (v & (int32_t)0xFF000000u) return 4;
    if (v & 0x00FF0000) return 3;
    if (v & 0x0000FF00) return 2;
    if ((int32_t)((uint32_t)v * 0xFFu) != 0) return 1;
    return 0;
}
__device__ inline uint32_t dnb64(int64_t v) {
    if (v & (int64_t)0xFF00000000000000ULL) return 8;
    if (v & 0x00FF000000000000LL) return 7;
    if (v & 0x0000FF0000000000LL) return 6;
    if (v & 0x000000FF00000000LL) return 5;
    return dnb32((int32_t)v);
}

// the canonical bytes of one packed pk as they are produced: counted, hashed (pk_route_hash's
// FNV-1a), compared with the input at the same position, written when WRITE
template <bool WRITE>
struct CanonOut {
    const uint8_t *in;
    uint64_t len;
    uint8_t *out;
    uint64_t o = 0, h = 0xCBF29CE484222325ULL;
    bool same = true;
    __device__ inline void put(uint8_t c) {
        if (WRITE) out[o] = c;
        h = (h ^ c) * 0x100000001B3ULL;
        if (o >= len || in[o] != c) same = false;
        o++;
    }
    __device__ inline void put_int(int64_t v, uint32_t nb) {
        for (uint32_t i = 0; i < nb; i++) put((uint8_t)((uint64_t)v >> (8 * (nb - 1 - i))));
    }
    __device__ inline uint64_t hash() const {
        uint64_t x = h;
        x ^= x >> 33;
        x *= 0xFF51AFD7ED558CCDULL;
        x ^= x >> 33;
        x *= 0xC4CEB9FE1A85EC53ULL;
        x ^= x >> 33;
        return x;
    }
};

__device__ inline bool dget_int(const uint8_t *p, uint64_t len, uint64_t &pos, uint32_t n, int64_t &v) {
    if (n > 8 || len - pos < n) return false;
    uint64_t x = 0;
    for (uint32_t i = 0; i < n; i++) x = (x << 8) | p[pos + i];
    if (n && n < 8 && ((x >> (8 * n - 1)) & 1)) x |= ~0ULL << (8 * n);
    pos += n;
    v = (int64_t)x;
    return true;
}

// pk_canonical (host, above) on the device: false when malformed
template <bool WRITE>
__device__ bool pk_canon_dev(const uint8_t *p, uint64_t len, CanonOut<WRITE> &co, bool &one_int, int64_t &ival) {
    if (len < 1) return false;
    uint64_t pos = 0;
    const uint32_t ncol = p[pos++];
    co.put((uint8_t)ncol);
    one_int = ncol == 1;
    for (uint32_t c = 0; c < ncol; c++) {
        if (pos >= len) return false;
        const uint8_t tb = p[pos++];
        const uint32_t type = tb & 7, intlen = tb >> 3;
        int64_t v = 0;
        if (type == CORRO_INTEGER) {
            if (!dget_int(p, len, pos, intlen, v)) return false;
            const uint32_t nb = dnb64(v);
            co.put((uint8_t)((nb << 3) | CORRO_INTEGER));
            co.put_int(v, nb);
            ival = v;
        } else if (type == CORRO_REAL) {
            if (len - pos < 8) return false;
            uint64_t bits = 0;
            for (int i = 0; i < 8; i++) bits = (bits << 8) | p[pos + i];
            pos += 8;
            if (bits == 0x8000000000000000ULL) bits = 0;  // -0.0 and 0.0 are one key
            co.put((uint8_t)CORRO_REAL);
            co.put_int((int64_t)bits, 8);
            one_int = false;
        } else if (type == CORRO_TEXT || type == CORRO_BLOB) {
            if (!dget_int(p, len, pos, intlen, v) || v < 0 || (uint64_t)v > len - pos) return false;
            const uint32_t nb = dnb32((int32_t)v);
            co.put((uint8_t)((nb << 3) | type));
            co.put_int(v, nb);
            for (uint64_t k = 0; k < (uint64_t)v; k++) co.put(p[pos + k]);
            pos += (uint64_t)v;
            one_int = false;
        } else if (type == CORRO_NULL) {
            co.put((uint8_t)CORRO_NULL);
            one_int = false;
        } else {
            return false;
        }
    }
    return true;
}

constexpr uint64_t PK_PENDING = 1ULL << 63;  // keys[i] during a call: a new key, claimed by change (key & ~bit)

struct PkArgs {
    PkRefs r;
    uint32_t table;
    uint32_t interned;
    uint64_t n;
    uint64_t *keys;     // the row keys (PK_PENDING | claimant while a new key is unresolved)
    uint8_t *bad;
    // per change, written only for the changes that need them (claimants and slow-path changes)
    uint32_t *clen;     // canonical length
    uint64_t *cref;     // where its canonical bytes are: input offset, or PK_SCRATCH | scratch offset
    uint64_t *h;        // route hash
    uint32_t *slotix;   // a claimant's slot
    uint32_t *firstof;  // a claimant's first-seen position (k_pk_mark: read before any commit overwrites the word)
    // (the claimants are not listed: one same-address append per wave of a cold call -- a million of them
    // at config 2 -- serialised at the memory side for ~20 ms; k_pk_mark / k_pk_newkeys find them by
    // keys[i] == PENDING | i in one streaming pass instead)
    uint32_t *slow;     // changes whose input is not canonical (ctl[2] of them): canonicalised, then probed
    uint32_t *newf;     // at each new key's first-seen position: 1
    uint32_t *newl;     // at each new key's first-seen position: its canonical length
    uint32_t *rank;     // inclusive scan of newf
    uint64_t *noff;     // inclusive scan of newl
    uint8_t *scratch;
    // [0] bad [1] max canonical length [2] slow changes [3] probe overflow [4] claims
    // [5] canonical bytes of the slow changes [6] scratch cursor
    unsigned long long *ctl;
    // the table
    PkSlot *slots;
    uint64_t nsl;       // slots, PK_PAD past the homes: a probe wraps here
    uint64_t nhome;     // home slots (a multiple of 8, not a power of two: sized for the MALL, see pk_slots_for)
    uint64_t *koff;
    uint8_t *kbytes;
    uint64_t *khash;
    uint64_t nkeys, nbytes;
};

// change i's packed bytes: 1 with (offset from base, length), 0 when it is not a change of this table
// (or has no reference), -1 when its reference lies outside the buffer (a corrupt exchange
// must not read past the received bytes)
__device__ inline int pk_src(const PkArgs &a, uint64_t i, uint64_t &at, uint64_t &len) {
    if (a.r.tcid && (a.r.tcid[i] >> 16) != a.table) return 0;
    if (a.r.off) {
        at = a.r.off[i];
        const uint64_t e = a.r.off[i + 1];
        if (e < at || e > a.r.limit) return -1;
        len = e - at;
        return 1;
    }
    const uint64_t x = a.r.ref[i];
    if (x == a.r.none) return 0;
    at = x >> a.r.len_bits;
    len = x & ((1ULL << a.r.len_bits) - 1);
    return at + len > a.r.limit ? -1 : 1;
}

__device__ inline const uint8_t *pk_cbytes(const PkArgs &a, uint64_t j) {
    const uint64_t c = a.cref[j];
    return (c & PK_SCRATCH) ? a.scratch + (c & ~PK_SCRATCH) : a.r.base + c;
}

__device__ inline bool pk_eq(const uint8_t *x, const uint8_t *y, uint32_t n) {
    for (uint32_t k = 0; k < n; k++)
        if (x[k] != y[k]) return false;
    return true;
}

// home slot: the hash's low mixed word scaled to the table size (multiply-high); probes run linearly
// and wrap at the end
__device__ inline uint64_t pk_slot_of(uint64_t h, uint64_t nsl) {
    return ((uint64_t)(uint32_t)(h ^ (h >> 31)) * nsl) >> 32;
}
__device__ inline uint64_t pk_next(uint64_t sl, uint64_t nsl) { return sl + 1 == nsl ? 0 : sl + 1; }
__device__ inline uint32_t pk_tag(uint64_t h) { return (uint32_t)(h >> 32) | 1u; }

// A short key (<= PK_INLINE bytes) as the three words of a slot's bytes 8..31: length, then the bytes,
// zero past the length. Its byte loads are independent (predicated, all issued at once), and a key is
// then compared by three word compares instead of a loop of dependent byte loads.
struct PkWords {
    uint64_t q[3];
};
// (round 6: read as the aligned 8-B words that hold the key's bytes -- at most four loads, none of them
// past the word of the key's last byte -- instead of 23 predicated byte loads)
__device__ inline PkWords pk_words(const uint8_t *p, uint32_t cl) {
    PkWords w{};
    w.q[0] = cl;
    if (cl == 0) return w;
    const uintptr_t a = reinterpret_cast<uintptr_t>(p);
    const uint64_t *ap = reinterpret_cast<const uint64_t *>(a & ~(uintptr_t)7);
    const uint32_t sh = (uint32_t)(a & 7) * 8;
    const uint32_t nw = (uint32_t)(((a + cl - 1) >> 3) - (a >> 3)) + 1;  // (1..4 words for cl <= 23)
    uint64_t v[4];
#pragma unroll
    for (uint32_t k = 0; k < 4; k++) v[k] = k < nw ? ap[k] : 0;
    uint64_t x[3];  // bytes [8k, 8k + 8) of the key, zero past its length
#pragma unroll
    for (uint32_t k = 0; k < 3; k++) {
        uint64_t y = v[k] >> sh;
        if (sh) y |= v[k + 1] << (64 - sh);
        const uint32_t have = cl > 8 * k ? min(cl - 8 * k, 8u) : 0u;
        x[k] = have == 8 ? y : (y & ((1ULL << (8 * have)) - 1));
    }
    w.q[0] = (uint64_t)cl | (x[0] << 8);
    w.q[1] = (x[0] >> 56) | (x[1] << 8);
    w.q[2] = (x[1] >> 56) | (x[2] << 8);
    return w;
}
__device__ inline bool pk_words_eq(const PkWords &x, const PkWords &y) {
    return x.q[0] == y.q[0] && x.q[1] == y.q[1] && x.q[2] == y.q[2];
}

// One 32-B slot read with plain loads: the claim word and the three inline words. Plain loads
// are exact here: inside a probe kernel a slot's claim word only goes 0 -> claim (a stale 0 is settled
// by the CAS that follows it), and committed words were written by an earlier kernel.
__device__ inline void pk_slot_read(const PkSlot *ps, unsigned long long &w, PkWords &q) {
    // (two 16-B loads, not four 8-B ones: a probe's lanes all read different lines, and the vector
    // memory pipeline's cost is per line per load instruction -- 4 x 8-B loads made the warm intern
    // 4.5 ms even with every slot in a 32-MB, cache-resident corner of the table. A 16-B load reads its
    // line once, so the 8-B claim word in it is never seen torn.)
    const uint4 *s4 = reinterpret_cast<const uint4 *>(ps);
    const uint4 x0 = s4[0], x1 = s4[1];
    w = (unsigned long long)x0.x | ((unsigned long long)x0.y << 32);
    q.q[0] = (uint64_t)x0.z | ((uint64_t)x0.w << 32);
    q.q[1] = (uint64_t)x1.x | ((uint64_t)x1.y << 32);
    q.q[2] = (uint64_t)x1.z | ((uint64_t)x1.w << 32);
}

// First-seen order of a new key (ids in first-seen order, as cr-sqlite's __crsql_key rowids
// are assigned): while a slot is claimed its inline bytes are still zero, so its first 32-bit inline
// word holds ~(the smallest index of a change of that key), raised by atomicMax from every change that
// finds the claim (a plain read first: the word only grows, so a read at or above ~i skips the atomic).
__device__ inline uint32_t *pk_first_word(PkSlot *ps) { return reinterpret_cast<uint32_t *>(ps) + 2; }
__device__ inline void pk_first_seen(PkSlot *ps, uint32_t i) {
#if PK_DIAG & 64  // (diagnostic: no first-seen atomics from the finders, ids not first-seen)
    if (true) return;
#endif
    uint32_t *f = pk_first_word(ps);
    if (*(volatile uint32_t *)f < ~i) atomicMax(f, ~i);
}

__device__ inline uint64_t pk_wave_min64(uint64_t x) {
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint64_t y = (uint64_t)__shfl_xor((unsigned long long)x, o);
        x = y < x ? y : x;
    }
    return x;
}
__device__ inline uint64_t pk_wave_max64(uint64_t x) {
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint64_t y = (uint64_t)__shfl_xor((unsigned long long)x, o);
        x = y > x ? y : x;
    }
    return x;
}
// wave-aggregated append: one atomic per wave; every lane of the wave calls it
__device__ inline uint32_t pk_wave_append(unsigned long long *ctr, bool take) {
    const uint64_t m = __ballot(take);
    if (!m) return 0;
    const uint32_t lane = threadIdx.x & 63;
    const int leader = __ffsll((unsigned long long)m) - 1;
    uint32_t base = 0;
    if ((int)lane == leader) base = (uint32_t)atomicAdd(ctr, (unsigned long long)__popcll(m));
    base = (uint32_t)__shfl((int)base, leader);
    return base + (uint32_t)__popcll(m & ((1ULL << lane) - 1));
}

// a committed key (claim word w = tag << 32 | id, inline words q) against my canonical bytes
__device__ inline bool pk_eq_committed(const PkArgs &a, uint32_t id, const PkWords &q, const uint8_t *mine,
                                       const PkWords &mw, uint32_t cl, uint64_t h) {
    if (cl <= PK_INLINE) return pk_words_eq(mw, q);
    return a.koff[id + 1] - a.koff[id] == cl && a.khash[id] == h && pk_eq(a.kbytes + a.koff[id], mine, cl);
}

// The wave's staging window: 64 consecutive changes whose packed bytes lie within one window (the
// common case: pack_columns output back to back, or a decoded frame) are copied into LDS with 16-B
// loads along the bytes; lanes then parse from LDS. Larger windows read their bytes from HBM.
constexpr uint32_t PK_WAVE_STAGE = 2048;
#ifndef PK_GRID_MAX
// k_pk_find workgroups (grid-stride beyond): four per CU of the MI355X's 256. More waves in flight only
// queue more random slot reads in the fabric -- warm intern 3.2 ms at 1024 workgroups, 3.4 at 2048, 4.0
// at 4096, 5.3 at the former 8192, 8.3 at 16384, and 5.1 at 512 (profiles/r06_pk_grid_ab.log)
#define PK_GRID_MAX 1024
#endif
#ifndef PK_DIAG
#define PK_DIAG 0  // diagnostic builds: 1 no probe, 2 no canonical parse, 4 no LDS staging
#endif
constexpr uint32_t PK_FIND_THREADS = 256;

// k_pk_find: the fused parse + probe (round 6; it replaces a parse kernel that wrote four columns per
// change and a probe kernel that re-read them and the key bytes): per change, the canonical check, the
// route hash and the key's slot words from the staged bytes, then the probe of the table with plain
// slot loads. A held key writes its id into keys[] here -- the warm call (every key held) is this one
// kernel. A new key is claimed by one 64-bit CAS of (tag, NEW | i); the changes that find the claim
// compare against the claimant's input bytes (read-only: a claimant here always has canonical input),
// take keys[i] = PENDING | claimant and raise the claim's first-seen word. Inputs that are not
// canonical are listed for the slow path (canonicalised into a scratch, then probed).
__global__ void __launch_bounds__(PK_FIND_THREADS) k_pk_find(PkArgs a) {
    __shared__ __attribute__((aligned(16))) uint8_t s_st[PK_FIND_THREADS / 64][PK_WAVE_STAGE];
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    uint8_t *st = s_st[wv];
    const uint64_t wstride = (uint64_t)gridDim.x * (PK_FIND_THREADS / 64) * 64;
    uint32_t nbad = 0, mx = 0, nclaim = 0;  // (nclaim: wave-uniform)
    unsigned long long slowb = 0;
    const uintptr_t base = reinterpret_cast<uintptr_t>(a.r.base);
    for (uint64_t w0 = ((uint64_t)blockIdx.x * (PK_FIND_THREADS / 64) + wv) * 64; w0 < a.n; w0 += wstride) {
        const uint64_t i = w0 + lane;
        uint64_t at = 0, len = 0;
        const int src = i < a.n ? pk_src(a, i, at, len) : 0;
        const uint64_t lo = pk_wave_min64(src == 1 ? at : ~0ULL), hi = pk_wave_max64(src == 1 ? at + len : 0);
        uintptr_t a0 = 0;
        bool staged = false;
        __builtin_amdgcn_wave_barrier();  // (the previous window's LDS reads are done)
        if (lo < hi) {
            a0 = (base + lo) & ~(uintptr_t)15;
            const uintptr_t span = base + hi - a0;
            if (span <= PK_WAVE_STAGE) {
                staged = true;
                // (an aligned 16-B chunk holding one byte of the buffer lies in that byte's page)
                const uint4 *src4 = reinterpret_cast<const uint4 *>(a.r.base + (intptr_t)(a0 - base));
                for (uint32_t c = lane; (uintptr_t)c * 16 < span; c += 64)
#if PK_DIAG & 16  // (the streamed bytes non-temporal: the slot table keeps the MALL)
                {
                    typedef unsigned int v4u __attribute__((ext_vector_type(4)));
                    const v4u x = __builtin_nontemporal_load(reinterpret_cast<const v4u *>(src4) + c);
                    *reinterpret_cast<v4u *>(st + 16 * c) = x;
                }
#else
                    *reinterpret_cast<uint4 *>(st + 16 * c) = src4[c];
#endif
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        bool slow = false, claimed = false;
        uint32_t cl = 0;
        uint64_t hh = 0, sl = 0;
        if (src < 0) {
            nbad++;
            if (a.bad) a.bad[i] = 1;
        } else if (src == 1) {
#if PK_DIAG & 4
            const uint8_t *p = a.r.base + at;
#else
            const uint8_t *p = staged ? st + (base + at - a0) : a.r.base + at;
#endif
            CanonOut<false> co{p, len, nullptr};
            bool one = false;
            int64_t v = 0;
#if PK_DIAG & 2  // (diagnostic: the hash of the input bytes only, no canonical parse -- canonical inputs)
            for (uint64_t k = 0; k < len; k++) co.put(p[k]);
            const bool ok = true;
#else
            const bool ok = pk_canon_dev<false>(p, len, co, one, v) && co.o < (1ULL << 24);
#endif
            if (!ok || (!a.interned && !one)) {
                nbad++;
                if (a.bad) a.bad[i] = 1;
            } else if (!a.interned) {
                a.keys[i] = (uint64_t)v;
            } else {
                cl = (uint32_t)co.o;
                mx = max(mx, cl);
                hh = co.hash();
                if (!(co.same && co.o == len)) {
                    slow = true;
                    a.clen[i] = cl;
                    a.h[i] = hh;
                    slowb += cl;
                } else if (PK_DIAG & 1) {  // (diagnostic: no probe, results not valid)
                    a.keys[i] = hh;
                } else if (!*(volatile unsigned long long *)&a.ctl[3]) {  // (retrying: seen late is fine)
                    const uint32_t tag = pk_tag(hh);
                    PkWords mw{};
                    if (cl <= PK_INLINE) mw = pk_words(p, cl);
                    sl = pk_slot_of(hh, a.nhome);
#if PK_DIAG & 40  // (diagnostic, results not valid: ONE slot read, at the home slot (32) or inside the
                  // first 2^20 slots (8), no compare, no claim)
                    if (PK_DIAG & 8) sl = pk_slot_of(hh, min(a.nhome, (uint64_t)1 << 20));
                    {
                        unsigned long long w;
                        PkWords q;
                        pk_slot_read(a.slots + sl, w, q);
                        a.keys[i] = w ^ q.q[0] ^ mw.q[0];
                    }
                    if (true) continue;
#endif
                    uint64_t res = ~0ULL;
                    for (uint32_t step = 0; step < PK_MAX_PROBE; step++, sl = pk_next(sl, a.nsl)) {
                        PkSlot *ps = a.slots + sl;
                        unsigned long long w;
                        PkWords q;
                        pk_slot_read(ps, w, q);
                        // (a plain read that shows an empty slot may be a stale L2 line -- the claims are
                        // atomics at the memory side: read the word coherently before paying for a CAS)
#if !(PK_DIAG & 128)
                        if (w == 0) w = __hip_atomic_load(&ps->w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#endif
                        if (w == 0) {
                            const unsigned long long want = ((unsigned long long)tag << 32) | (PK_NEW | (uint32_t)i);
                            w = atomicCAS(&ps->w, 0ULL, want);
                            if (w == 0) {
                                claimed = true;
                                res = PK_PENDING | i;
                                break;
                            }
                            q = PkWords{};  // (claimed by another change meanwhile: its inline words are not read)
                        }
                        if ((uint32_t)(w >> 32) != tag) continue;
                        const uint32_t vv = (uint32_t)w;
                        if (vv & PK_NEW) {
                            const uint32_t j = vv & ~PK_NEW;
                            uint64_t jat = 0, jlen = 0;
                            bool eq = pk_src(a, j, jat, jlen) == 1 && jlen == cl;  // (a claimant's input is canonical)
                            if (eq) {
                                const uint8_t *pj = a.r.base + jat;
                                eq = cl <= PK_INLINE ? pk_words_eq(pk_words(pj, cl), mw) : pk_eq(pj, p, cl);
                            }
                            if (eq) {
                                if ((uint32_t)i < j) pk_first_seen(ps, (uint32_t)i);  // (only a change before the claimant can be first)
                                res = PK_PENDING | j;
                                break;
                            }
                        } else if (pk_eq_committed(a, vv, q, p, mw, cl, hh)) {
                            res = vv;
                            break;
                        }
                    }
                    if (res == ~0ULL) {
                        atomicOr(&a.ctl[3], 1ULL);  // (the table is too full: the call retries)
                    } else {
#if PK_DIAG & 16
                        __builtin_nontemporal_store(res, &a.keys[i]);
#else
                        a.keys[i] = res;
#endif
                    }
                }
            }
        }
        // claimants counted (one atomic per wave at the end), slow changes listed (rare)
        nclaim += (uint32_t)__popcll(__ballot(claimed));
        if (claimed) {
            a.clen[i] = cl;
            a.h[i] = hh;
            a.cref[i] = at;
            a.slotix[i] = (uint32_t)sl;
            atomicMax(pk_first_word(a.slots + sl), ~(uint32_t)i);  // (its own: always, the finders' only below it)
        }
        const uint32_t sk = pk_wave_append(&a.ctl[2], slow);
        if (slow) a.slow[sk] = (uint32_t)i;
    }
    nbad = pk_wave_sum(nbad);
    mx = pk_wave_max(mx);
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) slowb += (unsigned long long)__shfl_xor(slowb, o);
    if ((threadIdx.x & 63) == 0) {
        if (nclaim) atomicAdd(&a.ctl[4], (unsigned long long)nclaim);
        if (nbad) atomicAdd(&a.ctl[0], (unsigned long long)nbad);
        if (mx) atomicMax(&a.ctl[1], (unsigned long long)mx);
        if (slowb) atomicAdd(&a.ctl[5], slowb);
    }
}

#define PK_LIST(k, cnt) for (uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; k < (cnt); k += (uint64_t)gridDim.x * blockDim.x)

// (slow path) the listed changes' canonical bytes into the scratch
__global__ void __launch_bounds__(256) k_pk_canon(PkArgs a, uint64_t nslow) {
    PK_LIST(k, nslow) {
        const uint32_t i = a.slow[k];
        uint64_t at = 0, len = 0;
        pk_src(a, i, at, len);
        const uint64_t o = atomicAdd(&a.ctl[6], (unsigned long long)a.clen[i]);
        CanonOut<true> co{a.r.base + at, len, a.scratch + o};
        bool one = false;
        int64_t v = 0;
        pk_canon_dev<true>(a.r.base + at, len, co, one, v);
        a.cref[i] = PK_SCRATCH | o;
    }
}

// (slow path) the listed changes probe the table; every claimant's canonical bytes, length and hash were
// written by an earlier kernel, so a claim is compared through cref / clen / h
__global__ void __launch_bounds__(256) k_pk_probe_slow(PkArgs a, uint64_t nslow) {
    const uint32_t lane = threadIdx.x & 63;
    (void)lane;
    for (uint64_t k0 = (uint64_t)blockIdx.x * blockDim.x; k0 < nslow; k0 += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t k = k0 + threadIdx.x;
        bool claimed = false;
        uint32_t i = 0;
        uint64_t sl = 0;
        if (k < nslow && !*(volatile unsigned long long *)&a.ctl[3]) {
            i = a.slow[k];
            const uint32_t cl = a.clen[i];
            const uint64_t h = a.h[i];
            const uint32_t tag = pk_tag(h);
            const uint8_t *mine = pk_cbytes(a, i);
            PkWords mw{};
            if (cl <= PK_INLINE) mw = pk_words(mine, cl);
            sl = pk_slot_of(h, a.nhome);
            uint64_t res = ~0ULL;
            for (uint32_t step = 0; step < PK_MAX_PROBE; step++, sl = pk_next(sl, a.nsl)) {
                PkSlot *ps = a.slots + sl;
                unsigned long long w;
                PkWords q;
                pk_slot_read(ps, w, q);
                if (w == 0) w = __hip_atomic_load(&ps->w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (w == 0) {
                    w = atomicCAS(&ps->w, 0ULL, ((unsigned long long)tag << 32) | (PK_NEW | i));
                    if (w == 0) {
                        claimed = true;
                        res = PK_PENDING | i;
                        break;
                    }
                    q = PkWords{};
                }
                if ((uint32_t)(w >> 32) != tag) continue;
                const uint32_t vv = (uint32_t)w;
                bool eq;
                if (vv & PK_NEW) {
                    const uint32_t j = vv & ~PK_NEW;
                    eq = a.clen[j] == cl && a.h[j] == h;
                    if (eq) eq = cl <= PK_INLINE ? pk_words_eq(pk_words(pk_cbytes(a, j), cl), mw) : pk_eq(pk_cbytes(a, j), mine, cl);
                    if (eq) {
                        if (i < j) pk_first_seen(ps, i);
                        res = PK_PENDING | j;
                        break;
                    }
                } else if (pk_eq_committed(a, vv, q, mine, mw, cl, h)) {
                    res = vv;
                    break;
                }
            }
            if (res == ~0ULL)
                atomicOr(&a.ctl[3], 1ULL);
            else
                a.keys[i] = res;
        }
        const uint32_t nc = (uint32_t)__popcll(__ballot(claimed));  // (rare: the slow path's claims)
        if (nc && (threadIdx.x & 63) == (uint32_t)(__ffsll((unsigned long long)__ballot(claimed)) - 1))
            atomicAdd(&a.ctl[4], (unsigned long long)nc);
        if (claimed) {
            a.slotix[i] = (uint32_t)sl;
            atomicMax(pk_first_word(a.slots + sl), ~i);
        }
    }
}

// each claim's first-seen position gets its new-key flag and length (the scans then number the new keys
// in first-seen order)
// a change that claimed a slot for a new key (keys[c] == PENDING | c, of this table, well formed)
__device__ inline bool pk_is_claimant(const PkArgs &a, uint64_t c) {
    if (a.keys[c] != (PK_PENDING | c)) return false;
    uint64_t at = 0, len = 0;
    return pk_src(a, c, at, len) == 1 && !(a.bad && a.bad[c]);
}

__global__ void __launch_bounds__(256) k_pk_mark(PkArgs a) {
    PK_LIST(c, a.n) {
        if (!pk_is_claimant(a, c)) continue;
        const uint32_t f = ~*pk_first_word(a.slots + a.slotix[c]);
        a.firstof[c] = f;
        a.newf[f] = 1;
        a.newl[f] = a.clen[c];
    }
}

// the slot's inline words from a key's canonical bytes (zero past the length; a key longer than the
// inline bytes keeps only its length there)
__device__ inline void pk_slot_fill(PkSlot &sl, const uint8_t *src, uint32_t cl) {
    PkWords w{};
    if (cl <= PK_INLINE) {
        w = pk_words(src, cl);
    } else {
        w.q[0] = min(cl, 255u);
    }
    uint64_t *q = reinterpret_cast<uint64_t *>(&sl) + 1;
    q[0] = w.q[0];
    q[1] = w.q[1];
    q[2] = w.q[2];
}

// per claim: its id (the table size + the rank of its first-seen position), its canonical bytes, offset
// and hash appended, its slot -> the id and the key's inline words; firstof[c] becomes the id
__global__ void __launch_bounds__(256) k_pk_newkeys(PkArgs a) {
    PK_LIST(c, a.n) {
        if (!pk_is_claimant(a, c)) continue;
        const uint32_t f = a.firstof[c];
        const uint32_t id = (uint32_t)a.nkeys + a.rank[f] - 1u;
        const uint32_t cl = a.clen[c];
        const uint64_t o = a.nbytes + a.noff[f] - cl;
        const uint8_t *src = pk_cbytes(a, c);
        PkSlot &sl = a.slots[a.slotix[c]];
        if (cl <= PK_INLINE) {
            // (a short key's bytes read once as its slot words -- independent aligned loads -- then
            // stored from registers: a byte loop alternating loads and stores waited on every load)
            const PkWords w = pk_words(src, cl);
            for (uint32_t b = 0; b < cl; b++) a.kbytes[o + b] = (uint8_t)(w.q[(b + 1) >> 3] >> (8 * ((b + 1) & 7)));
            uint64_t *q = reinterpret_cast<uint64_t *>(&sl) + 1;
            q[0] = w.q[0];
            q[1] = w.q[1];
            q[2] = w.q[2];
        } else {
            for (uint32_t b = 0; b < cl; b++) a.kbytes[o + b] = src[b];
            pk_slot_fill(sl, src, cl);
        }
        a.koff[id + 1] = o + cl;
        a.khash[id] = a.h[c];
        sl.w = ((unsigned long long)pk_tag(a.h[c]) << 32) | id;
        a.firstof[c] = id;
    }
}

// every change of a new key: keys[i] = its claim's id
__global__ void __launch_bounds__(256) k_pk_commit(PkArgs a) {
    PK_LIST(i, a.n) {
        const uint64_t key = a.keys[i];
        if (!(key & PK_PENDING)) continue;
        uint64_t at = 0, len = 0;
        if (pk_src(a, i, at, len) != 1 || (a.bad && a.bad[i])) continue;  // (another table's key, or a bad pk)
        a.keys[i] = a.firstof[(uint32_t)(key & ~PK_PENDING)];
    }
}

// the slots rebuilt from the keys (a larger table, a retry after a probe overflow, or the cleanup of a
// failed call's claims)
__global__ void __launch_bounds__(256) k_pk_rehash(PkSlot *slots, uint64_t nsl, uint64_t nhome, const uint64_t *khash,
                                                   const uint64_t *koff, const uint8_t *kbytes, uint64_t nkeys) {
    for (uint64_t id = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; id < nkeys; id += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t h = khash[id];
        const unsigned long long w = ((unsigned long long)pk_tag(h) << 32) | id;
        for (uint64_t sl = pk_slot_of(h, nhome);; sl = pk_next(sl, nsl))
            if (atomicCAS(&slots[sl].w, 0ULL, w) == 0ULL) {
                pk_slot_fill(slots[sl], kbytes + koff[id], (uint32_t)(koff[id + 1] - koff[id]));
                break;
            }
    }
}

// Ordered rebuild (round 6): the keys placed in home order, each at p_i = max(h_i, p_{i-1} + 1) =
// i + max_{j <= i}(h_j - j) over the home-sorted keys -- a max-scan, then one plain store per key. A
// key's probe then passes only keys of smaller or equal home: in a table filled by concurrent claims the
// longest probe of a wave's 64 lanes runs ~10 slots at load 0.6, in home order ~5
// (tools/sim_probe_order.py), and a wave waits for its longest lane (warm intern 5.48 -> 5.07 ms).
__global__ void __launch_bounds__(256) k_pk_homes(const uint64_t *khash, uint64_t nkeys, uint64_t nhome, uint64_t *home,
                                                  uint32_t *ids) {
    PK_LIST(id, nkeys) {
        home[id] = pk_slot_of(khash[id], nhome);
        ids[id] = (uint32_t)id;
    }
}
__global__ void __launch_bounds__(256) k_pk_shift(const uint64_t *home_s, uint64_t nkeys, uint64_t *v) {
    PK_LIST(i, nkeys) v[i] = home_s[i] + nkeys - i;  // (h_i - i, biased to stay positive)
}
__global__ void __launch_bounds__(256) k_pk_place(PkSlot *slots, uint64_t nsl, const uint64_t *vmax, const uint32_t *ids,
                                                  uint64_t nkeys, const uint64_t *khash, const uint64_t *koff,
                                                  const uint8_t *kbytes, unsigned long long *past) {
    PK_LIST(i, nkeys) {
        const uint64_t p = vmax[i] - nkeys + i;
        if (p >= nsl) {  // (the pad ran out: the caller rebuilds by claims instead)
            atomicOr(past, 1ULL);
            continue;
        }
        const uint32_t id = ids[i];
        pk_slot_fill(slots[p], kbytes + koff[id], (uint32_t)(koff[id + 1] - koff[id]));
        slots[p].w = ((unsigned long long)pk_tag(khash[id]) << 32) | id;
    }
}

#undef PK_LIST

dim3 pk_grid(uint64_t n) { return dim3((uint32_t)std::max<uint64_t>(1, std::min<uint64_t>((n + 255) / 256, 16384))); }

// Slots for `keys` keys at load `num / den`, a multiple of 8 (two 128-B lines), at least 4096. The table
// is not a power of two (round 6): a config-2-sized table (4.2 M keys) at load 3/4 is 179 MB, which the
// 256-MiB MALL holds beside the call's streamed bytes, where the round-5 table (load <= 1/2 rounded up
// to 2^23 slots: 268 MB) missed to HBM on nearly every probe.
uint64_t pk_slots_for(uint64_t keys, uint64_t num, uint64_t den) {
    const uint64_t ns = (keys * den + num - 1) / num;
    return std::max<uint64_t>(4096, (ns + 7) & ~7ULL);
}

// The committed keys placed into `slots` (nsl slots, homes in the first nhome) in home order; false
// when its scratch is not available or the pad runs out (the slots are then zero again).
int pk_place_ordered(corro_ctx *ctx, const PkTable &t, PkSlot *slots, uint64_t nsl, uint64_t nhome, bool &placed) {
    placed = false;
    hipStream_t s = ctx->stream;
    const uint64_t n = t.n;
    if (n >= (1ULL << 31)) return CORRO_OK;
    uint32_t bits = 1;
    while ((1ULL << bits) < nhome) bits++;
    size_t temp = 0, t1 = 0;
    if (int rc = ovf_sort_pairs(nullptr, &temp, nullptr, nullptr, nullptr, nullptr, (uint32_t)n, bits, s)) return rc;
    if (int rc = prim_inclusive_max_u64(nullptr, &t1, nullptr, nullptr, n, s)) return rc;
    temp = std::max(temp, t1);
    auto al = [](uint64_t x) { return (x + 255) & ~255ULL; };
    const uint64_t c8 = al(n * 8), c4 = al(n * 4);
    DevBuf sc;
    if (sc.ensure(2 * c8 + 2 * c4 + 256 + al(temp)) != CORRO_OK) return CORRO_OK;  // (no room: rebuild by claims)
    uint8_t *b = sc.as<uint8_t>();
    uint64_t *ki = reinterpret_cast<uint64_t *>(b), *ko = reinterpret_cast<uint64_t *>(b + c8);
    uint32_t *vi = reinterpret_cast<uint32_t *>(b + 2 * c8), *vo = reinterpret_cast<uint32_t *>(b + 2 * c8 + c4);
    auto *past = reinterpret_cast<unsigned long long *>(b + 2 * c8 + 2 * c4);
    void *tp = b + 2 * c8 + 2 * c4 + 256;
    CORRO_HIP_TRY(hipMemsetAsync(past, 0, 8, s));
    hipLaunchKernelGGL(k_pk_homes, pk_grid(n), dim3(256), 0, s, t.d_hash.as<uint64_t>(), n, nhome, ki, vi);
    CORRO_HIP_TRY(hipGetLastError());
    size_t tb = temp;
    if (int rc = ovf_sort_pairs(tp, &tb, ki, ko, vi, vo, (uint32_t)n, bits, s)) return rc;
    hipLaunchKernelGGL(k_pk_shift, pk_grid(n), dim3(256), 0, s, ko, n, ki);
    CORRO_HIP_TRY(hipGetLastError());
    tb = temp;
    if (int rc = prim_inclusive_max_u64(tp, &tb, ki, ko, n, s)) return rc;
    hipLaunchKernelGGL(k_pk_place, pk_grid(n), dim3(256), 0, s, slots, nsl, ko, vo, n, t.d_hash.as<uint64_t>(),
                       t.d_off.as<uint64_t>(), t.d_bytes.as<uint8_t>(), past);
    CORRO_HIP_TRY(hipGetLastError());
    unsigned long long h_past = 1;
    CORRO_HIP_TRY(hipMemcpyAsync(&h_past, past, 8, hipMemcpyDeviceToHost, s));
    CORRO_HIP_TRY(hipStreamSynchronize(s));
    if (h_past) {
        CORRO_HIP_TRY(hipMemsetAsync(slots, 0, nsl * sizeof(PkSlot), s));
        return CORRO_OK;
    }
    placed = true;
    return CORRO_OK;
}

// slots for `want` keys at load <= 3/4 (at least `min_slots` homes), rebuilt from the arena
int pk_slots_resize(corro_ctx *ctx, PkTable &t, uint64_t want, uint64_t min_slots = 0) {
    const uint64_t ns = std::max<uint64_t>(pk_slots_for(want, 3, 4), (min_slots + 7) & ~7ULL);
    if (ns + PK_PAD >= (1ULL << 32)) return fail(CORRO_E_RANGE, "interned pk table past 2^31 keys");
    const uint64_t nsl = ns + PK_PAD;
    hipStream_t s = ctx->stream;
    DevBuf nb;
    if (int rc = nb.ensure(nsl * sizeof(PkSlot))) return rc;
    CORRO_HIP_TRY(hipMemsetAsync(nb.p, 0, nsl * sizeof(PkSlot), s));
    bool placed = false;
    static const bool ordered = !std::getenv("CORRO_PK_ORDERED") || std::atoi(std::getenv("CORRO_PK_ORDERED")) != 0;
    if (t.n && ordered)
        if (int rc = pk_place_ordered(ctx, t, nb.as<PkSlot>(), nsl, ns, placed)) return rc;
    if (t.n && !placed)
        hipLaunchKernelGGL(k_pk_rehash, pk_grid(t.n), dim3(256), 0, s, nb.as<PkSlot>(), nsl, ns,
                           t.d_hash.as<uint64_t>(), t.d_off.as<uint64_t>(), t.d_bytes.as<uint8_t>(), t.n);
    CORRO_HIP_TRY(hipGetLastError());
    CORRO_HIP_TRY(hipStreamSynchronize(s));
    t.d_slots.release();
    t.d_slots = nb;
    nb.p = nullptr;
    t.nslots = ns;
    return CORRO_OK;
}

// A failed call leaves claim words (tag | NEW | change) and first-seen words in the slots; the next call
// would read them as claims of its own changes. Rebuild the slots from the committed keys;
// if even that fails, drop them so the next call builds them afresh.
void pk_drop_claims(corro_ctx *ctx, PkTable &t) {
    const std::string err = corro_last_error();
    if (pk_slots_resize(ctx, t, t.n, t.nslots) != CORRO_OK) {
        (void)hipStreamSynchronize(ctx->stream);
        t.d_slots.release();
        t.nslots = 0;
    }
    set_error(err);
}

}  // namespace

int pk_keys_device(corro_ctx *ctx, uint32_t table, const PkRefs &r, uint64_t n, uint64_t *keys, uint8_t *bad,
                   uint64_t *nbad) {
    if (nbad) *nbad = 0;
    if (n == 0) return CORRO_OK;
    if (table >= ctx->tables.size()) return fail(CORRO_E_UNKNOWN_TABLE, "no such table index");
    if (n >= (1ULL << 31)) return fail(CORRO_E_RANGE, "at most 2^31 - 1 pks per call");
    if (ctx->pk.size() < ctx->tables.size()) ctx->pk.resize(ctx->tables.size());
    PkTable &t = ctx->pk[table];
    hipStream_t s = ctx->stream;
    CORRO_HIP_TRY(hipSetDevice(ctx->device));
    // per-change columns (al256 each) + counters + rocPRIM temp
    auto al = [](uint64_t x) { return (x + 255) & ~255ULL; };
    size_t temp = 0, t1 = 0;
    if (int rc = prim_inclusive_scan_u32(nullptr, &temp, nullptr, nullptr, (uint32_t)n, s)) return rc;
    if (int rc = prim_inclusive_scan_u32_u64(nullptr, &t1, nullptr, nullptr, n, s)) return rc;
    temp = std::max(temp, t1);
    const uint64_t c4 = al(n * 4), c8 = al(n * 8);
    const uint64_t need = 8 * c4 + 3 * c8 + 256 + al(temp);
    if (int rc = ctx->d_pk_scratch.ensure(need)) return rc;
    uint8_t *base = ctx->d_pk_scratch.as<uint8_t>();
    PkArgs a{};
    a.r = r;
    a.table = table;
    a.interned = t.interned ? 1u : 0u;
    a.n = n;
    a.keys = keys;
    a.bad = bad;
    uint64_t o = 0;
    auto take = [&](uint64_t b) {
        uint8_t *p = base + o;
        o += b;
        return p;
    };
    a.clen = (uint32_t *)take(c4);
    a.slotix = (uint32_t *)take(c4);
    a.firstof = (uint32_t *)take(c4);
    (void)take(c4);  // (was the claimants' list)
    a.slow = (uint32_t *)take(c4);
    a.newf = (uint32_t *)take(c4);
    a.newl = (uint32_t *)take(c4);
    a.rank = (uint32_t *)take(c4);
    a.cref = (uint64_t *)take(c8);
    a.h = (uint64_t *)take(c8);
    a.noff = (uint64_t *)take(c8);
    a.ctl = (unsigned long long *)take(256);
    void *d_temp = take(al(temp));
    if (t.interned) {
        if (t.n + n > ((uint64_t)PK_NEW - 1)) return fail(CORRO_E_RANGE, "interned pk table past 2^31 keys");
        // slots for the held keys and a share of the call's at load <= 3/4; a call that brings more new
        // keys than that overflows a probe and retries with a table four times larger (rebuilt from the
        // arena). Sized by keys, not by changes: a warm call (every key held) probes a table sized by its
        // keys. (The call's estimated new keys: a sixteenth of its changes into an empty table, a
        // sixty-fourth into one that holds keys.)
        const uint64_t est_new = std::max<uint64_t>(t.n ? n / 64 : n / 16, 1ULL << 16);
        const uint64_t want = t.n + est_new;
        if (t.nslots < pk_slots_for(want, 3, 4)) TRY_PK(pk_slots_resize(ctx, t, want));
        a.koff = t.d_off.as<uint64_t>();
        a.kbytes = t.d_bytes.as<uint8_t>();
        a.khash = t.d_hash.as<uint64_t>();
        a.nkeys = t.n;
        a.nbytes = t.nbytes;
    }
    // from the first probe on, an error return drops this call's claims from the slots
    auto failc = [&](int rc) {
        if (t.interned && t.nslots) pk_drop_claims(ctx, t);
        return rc;
    };
#define TRY_PKC(x)                            \
    do {                                      \
        int rc_ = (x);                        \
        if (rc_ != CORRO_OK) return failc(rc_); \
    } while (0)
#define HIP_PKC(x)                                                                                   \
    do {                                                                                             \
        hipError_t e_ = (x);                                                                         \
        if (e_ != hipSuccess) return failc(fail(CORRO_E_DEVICE, std::string(#x) + ": " + hipGetErrorString(e_))); \
    } while (0)
    unsigned long long ctl[8] = {};
    DevBuf scratch;  // (non-canonical inputs: their canonical bytes)
    for (int attempt = 0;; attempt++) {
        a.slots = t.d_slots.as<PkSlot>();
        a.nsl = t.nslots + PK_PAD;
        a.nhome = t.nslots;
        HIP_PKC(hipMemsetAsync(a.ctl, 0, 64, s));
        if (bad) HIP_PKC(hipMemsetAsync(bad, 0, n, s));
        const uint32_t nwaves = (uint32_t)((n + 63) / 64);
        const uint32_t grid = std::max<uint32_t>(1, std::min<uint32_t>((nwaves + 3) / 4, PK_GRID_MAX));
        if (fault_armed("pk_find")) return failc(fail(CORRO_E_DEVICE, "injected fault (CORRO_FAULT): pk_find"));
        hipLaunchKernelGGL(k_pk_find, dim3(grid), dim3(PK_FIND_THREADS), 0, s, a);
        HIP_PKC(hipGetLastError());
        HIP_PKC(hipMemcpyAsync(ctl, a.ctl, 64, hipMemcpyDeviceToHost, s));
        HIP_PKC(hipStreamSynchronize(s));
        if (nbad) *nbad = ctl[0];
        if (ctl[0] && !bad) {
            return failc(t.interned ? fail(CORRO_E_INVALID, "malformed packed primary key (unpack_columns, or bytes "
                                                            "outside the buffer)")
                                    : fail(CORRO_E_RANGE, "table " + ctx->tables[table].name +
                                                              " keys rows by one INTEGER pk (or a pk is malformed): mark "
                                                              "it interned"));
        }
        if (!t.interned) return CORRO_OK;
        t.max_len = std::max<uint64_t>(t.max_len, ctl[1]);
        if (ctl[2] && !ctl[3]) {  // slow path: non-canonical inputs canonicalised, then probed
            HIP_PKC((scratch.ensure(std::max<uint64_t>(ctl[5], 1)) == CORRO_OK) ? hipSuccess : hipErrorOutOfMemory);
            a.scratch = scratch.as<uint8_t>();
            hipLaunchKernelGGL(k_pk_canon, pk_grid(ctl[2]), dim3(256), 0, s, a, (uint64_t)ctl[2]);
            hipLaunchKernelGGL(k_pk_probe_slow, pk_grid(ctl[2]), dim3(256), 0, s, a, (uint64_t)ctl[2]);
            HIP_PKC(hipGetLastError());
            HIP_PKC(hipMemcpyAsync(ctl + 3, a.ctl + 3, 16, hipMemcpyDeviceToHost, s));
            HIP_PKC(hipStreamSynchronize(s));
        }
        if (!ctl[3]) break;
        // a probe ran long: rebuild a table four times larger from the committed keys and probe again
        if (attempt == 6) return failc(fail(CORRO_E_DEVICE, "internal: interned pk probes do not terminate"));
        TRY_PKC(pk_slots_resize(ctx, t, t.n, 4 * t.nslots));
    }
    const uint64_t nclaims = ctl[4];
    if (!nclaims) return CORRO_OK;  // (a warm call: every key held, ids already in keys[])
    HIP_PKC(hipMemsetAsync(a.newf, 0, 4 * n, s));
    HIP_PKC(hipMemsetAsync(a.newl, 0, 4 * n, s));
    hipLaunchKernelGGL(k_pk_mark, pk_grid(n), dim3(256), 0, s, a);
    HIP_PKC(hipGetLastError());
    TRY_PKC(prim_inclusive_scan_u32(d_temp, &temp, a.newf, a.rank, (uint32_t)n, s));
    TRY_PKC(prim_inclusive_scan_u32_u64(d_temp, &temp, a.newl, a.noff, n, s));
    uint32_t nnew = 0;
    uint64_t nb = 0;
    HIP_PKC(hipMemcpyAsync(&nnew, a.rank + (n - 1), 4, hipMemcpyDeviceToHost, s));
    HIP_PKC(hipMemcpyAsync(&nb, a.noff + (n - 1), 8, hipMemcpyDeviceToHost, s));
    HIP_PKC(hipStreamSynchronize(s));
    if (nnew != nclaims) return failc(fail(CORRO_E_DEVICE, "internal: interned pk claims and first-seen marks differ"));
    // room for the new keys (offsets n + 1, hashes, bytes), keeping the committed ones
    const uint64_t nk = t.n + nnew, nbytes = t.nbytes + nb;
    TRY_PKC(grow_keep(t.d_off, (nk + 1) * 8, (t.n + 1) * 8 * (t.d_off.p ? 1 : 0), s));
    TRY_PKC(grow_keep(t.d_hash, std::max<uint64_t>(nk, 1) * 8, t.n * 8, s));
    TRY_PKC(grow_keep(t.d_bytes, std::max<uint64_t>(nbytes, 1), t.nbytes, s));
    if (t.n == 0) HIP_PKC(hipMemsetAsync(t.d_off.p, 0, 8, s));
    a.koff = t.d_off.as<uint64_t>();
    a.kbytes = t.d_bytes.as<uint8_t>();
    a.khash = t.d_hash.as<uint64_t>();
    if (fault_armed("pk_commit")) return failc(fail(CORRO_E_DEVICE, "injected fault (CORRO_FAULT): pk_commit"));
    hipLaunchKernelGGL(k_pk_newkeys, pk_grid(n), dim3(256), 0, s, a);
    hipLaunchKernelGGL(k_pk_commit, pk_grid(n), dim3(256), 0, s, a);
    HIP_PKC(hipGetLastError());
    HIP_PKC(hipStreamSynchronize(s));
    t.n = nk;
    t.nbytes = nbytes;
#undef TRY_PKC
#undef HIP_PKC
    // the next call starts at load <= 0.6; a call that placed a quarter of the keys by claims leaves
    // them rebuilt in home order (sized the same way: the next call's own pre-sizing would rebuild again)
    if (4 * t.n > 3 * t.nslots || (nnew >= 65536 && 4ULL * nnew >= t.n)) TRY_PK(pk_slots_resize(ctx, t, t.n + t.n / 4));
    return CORRO_OK;
}

std::string pack_int_pk(int64_t v) {
    std::string s;
    s.push_back((char)1);
    s.push_back((char)(uint8_t)((nbytes_i64(v) << 3) | CORRO_INTEGER));
    put_int(s, v, nbytes_i64(v));
    return s;
}

}  // namespace corro

using namespace corro;

extern "C" {

int corro_pk_canonical(const uint8_t *bytes, uint64_t len, uint8_t *out, uint64_t cap, uint64_t *out_len) {
    if ((!bytes && len) || !out_len || (cap && !out)) return fail(CORRO_E_INVALID, "NULL argument");
    std::string canon;
    if (!pk_canonical(bytes, len, canon, nullptr, nullptr))
        return fail(CORRO_E_INVALID, "malformed packed primary key (unpack_columns)");
    *out_len = canon.size();
    if (canon.size() > cap) return fail(CORRO_E_RANGE, "output buffer too small");
    std::memcpy(out, canon.data(), canon.size());
    return CORRO_OK;
}

int corro_table_set_pk_interned(corro_ctx *ctx, uint32_t table, int interned) {
    if (!ctx) return fail(CORRO_E_INVALID, "NULL argument");
    if (table >= ctx->tables.size()) return fail(CORRO_E_UNKNOWN_TABLE, "no such table index");
    if (ctx->pk.size() < ctx->tables.size()) ctx->pk.resize(ctx->tables.size());
    PkTable &t = ctx->pk[table];
    if ((t.interned != (interned != 0)) && (t.n || ctx->state_total))
        return fail(CORRO_E_INVALID, "a table's pk mode is fixed once it holds rows");
    t.interned = interned != 0;
    return CORRO_OK;
}

// host pks: staged into HBM and interned there (the one intern table, pk_keys_device)
int corro_pk_keys(corro_ctx *ctx, uint32_t table, const uint8_t *bytes, const uint64_t *off, uint64_t n,
                  uint64_t *keys) {
    if (!ctx || (n && (!bytes || !off || !keys))) return fail(CORRO_E_INVALID, "NULL argument");
    if (table >= ctx->tables.size()) return fail(CORRO_E_UNKNOWN_TABLE, "no such table index");
    if (n == 0) return CORRO_OK;
    for (uint64_t i = 0; i < n; i++)
        if (off[i + 1] < off[i]) return fail(CORRO_E_INVALID, "pk offsets must not decrease");
    CORRO_HIP_TRY(hipSetDevice(ctx->device));
    const uint64_t nb = off[n] - off[0];
    DevBuf st;
    const uint64_t ob = ((n + 1) * 8 + 255) & ~255ULL, kb = (n * 8 + 255) & ~255ULL;
    if (int rc = st.ensure(ob + kb + nb + 16)) return rc;
    uint64_t *doff = st.as<uint64_t>(), *dkeys = reinterpret_cast<uint64_t *>(st.as<uint8_t>() + ob);
    uint8_t *dbytes = st.as<uint8_t>() + ob + kb;
    std::vector<uint64_t> rel(n + 1);
    for (uint64_t i = 0; i <= n; i++) rel[i] = off[i] - off[0];
    hipStream_t s = ctx->stream;
    CORRO_HIP_TRY(hipMemcpyAsync(doff, rel.data(), (n + 1) * 8, hipMemcpyHostToDevice, s));
    if (nb) CORRO_HIP_TRY(hipMemcpyAsync(dbytes, bytes + off[0], nb, hipMemcpyHostToDevice, s));
    PkRefs r;
    r.base = dbytes;
    r.off = doff;
    r.limit = nb;
    if (int rc = pk_keys_device(ctx, table, r, n, dkeys, nullptr, nullptr)) return rc;
    CORRO_HIP_TRY(hipMemcpy(keys, dkeys, n * 8, hipMemcpyDeviceToHost));
    return CORRO_OK;
}

int corro_pk_keys_device(corro_ctx *ctx, uint32_t table, const uint8_t *bytes, const uint64_t *off, uint64_t n,
                         uint64_t *keys) {
    if (!ctx || (n && (!bytes || !off || !keys))) return fail(CORRO_E_INVALID, "NULL argument");
    PkRefs r;
    r.base = bytes;
    r.off = off;
    return pk_keys_device(ctx, table, r, n, keys, nullptr, nullptr);
}

int corro_pk_bytes(corro_ctx *ctx, uint32_t table, const uint64_t *keys, uint64_t n, uint8_t *bytes, uint64_t cap,
                   uint64_t *out_off) {
    if (!ctx || (n && (!keys || !out_off)) || (cap && !bytes)) return fail(CORRO_E_INVALID, "NULL argument");
    if (table >= ctx->tables.size()) return fail(CORRO_E_UNKNOWN_TABLE, "no such table index");
    if (ctx->pk.size() < ctx->tables.size()) ctx->pk.resize(ctx->tables.size());
    const PkTable &t = ctx->pk[table];
    // (export / extraction side: the intern arrays are read back; not on the merge path)
    std::vector<uint64_t> koff;
    std::vector<uint8_t> kb;
    if (t.interned && t.n) {
        CORRO_HIP_TRY(hipSetDevice(ctx->device));
        koff.resize(t.n + 1);
        kb.resize(t.nbytes);
        CORRO_HIP_TRY(hipMemcpy(koff.data(), t.d_off.p, (t.n + 1) * 8, hipMemcpyDeviceToHost));
        if (t.nbytes) CORRO_HIP_TRY(hipMemcpy(kb.data(), t.d_bytes.p, t.nbytes, hipMemcpyDeviceToHost));
    }
    uint64_t pos = 0;
    out_off[0] = 0;
    for (uint64_t i = 0; i < n; i++) {
        std::string s;
        if (t.interned) {
            if (keys[i] >= t.n) return fail(CORRO_E_INVALID, "unknown interned row key");
            s.assign(reinterpret_cast<const char *>(kb.data() + koff[keys[i]]), koff[keys[i] + 1] - koff[keys[i]]);
        } else {
            s = pack_int_pk((int64_t)keys[i]);
        }
        if (pos + s.size() <= cap) std::memcpy(bytes + pos, s.data(), s.size());
        pos += s.size();
        out_off[i + 1] = pos;
    }
    return pos <= cap ? CORRO_OK : fail(CORRO_E_RANGE, "pk byte buffer too small (out_off[n] = the size)");
}

}  // extern "C"
