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
// Device intern (pk_keys_device), per table, over the changes that reference packed bytes:
//   k_pk_parse   unpack_columns + pack_columns restated per change without writing: canonical length,
//                route hash of the canonical bytes (pk_route_hash), whether the input already is
//                canonical (the common case: pack_columns output), the value of a one-INTEGER pk
//   [k_pk_canon] only when some input is not canonical: its canonical bytes into a scratch (scan of
//                their lengths), the change's reference redirected there
//   k_pk_probe   each change probes the table's slots by its hash: a slot whose tag matches names an
//                existing id (bytes compared with the arena) or another change's claim of a new key
//                (bytes compared with that change's canonical bytes); an empty slot is claimed with
//                one 64-bit CAS of (tag, NEW | change). No change waits for another: a claim carries
//                everything a later prober compares against.
//   scans        claims -> new ids (table size + rank), their bytes -> arena offsets
//   k_pk_commit  keys; each claim's canonical bytes, offset and hash appended, its slot -> the id
// The slots (32 B: claim word, length, up to 23 canonical bytes inline) are sized by the keys the
// table holds (load <= 1/2 with a share of new ones), not by the changes of a call; a probe that runs
// past PK_MAX_PROBE slots marks the call for a retry with a table four times larger (rebuilt from the
// arena).
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

struct PkArgs {
    PkRefs r;
    uint32_t table;
    uint32_t interned;
    uint64_t n;
    uint64_t *keys;
    uint8_t *bad;
    // per change
    uint32_t *clen;     // canonical length (0: no reference of this table, or malformed)
    uint64_t *cref;     // where its canonical bytes are: input offset, or PK_SCRATCH | scratch offset
    uint64_t *h;        // route hash
    uint32_t *ncl;      // (non-canonical inputs) canonical length, for the scratch scan
    uint64_t *nclo;     // inclusive scan of ncl
    uint8_t *scratch;
    uint32_t *owner;    // id, or PK_NEW | claimant
    uint32_t *slotix;   // a claimant's slot
    uint32_t *newf;     // 1: a claimant (a new key)
    uint32_t *newl;     // a claimant's canonical length
    uint32_t *rank;     // inclusive scan of newf
    uint64_t *noff;     // inclusive scan of newl
    unsigned long long *ctl;  // [0] bad [1] max canonical length [2] non-canonical inputs [3] probe overflow
    // the table
    PkSlot *slots;
    uint64_t smask;
    uint64_t *koff;
    uint8_t *kbytes;
    uint64_t *khash;
    uint64_t nkeys, nbytes;
};

__device__ inline bool pk_src(const PkArgs &a, uint64_t i, const uint8_t *&p, uint64_t &len) {
    if (a.r.tcid && (a.r.tcid[i] >> 16) != a.table) return false;
    if (a.r.off) {
        p = a.r.base + a.r.off[i];
        len = a.r.off[i + 1] - a.r.off[i];
        return true;
    }
    const uint64_t x = a.r.ref[i];
    if (x == a.r.none) return false;
    p = a.r.base + (x >> a.r.len_bits);
    len = x & ((1ULL << a.r.len_bits) - 1);
    return true;
}

__device__ inline const uint8_t *pk_cbytes(const PkArgs &a, uint64_t j) {
    const uint64_t c = a.cref[j];
    return (c & PK_SCRATCH) ? a.scratch + (c & ~PK_SCRATCH) : a.r.base + c;
}

#define PK_LOOP(i) for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < a.n; i += (uint64_t)gridDim.x * blockDim.x)

// A pk of at most PK_STAGE bytes is parsed from a copy in LDS: the parse reads its bytes in a data-
// dependent order (column types, then lengths), which from HBM is a chain of dependent loads per byte
// (2.1 ms for config 2's 2^26 pks); the copy's loads are independent and issue at once.
constexpr uint32_t PK_STAGE = 32;

__global__ void __launch_bounds__(256) k_pk_parse(PkArgs a) {
    __shared__ __attribute__((aligned(16))) uint8_t s_pk[256 * PK_STAGE];
    uint8_t *mine_lds = s_pk + threadIdx.x * PK_STAGE;
    uint32_t nbad = 0, mx = 0, nnc = 0;
    PK_LOOP(i) {
        const uint8_t *p = nullptr;
        uint64_t len = 0;
        uint32_t cl = 0, nc = 0;
        if (pk_src(a, i, p, len)) {
            const uint8_t *q = p;
            if (len <= PK_STAGE) {
                uint8_t b[PK_STAGE];
#pragma unroll
                for (uint32_t k = 0; k < PK_STAGE; k++) b[k] = k < len ? p[k] : 0;
                uint32_t *w = reinterpret_cast<uint32_t *>(mine_lds);
#pragma unroll
                for (uint32_t k = 0; k < PK_STAGE / 4; k++)
                    w[k] = (uint32_t)b[4 * k] | ((uint32_t)b[4 * k + 1] << 8) | ((uint32_t)b[4 * k + 2] << 16) |
                           ((uint32_t)b[4 * k + 3] << 24);
                q = mine_lds;
            }
            CanonOut<false> co{q, len, nullptr};
            bool one = false;
            int64_t v = 0;
            const bool ok = pk_canon_dev<false>(q, len, co, one, v) && co.o < (1ULL << 24);
            if (!ok || (!a.interned && !one)) {
                nbad++;
                if (a.bad) a.bad[i] = 1;
            } else if (!a.interned) {
                a.keys[i] = (uint64_t)v;
            } else {
                cl = (uint32_t)co.o;
                mx = max(mx, cl);
                a.h[i] = co.hash();
                const bool canon = co.same && co.o == len;
                a.cref[i] = canon ? (uint64_t)(p - a.r.base) : PK_SCRATCH;
                if (!canon) {
                    nc = cl;
                    nnc++;
                }
            }
        }
        a.clen[i] = cl;
        a.ncl[i] = nc;
    }
    nbad = pk_wave_sum(nbad);
    nnc = pk_wave_sum(nnc);
    mx = pk_wave_max(mx);
    if ((threadIdx.x & 63) == 0) {
        if (nbad) atomicAdd(&a.ctl[0], (unsigned long long)nbad);
        if (mx) atomicMax(&a.ctl[1], (unsigned long long)mx);
        if (nnc) atomicAdd(&a.ctl[2], (unsigned long long)nnc);
    }
}

// (non-canonical inputs only) their canonical bytes into the scratch at the scan of their lengths
__global__ void __launch_bounds__(256) k_pk_canon(PkArgs a) {
    PK_LOOP(i) {
        if (!a.ncl[i]) continue;
        const uint8_t *p = nullptr;
        uint64_t len = 0;
        pk_src(a, i, p, len);
        const uint64_t o = a.nclo[i] - a.ncl[i];
        CanonOut<true> co{p, len, a.scratch + o};
        bool one = false;
        int64_t v = 0;
        pk_canon_dev<true>(p, len, co, one, v);
        a.cref[i] = PK_SCRATCH | o;
    }
}

__device__ inline bool pk_eq(const uint8_t *x, const uint8_t *y, uint32_t n) {
    for (uint32_t k = 0; k < n; k++)
        if (x[k] != y[k]) return false;
    return true;
}

__device__ inline uint64_t pk_slot_of(uint64_t h, uint64_t mask) { return (h ^ (h >> 31)) & mask; }
__device__ inline uint32_t pk_tag(uint64_t h) { return (uint32_t)(h >> 32) | 1u; }

// A short key (<= PK_INLINE bytes) as the three words of a slot's bytes 8..31: length, then the bytes,
// zero past the length. Its byte loads are independent (predicated, all issued at once), and a key is
// then compared by three word compares instead of a loop of dependent byte loads.
struct PkWords {
    uint64_t q[3];
};
__device__ inline PkWords pk_words(const uint8_t *p, uint32_t cl) {
    uint8_t b[PK_INLINE];
#pragma unroll
    for (uint32_t k = 0; k < PK_INLINE; k++) b[k] = k < cl ? p[k] : 0;
    PkWords w;
    w.q[0] = cl;
#pragma unroll
    for (uint32_t k = 0; k < 7; k++) w.q[0] |= (uint64_t)b[k] << (8 * (k + 1));
    w.q[1] = w.q[2] = 0;
#pragma unroll
    for (uint32_t k = 0; k < 8; k++) {
        w.q[1] |= (uint64_t)b[7 + k] << (8 * k);
        w.q[2] |= (uint64_t)b[15 + k] << (8 * k);
    }
    return w;
}
__device__ inline bool pk_words_eq(const PkWords &x, const PkSlot *ps) {
    const uint64_t *q = reinterpret_cast<const uint64_t *>(ps) + 1;  // (bytes 8..31: len, b[0..22])
    return q[0] == x.q[0] && q[1] == x.q[1] && q[2] == x.q[2];
}

// a committed key against my canonical bytes: inline in the slot (the line the claim word is on) or in
// the arena
__device__ inline bool pk_eq_slot(const PkArgs &a, const PkSlot *ps, uint32_t id, const uint8_t *mine, const PkWords &mw,
                                  uint32_t cl, uint64_t h) {
    if (cl <= PK_INLINE) return pk_words_eq(mw, ps);
    return a.koff[id + 1] - a.koff[id] == cl && a.khash[id] == h && pk_eq(a.kbytes + a.koff[id], mine, cl);
}

__global__ void __launch_bounds__(256) k_pk_probe(PkArgs a) {
    PK_LOOP(i) {
        a.newf[i] = 0;
        a.newl[i] = 0;
        const uint32_t cl = a.clen[i];
        if (!cl) continue;
        if (*(volatile unsigned long long *)&a.ctl[3]) continue;  // (retrying: a cached read, seen late is fine)
        const uint64_t h = a.h[i];
        const uint32_t tag = pk_tag(h);
        const uint8_t *mine = pk_cbytes(a, i);
        PkWords mw{};
        if (cl <= PK_INLINE) mw = pk_words(mine, cl);
        uint64_t sl = pk_slot_of(h, a.smask);
        uint32_t owner = ~0u;
        for (uint32_t step = 0; step < PK_MAX_PROBE; step++, sl = (sl + 1) & a.smask) {
            PkSlot *ps = a.slots + sl;
            unsigned long long w = __hip_atomic_load(&ps->w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (w == 0) {
                const unsigned long long want = ((unsigned long long)tag << 32) | (PK_NEW | (uint32_t)i);
                w = atomicCAS(&ps->w, 0ULL, want);
                if (w == 0) {  // claimed: a new key, its canonical bytes already where cref says
                    owner = PK_NEW | (uint32_t)i;
                    a.slotix[i] = (uint32_t)sl;
                    a.newf[i] = 1;
                    a.newl[i] = cl;
                    break;
                }
            }
            if ((uint32_t)(w >> 32) != tag) continue;
            const uint32_t v = (uint32_t)w;
            bool eq;
            if (v & PK_NEW) {
                const uint32_t j = v & ~PK_NEW;
                eq = a.clen[j] == cl && a.h[j] == h;
                if (eq && cl <= PK_INLINE) {
                    const PkWords jw = pk_words(pk_cbytes(a, j), cl);
                    eq = jw.q[0] == mw.q[0] && jw.q[1] == mw.q[1] && jw.q[2] == mw.q[2];
                } else if (eq) {
                    eq = pk_eq(pk_cbytes(a, j), mine, cl);
                }
            } else {
                eq = pk_eq_slot(a, ps, v, mine, mw, cl, h);  // (committed by an earlier kernel: plain loads)
            }
            if (eq) {
                owner = v;
                break;
            }
        }
        if (owner == ~0u) atomicOr(&a.ctl[3], 1ULL);  // (the table is too full: the call retries)
        a.owner[i] = owner;
    }
}

__device__ inline void pk_slot_fill(PkSlot &sl, const uint8_t *src, uint32_t cl) {
    sl.len = (uint8_t)min(cl, 255u);
    if (cl <= PK_INLINE)
        for (uint32_t k = 0; k < cl; k++) sl.b[k] = src[k];
}

__global__ void __launch_bounds__(256) k_pk_commit(PkArgs a) {
    PK_LOOP(i) {
        const uint32_t cl = a.clen[i];
        if (!cl) continue;
        const uint32_t o = a.owner[i];
        const uint32_t id = (o & PK_NEW) ? (uint32_t)a.nkeys + a.rank[o & ~PK_NEW] - 1u : o;
        a.keys[i] = id;
        if (!a.newf[i]) continue;
        const uint64_t at = a.nbytes + a.noff[i] - cl;
        const uint8_t *src = pk_cbytes(a, i);
        for (uint32_t k = 0; k < cl; k++) a.kbytes[at + k] = src[k];
        a.koff[id + 1] = at + cl;
        a.khash[id] = a.h[i];
        PkSlot &sl = a.slots[a.slotix[i]];
        pk_slot_fill(sl, src, cl);
        sl.w = ((unsigned long long)pk_tag(a.h[i]) << 32) | id;
    }
}

// the slots rebuilt from the keys (a larger table, or a retry after a probe overflow)
__global__ void __launch_bounds__(256) k_pk_rehash(PkSlot *slots, uint64_t mask, const uint64_t *khash,
                                                   const uint64_t *koff, const uint8_t *kbytes, uint64_t nkeys) {
    for (uint64_t id = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; id < nkeys; id += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t h = khash[id];
        const unsigned long long w = ((unsigned long long)pk_tag(h) << 32) | id;
        for (uint64_t sl = pk_slot_of(h, mask);; sl = (sl + 1) & mask)
            if (atomicCAS(&slots[sl].w, 0ULL, w) == 0ULL) {
                pk_slot_fill(slots[sl], kbytes + koff[id], (uint32_t)(koff[id + 1] - koff[id]));
                break;
            }
    }
}

#undef PK_LOOP

dim3 pk_grid(uint64_t n) { return dim3((uint32_t)std::max<uint64_t>(1, std::min<uint64_t>((n + 255) / 256, 16384))); }

// slots for `want` keys at load <= 1/2 (at least `min_slots`), rebuilt from the arena
int pk_slots_resize(corro_ctx *ctx, PkTable &t, uint64_t want, uint64_t min_slots = 0) {
    uint64_t ns = 1ULL << 12;
    while (ns < 2 * want || ns < min_slots) ns <<= 1;
    if (ns >= (1ULL << 32)) return fail(CORRO_E_RANGE, "interned pk table past 2^31 keys");
    hipStream_t s = ctx->stream;
    DevBuf nb;
    if (int rc = nb.ensure(ns * sizeof(PkSlot))) return rc;
    CORRO_HIP_TRY(hipMemsetAsync(nb.p, 0, ns * sizeof(PkSlot), s));
    if (t.n) hipLaunchKernelGGL(k_pk_rehash, pk_grid(t.n), dim3(256), 0, s, nb.as<PkSlot>(), ns - 1,
                                t.d_hash.as<uint64_t>(), t.d_off.as<uint64_t>(), t.d_bytes.as<uint8_t>(), t.n);
    CORRO_HIP_TRY(hipGetLastError());
    CORRO_HIP_TRY(hipStreamSynchronize(s));
    t.d_slots.release();
    t.d_slots = nb;
    nb.p = nullptr;
    t.nslots = ns;
    return CORRO_OK;
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
    const uint64_t need = 7 * c4 + 4 * c8 + 256 + al(temp);
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
    a.ncl = (uint32_t *)take(c4);
    a.owner = (uint32_t *)take(c4);
    a.slotix = (uint32_t *)take(c4);
    a.newf = (uint32_t *)take(c4);
    a.newl = (uint32_t *)take(c4);
    a.rank = (uint32_t *)take(c4);
    a.cref = (uint64_t *)take(c8);
    a.h = (uint64_t *)take(c8);
    a.nclo = (uint64_t *)take(c8);
    a.noff = (uint64_t *)take(c8);
    a.ctl = (unsigned long long *)take(256);
    void *d_temp = take(al(temp));
    CORRO_HIP_TRY(hipMemsetAsync(a.ctl, 0, 64, s));
    if (bad) CORRO_HIP_TRY(hipMemsetAsync(bad, 0, n, s));
    hipLaunchKernelGGL(k_pk_parse, pk_grid(n), dim3(256), 0, s, a);
    CORRO_HIP_TRY(hipGetLastError());
    unsigned long long ctl[4] = {0, 0, 0, 0};
    CORRO_HIP_TRY(hipMemcpyAsync(ctl, a.ctl, 32, hipMemcpyDeviceToHost, s));
    CORRO_HIP_TRY(hipStreamSynchronize(s));
    if (nbad) *nbad = ctl[0];
    if (ctl[0] && !bad) {
        return t.interned ? fail(CORRO_E_INVALID, "malformed packed primary key (unpack_columns)")
                          : fail(CORRO_E_RANGE, "table " + ctx->tables[table].name +
                                                    " keys rows by one INTEGER pk (or a pk is malformed): mark it interned");
    }
    if (!t.interned) return CORRO_OK;
    t.max_len = std::max<uint64_t>(t.max_len, ctl[1]);
    DevBuf scratch;  // (non-canonical inputs: their canonical bytes)
    if (ctl[2]) {
        TRY_PK(prim_inclusive_scan_u32_u64(d_temp, &temp, a.ncl, a.nclo, n, s));
        uint64_t tot = 0;
        CORRO_HIP_TRY(hipMemcpyAsync(&tot, a.nclo + (n - 1), 8, hipMemcpyDeviceToHost, s));
        CORRO_HIP_TRY(hipStreamSynchronize(s));
        if (int rc = scratch.ensure(std::max<uint64_t>(tot, 1))) return rc;
        a.scratch = scratch.as<uint8_t>();
        hipLaunchKernelGGL(k_pk_canon, pk_grid(n), dim3(256), 0, s, a);
        CORRO_HIP_TRY(hipGetLastError());
    }
    if (t.n + n > ((uint64_t)PK_NEW - 1)) return fail(CORRO_E_RANGE, "interned pk table past 2^31 keys");
    // slots for the held keys and a share of the call's (load <= 1/2); a call that brings more new keys
    // than that overflows a probe and retries with a table four times larger (rebuilt from the arena).
    // Sized by keys, not by changes: a warm call (every key held) probes a table that stays in the MALL.
    // (load <= 1/2 for the held keys, <= 3/4 with the call's estimated new keys: a sixteenth of its
    // changes into an empty table, a sixty-fourth into one that holds keys)
    const uint64_t est_new = std::max<uint64_t>(t.n ? n / 64 : n / 16, 1ULL << 16);
    const uint64_t want = std::max<uint64_t>(t.n, (t.n + est_new) * 2 / 3);
    if (t.nslots < 2 * want) TRY_PK(pk_slots_resize(ctx, t, want));
    a.slots = t.d_slots.as<PkSlot>();
    a.smask = t.nslots - 1;
    a.koff = t.d_off.as<uint64_t>();
    a.kbytes = t.d_bytes.as<uint8_t>();
    a.khash = t.d_hash.as<uint64_t>();
    a.nkeys = t.n;
    a.nbytes = t.nbytes;
    for (int attempt = 0;; attempt++) {
        hipLaunchKernelGGL(k_pk_probe, pk_grid(n), dim3(256), 0, s, a);
        CORRO_HIP_TRY(hipGetLastError());
        CORRO_HIP_TRY(hipMemcpyAsync(&ctl[3], a.ctl + 3, 8, hipMemcpyDeviceToHost, s));
        CORRO_HIP_TRY(hipStreamSynchronize(s));
        if (!ctl[3]) break;
        // a probe ran long: rebuild a table four times larger from the committed keys and probe again
        if (attempt == 6) return fail(CORRO_E_DEVICE, "internal: interned pk probes do not terminate");
        TRY_PK(pk_slots_resize(ctx, t, t.n, 4 * t.nslots));
        a.slots = t.d_slots.as<PkSlot>();
        a.smask = t.nslots - 1;
        CORRO_HIP_TRY(hipMemsetAsync(a.ctl + 3, 0, 8, s));
    }
    TRY_PK(prim_inclusive_scan_u32(d_temp, &temp, a.newf, a.rank, (uint32_t)n, s));
    uint32_t nnew = 0;
    uint64_t nb = 0;
    CORRO_HIP_TRY(hipMemcpyAsync(&nnew, a.rank + (n - 1), 4, hipMemcpyDeviceToHost, s));
    CORRO_HIP_TRY(hipStreamSynchronize(s));
    if (nnew) {  // (a warm call -- every key held -- needs no byte offsets)
        TRY_PK(prim_inclusive_scan_u32_u64(d_temp, &temp, a.newl, a.noff, n, s));
        CORRO_HIP_TRY(hipMemcpyAsync(&nb, a.noff + (n - 1), 8, hipMemcpyDeviceToHost, s));
        CORRO_HIP_TRY(hipStreamSynchronize(s));
    }
    // room for the new keys (offsets n + 1, hashes, bytes), keeping the committed ones
    const uint64_t nk = t.n + nnew, nbytes = t.nbytes + nb;
    if (int rc = grow_keep(t.d_off, (nk + 1) * 8, (t.n + 1) * 8 * (t.d_off.p ? 1 : 0), s)) return rc;
    if (int rc = grow_keep(t.d_hash, std::max<uint64_t>(nk, 1) * 8, t.n * 8, s)) return rc;
    if (int rc = grow_keep(t.d_bytes, std::max<uint64_t>(nbytes, 1), t.nbytes, s)) return rc;
    if (t.n == 0) CORRO_HIP_TRY(hipMemsetAsync(t.d_off.p, 0, 8, s));
    a.koff = t.d_off.as<uint64_t>();
    a.kbytes = t.d_bytes.as<uint8_t>();
    a.khash = t.d_hash.as<uint64_t>();
    hipLaunchKernelGGL(k_pk_commit, pk_grid(n), dim3(256), 0, s, a);
    CORRO_HIP_TRY(hipGetLastError());
    CORRO_HIP_TRY(hipStreamSynchronize(s));
    t.n = nk;
    t.nbytes = nbytes;
    if (2 * t.n > t.nslots) TRY_PK(pk_slots_resize(ctx, t, 2 * t.n));  // (the next call starts at load <= 1/4)
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
