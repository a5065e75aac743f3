// Row keys of primary keys (host side). corrosion ships a row's primary key as pack_columns bytes
// (/root/reference/crates/corro-types/src/pubsub.rs:2304-2358; unpack_columns :2396-2451); cr-sqlite
// keys its clock rows by `__crsql_key`, the rowid of the packed pk in `<t>__crsql_pks`. Here:
//   * a table whose primary key is one INTEGER column keys a row by that integer (the default);
//   * any other table (BLOB, TEXT, REAL or composite pk -- corro-tests' testsblob and wide) is
//     "interned": a row is keyed by a dense id handed out per table in first-seen order, the
//     `__crsql_pks` analogue, kept on the host next to the device state.
// pks are canonicalised before interning (unpacked and re-packed the way pack_columns packs), so
// non-canonical encodings of one key name one row, as cr-sqlite's re-packing makes them (SURVEY
// App. A.3).
#include <algorithm>
#include <cstring>
#include <string>
#include <unordered_map>
#include <vector>

#include "internal.h"

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
        PkTable &pt = ctx->pk[t];
        PkDir &d = dir[t];
        d = PkDir{};
        d.interned = pt.interned ? 1u : 0u;
        if (!pt.interned) continue;
        const uint64_t n = pt.keys.size();
        if (n > pt.dev_n) {  // append ids [dev_n, n)
            std::vector<uint64_t> off(n - pt.dev_n + 1), hs(n - pt.dev_n);
            std::string bytes;
            off[0] = pt.dev_bytes;
            for (uint64_t i = pt.dev_n; i < n; i++) {
                bytes += pt.keys[i];
                off[i - pt.dev_n + 1] = pt.dev_bytes + bytes.size();
                hs[i - pt.dev_n] = pt.hash[i];
            }
            if (int rc = grow_keep(pt.d_off, (n + 1) * 8, (pt.dev_n + 1) * 8 * (pt.dev_n ? 1 : 0), s)) return rc;
            if (int rc = grow_keep(pt.d_bytes, std::max<size_t>(pt.dev_bytes + bytes.size(), 1), pt.dev_bytes, s)) return rc;
            if (int rc = grow_keep(pt.d_hash, n * 8, pt.dev_n * 8, s)) return rc;
            CORRO_HIP_TRY(hipMemcpyAsync(pt.d_off.as<uint64_t>() + pt.dev_n, off.data(), off.size() * 8,
                                         hipMemcpyHostToDevice, s));
            if (!bytes.empty())
                CORRO_HIP_TRY(hipMemcpyAsync(pt.d_bytes.as<uint8_t>() + pt.dev_bytes, bytes.data(), bytes.size(),
                                             hipMemcpyHostToDevice, s));
            CORRO_HIP_TRY(hipMemcpyAsync(pt.d_hash.as<uint64_t>() + pt.dev_n, hs.data(), hs.size() * 8,
                                         hipMemcpyHostToDevice, s));
            pt.dev_n = n;
            pt.dev_bytes += bytes.size();
        }
        d.off = pt.d_off.as<uint64_t>();
        d.bytes = pt.d_bytes.as<uint8_t>();
        d.hash = pt.d_hash.as<uint64_t>();
        d.n = pt.dev_n;
    }
    if (int rc = ctx->d_pkdir.ensure(std::max<size_t>(dir.size(), 1) * sizeof(PkDir))) return rc;
    if (dir.empty()) dir.push_back(PkDir{});  // (no table: one zeroed entry, never an uninitialised one)
    CORRO_HIP_TRY(hipMemcpyAsync(ctx->d_pkdir.p, dir.data(), dir.size() * sizeof(PkDir), hipMemcpyHostToDevice, s));
    CORRO_HIP_TRY(hipStreamSynchronize(s));
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
    if ((t.interned != (interned != 0)) && (!t.keys.empty() || ctx->state_total))
        return fail(CORRO_E_INVALID, "a table's pk mode is fixed once it holds rows");
    t.interned = interned != 0;
    return CORRO_OK;
}

int corro_pk_keys(corro_ctx *ctx, uint32_t table, const uint8_t *bytes, const uint64_t *off, uint64_t n,
                  uint64_t *keys) {
    if (!ctx || (n && (!bytes || !off || !keys))) return fail(CORRO_E_INVALID, "NULL argument");
    if (table >= ctx->tables.size()) return fail(CORRO_E_UNKNOWN_TABLE, "no such table index");
    if (ctx->pk.size() < ctx->tables.size()) ctx->pk.resize(ctx->tables.size());
    PkTable &t = ctx->pk[table];
    std::string canon;
    for (uint64_t i = 0; i < n; i++) {
        if (off[i + 1] < off[i]) return fail(CORRO_E_INVALID, "pk offsets must not decrease");
        bool one_int = false;
        int64_t v = 0;
        if (!pk_canonical(bytes + off[i], off[i + 1] - off[i], canon, &one_int, &v))
            return fail(CORRO_E_INVALID, "malformed packed primary key (unpack_columns)");
        if (!t.interned) {
            if (!one_int) return fail(CORRO_E_RANGE, "table " + ctx->tables[table].name +
                                                         " keys rows by one INTEGER pk: mark it interned");
            keys[i] = (uint64_t)v;
            continue;
        }
        auto it = t.ids.find(canon);
        if (it == t.ids.end()) {
            const uint64_t id = t.keys.size();
            it = t.ids.emplace(canon, id).first;
            t.keys.push_back(canon);
            t.hash.push_back(pk_route_hash(canon));
            t.max_len = std::max<uint64_t>(t.max_len, canon.size());
        }
        keys[i] = it->second;
    }
    return CORRO_OK;
}

int corro_pk_bytes(corro_ctx *ctx, uint32_t table, const uint64_t *keys, uint64_t n, uint8_t *bytes, uint64_t cap,
                   uint64_t *out_off) {
    if (!ctx || (n && (!keys || !out_off)) || (cap && !bytes)) return fail(CORRO_E_INVALID, "NULL argument");
    if (table >= ctx->tables.size()) return fail(CORRO_E_UNKNOWN_TABLE, "no such table index");
    if (ctx->pk.size() < ctx->tables.size()) ctx->pk.resize(ctx->tables.size());
    const PkTable &t = ctx->pk[table];
    uint64_t pos = 0;
    out_off[0] = 0;
    for (uint64_t i = 0; i < n; i++) {
        std::string s;
        if (t.interned) {
            if (keys[i] >= t.keys.size()) return fail(CORRO_E_INVALID, "unknown interned row key");
            s = t.keys[keys[i]];
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
