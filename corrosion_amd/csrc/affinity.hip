// SQLite column affinity (schema from /root/reference/crates/corro-types/src/schema.rs:274).
// cr-sqlite writes a winning value into the base table, which applies the column's affinity, and
// later compares the NEXT incoming value (unconverted) against that stored (converted) value. Values
// already in the class the affinity keeps -- what corrosion's own writers send, since they read their
// changes back from the base tables -- merge exactly in every body. A value the affinity WOULD
// convert makes the outcome depend on the raw-vs-converted comparison order (and, for REAL -> TEXT
// and TEXT -> REAL, on SQLite's own decimal formatting and parsing), so the engine refuses it loudly:
// the batch fails with CORRO_E_RANGE before anything is merged, instead of merging it silently wrong.
//
// Which values an affinity converts (sqlite3 applyAffinity / applyNumericAffinity):
//   TEXT            INTEGER, REAL                      -> text
//   NUMERIC/INTEGER REAL holding an integer value      -> INTEGER;  TEXT that is a numeric literal -> number
//   REAL            INTEGER                            -> REAL;     TEXT that is a numeric literal -> REAL
//   BLOB (none)     nothing
// "numeric literal" = optional whitespace, sign, digits with an optional '.', optional exponent,
// optional whitespace (sqlite3AtoF accepting the whole string); the check errs on the side of refusing.
#include <hip/hip_runtime.h>

#include <cctype>
#include <cstring>
#include <string>

#include "internal.h"
#include "merge_kernels.h"

namespace corro {

__device__ inline bool aff_space(uint32_t c) { return c == ' ' || (c >= 9 && c <= 13); }
__device__ inline bool aff_digit(uint32_t c) { return c >= '0' && c <= '9'; }

// byte k of a TEXT value of the batch (inline: big-endian in v0 / v1; long: the staged bytes)
struct TextView {
    uint64_t w0, w1;
    const uint8_t *p;  // long values
    uint64_t len;
    __device__ inline uint32_t at(uint64_t k) const {
        if (p) return p[k];
        const uint64_t w = k < 8 ? w0 : w1;
        return (uint32_t)(w >> (8 * (7 - (k & 7)))) & 0xFFu;
    }
};

__device__ inline bool numeric_literal(const TextView &t) {
    uint64_t i = 0, n = t.len;
    while (i < n && aff_space(t.at(i))) i++;
    while (n > i && aff_space(t.at(n - 1))) n--;
    if (i < n && (t.at(i) == '+' || t.at(i) == '-')) i++;
    uint64_t digits = 0;
    while (i < n && aff_digit(t.at(i))) { i++; digits++; }
    if (i < n && t.at(i) == '.') {
        i++;
        while (i < n && aff_digit(t.at(i))) { i++; digits++; }
    }
    if (digits == 0) return false;
    if (i < n && (t.at(i) == 'e' || t.at(i) == 'E')) {
        i++;
        if (i < n && (t.at(i) == '+' || t.at(i) == '-')) i++;
        uint64_t ed = 0;
        while (i < n && aff_digit(t.at(i))) { i++; ed++; }
        if (ed == 0) return false;
    }
    return i == n;
}

// REAL holding an integer value in the int64 range (-0.0 included): NUMERIC/INTEGER store it as INTEGER
__device__ inline bool real_is_integral(uint64_t bits) {
    const double x = __longlong_as_double((long long)bits);
    if (!(x == x) || x >= 9223372036854775808.0 || x < -9223372036854775808.0) return false;
    return x == trunc(x);
}

__global__ void __launch_bounds__(256) k_affinity(BatchDev in, const uint8_t *__restrict__ aff, uint32_t ntables,
                                                  unsigned long long *misc) {
    uint32_t bad = 0;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < in.n; i += gridDim.x * blockDim.x) {
        const uint32_t tc = in.tcid[i], t = tc >> 16, cid = tc & 0xFFFFu;
        if (cid == 0 || cid > MAX_COLS || t >= ntables) continue;  // sentinels carry NULL; names checked elsewhere
        const uint32_t a = aff[t * (MAX_COLS + 1) + cid];
        if (a == CORRO_AFF_BLOB) continue;
        const uint32_t ty = in.vt ? in.vt[i] : (uint32_t)CORRO_INTEGER;
        if (a == CORRO_AFF_TEXT) {
            bad |= ty == CORRO_INTEGER || ty == CORRO_REAL;
            continue;
        }
        if (a == CORRO_AFF_REAL && ty == CORRO_INTEGER) { bad = 1; continue; }
        if (a != CORRO_AFF_REAL && ty == CORRO_REAL && real_is_integral(in.v0[i])) { bad = 1; continue; }
        if (ty == CORRO_TEXT) {
            const uint32_t ln = in.vl ? in.vl[i] : 0u;
            TextView tv{in.v0[i], in.v1 ? in.v1[i] : 0ULL, nullptr, ln};
            if (ln == VLEN_LONG) {
                // a malformed span is skipped here (k_validate / k_scatter report it): the same
                // bounds long_value() checks before any byte is read
                if (!in.voff || !in.vsz || !in.arena) continue;
                const uint64_t off = in.voff[i];
                const uint32_t sz = in.vsz[i];
                if (sz <= 16 || sz >= (1u << 24) || off > in.ldata || sz > in.ldata - off) continue;
                tv.p = in.arena + in.lbase + off;
                tv.len = sz;
            }
            bad |= numeric_literal(tv);
        }
    }
    if (__any(bad != 0) && (threadIdx.x & 63) == 0) atomicOr(&misc[0], 1ULL);
}

int affinity_check(corro_ctx *ctx, const BatchDev &bd) {
    if (!ctx->aff_any || bd.n == 0) return CORRO_OK;
    hipStream_t s = ctx->stream;
    unsigned long long *flag = ctx->d_affflag.as<unsigned long long>();
    CORRO_HIP_TRY(hipMemsetAsync(flag, 0, 8, s));
    hipLaunchKernelGGL(k_affinity, dim3((uint32_t)std::min<uint64_t>((bd.n + 255) / 256, 8192)), dim3(256), 0, s, bd,
                       ctx->d_aff.as<uint8_t>(), (uint32_t)ctx->tables.size(), flag);
    CORRO_HIP_TRY(hipGetLastError());
    uint64_t h = 0;
    CORRO_HIP_TRY(hipMemcpyAsync(&h, flag, 8, hipMemcpyDeviceToHost, s));
    CORRO_HIP_TRY(hipStreamSynchronize(s));
    if (h)
        return fail(CORRO_E_RANGE, "a value is not in its column's storage class (the column affinity would convert "
                                   "it): convert it before applying");
    return CORRO_OK;
}

}  // namespace corro

using namespace corro;

extern "C" int corro_affinity_of_type(const char *decl_type) {
    // sqlite3AffinityType, in its rule order
    std::string t;
    for (const char *p = decl_type ? decl_type : ""; *p; p++) t += (char)std::toupper((unsigned char)*p);
    if (t.find("INT") != std::string::npos) return CORRO_AFF_INTEGER;
    if (t.find("CHAR") != std::string::npos || t.find("CLOB") != std::string::npos ||
        t.find("TEXT") != std::string::npos)
        return CORRO_AFF_TEXT;
    if (t.find("BLOB") != std::string::npos || t.empty()) return CORRO_AFF_BLOB;
    if (t.find("REAL") != std::string::npos || t.find("FLOA") != std::string::npos ||
        t.find("DOUB") != std::string::npos)
        return CORRO_AFF_REAL;
    return CORRO_AFF_NUMERIC;
}

extern "C" int corro_table_set_affinity(corro_ctx *ctx, uint32_t table, const uint8_t *aff, uint32_t ncols) {
    if (!ctx || (!aff && ncols)) return fail(CORRO_E_INVALID, "NULL argument");
    if (table >= ctx->tables.size()) return fail(CORRO_E_UNKNOWN_TABLE, "no such table");
    if (ncols != ctx->tables[table].cols.size()) return fail(CORRO_E_INVALID, "one affinity per column of the table");
    const size_t W = MAX_COLS + 1;
    if (ctx->aff.size() != ctx->tables.size() * W) ctx->aff.assign(ctx->tables.size() * W, (uint8_t)CORRO_AFF_BLOB);
    for (uint32_t c = 0; c < ncols; c++) {
        if (aff[c] > CORRO_AFF_REAL) return fail(CORRO_E_INVALID, "unknown affinity code");
        ctx->aff[table * W + c + 1] = aff[c];
    }
    bool any = false;
    for (uint8_t a : ctx->aff) any |= a != CORRO_AFF_BLOB;
    CORRO_HIP_TRY(hipSetDevice(ctx->device));
    if (int rc = ctx->d_aff.ensure(ctx->aff.size())) return rc;
    if (int rc = ctx->d_affflag.ensure(64)) return rc;
    CORRO_HIP_TRY(hipMemcpy(ctx->d_aff.p, ctx->aff.data(), ctx->aff.size(), hipMemcpyHostToDevice));
    ctx->aff_any = any;
    return CORRO_OK;
}
