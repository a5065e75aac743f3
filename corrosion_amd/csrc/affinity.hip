// SQLite column affinity (schema from /root/reference/crates/corro-types/src/schema.rs:274).
// cr-sqlite writes a winning value into the base table, which applies the column's affinity, and
// compares the NEXT incoming value (unconverted) against that stored (converted) value. The engine
// does the same: before a batch is staged, k_aff_convert gives every change whose column affinity
// converts its value the converted (stored) value; the staged record carries it, the change's
// bucket takes the sequential general body, and there an incoming change is compared by its raw
// value (MergeArgs::raw) against the stored one.
//
// The conversion is SQLite 3.37.2's (applyAffinity / applyNumericAffinity / sqlite3AtoF /
// sqlite3VdbeIntegerAffinity, and "%!.15g" for REAL -> TEXT), which scales decimals in x87 80-bit
// long double: those operations are emulated here (X87: 64-bit significand, round to nearest even)
// so the results are SQLite's bit for bit. The oracle (oracle/affinity.c) restates the same
// algorithm with the host's long double and is pinned against the stdlib sqlite3
// (tests/test_affinity_oracle.py); tests/test_gpu_affinity.py checks this code against it.
//
//   TEXT            INTEGER -> decimal text; REAL -> "%!.15g" text
//   NUMERIC/INTEGER REAL holding an integer in (-2^63, 2^63) -> INTEGER; numeric TEXT -> INTEGER/REAL
//   REAL            as NUMERIC, then an INTEGER result is read back as REAL
//   BLOB (none)     nothing; NULL and BLOB values are never converted
//
// Version gap: the reference bundles SQLite through libsqlite3-sys 0.31.0
// (Cargo.lock:2444), a newer SQLite than the 3.37.2 this image holds and the fixtures pin. Newer
// SQLite rewrote sqlite3AtoF and the REAL -> TEXT rendering, so a conversion whose result hinges on
// 3.37.2's long-double rounding is not known to match the reference's base table. The default
// policy (CORRO_AFF_POLICY_SQLITE_3_37_2) converts every value as 3.37.2 does -- SQLite never
// refuses a change, and a refused batch would stall an actor's sync for good -- and counts such
// version-sensitive conversions (corro_metrics.aff_sensitive). The strict opt-in policy
// (CORRO_AFF_POLICY_PORTABLE) converts only what any correctly rounded implementation of these
// routines stores identically, and refuses the rest (CORRO_E_RANGE, before any write):
//   TEXT -> REAL   refused when a nonzero digit past the 19th is dropped, when the result
//                  overflows / is subnormal / takes the e > 307 double-scaling path, or when the
//                  long-double value lies within a margin of the double rounding midpoint (1 unit
//                  of 2^-64 when 10^e is exact, e <= 27; 32 otherwise -- above 3.37.2's scaling
//                  error, so outside it both 3.37.2 and a correctly rounded conversion pick the
//                  same double);
//   REAL -> TEXT   refused unless the "%!.15g" text converts back to the same double (then the
//                  15-digit rendering is far from a rounding tie and equals the shortest
//                  round-trip form as well), and for -0.0 (3.37.2 writes "0.0").
// Integer text, INTEGER -> TEXT / REAL and REAL -> INTEGER are exact and always converted.
// CORRO_AFF_POLICY_SQLITE_3_37_2 converts everything bit for bit as 3.37.2 does (the fixtures).
// The sensitive count is taken in the counting pass either way (one word per wave).
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

// ---- 128-bit helpers and the x87 extended format (value = m * 2^e, m normalised, 0 = zero) ----
struct U128 {
    uint64_t hi, lo;
};
__device__ inline U128 u_shl(U128 a, int k) {
    if (k == 0) return a;
    if (k >= 128) return {0, 0};
    if (k >= 64) return {a.lo << (k - 64), 0};
    return {(a.hi << k) | (a.lo >> (64 - k)), a.lo << k};
}
// shift right; *lost |= the bits shifted out
__device__ inline U128 u_shr(U128 a, int k, bool *lost) {
    if (k == 0) return a;
    if (k >= 128) {
        *lost |= (a.hi | a.lo) != 0;
        return {0, 0};
    }
    if (k >= 64) {
        *lost |= a.lo != 0 || (k > 64 && (a.hi << (128 - k)) != 0);
        return {0, a.hi >> (k - 64)};
    }
    *lost |= (a.lo << (64 - k)) != 0;
    return {a.hi >> k, (a.lo >> k) | (a.hi << (64 - k))};
}
__device__ inline U128 u_add(U128 a, U128 b) {
    const uint64_t lo = a.lo + b.lo;
    return {a.hi + b.hi + (lo < a.lo ? 1 : 0), lo};
}
__device__ inline U128 u_sub(U128 a, U128 b) {
    return {a.hi - b.hi - (a.lo < b.lo ? 1 : 0), a.lo - b.lo};
}
__device__ inline bool u_ge(U128 a, U128 b) { return a.hi != b.hi ? a.hi > b.hi : a.lo >= b.lo; }
__device__ inline int u_clz(U128 a) { return a.hi ? __clzll(a.hi) : 64 + (a.lo ? __clzll(a.lo) : 64); }

struct X87 {
    uint64_t m;
    int e;
};

// w * 2^e (+ a nonzero tail below w's last bit when sticky) rounded to 64 bits, nearest-even
__device__ inline X87 x_round(U128 w, int e, bool sticky) {
    if (!w.hi && !w.lo) return {0, 0};
    const int lz = u_clz(w);
    w = u_shl(w, lz);
    e -= lz;
    uint64_t hi = w.hi;
    const bool rb = (w.lo >> 63) != 0, st = sticky || (w.lo << 1) != 0;
    e += 64;
    if (rb && (st || (hi & 1))) {
        hi++;
        if (hi == 0) {
            hi = 1ULL << 63;
            e++;
        }
    }
    return {hi, e};
}
__device__ inline X87 x_u64(uint64_t u) { return x_round({0, u}, 0, false); }
__device__ inline X87 x_dbl(double d) {  // d >= 0, finite: exact
    const uint64_t b = (uint64_t)__double_as_longlong(d);
    const uint32_t ex = (uint32_t)(b >> 52) & 0x7FF;
    const uint64_t f = b & 0xFFFFFFFFFFFFFULL;
    if (ex == 0) return x_round({0, f}, -1074, false);
    return x_round({0, f | (1ULL << 52)}, (int)ex - 1075, false);
}
__device__ inline X87 x_mul(X87 a, X87 b) {
    if (!a.m || !b.m) return {0, 0};
    return x_round({__umul64hi(a.m, b.m), a.m * b.m}, a.e + b.e, false);
}
__device__ inline X87 x_div(X87 a, X87 b) {  // b != 0
    if (!a.m) return {0, 0};
    U128 r{0, a.m}, q{0, 0};
    const U128 d{0, b.m};
    for (int k = 0; k < 66; k++) {  // q = floor(a.m * 2^65 / b.m)
        q = u_shl(q, 1);
        if (u_ge(r, d)) {
            r = u_sub(r, d);
            q.lo |= 1;
        }
        r = u_shl(r, 1);
    }
    return x_round(q, a.e - b.e - 65, r.hi || r.lo);
}
__device__ inline int x_cmp(X87 a, X87 b) {
    if (!a.m || !b.m) return a.m ? 1 : (b.m ? -1 : 0);
    const int ea = a.e + 63, eb = b.e + 63;  // exponent of the top bit
    if (ea != eb) return ea > eb ? 1 : -1;
    return a.m == b.m ? 0 : (a.m > b.m ? 1 : -1);
}
__device__ inline X87 x_add(X87 a, X87 b) {  // a, b >= 0
    if (x_cmp(a, b) < 0) {
        const X87 t = a;
        a = b;
        b = t;
    }
    if (!b.m) return a;
    bool lost = false;
    const U128 A = u_shl({0, a.m}, 63), B = u_shr(u_shl({0, b.m}, 63), a.e - b.e, &lost);
    return x_round(u_add(A, B), a.e - 63, lost);
}
__device__ inline X87 x_sub(X87 a, X87 b) {  // a >= b >= 0
    if (!b.m) return a;
    bool lost = false;
    const U128 A = u_shl({0, a.m}, 63);
    U128 B = u_shr(u_shl({0, b.m}, 63), a.e - b.e, &lost);
    if (lost) B = u_add(B, {0, 1});  // true difference lies in (A - B - 1, A - B): round from below, sticky
    return x_round(u_sub(A, B), a.e - 63, lost);
}
__device__ inline uint64_t x_trunc(X87 a) {  // a < 2^64
    if (!a.m || a.e <= -64) return 0;
    return a.e >= 0 ? a.m << a.e : a.m >> (-a.e);
}
// to double, round to nearest even (subnormal and overflow results included)
__device__ inline double x_to_dbl(X87 a) {
    if (!a.m) return 0.0;
    int E = a.e + 63;
    if (E > 1023) return __longlong_as_double(0x7FF0000000000000LL);
    int sh = 11;
    if (E < -1022) sh += -1022 - E;
    if (sh > 64) return 0.0;
    uint64_t mant = sh == 64 ? 0 : a.m >> sh;
    const uint64_t rem = sh == 64 ? a.m : a.m & ((1ULL << sh) - 1), half = 1ULL << (sh - 1);
    if (rem > half || (rem == half && (mant & 1))) mant++;
    if (E < -1022) return __longlong_as_double((long long)mant);  // (a carry into bit 52 makes it normal)
    if (mant == (1ULL << 53)) {
        mant >>= 1;
        E++;
        if (E > 1023) return __longlong_as_double(0x7FF0000000000000LL);
    }
    return __longlong_as_double((long long)(((uint64_t)(E + 1023) << 52) | (mant & 0xFFFFFFFFFFFFFULL)));
}

// sqlite3Pow10: 10^E by binary powering, in long double
__device__ inline X87 x_pow10(int E) {
    X87 x = x_u64(10), r = x_u64(1);
    while (true) {
        if (E & 1) r = x_mul(r, x);
        E >>= 1;
        if (E == 0) break;
        x = x_mul(x, x);
    }
    return r;
}

// sqlite3AtoF (UTF-8): 1 = pure integer, 2+ = '.' and/or exponent, <= 0 = not a number (-1: a numeric
// prefix with '.'/exponent and trailing text)
// *sens: the result is not known to be version-independent (the header's PORTABLE rules).
__device__ int aff_atof(const TextView &t, double *out, bool *sens) {
    constexpr int64_t LARGEST = 0x7fffffffffffffffLL;
    *sens = false;
    uint64_t z = 0;
    const uint64_t zEnd = t.len;
    int sign = 1, d = 0, esign = 1, e = 0, eValid = 1, nDigit = 0, eType = 1;
    int64_t s = 0;
    double result;
    *out = 0.0;
    while (z < zEnd && aff_space(t.at(z))) z++;
    if (z >= zEnd) return 0;
    if (t.at(z) == '-') {
        sign = -1;
        z++;
    } else if (t.at(z) == '+') {
        z++;
    }
    while (z < zEnd && aff_digit(t.at(z))) {
        s = s * 10 + (int64_t)(t.at(z) - '0');
        z++;
        nDigit++;
        if (s >= ((LARGEST - 9) / 10))
            while (z < zEnd && aff_digit(t.at(z))) {
                *sens |= t.at(z) != '0';  // a dropped digit
                z++;
                d++;
            }
    }
    if (z < zEnd && t.at(z) == '.') {
        z++;
        eType++;
        while (z < zEnd && aff_digit(t.at(z))) {
            if (s < ((LARGEST - 9) / 10)) {
                s = s * 10 + (int64_t)(t.at(z) - '0');
                d--;
                nDigit++;
            } else {
                *sens |= t.at(z) != '0';  // a dropped digit
            }
            z++;
        }
    }
    if (z < zEnd && (t.at(z) == 'e' || t.at(z) == 'E')) {
        z++;
        eValid = 0;
        eType++;
        if (z < zEnd) {
            if (t.at(z) == '-') {
                esign = -1;
                z++;
            } else if (t.at(z) == '+') {
                z++;
            }
            while (z < zEnd && aff_digit(t.at(z))) {
                e = e < 10000 ? (e * 10 + (int)(t.at(z) - '0')) : 10000;
                z++;
                eValid = 1;
            }
        }
    }
    while (z < zEnd && aff_space(t.at(z))) z++;
    // (SQLite jumps past the trailing-space skip when the text ends early: the same, nothing is left)
    e = (e * esign) + d;
    if (e < 0) {
        esign = -1;
        e = -e;
    } else {
        esign = 1;
    }
    if (s == 0) {
        result = sign < 0 ? -0.0 : 0.0;
    } else {
        while (e > 0) {
            if (esign > 0) {
                if (s >= LARGEST / 10) break;
                s *= 10;
            } else {
                if (s % 10 != 0) break;
                s /= 10;
            }
            e--;
        }
        if (e == 0) {
            result = (double)(sign < 0 ? -s : s);
        } else if (e > 307 && e >= 342) {
            *sens = true;
            result = esign < 0 ? (sign < 0 ? -0.0 : 0.0)
                               : __longlong_as_double(sign < 0 ? (long long)0xFFF0000000000000ULL : 0x7FF0000000000000LL);
        } else {
            const X87 S = x_u64((uint64_t)s);  // s > 0 here; the sign is applied to the result
            if (e > 307) {
                *sens = true;
                const X87 scale = x_pow10(e - 308);
                double r = x_to_dbl(esign < 0 ? x_div(S, scale) : x_mul(S, scale));
                r = esign < 0 ? r / 1.0e+308 : r * 1.0e+308;
                result = sign < 0 ? -r : r;
            } else {
                const X87 scale = x_pow10(e);
                const X87 q = esign < 0 ? x_div(S, scale) : x_mul(S, scale);
                const double r = x_to_dbl(q);
                const int E = q.e + 63;  // the double's exponent
                const int low = (int)(q.m & 0x7FFu);  // the 11 bits the double drops: tie at 0x400
                // 3.37.2's error in 2^-64 units: half of one when 10^e is exact (e <= 27: one rounding),
                // a few per rounding of the binary powering otherwise (margin 32)
                const int margin = e <= 27 ? 1 : 32;
                if (E > 1023 || E < -1022 || (low >= 0x400 - margin && low <= 0x400 + margin)) *sens = true;
                result = sign < 0 ? -r : r;
            }
        }
    }
    *out = result;
    if (z == zEnd && nDigit > 0 && eValid && eType > 0) return eType;
    if (eType >= 2 && (eType == 3 || eValid) && nDigit > 0) return -1;
    return 0;
}

// sqlite3Atoi64 == 0: pure-integer text that fits in int64
__device__ bool aff_atoi64(const TextView &t, int64_t *out) {
    uint64_t i = 0, u = 0;
    const uint64_t n = t.len;
    bool neg = false;
    int nd = 0;
    while (i < n && aff_space(t.at(i))) i++;
    if (i < n && (t.at(i) == '-' || t.at(i) == '+')) neg = t.at(i++) == '-';
    while (i < n && t.at(i) == '0') i++;
    for (; i < n && aff_digit(t.at(i)); i++) {
        if (++nd > 19) return false;
        u = u * 10 + (t.at(i) - '0');
    }
    while (i < n && aff_space(t.at(i))) i++;
    if (i != n) return false;
    if (neg ? u > (1ULL << 63) : u > 0x7fffffffffffffffULL) return false;
    *out = neg ? (int64_t)(0 - u) : (int64_t)u;
    return true;
}

// sqlite3VdbeIntegerAffinity: a REAL holding an integer strictly inside (-2^63, 2^63)
__device__ inline bool aff_real_int(double r, int64_t *out) {
    if (!(r > -9223372036854775808.0 && r < 9223372036854775808.0)) return false;
    const int64_t ix = (int64_t)r;
    if ((double)ix != r) return false;
    *out = ix;
    return true;
}

__device__ uint32_t aff_int_text(int64_t v, uint8_t *out) {
    uint8_t buf[24];
    int k = 0;
    uint64_t u = v < 0 ? 0 - (uint64_t)v : (uint64_t)v;
    do {
        buf[k++] = (uint8_t)('0' + u % 10);
        u /= 10;
    } while (u);
    uint32_t n = 0;
    if (v < 0) out[n++] = '-';
    while (k) out[n++] = buf[--k];
    return n;
}

// "%!.15g" (sqlite3_str_vappendf, etGENERIC with flag_altform2), SQLite's long double steps
__device__ uint32_t aff_real_text(double r, uint8_t *out) {
    uint32_t n = 0;
    const bool neg = r < 0.0;
    const double ar = neg ? -r : r;
    if (neg) out[n++] = '-';
    if (ar == __longlong_as_double(0x7FF0000000000000LL)) {
        out[n++] = 'I', out[n++] = 'n', out[n++] = 'f';
        return n;
    }
    int precision = 14, exp = 0;  // 15 significant digits, generic: precision - 1
    const double rounder = 5.0e-05 * 1.0e-10;
    X87 v = x_dbl(ar);
    if (v.m) {
        X87 scale = x_u64(1);
        const X87 e100 = x_dbl(1e100), e10 = x_dbl(1e10), ten = x_u64(10);
        while (x_cmp(v, x_mul(e100, scale)) >= 0 && exp <= 350) {
            scale = x_mul(scale, e100);
            exp += 100;
        }
        while (x_cmp(v, x_mul(e10, scale)) >= 0 && exp <= 350) {
            scale = x_mul(scale, e10);
            exp += 10;
        }
        while (x_cmp(v, x_mul(ten, scale)) >= 0 && exp <= 350) {
            scale = x_mul(scale, ten);
            exp++;
        }
        v = x_div(v, scale);
        const X87 em8 = x_dbl(1e-8), e8 = x_dbl(1.0e8), one = x_u64(1);
        while (x_cmp(v, em8) < 0) {
            v = x_mul(v, e8);
            exp -= 8;
        }
        while (x_cmp(v, one) < 0) {
            v = x_mul(v, ten);
            exp--;
        }
    }
    v = x_add(v, x_dbl(rounder));
    if (x_cmp(v, x_u64(10)) >= 0) {
        v = x_mul(v, x_dbl(0.1));
        exp++;
    }
    const bool xexp = exp < -4 || exp > precision;
    int e2 = 0;
    if (!xexp) {
        precision -= exp;
        e2 = exp;
    }
    int nsd = 26;
    auto digit = [&]() -> uint8_t {  // et_getdigit
        if (nsd <= 0) return '0';
        nsd--;
        const uint64_t dg = x_trunc(v);
        v = x_mul(x_sub(v, x_u64(dg)), x_u64(10));
        return (uint8_t)('0' + dg);
    };
    if (e2 < 0) {
        out[n++] = '0';
    } else {
        for (; e2 >= 0; e2--) out[n++] = digit();
    }
    out[n++] = '.';
    for (e2++; e2 < 0; precision--, e2++) out[n++] = '0';
    while ((precision--) > 0) out[n++] = digit();
    while (out[n - 1] == '0') n--;
    if (out[n - 1] == '.') out[n++] = '0';
    if (xexp) {
        out[n++] = 'e';
        if (exp < 0) {
            out[n++] = '-';
            exp = -exp;
        } else {
            out[n++] = '+';
        }
        if (exp >= 100) {
            out[n++] = (uint8_t)(exp / 100 + '0');
            exp %= 100;
        }
        out[n++] = (uint8_t)(exp / 10 + '0');
        out[n++] = (uint8_t)(exp % 10 + '0');
    }
    return n;
}

// The value a column of affinity `aff` stores for (ty, v0, text t). True = converted: *oty, *ov0
// (INTEGER / REAL bits) or txt/len (TEXT, at most 24 bytes).
// *sens: the conversion is not known to be version-independent (the header's PORTABLE rules).
__device__ bool aff_convert(uint32_t aff, uint32_t ty, uint64_t v0, const TextView &t, uint32_t *oty,
                            uint64_t *ov0, uint8_t *txt, uint32_t *len, bool *sens) {
    *len = 0;
    *sens = false;
    if (aff == CORRO_AFF_BLOB || ty == CORRO_NULL || ty == CORRO_BLOB) return false;
    if (aff == CORRO_AFF_TEXT) {
        if (ty == CORRO_INTEGER) {
            *len = aff_int_text((int64_t)v0, txt);
        } else if (ty == CORRO_REAL) {
            const double r = __longlong_as_double((long long)v0);
            *len = aff_real_text(r, txt);
            TextView back{0, 0, txt, *len};
            double rb;
            bool sb;  // (unused: 3.37.2's re-read is enough -- when it gives r back, r lies within
                      // about half an ulp of the 15-digit text, far from a 15th-digit tie)
            // must round-trip; -0.0 renders as "0.0" in 3.37.2 (its sign test is r < 0.0), a
            // rendering later versions need not share
            *sens = aff_atof(back, &rb, &sb) <= 0 || rb != r || (r == 0.0 && signbit(r));
        } else {
            return false;
        }
        *oty = CORRO_TEXT;
        *ov0 = 0;
        return true;
    }
    uint32_t rt = ty;
    int64_t iv = (int64_t)v0;
    double rv = __longlong_as_double((long long)v0);
    if (ty == CORRO_TEXT) {
        double r;
        bool sr;
        const int rc = aff_atof(t, &r, &sr);
        if (rc <= 0) return false;
        int64_t i;
        if (rc == 1 && aff_atoi64(t, &i)) {  // alsoAnInt (exact)
            rt = CORRO_INTEGER;
            iv = i;
        } else if (aff_real_int(r, &i)) {
            rt = CORRO_INTEGER;
            iv = i;
            *sens = sr;
        } else {
            rt = CORRO_REAL;
            rv = r;
            *sens = sr;
        }
    } else if (ty == CORRO_REAL) {
        int64_t i;
        if (aff_real_int(rv, &i)) {
            rt = CORRO_INTEGER;
            iv = i;
        }
    }
    if (aff == CORRO_AFF_REAL && rt == CORRO_INTEGER) {
        rt = CORRO_REAL;
        rv = (double)iv;
    }
    *oty = rt;
    *ov0 = rt == CORRO_INTEGER ? (uint64_t)iv : (uint64_t)__double_as_longlong(rv);
    return rt != ty || *ov0 != v0;
}

// Pass 0 (write = false): conv[i] = 1 for every change its column's affinity converts; counts in
// cnt[0] (conversions) and cnt[1] (converted values longer than 16 bytes). Pass 1 (write = true)
// over the flagged changes: the converted value as a staged record holds it -- meta (type | len),
// words 0 / 1 (a long text's bytes go to a 24-byte arena slot: word 1 = its handle).
template <bool WRITE>
__global__ void __launch_bounds__(256) k_aff_convert(BatchDev in, const uint8_t *__restrict__ aff, uint32_t ntables,
                                                     uint8_t *conv, uint64_t *cv0, uint64_t *cv1, uint32_t *cmeta,
                                                     uint8_t *arena, uint64_t slot_base,
                                                     unsigned long long *cnt) {
    uint32_t nconv = 0, nlong = 0, nsens = 0;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < in.n; i += gridDim.x * blockDim.x) {
        if (WRITE && !conv[i]) continue;
        const uint32_t tc = in.tcid[i], t = tc >> 16, cid = tc & 0xFFFFu;
        uint8_t c = 0;
        if (cid != 0 && cid <= MAX_COLS && t < ntables) {  // sentinels carry NULL; names checked elsewhere
            const uint32_t a = aff[t * (MAX_COLS + 1) + cid];
            const uint32_t ty = in.vt ? in.vt[i] : (uint32_t)CORRO_INTEGER;
            bool go = a != CORRO_AFF_BLOB && ty != CORRO_NULL && ty != CORRO_BLOB && ty >= 1 && ty <= 5;
            const uint32_t ln = in.vl ? in.vl[i] : 0u;
            TextView tv{in.v0[i], in.v1 ? in.v1[i] : 0ULL, nullptr, ln};
            if (go && ty == CORRO_TEXT && ln == VLEN_LONG) {
                // a malformed span is left alone here (k_scatter reports it): long_value's bounds
                if (!in.voff || !in.vsz || !in.arena) {
                    go = false;
                } else {
                    const uint64_t off = in.voff[i];
                    const uint32_t sz = in.vsz[i];
                    go = sz > 16 && sz < (1u << 24) && off <= in.ldata && sz <= in.ldata - off;
                    if (go) {
                        tv.p = in.arena + in.lbase + off;
                        tv.len = sz;
                    }
                }
            } else if (go && ty == CORRO_TEXT && ln > 16) {
                go = false;
            }
            uint32_t oty = 0, olen = 0;
            uint64_t ov0 = 0;
            uint8_t txt[32];
            bool sens = false;
            if (go && aff_convert(a, ty, in.v0[i], tv, &oty, &ov0, txt, &olen, &sens)) {
                c = 1;
                nconv++;
                nsens += sens;
                nlong += olen > 16;
                if (WRITE) {
                    uint64_t w0 = 0, w1 = 0;
                    uint32_t meta = oty;
                    if (oty != CORRO_TEXT) {
                        w0 = ov0;
                    } else {
                        for (uint32_t k = 0; k < 8 && k < olen; k++) w0 |= (uint64_t)txt[k] << (56 - 8 * k);
                        if (olen <= 16) {
                            for (uint32_t k = 8; k < olen; k++) w1 |= (uint64_t)txt[k] << (56 - 8 * (k - 8));
                            meta |= olen << 8;
                        } else {
                            const uint64_t off = slot_base + 24ULL * atomicAdd(&cnt[2], 1ULL);
                            for (uint32_t k = 0; k < olen; k++) arena[off + k] = txt[k];
                            w1 = (off << 24) | olen;
                            meta |= VLEN_LONG << 8;
                        }
                    }
                    cv0[i] = w0;
                    cv1[i] = w1;
                    cmeta[i] = meta;
                }
            }
        }
        if (!WRITE) conv[i] = c;
    }
    if (!WRITE) {
        nconv = wave_sum_u32(nconv);
        nlong = wave_sum_u32(nlong);
        nsens = wave_sum_u32(nsens);
        if ((threadIdx.x & 63) == 0 && nconv) {
            atomicAdd(&cnt[0], (unsigned long long)nconv);
            atomicAdd(&cnt[1], (unsigned long long)nlong);
            if (nsens) atomicAdd(&cnt[3], (unsigned long long)nsens);
        }
    }
}

int arena_reserve(corro_ctx *ctx, uint64_t add);  // engine.hip
#define AFF_TRY(x)                   \
    do {                             \
        if (int rc_ = (x)) return rc_; \
    } while (0)

// The converted values of the batch (affinity.hip header comment): bd.conv / cv0 / cv1 / cmeta set
// when some change is converted, left null otherwise.
int affinity_convert(corro_ctx *ctx, BatchDev &bd) {
    if (!ctx->aff_any || bd.n == 0) return CORRO_OK;
    hipStream_t s = ctx->stream;
    const uint64_t n = bd.n;
    AFF_TRY(ctx->d_aff_conv.ensure(n));
    unsigned long long *cnt = ctx->d_affflag.as<unsigned long long>();
    CORRO_HIP_TRY(hipMemsetAsync(cnt, 0, 32, s));
    uint8_t *conv = ctx->d_aff_conv.as<uint8_t>();
    const dim3 grid((uint32_t)std::min<uint64_t>((n + 255) / 256, 8192));
    const uint32_t nt = (uint32_t)ctx->tables.size();
    hipLaunchKernelGGL(k_aff_convert<false>, grid, dim3(256), 0, s, bd, ctx->d_aff.as<uint8_t>(), nt, conv, nullptr,
                       nullptr, nullptr, nullptr, 0ULL, cnt);
    CORRO_HIP_TRY(hipGetLastError());
    uint64_t h[4] = {0, 0, 0, 0};
    CORRO_HIP_TRY(hipMemcpyAsync(h, cnt, 32, hipMemcpyDeviceToHost, s));
    CORRO_HIP_TRY(hipStreamSynchronize(s));
    if (!h[0]) return CORRO_OK;
    if (h[3] && ctx->aff_policy == CORRO_AFF_POLICY_PORTABLE)
        return fail(CORRO_E_RANGE, std::to_string(h[3]) + " change(s) need a column-affinity conversion whose result "
                                   "depends on the SQLite version (TEXT <-> REAL rounding): refused under "
                                   "CORRO_AFF_POLICY_PORTABLE (corro_set_affinity_policy)");
    ctx->metrics.aff_sensitive += h[3];  // (counted at staging: a batch that later fails is counted too)
    // 20 bytes per change of the batch: cv0 | cv1 | cmeta
    AFF_TRY(ctx->d_aff_vals.ensure(n * 20));
    uint64_t *cv0 = ctx->d_aff_vals.as<uint64_t>(), *cv1 = cv0 + n;
    uint32_t *cmeta = (uint32_t *)(cv1 + n);
    uint64_t slot_base = 0;
    if (h[1]) {
        AFF_TRY(arena_reserve(ctx, h[1] * 24));
        slot_base = ctx->arena_top;
        ctx->arena_top += h[1] * 24;
    }
    hipLaunchKernelGGL(k_aff_convert<true>, grid, dim3(256), 0, s, bd, ctx->d_aff.as<uint8_t>(), nt, conv, cv0, cv1,
                       cmeta, ctx->d_arena.as<uint8_t>(), slot_base, cnt);
    CORRO_HIP_TRY(hipGetLastError());
    bd.conv = conv;
    bd.cv0 = cv0;
    bd.cv1 = cv1;
    bd.cmeta = cmeta;
    bd.arena = ctx->d_arena.as<uint8_t>();
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

extern "C" int corro_set_affinity_policy(corro_ctx *ctx, int policy) {
    if (!ctx) return fail(CORRO_E_INVALID, "NULL argument");
    if (policy != CORRO_AFF_POLICY_PORTABLE && policy != CORRO_AFF_POLICY_SQLITE_3_37_2)
        return fail(CORRO_E_INVALID, "unknown affinity policy");
    ctx->aff_policy = policy;
    return CORRO_OK;
}
