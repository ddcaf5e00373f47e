// textio.hpp -- the once-per-run host work of the reference moved onto the
// device, its own translation unit (textio.hip):
//
//   * device init: Trainer::prepTrain's randn draws (common/trainer.cpp:34-58,
//     common/utils.cpp:26-38) taken from the same glibc stream, value for
//     value -- the engine's rng is advanced by exactly the words the reference
//     consumes, so the sample stream that follows is unchanged;
//   * "%.6lf\t" table writer (common/trainer.cpp:109-127, transh/trainer.cpp:
//     94-105, transr/trainer.cpp:128-142): formatted on the device, byte for
//     byte glibc printf's output (exact decimal rounding, ties to even);
//   * "%lf" table reader (transr/trainer.cpp:88-113 seed files, the
//     evaluators' table loads): tokens split and converted on the device.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <functional>
#include <string>

#include "glibc_rand.hpp"

namespace kb2e {

// ---- %.6lf formatting, shared by host and device --------------------------
//
// Writes the "%.6lf" text of v into out (no terminator) and returns its
// length; out == nullptr only measures.  Exact: v = m 2^e, the six-digit
// fraction is floor/round of m 10^6 2^e computed in 128-bit integers with
// round-half-even on the exact remainder (glibc's rounding in the default
// mode); |v| >= 2^64 takes a multi-limb conversion of the integer part.
constexpr int kFmtMax = 320;  // longest "%.6lf" text: "-" + 309 digits + ".000000"

__host__ __device__ inline int fmt_u64(uint64_t x, char* out) {  // decimal digits of x
    char tmp[20];
    int k = 0;
    do {
        tmp[k++] = (char)('0' + x % 10);
        x /= 10;
    } while (x);
    if (out)
        for (int q = 0; q < k; ++q) out[q] = tmp[k - 1 - q];
    return k;
}

// Digits of m * 2^e (m < 2^53, 11 <= e <= 971) by repeated division by 10^9.
__host__ __device__ inline int fmt_bigint(uint64_t m, int e, char* out) {
    uint32_t limb[34];  // little endian, up to 1024 + 53 bits
    int nl = 0;
    for (int q = 0; q < 34; ++q) limb[q] = 0;
    const int ws = e / 32, bs = e % 32;
    const unsigned __int128 sh = (unsigned __int128)m << bs;
    for (int q = 0; q < 3; ++q) limb[ws + q] = (uint32_t)(sh >> (32 * q));
    nl = ws + 3;
    while (nl > 0 && limb[nl - 1] == 0) --nl;
    uint32_t groups[40];  // base-10^9 groups, least significant first
    int ng = 0;
    while (nl > 0) {
        uint64_t rem = 0;
        for (int q = nl - 1; q >= 0; --q) {
            const uint64_t cur = (rem << 32) | limb[q];
            limb[q] = (uint32_t)(cur / 1000000000u);
            rem = cur % 1000000000u;
        }
        groups[ng++] = (uint32_t)rem;
        while (nl > 0 && limb[nl - 1] == 0) --nl;
    }
    int len = fmt_u64(groups[ng - 1], out);
    for (int g = ng - 2; g >= 0; --g) {
        uint32_t v = groups[g];
        if (out)
            for (int d = 8; d >= 0; --d) {
                out[len + d] = (char)('0' + v % 10);
                v /= 10;
            }
        len += 9;
    }
    return len;
}

__host__ __device__ inline int fmt_fixed6(double v, char* out) {
    uint64_t bits;
    memcpy(&bits, &v, 8);
    const bool neg = bits >> 63;
    const int be = (int)((bits >> 52) & 0x7ff);
    const uint64_t frac = bits & ((1ull << 52) - 1);
    int len = 0;
    if (be == 0x7ff) {  // glibc: "inf" / "nan", sign shown
        const char* s = frac ? "nan" : "inf";
        if (neg) {
            if (out) out[len] = '-';
            ++len;
        }
        for (int q = 0; q < 3; ++q) {
            if (out) out[len] = s[q];
            ++len;
        }
        return len;
    }
    if (neg) {
        if (out) out[0] = '-';
        len = 1;
    }
    const uint64_t m = be ? (frac | (1ull << 52)) : frac;
    const int e = be ? be - 1075 : -1074;
    uint64_t ip = 0, fr = 0;  // integer part, six fraction digits
    if (e >= 0) {
        if (e > 10) {  // >= 2^63: the integer part by limbs, fraction zero
            len += fmt_bigint(m, e, out ? out + len : nullptr);
            goto fraction;
        }
        ip = m << e;
    } else {
        const int sh = -e;
        ip = sh < 64 ? (m >> sh) : 0;
        const uint64_t f = sh < 64 ? (m & ((1ull << sh) - 1)) : m;  // fraction numerator over 2^sh
        if (sh <= 74) {  // f 10^6 < 2^73: for sh > 74 the fraction is < 2^-21 and rounds to 0
            const unsigned __int128 p = (unsigned __int128)f * 1000000u;
            uint64_t d = (uint64_t)(p >> sh);
            const unsigned __int128 rem = p - ((unsigned __int128)d << sh);
            const unsigned __int128 half = (unsigned __int128)1 << (sh - 1);
            if (rem > half || (rem == half && (d & 1))) ++d;
            if (d == 1000000u) {
                d = 0;
                ++ip;
            }
            fr = d;
        }
    }
    len += fmt_u64(ip, out ? out + len : nullptr);
fraction:
    if (out) {
        out[len] = '.';
        for (int d = 6; d >= 1; --d) {
            out[len + d] = (char)('0' + fr % 10);
            fr /= 10;
        }
    }
    return len + 7;
}

// ---- %lf token parsing, shared by host and device -------------------------
//
// Exact fast path: [+-] digits [. digits] [(e|E) [+-] digits] with at most 19
// significant digits N and decimal exponent q: when N < 2^53 and |q| <= 22
// both N and 10^|q| are exact doubles and one IEEE multiply / divide gives the
// correctly rounded value -- strtod's result (every "%.6lf" field of magnitude
// below 9e9 is such a token).  Returns 0 ok, 1 anything else -- the caller
// converts it with strtod (hex floats, inf / nan, long mantissas, huge
// exponents) and rejects the token if strtod does not consume all of it.
__host__ __device__ inline int parse_fast(const char* s, int64_t n, double* out) {
    constexpr double p10[23] = {1e0,  1e1,  1e2,  1e3,  1e4,  1e5,  1e6,  1e7,  1e8,  1e9,  1e10, 1e11,
                                1e12, 1e13, 1e14, 1e15, 1e16, 1e17, 1e18, 1e19, 1e20, 1e21, 1e22};
    int64_t k = 0;
    bool neg = false;
    if (k < n && (s[k] == '+' || s[k] == '-')) neg = s[k++] == '-';
    uint64_t N = 0;
    int sig = 0, q = 0, digits = 0;
    bool dropped = false;
    for (; k < n && s[k] >= '0' && s[k] <= '9'; ++k, ++digits) {
        if (sig < 19) {
            if (N || s[k] != '0') {
                N = N * 10 + (uint64_t)(s[k] - '0');
                ++sig;
            }
        } else {
            ++q;
            dropped |= s[k] != '0';
        }
    }
    if (k < n && s[k] == '.') {
        for (++k; k < n && s[k] >= '0' && s[k] <= '9'; ++k, ++digits) {
            if (sig < 19) {
                if (N || s[k] != '0') {
                    N = N * 10 + (uint64_t)(s[k] - '0');
                    ++sig;
                }
                --q;
            } else {
                dropped |= s[k] != '0';
            }
        }
    }
    if (digits == 0) return 1;
    if (k < n && (s[k] == 'e' || s[k] == 'E')) {
        int64_t j = k + 1;
        bool eneg = false;
        if (j < n && (s[j] == '+' || s[j] == '-')) eneg = s[j++] == '-';
        if (j >= n || s[j] < '0' || s[j] > '9') return 1;  // "1e" / "1e+": strtod stops before the e
        int ex = 0;
        for (; j < n && s[j] >= '0' && s[j] <= '9'; ++j) ex = ex < 100000 ? ex * 10 + (s[j] - '0') : ex;
        q += eneg ? -ex : ex;
        k = j;
    }
    if (k != n) return 1;  // not a plain decimal (hex, inf, trailing characters)
    if (dropped) return 1;
    double v;
    if (N == 0) v = 0.0;
    else if (N < (1ull << 53) && q >= -22 && q <= 22) v = q >= 0 ? (double)N * p10[q] : (double)N / p10[-q];
    else return 1;
    *out = neg ? -v : v;
    return 0;
}

// ---- device entry points (textio.hip) --------------------------------------

// common::randn(miu, sigma, lo, hi) (common/utils.cpp:26-38) `count` times from
// `rng`'s stream, into the device array out[count]; `rng` is advanced by
// exactly the words those calls consume.  jump = the glibc jump table (L words
// a block, device memory).  Returns the number of accept/reject decisions whose
// margin was within a few ulps of the density (where the device exp and
// glibc's could round differently; 0 in every run measured).
int64_t device_randn(GlibcRand& rng, const uint32_t* jump, int L, double miu, double sigma, double lo, double hi,
                     int64_t count, double* out, hipStream_t st);

// dst[r][0..n) (leading dimension ld, double or float) = vals[r*n .. r*n+n),
// then common::norm(row, ignore_short) (common/utils.cpp:70-77) with the
// reference's sequential sum of squares.
void place_rows(const double* vals, int64_t rows, int n, int ld, void* dst, bool f64, bool norm, bool ignore_short,
                hipStream_t st);

// TransR Mr = identity (transr/trainer.cpp:73-86), [r][j][i] rows of ld.
void identity_weights(void* w, int64_t nr, int n, int ld, bool f64, hipStream_t st);

// A device table (rows x n, leading dimension ld) as the reference's text:
// "%.6lf\t" per value, "\n" per row.  The bytes are handed to `sink` in order,
// chunk by chunk.  Returns the total length.
int64_t format_table(const void* table, bool f64, int64_t rows, int n, int ld, hipStream_t st,
                     const std::function<void(const char*, size_t)>& sink);

// The first `count` whitespace-separated "%lf" tokens of text[0..len) into the
// device array out[count].  Returns the number of tokens converted (< count:
// the text ran out, as fscanf returning EOF); *bad = index of the first token
// that is not a number (fscanf returning 0), or -1.  Tokens outside the exact
// fast path (> 19 significant digits, |exponent| beyond 10^22, hex, inf / nan)
// are counted in *slow and converted with strtod on the host; a token strtod
// does not consume whole is not a number.
int64_t parse_doubles(const char* text, int64_t len, int64_t count, double* out, hipStream_t st, int64_t* bad,
                      int64_t* slow);

}  // namespace kb2e
