// textio_check.cpp -- host check of the shared "%.6lf" formatter and "%lf"
// fast-path parser (kb2e_amd/csrc/textio.hpp) against glibc's own snprintf and
// strtod, which the reference's fprintf / fscanf use.  The same inline
// functions run in the device kernels (textio.hip).  Test infrastructure.
//   textio_check [count] [seed]  -> prints "ok <n>" or the first mismatch.
#include <cinttypes>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "../../kb2e_amd/csrc/textio.hpp"

static int check_one(double v) {
    char want[400], got[400];
    const int wl = snprintf(want, sizeof want, "%.6lf", v);
    const int gl = kb2e::fmt_fixed6(v, got);
    const int ml = kb2e::fmt_fixed6(v, nullptr);
    if (wl != gl || ml != gl || memcmp(want, got, (size_t)wl) != 0) {
        got[gl < 399 ? gl : 399] = 0;
        printf("FORMAT MISMATCH %a: want '%s' got '%s'\n", v, want, got);
        return 1;
    }
    if (std::isfinite(v)) {  // the written text parses back to strtod's value
        double p = 0;
        const int st = kb2e::parse_fast(want, wl, &p);
        const double s = strtod(want, nullptr);
        if (st == 0 && memcmp(&p, &s, 8) != 0) {
            printf("PARSE MISMATCH '%s': strtod %a fast %a\n", want, s, p);
            return 1;
        }
    }
    return 0;
}

static int check_token(const char* tok) {
    double p = 0;
    const int st = kb2e::parse_fast(tok, (int64_t)strlen(tok), &p);
    char* end = nullptr;
    const double s = strtod(tok, &end);
    if (st == 0 && (*end != 0 || memcmp(&p, &s, 8) != 0)) {
        printf("TOKEN MISMATCH '%s': strtod %a fast %a\n", tok, s, p);
        return 1;
    }
    return 0;
}

int main(int argc, char** argv) {
    const long count = argc > 1 ? atol(argv[1]) : 2000000;
    std::mt19937_64 rng(argc > 2 ? strtoull(argv[2], nullptr, 10) : 1);
    int bad = 0;
    long n = 0;
    // edge cases: ties at the 7th digit, signed zeros, subnormals, huge, non-finite
    const double edges[] = {0.0, -0.0, 0.0078125, 0.0234375, -0.0234375, 5e-7, 4.9999999999999998e-7, 5.0000000000000004e-7,
                            -1e-9, 0.9999995, 0.99999949999999995, 1.0, -1.0, 123456.7890125, 4.94e-324, 2.2250738585072014e-308,
                            9007199254740992.0, 9007199254740993.0, 1.8446744073709552e19, 1e22, 1e300, 1.7976931348623157e308,
                            -1.7976931348623157e308, INFINITY, -INFINITY, NAN, -NAN, 0.5, 1.5, 2.5, 1e-6, 1.5e-6, 2.5e-6};
    for (double e : edges) bad += check_one(e), ++n;
    // every tie k + 0.5 ulp at 1e-6 representable as a dyadic: (2j+1) / 2^7 / 5^6 * 5^6 ...
    for (int j = 0; j < 20000; ++j) bad += check_one((2.0 * j + 1) / 128.0), bad += check_one(-(2.0 * j + 1) / 2048.0), n += 2;
    std::uniform_real_distribution<double> u(-1.0, 1.0);
    std::uniform_int_distribution<uint64_t> bits;
    for (long k = 0; k < count && bad == 0; ++k) {
        double v;
        switch (k % 4) {
            case 0: v = u(rng); break;                                   // embedding-like
            case 1: v = u(rng) * 1e-5; break;                            // near the last digit
            case 2: v = std::ldexp(u(rng), (int)(bits(rng) % 140) - 70); break;
            default: {
                uint64_t b = bits(rng);
                memcpy(&v, &b, 8);
            }
        }
        bad += check_one(v);
        ++n;
    }
    const char* toks[] = {"0.000000", "-0.000000", "1", "-1", "+1.5", ".5", "5.", "1e5", "1E-5", "2.5e+3", "0.1234567890123456789",
                          "12345678901234567890", "123456789012345678901234", "1e-400", "1e400", "abc", "-", ".", "1.2.3",
                          "0x1p3", "inf", "nan", "1e", "00000000000000000000001.5", "0.000000000000000000000000001"};
    for (const char* t : toks) bad += check_token(t), ++n;
    char buf[64];
    for (long k = 0; k < count / 4 && bad == 0; ++k) {  // random decimal tokens
        const int digits = 1 + (int)(bits(rng) % 18), point = (int)(bits(rng) % (digits + 1));
        int p = 0;
        if (bits(rng) & 1) buf[p++] = '-';
        for (int d = 0; d < digits; ++d) {
            if (d == point) buf[p++] = '.';
            buf[p++] = (char)('0' + bits(rng) % 10);
        }
        if (bits(rng) % 4 == 0) p += snprintf(buf + p, 16, "e%d", (int)(bits(rng) % 60) - 30);
        buf[p] = 0;
        bad += check_token(buf);
        ++n;
    }
    if (bad) return 1;
    printf("ok %ld\n", n);
    return 0;
}
