// glibc_rand.hpp -- the reference's random stream, restated natively.
//
// The reference draws every random number from the process-global glibc
// rand() seeded once in main() (transe/bin/trainTransE.cpp:13).  glibc's
// rand() is random_r() with the default TYPE_3 state: an additive lagged
// Fibonacci generator r[i] = r[i-3] + r[i-31] (mod 2^32), output r >> 1,
// seeded by a Park-Miller LCG and warmed up by 310 discarded outputs.  Keeping
// our own copy of that state (instead of calling libc) lets the engine hand the
// exact state to the device sampler and advance it by jump-ahead.
#pragma once

#include <cmath>
#include <cstdint>
#include <cstring>

namespace kb2e {

struct GlibcRand {
    static constexpr int kDeg = 31;  // TYPE_3 degree
    static constexpr int kSep = 3;   // TYPE_3 separation
    int32_t state[kDeg];
    int f = kSep;  // buf->fptr - state
    int r = 0;     // buf->rptr - state

    explicit GlibcRand(uint32_t seed = 1) { seed_with(seed); }

    // srandom_r: Park-Miller "minimal standard" fill, then 10 * deg discards.
    void seed_with(uint32_t seed) {
        if (seed == 0) seed = 1;
        state[0] = (int32_t)seed;
        int32_t word = (int32_t)seed;
        for (int i = 1; i < kDeg; ++i) {
            long hi = word / 127773;
            long lo = word % 127773;
            word = (int32_t)(16807 * lo - 2836 * hi);
            if (word < 0) word += 2147483647;
            state[i] = word;
        }
        f = kSep;
        r = 0;
        for (int k = 0; k < kDeg * 10; ++k) (void)next();
    }

    // random_r: one output in [0, RAND_MAX].
    inline int32_t next() {
        uint32_t val = (uint32_t)state[f] + (uint32_t)state[r];
        state[f] = (int32_t)val;
        int32_t result = (int32_t)(val >> 1);
        if (++f >= kDeg) {
            f = 0;
            ++r;
        } else if (++r >= kDeg) {
            r = 0;
        }
        return result;
    }

    // One raw 32-bit word (the value random_r stores; rand() returns it >> 1).
    inline uint32_t next_raw() {
        uint32_t val = (uint32_t)state[f] + (uint32_t)state[r];
        state[f] = (int32_t)val;
        if (++f >= kDeg) {
            f = 0;
            ++r;
        } else if (++r >= kDeg) {
            r = 0;
        }
        return val;
    }

    // The 31 most recent raw words, oldest first (the word the next call adds
    // to is w[0], lag 31; w[28] is lag 3).
    void window(uint32_t w[kDeg]) const {
        for (int m = 0; m < kDeg; ++m) w[m] = (uint32_t)state[(f + m) % kDeg];
    }
    void set_window(const uint32_t w[kDeg]) {
        for (int m = 0; m < kDeg; ++m) state[m] = (int32_t)w[m];
        f = 0;
        r = kDeg - kSep;
    }

    // Advance this generator past `m` words whose raw values `vals[0..m)` were
    // generated from exactly this state (f and r always move together, r = f - 3
    // mod 31, and the word made at step q lands in slot (f + q) mod 31).
    void commit(const uint32_t* vals, int64_t m) {
        if (m < kDeg) {
            for (int64_t q = 0; q < m; ++q) (void)next_raw();
            return;
        }
        const int f0 = f;
        for (int64_t q = m - kDeg; q < m; ++q) state[(f0 + q) % kDeg] = (int32_t)vals[q];
        f = (int)((f0 + m) % kDeg);
        r = (f + kDeg - kSep) % kDeg;
    }
};

// Jump table of the TYPE_3 recurrence r[i] = r[i-3] + r[i-31] (mod 2^32):
// r[i0 + t] = sum_m C[m][t] * r[i0 - 31 + m] for 0 <= t < L, stored m-major
// (C[m * L + t]) so consecutive t are consecutive words.  With it the device
// makes a whole epoch's words in parallel from one 31-word window.
inline void glibc_jump_table(int L, uint32_t* C) {
    constexpr int D = GlibcRand::kDeg;
    // coef(t) for t >= -31: unit vectors before i0, then coef(t-3) + coef(t-31)
    auto at = [&](int t, int m) -> uint32_t {
        return t < 0 ? (uint32_t)(m == D + t ? 1u : 0u) : C[(size_t)m * L + t];
    };
    for (int t = 0; t < L; ++t)
        for (int m = 0; m < D; ++m) C[(size_t)m * L + t] = at(t - GlibcRand::kSep, m) + at(t - D, m);
}

// common/utils.cpp:113-120 -- (rand() * rand()) % x in int32 with wrap-around
// (the product overflows in practice; both factors are consumed either way).
inline int32_t rand_max(GlibcRand& g, int32_t x) {
    uint32_t a = (uint32_t)g.next();
    uint32_t b = (uint32_t)g.next();
    int32_t res = (int32_t)(a * b) % x;
    while (res < 0) res += x;
    return res;
}

// common/utils.cpp:18-20
inline double rand_range(GlibcRand& g, double min, double max) {
    return min + (max - min) * g.next() / (2147483647 + 1.0);
}

// common/utils.cpp:22-24
inline double normal_pdf(double x, double miu, double sigma) {
    const double pi = 3.1415926535897932384626433832795;
    return 1.0 / std::sqrt(2 * pi) / sigma * std::exp(-1 * ((x - miu) * (x - miu)) / (2 * (sigma * sigma)));
}

// common/utils.cpp:26-38 -- uniform-proposal rejection sampler.
inline double randn(GlibcRand& g, double miu, double sigma, double min, double max) {
    double x, y, scope;
    do {
        x = rand_range(g, min, max);
        y = normal_pdf(x, miu, sigma);
        scope = rand_range(g, 0.0, normal_pdf(miu, miu, sigma));
    } while (scope > y);
    return x;
}

}  // namespace kb2e
