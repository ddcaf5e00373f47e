// kernels_glibc.hpp -- the glibc TYPE_3 rand() stream made on the device from
// a 31-word window (glibc_rand.hpp's jump table).  Used by the epoch sampler
// (kernels_sampler.hpp, engine.hip) and the device init (textio.hip); the
// kernels have internal linkage so each translation unit keeps its own copy.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace kb2e {
namespace {

// glibc_starts: one wave walks the epoch in blocks of L words: the window
//   before block p+1 is rows L-31..L-1 of the jump table applied to the window
//   before block p (31 x 31 multiply-adds mod 2^32 per block).
// glibc_words: word i = pL + t is sum_m C[m][t] * start_p[m], independently.
// raw[0..31) = the starting window, raw[31 + i] = word i (raw), words[i] =
// raw >> 1 (what rand() returns).
struct GlibcWindow {
    uint32_t w[31];
};

[[maybe_unused]] __global__ __launch_bounds__(64) void glibc_starts_kernel(GlibcWindow win, const uint32_t* C, int32_t L,
                                                          int32_t nblocks, uint32_t* starts, uint32_t* raw) {
    __shared__ uint32_t cur[32];
    __shared__ uint32_t tail[31][32];  // tail[j][m] = C[m][L - 31 + j]
    const int l = threadIdx.x;
    for (int q = l; q < 31 * 31; q += 64) {
        const int j = q / 31, m = q % 31;
        tail[j][m] = C[(size_t)m * L + (L - 31 + j)];
    }
    if (l < 31) {
        cur[l] = win.w[l];
        raw[l] = win.w[l];
    }
    __syncthreads();
    for (int p = 0; p < nblocks; ++p) {
        uint32_t v = 0;
        if (l < 31) {
            starts[(size_t)p * 31 + l] = cur[l];
#pragma unroll
            for (int m = 0; m < 31; ++m) v += tail[l][m] * cur[m];
        }
        __syncthreads();
        if (l < 31) cur[l] = v;
        __syncthreads();
    }
}

// glibc_starts_pow: the same windows with no walk: the window before block p is
//   M^p applied to the starting window (M = the L-word jump, rows L-31..L-1 of
//   the table), one workgroup per block multiplying by the precomputed squares
//   M^(2^k) of p's set bits (row-major 31 x 31, k < kGlibcPowLevels).  Block 0
//   also writes raw[0..31) and clears *clear (the sampler's overflow flag).
constexpr int kGlibcPowLevels = 24;

[[maybe_unused]] __global__ __launch_bounds__(64) void glibc_starts_pow_kernel(GlibcWindow win, const uint32_t* P,
                                                                              uint32_t* starts, uint32_t* raw,
                                                                              int32_t* clear) {
    __shared__ uint32_t cur[32];
    const int l = threadIdx.x;
    const int p = blockIdx.x;
    if (l < 31) cur[l] = win.w[l];
    if (p == 0) {
        if (l < 31) raw[l] = win.w[l];
        if (l == 0 && clear) *clear = 0;
    }
    __syncthreads();
    for (int k = 0; (p >> k) != 0; ++k) {
        if (!((p >> k) & 1)) continue;
        uint32_t v = 0;
        if (l < 31) {
            const uint32_t* row = P + ((size_t)k * 31 + l) * 31;
#pragma unroll
            for (int m = 0; m < 31; ++m) v += row[m] * cur[m];
        }
        __syncthreads();
        if (l < 31) cur[l] = v;
        __syncthreads();
    }
    if (l < 31) starts[(size_t)p * 31 + l] = cur[l];
}

__global__ __launch_bounds__(256) void glibc_words_kernel(const uint32_t* C, int32_t L, const uint32_t* starts,
                                                          int64_t nraw, uint32_t* raw, int32_t* words) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nraw) return;
    const int64_t p = i / L;
    const int t = (int)(i - p * L);
    const uint32_t* st = starts + p * 31;
    uint32_t v = 0;
#pragma unroll
    for (int m = 0; m < 31; ++m) v += C[(size_t)m * L + t] * st[m];
    raw[31 + i] = v;
    words[i] = (int32_t)(v >> 1);
}

// The generator window after the epoch's `consumed` words: raw[used .. used + 31).
[[maybe_unused]] __global__ void glibc_window_kernel(const uint32_t* raw, const int64_t* consumed, uint32_t* out) {
    const int l = threadIdx.x;
    const int64_t used = *consumed;
    if (l < 31) out[l] = used >= 0 ? raw[used + l] : 0u;
}

}  // namespace
}  // namespace kb2e
