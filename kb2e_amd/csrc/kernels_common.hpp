// kernels_common.hpp -- shared device helpers for the kb2e_amd engine (gfx950).
//
// Row layout in HBM: every table is row-major with a leading dimension `ld`
// (elements) rounded up to a multiple of 2, 16-byte aligned for FP64 pairs.
// One 64-lane wave owns one row: lane l holds elements {128 c + 2 l, +1} for
// chunks c < CH (CH = ceil(n / 128)).  Padding elements are zero and are never
// written.  Reductions are deterministic xor-butterflies over the 64 lanes.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace kb2e {

constexpr int kWave = 64;
constexpr int kVec = 2;  // elements per lane per chunk

// DPP lane moves.  Every lane the result is read from is written, so no
// `old` operand (and no zero-initialisation) is needed.
//   ROR<N>:  row_ror:N within each 16-lane row
//   BC15:    row_bcast:15 (lane 15 of row k to every lane of row k+1)
//   BC31:    row_bcast:31 (lane 31 to rows 2 and 3)
template <int CTRL>
__device__ __forceinline__ float dpp_mov(float x) {
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), CTRL, 0xF, 0xF, false));
}
template <int CTRL>
__device__ __forceinline__ double dpp_mov(double x) {
    const long long b = __double_as_longlong(x);
    const int lo = __builtin_amdgcn_mov_dpp((int)(b & 0xffffffff), CTRL, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_mov_dpp((int)(b >> 32), CTRL, 0xF, 0xF, false);
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
template <int N, typename T>
__device__ __forceinline__ T dpp_ror(T x) { return dpp_mov<0x120 + N>(x); }
constexpr int kDppBcast15 = 0x142, kDppBcast31 = 0x143;

__device__ __forceinline__ float readlane_f(float x, int l) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), l));
}
__device__ __forceinline__ double readlane_f(double x, int l) {
    const long long b = __double_as_longlong(x);
    const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffff), l);
    const int hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

// Sum over the 64 lanes, identical in every lane.  Four DPP rotate steps make
// every lane of a 16-lane row k hold its row sum R_k (each step pairs lanes
// symmetrically, so all lanes of a row add the same two numbers); two
// row_bcast steps then leave (R3 + R2) + (R1 + R0) in row 3 (rows 0-2 end up
// with partial or meaningless values), and lane 63 is broadcast.  The result
// is bit-identical to (R0 + R1) + (R2 + R3).  No LDS traffic.
template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
    v += dpp_ror<8>(v);
    v += dpp_ror<4>(v);
    v += dpp_ror<2>(v);
    v += dpp_ror<1>(v);
    v += dpp_mov<kDppBcast15>(v);  // rows 1, 3: R1 + R0, R3 + R2
    v += dpp_mov<kDppBcast31>(v);  // row 3: (R3 + R2) + (R1 + R0)
    return readlane_f(v, 63);
}

// a / b for many a and one b, bit-identical to IEEE division: with y the
// correctly rounded 1/b, q = RN(a y) is within an ulp of a/b, the residual
// a - q b is exact by FMA, and RN(q + r y) is the correctly rounded quotient
// (Markstein's theorem; no overflow / underflow in our ranges).  3 ops
// instead of the ~10 of a full division.
template <typename T>
__device__ __forceinline__ T div_markstein(T a, T b, T y) {
    const T q = a * y;
    const T r = fma(-q, b, a);
    return fma(r, y, q);
}

// Keep a value in registers from here on: an empty asm that "modifies" it
// stops the compiler from re-loading it later from LDS (which would turn a
// one-step-ahead prefetch back into a load-and-wait at the point of use).
__device__ __forceinline__ void pin(double& x) { asm volatile("" : "+v"(x)); }
__device__ __forceinline__ void pin(float& x) { asm volatile("" : "+v"(x)); }
__device__ __forceinline__ void pin(uint64_t& x) { asm volatile("" : "+v"(x)); }
__device__ __forceinline__ void pin(double4& x) {
    pin(x.x);
    pin(x.y);
    pin(x.z);
    pin(x.w);
}

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }

// Order LDS traffic between the lanes of ONE wave (no workgroup barrier: the
// other waves of the block may be elsewhere).
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
}

// Read a wave-uniform 64-bit value held by lane `src` (src wave-uniform).
__device__ __forceinline__ uint64_t readlane_u64(uint64_t v, int src) {
    uint32_t lo = __builtin_amdgcn_readlane((int)(uint32_t)v, src);
    uint32_t hi = __builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), src);
    return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ int readlane_i32(int v, int src) { return __builtin_amdgcn_readlane(v, src); }

template <typename T, int CH>
struct RowReg {
    T v[CH][kVec];

    __device__ __forceinline__ void load(const T* __restrict__ row, int n) {
        const int l = lane_id();
#pragma unroll
        for (int c = 0; c < CH; ++c) {
            const int e = c * (kWave * kVec) + l * kVec;
            if (e < n) {
                // ld is a multiple of 2, so the pair stays inside the row.
                v[c][0] = row[e];
                v[c][1] = row[e + 1];
            } else {
                v[c][0] = T(0);
                v[c][1] = T(0);
            }
        }
    }

    __device__ __forceinline__ void store(T* __restrict__ row, int n) const {
        const int l = lane_id();
#pragma unroll
        for (int c = 0; c < CH; ++c) {
            const int e = c * (kWave * kVec) + l * kVec;
            if (e < n) row[e] = v[c][0];
            if (e + 1 < n) row[e + 1] = v[c][1];
        }
    }

    // sum of squares over the wave (common/utils.cpp:44-51 computes it serially)
    __device__ __forceinline__ T sumsq() const {
        T s = T(0);
#pragma unroll
        for (int c = 0; c < CH; ++c) s += v[c][0] * v[c][0] + v[c][1] * v[c][1];
        return wave_sum(s);
    }

    // common::norm (common/utils.cpp:70-77): scale to unit length if
    // !ignoreShort or the length exceeds 1.  Division, as the reference.
    __device__ __forceinline__ void norm(int n, bool ignore_short) {
        const T len = sqrt(sumsq());
        if (!ignore_short || len > T(1)) {
            const int l = lane_id();
#pragma unroll
            for (int c = 0; c < CH; ++c) {
                const int e = c * (kWave * kVec) + l * kVec;
                if (e < n) v[c][0] = v[c][0] / len;
                if (e + 1 < n) v[c][1] = v[c][1] / len;
            }
        }
    }
};

// Is element (c, k) of this lane inside the row?
__device__ __forceinline__ bool elem_valid(int c, int k, int n) {
    return c * (kWave * kVec) + lane_id() * kVec + k < n;
}

// Sign bits of an update direction x: word (c * 2 + k) holds, at bit l, the
// sign (x > 0) of element 128 c + 2 l + k.
__device__ __forceinline__ bool xbit(const uint64_t* words, int c, int k) {
    return (words[c * kVec + k] >> lane_id()) & 1ull;
}

// ---- diagnostic build only (make prof): per-phase cycle accounting
#ifdef KB2E_OWNER_PROF
constexpr int kProfOwners = 1024;
__device__ unsigned long long g_owner_prof[kProfOwners][16];  // relation owners
__device__ unsigned long long g_fold_prof[2][16];              // fold: [0] segments >= 512 events, [1] shorter
__device__ unsigned long long g_long_prof[16];                 // 4-wave long-segment fold
struct PhaseClock {
    unsigned long long t, acc[16];
    __device__ void start() {
        for (int k = 0; k < 16; ++k) acc[k] = 0;
        t = clock64();
    }
    __device__ void mark(int k) {
        const unsigned long long n = clock64();
        acc[k] += n - t;
        t = n;
    }
    __device__ void count(int k, unsigned long long v = 1) { acc[k] += v; }
    __device__ void flush(unsigned long long* dst) {
        if (lane_id() == 0 && dst)
            for (int k = 0; k < 16; ++k) atomicAdd(&dst[k], acc[k]);
    }
};
#define OWNER_PC_PARAM , PhaseClock& pc
#define OWNER_PC_ARG , pc
#define OWNER_MARK(k) pc.mark(k)
#define OWNER_COUNT(k) pc.count(k)
#else
#define OWNER_PC_PARAM
#define OWNER_PC_ARG
#define OWNER_MARK(k)
#define OWNER_COUNT(k)
#endif

// ---- event keys: [batch | row | kk | u | roles] (most to least significant)
struct KeyLayout {
    int kk_bits, row_bits, batch_bits;
    __host__ __device__ int kk_shift() const { return 4; }
    __host__ __device__ int row_shift() const { return 4 + kk_bits; }
    __host__ __device__ int batch_shift() const { return 4 + kk_bits + row_bits; }
    __host__ __device__ int total_bits() const { return 4 + kk_bits + row_bits + batch_bits; }
    __host__ __device__ uint64_t make(uint64_t batch, uint64_t row, uint64_t kk, uint64_t u,
                                      uint64_t roles) const {
        return (batch << batch_shift()) | (row << row_shift()) | (kk << kk_shift()) | (u << 3) | roles;
    }
    __host__ __device__ uint64_t seg_part(uint64_t key) const { return key >> row_shift(); }
    __host__ __device__ int batch_of(uint64_t key) const { return (int)(key >> batch_shift()); }
    __host__ __device__ int row_of(uint64_t key) const {
        return (int)((key >> row_shift()) & ((1ull << row_bits) - 1));
    }
    __host__ __device__ int kk_of(uint64_t key) const {
        return (int)((key >> kk_shift()) & ((1ull << kk_bits) - 1));
    }
};

constexpr uint64_t kSentinelKey = ~0ull;
enum : uint32_t { kRoleHead = 1, kRoleTail = 2, kRoleEntRel = 4 };

}  // namespace kb2e
