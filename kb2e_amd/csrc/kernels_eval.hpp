// kernels_eval.hpp -- link-prediction evaluation (common/evaluation.cpp:124-251).
//
// For every test triple and both corruption sides the reference scores all
// |E| candidate triples, sorts them and reads off the raw rank (position of
// the true triple) and the filtered rank (1 + candidates ranked above it that
// are not known triples).  Here:
//   * eval_project_kernel writes the model's projection of every entity for
//     one relation into a TRANSPOSED table PT[k][i] (TransE: the entity rows;
//     TransH: e - (w.e) w, transh/transh.cpp:18-26; TransR: W^T e,
//     transr/transr.cpp:20-25 with zeroed work vectors), so a wave reading
//     dimension k of 64 consecutive entities is one coalesced load;
//   * eval_rank_kernel gives one thread per candidate entity and a tile of up
//     to kQ queries of that relation in LDS; each thread sums |(P(t) - P(h)) -
//     r| (or the squares) over k in the reference's serial order, so every
//     energy is bit-identical to the reference's FP64 value, and counts
//     candidates strictly below the true triple's energy (raw) and those of
//     them that are not in the filter set (filtered).
// Ties with the true energy are not counted (std::sort leaves their order
// unspecified; the oracle uses the same rule).
#pragma once

#include "kernels_common.hpp"
#include "kernels_sampler.hpp"  // dev_mix64

namespace kb2e {

constexpr int kQ = 16;

template <typename T>
struct EvalArgs {
    int32_t model, n, ld, ne, l1;
    const T* ent;
    const T* rel;
    const T* w;
    int32_t r;
    double* PT;    // [n][ne]
    double* relv;  // [n] relation r in FP64
};

// One thread per entity: its projection for relation r, in FP64, summed in the
// reference's order.
template <typename T>
__global__ __launch_bounds__(256) void eval_project_kernel(EvalArgs<T> a) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < a.n) a.relv[i] = (double)a.rel[(int64_t)a.r * a.ld + i];
    if (i >= a.ne) return;
    const T* e = a.ent + (int64_t)i * a.ld;
    if (a.model == 0) {
        for (int k = 0; k < a.n; ++k) a.PT[(int64_t)k * a.ne + i] = (double)e[k];
    } else if (a.model == 1) {
        const T* w = a.w + (int64_t)a.r * a.ld;
        double s = 0;
        for (int k = 0; k < a.n; ++k) s += (double)w[k] * (double)e[k];
        for (int k = 0; k < a.n; ++k) a.PT[(int64_t)k * a.ne + i] = (double)e[k] - s * (double)w[k];
    } else {
        const T* W = a.w + (int64_t)a.r * a.n * a.ld;
        for (int k = 0; k < a.n; ++k) {
            double s = 0;
            for (int j = 0; j < a.n; ++j) s += (double)W[(int64_t)j * a.ld + k] * (double)e[j];
            a.PT[(int64_t)k * a.ne + i] = s;
        }
    }
}

struct RankArgs {
    const double* PT;     // [n][ne]
    const double* relv;   // [n] relation vector (FP64)
    int32_t n, ne, l1;
    int32_t r;
    const int32_t* qh;    // queries of this relation
    const int32_t* qt;
    int32_t nq;
    const uint64_t* slots;  // eval filter (test + train + valid)
    uint64_t mask, nr64, ne64;
    unsigned long long* counts;  // [nq][2 sides][2: raw, filtered]
    double* target;              // [nq][2] true energies (head side, tail side)
};

__device__ __forceinline__ bool eval_filter_has(const RankArgs& a, int64_t h, int64_t t) {
    const uint64_t k = ((uint64_t)h * a.nr64 + (uint64_t)a.r) * a.ne64 + (uint64_t)t;
    uint64_t p = dev_mix64(k) & a.mask;
    while (true) {
        const uint64_t s = a.slots[p];
        if (s == k) return true;
        if (s == ~0ull) return false;
        p = (p + 1) & a.mask;
    }
}

// Energy of (h, t) from the projection table, serial over k (the reference's order).
__device__ __forceinline__ double eval_energy(const RankArgs& a, int h, int t) {
    double e = 0;
    for (int k = 0; k < a.n; ++k) {
        const double d = a.PT[(int64_t)k * a.ne + t] - a.PT[(int64_t)k * a.ne + h] - a.relv[k];
        e += a.l1 ? fabs(d) : d * d;
    }
    return e;
}

__global__ __launch_bounds__(256) void eval_target_kernel(RankArgs a) {
    const int q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= a.nq) return;
    const double e = eval_energy(a, a.qh[q], a.qt[q]);
    a.target[2 * q] = e;
    a.target[2 * q + 1] = e;
}

// grid.x: entity blocks of 256; grid.y: query tiles of kQ.
__global__ __launch_bounds__(256) void eval_rank_kernel(RankArgs a) {
    __shared__ double th[kQ][128], tt[kQ][128];  // P(true head), P(true tail), n <= 128
    __shared__ double rv[128];
    __shared__ unsigned int cnt[kQ][4];
    const int q0 = blockIdx.y * kQ;
    const int nq = min(kQ, a.nq - q0);
    for (int x = threadIdx.x; x < kQ * a.n; x += blockDim.x) {
        const int q = x / a.n, k = x % a.n;
        if (q < nq) {
            th[q][k] = a.PT[(int64_t)k * a.ne + a.qh[q0 + q]];
            tt[q][k] = a.PT[(int64_t)k * a.ne + a.qt[q0 + q]];
        }
    }
    for (int k = threadIdx.x; k < a.n; k += blockDim.x) rv[k] = a.relv[k];
    if (threadIdx.x < kQ * 4) cnt[threadIdx.x / 4][threadIdx.x % 4] = 0;
    __syncthreads();
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < a.ne) {
        double eh[kQ], et[kQ];  // head replaced by i / tail replaced by i
#pragma unroll
        for (int q = 0; q < kQ; ++q) eh[q] = et[q] = 0;
        for (int k = 0; k < a.n; ++k) {
            const double v = a.PT[(int64_t)k * a.ne + i];
            const double r = rv[k];
#pragma unroll
            for (int q = 0; q < kQ; ++q) {
                const double dh = tt[q][k] - v - r;   // (P(t) - P(i)) - r
                const double dt = v - th[q][k] - r;   // (P(i) - P(h)) - r
                eh[q] += a.l1 ? fabs(dh) : dh * dh;
                et[q] += a.l1 ? fabs(dt) : dt * dt;
            }
        }
#pragma unroll
        for (int q = 0; q < kQ; ++q) {
            if (q >= nq) continue;
            const int h = a.qh[q0 + q], t = a.qt[q0 + q];
            const double target = a.target[2 * (q0 + q)];
            if (i != h && eh[q] < target) {
                atomicAdd(&cnt[q][0], 1u);
                if (!eval_filter_has(a, i, t)) atomicAdd(&cnt[q][1], 1u);
            }
            if (i != t && et[q] < target) {
                atomicAdd(&cnt[q][2], 1u);
                if (!eval_filter_has(a, h, i)) atomicAdd(&cnt[q][3], 1u);
            }
        }
    }
    __syncthreads();
    if (threadIdx.x < nq * 4) {
        const int q = threadIdx.x / 4, c = threadIdx.x % 4;
        if (cnt[q][c]) atomicAdd(&a.counts[(int64_t)(q0 + q) * 4 + c], (unsigned long long)cnt[q][c]);
    }
}

}  // namespace kb2e
