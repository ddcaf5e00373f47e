// kernels_parallel.hpp -- phase B of the PARALLEL schedule (kb2e_config.schedule
// = KB2E_SCHEDULE_PARALLEL).
//
// The reference computes every update direction of a batch from the
// start-of-batch snapshot (common/trainer.cpp:130-149 via prebatch/postbatch,
// transe/trainer.cpp:48-56) and then applies the updates one sample at a time,
// renormalising after each (transe/trainer.cpp:38-45).  The ORDERED schedule
// (kernels_transe.hpp, kernels_relowner.hpp) replays exactly that sequence.
// The PARALLEL schedule keeps the snapshot gradients -- the same sample stream,
// energies, hinge decisions and update directions -- and applies each row's
// summed delta once, followed by one common::norm:
//
//     next_row = norm(row + sum_k delta_k)            (ordered: norm(...norm(row + delta_0)... + delta_k))
//
// A row with one event per batch gets exactly the reference's value; a row with
// several events differs at O(lr^2).  Every row is owned by one wave (or one
// workgroup for long segments), accumulation order is fixed: the result is
// deterministic.  HBM-bound: each event reads its sign words (L1) or direction
// row (L2); each touched row is read and written once.
#pragma once

#include "kernels_transe.hpp"

namespace kb2e {

// Per-lane accumulator of one row's summed delta: L1 keeps the integer count
// sum_k s_k x_k (x_k in {+-1}, exact), L2 the real sum sum_k s_k x_k.
template <typename T, int CH, bool L1>
struct DeltaAcc {
    using A = typename std::conditional<L1, int, double>::type;
    A v[CH][kVec];
    bool dirty;  // some active event normalises the row
    __device__ __forceinline__ void zero() {
#pragma unroll
        for (int c = 0; c < CH; ++c)
#pragma unroll
            for (int k = 0; k < kVec; ++k) v[c][k] = A(0);
        dirty = false;
    }
};

// Transpose a 64 x 64 bit matrix held one row per lane: afterwards bit e of
// lane l is bit l of lane e's input.  Six block-swap stages (rows e and e ^ j
// exchange the off-diagonal j x j blocks); stage 32 is one v_permlane32_swap
// of the word halves, the others are lane shuffles.
__device__ __forceinline__ uint64_t wave_transpose64(uint64_t x) {
    const int l = lane_id();
    uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
    {  // j = 32: lanes < 32 take the partner's low half as their high half, and back
        const auto r = __builtin_amdgcn_permlane32_swap(lo, hi, false, false);
        lo = r[0];
        hi = r[1];
    }
    x = ((uint64_t)hi << 32) | lo;
    constexpr uint64_t kMask[5] = {0xFFFF0000FFFF0000ull, 0xFF00FF00FF00FF00ull, 0xF0F0F0F0F0F0F0F0ull,
                                   0xCCCCCCCCCCCCCCCCull, 0xAAAAAAAAAAAAAAAAull};
#pragma unroll
    for (int q = 0; q < 5; ++q) {
        const int j = 16 >> q;
        const uint64_t M = kMask[q];
        const uint32_t ylo = (uint32_t)__shfl_xor((int)(uint32_t)x, j);
        const uint32_t yhi = (uint32_t)__shfl_xor((int)(uint32_t)(x >> 32), j);
        const uint64_t y = ((uint64_t)yhi << 32) | ylo;
        x = (l & j) ? ((x & M) | ((y >> j) & ~M)) : ((x & ~M) | ((y << j) & M));
    }
    return x;
}

template <typename T, int CH, bool L1>
struct ApplyChunk {
    uint64_t xw[2 * CH];
    int sgn, nn, xrow;
    __device__ __forceinline__ void load(const FoldArgs<T>& a, const EventRecs& er, int base, int p1) {
        const int l = lane_id();
        const bool valid = base + l < p1;
        const int32_t meta = valid ? er.meta[base + l] : 1;
        sgn = (meta & 3) - 1;
        nn = (meta >> 2) & 3;
        xrow = meta >> 4;
#pragma unroll
        for (int q = 0; q < 2 * CH; ++q) xw[q] = 0ull;
        if (L1 && valid) {  // same load level as meta; events with s = 0 are masked out later
#pragma unroll
            for (int q = 0; q < 2 * CH; ++q)
                if (q < a.nw) xw[q] = er.words[(int64_t)(base + l) * a.nw + q];
        }
    }
};

// Accumulate chunks first, first + stride, ... of segment [p0, p1).
// L1: per sign word, transpose the chunk's 64 words so lane l holds element
// l's 64 sign bits, then sum_k s_k x_k = 2 (#{s=+1, bit} - #{s=-1, bit})
// - #{s=+1} + #{s=-1}: popcounts instead of a per-event loop.
template <typename T, int CH, bool L1>
__device__ __forceinline__ void accumulate_segment(const FoldArgs<T>& a, const EventRecs& er, int p0, int p1,
                                                   int first, int stride, DeltaAcc<T, CH, L1>& acc) {
    const int l = lane_id();
    for (int base = p0 + first * kWave; base < p1; base += stride * kWave) {
        ApplyChunk<T, CH, L1> ck;
        ck.load(a, er, base, p1);
        if (__ballot(ck.nn > 0)) acc.dirty = true;
        if (L1) {
            const uint64_t mp = __ballot(ck.sgn > 0), mn = __ballot(ck.sgn < 0);
            if (!(mp | mn)) continue;
            const int bias = __popcll(mn) - __popcll(mp);
#pragma unroll
            for (int c = 0; c < CH; ++c)
#pragma unroll
                for (int k = 0; k < kVec; ++k) {
                    if (c * (kWave * kVec) >= a.n) continue;  // wave-uniform: chunk past the row
                    const uint64_t col = wave_transpose64(ck.xw[c * kVec + k]);
                    acc.v[c][k] += 2 * (__popcll(col & mp) - __popcll(col & mn)) + bias;
                }
        } else {
            uint64_t m = __ballot(ck.sgn != 0);
            while (m) {
                const int e = __builtin_ctzll(m);
                m &= m - 1;
                const int s = readlane_i32(ck.sgn, e);
                const T* xr = a.xreal + (int64_t)readlane_i32(ck.xrow, e) * a.ld;
#pragma unroll
                for (int c = 0; c < CH; ++c)
#pragma unroll
                    for (int k = 0; k < kVec; ++k) {
                        const int el = c * (kWave * kVec) + l * kVec + k;
                        if (el < a.n) acc.v[c][k] += (double)s * (double)xr[el];
                    }
            }
        }
    }
}

// row <- norm(row + lr * acc)  (transe/trainer.cpp:38-45 with the deltas summed);
// V holds the row as loaded.
template <typename T, int CH, bool L1>
__device__ __forceinline__ void apply_row(const FoldArgs<T>& a, T* ptr, RowReg<T, CH>& V,
                                          const DeltaAcc<T, CH, L1>& acc) {
    if (!acc.dirty) return;
#pragma unroll
    for (int c = 0; c < CH; ++c)
#pragma unroll
        for (int k = 0; k < kVec; ++k)
            if (elem_valid(c, k, a.n)) V.v[c][k] = V.v[c][k] + (T)(a.lr * (double)acc.v[c][k]);
    V.norm(a.n, true);
    V.store(ptr, a.n);
}

template <typename T>
__device__ __forceinline__ T* row_ptr(const FoldArgs<T>& a, int row) {
    return row >= a.ne ? a.rel + (int64_t)(row - a.ne) * a.ld : a.ent + (int64_t)row * a.ld;
}

// Per epoch: position of every emitted key in the sorted order, and the row of
// every segment.
__global__ __launch_bounds__(256) void inverse_perm_kernel(const int32_t* sorted_slot, int64_t n, int32_t* inv) {
    const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p < n) inv[sorted_slot[p]] = (int32_t)p;
}

__global__ __launch_bounds__(256) void seg_rows_kernel(const uint64_t* keys, const int32_t* seg_start,
                                                       const int32_t* nseg_p, KeyLayout kl, int32_t* seg_row) {
    const int nseg = *nseg_p;
    for (int s = blockIdx.x * blockDim.x + threadIdx.x; s < nseg; s += gridDim.x * blockDim.x)
        seg_row[s] = kl.row_of(keys[seg_start[s]]);
}

// Per epoch: the (batch, row) segments with at least long_min events, listed
// per batch (list[b * cap ...], count[b]).
__global__ __launch_bounds__(1024) void long_lists_kernel(const int32_t* seg_start, const int32_t* batch_seg,
                                                          int32_t long_min, int32_t cap, int32_t* list,
                                                          int32_t* count) {
    __shared__ int n;
    if (threadIdx.x == 0) n = 0;
    __syncthreads();
    const int b = blockIdx.x;
    const int s0 = batch_seg[b], s1 = batch_seg[b + 1];
    for (int s = s0 + threadIdx.x; s < s1; s += blockDim.x)
        if (seg_start[s + 1] - seg_start[s] >= long_min) {
            const int q = atomicAdd(&n, 1);
            if (q < cap) list[(int64_t)b * cap + q] = s;
        }
    __syncthreads();
    if (threadIdx.x == 0) count[b] = min(n, cap);
}

// Phase B of one batch in one launch of 1024-thread workgroups.  Long segments
// (the hot relations and entities): one workgroup each, its 16 waves taking
// interleaved chunks, partial sums combined in wave order through LDS.  All
// other segments: one wave each; workgroups that had a long segment take the
// last share of them.
constexpr int kApplyWaves = 16;

// (the body takes its workgroup index and count: TransH runs it in one launch
// with the relation-normal sums, transh_phase_b_kernel; arguments by value)
template <typename T, int CH, bool L1>
__device__ __forceinline__ void transe_apply_body(FoldArgs<T> a, EventRecs er, const int32_t* long_list,
                                                  const int32_t* long_count, int32_t cap, int bid, int G) {
    using A = typename DeltaAcc<T, CH, L1>::A;
    __shared__ A part[kApplyWaves][CH * kVec][kWave];
    __shared__ int dirty_any;
    const int w = threadIdx.x >> 6, l = lane_id();
    const int nlong = a.long_min > 0 ? long_count[a.batch] : 0;
    const int32_t* list = long_list + (int64_t)a.batch * cap;
    for (int q = bid; q < nlong; q += G) {
        const int s = list[q];
        const int p0 = a.seg_start[s], p1 = a.seg_start[s + 1];
        T* ptr = row_ptr(a, er.seg_row[s]);
        RowReg<T, CH> V;
        if (w == 0) V.load(ptr, a.n);  // in flight while the events are summed
        if (threadIdx.x == 0) dirty_any = 0;
        __syncthreads();
        DeltaAcc<T, CH, L1> acc;
        acc.zero();
        accumulate_segment<T, CH, L1>(a, er, p0, p1, w, kApplyWaves, acc);
#pragma unroll
        for (int c = 0; c < CH; ++c)
#pragma unroll
            for (int k = 0; k < kVec; ++k) part[w][c * kVec + k][l] = acc.v[c][k];
        if (acc.dirty && l == 0) dirty_any = 1;
        __syncthreads();
        if (w == 0) {
#pragma unroll
            for (int c = 0; c < CH; ++c)
#pragma unroll
                for (int k = 0; k < kVec; ++k) {
                    A sum = part[0][c * kVec + k][l];
                    for (int v = 1; v < kApplyWaves; ++v) sum += part[v][c * kVec + k][l];
                    acc.v[c][k] = sum;
                }
            acc.dirty = dirty_any != 0;
            apply_row<T, CH, L1>(a, ptr, V, acc);
        }
        __syncthreads();
    }
    const int s0 = a.batch_seg[a.batch], s1 = a.batch_seg[a.batch + 1];
    const int rot = (bid + G - (nlong % G)) % G;
    const int wave = rot * kApplyWaves + w;
    for (int s = s0 + wave; s < s1; s += G * kApplyWaves) {
        const int p0 = a.seg_start[s], p1 = a.seg_start[s + 1];
        if (a.long_min > 0 && p1 - p0 >= a.long_min) continue;
        T* ptr = row_ptr(a, er.seg_row[s]);
        RowReg<T, CH> V;
        V.load(ptr, a.n);  // in flight while the events are summed
        DeltaAcc<T, CH, L1> acc;
        acc.zero();
        accumulate_segment<T, CH, L1>(a, er, p0, p1, 0, 1, acc);
        apply_row<T, CH, L1>(a, ptr, V, acc);
    }
}

template <typename T, int CH, bool L1>
__global__ __launch_bounds__(1024) void transe_apply_kernel(FoldArgs<T> a, EventRecs er, const int32_t* long_list,
                                                            const int32_t* long_count, int32_t cap) {
    transe_apply_body<T, CH, L1>(a, er, long_list, long_count, cap, blockIdx.x, gridDim.x);
}

}  // namespace kb2e
