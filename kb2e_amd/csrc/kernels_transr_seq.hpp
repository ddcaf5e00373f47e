// kernels_transr_seq.hpp -- transRNorm of the PARALLEL TransR schedule per
// relation, the relation's pairs one after another, each against the matrix the
// earlier ones left (transr/trainer.cpp:35-64, :185-187; CPU model:
// oracle/parallel.py transr_constraint, cons="chunk1").
//
// Why per relation, in order.  The reference calls transRNorm(h', W'_r),
// transRNorm(t', W'_r) and transRNorm(entity'[r], W'_r) after every update of
// relation r, each on the matrix the previous calls left: a later pair only
// shrinks W'_r if it still violates |W^T a|^2 <= 1 after the earlier pairs'
// shrinks.  Computing every pair of the batch against the same W'_r and summing
// the corrections (the tile kernels' Jacobi form) over-shrinks W'_r along the
// directions the relation's entities share: on FB15k-shaped data the compat
// loss ends 20% below the reference's, outside its seed envelope
// (profiles/seed_envelope_r17_fb15k_R_compat.jsonl); in order it is inside
// (profiles/seed_envelope_r18_*).
//
// The pairs (the (h', r), (t', r) pairs of the active updates in (sample,
// update, role) order, first occurrences per relation per batch -- the gradient
// kernel's compacted lists bf.cpairs -- then (entity'[r], r)), per violator v
// (|p_v|^2 > 1, p_v = a_v W_c, a_v the entity row after its unit norm):
//   V = p_v K0                     (K0 = W'^T W', made at the relation's first violator)
//   the rounds of transRNorm's loop along p and w (transr_norm_rounds): with
//   v = V + |a|^2 p = kappa p + w, rho = 1 - 2 lr kappa,
//   m = the first round t with rho^2t |p|^2 + (2 lr t)^2 rho^(2t-2) |w|^2 <= 1,
//   g = 2 (S0 + 2 lr S1 kappa) p - 4 lr S1 v   (S0 = sum rho^t, S1 = sum t rho^(t-1))
//   W_c <- W_c - lr a_v^T g
// The pairs of the relation's last update and (entity'[r], r) come last, after
// W_c's rows are renormalised (the reference renormalises W' at every update, so
// only the last update's shrinks outlive the batch); the entity pass
// renormalises a row between the deltas of its earlier pairs and those of its
// own last update (bf.last_renorm, kernels_transr_parallel.hpp).
//
// This file holds the semantics above and what the chain kernels share (the
// rounds, wave sums, the block -> relation map, the pair records); the kernels
// are kernels_transr_pipe.hpp (n <= 64), kernels_transr_chainwp.hpp (64 < n <=
// 100), kernels_transr_chainw.hpp (the lockstep form) and kernels_transr_chaing.hpp
// (FP32 and the other widths).
#pragma once

#include "kernels_transr_mfma.hpp"

namespace kb2e {

constexpr int kChainRows = 32;      // pairs a chunk: two MFMA row tiles of projections and Gram rows
constexpr int kChainThreads = 256;  // four waves; wave w < NB owns column slice w
constexpr int kSeqMaxTiles = 256;   // tiles of one relation a window (the prefix table)

// KB2E_RPAR_STATS: 0 relations, 1 chunks, 2 violators, 3 rounds, 4 cycles sum, 5 max, 6 most chunks, 7 most rounds,
// 8..23 cycles of the phases (thread 0: prologue, load issue, S1 MFMA issue, S1 sums, B1, mask + K0, S3 MFMA
// issue, S3 sums, rows + B2, rounds, shuffles, S5, S6), 24..39 the same over relations of >= 40 chunks,
// 40 their chunks, 41 their count
static __device__ unsigned long long g_seq_stats[64];

// sums over the 16 lanes of a DPP row (lanes l & ~15 ... l | 15), in every lane of
// the row, of K values at once (independent chains, interleaved): the first four
// steps of wave_sum (kernels_common.hpp)
template <typename T, int K>
__device__ __forceinline__ void row16_sums(T (&v)[K]) {
#pragma unroll
    for (int k = 0; k < K; ++k) v[k] += dpp_ror<8>(v[k]);
#pragma unroll
    for (int k = 0; k < K; ++k) v[k] += dpp_ror<4>(v[k]);
#pragma unroll
    for (int k = 0; k < K; ++k) v[k] += dpp_ror<2>(v[k]);
#pragma unroll
    for (int k = 0; k < K; ++k) v[k] += dpp_ror<1>(v[k]);
}

// wave-wide sums of K values at once (interleaved DPP chains, kernels_common.hpp
// wave_sum), the totals in every lane
template <typename T, int K>
__device__ __forceinline__ void wave_sums(T (&v)[K]) {
    row16_sums<T, K>(v);
#pragma unroll
    for (int k = 0; k < K; ++k) v[k] += dpp_mov<kDppBcast15>(v[k]);
#pragma unroll
    for (int k = 0; k < K; ++k) v[k] += dpp_mov<kDppBcast31>(v[k]);
#pragma unroll
    for (int k = 0; k < K; ++k) v[k] = readlane_f(v[k], 63);
}

// The rounds m of transRNorm's loop and the sums S0 = sum_{t<m} rho^t,
// S1 = sum_{t<m} t rho^(t-1) (oracle/parallel.py transr_norm_rounds): m is the
// first t with rho^2t Q0 + eps^2 t^2 rho^(2t-2) w2 <= 1.  A handful of FMAs a
// round (m is 1-3 for almost every violator), cheaper than the closed form's pow.
template <typename T>
__device__ __forceinline__ int transr_rounds(T Q0, T w2, T eps, T rho, T& S0, T& S1) {
    const T e2w = eps * eps * w2;
    T rt = T(1), rtm1 = T(0);  // rho^t, rho^(t-1) (0 at t = 0)
    S0 = T(0);
    S1 = T(0);
    int m = 0;
    while (m < kRParMaxIter && rt * rt * Q0 + e2w * (T)m * (T)m * rtm1 * rtm1 > T(1)) {
        S0 += rt;
        S1 += (T)m * rtm1;
        rtm1 = rt;
        rt *= rho;
        ++m;
    }
    return m;
}

// transr_rounds for a violator (Q0 > 1: round 0 always runs), from round 1
template <typename T>
__device__ __forceinline__ int transr_rounds_violator(T Q0, T w2, T eps, T rho, T& S0, T& S1) {
    const T e2w = eps * eps * w2;
    T rt = rho, rtm1 = T(1);  // rho^t, rho^(t-1) at t = 1
    S0 = T(1);
    S1 = T(0);
    int m = 1;
    while (m < kRParMaxIter && rt * rt * Q0 + e2w * (T)m * (T)m * rtm1 * rtm1 > T(1)) {
        S0 += rt;
        S1 += (T)m * rtm1;
        rtm1 = rt;
        rt *= rho;
        ++m;
    }
    return m;
}

// transr_rounds_violator with the first four rounds as straight-line code: the
// powers rho^t are the loop's products (the same bits), the four tests are
// independent, and S0 / S1 add the same terms in the same order (+0 where a round
// does not run), so the results are bit-identical to the loop's.  A violator
// runs 1-3 rounds almost always (r21 counters: 2.8 on average); more than four
// continue in the loop.  Without the branches between rounds the tests overlap
// (a dependent FP64 chain of ~6 instead of ~25).
template <typename T>
__device__ __forceinline__ int transr_rounds_violator4(T Q0, T w2, T eps, T rho, T& S0, T& S1) {
    const T e2w = eps * eps * w2;
    const T r1 = rho, r2 = r1 * rho, r3 = r2 * rho, r4 = r3 * rho;
    // (bitwise &: no short-circuit branches between the tests)
    const bool c1 = r1 * r1 * Q0 + e2w * T(1) * T(1) * T(1) * T(1) > T(1);
    const bool c2 = c1 & (r2 * r2 * Q0 + e2w * T(2) * T(2) * r1 * r1 > T(1));
    const bool c3 = c2 & (r3 * r3 * Q0 + e2w * T(3) * T(3) * r2 * r2 > T(1));
    const bool c4 = c3 & (r4 * r4 * Q0 + e2w * T(4) * T(4) * r3 * r3 > T(1));
    S0 = T(1);
    S1 = T(0);
    S0 += c1 ? r1 : T(0);
    S1 += c1 ? T(1) * T(1) : T(0);
    S0 += c2 ? r2 : T(0);
    S1 += c2 ? T(2) * r1 : T(0);
    S0 += c3 ? r3 : T(0);
    S1 += c3 ? T(3) * r2 : T(0);
    S0 += c4 ? r4 : T(0);
    S1 += c4 ? T(4) * r3 : T(0);
    int m = 1 + (int)c1 + (int)c2 + (int)c3 + (int)c4;
    if (c4) {  // (uniform: every lane holds the same scalars)
        T rt = r4 * rho, rtm1 = r4;
        while (m < kRParMaxIter && rt * rt * Q0 + e2w * (T)m * (T)m * rtm1 * rtm1 > T(1)) {
            S0 += rt;
            S1 += (T)m * rtm1;
            rtm1 = rt;
            rt *= rho;
            ++m;
        }
    }
    return m;
}

// The chain kernels' block -> relation map: block b takes the batch's b-th most
// frequent relation (a.brel), so the hot relations' long chains start first instead
// of waiting for a dispatch slot behind short ones; its first tile g0 within the
// batch by binary search over the batch's tile relations (tiles follow the
// relation segments, sorted by relation).  False: the relation is not in the batch.
__device__ __forceinline__ bool chain_first_tile(const RParArgs& a, int t0, int t1, int& g0, int& r) {
    r = a.brel[blockIdx.x];
    int lo = t0, hi = t1;  // first tile with td_r >= r
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (a.td_r[mid] < r) lo = mid + 1;
        else hi = mid;
    }
    if (lo >= t1 || a.td_r[lo] != r) return false;
    g0 = lo - t0;
    return true;
}

// The relation's pair records G -> da = -lr W G with its final matrix
// (transr/trainer.cpp:59-60; first order in lr the same as the matrix at the
// pair's chunk), at the end of its chain: the nvt violator slots in vio (written
// during the chain), W_c in LDS (stride L), `stage` (stage_cap doubles) free LDS: [4][L] rows, then the slot list.  A wave a
// record: the G row staged in LDS, lane j makes da_j = sum_i W[j][i] G_i (four
// chains).  (Made here, the records of the ~440 relations that finish early
// overlap the hottest relation's chain instead of following it in a kernel of
// their own.)
template <typename T, int NP, int L>
__device__ __forceinline__ void chain_records(const RParArgs& a, const RParBufs<T>& bf, int r, const int32_t* vio,
                                              int nvt, const T* Wc, T* stage, int stage_cap) {
    const int n = a.n, ld = a.ld, w = threadIdx.x >> 6, l = lane_id();
    const int nw = blockDim.x >> 6;
    T* gs = stage + w * L;
    // the violator slots in LDS when they fit (after the waves' staged rows), so a
    // record's G row load waits on no global slot load; the rows prefetched PF
    // records ahead (a hot relation has ~150 records a batch: ~40 a wave)
    int* sl_l = (int*)(stage + nw * L);
    const bool lds_sl = nvt <= 2 * (stage_cap - nw * L);
    if (lds_sl) {
        for (int i = threadIdx.x; i < nvt; i += blockDim.x) sl_l[i] = vio[i];
        __syncthreads();
    }
    auto row_of = [&](int k) {
        const int sl = lds_sl ? sl_l[k] : vio[k];
        return sl >= 0 ? bf.pair + (int64_t)sl * ld : bf.relpair + (int64_t)r * ld;
    };
    constexpr int PF = 4;
    T pre[PF];
#pragma unroll
    for (int p = 0; p < PF; ++p) {
        const int k = w + p * nw;
        pre[p] = k < nvt && l < n ? row_of(k)[l] : T(0);
    }
    for (int k = w; k < nvt; k += nw) {
        T* row = row_of(k);
        if (l < NP) gs[l] = pre[0];
#pragma unroll
        for (int p = 0; p + 1 < PF; ++p) pre[p] = pre[p + 1];
        {
            const int kn = k + PF * nw;
            pre[PF - 1] = kn < nvt && l < n ? row_of(kn)[l] : T(0);
        }
        wave_lds_sync();
        T acc[4] = {T(0), T(0), T(0), T(0)};
        const int j = l < NP ? l : 0;
#pragma unroll
        for (int i = 0; i < NP; i += 4)
#pragma unroll
            for (int u = 0; u < 4; ++u) acc[u] = fma(Wc[j * L + i + u], gs[i + u], acc[u]);
        const T da = (acc[0] + acc[1]) + (acc[2] + acc[3]);
        wave_lds_sync();  // (every lane has read the staged row before the next one lands)
        if (l < n) row[l] = -(T)a.lr * da;
    }
}


}  // namespace kb2e
