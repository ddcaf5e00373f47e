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
// The work is cut so that only the violators are sequential.  Per chunk of 32
// pairs, all four waves make P = A W_c and the Gram matrix A A^T on the matrix
// cores (16 x 16 tiles); then one wave walks the chunk's pairs: the first pair
// with |p_j|^2 > 1 is the next violator v, its V row, scalars, rounds and g are
// made with lane c holding column c, and its shrink reaches every later pair of
// the chunk as P_j -= lr (a_j . a_v) g (the Gram entry), |p_j|^2 made afresh --
// no barrier between violators.  The chunk's violators then update W_c (the G
// rows kept in P), before the next chunk's P.  ~1.7 of 16 pairs violate on
// FB15k-shaped data.  The pair records da = -lr W G are made at the end of the
// relation's chain over its final matrix (chain_records: first order the same).
#pragma once

#include "kernels_transr_mfma.hpp"

namespace kb2e {

constexpr int kChainRows = 32;      // pairs a chunk: two MFMA row tiles of projections and Gram rows
constexpr int kChainThreads = 256;  // four waves; wave w < NB owns column slice w
constexpr int kSeqMaxTiles = 256;   // tiles of one relation a window (the prefix table)
constexpr int kChainList = 2048;    // pairs of one relation a window (entity and slot lists in LDS)

// LDS (elements of T): W_c [NP][L] | K0 [NP][L] | A [2][R][L] | P [R][L] |
// Gram [R][R + 1] | |p|^2 partials [4][R] | row partials [4][NP] ; ints: pair
// entities, slots [2][kChainList] | pre [kSeqMaxTiles + 1] | misc [8]
template <typename T>
__host__ __device__ constexpr size_t chain_lds(int n) {
    return sizeof(T) * ((size_t)rm_np(n) * rm_ld(n) * 2 + 3 * (size_t)kChainRows * rm_ld(n) +
                        (size_t)kChainRows * (kChainRows + 1) + 4 * kChainRows + 4 * (size_t)rm_np(n)) +
           sizeof(int) * (size_t)(2 * kChainList + kSeqMaxTiles + 1 + 8);
}

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

// The chain kernels' block -> relation map: block b takes the b-th most frequent
// relation (a.rel_order), so the hot relations' long chains start first instead
// of waiting for a dispatch slot behind short ones; its first tile g0 within the
// batch by binary search over the batch's tile relations (tiles follow the
// relation segments, sorted by relation).  False: the relation is not in the batch.
__device__ __forceinline__ bool chain_first_tile(const RParArgs& a, int t0, int t1, int& g0, int& r) {
    r = a.rel_order[blockIdx.x];
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

// KS = ceil(n / 4): the live k-steps of a contraction over n, a compile-time
// count so that the MFMA chains are straight-line code (no per-step branches)
template <typename T, int KS>
__global__ __launch_bounds__(kChainThreads) void transr_cons_chain_kernel(RParArgs a, RParBufs<T> bf) {
    using M = Mfma16<T>;
    static_assert(sizeof(T) == 8, "the D-row / k-step identity below is the FP64 fragment layout");
    constexpr int NB = (4 * KS + 15) / 16;  // column slices of 16
    constexpr int NP = 16 * NB, L = NP + 2, R = kChainRows, LG = R + 1;
    const int t0 = a.batch_t0[a.batch], t1 = a.batch_t0[a.batch + 1];
    int g0, r;  // the relation's first tile within the batch
    if (!chain_first_tile(a, t0, t1, g0, r)) return;
    const int n = a.n, ld = a.ld;
    const int w = threadIdx.x >> 6, l = lane_id(), kq = l >> 4, l16 = l & 15;
    const bool mine = w < NB;  // this wave owns a column slice (K0, the W_c update)
    const int col = 16 * w + l16;
    const T lr = (T)a.lr;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    T* Wc = (T*)smem;
    T* K0 = Wc + NP * L;
    T* Abuf = K0 + NP * L;      // [2][R][L] the chunk's entity rows (double buffered)
    T* P = Abuf + 2 * R * L;    // [R][L] projections, then G rows of the violators
    T* Gm = P + R * L;          // [R][LG] Gram matrix A A^T of the chunk
    T* qpart = Gm + R * LG;     // [NB][R] |p|^2 partials of the column slices
    T* rp = qpart + 4 * R;      // [4][NP] row partials of the tail renorm
    int* pe = (int*)(rp + 4 * NP);  // the window's pairs: entities [kChainList], slots [kChainList]
    int* ps = pe + kChainList;
    int* pre = ps + kChainList;
    int* misc = pre + kSeqMaxTiles + 1;
    const long long ck0 = clock64();
    unsigned long long n_chunks = 0, n_vio = 0, n_rounds = 0, max_m = 0;
    unsigned long long ph[16] = {};  // stats: cycles of the phases (thread 0; see g_seq_stats)
    long long tq = ck0;
    auto tick = [&](int k) {
        if (bf.stats && threadIdx.x == 0) {
            const long long t = clock64();
            ph[k] += (unsigned long long)(t - tq);
            tq = t;
        }
    };

    // W'_r, zero padded to NP x NP
    for (int idx = threadIdx.x; idx < NP * NP; idx += kChainThreads) {
        const int j = idx / NP, i = idx % NP;
        Wc[j * L + i] = (j < n && i < n) ? bf.W[((int64_t)r * n + j) * ld + i] : T(0);
    }
    // The relation's pairs in order: its tiles' compacted lists, except that the
    // (entity'[r], r) pair, which the gradient kernel appends to the relation's
    // first tile, goes last (the order, and so the result, does not depend on the
    // tile size); the relation's last active sample kl, its tile, and how many
    // of the pairs belong to kl's corrupted-triple update (the tail).
    if (w == 0) {
        int run = 0;
        for (int m0 = 0;; m0 += kWave) {
            const int g = g0 + m0 + l;
            const uint64_t b = __ballot(t0 + g < t1 && a.td_r[t0 + g] == r);
            const int k = b == ~0ull ? kWave : __builtin_ctzll(~b);
            run += k;
            if (k < kWave) break;
        }
        const int c0 = bf.cnrows[g0] & 127;
        const int rel = c0 > 0 && bf.cpairs[(int64_t)g0 * 2 * kCPairs + kCPairs + c0 - 1] == -2;
        int kl = -1, gt = -1;
        for (int g = g0 + run - 1; g >= g0 && kl < 0; --g) {
            const int cs = a.td_cnt[t0 + g] & 255;
            const int kk = l < cs ? a.td_kk[(t0 + g) * 8 + l] : -1;
            const uint64_t b = __ballot(kk >= 0 && a.act[kk]);
            if (b) {
                kl = __shfl(kk, 63 - __builtin_clzll(b));
                gt = g;
            }
        }
        int ntail = 0;
        if (gt >= 0) {
            const int cp = bf.cnrows[gt] & 127;
            const int sl = l < cp ? bf.cpairs[(int64_t)gt * 2 * kCPairs + kCPairs + l] : -3;
            ntail = __builtin_popcountll(__ballot(sl >= 0 && (sl >> 1) == kl * 2 + 1));
        }
        if (l == 0) {
            misc[3] = rel;
            misc[4] = gt;
            misc[5] = run;
            misc[6] = ntail;
        }
    }
    __syncthreads();
    const int run = misc[5], has_rel = misc[3], g_tail = misc[4], n_tail = misc[6];
    bool have_k0 = false, changed = false;
    int32_t* const vio = bf.vio + (int64_t)g0 * kCPairs;  // the relation's violators (run * kCPairs >= its pairs)
    int nvt = 0;
    T k0c[4 * KS];  // wave 0: K0's column l (the violators' V rows), loaded once K0 is made
    tick(0);
    int chunk_no = 0;  // chunks so far (row buffer parity)
    const int tile_cap = bf.chain_tiles >= 1 && bf.chain_tiles < kSeqMaxTiles ? bf.chain_tiles : kSeqMaxTiles;
    // windows of at most kSeqMaxTiles tiles and kChainList - 1 pairs (FB15k's hottest
    // relation holds ~1000 pairs a batch: one window)
    for (int gw = g0; gw < g0 + run || gw == g0;) {
        if (w == 0) {  // exclusive prefix of the window's tile pair counts (the relation pair left out)
            const int nt = g0 + run - gw < tile_cap ? g0 + run - gw : tile_cap;
            int carry = 0, fit = 0;
            for (int m0 = 0; m0 < nt; m0 += kWave) {
                const int g = m0 + l;
                int c = g < nt ? (bf.cnrows[gw + g] & 127) : 0;
                if (gw + g == g0 && has_rel) c -= 1;
                int x = c;
#pragma unroll
                for (int s = 1; s < kWave; s <<= 1) {
                    const int y = __shfl_up(x, s);
                    if (l >= s) x += y;
                }
                if (g < nt) pre[g] = carry + x - c;
                // tiles whose pairs (and the relation pair) still fit the list
                fit += __builtin_popcountll(__ballot(g < nt && carry + x <= kChainList - 1));
                carry += __shfl(x, kWave - 1);
            }
            if (l == 0) {
                if (fit == nt) pre[nt] = carry;
                misc[0] = fit;
            }
        }
        __syncthreads();
        const int ntile = misc[0];
        // the window holding the relation's last active sample is its last: the
        // tiles after it hold no pairs (only inactive samples), so a window cut by
        // the tile cap after it would otherwise lose the tail's renorm
        const bool last = gw + ntile == g0 + run || (g_tail >= 0 && gw + ntile > g_tail);
        const int ntp = pre[ntile];
        const int npairs = ntp + (last && has_rel ? 1 : 0);
        const int tail_start = last && g_tail >= gw ? ntp - n_tail : npairs;
        // the window's pairs into LDS, every thread a pair at a time
        for (int f = threadIdx.x; f < npairs; f += kChainThreads) {
            int e = r, sl = -2;
            if (f < ntp) {
                int lo = 0, hi = ntile - 1;
                while (lo < hi) {
                    const int mid = (lo + hi + 1) >> 1;
                    if (pre[mid] <= f) lo = mid;
                    else hi = mid - 1;
                }
                const int32_t* cp = bf.cpairs + (int64_t)(gw + lo) * 2 * kCPairs;
                e = cp[f - pre[lo]];
                sl = cp[kCPairs + f - pre[lo]];
            }
            pe[f] = e;
            ps[f] = sl;
        }
        // chunks of R pairs; the relation's last update's pairs (and (entity'[r], r)) alone
        auto chunk_end = [&](int b) {
            return b < tail_start ? (b + R < tail_start ? b + R : tail_start) : npairs;
        };
        // rows of the chunk [b, e): R x NP elements, R NP / 256 a thread, into registers.
        // Every load is issued (a valid address when the element is padding) and the
        // padding zeroed when stored, so no register is written under a branch while a
        // load into it may be in flight.
        constexpr int kRowsPer = R * NP / kChainThreads;
        T rows[kRowsPer];
        uint32_t rows_ok = 0;
        auto load_rows = [&](int b, int e) {
            int ent[kRowsPer];
#pragma unroll
            for (int q = 0; q < kRowsPer; ++q) {
                const int f = b + (threadIdx.x + q * kChainThreads) / NP;
                ent[q] = pe[f < kChainList ? f : kChainList - 1];
            }
            rows_ok = 0;
#pragma unroll
            for (int q = 0; q < kRowsPer; ++q) {
                const int idx = threadIdx.x + q * kChainThreads;
                const int k = idx / NP, j = idx % NP;
                const bool ok = b + k < e && ent[q] >= 0 && j < n;
                rows[q] = bf.ent[ok ? (uint32_t)ent[q] * (uint32_t)ld + (uint32_t)j : 0u];
                rows_ok |= (ok ? 1u : 0u) << q;
            }
        };
        auto store_rows = [&](int b) {
#pragma unroll
            for (int q = 0; q < kRowsPer; ++q) {
                const int idx = threadIdx.x + q * kChainThreads;
                Abuf[b * R * L + (idx / NP) * L + idx % NP] = ((rows_ok >> q) & 1) ? rows[q] : T(0);
            }
        };
        __syncthreads();
        {
            const int e0 = chunk_end(0);
            load_rows(0, e0);
            store_rows(chunk_no & 1);
            load_rows(e0, e0 < npairs ? chunk_end(e0) : e0);  // the second chunk's rows in flight
        }
        __syncthreads();
        for (int base = 0; base < npairs; ++chunk_no) {
            const int nbase = chunk_end(base);
            const int cc = nbase - base;
            const int nrt = cc > 16 ? 2 : 1;  // row tiles of the chunk
            const T* A = Abuf + (chunk_no & 1) * R * L;
            ++n_chunks;
            if (base == tail_start && changed) {
                // the relation's last update renormalises the rows before its own pairs'
                // shrinks (transr/trainer.cpp:178-180): row sums over the slices, then each
                // wave scales its own columns
                if (mine && l < NP) {
                    T sq = T(0);
                    if (l < n)
                        for (int i = 0; i < 16; ++i) sq += Wc[l * L + 16 * w + i] * Wc[l * L + 16 * w + i];
                    rp[w * NP + l] = sq;
                }
                __syncthreads();
                if (mine && l < n) {
                    T ss = rp[l];
                    for (int v = 1; v < NB; ++v) ss += rp[v * NP + l];
                    const T len = sqrt(ss);
                    for (int i = 0; i < 16; ++i) Wc[l * L + 16 * w + i] = Wc[l * L + 16 * w + i] / len;
                }
                __syncthreads();
            }
            tick(1);
            // Phase A, all waves: P = A W_c and the Gram matrix A A^T of the chunk, 16 x 16
            // MFMA tiles dealt round the waves; |p|^2 partials per column slice.
            {
                // Gram tiles (0, 0), (1, 0), (1, 1): only a_j . a_v with j > v is read
                const int ntiles = nrt * NB + (nrt == 2 ? 3 : 1);
                for (int tl = w; tl < ntiles; tl += kChainThreads / kWave) {
                    const bool gram = tl >= nrt * NB;
                    const int gi = tl - nrt * NB;
                    const int rt = gram ? (gi == 0 ? 0 : 1) : tl / NB;
                    const int cb = gram ? (gi == 2 ? 1 : 0) : tl % NB;
                    typename M::acc_t acc = {T(0), T(0), T(0), T(0)};
                    T av[KS], bv[KS];
#pragma unroll
                    for (int s = 0; s < KS; ++s) {
                        av[s] = A[(rt * 16 + l16) * L + 4 * s + kq];
                        bv[s] = gram ? A[(cb * 16 + l16) * L + 4 * s + kq] : Wc[(4 * s + kq) * L + cb * 16 + l16];
                    }
#pragma unroll
                    for (int s = 0; s < KS; ++s) acc = M::mma(av[s], bv[s], acc);
                    if (gram) {
#pragma unroll
                        for (int q = 0; q < 4; ++q) Gm[(rt * 16 + kq + 4 * q) * LG + cb * 16 + l16] = acc[q];
                    } else {
                        T sp[4];
#pragma unroll
                        for (int q = 0; q < 4; ++q) {
                            P[(rt * 16 + kq + 4 * q) * L + cb * 16 + l16] = acc[q];
                            sp[q] = acc[q] * acc[q];
                        }
                        row16_sums<T, 4>(sp);
                        if (l16 == 0) {
#pragma unroll
                            for (int q = 0; q < 4; ++q) qpart[cb * R + rt * 16 + kq + 4 * q] = sp[q];
                        }
                    }
                }
            }
            // the next chunk's rows (loaded a chunk ago) into the other buffer, then the
            // rows of the chunk after it in flight for a whole chunk (before wave 0's
            // record stores: waiting for a load waits for every global access issued
            // before it)
            store_rows((chunk_no & 1) ^ 1);  // (zeros past the window's last chunk: unread)
            {
                const int n2 = nbase < npairs ? chunk_end(nbase) : nbase;
                load_rows(n2, n2 < npairs ? chunk_end(n2) : n2);
            }
            __syncthreads();  // B1
            tick(2);
            // |p_j|^2 of pair j on lanes j and j + 32 of every wave
            const int j = l & (R - 1);
            T q = T(0);
            if (j < cc) {
                q = qpart[j];
                for (int v = 1; v < NB; ++v) q += qpart[v * R + j];
            }
            const bool anyv = __ballot(j < cc && q > T(1)) != 0;
            if (anyv && !have_k0) {  // K0[:, slice] = W^T W[:, slice] (W_c is still W'_r here)
                have_k0 = true;
                if (mine) {
#pragma unroll
                    for (int ib = 0; ib < NB; ++ib) {
                        typename M::acc_t acc = {T(0), T(0), T(0), T(0)};
                        T av[KS], bv[KS];
#pragma unroll
                        for (int s = 0; s < KS; ++s) {
                            av[s] = Wc[(4 * s + kq) * L + ib * 16 + l16];
                            bv[s] = Wc[(4 * s + kq) * L + col];
                        }
#pragma unroll
                        for (int s = 0; s < KS; ++s) acc = M::mma(av[s], bv[s], acc);
#pragma unroll
                        for (int qq = 0; qq < 4; ++qq) K0[(ib * 16 + kq + 4 * qq) * L + col] = acc[qq];
                    }
                }
                __syncthreads();
                if (w == 0) {
                    const int cK = l < NP ? l : 0;
#pragma unroll
                    for (int i = 0; i < 4 * KS; ++i) k0c[i] = K0[i * L + cK];
                }
            }
            tick(3);
            // Phase B, wave 0: the pairs in order, each against the matrix the earlier
            // ones left (transr/trainer.cpp:35-64 per pair).  A violator v's shrink
            // W_c -= lr a_v^T g_v moves every later pair's projection by
            // -lr (a_j . a_v) g_v: applied to the P rows and |p_j|^2 at once; lane c
            // holds column c for the violator's own quantities.
            if (w == 0 && anyv) {
                uint32_t vmask = 0;
                int cursor = 0;
                const T eps = T(2) * lr;
                for (;;) {
                    const uint64_t cand = __ballot(l < R && j < cc && j >= cursor && q > T(1));
                    if (!cand) break;
                    const int v = __builtin_ctzll(cand);
                    const int c = l;  // column
                    const T pv = c < NP ? P[v * L + c] : T(0);
                    // V[c] = sum_i p_v[i] K0[i][c] (K0's column c in lane c's registers), four chains
                    T vv4[4] = {T(0), T(0), T(0), T(0)};
#pragma unroll
                    for (int t = 0; t < KS; ++t)
#pragma unroll
                        for (int u = 0; u < 4; ++u) vv4[u] = fma(P[v * L + 4 * t + u], k0c[4 * t + u], vv4[u]);
                    const T Vc = c < n ? (vv4[0] + vv4[1]) + (vv4[2] + vv4[3]) : T(0);
                    tick(7);
                    T s2[2] = {pv * Vc, Vc * Vc};
                    wave_sums<T, 2>(s2);
                    tick(8);
                    const T pp = readlane_f(q, v);
                    const T pV = s2[0], VV = s2[1], aa = Gm[v * LG + v];  // |a_v|^2: the Gram diagonal
                    const T pvd = pV + aa * pp, vvd = VV + T(2) * aa * pV + aa * aa * pp;
                    const T kappa = pvd / pp;
                    const T w2t = vvd - kappa * pvd;
                    const T w2 = w2t > T(0) ? w2t : T(0);
                    const T rho = T(1) - eps * kappa;
                    T S0, S1;
                    const int m = transr_rounds_violator(pp, w2, eps, rho, S0, S1);
                    n_rounds += (unsigned long long)m;
                    max_m = max_m > (unsigned long long)m ? max_m : (unsigned long long)m;
                    const T cpf = T(2) * (S0 + eps * S1 * kappa), cvf = T(2) * eps * S1;
                    const T g = c < n ? cpf * pv - cvf * (Vc + aa * pv) : T(0);
                    tick(9);
                    if (c < NP) P[v * L + c] = g;  // the violator's row now holds G (records after B2)
                    tick(10);
                    // the later pairs: P[j] -= lr (a_j . a_v) g, |p_j|^2 afresh (lane j: half
                    // l >> 5 of the columns)
                    if (j > v && j < cc) {
                        // blocks of 16 columns: all loads of a block, then its stores (a store
                        // between loads would make every load wait for it)
                        const T gl = -lr * Gm[j * LG + v];
                        const int c0 = (l >> 5) * (NP / 2);
                        constexpr int KB = (NP / 2) % 16 == 0 ? 16 : 8;  // divides NP / 2
                        T s4[4] = {T(0), T(0), T(0), T(0)};
#pragma unroll
                        for (int b0 = 0; b0 < NP / 2; b0 += KB) {
                            T x[KB], gg[KB];
#pragma unroll
                            for (int u = 0; u < KB; ++u) {
                                x[u] = P[j * L + c0 + b0 + u];
                                gg[u] = P[v * L + c0 + b0 + u];
                            }
#pragma unroll
                            for (int u = 0; u < KB; ++u) {
                                x[u] = fma(gl, gg[u], x[u]);
                                s4[u & 3] = fma(x[u], x[u], s4[u & 3]);
                            }
#pragma unroll
                            for (int u = 0; u < KB; ++u) P[j * L + c0 + b0 + u] = x[u];
                        }
                        q = (s4[0] + s4[1]) + (s4[2] + s4[3]);
                    }
                    {
                        const T other = __shfl_xor(q, 32);
                        if (j > v && j < cc) q += other;
                    }
                    vmask |= 1u << v;
                    cursor = v + 1;
                    ++n_vio;
                    tick(11);
                }
                if (l < cc) {  // the chunk's pair flags; (entity'[r], r) marks the relation
                    const int sl = ps[base + l];
                    const bool vio = (vmask >> l) & 1;
                    if (sl >= 0) bf.pflag[sl] = vio ? 1 : 0;
                    else if (vio) bf.relpair_stamp[r] = bf.stamp;
                }
                if (l == 0) misc[1] = (int)vmask;
            } else if (w == 0 && l < cc) {
                const int sl = ps[base + l];
                if (sl >= 0) bf.pflag[sl] = 0;
            }
            tick(4);
            __syncthreads();  // B2
            tick(5);
            if (anyv) {
                const uint32_t vmask = (uint32_t)misc[1];
                {  // the violators' pair records G (da = -lr W G at the end), a wave each
                    uint32_t mm = vmask;
                    for (int k = 0; k < w && mm; ++k) mm &= mm - 1;
                    while (mm) {
                        const int v = __builtin_ctz(mm);
                        const int sl = ps[base + v];
                        T* dst = sl >= 0 ? bf.pair + (int64_t)sl * ld : bf.relpair + (int64_t)r * ld;
                        if (l < n) dst[l] = P[v * L + l];
                        if (l == 0) vio[nvt + __builtin_popcount(vmask & ((1u << v) - 1u))] = sl;
                        for (int k = 0; k < 4 && mm; ++k) mm &= mm - 1;
                    }
                    nvt += __builtin_popcount(vmask);
                }
                // W_c[:, slice] -= lr sum_v A[v]^T G[v] over the chunk's violators
                if (vmask) changed = true;
                if (mine) {
                    T wv[KS];
#pragma unroll
                    for (int t = 0; t < KS; ++t) wv[t] = Wc[(kq + 4 * t) * L + col];
                    for (uint32_t mm = vmask; mm; mm &= mm - 1) {
                        const int v = __builtin_ctz(mm);
                        const T gl = -lr * P[v * L + col];
#pragma unroll
                        for (int t = 0; t < KS; ++t) wv[t] = fma(A[v * L + kq + 4 * t], gl, wv[t]);
                    }
#pragma unroll
                    for (int t = 0; t < KS; ++t) Wc[(kq + 4 * t) * L + col] = wv[t];
                }
            }
            __syncthreads();  // B3: W_c
            tick(6);
            base = nbase;
        }
        gw += ntile;
        if (last || gw >= g0 + run) break;
    }
    // the relation's matrix back: each wave its column slice (the transRNorm pass adds no partials)
    if (mine && col < n)
        for (int jj = 0; jj < n; ++jj) bf.W[((int64_t)r * n + jj) * ld + col] = Wc[jj * L + col];
    __syncthreads();  // (the last records written; P free)
    chain_records<T, NP, L>(a, bf, r, vio, nvt, Wc, P, R * L);
    if (bf.stats) {
        if (threadIdx.x == 0) {
            const unsigned long long cyc = (unsigned long long)(clock64() - ck0);
            atomicAdd(&g_seq_stats[0], 1ull);
            atomicAdd(&g_seq_stats[1], n_chunks);
            atomicAdd(&g_seq_stats[2], n_vio);
            atomicAdd(&g_seq_stats[3], n_rounds);
            atomicAdd(&g_seq_stats[4], cyc);
            atomicMax(&g_seq_stats[5], cyc);
            atomicMax(&g_seq_stats[6], n_chunks);
            atomicMax(&g_seq_stats[7], max_m);
            for (int k = 0; k < 16; ++k) atomicAdd(&g_seq_stats[8 + k], ph[k]);
            if (n_chunks >= 20) {  // the hot relations alone
                for (int k = 0; k < 16; ++k) atomicAdd(&g_seq_stats[24 + k], ph[k]);
                atomicAdd(&g_seq_stats[40], n_chunks);
                atomicAdd(&g_seq_stats[41], 1ull);
                atomicAdd(&g_seq_stats[42], n_vio);
            }
        }
    }
}

}  // namespace kb2e
