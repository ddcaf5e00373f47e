// kernels_transr_chainwp.hpp -- transRNorm of the PARALLEL TransR schedule per
// relation, pair by pair, software-pipelined, for 64 < n <= 100 (FP64; K5's
// n = 100, BASELINE configs[4]).  Same model and the same records as
// transr_cons_chain_wide_kernel (kernels_transr_chainw.hpp; oracle/parallel.py
// transr_constraint, cons="chunk1"; the reference's calls are
// transr/trainer.cpp:185-187 on the loop at :35-64): the relation's pairs in
// (sample, update, role) order, first occurrences, each against the matrix the
// earlier violators left, the last update's pairs and (entity'[r], r) after
// W_c's rows are renormalised.
//
// The wide kernel walks a chunk with all eight waves in lockstep: the chunk's
// projections (MFMA) and its walk follow one another, and every violator costs
// three block barriers.  On a hot relation (K5: ~1,200 chunks of 16 pairs a
// batch, ~1.5 violators a chunk) that chain is the batch's critical path.  Here,
// as in kernels_transr_pipe.hpp for n <= 64:
//  * wave 0 walks chunk k alone (no barriers inside the walk): the chunk's
//    projection rows in registers (lane (j, h): quarter h of row j), V = p K0
//    from K0 = W'^T W' in LDS (two columns a lane), the dots a_j . a_v from the
//    chunk's rows (quarters, two shuffles), the closed-form rounds;
//  * waves 1-7 own the working matrix W_c as the MFMA B fragments of one column
//    tile each (tile cb on wave 1 + cb), and meanwhile pay chunk k-1's debt
//    (W_c -= lr A_{k-1}^T G_{k-1} on their tile, the pair records G) and make the
//    next chunk's projections X_{k+1} = A_{k+1} W_c;
//  * after the walk all 512 threads fold chunk k's violators into X_{k+1}
//    (P_{k+1} = X_{k+1} - lr (A_{k+1} a_v) g_v, the dots on the fly) and take
//    the new |p|^2 -- two block barriers a chunk, whatever its violators.
// The k-steps run over 4 KS >= n columns (KS a template parameter: 25 at n = 100,
// no MFMA on the 112-column padding of the wide kernel), which is also what
// lets K0 [4 KS][4 KS + 1], three row slots and two projection buffers fit
// the 160 KiB of LDS.
#pragma once

#include "kernels_transr_chainw.hpp"

namespace kb2e {

constexpr int kWPThreads = 512;       // eight waves: the walker and seven helpers
constexpr int kWPRows = 16;           // pairs a chunk: one MFMA row tile
constexpr int kWPWin = 256;           // samples a window
constexpr int kWPPairs = 4 * kWPWin;  // pairs a window, at most
constexpr int kWPMaxN = 100;          // K0 [100][100] + the buffers: 159 KiB

__host__ __device__ constexpr int wp_ks(int n) {  // the k-steps: an instantiated KS >= ceil(n / 4)
    return n <= 72 ? 18 : n <= 80 ? 20 : n <= 88 ? 22 : n <= 96 ? 24 : 25;
}

// LDS bytes: K0 / W' [4 KS][4 KS + 2] | A [3][R][4 KS + 2] | P [2][R][4 KS + 2] |
// Gram [2][R][R + 1] | cross Gram [R][R + 1] | qpart [R] ; ints pe, ps [kWPPairs] | vlist [2][R] | wsum [8] | misc [8] ; vflag [kWPPairs]
__host__ __device__ constexpr size_t chainwp_lds_ks(int KS) {
    return sizeof(double) * ((size_t)(4 * KS) * (4 * KS + 2) + 5 * (size_t)kWPRows * (4 * KS + 2) +
                             3 * (size_t)kWPRows * (kWPRows + 1) + kWPRows) +
           sizeof(int) * (2 * (size_t)kWPPairs + 2 * kWPRows + 16) + (size_t)kWPPairs;
}
__host__ __device__ constexpr size_t chainwp_lds(int n) { return chainwp_lds_ks(wp_ks(n)); }

template <int KS>
__global__ __launch_bounds__(kWPThreads) void transr_cons_chain_wpipe_kernel(RParArgs a, RParBufs<double> bf) {
    using T = double;
    using M = Mfma16<T>;
    constexpr int NC = 4 * KS;                 // the columns the chain keeps (>= n; zeros past n)
    constexpr int NB = (NC + 15) / 16;         // MFMA column tiles
    constexpr int LA = NC + 2, R = kWPRows, LG = R + 1, NT = kWPThreads, NW = NT / 64;
    static_assert(NB <= NW - 1, "a column tile a helper wave");
    static_assert(2 * R * LA >= NB * NC, "the renorm's row partials borrow the P buffers");
    // block b takes the b-th most frequent relation (the hot chains start first)
    const int r = a.brel[blockIdx.x];
    int s;
    {
        int lo = a.rel_begin[a.batch], hi = a.batch_seg[a.batch + 1] - 1;
        if (lo > hi) return;
        const int want = a.ne + r;
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (a.seg_row[mid] < want) lo = mid + 1;
            else hi = mid;
        }
        if (a.seg_row[lo] != want) return;
        s = lo;
    }
    const int n = a.n, ld = a.ld;
    const int p0 = a.seg_start[s], ns = (a.seg_start[s + 1] - p0) / 2;
    const int tid = threadIdx.x, w = tid >> 6, l = lane_id(), kq = l >> 4, l16 = l & 15;
    const int cb = w - 1;                  // helper wave: its column tile
    const bool own = w >= 1 && cb < NB;
    const int col = 16 * cb + l16;         // (helpers) the fragment column
    const T lr = (T)a.lr;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    T* K0 = (T*)smem;              // [NC][LA] W' (prologue), then K0 as [NC / 2][NC] pairs (K0[2 i2 + e][c] at (i2 NC + c) 2 + e)
    T* Abuf = K0 + NC * LA;        // [3][R][LA] entity rows of chunks k - 1 / k + 2, k, k + 1
    T* Pbuf = Abuf + 3 * R * LA;   // [2][R][LA] projections of chunks k, k + 1 (violator rows: G)
    T* Gbuf = Pbuf + 2 * R * LA;   // [2][R][LG] Gram matrices A A^T of chunks k, k + 1
    T* Cx = Gbuf + 2 * R * LG;     // [R][LG] cross Gram A_{k+1} A_k^T (next x current)
    T* qpart = Cx + R * LG;        // [R] |p_j|^2 of the next chunk
    int* pe = (int*)(qpart + R);   // [kWPPairs]
    int* ps = pe + kWPPairs;       // [kWPPairs]
    int* vlist = ps + kWPPairs;    // [2][R] the violators of a chunk, by chunk parity
    int* wsum = vlist + 2 * R;     // [8]
    int* misc = wsum + 8;          // [8]
    uint8_t* vflag = (uint8_t*)(misc + 8);  // [kWPPairs]
    const long long ck0 = clock64();
    unsigned long long n_chunks = 0, n_vio = 0, n_rounds = 0, max_m = 0;
    // KB2E_RPAR_STATS: cycles on thread 0 (the walker; g_seq_stats 8..23, relations of
    // >= 200 chunks also 24..39): 0 prologue + K0, 1 window list, 2 walk, 3 B1 wait,
    // 4 row stores + fold, 5 B2 wait, 6 drain, 7 window flags, 8 tail, 9 write-back + records;
    // thread 64 (helper wave 1): 10 debt (W update + records; from its last tick: the
    // fold and B2 too), 11 X tile, 12 B1 wait; the walk's violators split into 13
    // (row to LDS + V), 14 (sums, rounds, g), 15 (later rows; phase 2 keeps the rest)
    __shared__ unsigned long long ph[16];
    if (tid < 16) ph[tid] = 0;
    long long tq = ck0;
    auto tick = [&](int k) {
        if (bf.stats && ((k >= 10 && k <= 12) ? tid == 64 : tid == 0)) {
            const long long t = clock64();
            atomicAdd(&ph[k], (unsigned long long)(t - tq));
            tq = t;
        }
    };

    // the relation's last active sample (from the end, NT samples a round)
    if (tid == 0) misc[0] = -1;
    __syncthreads();
    for (int qb = ns - NT;; qb -= NT) {
        const int q = qb + tid;
        const bool act = q >= 0 && q < ns && a.act[a.kl.kk_of(a.keys[p0 + 2 * q])];
        const uint64_t b = __ballot(act);
        if (b && l == 0) atomicMax(&misc[0], qb + (w << 6) + 63 - __builtin_clzll(b));
        __syncthreads();
        const int found = misc[0];
        __syncthreads();
        if (found >= 0 || qb <= 0) break;
    }
    const int klq = misc[0];
    if (klq < 0) return;  // no active update: the gradient step left the relation alone
    const int kl = a.kl.kk_of(a.keys[p0 + 2 * klq]);
    const bool has_rel = r < a.ne && ptab_first(a, r, r) < 0;  // (entity'[r], r), transr/trainer.cpp:187

    // W'_r [NC][LA] (zeros past n), the helpers' fragments, K0 = W'^T W' on the
    // matrix cores (upper tiles, mirrored), then K0 in place of W'
    for (int idx = tid; idx < NC * NC; idx += NT) {
        const int j = idx / NC, i = idx % NC;
        K0[j * LA + i] = (j < n && i < n) ? bf.W[((int64_t)r * n + j) * ld + i] : T(0);
    }
    __syncthreads();
    T bW[KS];  // helpers: W_c[4 s + kq][col]
#pragma unroll
    for (int q = 0; q < KS; ++q) bW[q] = own && col < NC ? K0[(4 * q + kq) * LA + col] : T(0);
    {
        constexpr int NUT = NB * (NB + 1) / 2;  // upper tiles (ib <= jb)
        constexpr int TPW = (NUT + NW - 1) / NW;
        typename M::acc_t kacc[TPW];
#pragma unroll
        for (int t = 0; t < TPW; ++t) {
            kacc[t] = typename M::acc_t{T(0), T(0), T(0), T(0)};
            const int u = w + NW * t;
            if (u >= NUT) continue;
            int ib = 0, rem = u;
            while (rem >= NB - ib) {
                rem -= NB - ib;
                ++ib;
            }
            const int jb = ib + rem;
            const int ci = 16 * ib + l16, cj = 16 * jb + l16;
#pragma unroll 5
            for (int q = 0; q < KS; ++q) {
                const T av = ci < NC ? K0[(4 * q + kq) * LA + ci] : T(0);
                const T bv = cj < NC ? K0[(4 * q + kq) * LA + cj] : T(0);
                kacc[t] = M::mma(av, bv, kacc[t]);
            }
        }
        __syncthreads();  // every thread done with W'
#pragma unroll
        for (int t = 0; t < TPW; ++t) {
            const int u = w + NW * t;
            if (u >= NUT) continue;
            int ib = 0, rem = u;
            while (rem >= NB - ib) {
                rem -= NB - ib;
                ++ib;
            }
            const int jb = ib + rem;
            const int cj = 16 * jb + l16;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int ri = 16 * ib + M::row(l, q);
                if (ri < NC && cj < NC) {  // K0[i][c] at pair (i / 2, c), element i & 1
                    K0[((ri >> 1) * NC + cj) * 2 + (ri & 1)] = kacc[t][q];
                    K0[((cj >> 1) * NC + ri) * 2 + (cj & 1)] = kacc[t][q];
                }
            }
        }
    }
    bool changed = false;
    // the chunk whose W_c update and pair records the helpers still owe (nv 0: none)
    int pend_nv = 0, pend_par = 0, pend_pc = 0, pend_ka = 0, pend_base = 0;
    __syncthreads();
    tick(0);

    // rows of chunk [b, e) of the list: R x NC elements, RPT a thread, into registers
    constexpr int RPT = (R * NC + NT - 1) / NT;
    T rows[RPT];
    uint32_t rows_ok = 0;
    auto load_rows = [&](int b, int e) {
        int ent[RPT];
#pragma unroll
        for (int q = 0; q < RPT; ++q) {
            const int idx = tid + q * NT;
            const int f = b + idx / NC;
            ent[q] = idx < R * NC && f < e ? pe[f] : -1;
        }
        rows_ok = 0;
#pragma unroll
        for (int q = 0; q < RPT; ++q) {
            const int j = (tid + q * NT) % NC;
            const bool ok = ent[q] >= 0 && j < n;
            rows[q] = bf.ent[ok ? (uint32_t)ent[q] * (uint32_t)ld + (uint32_t)j : 0u];
            rows_ok |= (ok ? 1u : 0u) << q;
        }
    };
    auto store_rows = [&](int slot) {
#pragma unroll
        for (int q = 0; q < RPT; ++q) {
            const int idx = tid + q * NT;
            if (idx < R * NC) Abuf[slot * R * LA + (idx / NC) * LA + idx % NC] = ((rows_ok >> q) & 1) ? rows[q] : T(0);
        }
    };
    // helpers: X = A W_c on their column tile (KS k-steps, B from the registers);
    // wave 4 also the chunk's Gram matrix A A^T (its B operand is its A operand),
    // wave 5 the cross Gram A A_c^T with the current chunk (Ac; none for a fresh chunk)
    // The Gram matrices ride on waves 6 / 7 (NB = 7), off the walker's SIMD (wave w runs on
    // SIMD w mod 4): 4% on the K5 line (KB2E_CONS_DBG bit 1: waves 4 / 5, A/B; same results)
    const int gw = !(bf.dbg & 2) && NB >= 7 ? 6 : 4, cw = !(bf.dbg & 2) && NB >= 7 ? 7 : 5;
    auto x_tile = [&](const T* Ar, T* out, T* G, const T* Ac) {
        if (!own) return;
        typename M::acc_t acc = {T(0), T(0), T(0), T(0)};
        T av[KS];
#pragma unroll
        for (int q = 0; q < KS; ++q) av[q] = Ar[l16 * LA + 4 * q + kq];
#pragma unroll
        for (int q = 0; q < KS; ++q) acc = M::mma(av[q], bW[q], acc);
        if (col < NC) {
#pragma unroll
            for (int q = 0; q < 4; ++q) out[(kq + 4 * q) * LA + col] = acc[q];
        }
        if (w == gw) {
            typename M::acc_t ga = {T(0), T(0), T(0), T(0)};
#pragma unroll
            for (int q = 0; q < KS; ++q) ga = M::mma(av[q], av[q], ga);
#pragma unroll
            for (int q = 0; q < 4; ++q) G[(kq + 4 * q) * LG + l16] = ga[q];
        }
        if (w == cw && Ac) {  // the cross Gram with the current chunk's rows (the fold's dots)
            typename M::acc_t ca = {T(0), T(0), T(0), T(0)};
#pragma unroll
            for (int q = 0; q < KS; ++q) ca = M::mma(av[q], Ac[l16 * LA + 4 * q + kq], ca);
#pragma unroll
            for (int q = 0; q < 4; ++q) Cx[(kq + 4 * q) * LG + l16] = ca[q];
        }
    };
    // the helpers' debt: the pending chunk's W_c -= lr A^T G on their tile (G rows in
    // P buffer pend_pc, a rows in A slot pend_ka) and its pair records (their columns)
    auto apply_pending = [&]() {
        if (!own || pend_nv == 0) return;
        const T* Pp = Pbuf + pend_pc * R * LA;
        const T* Ap = Abuf + pend_ka * R * LA;
        const int* vl = vlist + pend_par * R;
        // the violators' rows as wave-uniform values (one LDS read for all of them); the
        // next violator's reads in flight while this one's FMAs run
        const int vmine = l < pend_nv ? vl[l] : 0;
        T an[KS], gn = T(0);
        auto ldv = [&](int k) {
            const int v = __builtin_amdgcn_readlane(vmine, k);
#pragma unroll
            for (int q = 0; q < KS; ++q) an[q] = Ap[v * LA + 4 * q + kq];
            gn = col < NC ? -lr * Pp[v * LA + col] : T(0);
        };
        ldv(0);
        for (int k = 0; k < pend_nv; ++k) {
            T ac[KS];
#pragma unroll
            for (int q = 0; q < KS; ++q) ac[q] = an[q];
            const T gl = gn;
            if (k + 1 < pend_nv) ldv(k + 1);
#pragma unroll
            for (int q = 0; q < KS; ++q) bW[q] = fma(ac[q], gl, bW[q]);
        }
        for (int k = kq; k < pend_nv; k += 4) {
            const int v = vl[k];
            const int sl = ps[pend_base + v];
            T* dst = sl >= 0 ? bf.pair + (int64_t)sl * ld : bf.relpair + (int64_t)r * ld;
            if (col < n) dst[col] = Pp[v * LA + col];
            if (sl < 0 && cb == 0 && l16 == 0) bf.relpair_stamp[r] = bf.stamp;
        }
    };
    // all threads: P_n[j] -= lr sum_v (a_n[j] . a_v) g_v over the current chunk's nv
    // violators (vl; the dots from the cross Gram Cx, g_v in Pc), then |p_j|^2 into
    // qpart; 32 threads a row, four columns each
    auto fold = [&](T* Pn, int cn, int nv, const T* Pc, const int* vl) {
        const int j = tid >> 5, c0 = 4 * (tid & 31);
        const bool okr = j < cn && c0 < NC;
        T x[4] = {T(0), T(0), T(0), T(0)};
        if (okr) {
#pragma unroll
            for (int u = 0; u < 4; ++u) x[u] = Pn[j * LA + c0 + u];
        }
        if (nv > 0) {
            for (int k = 0; k < nv; ++k) {
                const int v = vl[k];
                if (okr) {
                    const T gl = -lr * Cx[j * LG + v];
#pragma unroll
                    for (int u = 0; u < 4; ++u) x[u] = fma(gl, Pc[v * LA + c0 + u], x[u]);
                }
            }
            if (okr) {
#pragma unroll
                for (int u = 0; u < 4; ++u) Pn[j * LA + c0 + u] = x[u];
            }
        }
        T sq = (x[0] * x[0] + x[1] * x[1]) + (x[2] * x[2] + x[3] * x[3]);
        // the row's 32 lanes: quad perms, half-row and row mirrors (DPP), then the
        // other row of the pair (the same sums as xor 1 .. 16)
        sq += dpp_mov<0xB1>(sq);
        sq += dpp_mov<0x4E>(sq);
        sq += dpp_mov<0x141>(sq);
        sq += dpp_mov<0x140>(sq);
        sq += __shfl_xor(sq, 16);
        if ((tid & 31) == 0 && j < R) qpart[j] = j < cn ? sq : T(0);
    };
    // W_c's unit rows (transr/trainer.cpp:178-180) before the last update's pairs;
    // row sums of the tiles in DPP rows, then LDS (the P buffers are free: drained)
    auto renorm = [&] {
        T* rp = Pbuf;  // [NB][NC]
        if (own) {
#pragma unroll
            for (int q = 0; q < KS; ++q) {
                T x[1] = {bW[q] * bW[q]};
                row16_sums<T, 1>(x);
                if (l16 == 0) rp[cb * NC + 4 * q + kq] = x[0];
            }
        }
        __syncthreads();
        if (own) {
#pragma unroll
            for (int q = 0; q < KS; ++q) {
                const int jr = 4 * q + kq;
                T ss = rp[jr];
                for (int v = 1; v < NB; ++v) ss += rp[v * NC + jr];
                if (jr < n) bW[q] = bW[q] / sqrt(ss);
            }
        }
        __syncthreads();
    };
    // the walk of one chunk (wave 0): pairs [base, base + cc), projections in P (rows
    // j < cc), |p_j|^2 in qpart, rows in A; the violators' rows of P become G
    auto walk = [&](T* P, const T* Gm, int cc, int base, int* vl) {
        const int j = l & (R - 1), h = l >> 4;  // lane: quarter h of row j
        T q = j < cc ? qpart[j] : T(0);
        uint32_t vmask = 0;
        if (__ballot(j < cc && q > T(1)) != 0) {
            T x[KS];
#pragma unroll
            for (int u = 0; u < KS; ++u) x[u] = P[j * LA + h * KS + u];
            const T eps = T(2) * lr;
            const int c1 = l + 64;  // the lane's second column (c1 < NC)
            int cursor = 0;
            for (;;) {
                const uint64_t cand = __ballot(j < cc && j >= cursor && q > T(1));
                if (!cand) break;
                const int v = __builtin_ctzll(cand) & (R - 1);
                // the violator's current row to LDS (column layout below)
                if (j == v) {
#pragma unroll
                    for (int u = 0; u < KS; ++u) P[v * LA + h * KS + u] = x[u];
                }
                if (bf.dbg & 4) tick(7);  // (timing experiment: the pick and row store apart from V)
                // a_j . a_v for every row, from the chunk's Gram matrix
                const T dp = Gm[j * LG + v];
                // V_c = sum_i p_v[i] K0[i][c], c = l and l + 64: 16-byte reads of K0's row
                // pairs (consecutive lanes, consecutive pairs), p_v as broadcasts; the
                // second column's reads are clamped, not branched (its lanes >= NC - 64
                // read one address and discard the sums)
                const T* pr = P + v * LA;
                const double2* kp = (const double2*)K0;
                const double2* pp2 = (const double2*)pr;
                const int c1r = c1 < NC ? c1 : NC - 1;  // (lanes past the columns: one broadcast address)
                T va[4] = {T(0), T(0), T(0), T(0)}, vb[4] = {T(0), T(0), T(0), T(0)};
                // software-pipelined over the NC / 2 row pairs: the reads of the next D pairs
                // (three 16-byte reads a pair, 3 D <= 15 in flight: the LDS counter's range)
                // are issued while the current pair's four FMAs run.  The slots rotate
                // without copies and every condition is a compile-time one (a runtime one
                // turns the slots into phi copies that wait for every read)
                constexpr int NP2 = NC / 2, D = 4, NG = NP2 / D, REM = NP2 % D;
                static_assert(NG >= 1, "a full group of pairs");
                double2 bp[D], ba[D], bb[D];
                auto ld = [&](int i, int t) {
                    bp[t] = pp2[i];
                    ba[t] = kp[i * NC + l];
                    bb[t] = kp[i * NC + c1r];
                };
                auto fm = [&](int t) {  // (pair parity = t's: D even)
                    const int e = (t & 1) * 2;
                    va[e] = fma(bp[t].x, ba[t].x, va[e]);
                    va[e + 1] = fma(bp[t].y, ba[t].y, va[e + 1]);
                    vb[e] = fma(bp[t].x, bb[t].x, vb[e]);
                    vb[e + 1] = fma(bp[t].y, bb[t].y, vb[e + 1]);
                };
#pragma unroll
                for (int t = 0; t < D; ++t) ld(t, t);
                // groups of D pairs, rolled (unrolled, the scheduler hoists every read and
                // spills), each refill pinned right behind its slot's FMAs
#pragma unroll 1
                for (int g = 0; g + 1 < NG; ++g) {
#pragma unroll
                    for (int t = 0; t < D; ++t) {
                        fm(t);
                        ld((g + 1) * D + t, t);
                        __builtin_amdgcn_sched_barrier(0);
                    }
                }
#pragma unroll
                for (int t = 0; t < D; ++t) {  // the last full group, refilling the remainder
                    fm(t);
                    if (t < REM) ld(NG * D + t, t);
                }
#pragma unroll
                for (int t = 0; t < REM; ++t) fm(t);
                const T V0 = (va[0] + va[1]) + (va[2] + va[3]);
                const T V1 = c1 < NC ? (vb[0] + vb[1]) + (vb[2] + vb[3]) : T(0);
                tick(13);
                const T pv0 = pr[l], pv1 = c1 < NC ? pr[c1] : T(0);
                T s2[2] = {pv0 * V0 + pv1 * V1, V0 * V0 + V1 * V1};
                wave_sums<T, 2>(s2);
                const T pp = readlane_f(q, v);
                const T aa = readlane_f(dp, v);  // |a_v|^2
                const T pV = s2[0], VV = s2[1];
                const T pvd = pV + aa * pp, vvd = VV + T(2) * aa * pV + aa * aa * pp;
                T rpp = __builtin_amdgcn_rcp(pp);  // v_rcp_f64 and two Newton steps (as the pipe kernel)
                rpp = fma(fma(-pp, rpp, T(1)), rpp, rpp);
                rpp = fma(fma(-pp, rpp, T(1)), rpp, rpp);
                const T kappa = pvd * rpp;
                const T w2t = vvd - kappa * pvd;
                const T w2 = w2t > T(0) ? w2t : T(0);
                const T rho = T(1) - eps * kappa;
                T S0, S1;
                const int m = transr_rounds_violator4(pp, w2, eps, rho, S0, S1);
                n_rounds += (unsigned long long)m;
                max_m = max_m > (unsigned long long)m ? max_m : (unsigned long long)m;
                const T cpf = T(2) * (S0 + eps * S1 * kappa), cvf = T(2) * eps * S1;
                // g (zero past n: p and K0 are); the violator's row now holds G
                P[v * LA + l] = cpf * pv0 - cvf * (V0 + aa * pv0);
                if (c1 < NC) P[v * LA + c1] = cpf * pv1 - cvf * (V1 + aa * pv1);
                tick(14);
                // the later rows: p_j -= lr (a_j . a_v) g, |p_j|^2 afresh
                const bool upd = j > v && j < cc;
                T qh = T(0);
                if (upd) {
                    const T gl = -lr * dp;
                    T s4[4] = {T(0), T(0), T(0), T(0)};
#pragma unroll
                    for (int u = 0; u < KS; ++u) {
                        x[u] = fma(gl, P[v * LA + h * KS + u], x[u]);
                        s4[u & 3] = fma(x[u], x[u], s4[u & 3]);
                    }
                    qh = (s4[0] + s4[1]) + (s4[2] + s4[3]);
                }
                qh += __shfl_xor(qh, 16);
                qh += __shfl_xor(qh, 32);
                if (upd) q = qh;
                vmask |= 1u << v;
                cursor = v + 1;
                ++n_vio;
                tick(15);
            }
        }
        if (l < R && ((vmask >> l) & 1u)) {
            vl[__builtin_popcount(vmask & ((1u << l) - 1u))] = l;
            vflag[base + l] = 1;
        }
        if (l == 0) {
            misc[1] = (int)vmask;
            misc[2] = __builtin_popcount(vmask);
        }
    };
    // the pipeline over the list's pairs [0, npw) (pe / ps), chunks of R; ends
    // drained (the last chunk's debt paid) after a barrier
    auto run_list = [&](int npw) {
        const int nch = (npw + R - 1) / R;
        auto csz = [&](int k) { return k < nch ? min(R, npw - k * R) : 0; };
        load_rows(0, csz(0));
        store_rows(0);
        if (nch > 1) {
            load_rows(R, R + csz(1));
            store_rows(1);
        }
        if (nch > 2) load_rows(2 * R, 2 * R + csz(2));
        __syncthreads();
        x_tile(Abuf, Pbuf, Gbuf, nullptr);  // chunk 0 afresh
        __syncthreads();
        fold(Pbuf, csz(0), 0, nullptr, nullptr);
        __syncthreads();
        // after B1, everyone: chunk k's debt noted for the helpers, the row slots, the fold
        auto after_b1 = [&](int k) {
            const int cn = csz(k + 1), pc = k & 1;
            const int nv = misc[2];
            pend_nv = nv;
            pend_par = pc;
            pend_pc = pc;
            pend_ka = k % 3;
            pend_base = k * R;
            if (nv) changed = true;
            // chunk k + 2's rows into the slot chunk k - 1 left, chunk k + 3's in flight
            if (k + 2 < nch) {
                store_rows((k + 2) % 3);
                if (k + 3 < nch) load_rows((k + 3) * R, (k + 3) * R + csz(k + 3));
            }
            if (cn > 0) fold(Pbuf + (pc ^ 1) * R * LA, cn, nv, Pbuf + pc * R * LA, vlist + pc * R);
        };
        // one loop a role: the walker's holds no W_c fragment (zeros on wave 0, restated as
        // such after its loop, so that they are not live across the walk)
        if (w == 0) {
            for (int k = 0; k < nch; ++k) {
                const int pc = k & 1;
                ++n_chunks;
                walk(Pbuf + pc * R * LA, Gbuf + pc * R * LG, csz(k), k * R, vlist + pc * R);
                tick(2);
                __syncthreads();  // B1: the walk's G rows and violators, X_{k+1}
                tick(3);
                after_b1(k);
                tick(4);
                __syncthreads();  // B2: P_{k+1} and its |p|^2
                tick(5);
            }
#pragma unroll
            for (int q = 0; q < KS; ++q) bW[q] = T(0);
        } else {
            for (int k = 0; k < nch; ++k) {
                const int cn = csz(k + 1), pc = k & 1;
                ++n_chunks;
                apply_pending();  // chunk k - 1's
                tick(10);
                if (cn > 0)
                    x_tile(Abuf + ((k + 1) % 3) * R * LA, Pbuf + (pc ^ 1) * R * LA, Gbuf + (pc ^ 1) * R * LG,
                           Abuf + (k % 3) * R * LA);
                tick(11);
                __syncthreads();  // B1
                tick(12);
                after_b1(k);
                __syncthreads();  // B2
            }
        }
        apply_pending();
        pend_nv = 0;
        __syncthreads();
        tick(6);
    };

    // windows of kWPWin samples up to the last active one; the last update's slots wait for the tail
    for (int wq = 0; wq <= klq; wq += kWPWin) {
        const int q = wq + tid;
        int kk = -1, ents[4] = {-1, -1, -1, -1};
        uint32_t keep = 0;
        if (tid < kWPWin && q <= klq) {
            kk = a.kl.kk_of(a.keys[p0 + 2 * q]);
            if (a.act[kk]) {
                const int i0 = a.si[kk], jj = a.sj[kk];
                const int hh = a.heads[i0], tt = a.tails[i0];
                const bool sd = a.side[kk] != 0;
                ents[0] = hh;
                ents[1] = tt;
                ents[2] = sd ? hh : jj;
                ents[3] = sd ? jj : tt;
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const int sl = kk * 4 + k;
                    const bool tail = kk == kl && k >= 2;
                    if (!tail && ptab_first(a, r, ents[k]) == sl) keep |= 1u << k;
                }
            } else {
                kk = -1;
            }
        }
        const int cnt = __builtin_popcount(keep);
        int x = cnt;
#pragma unroll
        for (int sh = 1; sh < kWave; sh <<= 1) {
            const int y = __shfl_up(x, sh);
            if (l >= sh) x += y;
        }
        if (l == kWave - 1) wsum[w] = x;
        __syncthreads();
        int off = 0, npw = 0;
#pragma unroll
        for (int k = 0; k < NW; ++k) {
            const int ws = wsum[k];
            off += k < w ? ws : 0;
            npw += ws;
        }
        const int pos0 = off + x - cnt;
        {
            int pos = pos0;
#pragma unroll
            for (int k = 0; k < 4; ++k)
                if ((keep >> k) & 1) {
                    pe[pos] = ents[k];
                    ps[pos] = kk * 4 + k;
                    vflag[pos] = 0;
                    ++pos;
                }
        }
        __syncthreads();  // the window's list
        tick(1);
        if (npw > 0) run_list(npw);
        // the flags of the window's slots (the tail's wait)
        if (kk >= 0) {
            int pos = pos0;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                if (kk == kl && k >= 2) continue;
                uint8_t f = 0;
                if ((keep >> k) & 1) f = vflag[pos++];
                bf.pflag[kk * 4 + k] = f;
            }
        }
        __syncthreads();  // the list is rebuilt by the next window
        tick(7);
    }

    // the tail: the last update's pairs and (entity'[r], r), after the rows' renorm
    int ntail = 0;
    uint32_t tkeep = 0;
    {
        const int i0 = a.si[kl], jj = a.sj[kl];
        const int hh = a.heads[i0], tt = a.tails[i0];
        const bool sd = a.side[kl] != 0;
        const int e2[2] = {sd ? hh : jj, sd ? jj : tt};
        for (int k = 0; k < 2; ++k)
            if (ptab_first(a, r, e2[k]) == kl * 4 + 2 + k) {
                tkeep |= 1u << k;
                if (tid == 0) {
                    pe[ntail] = e2[k];
                    ps[ntail] = kl * 4 + 2 + k;
                    vflag[ntail] = 0;
                }
                ++ntail;
            }
        if (has_rel) {
            if (tid == 0) {
                pe[ntail] = r;
                ps[ntail] = -2;
                vflag[ntail] = 0;
            }
            ++ntail;
        }
    }
    if (ntail > 0) {
        if (changed) renorm();  // (ends with a barrier: the tail list is visible)
        else __syncthreads();
        run_list(ntail);
    }
    if (tid == 0) {
        int pos = 0;
        for (int k = 0; k < 2; ++k) bf.pflag[kl * 4 + 2 + k] = ((tkeep >> k) & 1) ? vflag[pos++] : 0;
    }
    tick(8);
    // the relation's matrix back, from the fragments, and transposed into LDS (K0's
    // space) for the pair records da = -lr W G, made here: the other relations' blocks
    // finish long before the hottest chain, so their records cost no batch time
    const int LT = (n + 1) & ~1;
    static_assert(NC * LA >= NC * NC, "Wt fits K0's space");
    static_assert(3 * R * LA >= (NT / 64) * NC, "a G row a wave fits the row slots");
    static_assert(2 * kWPPairs + 2 * R >= 4 * NT + 1, "the record list fits the pair lists (and the violator lists)");
    __syncthreads();  // every walk done with K0
    if (own && col < n) {
#pragma unroll
        for (int q = 0; q < KS; ++q)
            if (4 * q + kq < n) {
                bf.W[((int64_t)r * n + 4 * q + kq) * ld + col] = bW[q];
                K0[col * LT + 4 * q + kq] = bW[q];
            }
    }
    __syncthreads();
    relation_records<NT>(a, bf, r, p0, ns, K0, LT, Abuf, pe, wsum);
    tick(9);
    if (bf.stats) {
        __syncthreads();
        if (tid == 0) {
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
            if (n_chunks >= 200) {  // the hot relations alone
                for (int k = 0; k < 16; ++k) atomicAdd(&g_seq_stats[24 + k], ph[k]);
                atomicAdd(&g_seq_stats[40], n_chunks);
                atomicAdd(&g_seq_stats[41], 1ull);
                atomicAdd(&g_seq_stats[42], n_vio);
            }
        }
    }
}

}  // namespace kb2e
