// kernels_transr_chainwv.hpp -- transRNorm of the PARALLEL TransR schedule per
// relation, pair by pair, for 64 < n <= 100 (FP64; K5's n = 100, BASELINE
// configs[4]), with V = p K0 made by the helper waves.  The same model and records
// as the other chain kernels (oracle/parallel.py transr_constraint, cons="chunk1";
// the reference's calls are transr/trainer.cpp:185-187 on the loop at :35-64).
//
// kernels_transr_chainwp.hpp walks each chunk on wave 0 with K0 = W'^T W' in LDS:
// per violator V = p_v K0 is 100 x 100 FMAs on one wave fed from 80 KB of LDS,
// ~6k of the walk's ~9k cycles a violator (r22 counters), and after the walk all
// waves fold the chunk's violators into the next chunk's projections behind a
// second barrier -- the walker's path is the chunk's critical path.  Here:
//  * the seven helper waves hold K0 as well as W_c, one column tile each (K0's
//    fragments kf[q] = K0[4 q + kq][col] beside W_c's), and answer the walker's
//    V requests: the walker writes the violator's row to LDS and a request
//    number, each helper makes its 16 columns of V (25 FMAs a lane over
//    broadcasts of the row, two shuffles) and counts itself in, the walker reads
//    V from LDS.  The helpers look for requests between every few steps of their
//    own work (the debt, the projection tile) and while they wait;
//  * the helpers fold each violator into the next chunk's projections as the
//    walker publishes its G row (their own columns, the dots from the cross Gram
//    matrix), and take the next chunk's |p|^2 partials of their columns: one block
//    barrier a chunk, no fold on the walker's path.
#pragma once

#include "kernels_transr_chainwp.hpp"

namespace kb2e {

// LDS bytes: as kernels_transr_chainwp.hpp, with K0 [NC][LA] in normal layout (the
// prologue's; the V row after it) and qpart [NB][R]
__host__ __device__ constexpr size_t chainwv_lds_ks(int KS) {
    return chainwp_lds_ks(KS) + sizeof(double) * (size_t)(((4 * KS + 15) / 16) - 1) * kWPRows;
}
__host__ __device__ constexpr size_t chainwv_lds(int n) { return chainwv_lds_ks(wp_ks(n)); }

template <int KS>
__global__ __launch_bounds__(kWPThreads) void transr_cons_chain_wv_kernel(RParArgs a, RParBufs<double> bf) {
    using T = double;
    using M = Mfma16<T>;
    constexpr int NC = 4 * KS;                 // the columns the chain keeps (>= n; zeros past n)
    constexpr int NB = (NC + 15) / 16;         // MFMA column tiles
    constexpr int LA = NC + 2, R = kWPRows, LG = R + 1, NT = kWPThreads, NW = NT / 64;
    static_assert(NB <= NW - 1, "a column tile a helper wave");
    static_assert(NB >= 5, "waves 4 and 5 own a tile (the Gram matrices ride on them)");
    static_assert(2 * R * LA >= NB * NC, "the renorm's row partials borrow the P buffers");
    const int r = a.rel_order[blockIdx.x];
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
    T* K0 = (T*)smem;              // [NC][LA] W', then K0 (prologue); then the V row [NC]
    T* Vrow = K0;
    T* Abuf = K0 + NC * LA;        // [3][R][LA] entity rows of chunks k - 1 / k + 2, k, k + 1
    T* Pbuf = Abuf + 3 * R * LA;   // [2][R][LA] projections of chunks k, k + 1 (violator rows: G)
    T* Gbuf = Pbuf + 2 * R * LA;   // [2][R][LG] Gram matrices A A^T of chunks k, k + 1
    T* Cx = Gbuf + 2 * R * LG;     // [R][LG] cross Gram A_{k+1} A_k^T (next x current)
    T* qpart = Cx + R * LG;        // [NB][R] |p_j|^2 of the next chunk, a partial a column tile
    int* pe = (int*)(qpart + NB * R);  // [kWPPairs]
    int* ps = pe + kWPPairs;       // [kWPPairs]
    int* vlist = ps + kWPPairs;    // [2][R] the violators of a chunk, by chunk parity
    int* wsum = vlist + 2 * R;     // [8]
    int* misc = wsum + 8;          // [8]
    uint8_t* vflag = (uint8_t*)(misc + 8);  // [kWPPairs]
    // misc: 0 (scans); 1, 2 the chunk's violator mask / count (by parity: 1 + 2 pc, 2 + 2 pc);
    // 5 helper arrivals (helper_sync); 6 the chunk whose walk is complete; 7 (chunk << 6) |
    // violators published; during a run of chunks wsum[4] the request's row, wsum[5]
    // requests made, wsum[6] V tiles answered (NB a request)
    int* vreq = wsum + 4;
    const long long ck0 = clock64();
    unsigned long long n_chunks = 0, n_vio = 0, n_rounds = 0, max_m = 0;
    // KB2E_RPAR_STATS (g_seq_stats 8..23; relations of >= 200 chunks also 24..39): thread 0
    // (walker) 0 prologue + K0, 1 window list, 2 walk, 3 B1 wait, 6 drain, 7 window flags,
    // 8 tail, 9 write-back + records, 5 pick + row + request, 13 V wait, 14 sums + rounds + g,
    // 15 later rows; thread 64 (helper wave 1) 10 debt, 11 X tile + sync, 12 rows + fold
    // until the walk ends + |p|^2, 4 B1 wait
    __shared__ unsigned long long ph[16];
    if (tid < 16) ph[tid] = 0;
    long long tq = ck0;
    auto tick = [&](int k) {
        if (bf.stats && ((k >= 10 && k <= 12) || k == 4 ? tid == 64 : tid == 0)) {
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

    // W'_r [NC][LA] (zeros past n), the helpers' W_c fragments, K0 = W'^T W' on the matrix
    // cores (upper tiles, mirrored) into the same LDS, then the helpers' K0 fragments
    for (int idx = tid; idx < NC * NC; idx += NT) {
        const int j = idx / NC, i = idx % NC;
        K0[j * LA + i] = (j < n && i < n) ? bf.W[((int64_t)r * n + j) * ld + i] : T(0);
    }
    __syncthreads();
    T bW[KS];  // helpers: W_c[4 q + kq][col]
    T kf[KS];  // helpers: K0[4 q + kq][col]
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
                if (ri < NC && cj < NC) {
                    K0[ri * LA + cj] = kacc[t][q];
                    K0[cj * LA + ri] = kacc[t][q];
                }
            }
        }
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < KS; ++q) kf[q] = own && col < NC ? K0[(4 * q + kq) * LA + col] : T(0);
    bool changed = false;
    // the chunk whose W_c update and pair records the helpers still owe (nv 0: none)
    int pend_nv = 0, pend_par = 0, pend_pc = 0, pend_ka = 0, pend_base = 0;
    int vreqs = 0;  // V requests made (walker) / answered (helpers) in the current run of chunks
    if (tid == 0) {
        misc[5] = 0;   // helper-wave arrivals (helper_sync)
        misc[6] = -1;  // the chunk whose walk is complete
        misc[7] = -1;  // (chunk << 6) | violators published so far
    }
    __syncthreads();  // (K0's region holds the V row from here)
    tick(0);

    // rows of chunk [b, e) of the list: R x NC elements, staged by the helper waves
    constexpr int kRT = NT - 64;
    constexpr int RPT = (R * NC + kRT - 1) / kRT;
    static_assert(RPT <= 32, "rows_ok bits");
    const int rt_ = tid - 64;
    T rows[RPT];
    uint32_t rows_ok = 0;
    auto load_rows = [&](int b, int e) {
        if (w == 0) return;
        int ent[RPT];
#pragma unroll
        for (int q = 0; q < RPT; ++q) {
            const int idx = rt_ + q * kRT;
            const int f = b + idx / NC;
            ent[q] = idx < R * NC && f < e ? pe[f] : -1;
        }
        rows_ok = 0;
#pragma unroll
        for (int q = 0; q < RPT; ++q) {
            const int j = (rt_ + q * kRT) % NC;
            const bool ok = ent[q] >= 0 && j < n;
            rows[q] = bf.ent[ok ? (uint32_t)ent[q] * (uint32_t)ld + (uint32_t)j : 0u];
            rows_ok |= (ok ? 1u : 0u) << q;
        }
    };
    auto store_rows = [&](int slot) {
        if (w == 0) return;
#pragma unroll
        for (int q = 0; q < RPT; ++q) {
            const int idx = rt_ + q * kRT;
            if (idx < R * NC) Abuf[slot * R * LA + (idx / NC) * LA + idx % NC] = ((rows_ok >> q) & 1) ? rows[q] : T(0);
        }
    };
    // helpers: the walker's V requests so far (one at a time: it waits for each), V of
    // row vreq[0] of P on their column tile into the V row
    auto answer = [&](const T* P) {
        if (!own) return;
        while (__hip_atomic_load(&vreq[1], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) > vreqs) {
            const T* pr = P + vreq[0] * LA;
            T h[5] = {T(0), T(0), T(0), T(0), T(0)};
#pragma unroll
            for (int q = 0; q < KS; ++q) h[q % 5] = fma(pr[4 * q + kq], kf[q], h[q % 5]);
            T hp = ((h[0] + h[1]) + (h[2] + h[3])) + h[4];
            hp += __shfl_xor(hp, 16);
            hp += __shfl_xor(hp, 32);
            if (kq == 0 && col < NC) Vrow[col] = hp;
            ++vreqs;
            if (l == 0)  // (release: this wave's V columns before the count)
                __hip_atomic_fetch_add(&vreq[2], 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
    };
    // the helper waves meet without the walker, answering its requests meanwhile
    // (bounded; a timeout sets *bf.err and gives up)
    int hsync_target = 0;
    auto helper_sync = [&](const T* P) {
        hsync_target += NW - 1;
        if (l == 0) __hip_atomic_fetch_add(&misc[5], 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        for (uint32_t sp = 0;
             __hip_atomic_load(&misc[5], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < hsync_target; ++sp) {
            answer(P);
            if (sp > (1u << 22)) {
                if (l == 0) __hip_atomic_store(bf.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
    };
    // helpers: X = A W_c on their column tile; wave gw also the chunk's Gram matrix A A^T,
    // wave cw the cross Gram A A_c^T with the current chunk (none for a fresh chunk);
    // the walker's requests answered between groups of five k-steps (P: its chunk).
    // (the Gram matrices on waves 6 / 7 at NB = 7, off the walker's SIMD; KB2E_CONS_DBG bit 1:
    // waves 4 / 5, A/B; same results)
    const int gw = !(bf.dbg & 2) && NB >= 7 ? 6 : 4, cw = !(bf.dbg & 2) && NB >= 7 ? 7 : 5;
    auto x_tile = [&](const T* Ar, T* out, T* G, const T* Ac, const T* P) {
        if (!own) return;
        typename M::acc_t acc = {T(0), T(0), T(0), T(0)};
        typename M::acc_t ga = {T(0), T(0), T(0), T(0)};
#pragma unroll
        for (int q0 = 0; q0 < KS; q0 += 5) {
#pragma unroll
            for (int q = q0; q < q0 + 5 && q < KS; ++q) {
                const T av = Ar[l16 * LA + 4 * q + kq];
                acc = M::mma(av, bW[q], acc);
                if (w == gw) ga = M::mma(av, av, ga);
                else if (w == cw && Ac) ga = M::mma(av, Ac[l16 * LA + 4 * q + kq], ga);
            }
            if (P) answer(P);
        }
        if (col < NC) {
#pragma unroll
            for (int q = 0; q < 4; ++q) out[(kq + 4 * q) * LA + col] = acc[q];
        }
        if (w == gw) {
#pragma unroll
            for (int q = 0; q < 4; ++q) G[(kq + 4 * q) * LG + l16] = ga[q];
        }
        if (w == cw && Ac) {
#pragma unroll
            for (int q = 0; q < 4; ++q) Cx[(kq + 4 * q) * LG + l16] = ga[q];
        }
    };
    // helpers: |p_j|^2 partials of their columns (qpart[cb][j]) for the chunk's cc rows
    auto q_tile = [&](const T* Pr, int cc) {
        if (!own) return;
        T sq[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const T x = col < NC ? Pr[(kq + 4 * q) * LA + col] : T(0);
            sq[q] = x * x;
        }
        row16_sums<T, 4>(sq);
        if (l16 == 0) {
#pragma unroll
            for (int q = 0; q < 4; ++q) qpart[cb * R + kq + 4 * q] = kq + 4 * q < cc ? sq[q] : T(0);
        }
    };
    // the helpers' debt: the pending chunk's W_c -= lr A^T G on their tile and its pair
    // records; requests answered between violators (P: the current chunk)
    auto apply_pending = [&](const T* P) {
        if (!own || pend_nv == 0) return;
        const T* Pp = Pbuf + pend_pc * R * LA;
        const T* Ap = Abuf + pend_ka * R * LA;
        const int* vl = vlist + pend_par * R;
        for (int k = 0; k < pend_nv; ++k) {
            const int v = vl[k];
            const T gl = col < NC ? -lr * Pp[v * LA + col] : T(0);
#pragma unroll
            for (int q = 0; q < KS; ++q) bW[q] = fma(Ap[v * LA + 4 * q + kq], gl, bW[q]);
            if (P) answer(P);
        }
        for (int k = kq; k < pend_nv; k += 4) {
            const int v = vl[k];
            const int sl = ps[pend_base + v];
            T* dst = sl >= 0 ? bf.pair + (int64_t)sl * ld : bf.relpair + (int64_t)r * ld;
            if (col < n) dst[col] = Pp[v * LA + col];
            if (sl < 0 && cb == 0 && l16 == 0) bf.relpair_stamp[r] = bf.stamp;
        }
    };
    // helpers, until the walk of chunk ck ends: its requests, and each violator it
    // publishes (k-th of the chunk, vl[k]) folded into the next chunk's projections on
    // their columns, P_n[j] -= lr (a_n[j] . a_v) g_v (rows kq + 4 q < cn; no next chunk: cn 0)
    auto serve = [&](const T* P, const int* vl, int ck, T* Pn, int cn) {
        if (!own) return;
        int used = 0;
        for (uint32_t sp = 0;; ++sp) {
            answer(P);
            const bool done = __hip_atomic_load(&misc[6], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) == ck;
            const int pw = __hip_atomic_load(&misc[7], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
            const int avail = (pw >> 6) == ck ? (pw & 63) : 0;
            for (; used < avail; ++used) {
                if (cn == 0) continue;
                const int v = vl[used];
                const T gv = col < NC ? P[v * LA + col] : T(0);
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const int j = kq + 4 * q;
                    if (j < cn && col < NC) Pn[j * LA + col] = fma(-lr * Cx[j * LG + v], gv, Pn[j * LA + col]);
                }
            }
            if (done) break;
            if (sp > (1u << 22)) {
                if (l == 0) __hip_atomic_store(bf.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
    };
    // W_c's unit rows (transr/trainer.cpp:178-180) before the last update's pairs
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
    // j < cc), |p_j|^2 as qpart partials, the Gram matrix; the violators' rows of P become
    // G, each published to the helpers as it is made
    auto walk = [&](T* P, const T* Gm, int cc, int base, int* vl, int ck, int par) {
        const int j = l & (R - 1), h = l >> 4;  // lane: quarter h of row j
        T q = T(0);
        if (j < cc) {
            q = qpart[j];
            for (int v = 1; v < NB; ++v) q += qpart[v * R + j];
        }
        uint32_t vmask = 0;
        int npub = 0;
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
                // the violator's current row to LDS, then the request for its V
                if (j == v) {
#pragma unroll
                    for (int u = 0; u < KS; ++u) P[v * LA + h * KS + u] = x[u];
                }
                ++vreqs;
                if (l == 0) {
                    vreq[0] = v;
                    __hip_atomic_store(&vreq[1], vreqs, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
                }
                const T dp = Gm[j * LG + v];  // a_j . a_v for every row
                const T* pr = P + v * LA;
                const T pv0 = pr[l], pv1 = c1 < NC ? pr[c1] : T(0);
                const T pp = readlane_f(q, v);
                const T aa = readlane_f(dp, v);  // |a_v|^2
                T rpp = __builtin_amdgcn_rcp(pp);  // v_rcp_f64 and one Newton step
                rpp = fma(fma(-pp, rpp, T(1)), rpp, rpp);
                tick(5);
                for (uint32_t sp = 0;
                     __hip_atomic_load(&vreq[2], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < NB * vreqs; ++sp) {
                    if (sp > (1u << 24)) {
                        if (l == 0) __hip_atomic_store(bf.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        break;
                    }
                }
                const T V0 = Vrow[l], V1 = c1 < NC ? Vrow[c1] : T(0);
                tick(13);
                T s2[2] = {pv0 * V0 + pv1 * V1, V0 * V0 + V1 * V1};
                wave_sums<T, 2>(s2);
                const T pV = s2[0], VV = s2[1];
                const T pvd = pV + aa * pp, vvd = VV + T(2) * aa * pV + aa * aa * pp;
                const T kappa = pvd * rpp;
                const T w2t = vvd - kappa * pvd;
                const T w2 = w2t > T(0) ? w2t : T(0);
                const T rho = T(1) - eps * kappa;
                T S0, S1;
                const int m = transr_rounds_violator4(pp, w2, eps, rho, S0, S1);
                n_rounds += (unsigned long long)m;
                max_m = max_m > (unsigned long long)m ? max_m : (unsigned long long)m;
                const T cpf = T(2) * (S0 + eps * S1 * kappa), cvf = T(2) * eps * S1;
                // g (zero past n: p and V are); the violator's row now holds G
                P[v * LA + l] = cpf * pv0 - cvf * (V0 + aa * pv0);
                if (c1 < NC) P[v * LA + c1] = cpf * pv1 - cvf * (V1 + aa * pv1);
                // published to the helpers (its G row above and its vl entry first)
                if (l == 0) {
                    vl[npub] = v;
                    __hip_atomic_store(&misc[7], (ck << 6) | (npub + 1), __ATOMIC_RELEASE,
                                       __HIP_MEMORY_SCOPE_WORKGROUP);
                }
                ++npub;
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
        if (l < R && ((vmask >> l) & 1u)) vflag[base + l] = 1;
        if (l == 0) {
            misc[1 + 2 * par] = (int)vmask;
            misc[2 + 2 * par] = npub;
            __hip_atomic_store(&misc[6], ck, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
    };
    // the pipeline over the list's pairs [0, npw) (pe / ps), chunks of R; ends drained
    // (the last chunk's debt paid) after a barrier
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
        if (tid == 0) {
            vreq[1] = 0;
            vreq[2] = 0;
        }
        vreqs = 0;
        __syncthreads();
        x_tile(Abuf, Pbuf, Gbuf, nullptr, nullptr);  // chunk 0 afresh
        __syncthreads();
        q_tile(Pbuf, csz(0));
        __syncthreads();
        // one loop a role (the walker's path holds no helper fragment: they are dead there,
        // zeros on wave 0, and restated as such after its loop)
        if (w == 0) {
            for (int k = 0; k < nch; ++k) {
                const int pc = k & 1;
                const int ck = (int)n_chunks;  // the chunk's tag in the publish words (misc[6], misc[7])
                ++n_chunks;
                walk(Pbuf + pc * R * LA, Gbuf + pc * R * LG, csz(k), k * R, vlist + pc * R, ck, pc);
                tick(2);
                __syncthreads();  // B1: the walk, P_{k+1} and its |p|^2 partials
                tick(3);
                if (misc[2 + 2 * pc]) changed = true;
            }
#pragma unroll
            for (int q = 0; q < KS; ++q) bW[q] = kf[q] = T(0);
#pragma unroll
            for (int q = 0; q < RPT; ++q) rows[q] = T(0);
            rows_ok = 0;
        } else {
            for (int k = 0; k < nch; ++k) {
                const int cn = csz(k + 1);
                const int ka = k % 3, kn = (k + 1) % 3, pc = k & 1;
                const T* A = Abuf + ka * R * LA;
                const T* An = Abuf + kn * R * LA;
                const T* P = Pbuf + pc * R * LA;
                T* Pn = Pbuf + (pc ^ 1) * R * LA;
                T* Gn = Gbuf + (pc ^ 1) * R * LG;
                const int* vl = vlist + pc * R;
                const int ck = (int)n_chunks;
                ++n_chunks;
                apply_pending(P);  // chunk k - 1's
                tick(10);
                if (cn > 0) x_tile(An, Pn, Gn, A, P);
                helper_sync(P);  // the cross Gram (wave 5); every helper done with A slot k - 1
                tick(11);
                if (k + 2 < nch) {  // chunk k + 2's rows into the slot chunk k - 1 left, k + 3's in flight
                    store_rows((k + 2) % 3);
                    if (k + 3 < nch) load_rows((k + 3) * R, (k + 3) * R + csz(k + 3));
                }
                serve(P, vl, ck, Pn, cn);  // the rest of the walk
                if (cn > 0) q_tile(Pn, cn);
                tick(12);
                __syncthreads();  // B1
                tick(4);
                const int nv = misc[2 + 2 * pc];
                pend_nv = nv;
                pend_par = pc;
                pend_pc = pc;
                pend_ka = ka;
                pend_base = k * R;
                if (nv) changed = true;
            }
        }
        apply_pending(nullptr);
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
        __syncthreads();  // the window's list (and every thread past wsum: the requests reuse it)
        tick(1);
        if (npw > 0) run_list(npw);
        if (kk >= 0) {  // the flags of the window's slots (the tail's wait)
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
    // region) for the pair records da = -lr W G, made here
    const int LT = (n + 1) & ~1;
    static_assert(NC * LA >= NC * NC, "Wt fits K0's region");
    static_assert(3 * R * LA >= (NT / 64) * NC, "a G row a wave fits the row slots");
    static_assert(2 * kWPPairs + 2 * R >= 4 * NT + 1, "the record list fits the pair lists (and the violator lists)");
    __syncthreads();  // every walk done with the V row
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
            if (n_chunks >= 200) {
                for (int k = 0; k < 16; ++k) atomicAdd(&g_seq_stats[24 + k], ph[k]);
                atomicAdd(&g_seq_stats[40], n_chunks);
                atomicAdd(&g_seq_stats[41], 1ull);
                atomicAdd(&g_seq_stats[42], n_vio);
            }
        }
    }
}

}  // namespace kb2e
