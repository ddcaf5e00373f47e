// kernels_transr_wave.hpp -- the PARALLEL TransR tile passes without LDS
// staging of the small operands (companion of kernels_transr_cons.hpp).
//
// Gradient partials (transr/trainer.cpp:166-167, :171): per tile of <= St
// samples of relation r, over its updates u = 2 q + side (beta_u = +1 for the
// corrupted triple, -1 for the training one, coefficient c_u = -lr beta_u if
// the sample is hinge-active, else 0)
//   dW[j][i] = sum_u c_u d_u[j] x_u[i]      d = h - t (snapshot), x the direction
//   dr[i]    = sum_u c_u x_u[i]
// dW is an MFMA product with the updates as the contraction: its A and B
// fragments are exactly rows of the phase-A exports bf.d and bf.x read from
// L2 (lane l & 15 -> column, lane l >> 4 -> update), so the kernel needs no
// LDS and no barrier; every operand load of a wave is issued before its MFMAs.
//
// Phase A (transr/trainer.cpp:147-164, transr/transr.cpp:13-35): per tile the
// projections P = V W0 of the rows v = h, t, h', t' of its samples, taken
// transposed (P^T = W0^T V^T) with the V rows as the MFMA's N dimension: rows
// 4 q + {0, 1, 2, 3} of a 16-row block are one sample's h, t, h', t' and sit
// in one DPP quad of every lane group, so d_p = p_t - p_h - r and x (the L1
// sign / L2 2 d_p), the energies and the raw d = h - t come from quad_perm
// moves, y = W0 x is the MFMA product Y^T = W0 X^T with the x fragments as
// the B operand, and only W0 is staged in LDS (its live rows, 27.5 KB at
// n = 50: five workgroups of two waves per CU).
#pragma once

#include "kernels_transr_cons.hpp"

namespace kb2e {

// the value of quad lane Q (lanes 4 (l / 4) + Q) in every lane of the quad
template <int Q>
__device__ __forceinline__ float quad_bcast(float x) {
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), Q * 0x55, 0xF, 0xF, false));
}
template <int Q>
__device__ __forceinline__ double quad_bcast(double x) {
    const long long b = __double_as_longlong(x);
    const int lo = __builtin_amdgcn_mov_dpp((int)(b & 0xffffffff), Q * 0x55, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_mov_dpp((int)(b >> 32), Q * 0x55, 0xF, 0xF, false);
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

constexpr int kProjWaves = 2;  // 4 St <= 32 rows: two 16-row blocks

// W0 rows transr_proj_wave_kernel stages: FP64 reads rows k = kmap(s, kq) < 4 KS
// only (rows >= n are zero, so the y product masks the rest instead of reading
// them: 27.5 KB instead of 34 KB at n = 50, five workgroups a CU instead of four)
template <typename T>
__host__ __device__ constexpr int proj_wave_rows(int KS) {
    return sizeof(T) == 8 ? 4 * KS : 16 * ((KS + 3) / 4);
}

template <typename T, int KS>
__global__ __launch_bounds__(128) void transr_proj_wave_kernel(RParArgs a, RParBufs<T> bf) {
    using M = Mfma16<T>;
    constexpr int NB = (KS + 3) / 4, NP = 16 * NB, L = NP + 2, NS = NP / 4, R = proj_wave_rows<T>(KS);
    extern __shared__ __attribute__((aligned(16))) char smem[];
    // fixed energy: this kernel fills the pair-dedupe table (every thread of the grid
    // clears its share of the next batch's first)
    if (!a.compat) ptab_clear_next(a, (int64_t)blockIdx.x * blockDim.x + threadIdx.x, (int64_t)gridDim.x * blockDim.x);
    // the tile from the per-epoch descriptors: two dependent loads to the rows
    const int t = a.batch_t0[a.batch] + blockIdx.x;
    if (t >= a.batch_t0[a.batch + 1]) return;
    const int r = a.td_r[t], cnt = a.td_cnt[t] & 255;
    const int n = a.n, ld = a.ld;
    const int w = threadIdx.x >> 6, l = lane_id(), kq = l >> 4, l16 = l & 15;
    T* Wl = (T*)smem;
    // this lane's row: sample q, role which (0 h, 1 t, 2 h', 3 t')
    const int q = w * 4 + (l16 >> 2), which = l16 & 3;
    const bool has = q < cnt;
    const int kk = a.td_kk[t * 8 + q];
    const int ed = a.td_ent[(t * 8 + q) * 4 + which];
    const int e = ed < 0 ? 0 : ed;
    {  // W0 as element pairs, every load in flight before the LDS stores
        using T2 = typename std::conditional<sizeof(T) == 8, double2, float2>::type;
        constexpr int kPairs = R * L / 2, kThreads = kProjWaves * kWave;
        constexpr int kPer = (kPairs + kThreads - 1) / kThreads;
        const T2* Wg = (const T2*)(bf.W + (int64_t)r * n * ld);
        const int hp = ld / 2;
        T2 v[kPer];
#pragma unroll
        for (int p = 0; p < kPer; ++p) {
            const int idx = threadIdx.x + p * kThreads;
            const int j = idx / (L / 2), ip = idx % (L / 2);
            const bool ok = idx < kPairs && j < n && ip < hp;
            const T2 g = Wg[ok ? j * hp + ip : 0];
            v[p] = ok ? g : T2{T(0), T(0)};
        }
#pragma unroll
        for (int p = 0; p < kPer; ++p) {
            const int idx = threadIdx.x + p * kThreads;
            if (idx < kPairs) ((T2*)Wl)[idx] = v[p];
        }
    }
    // the V row and the relation vector as B fragments (unconditional in-row loads, masked)
    T vf[KS], rf[KS];
    {
        const T* vr = bf.ent + (int64_t)e * ld;
        const T* rr = bf.rel + (int64_t)r * ld;
#pragma unroll
        for (int s = 0; s < KS; ++s) {
            const int k = kmap<T>(s, kq);
            const T m = (has && k < n) ? T(1) : T(0);
            vf[s] = vr[k < n ? k : 0] * m;
            rf[s] = rr[k < n ? k : 0] * m;
        }
    }
    __syncthreads();
    if (w * 16 >= 4 * cnt) return;  // no sample in this block
    // P^T = W0^T V^T
    T pf[NS];
#pragma unroll
    for (int ib = 0; ib < NB; ++ib) {
        typename M::acc_t acc = {T(0), T(0), T(0), T(0)};
#pragma unroll
        for (int s = 0; s < KS; ++s) acc = M::mma(Wl[kmap<T>(s, kq) * L + ib * 16 + l16], vf[s], acc);
#pragma unroll
        for (int k = 0; k < 4; ++k) pf[4 * ib + k] = acc[k];
    }
    // the t / t' lanes: d_p = p_t - p_h - r (x from it), d = h - t; compat: every row's projection
    const bool upd = has && (which & 1);
    const int u = which >> 1;  // 0: the training triple, 1: the corrupted one
    T xf[NS];
    T en = T(0);
    T* xrow = bf.x + ((int64_t)kk * 2 + u) * ld;
    T* drow = bf.d + ((int64_t)kk * 2 + u) * ld;
    double* prow = a.proj + ((int64_t)kk * 4 + which) * ld;
#pragma unroll
    for (int s = 0; s < NS; ++s) xf[s] = T(0);
#pragma unroll
    for (int s = 0; s < KS; ++s) {
        const int k = kmap<T>(s, kq);
        const T ph = (which & 2) ? quad_bcast<2>(pf[s]) : quad_bcast<0>(pf[s]);
        const T vh = (which & 2) ? quad_bcast<2>(vf[s]) : quad_bcast<0>(vf[s]);
        const T dp = pf[s] - ph - rf[s];
        en += a.l1 ? fabs(dp) : dp * dp;
        xf[s] = upd && k < n ? (a.l1 ? (dp > T(0) ? T(1) : T(-1)) : T(2) * dp) : T(0);
        if (upd && k < n) {
            xrow[k] = xf[s];
            drow[k] = vh - vf[s];
        }
        if (a.compat && has && k < n) prow[k] = (double)pf[s];
    }
    if (!a.compat) {  // energies, hinge (common/trainer.cpp:138-141) on the t' lane of the sample
        const T er = row4_sum(en);
        const T ep = quad_bcast<1>(er);
        if (has && which == 3 && kq == 0) {
            const bool active = (double)ep + a.margin > (double)er;
            a.act[kk] = active ? 1 : 0;
            a.loss[kk] = active ? a.margin + (double)ep - (double)er : 0.0;
        }
        // every row of an active sample records its (entity, r) slot for the pair dedupe
        const T en3 = quad_bcast<3>(er);
        if (has && kq == 0 && (double)ep + a.margin > (double)en3) ptab_insert(a, r, e, kk * 4 + which);
    }
    // y = W0 x (transr/trainer.cpp:168-169): Y^T = W0 X^T, the t / t' columns
    T* yrow = bf.y + ((int64_t)kk * 2 + u) * ld;
#pragma unroll
    for (int jb = 0; jb < NB; ++jb) {
        typename M::acc_t acc = {T(0), T(0), T(0), T(0)};
#pragma unroll
        for (int s = 0; s < KS; ++s) {
            const int jr = jb * 16 + l16;  // rows >= R (all >= n) are zero
            acc = M::mma(jr < R ? Wl[jr * L + kmap<T>(s, kq)] : T(0), xf[s], acc);
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int j = jb * 16 + M::row(l, k);
            if (upd && j < n) yrow[j] = acc[k];
        }
    }
}

template <typename T, int KS>
__global__ __launch_bounds__(256) void transr_grad_wave_kernel(RParArgs a, RParBufs<T> bf) {
    using M = Mfma16<T>;
    constexpr int NB = (KS + 3) / 4;
    constexpr int kOut = (NB * NB + kConsWaves - 1) / kConsWaves;  // output tiles per wave
    constexpr int kSteps = 4;  // 2 St <= 16 updates (St <= 8 on the matrix-core path)
    const int t = a.batch_t0[a.batch] + blockIdx.x;
    if (t >= a.batch_t0[a.batch + 1]) return;
    const int r = a.td_r[t], cnt = a.td_cnt[t] & 255, single = (a.td_cnt[t] >> 8) & 1;
    const int n = a.n, ld = a.ld;
    const int w = threadIdx.x >> 6, l = lane_id(), kq = l >> 4, l16 = l & 15;
    const int nu = 2 * cnt;
    // this lane's update of every k-step (u = 4 s + l / 16: sample u / 2, update u & 1):
    // export row and coefficient
    int rowu[kSteps];
    T cu[kSteps];
#pragma unroll
    for (int s = 0; s < kSteps; ++s) {
        const int u = 4 * s + kq;
        const int kk = a.td_kk[t * 8 + (u >> 1)], side = u & 1;
        rowu[s] = kk * 2 + side;
        cu[s] = (u < nu && a.act[kk]) ? (T)(-(side ? 1.0 : -1.0) * a.lr) : T(0);
    }
    T* const wp = bf.wpart + (int64_t)blockIdx.x * n * ld;
#pragma unroll
    for (int q = 0; q < kOut; ++q) {
        const int tile = w + kConsWaves * q;
        if (tile >= NB * NB) break;
        const int jb = tile / NB, ib = tile % NB;
        const int j = jb * 16 + l16, i = ib * 16 + l16;
        T av[kSteps], bv[kSteps];
#pragma unroll
        for (int s = 0; s < kSteps; ++s) {  // unconditional in-row loads, masked by products
            av[s] = cu[s] * bf.d[(int64_t)rowu[s] * ld + (j < n ? j : 0)] * (j < n ? T(1) : T(0));
            bv[s] = bf.x[(int64_t)rowu[s] * ld + (i < n ? i : 0)] * (i < n ? T(1) : T(0));
        }
        typename M::acc_t acc = {T(0), T(0), T(0), T(0)};
#pragma unroll
        for (int s = 0; s < kSteps; ++s) acc = M::mma(av[s], bv[s], acc);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int jj = jb * 16 + M::row(l, k);
            if (jj < n && i < n) wp[(int64_t)jj * ld + i] = acc[k];
        }
        if (jb == 0) {  // dr over this column block: row 0 of (c^T) X, c in row 0 of A
            typename M::acc_t dr = {T(0), T(0), T(0), T(0)};
#pragma unroll
            for (int s = 0; s < kSteps; ++s) dr = M::mma(l16 == 0 ? cu[s] : T(0), bv[s], dr);
            if (M::row(l, 0) == 0 && i < n) bf.rpart[(int64_t)blockIdx.x * ld + i] = dr[0];
        }
    }
    if (w == 0) {  // the tile's active updates: lane u holds update u (nu <= 16), one ballot
        const bool au = l < nu && a.act[a.td_kk[t * 8 + (l >> 1)]] != 0;
        const uint64_t m = __ballot(au);
        if (l == 0) a.tile_act[t] = __builtin_popcountll(m);
    }
    if (w == kConsWaves - 1) {
        // the tile's transRNorm pairs for transr_cons_wave_kernel: (h', r), (t', r) of the
        // active updates in (sample, update, role) order -- phase A's V rows -- then
        // (entity'[r], r) on the relation's first tile if any of its samples is active;
        // first occurrences per relation per batch only (transr_pair_dup: across the
        // relation's tiles; the LDS check below catches nothing more), compacted;
        // pairs without a row get pflag 0
        __shared__ int ents[kCPairs];
        const RTile tl = a.tiles[t];
        bool relpair = false;
        if (tl.q == 0 && r < a.ne) {
            const int p0 = a.seg_start[tl.seg], ns = (a.seg_start[tl.seg + 1] - p0) / 2;
            for (int m0 = 0; m0 < ns && !relpair; m0 += kWave)
                relpair = __ballot(m0 + l < ns && a.act[a.kl.kk_of(a.keys[p0 + 2 * (m0 + l)])]) != 0;
        }
        const int pq = l;
        int ent = -1, slot = -1;
        if (pq < 4 * cnt) {
            const int q = pq >> 2, u = (pq >> 1) & 1, role = pq & 1;
            const int kk = a.td_kk[t * 8 + q];
            if (a.act[kk]) {
                slot = (kk * 2 + u) * 2 + role;
                const int e = a.td_ent[t * 32 + pq];
                if (!transr_pair_dup(a, slot, r, e)) ent = e;
            }
        } else if (pq == 4 * cnt && relpair && !transr_relpair_dup(a, r)) {
            ent = r;  // entityVec_next_[relation] (transr/trainer.cpp:187)
            slot = -2;
        }
        ents[pq] = ent;
        wave_lds_sync();
        bool dup = false;
        for (int k = 0; k < kCPairs; k += 4) {
            const int4 e4 = *(const int4*)(ents + k);
            dup |= (k < pq && e4.x == ent) | (k + 1 < pq && e4.y == ent) | (k + 2 < pq && e4.z == ent) |
                   (k + 3 < pq && e4.w == ent);
        }
        const bool live = ent >= 0 && !dup;
        const uint64_t m = __ballot(live);
        const int pos = __builtin_popcountll(m & ((1ull << l) - 1));
        int32_t* cp = bf.cpairs + (int64_t)blockIdx.x * 2 * kCPairs;
        if (live) {
            cp[pos] = ent;
            cp[kCPairs + pos] = slot;
        } else if (slot >= 0) {
            bf.pflag[slot] = 0;
        }
        // rows | the relation's only tile | relation, for the transRNorm kernel
        if (l == 0) bf.cnrows[blockIdx.x] = __builtin_popcountll(m) | (single << 7) | (r << 8);
    }
}

}  // namespace kb2e
