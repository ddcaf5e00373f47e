// kernels_transe.hpp -- TransE batch kernels.
//
// score: phase A of one batch.  One wave per sample: gather the rows h, t, r
//   and the corrupting entity from the start-of-batch tables, both energies
//   (transe/transe.cpp:10-28), the hinge (common/trainer.cpp:130-149), and the
//   update directions x = 2((t - h) - r) (transe/trainer.cpp:29-35) -- as sign
//   bits for L1, as reals for L2.
// fold:  phase B.  One wave per (batch,row) segment replays that row's events
//   in sample order: the delta of each active update followed by common::norm
//   (transe/trainer.cpp:38-45).  TransE rows never interact inside a batch, so
//   the per-row fold is exactly the reference's sequential *_next_ update, and
//   it runs in place: every delta reads only phase-A outputs.
#pragma once

#include "kernels_common.hpp"

namespace kb2e {

template <typename T>
struct ScoreArgs {
    const int32_t* heads;
    const int32_t* tails;
    const int32_t* rels;
    const int32_t* si;  // sample stream of this batch (already offset)
    const int32_t* sj;
    const uint8_t* side;
    int32_t B, n, ld, nw;
    const T* ent;
    const T* rel;
    const T* w;  // TransH normals (R x ld) / TransR matrices
    double margin;
    uint8_t* act;       // [B]
    double* loss;       // [B]
    uint64_t* xbits;    // [B][2][nw]
    T* xreal;           // [B][2][ld] (L2 only)
};

template <typename T, int CH, bool L1>
__global__ __launch_bounds__(256) void transe_score_kernel(ScoreArgs<T> a) {
    const int kk = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (kk >= a.B) return;
    const int l = lane_id();
    const int i = a.si[kk], j = a.sj[kk];
    const int h = a.heads[i], t = a.tails[i], r = a.rels[i];
    const int nh = a.side[kk] ? h : j, nt = a.side[kk] ? j : t;
    RowReg<T, CH> H, Tt, R, NH, NT;
    H.load(a.ent + (int64_t)h * a.ld, a.n);
    Tt.load(a.ent + (int64_t)t * a.ld, a.n);
    R.load(a.rel + (int64_t)r * a.ld, a.n);
    NH.load(a.ent + (int64_t)nh * a.ld, a.n);
    NT.load(a.ent + (int64_t)nt * a.ld, a.n);
    T dp[CH][kVec], dn[CH][kVec];
    T ep = T(0), en = T(0);
#pragma unroll
    for (int c = 0; c < CH; ++c)
#pragma unroll
        for (int k = 0; k < kVec; ++k) {
            dp[c][k] = Tt.v[c][k] - H.v[c][k] - R.v[c][k];
            dn[c][k] = NT.v[c][k] - NH.v[c][k] - R.v[c][k];
            if (L1) {
                ep += fabs(dp[c][k]);
                en += fabs(dn[c][k]);
            } else {
                ep += dp[c][k] * dp[c][k];
                en += dn[c][k] * dn[c][k];
            }
        }
    ep = wave_sum(ep);
    en = wave_sum(en);
    // train_kb uses double arithmetic on the returned energies.
    const double e_pos = (double)ep, e_neg = (double)en;
    const bool active = e_pos + a.margin > e_neg;
    if (l == 0) {
        a.act[kk] = active ? 1 : 0;
        a.loss[kk] = active ? a.margin + e_pos - e_neg : 0.0;
    }
    if (!active) return;
    if (L1) {
#pragma unroll
        for (int c = 0; c < CH; ++c)
#pragma unroll
            for (int k = 0; k < kVec; ++k) {
                // x = 2 * d > 0  <=>  d > 0
                const bool valid = elem_valid(c, k, a.n);
                const uint64_t bp = __ballot(valid && dp[c][k] > T(0));
                const uint64_t bn = __ballot(valid && dn[c][k] > T(0));
                if (l == 0) {
                    a.xbits[((int64_t)kk * 2 + 0) * a.nw + c * kVec + k] = bp;
                    a.xbits[((int64_t)kk * 2 + 1) * a.nw + c * kVec + k] = bn;
                }
            }
    } else {
        T* xp = a.xreal + ((int64_t)kk * 2 + 0) * a.ld;
        T* xn = a.xreal + ((int64_t)kk * 2 + 1) * a.ld;
#pragma unroll
        for (int c = 0; c < CH; ++c)
#pragma unroll
            for (int k = 0; k < kVec; ++k) {
                const int e = c * (kWave * kVec) + l * kVec + k;
                if (e < a.n) {
                    xp[e] = T(2.0) * dp[c][k];
                    xn[e] = T(2.0) * dn[c][k];
                }
            }
    }
}

template <typename T>
struct FoldArgs {
    const uint64_t* keys;
    const int32_t* seg_start;
    const int32_t* batch_seg;
    int32_t batch;
    KeyLayout kl;
    int32_t ne, n, ld, nw;
    T* ent;
    T* rel;
    double lr;
    const uint8_t* act;     // [B] of this batch
    const uint64_t* xbits;  // [B][2][nw]
    const T* xreal;         // [B][2][ld]
    int32_t gram_min;       // segments at least this long take the scalar-recurrence path (0: never)
};

// ---- long L1 segments: the renormalisation recurrence on scalars ----------
//
// A row's events are v <- v + e_k then "if |v| > 1: v /= |v|", with
// e_k = s_k * lr * x_k, x_k in {+-1}^n (s_k = -1 relation / head role, +1 tail
// role, 0 when the update uses the row as head AND tail, whose two deltas
// cancel; transe/trainer.cpp:38-45).  Write v = A * u with
// u = v0 + sum_j beta_j e_j (beta_j = 1/A when e_j was added).  Then
//   |v + e_k|^2 = N + 2 A (v0.e_k + sum_{j<k} beta_j e_j.e_k) + |e_k|^2,
// with N = |v|^2, and e_j.e_k = s_j s_k lr^2 (n - 2 popcount(bits_j ^ bits_k)).
// Per chunk of 64 events: one reduction for N, 64 independent dot products
// v0.e_m (lane m), a scalar chain (sqrt, reciprocal) per event while each lane
// m accumulates S_m = sum_j beta_j e_j.e_m, and one elementwise
// materialisation v = A (v0 + sum beta_j e_j).  Same decisions as the
// reference; values agree to a few ulps per chunk.
// 1/sqrt(x) to ~full FP64 precision: hardware estimate + two Newton steps.
__device__ __forceinline__ double rsqrt_nr(double x) {
    double y = __builtin_amdgcn_rsq(x);
    y = y * (1.5 - 0.5 * x * y * y);
    y = y * (1.5 - 0.5 * x * y * y);
    return y;
}

template <typename T, int CH>
__device__ void fold_segment_gram(const FoldArgs<T>& a, int p0, int p1, bool is_rel, RowReg<T, CH>& V,
                                  double* lds_v, bool& dirty) {
    const int l = lane_id();
    const double lr = a.lr;
    const double lr2 = lr * lr;
    const double eps = lr2 * (double)a.n;
    for (int base = p0; base < p1; base += kWave) {
        const int cnt = min(kWave, p1 - base);
        uint64_t xw[2 * CH];
        int sgn = 0, nn = 0;
#pragma unroll
        for (int q = 0; q < 2 * CH; ++q) xw[q] = 0ull;
        if (l < cnt) {
            const uint64_t key = a.keys[base + l];
            const int kk = a.kl.kk_of(key);
            if (a.act[kk]) {
                const int u = (int)((key >> 3) & 1);
                const uint32_t roles = (uint32_t)(key & 7);
                // e = s * lr * x: relation and head rows take -d, tail rows +d,
                // d = (neg update ? +1 : -1) * lr * x (transe/trainer.cpp:26, 38-40)
                const int us = u ? 1 : -1;
                if (is_rel) {
                    sgn = -us;
                    nn = 1;
                } else {
                    const bool hd = roles & kRoleHead, tl = roles & kRoleTail;
                    sgn = (hd && tl) ? 0 : (hd ? -us : us);
                    nn = (hd ? 1 : 0) + (tl ? 1 : 0);
                }
#pragma unroll
                for (int q = 0; q < 2 * CH; ++q) xw[q] = a.xbits[((int64_t)kk * 2 + u) * a.nw + q];
            }
        }
        const uint64_t m_act = __ballot(nn > 0);
        if (!m_act) continue;
        const uint64_t m_sgn = __ballot(sgn != 0), m_n2 = __ballot(nn == 2);
        dirty = true;
        // p_m = s_m lr (v0 . x_m): v0 to LDS, lane m walks the row
#pragma unroll
        for (int c = 0; c < CH; ++c)
#pragma unroll
            for (int k = 0; k < kVec; ++k) {
                const int e = c * (kWave * kVec) + l * kVec + k;
                if (e < a.n) lds_v[e] = (double)V.v[c][k];
            }
        wave_lds_sync();
        double pm = 0;
        for (int e = 0; e < a.n; ++e) {
            const int c = e / (kWave * kVec), r = e % (kWave * kVec);
            const double v = lds_v[e];
            pm += ((xw[c * kVec + (r & 1)] >> (r >> 1)) & 1ull) ? v : -v;
        }
        pm *= (double)sgn * lr;
        // e_k . e_m / lr^2 = s_k s_m (n - 2 popcount(bits_k ^ bits_m)), for every k (lane m)
        int gk[kWave];
#pragma unroll
        for (int k = 0; k < kWave; ++k) {
            uint32_t dis = 0;
#pragma unroll
            for (int q = 0; q < 2 * CH; ++q) dis += (uint32_t)__popcll(xw[q] ^ readlane_u64(xw[q], k));
            gk[k] = readlane_i32(sgn, k) * sgn * (a.n - 2 * (int)dis);
        }
        double N = (double)V.sumsq();
        double A = 1.0, invA = 1.0, S = 0.0, beta_mine = 0.0;
#pragma unroll
        for (int k = 0; k < kWave; ++k) {
            if (!((m_act >> k) & 1ull)) continue;  // wave-uniform
            const double z2 = N + 2.0 * A * (readlane_f(pm, k) + readlane_f(S, k)) +
                              (((m_sgn >> k) & 1ull) ? eps : 0.0);
            beta_mine = (l == k) ? invA : beta_mine;
            S += invA * lr2 * (double)gk[k];
            double nz = z2;
            if (z2 > 1.0) {  // common::norm: len > 1 -> v /= len
                const double y = rsqrt_nr(z2);
                A *= y;
                invA *= z2 * y;
                nz = z2 * y * y;
            }
            if (((m_n2 >> k) & 1ull) && nz > 1.0) {  // second role of the same row
                const double y = rsqrt_nr(nz);
                A *= y;
                invA *= nz * y;
                nz = nz * y * y;
            }
            N = nz;
        }
        // v = A * (v0 + sum_k beta_k s_k lr x_k)
        double u[CH][kVec];
#pragma unroll
        for (int c = 0; c < CH; ++c)
#pragma unroll
            for (int k = 0; k < kVec; ++k) u[c][k] = (double)V.v[c][k];
#pragma unroll
        for (int k = 0; k < kWave; ++k) {
            if (!((m_sgn >> k) & 1ull)) continue;
            const double w = readlane_f(beta_mine, k) * (double)readlane_i32(sgn, k) * lr;
            uint64_t words[2 * CH];
#pragma unroll
            for (int q = 0; q < 2 * CH; ++q) words[q] = readlane_u64(xw[q], k);
#pragma unroll
            for (int c = 0; c < CH; ++c)
#pragma unroll
                for (int kv = 0; kv < kVec; ++kv) u[c][kv] += xbit(words, c, kv) ? w : -w;
        }
#pragma unroll
        for (int c = 0; c < CH; ++c)
#pragma unroll
            for (int k = 0; k < kVec; ++k) V.v[c][k] = elem_valid(c, k, a.n) ? (T)(A * u[c][k]) : T(0);
        wave_lds_sync();
    }
}

template <typename T, int CH, bool L1>
__global__ __launch_bounds__(256) void transe_fold_kernel(FoldArgs<T> a) {
    __shared__ double lds_v[4 * CH * kWave * kVec];  // one row per wave (gram path)
    const int s0 = a.batch_seg[a.batch], s1 = a.batch_seg[a.batch + 1];
    const int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int nwaves = (gridDim.x * blockDim.x) >> 6;
    const int l = lane_id();
    // Relation rows sort last and carry the longest event chains: start them first.
    for (int s = s1 - 1 - wave; s >= s0; s -= nwaves) {
        const int p0 = a.seg_start[s], p1 = a.seg_start[s + 1];
        const int row = a.kl.row_of(a.keys[p0]);
        const bool is_rel = row >= a.ne;
        T* ptr = is_rel ? a.rel + (int64_t)(row - a.ne) * a.ld : a.ent + (int64_t)row * a.ld;
        RowReg<T, CH> V;
        V.load(ptr, a.n);
        bool dirty = false;
        if (L1 && a.gram_min > 0 && p1 - p0 >= a.gram_min) {
            fold_segment_gram<T, CH>(a, p0, p1, is_rel, V, lds_v + (threadIdx.x >> 6) * (CH * kWave * kVec), dirty);
            if (dirty) V.store(ptr, a.n);
            continue;
        }
        for (int base = p0; base < p1; base += kWave) {
            // Prefetch up to 64 events: lane q holds event base+q.
            const int cnt = min(kWave, p1 - base);
            uint64_t key = 0;
            int active = 0;
            uint64_t xw[2 * CH];
            if (l < cnt) {
                key = a.keys[base + l];
                const int kk = a.kl.kk_of(key);
                active = a.act[kk];
                if (L1 && active) {
                    const int u = (int)((key >> 3) & 1);
#pragma unroll
                    for (int q = 0; q < 2 * CH; ++q) xw[q] = a.xbits[((int64_t)kk * 2 + u) * a.nw + q];
                }
            }
            for (int e = 0; e < cnt; ++e) {
                if (!readlane_i32(active, e)) continue;
                const uint64_t ke = readlane_u64(key, e);
                const int u = (int)((ke >> 3) & 1);
                const uint32_t roles = (uint32_t)(ke & 7);
                const int kk = a.kl.kk_of(ke);
                // modifier * learningRate_ (transe/trainer.cpp:26, 38-40)
                const T c = (T)((u ? 1.0 : -1.0) * a.lr);
                T d[CH][kVec];
                if (L1) {
                    uint64_t words[2 * CH];
#pragma unroll
                    for (int q = 0; q < 2 * CH; ++q) words[q] = readlane_u64(xw[q], e);
#pragma unroll
                    for (int cc = 0; cc < CH; ++cc)
#pragma unroll
                        for (int k = 0; k < kVec; ++k) d[cc][k] = xbit(words, cc, k) ? c : -c;
                } else {
                    const T* xr = a.xreal + ((int64_t)kk * 2 + u) * a.ld;
#pragma unroll
                    for (int cc = 0; cc < CH; ++cc)
#pragma unroll
                        for (int k = 0; k < kVec; ++k) {
                            const int el = cc * (kWave * kVec) + l * kVec + k;
                            d[cc][k] = el < a.n ? c * xr[el] : T(0);
                        }
                }
                int nnorm = 1;
#pragma unroll
                for (int cc = 0; cc < CH; ++cc)
#pragma unroll
                    for (int k = 0; k < kVec; ++k) {
                        if (!elem_valid(cc, k, a.n)) continue;
                        if (is_rel) {
                            V.v[cc][k] = V.v[cc][k] - d[cc][k];
                        } else {
                            if (roles & kRoleHead) V.v[cc][k] = V.v[cc][k] - d[cc][k];
                            if (roles & kRoleTail) V.v[cc][k] = V.v[cc][k] + d[cc][k];
                        }
                    }
                if (!is_rel) nnorm = ((roles & kRoleHead) ? 1 : 0) + ((roles & kRoleTail) ? 1 : 0);
                for (int q = 0; q < nnorm; ++q) V.norm(a.n, true);
                dirty = true;
            }
        }
        if (dirty) V.store(ptr, a.n);
    }
}

}  // namespace kb2e
