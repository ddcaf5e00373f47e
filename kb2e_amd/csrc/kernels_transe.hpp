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
};

template <typename T, int CH, bool L1>
__global__ __launch_bounds__(256) void transe_fold_kernel(FoldArgs<T> a) {
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
