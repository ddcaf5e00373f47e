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
    int32_t B, n, ld, nw, ne;
    const T* ent;
    const T* rel;
    const T* w;  // TransH normals (R x ld) / TransR matrices
    double margin;
    uint8_t* act;       // [B]
    double* loss;       // [B]
    uint64_t* xbits;    // [B][2][nw]
    T* xreal;           // [B][2][ld] (L2 only)
};

// Per-event records written by phase A in sorted-event order (position p of
// the epoch's event index): meta = (s + 1) | nn << 2 | (2 kk + u) << 4 with s
// the sign of the event's delta (0: none) and nn its norm count; L1 also the
// event's sign words.  Phase B then reads each segment's events contiguously.
struct EventRecs {
    int32_t* meta;     // [nkeys]
    uint64_t* words;   // [nkeys][nw] (L1)
    const int32_t* inv;       // unsorted slot -> sorted position
    const uint64_t* keys;     // unsorted keys (emit order: sample * slots + slot)
    const int32_t* seg_row;   // [nseg] row of each segment
    int32_t slots;
};

__device__ __forceinline__ int32_t pack_meta(int sgn, int nn, int xrow) { return (sgn + 1) | (nn << 2) | (xrow << 4); }

// Phase A side: lanes 0..slots-1 of the sample's wave write the records of the
// sample's events (transe/trainer.cpp:36-40 signs: relation and head rows -d,
// tail rows +d, d = (corrupted ? +1 : -1) lr x).  The slot's key and sorted
// position are fetched at kernel start (prefetch) and used at the end (write).
struct EventSlot {
    uint64_t key = kSentinelKey;
    int p = 0;
    __device__ __forceinline__ void prefetch(const EventRecs& er, int64_t k) {
        const int l = lane_id();
        if (l < er.slots) {
            key = er.keys[k * er.slots + l];
            p = er.inv[k * er.slots + l];
        }
    }
    template <int NW>
    __device__ __forceinline__ void write(const EventRecs& er, const KeyLayout& kl, int32_t ne, int kk, bool active,
                                          const uint64_t (&bp)[NW], const uint64_t (&bn)[NW], int nw) const {
        if (key == kSentinelKey) return;
        const int u = (int)((key >> 3) & 1);
        const uint32_t roles = (uint32_t)(key & 7);
        const bool is_rel = kl.row_of(key) >= ne;
        int sgn = 0, nn = 0;
        if (active) {
            const int us = u ? 1 : -1;
            if (is_rel) {
                sgn = -us;
                nn = 1;
            } else {
                const bool hd = roles & kRoleHead, tl = roles & kRoleTail;
                sgn = (hd && tl) ? 0 : (hd ? -us : us);
                nn = (hd ? 1 : 0) + (tl ? 1 : 0);
            }
            if (sgn != 0)
                for (int w = 0; w < nw; ++w) er.words[(int64_t)p * nw + w] = u ? bn[w] : bp[w];
        }
        er.meta[p] = pack_meta(sgn, nn, kk * 2 + u);
    }
};

// EMIT (PARALLEL schedule): also write the sample's event records.
template <typename T, int CH, bool L1, bool EMIT = false>
__global__ __launch_bounds__(256) void transe_score_kernel(ScoreArgs<T> a, EventRecs er = {}, KeyLayout kl = {},
                                                           int64_t kbase = 0) {
    const int kk = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (kk >= a.B) return;
    const int l = lane_id();
    EventSlot slot;
    if (EMIT) slot.prefetch(er, kbase + kk);
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
    uint64_t bpw[CH * kVec], bnw[CH * kVec];
    if (!active) {
        if (EMIT) slot.write<CH * kVec>(er, kl, a.ne, kk, false, bpw, bnw, a.nw);
        return;
    }
    if (L1) {
#pragma unroll
        for (int c = 0; c < CH; ++c)
#pragma unroll
            for (int k = 0; k < kVec; ++k) {
                // x = 2 * d > 0  <=>  d > 0
                const bool valid = elem_valid(c, k, a.n);
                const uint64_t bp = __ballot(valid && dp[c][k] > T(0));
                const uint64_t bn = __ballot(valid && dn[c][k] > T(0));
                bpw[c * kVec + k] = bp;
                bnw[c * kVec + k] = bn;
                if (!EMIT && l == 0) {
                    a.xbits[((int64_t)kk * 2 + 0) * a.nw + c * kVec + k] = bp;
                    a.xbits[((int64_t)kk * 2 + 1) * a.nw + c * kVec + k] = bn;
                }
            }
        if (EMIT) slot.write<CH * kVec>(er, kl, a.ne, kk, true, bpw, bnw, a.nw);
    } else {
        if (EMIT) slot.write<CH * kVec>(er, kl, a.ne, kk, true, bpw, bnw, 0);
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
    int32_t long_min;       // segments at least this long are left to transe_fold_long_kernel (0: none)
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
// 1/sqrt(x) to ~full FP64 precision: hardware estimate (rel. error ~5e-8 on
// gfx950, tools/diag/rsq_accuracy.hip) + one third-order correction:
// 1/sqrt(x) = y (1 - r)^-1/2 = y (1 + r/2 + 3r^2/8 + O(r^3)), r = 1 - x y^2.
// 5 dependent operations instead of the 8 of two Newton steps.
__device__ __forceinline__ double rsqrt_nr(double x) {
    const double y = __builtin_amdgcn_rsq(x);
    const double xy = x * y;
    const double r = fma(-xy, y, 1.0);
    const double p = fma(r, 0.375, 0.5);
    return fma(y, r * p, y);
}

// Per-wave LDS of the recurrence path.
template <int CH>
struct GramLds {
    double v[CH * kWave * kVec];   // v0 of the chunk (broadcast reads)
    uint64_t x[kWave][2 * CH];     // sign words of the chunk's active events, compacted
    double4 ev[kWave];             // per active event: {lr v0.x, 2 s, |e|^2, s lr^2}
    int s[kWave];                  // s of the active events, compacted
};

// Events of one chunk, one per lane: s (sign of e), number of norms, x words.
template <int CH>
struct ChunkEvents {
    int sgn, nn;
    uint64_t xw[2 * CH];
};

// Raw loads of a chunk's event data (decoded later, so issuing them does not
// wait for them).
template <typename T, int CH>
struct ChunkLoads {
    uint64_t key;
    uint32_t act;
    uint64_t xw[2 * CH];
    __device__ __forceinline__ void issue(const FoldArgs<T>& a, bool valid) {
        act = 0;
#pragma unroll
        for (int q = 0; q < 2 * CH; ++q) xw[q] = 0ull;
        if (valid) {
            const int kk = a.kl.kk_of(key);
            const int u = (int)((key >> 3) & 1);
            act = a.act[kk];
#pragma unroll
            for (int q = 0; q < 2 * CH; ++q) xw[q] = a.xbits[((int64_t)kk * 2 + u) * a.nw + q];
        }
    }
    __device__ __forceinline__ ChunkEvents<CH> decode(bool valid, bool is_rel) const {
        ChunkEvents<CH> ev;
        ev.sgn = 0;
        ev.nn = 0;
#pragma unroll
        for (int q = 0; q < 2 * CH; ++q) ev.xw[q] = 0ull;
        if (valid && act) {
            // e = s * lr * x: relation and head rows take -d, tail rows +d,
            // d = (neg update ? +1 : -1) * lr * x (transe/trainer.cpp:26, 38-40)
            const int us = ((key >> 3) & 1) ? 1 : -1;
            const uint32_t roles = (uint32_t)(key & 7);
            if (is_rel) {
                ev.sgn = -us;
                ev.nn = 1;
            } else {
                const bool hd = roles & kRoleHead, tl = roles & kRoleTail;
                ev.sgn = (hd && tl) ? 0 : (hd ? -us : us);
                ev.nn = (hd ? 1 : 0) + (tl ? 1 : 0);
            }
#pragma unroll
            for (int q = 0; q < 2 * CH; ++q) ev.xw[q] = xw[q];
        }
        return ev;
    }
};

template <typename T, int CH>
__device__ void fold_segment_gram(const FoldArgs<T>& a, int p0, int p1, bool is_rel, RowReg<T, CH>& V,
                                  GramLds<CH>* L, bool& dirty) {
    constexpr int NW = 2 * CH;
    const int l = lane_id();
    const double lr = a.lr;
    const double lr2 = lr * lr;
    const double eps = lr2 * (double)a.n;
    // first chunk: synchronous
    ChunkLoads<T, CH> ld;
    ld.key = p0 + l < p1 ? a.keys[p0 + l] : 0ull;
    ld.issue(a, p0 + l < p1);
    ChunkEvents<CH> ev = ld.decode(p0 + l < p1, is_rel);
#ifdef KB2E_OWNER_PROF
    PhaseClock pc;
    pc.start();
#endif
    for (int base = p0; base < p1; base += kWave) {
        const int nbase = base + kWave;
        const bool nvalid = nbase + l < p1;
        ChunkLoads<T, CH> nld;
        nld.key = nvalid ? a.keys[nbase + l] : 0ull;  // level 1 of the next chunk
        const uint64_t m_act = __ballot(ev.nn > 0);
        if (m_act) {
            dirty = true;
            // Active events only, in order, moved to lanes 0..cnt-1 (inactive
            // samples leave the row untouched).
            const int cnt = __popcll(m_act);
            const int pos = __builtin_amdgcn_mbcnt_hi((uint32_t)(m_act >> 32),
                                                      __builtin_amdgcn_mbcnt_lo((uint32_t)m_act, 0u));
            if (ev.nn > 0) {
#pragma unroll
                for (int q = 0; q < NW; ++q) L->x[pos][q] = ev.xw[q];
                L->s[pos] = ev.sgn;
            }
            // v0 (zero padding included) to LDS
#pragma unroll
            for (int c = 0; c < CH; ++c)
#pragma unroll
                for (int k = 0; k < kVec; ++k) L->v[c * (kWave * kVec) + l * kVec + k] = (double)V.v[c][k];
            wave_lds_sync();
            uint64_t xw[NW];
#pragma unroll
            for (int q = 0; q < NW; ++q) xw[q] = l < cnt ? L->x[l][q] : 0ull;
            const int sg = l < cnt ? L->s[l] : 0;
            // pm_m = lr (v0 . x_m): element pair (128c + 2j, +1) has sign bits j
            // of words 2c and 2c + 1; four partial sums, groups of 8 pairs past
            // the row's end skipped.
            double pq[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
            for (int c = 0; c < CH; ++c)
#pragma unroll
                for (int j0 = 0; j0 < kWave; j0 += 8) {
                    if (c * (kWave * kVec) + 2 * j0 >= a.n) continue;  // wave-uniform
#pragma unroll
                    for (int j = j0; j < j0 + 8; ++j) {
                        const double2 vv = *reinterpret_cast<const double2*>(&L->v[c * (kWave * kVec) + 2 * j]);
                        const bool b0 = (xw[c * kVec] >> j) & 1ull, b1 = (xw[c * kVec + 1] >> j) & 1ull;
                        pq[(2 * j) & 3] += b0 ? vv.x : -vv.x;
                        pq[(2 * j + 1) & 3] += b1 ? vv.y : -vv.y;
                    }
                }
            const double sd = (double)sg;
            L->ev[l] = make_double4(((pq[0] + pq[1]) + (pq[2] + pq[3])) * lr, 2.0 * sd, sg != 0 ? eps : 0.0,
                                    sd * lr2);
            wave_lds_sync();
            nld.issue(a, nvalid);  // level 2 of the next chunk: in flight during the chain
            OWNER_MARK(1);
            // The chain, one active event per step, branch free.  With
            // e_k = s_k lr x_k, write v = A (v0 + sum_{j<k} beta_j e_j); then
            //   |v + e_k|^2 = N + 2 A s_k (lr v0.x_k + T_k) + |e_k|^2,
            //   T_m = sum_{j<m} beta_j s_j lr^2 (n - 2 popcount(bits_j ^ bits_m)),
            // which lane m accumulates one event at a time (x_j . x_m from the
            // sign words).  Only z2 -> rsqrt -> scale -> next z2 is serial: the
            // next event's 2 A s (pm + T) is formed from values known at the
            // start of a step, and a renormalised row's squared length is
            // tracked as exactly 1 (so a row used as head and tail, e = 0 with
            // two norms, needs one step).  Event k+1's table entry and sign
            // words are read from LDS one step ahead.
            double N = (double)V.sumsq();
            double A = 1.0, invA = 1.0, Tm = 0.0, beta_mine = 0.0;
            double f = 1.0;  // scale applied by the previous step
            // event table entries read two steps ahead, sign words one step
            auto tcoef = [&](const uint64_t (&xk)[NW]) {
                uint32_t dis = 0;
#pragma unroll
                for (int q = 0; q < NW; ++q) dis += (uint32_t)__popcll(xw[q] ^ xk[q]);
                return (double)(a.n - 2 * (int)dis);
            };
            double4 ek = L->ev[0], e1 = L->ev[1];
            double P = ek.y * ek.x;  // 2 A_{-1} s_0 (pm_0 + T_0), A_{-1} = 1, T_0 = 0
            uint64_t x1[NW];
#pragma unroll
            for (int q = 0; q < NW; ++q) x1[q] = L->x[0][q];
            double tk = tcoef(x1);
#pragma unroll
            for (int q = 0; q < NW; ++q) x1[q] = L->x[1][q];
#pragma unroll 1
            for (int k = 0; k < cnt; ++k) {
                const int k1 = k + 1 < kWave ? k + 1 : k;
                const int k2 = k + 2 < kWave ? k + 2 : kWave - 1;
                double4 e2 = L->ev[k2];
                uint64_t x2[NW];
#pragma unroll
                for (int q = 0; q < NW; ++q) x2[q] = L->x[k2][q];
                const double z2 = fma(f, P, N + ek.z);
                const bool big = z2 > 1.0;  // common::norm: len > 1 -> v /= len
                const double y = rsqrt_nr(z2);
                // off the serial path
                A *= f;
                beta_mine = (l == k) ? invA : beta_mine;
                Tm = fma(invA * ek.w, tk, Tm);
                const double Pn = (A * e1.y) * (e1.x + readlane_f(Tm, k1));
                tk = tcoef(x1);
                // serial tail
                f = big ? y : 1.0;
                invA = big ? invA * (z2 * y) : invA;
                N = big ? 1.0 : z2;
                P = Pn;
                ek = e1;
                e1 = e2;
                pin(ek);
                pin(e1);
#pragma unroll
                for (int q = 0; q < NW; ++q) {
                    x1[q] = x2[q];
                    pin(x1[q]);
                }
            }
            A *= f;
#ifdef KB2E_OWNER_PROF
            pc.mark(2);
            pc.count(10, (unsigned long long)cnt);
            pc.count(11, (unsigned long long)cnt);
#endif
            // v = A (v0 + sum_k w_k x_k), w_k = beta_k s_k lr.  Event k's sign
            // word for element parity kv of chunk c is itself the lane mask
            // (bit l <-> lane l) that picks +w_k or -w_k.
            const double w_mine = beta_mine * (double)sg * lr;
            double u[CH][kVec];
#pragma unroll
            for (int c = 0; c < CH; ++c)
#pragma unroll
                for (int k = 0; k < kVec; ++k) u[c][k] = (double)V.v[c][k];
#pragma unroll 1
            for (int k = 0; k < cnt; ++k) {
                const double w = readlane_f(w_mine, k);
                const uint32_t wlo = (uint32_t)__double_as_longlong(w);
                const uint32_t whi = (uint32_t)(__double_as_longlong(w) >> 32);
                const uint32_t whn = whi ^ 0x80000000u;  // -w differs in the sign bit only
#pragma unroll
                for (int c = 0; c < CH; ++c)
#pragma unroll
                    for (int kv = 0; kv < kVec; ++kv) {
                        const uint64_t word = readlane_u64(xw[c * kVec + kv], k);
                        uint32_t hi;
                        asm volatile("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(hi) : "v"(whn), "v"(whi), "s"(word));
                        u[c][kv] += __longlong_as_double(((long long)hi << 32) | wlo);
                    }
            }
#pragma unroll
            for (int c = 0; c < CH; ++c)
#pragma unroll
                for (int k = 0; k < kVec; ++k) V.v[c][k] = elem_valid(c, k, a.n) ? (T)(A * u[c][k]) : T(0);
            wave_lds_sync();
            OWNER_MARK(3);
        } else {
            nld.issue(a, nvalid);
        }
        ev = nld.decode(nvalid, is_rel);
        OWNER_MARK(4);
        OWNER_COUNT(12);
    }
#ifdef KB2E_OWNER_PROF
    pc.flush(g_fold_prof[p1 - p0 >= 512 ? 0 : 1]);
#endif
}

template <typename T, int CH, bool L1>
__global__ __launch_bounds__(256) void transe_fold_kernel(FoldArgs<T> a) {
    __shared__ GramLds<CH> glds[4];  // one per wave (recurrence path)
    const int s0 = a.batch_seg[a.batch], s1 = a.batch_seg[a.batch + 1];
    const int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int nwaves = (gridDim.x * blockDim.x) >> 6;
    const int l = lane_id();
    // Relation rows sort last and carry the longest event chains: start them first.
    for (int s = s1 - 1 - wave; s >= s0; s -= nwaves) {
        const int p0 = a.seg_start[s], p1 = a.seg_start[s + 1];
        if (a.long_min > 0 && p1 - p0 >= a.long_min) continue;  // transe_fold_long_kernel's
        const int row = a.kl.row_of(a.keys[p0]);
        const bool is_rel = row >= a.ne;
        T* ptr = is_rel ? a.rel + (int64_t)(row - a.ne) * a.ld : a.ent + (int64_t)row * a.ld;
        RowReg<T, CH> V;
        V.load(ptr, a.n);
        bool dirty = false;
        if (L1 && a.gram_min > 0 && p1 - p0 >= a.gram_min) {
            fold_segment_gram<T, CH>(a, p0, p1, is_rel, V, &glds[threadIdx.x >> 6], dirty);
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
