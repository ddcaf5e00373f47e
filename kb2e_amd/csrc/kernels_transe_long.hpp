// kernels_transe_long.hpp -- the TransE row fold for long event segments:
// one workgroup of four cooperating waves per row.
//
// The per-row fold (kernels_transe.hpp) replays a row's events in sample
// order.  For the longest rows (the most frequent relations and entities) that
// chain is the critical path of the whole batch, and one wave running it is
// issue-bound: of ~530 cycles per event only ~60% is the serial recurrence
// itself.  Here wave 0 runs nothing but the recurrence (fold_segment_gram's
// chain) while three helper waves prepare the next chunks and materialise the
// previous one, one chunk-phase apart, separated by workgroup barriers:
//
//   phase c   wave 0: pm of chunk c (see below), chain over chunk c
//             wave 1: materialise v_c (the row at the start of chunk c) from
//                     chunk c-1's weights; P0_{c+1} = lr x_m . v_c
//             wave 2: decode chunk c+2 (keys, hinge flags, sign words,
//                     compaction of active events); t-matrix of chunk c+1
//             wave 3: cross t-matrix between chunks c+1 and c; event table
//                     of chunk c+1
//
// with t(k, m) = n - 2 popcount(bits_k ^ bits_m) = x_k . x_m.  The chain needs
// pm_m = lr x_m . v_c for its chunk; since v_c = A_{c-1} (v_{c-1} + sum_k w_k
// x_k) (k over chunk c-1), wave 0 forms it after the barrier as
//   pm_m = A_{c-1} (P0_m + lr sum_k w_k t_c(k, m)),
// a 64-term sum per lane, instead of waiting for the materialisation.  The
// row's squared length is carried by the chain across chunks.
#pragma once

#include "kernels_transe.hpp"

namespace kb2e {

template <int CH>
struct LongLds {
    uint64_t x[4][kWave][2 * CH];  // compacted sign words, chunk c in slot c % 4
    int s[4][kWave];               // compacted signs s_k
    int cnt[4];                    // active events of the chunk
    float tt[2][kWave][kWave];     // tt[c&1][k][m] = t(k, m) within chunk c
    float tc[2][kWave][kWave];     // tc[c&1][k][m] = t(event k of chunk c-1, event m of chunk c)
    double4 ev[2][kWave];          // chain table of chunk c: {pm, 2 s, |e|^2, s lr^2}
    double P0[2][kWave];           // lr x_m . v_{c-1} for chunk c
    double w[2][kWave];            // w_k = beta_k s_k lr of chunk c
    double Asc[2];                 // final scale A of chunk c
    double N0;                     // |v_0|^2
    double v[CH * kWave * kVec];   // materialised row (wave 1)
};

template <typename T, int CH>
__host__ __device__ constexpr size_t fold_long_lds_bytes() {
    return sizeof(LongLds<CH>);
}

// Wave 2: events of chunk ci of segment [p0, p1), compacted into slot ci % 4.
template <typename T, int CH>
__device__ __forceinline__ void long_decode(const FoldArgs<T>& a, LongLds<CH>& L, int p0, int p1, int ci,
                                            bool is_rel) {
    constexpr int NW = 2 * CH;
    const int l = lane_id();
    const int p = p0 + ci * kWave + l;
    const bool valid = p < p1;
    ChunkLoads<T, CH> ld;
    ld.key = valid ? a.keys[p] : 0ull;
    ld.issue(a, valid);
    const ChunkEvents<CH> ev = ld.decode(valid, is_rel);
    const uint64_t m_act = __ballot(ev.nn > 0);
    const int pos = __builtin_amdgcn_mbcnt_hi((uint32_t)(m_act >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m_act, 0u));
    const int slot = ci & 3;
    if (ev.nn > 0) {
#pragma unroll
        for (int q = 0; q < NW; ++q) L.x[slot][pos][q] = ev.xw[q];
        L.s[slot][pos] = ev.sgn;
    }
    if (l == 0) L.cnt[slot] = __popcll(m_act);
}

// t(k, m) for m = this lane against every event k of words `src` (count ck),
// written as dst[k][m]; lanes past `cm` events write zeros.
template <int CH>
__device__ __forceinline__ void long_tmatrix(const uint64_t (*src)[2 * CH], int ck, const uint64_t (&xm)[2 * CH],
                                             int cm, int n, float (*dst)[kWave]) {
    constexpr int NW = 2 * CH;
    const int l = lane_id();
#pragma unroll 4
    for (int k = 0; k < ck; ++k) {
        uint32_t dis = 0;
#pragma unroll
        for (int q = 0; q < NW; ++q) dis += (uint32_t)__popcll(xm[q] ^ src[k][q]);
        dst[k][l] = l < cm ? (float)(n - 2 * (int)dis) : 0.0f;
    }
    if (ck < kWave) dst[ck][l] = 0.0f;  // the padding step of an odd count reads this row
}

// Wave 1: p0[m] = lr x_m . v with v in L.v (four partial sums over the row).
template <int CH>
__device__ __forceinline__ double long_xdotv(const LongLds<CH>& L, const uint64_t (&xw)[2 * CH], int n, double lr) {
    double pq[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int c = 0; c < CH; ++c)
#pragma unroll
        for (int j0 = 0; j0 < kWave; j0 += 8) {
            if (c * (kWave * kVec) + 2 * j0 >= n) continue;  // wave-uniform
#pragma unroll
            for (int j = j0; j < j0 + 8; ++j) {
                const double2 vv = *reinterpret_cast<const double2*>(&L.v[c * (kWave * kVec) + 2 * j]);
                const bool b0 = (xw[c * kVec] >> j) & 1ull, b1 = (xw[c * kVec + 1] >> j) & 1ull;
                pq[(2 * j) & 3] += b0 ? vv.x : -vv.x;
                pq[(2 * j + 1) & 3] += b1 ? vv.y : -vv.y;
            }
        }
    return ((pq[0] + pq[1]) + (pq[2] + pq[3])) * lr;
}

// Wave 1: u = v + sum_k w_k x_k over the cnt events of slot `slot`; the sign
// word of event k is the lane mask that picks +w_k or -w_k.
template <int CH>
__device__ __forceinline__ void long_materialise(const LongLds<CH>& L, int slot, int wb, int cnt,
                                                 double (&u)[CH][kVec]) {
#pragma unroll 1
    for (int k = 0; k < cnt; ++k) {
        const double w = L.w[wb][k];
        const uint32_t wlo = (uint32_t)__double_as_longlong(w);
        const uint32_t whi = (uint32_t)(__double_as_longlong(w) >> 32);
        const uint32_t whn = whi ^ 0x80000000u;
#pragma unroll
        for (int c = 0; c < CH; ++c)
#pragma unroll
            for (int kv = 0; kv < kVec; ++kv) {
                const uint64_t wd = L.x[slot][k][c * kVec + kv];
                const uint64_t word = ((uint64_t)__builtin_amdgcn_readfirstlane((int)(wd >> 32)) << 32) |
                                      (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)wd);
                uint32_t hi;
                asm volatile("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(hi) : "v"(whn), "v"(whi), "s"(word));
                u[c][kv] += __longlong_as_double(((long long)hi << 32) | wlo);
            }
    }
}

template <typename T, int CH>
__global__ __launch_bounds__(256) void transe_fold_long_kernel(FoldArgs<T> a, const int32_t* long_list,
                                                               const int32_t* long_count) {
    constexpr int NW = 2 * CH;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    LongLds<CH>& L = *reinterpret_cast<LongLds<CH>*>(smem);
    const int wv = threadIdx.x >> 6, l = lane_id();
    const double lr = a.lr;
    const double lr2 = lr * lr;
    const double eps = lr2 * (double)a.n;
    const int nlong = *long_count;
    for (int li = blockIdx.x; li < nlong; li += gridDim.x) {
        const int sidx = long_list[li];
        const int p0 = a.seg_start[sidx], p1 = a.seg_start[sidx + 1];
        const int row = a.kl.row_of(a.keys[p0]);
        const bool is_rel = row >= a.ne;
        T* ptr = is_rel ? a.rel + (int64_t)(row - a.ne) * a.ld : a.ent + (int64_t)row * a.ld;
        const int C = (p1 - p0 + kWave - 1) / kWave;
        RowReg<T, CH> V;  // wave 1: the row
        // ---- prologue: chunks 0 and 1 decoded, row loaded, chunk 0's tables
        if (wv == 1) {
            V.load(ptr, a.n);
#pragma unroll
            for (int c = 0; c < CH; ++c)
#pragma unroll
                for (int k = 0; k < kVec; ++k) L.v[c * (kWave * kVec) + l * kVec + k] = (double)V.v[c][k];
            const double n0 = (double)V.sumsq();
            if (l == 0) L.N0 = n0;
        } else if (wv == 2) {
            long_decode<T, CH>(a, L, p0, p1, 0, is_rel);
        } else if (wv == 3 && C > 1) {
            long_decode<T, CH>(a, L, p0, p1, 1, is_rel);
        }
        __syncthreads();
        if (wv >= 1) {
            const int cnt0 = L.cnt[0];
            uint64_t xm[NW];
#pragma unroll
            for (int q = 0; q < NW; ++q) xm[q] = l < cnt0 ? L.x[0][l][q] : 0ull;
            const int sg = l < cnt0 ? L.s[0][l] : 0;
            if (wv == 1) {
                L.ev[0][l].x = long_xdotv<CH>(L, xm, a.n, lr);  // pm of chunk 0: v_0 is the loaded row
            } else if (wv == 2) {
                long_tmatrix<CH>(L.x[0], cnt0, xm, cnt0, a.n, L.tt[0]);
            } else {
                const double sd = (double)sg;
                L.ev[0][l].y = 2.0 * sd;
                L.ev[0][l].z = sg != 0 ? eps : 0.0;
                L.ev[0][l].w = sd * lr2;
            }
        }
        __syncthreads();
        double N = L.N0;  // wave 0: the row's squared length, carried across chunks
#ifdef KB2E_OWNER_PROF
        PhaseClock pc;
        pc.start();
#endif
        for (int c = 0; c < C; ++c) {
            const int b = c & 1, slot = c & 3;
            if (wv == 0) {
                const int cnt = L.cnt[slot];
                if (c > 0) {  // pm of chunk c from P0 and chunk c-1's weights
                    const int cprev = L.cnt[(c - 1) & 3];
                    double acc = 0.0;
#pragma unroll 4
                    for (int k = 0; k < cprev; ++k) acc = fma(L.w[b ^ 1][k], (double)L.tc[b][k][l], acc);
                    L.ev[b][l].x = L.Asc[b ^ 1] * (L.P0[b][l] + lr * acc);
                }
                wave_lds_sync();
                const int sg = l < cnt ? L.s[slot][l] : 0;
                double A = 1.0, invA = 1.0, Tm = 0.0, beta_mine = 0.0, f = 1.0;
                if (cnt > 0) {
                    // Two steps per iteration (cnt rounded up: past the last event
                    // the table holds zeros, and once a step has run the tracked
                    // squared length is <= 1, so padding steps change nothing).
                    // Table entries are read two steps ahead, t-matrix rows one.
                    double4 e0 = L.ev[b][0], e1 = L.ev[b][1];
                    double P = e0.y * e0.x;
                    double t0 = (double)L.tt[b][0][l];
                    auto step = [&](int k, const double4& ek, const double4& en, double tk) {
                        const double z2 = fma(f, P, N + ek.z);
                        const bool big = z2 > 1.0;  // common::norm: len > 1 -> v /= len
                        const double y = rsqrt_nr(z2);
                        A *= f;
                        beta_mine = (l == k) ? invA : beta_mine;
                        Tm = fma(invA * ek.w, tk, Tm);
                        P = (A * en.y) * (en.x + readlane_f(Tm, (k + 1) & (kWave - 1)));
                        f = big ? y : 1.0;
                        invA = big ? invA * (z2 * y) : invA;
                        N = big ? 1.0 : z2;
                    };
#pragma unroll 1
                    for (int k = 0; k < cnt; k += 2) {
                        // k + 3 <= 64 since cnt <= 64 and k is even
                        const double4 e2 = L.ev[b][k + 2 < kWave ? k + 2 : kWave - 1];
                        const double t1 = (double)L.tt[b][k + 1][l];
                        step(k, e0, e1, t0);
                        const double4 e3 = L.ev[b][k + 3 < kWave ? k + 3 : kWave - 1];
                        const double t2 = (double)L.tt[b][k + 2 < kWave ? k + 2 : kWave - 1][l];
                        step(k + 1, e1, e2, t1);
                        e0 = e2;
                        e1 = e3;
                        t0 = t2;
                        pin(e0);
                        pin(e1);
                        pin(t0);
                    }
                    A *= f;
                }
                L.w[b][l] = beta_mine * (double)sg * lr;
                if (l == 0) L.Asc[b] = A;
            } else if (wv == 1) {
                if (c > 0) {  // v_c = A_{c-1} (v_{c-1} + sum_k w_k x_k)
                    double u[CH][kVec];
#pragma unroll
                    for (int cc = 0; cc < CH; ++cc)
#pragma unroll
                        for (int k = 0; k < kVec; ++k) u[cc][k] = (double)V.v[cc][k];
                    long_materialise<CH>(L, (c - 1) & 3, b ^ 1, L.cnt[(c - 1) & 3], u);
                    const double Ap = L.Asc[b ^ 1];
#pragma unroll
                    for (int cc = 0; cc < CH; ++cc)
#pragma unroll
                        for (int k = 0; k < kVec; ++k) {
                            V.v[cc][k] = elem_valid(cc, k, a.n) ? (T)(Ap * u[cc][k]) : T(0);
                            L.v[cc * (kWave * kVec) + l * kVec + k] = (double)V.v[cc][k];
                        }
                    wave_lds_sync();
                }
                if (c + 1 < C) {
                    const int sn = (c + 1) & 3, cn = L.cnt[sn];
                    uint64_t xm[NW];
#pragma unroll
                    for (int q = 0; q < NW; ++q) xm[q] = l < cn ? L.x[sn][l][q] : 0ull;
                    L.P0[b ^ 1][l] = long_xdotv<CH>(L, xm, a.n, lr);
                }
            } else if (wv == 2) {
                if (c + 2 < C) long_decode<T, CH>(a, L, p0, p1, c + 2, is_rel);
                if (c + 1 < C) {
                    const int sn = (c + 1) & 3, cn = L.cnt[sn];
                    uint64_t xm[NW];
#pragma unroll
                    for (int q = 0; q < NW; ++q) xm[q] = l < cn ? L.x[sn][l][q] : 0ull;
                    long_tmatrix<CH>(L.x[sn], cn, xm, cn, a.n, L.tt[b ^ 1]);
                }
            } else {
                if (c + 1 < C) {
                    const int sn = (c + 1) & 3, cn = L.cnt[sn];
                    uint64_t xm[NW];
#pragma unroll
                    for (int q = 0; q < NW; ++q) xm[q] = l < cn ? L.x[sn][l][q] : 0ull;
                    long_tmatrix<CH>(L.x[slot], L.cnt[slot], xm, cn, a.n, L.tc[b ^ 1]);
                    const int sg = l < cn ? L.s[sn][l] : 0;
                    const double sd = (double)sg;
                    L.ev[b ^ 1][l].y = 2.0 * sd;
                    L.ev[b ^ 1][l].z = sg != 0 ? eps : 0.0;
                    L.ev[b ^ 1][l].w = sd * lr2;
                }
            }
#ifdef KB2E_OWNER_PROF
            pc.mark(wv);  // work of this wave's phase
#endif
            __syncthreads();
#ifdef KB2E_OWNER_PROF
            pc.mark(4 + wv);  // waiting at the barrier
            if (wv == 0) pc.count(10, (unsigned long long)L.cnt[c & 3]);
            pc.count(12);
#endif
        }
#ifdef KB2E_OWNER_PROF
        pc.flush(&g_long_prof[0]);
#endif
        // ---- epilogue: the final row
        if (wv == 1) {
            const int cl = (C - 1) & 3, bl = (C - 1) & 1;
            double u[CH][kVec];
#pragma unroll
            for (int cc = 0; cc < CH; ++cc)
#pragma unroll
                for (int k = 0; k < kVec; ++k) u[cc][k] = (double)V.v[cc][k];
            long_materialise<CH>(L, cl, bl, L.cnt[cl], u);
            const double Ap = L.Asc[bl];
#pragma unroll
            for (int cc = 0; cc < CH; ++cc)
#pragma unroll
                for (int k = 0; k < kVec; ++k) V.v[cc][k] = elem_valid(cc, k, a.n) ? (T)(Ap * u[cc][k]) : T(0);
            V.store(ptr, a.n);
        }
        __syncthreads();
    }
}

// The batch's segments of at least `long_min` events (order irrelevant: rows
// are independent).  One workgroup.
__global__ __launch_bounds__(1024) void long_segments_kernel(const int32_t* seg_start, const int32_t* batch_seg,
                                                             int32_t batch, int32_t long_min, int32_t* list,
                                                             int32_t* count) {
    __shared__ int n;
    if (threadIdx.x == 0) n = 0;
    __syncthreads();
    const int s0 = batch_seg[batch], s1 = batch_seg[batch + 1];
    for (int s = s0 + threadIdx.x; s < s1; s += blockDim.x)
        if (seg_start[s + 1] - seg_start[s] >= long_min) list[atomicAdd(&n, 1)] = s;
    __syncthreads();
    if (threadIdx.x == 0) *count = n;
}

}  // namespace kb2e
