// kernels_transr_cons.hpp -- transRNorm of the PARALLEL TransR schedule
// (transr/trainer.cpp:35-64, model: oracle/parallel.py transr_constraint) with
// each 16-row block of pairs iterated by ONE wave, without workgroup barriers.
//
// Same pairs and rules as transr_cons_tile_kernel (kernels_transr_mfma.hpp):
// per tile, the (h', r), (t', r) pairs of its active updates and (entity'[r], r)
// on the relation's first tile, first occurrences per relation per batch only
// (transr_pair_dup); with W0 = W'_r,
// K = W0^T W0 and p = W0^T a0, while |p|^2 > 1:  G += 2 p,
// p <- p - 2 lr K p - 2 lr |a0|^2 p, a row freezing at its own first
// non-violation; then da = -lr W0 G (pair records) and dW = -lr a0 G^T (matrix
// partials).  What changes is where the rounds live:
//   * products are taken transposed, the pair rows as the MFMA's N dimension,
//     so a row block's p sits in B-operand fragments and the D fragment of
//     output block ib, register r IS the B fragment of k-step 4 ib + r (kmap):
//     a block with many moving rows iterates as one MFMA chain (Q^T = K P^T)
//     in one wave's registers, no LDS round trip, no barrier;
//   * once at most kValuRows rows of a block still move (almost always from
//     the start: a typical block has one or two violators), the rounds run on
//     the VALU, lane i holding element i of each row's p and G: q_i = K[i] . p
//     with row i of K read contiguously and p as LDS broadcasts, every load of
//     a chunk in flight before its FMAs (an MFMA round costs the same for 1 or
//     16 moving rows; measured on gfx950: ~1.2k cycles a VALU round for one
//     row against ~3.3k for an MFMA round, tools/diag/cons_round.hip);
//   * the tile's matrix partial -lr A0^T G is one more MFMA product, its rows
//     (a0 re-read from L2, G from the fragments) staged through the W0 / K
//     image once every wave's rounds are done (a workgroup lives as long as
//     its slowest wave anyway).
// The workgroup synchronises after staging W0 and the pairs, after the check
// (K = W0^T W0 is computed by all four waves only when the tile has a
// violator), after K, and around the partial's staging.  |p|^2 is summed over a lane's k-steps and then over the four
// lanes that share a row (lanes l, l ^ 16, l ^ 32, l ^ 48: two permlane
// swaps), so all four see the same bits; on the VALU it is a wave_sum.
#pragma once

#include <type_traits>

#include "kernels_transr_mfma.hpp"
#include "transr_cons.hpp"

namespace kb2e {

// The k index lane group kq = l >> 4 carries in k-step s of a register-resident
// B operand (P^T, T^T, G^T, A0^T): chosen so that D of output block ib,
// register r IS k-step 4 ib + r.  FP64 D rows are (l >> 4) + 4 r, FP32 ones 4 (l >> 4) + r.
template <typename T>
__device__ __forceinline__ constexpr int kmap(int s, int kq) {
    if constexpr (sizeof(T) == 8) return 4 * s + kq;
    else return (s >> 2) * 16 + 4 * kq + (s & 3);
}

// x + x[l ^ 16] (FP addition commutes: both lanes of a pair get the same bits)
__device__ __forceinline__ float pair_sum16(float v) {
    const uint32_t b = __float_as_uint(v);
    const auto r = __builtin_amdgcn_permlane16_swap(b, b, false, false);
    return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ __forceinline__ double pair_sum16(double v) {
    const uint64_t b = (uint64_t)__double_as_longlong(v);
    const auto lo = __builtin_amdgcn_permlane16_swap((uint32_t)b, (uint32_t)b, false, false);
    const auto hi = __builtin_amdgcn_permlane16_swap((uint32_t)(b >> 32), (uint32_t)(b >> 32), false, false);
    return __longlong_as_double((long long)(((uint64_t)hi[0] << 32) | lo[0])) +
           __longlong_as_double((long long)(((uint64_t)hi[1] << 32) | lo[1]));
}
__device__ __forceinline__ float pair_sum32(float v) {
    const uint32_t b = __float_as_uint(v);
    const auto r = __builtin_amdgcn_permlane32_swap(b, b, false, false);
    return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ __forceinline__ double pair_sum32(double v) {
    const uint64_t b = (uint64_t)__double_as_longlong(v);
    const auto lo = __builtin_amdgcn_permlane32_swap((uint32_t)b, (uint32_t)b, false, false);
    const auto hi = __builtin_amdgcn_permlane32_swap((uint32_t)(b >> 32), (uint32_t)(b >> 32), false, false);
    return __longlong_as_double((long long)(((uint64_t)hi[0] << 32) | lo[0])) +
           __longlong_as_double((long long)(((uint64_t)hi[1] << 32) | lo[1]));
}
// sum over the four lanes of one pair row (identical bits in all four)
template <typename T>
__device__ __forceinline__ T row4_sum(T v) {
    return pair_sum32(pair_sum16(v));
}

constexpr int kConsWaves = 4;  // PP / 16 <= 4 row blocks (4 St + 1 <= 64)
constexpr int kValuRows = 4;   // a block with this few moving rows iterates on the VALU

// LDS (bytes): W0 [NP][NP + 2] | K [NP][NP + 2] | per wave SP [kValuRows][NP] | int misc [8]
// (75 KB at n = 50 in FP64: two workgroups per CU)
template <typename T>
__host__ __device__ constexpr size_t rcons_lds(int n, int St) {
    return sizeof(T) * (2 * (size_t)rm_np(n) * rm_ld(n) + (size_t)kConsWaves * kValuRows * rm_np(n)) +
           sizeof(int) * 8 + 0 * (size_t)St;
}

// k-steps (of kmap) that hold a column below n: a prefix 0 .. KS - 1 of the
// 4 ceil(n / 16) steps, for both layouts
template <typename T>
__host__ __device__ constexpr int cons_live_steps(int n) {
    const int nb = (n + 15) / 16, tail = n - 16 * (nb - 1);
    return 4 * (nb - 1) + (sizeof(T) == 8 ? (tail + 3) / 4 : (tail < 4 ? tail : 4));
}

// The rest of a block's rounds once at most R of its rows still move (rows rr,
// their 2 lr |a0|^2 in c2): their p from the fragments into SP, then rounds
// with lane i holding p_i and this phase's G_i (q_i = K[i] . p over KN
// columns, chunks of CH with every load in flight before the FMAs);
// afterwards that G is added to the rows' fragments gs.  Returns the rounds run.
template <typename T, int R, int NP, int L, int KN>
__device__ __forceinline__ int cons_valu_rounds(const T* KX, T* SP, T lr, const int (&rr)[kValuRows],
                                                const T (&c2)[kValuRows], const T (&ps)[NP / 4], T (&gs)[NP / 4],
                                                int m) {
    constexpr int CH = R == 1 ? 16 : R == 2 ? 8 : 4;  // about 16 loads in flight a chunk
    const int l = lane_id(), kq = l >> 4, l16 = l & 15;
    const bool mine = l < NP;  // lane l < NP holds element l (zeros past n)
    const T* Ki = KX + (mine ? l : 0) * L;  // row i of K = column i (symmetric)
#pragma unroll
    for (int j = 0; j < R; ++j)
        if (l16 == rr[j])
#pragma unroll
            for (int s = 0; s < NP / 4; ++s) SP[j * NP + kmap<T>(s, kq)] = ps[s];
    wave_lds_sync();
    T pv[R], g2[R];
    bool lj[R];
#pragma unroll
    for (int j = 0; j < R; ++j) {
        pv[j] = mine ? SP[j * NP + l] : T(0);
        g2[j] = T(0);
        lj[j] = true;
    }
    int rounds = 0;
    for (; m < kRParMaxIter; ++m) {
        bool any = false;
#pragma unroll
        for (int j = 0; j < R; ++j) any |= lj[j];
        if (!any) break;
        ++rounds;
#pragma unroll
        for (int j = 0; j < R; ++j)
            if (lj[j]) g2[j] += T(2) * pv[j];
        T acc[R][4];
#pragma unroll
        for (int j = 0; j < R; ++j) acc[j][0] = acc[j][1] = acc[j][2] = acc[j][3] = T(0);
        // C columns from k0: every load issued (pinned) before the chunk's FMAs
        auto chunk = [&](int k0, auto cw) {
            constexpr int C = decltype(cw)::value;
            T kk[C], pk[R][C];
#pragma unroll
            for (int k = 0; k < C; ++k) {
                kk[k] = Ki[k0 + k];
#pragma unroll
                for (int j = 0; j < R; ++j) pk[j][k] = SP[j * NP + k0 + k];
            }
#pragma unroll
            for (int k = 0; k < C; ++k) {
                pin(kk[k]);
#pragma unroll
                for (int j = 0; j < R; ++j) pin(pk[j][k]);
            }
#pragma unroll
            for (int k = 0; k < C; ++k)
#pragma unroll
                for (int j = 0; j < R; ++j) acc[j][k & 3] = fma(kk[k], pk[j][k], acc[j][k & 3]);
        };
        int k0 = 0;
#pragma unroll 1
        for (; k0 + CH <= KN; k0 += CH) chunk(k0, std::integral_constant<int, CH>());  // one chunk's registers at a time
        if constexpr (KN % CH != 0) chunk(k0, std::integral_constant<int, KN % CH>());
        T nr[R];
#pragma unroll
        for (int j = 0; j < R; ++j) {
            const T q = (acc[j][0] + acc[j][1]) + (acc[j][2] + acc[j][3]);
            if (lj[j] && mine) pv[j] = pv[j] - T(2) * lr * q - c2[j] * pv[j];
            nr[j] = wave_sum(pv[j] * pv[j]);
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // every lane's reads of SP are done
#pragma unroll
        for (int j = 0; j < R; ++j) {
            lj[j] = lj[j] && nr[j] > T(1);
            if (mine) SP[j * NP + l] = pv[j];
        }
        wave_lds_sync();
    }
#pragma unroll
    for (int j = 0; j < R; ++j)
        if (mine) SP[j * NP + l] = g2[j];
    wave_lds_sync();
#pragma unroll
    for (int j = 0; j < R; ++j)
        if (l16 == rr[j])
#pragma unroll
            for (int s = 0; s < NP / 4; ++s) gs[s] += SP[j * NP + kmap<T>(s, kq)];
    wave_lds_sync();
    return rounds;
}

// round statistics (KB2E_RPAR_STATS), the layout of g_rpar_rounds
static __device__ unsigned long long g_cons_stats[16];

// KS: the live k-steps, a compile-time constant (NB = ceil(KS / 4) column
// blocks): every MFMA loop is straight-line code without per-step guards.
template <typename T, int KS>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) void transr_cons_wave_kernel(RParArgs a, RParBufs<T> bf) {
    using M = Mfma16<T>;
    constexpr int NB = (KS + 3) / 4, NP = 16 * NB, L = NP + 2, NS = NP / 4;
    // the VALU rounds' contraction length: natural k below n (FP64: 4 KS; FP32 up to NP)
    constexpr int KN = sizeof(T) == 8 ? 4 * KS : NP;
    constexpr int kOut = (NB * NB + kConsWaves - 1) / kConsWaves;  // K output tiles per wave
    extern __shared__ __attribute__((aligned(16))) char smem[];
    // the tile's pair count and relation from the gradient kernel (one load before
    // the W0 staging), read beside the batch's tile range
    const int cn = bf.cnrows[blockIdx.x];
    if ((int)blockIdx.x >= a.batch_t0[a.batch + 1] - a.batch_t0[a.batch]) return;
    const int r = cn >> 8;
    // the relation's only tile: its matrix partial goes straight into W'_r (the row
    // pass would add this one partial to the same values), no partial round trip
    const bool single = (cn >> 7) & 1;
    const int n = a.n, ld = a.ld;
    const int w = threadIdx.x >> 6, l = lane_id(), kq = l >> 4, l16 = l & 15;
    T* Wl = (T*)smem;
    T* KX = Wl + NP * L;
    T* SP = KX + NP * L + w * kValuRows * NP;  // this wave's VALU rounds: p rows
    int* misc = (int*)(KX + NP * L + kConsWaves * kValuRows * NP);  // [1] the tile has a violator, [2 + b] block b has one
    const unsigned long long ck0 = bf.stats ? clock64() : 0ull;
    const T lr = (T)a.lr;
    // this wave's pair rows (compacted by transr_grad_wave_kernel) and their a0 rows as
    // B fragments (not kept: the matrix partial re-reads them), loads issued before the barrier
    const int nrows = cn & 127;
    const int nblk = (nrows + 15) >> 4;
    const bool mine = w < nblk;  // this wave owns pair rows [16 w, 16 w + 16)
    const int32_t* cp = bf.cpairs + (int64_t)blockIdx.x * 2 * kCPairs;
    const int row = w * 16 + l16;
    const int e = row < nrows ? cp[row] : -1;
    const int sl = row < nrows ? cp[kCPairs + row] : -1;
    T af[KS];
    {
        const T* ar = bf.ent + (int64_t)(e < 0 ? 0 : e) * ld;
#pragma unroll
        for (int s = 0; s < KS; ++s) {  // unconditional loads (in-row index), masked by a
            const int k = kmap<T>(s, kq);  // product: a select lets the compiler branch around each load
            af[s] = ar[k < n ? k : 0] * ((e >= 0 && k < n) ? T(1) : T(0));
        }
    }
    if (w == 0) {
        if (l < 8) misc[l] = 0;
    } else {
        // W0 as element pairs (ld is even and the row padding is zero), every
        // load of the thread in flight before the first LDS store
        using T2 = typename std::conditional<sizeof(T) == 8, double2, float2>::type;
        constexpr int kPairs = NP * L / 2, kThreads = (kConsWaves - 1) * kWave;
        constexpr int kPer = (kPairs + kThreads - 1) / kThreads;
        const T2* Wg = (const T2*)(bf.W + (int64_t)r * n * ld);
        const int hp = ld / 2;  // pairs of a row in HBM
        T2 v[kPer];
#pragma unroll
        for (int q = 0; q < kPer; ++q) {
            const int idx = threadIdx.x - kWave + q * kThreads;
            const int j = idx / (L / 2), ip = idx % (L / 2);
            const bool ok = idx < kPairs && j < n && ip < hp;
            const T2 g = Wg[ok ? j * hp + ip : 0];
            v[q] = ok ? g : T2{T(0), T(0)};
        }
#pragma unroll
        for (int q = 0; q < kPer; ++q) {
            const int idx = threadIdx.x - kWave + q * kThreads;
            if (idx < kPairs) ((T2*)Wl)[idx] = v[q];
        }
    }
    __syncthreads();  // W0 in place
    const unsigned long long ck1 = bf.stats ? clock64() : 0ull;
    T ps[NS], gs[NS];
#pragma unroll
    for (int s = 0; s < NS; ++s) ps[s] = gs[s] = T(0);
    T c2 = T(0);
    bool lv = false;
    uint32_t vm16 = 0;
    if (mine) {
        // |a0|^2, then P0^T = W0^T A0^T and the check
        T ss = T(0);
#pragma unroll
        for (int s = 0; s < KS; ++s) ss += af[s] * af[s];
        c2 = T(2) * lr * row4_sum(ss);
#pragma unroll
        for (int ib = 0; ib < NB; ++ib) {
            typename M::acc_t acc = {T(0), T(0), T(0), T(0)};
#pragma unroll
            for (int s = 0; s < KS; ++s) acc = M::mma(Wl[kmap<T>(s, kq) * L + ib * 16 + l16], af[s], acc);
#pragma unroll
            for (int q = 0; q < 4; ++q) ps[4 * ib + q] = acc[q];
        }
        T nr0 = T(0);
#pragma unroll
        for (int s = 0; s < KS; ++s) nr0 += ps[s] * ps[s];
        lv = row < nrows && row4_sum(nr0) > T(1);
        if (kq == 0 && sl >= 0) bf.pflag[sl] = lv ? 1 : 0;
        vm16 = (uint32_t)__ballot(lv) & 0xFFFFu;  // lanes 0-15: one per row
        if (vm16 && l == 0) {
            misc[1] = 1;
            misc[2 + w] = 1;
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) bf.cons_tile[blockIdx.x] = misc[1] && !single;
    if (!misc[1]) {  // no violator in the tile
        if (bf.stats && threadIdx.x == 0) {
            atomicAdd(&g_cons_stats[3], ck1 - ck0);
            atomicAdd(&g_cons_stats[4], clock64() - ck1);
            atomicAdd(&g_cons_stats[7], 1ull);
        }
        return;
    }
    // K = W0^T W0 (symmetric, zero past n) by all four waves, over the live k-steps
#pragma unroll
    for (int q = 0; q < kOut; ++q) {
        if (bf.dbg & 1) break;
        const int tile = w + kConsWaves * q;
        if (tile >= NB * NB) break;
        const int mb = tile / NB, cb = tile % NB;
        typename M::acc_t acc = {T(0), T(0), T(0), T(0)};
#pragma unroll
        for (int s = 0; s < KS; ++s) {
            const int k = kmap<T>(s, kq);
            acc = M::mma(Wl[k * L + mb * 16 + l16], Wl[k * L + cb * 16 + l16], acc);
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) KX[(mb * 16 + M::row(l, k)) * L + cb * 16 + l16] = acc[k];
    }
    __syncthreads();
    const bool vio0 = lv;
    int rounds = 0;
    const unsigned long long ck2r = bf.stats ? clock64() : 0ull;
    if (vm16) {
    // the rounds, on the matrix cores while more than kValuRows rows move
    for (int m = (bf.dbg & 2) ? kRParMaxIter : 0; m < kRParMaxIter; ++m) {
        const uint32_t live16 = (uint32_t)__ballot(lv) & 0xFFFFu;
        if (!live16) break;
        const int nl = __builtin_popcount(live16);
        if (nl <= kValuRows) {
            int rr[kValuRows];
            T cj[kValuRows];
            uint32_t mm = live16;
#pragma unroll
            for (int j = 0; j < kValuRows; ++j) {
                rr[j] = mm ? __builtin_ctz(mm) : 0;
                mm &= mm - 1;
                cj[j] = readlane_f(c2, rr[j]);
            }
            if (bf.stats && l == 0) {
                atomicAdd(&g_cons_stats[12], (unsigned long long)rounds);
                atomicAdd(&g_cons_stats[13], 1ull);
            }
            if (nl == 1) rounds += cons_valu_rounds<T, 1, NP, L, KN>(KX, SP, lr, rr, cj, ps, gs, m);
            else if (nl == 2) rounds += cons_valu_rounds<T, 2, NP, L, KN>(KX, SP, lr, rr, cj, ps, gs, m);
            else if (nl == 3) rounds += cons_valu_rounds<T, 3, NP, L, KN>(KX, SP, lr, rr, cj, ps, gs, m);
            else rounds += cons_valu_rounds<T, 4, NP, L, KN>(KX, SP, lr, rr, cj, ps, gs, m);
            break;
        }
        ++rounds;
#pragma unroll
        for (int s = 0; s < NS; ++s)
            if (lv) gs[s] += T(2) * ps[s];
        typename M::acc_t q[NB];
#pragma unroll
        for (int ib = 0; ib < NB; ++ib) q[ib] = typename M::acc_t{T(0), T(0), T(0), T(0)};
#pragma unroll
        for (int s = 0; s < KS; ++s) {
#pragma unroll
            for (int ib = 0; ib < NB; ++ib) q[ib] = M::mma(KX[(ib * 16 + l16) * L + kmap<T>(s, kq)], ps[s], q[ib]);
        }
        T nr = T(0);
#pragma unroll
        for (int ib = 0; ib < NB; ++ib)
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int s = 4 * ib + k;
                if (lv) ps[s] = ps[s] - T(2) * lr * q[ib][k] - c2 * ps[s];
                nr += ps[s] * ps[s];
            }
        lv = lv && row4_sum(nr) > T(1);
    }
    // pair records da = -lr W0 G
    const uint32_t v16 = (uint32_t)__ballot(vio0) & 0xFFFFu;
    const bool valu_rec = __builtin_popcount(v16) <= kValuRows;
    if (valu_rec && !(bf.dbg & 4)) {
        // few violating rows (the usual case): on the VALU, one row at a time, lane j
        // element j: da_j = W0[j] . G, G through this wave's SP rows
        int rv[kValuRows];
        uint32_t mm = v16;
#pragma unroll
        for (int j = 0; j < kValuRows; ++j) {
            rv[j] = mm ? (int)__builtin_ctz(mm) : -1;
            mm &= mm - 1;
        }
#pragma unroll
        for (int j = 0; j < kValuRows; ++j)
            if (l16 == rv[j])
#pragma unroll
                for (int s = 0; s < NS; ++s) SP[j * NP + kmap<T>(s, kq)] = gs[s];
        wave_lds_sync();
        const T* Wj = Wl + (l < n ? l : 0) * L;
#pragma unroll 1
        for (int j = 0; j < kValuRows; ++j) {
            if (rv[j] < 0) break;
            const int slj = readlane_i32(sl, rv[j]);
            T acc[4] = {T(0), T(0), T(0), T(0)};
#pragma unroll
            for (int k = 0; k < KN; ++k) acc[k & 3] = fma(Wj[k], SP[j * NP + k], acc[k & 3]);
            T* dj = slj >= 0 ? bf.pair + (int64_t)slj * ld : bf.relpair + (int64_t)r * ld;
            if (l < n) dj[l] = -lr * ((acc[0] + acc[1]) + (acc[2] + acc[3]));
            if (slj == -2 && l == 0) bf.relpair_stamp[r] = bf.stamp;
        }
        wave_lds_sync();
    }
    // (da^T = W0 G^T, G^T the B operand)
    T* dst = sl >= 0 ? bf.pair + (int64_t)sl * ld : bf.relpair + (int64_t)r * ld;
#pragma unroll
    for (int jb = 0; jb < NB; ++jb) {
        if ((bf.dbg & 4) || valu_rec) break;
        typename M::acc_t acc = {T(0), T(0), T(0), T(0)};
#pragma unroll
        for (int s = 0; s < KS; ++s) acc = M::mma(Wl[(jb * 16 + l16) * L + kmap<T>(s, kq)], gs[s], acc);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int j = jb * 16 + M::row(l, q);
            if (vio0 && j < n) dst[j] = -lr * acc[q];
        }
    }
    if (vio0 && sl == -2 && !valu_rec) bf.relpair_stamp[r] = bf.stamp;
    }  // vm16
    const unsigned long long ck2 = bf.stats ? clock64() : ck2r;
    // the tile's matrix partial dW[j][i] = sum_p (-lr a0[p][j]) G[p][i]: the
    // (a0, G) rows of NB row blocks at a time (32 rows each) through the image
    // (W0 and K: 2 NP rows), free once every wave's rounds and records are done
    typename M::acc_t dw[kOut];
#pragma unroll
    for (int q = 0; q < kOut; ++q) dw[q] = typename M::acc_t{T(0), T(0), T(0), T(0)};
    // the relation's only tile: this lane's W'_r elements from the W0 image (= W'_r:
    // nothing else writes the relation), read before the image is reused below
    T wold[kOut][4];
#pragma unroll
    for (int q = 0; q < kOut; ++q) {
        const int tile = w + kConsWaves * q;
        const int jb = tile / NB, ib = tile % NB;
#pragma unroll
        for (int k = 0; k < 4; ++k)
            wold[q][k] = (single && tile < NB * NB) ? Wl[(jb * 16 + M::row(l, k)) * L + ib * 16 + l16] : T(0);
    }
    T* const CX = Wl;
    for (int c0 = 0; c0 < nblk; c0 += NB) {
        __syncthreads();  // the W0 / K reads (c0 = 0) or the previous chunks' reads are done
        if (vm16 && w >= c0 && w < c0 + NB) {
            T* A0c = CX + 32 * (w - c0) * L;
            T* Gc = A0c + 16 * L;
#pragma unroll
            for (int s = 0; s < NS; ++s) Gc[l16 * L + kmap<T>(s, kq)] = gs[s];
            // the block's a0 rows again, row-wise (coalesced, L2), all loads in flight
            T a0v[16];
#pragma unroll
            for (int q = 0; q < 16; ++q) {
                const int rq = w * 16 + q;
                const int eq = rq < nrows ? readlane_i32(e, q) : 0;  // lane q holds row 16 w + q
                a0v[q] = bf.ent[(int64_t)eq * ld + (l < n ? l : 0)] * ((rq < nrows && l < n) ? T(1) : T(0));
            }
            if (l < NP)
#pragma unroll
                for (int q = 0; q < 16; ++q) A0c[q * L + l] = a0v[q];
        }
        __syncthreads();
#pragma unroll
        for (int q = 0; q < kOut; ++q) {
            const int tile = w + kConsWaves * q;
            if (tile >= NB * NB) break;
            const int jb = tile / NB, ib = tile % NB;
            for (int b = c0; b < c0 + NB && b < nblk; ++b) {
                if (!misc[2 + b] || (bf.dbg & 8)) continue;
                const T* A0c = CX + 32 * (b - c0) * L;
                const T* Gc = A0c + 16 * L;
#pragma unroll
                for (int s = 0; s < 4; ++s) {
                    const int p = 4 * s + kq;
                    dw[q] = M::mma(A0c[p * L + jb * 16 + l16], Gc[p * L + ib * 16 + l16], dw[q]);
                }
            }
        }
    }
    T* const wp = single ? bf.W + (int64_t)r * n * ld : bf.wpart + (int64_t)blockIdx.x * n * ld;
#pragma unroll
    for (int q = 0; q < kOut; ++q) {
        const int tile = w + kConsWaves * q;
        if (tile >= NB * NB) break;
        const int jb = tile / NB, ib = tile % NB;
        const int i = ib * 16 + l16;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int j = jb * 16 + M::row(l, k);
            if (j < n && i < n) wp[(int64_t)j * ld + i] = single ? wold[q][k] + -lr * dw[q][k] : -lr * dw[q][k];
        }
    }
    if (bf.stats && l == 0 && vm16) {
        const unsigned long long ck3 = clock64();
        atomicAdd(&g_cons_stats[0], (unsigned long long)rounds);
        atomicMax(&g_cons_stats[2], (unsigned long long)rounds);
        atomicAdd(&g_cons_stats[1], 1ull);
        atomicAdd(&g_cons_stats[3], ck1 - ck0);
        atomicAdd(&g_cons_stats[4], ck2 - ck1);
        atomicAdd(&g_cons_stats[5], ck3 - ck2);
        atomicMax(&g_cons_stats[6], ck3 - ck0);
        atomicAdd(&g_cons_stats[7], 1ull);
        atomicMax(&g_cons_stats[8], ck1 - ck0);
        atomicMax(&g_cons_stats[9], ck2 - ck1);
        atomicMax(&g_cons_stats[10], ck3 - ck2);
    }
}

}  // namespace kb2e
