// kernels_transr_mfma.hpp -- the PARALLEL TransR tile and transRNorm kernels on
// the matrix cores (v_mfma_f64_16x16x4_f64 / v_mfma_f32_16x16x4_f32).
//
// Same arithmetic contract as kernels_transr_parallel.hpp (whose VALU kernels
// remain the path when the LDS image below does not fit), recast as the dense
// contractions they are:
//   projections   P = V W          V: the tile's h, t, h', t' rows   (4 St x n) . (n x n)
//   directions    Y = X W^T        X: the updates' x rows            (2 St x n) . (n x n)
//   matrix step   dW = D^T X       D: -lr beta (h - t) rows          (n x 2 St) . (2 St x n)
//   transRNorm    Pm = A W, A -= lr (2 Pm) W^T, dW = (-lr A0)^T G  per Jacobi round over the tile's pairs
// Matrices live in LDS padded to NP = 16 ceil(n / 16) columns (zeros), row
// stride L = NP + 2 (bank spread).  MFMA fragment maps (cdna_hip_programming.md
// "Fragment layout"): A[i = l & 15][k = l >> 4], B[k = l >> 4][j = l & 15];
// D col = l & 15, row = (l >> 4) + 4 r for f64 and 4 (l >> 4) + r for f32.
#pragma once

#include "kernels_transr_parallel.hpp"

namespace kb2e {

template <typename T>
struct Mfma16;

template <>
struct Mfma16<double> {
    typedef double acc_t __attribute__((ext_vector_type(4)));
    static __device__ __forceinline__ acc_t mma(double a, double b, acc_t c) {
        return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
    }
    static __device__ __forceinline__ int row(int l, int r) { return (l >> 4) + 4 * r; }
};

template <>
struct Mfma16<float> {
    typedef float acc_t __attribute__((ext_vector_type(4)));
    static __device__ __forceinline__ acc_t mma(float a, float b, acc_t c) {
        return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
    }
    static __device__ __forceinline__ int row(int l, int r) { return 4 * (l >> 4) + r; }
};

// C = A B over 16 x 16 output tiles (MT x NT of them) and K (multiple of 4; rm_k4(n)
// for a contraction over the n columns of an NP-padded image),
// tiles dealt to the waves of the block; put(m, n, v) receives every element.
// The fragments of eight k-steps are read from LDS before their MFMAs issue,
// so the LDS latency is paid once per eight steps, not once per step.
template <typename T, class FA, class FB, class FP>
__device__ __forceinline__ void block_gemm(int MT, int NT, int K, FA A, FB B, FP put) {
    using M = Mfma16<T>;
    const int l = lane_id(), w = threadIdx.x >> 6, nw = blockDim.x >> 6;
    for (int idx = w; idx < MT * NT; idx += nw) {
        const int mb = idx / NT, nb = idx % NT;
        typename M::acc_t acc = {T(0), T(0), T(0), T(0)};
        const int ar = mb * 16 + (l & 15), bc = nb * 16 + (l & 15), kq = l >> 4;
        for (int kb = 0; kb < K; kb += 32) {
            T av[8], bv[8];
#pragma unroll
            for (int s = 0; s < 8; ++s) {
                const int k = kb + 4 * s + kq;
                const bool ok = kb + 4 * s < K;  // past K: zero operands add nothing
                av[s] = ok ? A(ar, k) : T(0);
                bv[s] = ok ? B(k, bc) : T(0);
            }
#pragma unroll
            for (int s = 0; s < 8; ++s)
                if (kb + 4 * s < K) acc = M::mma(av[s], bv[s], acc);  // no MFMA on the zero padding
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) put(mb * 16 + M::row(l, r), bc, acc[r]);
    }
}

// block_gemm over a K whose bound KP is a compile-time multiple of 16 (the NP
// padding of an image): loads without runtime guards, MFMAs only below K4.
// (D: the k-steps whose fragments are loaded ahead of their MFMAs)
template <typename T, int KP, class FA, class FB, class FP, int D = 8>
__device__ __forceinline__ void block_gemm_k(int MT, int NT, int K4, FA A, FB B, FP put) {
    using M = Mfma16<T>;
    const int l = lane_id(), w = threadIdx.x >> 6, nw = blockDim.x >> 6;
    for (int idx = w; idx < MT * NT; idx += nw) {
        const int mb = idx / NT, nb = idx % NT;
        typename M::acc_t acc = {T(0), T(0), T(0), T(0)};
        const int ar = mb * 16 + (l & 15), bc = nb * 16 + (l & 15), kq = l >> 4;
#pragma unroll
        for (int kb = 0; kb < KP; kb += 4 * D) {
            T av[D], bv[D];
#pragma unroll
            for (int s = 0; s < D; ++s) {
                const int k = kb + 4 * s + kq;
                const bool ok = kb + 4 * s < KP;  // compile time
                av[s] = ok ? A(ar, k) : T(0);
                bv[s] = ok ? B(k, bc) : T(0);
            }
#pragma unroll
            for (int s = 0; s < D; ++s)
                if (kb + 4 * s < K4) acc = M::mma(av[s], bv[s], acc);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) put(mb * 16 + M::row(l, r), bc, acc[r]);
    }
}

__host__ __device__ constexpr int rm_np(int n) { return (n + 15) & ~15; }
__host__ __device__ constexpr int rm_ld(int n) { return rm_np(n) + 2; }
__host__ __device__ constexpr int rm_up16(int v) { return (v + 15) & ~15; }
__host__ __device__ constexpr int rm_k4(int n) { return (n + 3) & ~3; }

constexpr int kTileGroupMax = 8;  // tiles a gradient block runs at most (KB2E_RPAR_TGROUP is capped here)

// Tile kernel LDS (elements of T): V [MV][L] | P [MV][L] (PROJ) | X [UY][L] | D [UY][L] |
// coef [UY] (GRAD) | int ids [MV], kk [kTileGroupMax St].  A projection-only launch needs no D, a
// gradient-only one (compat) neither V nor P.  W_r is not staged: the MFMA B
// fragments come from global memory (L2; a tile group reads the same matrix), so
// the image is small enough for two or more workgroups a CU to overlap their
// gathers and HBM latencies (K5: one 160 KiB workgroup a CU spent the phase waiting).
template <typename T>
__host__ __device__ constexpr size_t rmfma_tile_lds(int n, int St, bool proj = true, bool grad = true) {
    return sizeof(T) * ((proj ? 2 * (size_t)rm_up16(4 * St) * rm_ld(n) : 0) +
                        (grad ? 2 : 1) * (size_t)rm_up16(2 * St) * rm_ld(n) + rm_up16(2 * St)) +
           sizeof(int) * ((size_t)rm_up16(4 * St) + kTileGroupMax * (size_t)St);
}

// transRNorm kernel LDS: W [NP][L] | K [NP][L] | A0 [PP][L] | PG, PG2 [PP + 1][L] | s0 [PP + 2] |
// int ent_of, slot_of, rowmap, posmap, vio [PP] | 8 | npart [2][PP][NP / 16] | int vrow [PP]
template <typename T>
__host__ __device__ constexpr size_t rmfma_cons_lds(int n, int St) {
    return sizeof(T) * (2 * (size_t)rm_np(n) * rm_ld(n) + (3 * (size_t)rm_up16(4 * St + 1) + 2) * rm_ld(n) + 2 +
                        (1 + 2 * (rm_np(n) / 16)) * (size_t)rm_up16(4 * St + 1)) +
           sizeof(int) * (6 * (size_t)rm_up16(4 * St + 1) + 8);
}

// NP: the padded width rm_np(n), a compile-time constant at the call sites
// (index arithmetic by constants, not runtime integer division)
template <typename T, int NP>
__device__ __forceinline__ void stage_matrix_padded(T* Wl, const T* Wg, int n, int ld) {
    constexpr int L = NP + 2;
#pragma unroll 8
    for (int idx = threadIdx.x; idx < NP * L; idx += blockDim.x) {
        const int j = idx / L, i = idx % L;
        Wl[idx] = (j < n && i < n) ? Wg[(int64_t)j * ld + i] : T(0);
    }
}

// rows[row][0..L) = table row ids[row] (zeros past n, or for ids < 0), every
// thread of the block issuing independent loads (no per-row dependent chains).
template <typename T, int NP>
__device__ __forceinline__ void gather_rows(T* rows, const int* ids, int nrows, const T* table, int n, int ld) {
    constexpr int L = NP + 2;
#pragma unroll 8
    for (int idx = threadIdx.x; idx < nrows * L; idx += blockDim.x) {
        const int row = idx / L, i = idx % L;
        const int e = ids[row];
        rows[idx] = (e >= 0 && i < n) ? table[(int64_t)e * ld + i] : T(0);
    }
}

// y_j = sum_i W[j][i] x_i from the transposed image (lane l: j = 2l, 2l+1; LDS
// reads contiguous across lanes, x as broadcasts).
template <typename T>
__device__ __forceinline__ void matvec_t(const T* WT, int L, int n, const T* xl, T (&y)[2]) {
    const int j = 2 * lane_id();
    y[0] = y[1] = T(0);
    if (j >= n) return;
    T s[4][2] = {};  // four interleaved partial sums: independent LDS reads in flight
    int i = 0;
    for (; i + 4 <= n; i += 4) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const T xi = xl[i + q];
            s[q][0] += WT[(i + q) * L + j] * xi;
            s[q][1] += WT[(i + q) * L + j + 1] * xi;
        }
    }
    for (; i < n; ++i) {
        const T xi = xl[i];
        s[0][0] += WT[i * L + j] * xi;
        s[0][1] += WT[i * L + j + 1] * xi;
    }
    y[0] = (s[0][0] + s[1][0]) + (s[2][0] + s[3][0]);
    y[1] = (s[0][1] + s[1][1]) + (s[2][1] + s[3][1]);
}

// Tile: phase A (projections, energies / compat projections, x, d, y = W x) and
// the gradient partials dW = D^T X, dr, as transr_tile_kernel.
// Tile groups (a.tgroup > 1, eight-wave blocks): the block of a relation's tile
// q = 0 (mod tgroup) runs tiles q .. q + tgroup - 1 of that relation one after
// another -- W staged once, dW accumulated in the waves' MFMA registers -- and
// writes ONE matrix partial (on the group's first tile; the others flag zero
// updates, so the relation-row pass skips them).  The blocks of the other tiles
// exit at once.  Sums regroup (partials of up to tgroup tiles instead of one):
// rounding-level differences only.
template <typename T, bool PROJ, bool GRAD, int kNB>
__global__ __launch_bounds__(512, 4) void transr_tile_mfma_kernel(RParArgs a, RParBufs<T> bf) {  // 4 waves an EU: two workgroups a CU
    using M = Mfma16<T>;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int t0 = a.tile_first[a.batch_seg[a.batch]] + blockIdx.x;
    if (t0 >= a.tile_first[a.batch_seg[a.batch + 1]]) return;
    const int w = threadIdx.x >> 6, nw = blockDim.x >> 6, l = lane_id();
    // (a projection-only launch has no partial to share: a tile a block, all in parallel;
    // the register partial needs eight waves)
    const int G = GRAD && nw == 8 && a.tgroup > 1 ? min(a.tgroup, kTileGroupMax) : 1;
    const RTile tl0 = a.tiles[t0];
    if (tl0.q % G != 0) return;  // another block runs this tile
    const int ntl = min(G, a.tile_first[tl0.seg + 1] - t0);
    // the group's relation segment (its tiles are consecutive chunks of St samples)
    const int sp0 = a.seg_start[tl0.seg], sns = (a.seg_start[tl0.seg + 1] - sp0) / 2;
    const int r = a.seg_row[tl0.seg] - a.ne;
    constexpr int NP = 16 * kNB, L = NP + 2;  // kNB = rm_np(n) / 16, exactly
    const int n = a.n, ld = a.ld;
    const int MV = rm_up16(4 * a.St), UY = rm_up16(2 * a.St);
    T* V = (T*)smem;
    T* P = V + (PROJ ? MV * L : 0);
    T* X = P + (PROJ ? MV * L : 0);
    T* D = X + UY * L;  // GRAD only
    T* coef = D + (GRAD ? UY * L : 0);
    int* ids = (int*)(coef + UY);  // entity of every V row
    int* kks = ids + MV;           // sample index of every tile sample (!PROJ: of the group's tiles)
    if (!PROJ) {  // the gradient-only launch needs the samples alone: the whole group's at once
        for (int i = threadIdx.x; i < ntl * a.St; i += blockDim.x) {
            const int f = tl0.q * a.St + i;
            kks[i] = f < sns ? a.kl.kk_of(a.keys[sp0 + 2 * f]) : -1;
        }
    }
    // the group's matrix partial: wave w holds output tiles w, w + 8, ... of the kNB x kNB grid
    constexpr int kAcc = (kNB * kNB + 7) / 8;
    typename M::acc_t gacc[kAcc];
#pragma unroll
    for (int k = 0; k < kAcc; ++k) gacc[k] = typename M::acc_t{T(0), T(0), T(0), T(0)};
    T dr[2] = {T(0), T(0)};  // wave 0: the relation-vector partial
    int nact = 0;
    for (int ti = 0; ti < ntl; ++ti) {
        const int fq = (tl0.q + ti) * a.St;  // (tile_range without its loads)
        const int e0 = sp0 + 2 * fq, cnt = min(a.St, sns - fq);
        const int* kt = PROJ ? kks : kks + ti * a.St;
        // samples of the tile: ids resolved by one thread each, then the rows gathered by all
        for (int row = threadIdx.x; PROJ && row < MV; row += blockDim.x) {
            const int q = row >> 2, which = row & 3;
            int e = -1;
            if (q < cnt) {
                if (a.td_ent) {  // the epoch's tile descriptors (rtile_desc_kernel, side stream)
                    const int64_t td = (int64_t)(t0 + ti) * 8 + q;
                    if (which == 0) kks[q] = a.td_kk[td];
                    e = a.td_ent[td * 4 + which];
                } else {
                    const int kk = a.kl.kk_of(a.keys[e0 + 2 * q]);
                    if (which == 0) kks[q] = kk;
                    const int i0 = a.si[kk], jj = a.sj[kk];
                    const int h = a.heads[i0], tt = a.tails[i0];
                    e = which == 0 ? h : which == 1 ? tt : which == 2 ? (a.side[kk] ? h : jj) : (a.side[kk] ? jj : tt);
                }
            }
            ids[row] = e;
        }
        for (int idx = threadIdx.x; idx < UY * L; idx += blockDim.x) {
            X[idx] = T(0);
            if (GRAD) D[idx] = T(0);
        }
        for (int idx = threadIdx.x; idx < UY; idx += blockDim.x) coef[idx] = T(0);
        __syncthreads();
        if (PROJ) {  // V rows 4q + {0,1,2,3} = h, t, h', t' of sample q (zeros past the data)
            gather_rows<T, NP>(V, ids, MV, bf.ent, n, ld);
            __syncthreads();
            const T* Wg = bf.W + (int64_t)r * n * ld;  // W_r: B fragments from global memory (L2)
            auto va = [&](int m, int k) { return V[m * L + k]; };
            auto wb = [&](int k, int c) { return k < n && c < n ? Wg[(int64_t)k * ld + c] : T(0); };
            auto pput = [&](int m, int c, T v) { P[m * L + c] = v; };
            block_gemm_k<T, NP, decltype(va), decltype(wb), decltype(pput), 4>(MV / 16, kNB, rm_k4(n), va, wb, pput);
            __syncthreads();
            // one wave per sample: energies, hinge, x, d (transr/trainer.cpp:147-164, transr/transr.cpp:26-35)
            for (int q = w; q < cnt; q += nw) {
                const int kk = kks[q];
                const T* ph = P + (4 * q + 0) * L;
                const T* pt = P + (4 * q + 1) * L;
                const T* pnh = P + (4 * q + 2) * L;
                const T* pnt = P + (4 * q + 3) * L;
                T vr[2];
                lane_pair_load(bf.rel + (int64_t)r * ld, n, vr);
                T ep = T(0), en = T(0), xp[2], xn[2];
#pragma unroll
                for (int k = 0; k < 2; ++k) {
                    const int i = 2 * l + k;
                    const bool ok = i < n;
                    const T dp = ok ? pt[i] - ph[i] - vr[k] : T(0);
                    const T dn = ok ? pnt[i] - pnh[i] - vr[k] : T(0);
                    ep += a.l1 ? fabs(dp) : dp * dp;
                    en += a.l1 ? fabs(dn) : dn * dn;
                    xp[k] = ok ? (a.l1 ? (dp > T(0) ? T(1) : T(-1)) : T(2) * dp) : T(0);
                    xn[k] = ok ? (a.l1 ? (dn > T(0) ? T(1) : T(-1)) : T(2) * dn) : T(0);
                }
                T dpos[2], dneg[2];
#pragma unroll
                for (int k = 0; k < 2; ++k) {
                    const int i = 2 * l + k;
                    dpos[k] = i < n ? V[(4 * q + 0) * L + i] - V[(4 * q + 1) * L + i] : T(0);
                    dneg[k] = i < n ? V[(4 * q + 2) * L + i] - V[(4 * q + 3) * L + i] : T(0);
                }
                lane_pair_store(bf.x + ((int64_t)kk * 2 + 0) * ld, n, xp);
                lane_pair_store(bf.x + ((int64_t)kk * 2 + 1) * ld, n, xn);
                lane_pair_store(bf.d + ((int64_t)kk * 2 + 0) * ld, n, dpos);
                lane_pair_store(bf.d + ((int64_t)kk * 2 + 1) * ld, n, dneg);
                lane_pair_store(X + (2 * q + 0) * L, n, xp);
                lane_pair_store(X + (2 * q + 1) * L, n, xn);
                if (a.compat) {
                    double* pr = a.proj + (int64_t)kk * 4 * ld;
#pragma unroll
                    for (int k = 0; k < 2; ++k) {
                        const int i = 2 * l + k;
                        if (i >= n) continue;
                        pr[i] = (double)ph[i];
                        pr[ld + i] = (double)pt[i];
                        pr[2 * ld + i] = (double)pnh[i];
                        pr[3 * ld + i] = (double)pnt[i];
                    }
                } else {
                    ep = wave_sum(ep);
                    en = wave_sum(en);
                    const bool active = (double)ep + a.margin > (double)en;
                    if (l == 0) {
                        a.act[kk] = active ? 1 : 0;
                        a.loss[kk] = active ? a.margin + (double)ep - (double)en : 0.0;
                    }
                    if (GRAD) {
#pragma unroll
                        for (int u = 0; u < 2; ++u) {
                            const T c = active ? (T)(-(u ? 1.0 : -1.0) * a.lr) : T(0);  // -lr beta
                            const T* dv = u ? dneg : dpos;
                            const T dsc[2] = {c * dv[0], c * dv[1]};
                            lane_pair_store(D + (2 * q + u) * L, n, dsc);
                            if (l == 0) coef[2 * q + u] = c;
                        }
                    }
                }
            }
            __syncthreads();
            // y = W x for every update (transr/trainer.cpp:168-169): Y = X W^T
            auto xa = [&](int m, int k) { return X[m * L + k]; };
            auto wtb = [&](int k, int c) { return k < n && c < n ? Wg[(int64_t)c * ld + k] : T(0); };
            auto yput = [&](int m, int c, T v) {
                if (m < 2 * cnt && c < n) bf.y[((int64_t)kks[m >> 1] * 2 + (m & 1)) * ld + c] = v;
            };
            block_gemm_k<T, NP, decltype(xa), decltype(wtb), decltype(yput), 4>(UY / 16, kNB, rm_k4(n), xa, wtb, yput);
        }
        if (GRAD) {
            if (!PROJ) {  // compat: directions from phase A, hinge from the work-vector scan
                for (int q = w; q < cnt; q += nw) {
                    const int kk = kt[q];
                    const bool act = a.act[kk] != 0;
#pragma unroll
                    for (int u = 0; u < 2; ++u) {
                        const T c = act ? (T)(-(u ? 1.0 : -1.0) * a.lr) : T(0);
                        T xv[2], dv[2];
                        lane_pair_load(bf.x + ((int64_t)kk * 2 + u) * ld, n, xv);
                        lane_pair_load(bf.d + ((int64_t)kk * 2 + u) * ld, n, dv);
                        dv[0] *= c;
                        dv[1] *= c;
                        lane_pair_store(X + (2 * q + u) * L, n, xv);
                        lane_pair_store(D + (2 * q + u) * L, n, dv);
                        if (l == 0) coef[2 * q + u] = c;
                    }
                }
            }
            __syncthreads();
            // dW[j][i] = sum_u D[u][j] X[u][i]  (transr/trainer.cpp:166-167)
            if (nw == 8) {  // into the group's register partial
                const int K4 = (2 * cnt + 3) & ~3, kq = l >> 4, c16 = l & 15;
#pragma unroll
                for (int k = 0; k < kAcc; ++k) {
                    const int idx = w + 8 * k;
                    if (idx >= kNB * kNB) continue;
                    const int jc = (idx / kNB) * 16 + c16, ic = (idx % kNB) * 16 + c16;
                    for (int kb = 0; kb < K4; kb += 16) {
                        T av[4], bv[4];
#pragma unroll
                        for (int s = 0; s < 4; ++s) {
                            const int u = kb + 4 * s + kq;
                            av[s] = u < UY ? D[u * L + jc] : T(0);
                            bv[s] = u < UY ? X[u * L + ic] : T(0);
                        }
#pragma unroll
                        for (int s = 0; s < 4; ++s)
                            if (kb + 4 * s < K4) gacc[k] = M::mma(av[s], bv[s], gacc[k]);
                    }
                }
            } else {  // four waves: one tile a block, written directly
                T* wp = bf.wpart + (int64_t)blockIdx.x * n * ld;
                block_gemm<T>(kNB, kNB, UY, [&](int j, int u) { return D[u * L + j]; },
                              [&](int u, int i) { return X[u * L + i]; }, [&](int j, int i, T v) {
                                  if (j < n && i < n) wp[(int64_t)j * ld + i] = v;
                              });
            }
            if (w == 0) {  // dr = sum_u (-lr beta) x_u
                for (int u = 0; u < 2 * cnt; ++u) {
                    const T c = coef[u];
                    dr[0] += c * X[u * L + 2 * l];
                    dr[1] += c * X[u * L + 2 * l + 1];
                    nact += c != T(0);
                }
            }
        }
        if (ti + 1 < ntl) __syncthreads();  // the next tile's ids, X, D
    }
    if (!GRAD) return;
    if (nw == 8) {
        T* wp = bf.wpart + (int64_t)blockIdx.x * n * ld;
#pragma unroll
        for (int k = 0; k < kAcc; ++k) {
            const int idx = w + 8 * k;
            if (idx >= kNB * kNB) continue;
            const int i = (idx % kNB) * 16 + (l & 15);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int j = (idx / kNB) * 16 + M::row(l, q);
                if (j < n && i < n) wp[(int64_t)j * ld + i] = gacc[k][q];
            }
        }
    }
    if (w == 0) {
        lane_pair_store(bf.rpart + (int64_t)blockIdx.x * ld, n, dr);
        if (l == 0) {
            a.tile_act[t0] = nact;
            for (int ti = 1; ti < ntl; ++ti) a.tile_act[t0 + ti] = 0;  // the group's partial is on t0
        }
    }
}

// transRNorm (transr/trainer.cpp:35-64) per tile on the matrix cores, pairs and
// rules of transr_constraint_kernel: the pairs (h', r), (t', r) of the tile's
// active updates and (entity'[r], r) on the relation's first tile, first
// occurrences only, compacted.  With W0 = W'_r and K = W0^T W0 (MFMA, once):
//   P = A0 W0 for all pairs (MFMA), |p|^2 reduced from the accumulators;
//   Jacobi rounds on the violators, one wave per 16-row block with its P and
//   G fragments in registers:  G += 2 p,  p <- p - 2 lr K p - 2 lr (a0.a0) p
//   while |p|^2 > 1 (a row stops at its own first non-violation);
//   pair records da = -lr W0 G (MFMA), the tile's matrix partial -lr A0^T G
//   (MFMA), a flag per update slot (bf.pflag: the record is valid) and the
//   tile's violator count (bf.cons_tile: 0 = no partial).
// transRNorm statistics (tools): rounds summed over row blocks, tiles with violators, most rounds of a block
static __device__ unsigned long long g_rpar_rounds[16];

// kConsNB: the column blocks of 16, exactly (NP = 16 kConsNB): every loop over
// them and over the k-steps below NP has a compile-time trip count.
template <typename T, int kConsNB>
__global__ __launch_bounds__(512) void transr_cons_tile_kernel(RParArgs a, RParBufs<T> bf) {
    using M = Mfma16<T>;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int tb = a.tile_first[a.batch_seg[a.batch]];
    const int t = tb + blockIdx.x;
    if (t >= a.tile_first[a.batch_seg[a.batch + 1]]) return;
    int r, e0, cnt;
    tile_range(a, t, r, e0, cnt);
    constexpr int NB = kConsNB, NP = 16 * NB, L = NP + 2;
    const int n = a.n, ld = a.ld;
    const int PP = rm_up16(4 * a.St + 1);
    T* Wl = (T*)smem;
    T* K = Wl + NP * L;
    T* A0 = K + NP * L;
    T* PG = A0 + PP * L;  // P during the rounds, then G; row PP: zeros (the rounds' padding rows)
    T* PG2 = PG + (PP + 1) * L;  // the rounds' second P buffer, row PP zeros
    T* s0 = PG2 + (PP + 1) * L;  // [PP + 1], s0[PP] = 0
    int* ent_of = (int*)(s0 + PP + 1 + 1);
    int* slot_of = ent_of + PP;  // pair slot (kk * 2 + u) * 2 + role, -2 for (entity[r], r), -1 none
    int* rowmap = slot_of + PP;  // compacted row -> pq
    int* posmap = rowmap + PP;   // pq -> compacted row or -1
    int* vio = posmap + PP;      // compacted row violates (its pair moves)
    int* misc = vio + PP;  // [0] live rows, [1] violators, [2 + 3 (m & 1) + b] row block b live at round m
    T* npart = (T*)(misc + 8);   // [2][PP][kConsNB]: |p|^2 of a row over one column block, per round parity
    int* vrow = (int*)(npart + 2 * kConsNB * PP);  // the violators' rows, compacted: the rounds' row blocks
    const int w = threadIdx.x >> 6, nw = blockDim.x >> 6, l = lane_id();
    const RTile tl = a.tiles[t];
    const unsigned long long ck0 = bf.stats ? clock64() : 0ull;
    bool relpair = false;
    if (tl.q == 0) {
        int any = 0;
        for (int q = a.tile_first[tl.seg]; q < a.tile_first[tl.seg + 1]; ++q) any |= a.tile_act[q];
        relpair = any != 0 && r < a.ne;
    }
    const int npairs = 4 * cnt + (relpair ? 1 : 0);
    if (threadIdx.x == 0) misc[1] = 0;
    if (w == 0) {
        // the pairs, then the first occurrence of each entity compacted in pair
        // order (PP <= kWave: one lane per pair) while the other waves stage W
        const int pq = l;
        int ent = -1, slot = -1;
        if (pq < 4 * cnt) {
            const int q = pq >> 2, u = (pq >> 1) & 1, role = pq & 1;
            const int kk = a.kl.kk_of(a.keys[e0 + 2 * q]);
            if (a.act[kk]) {
                slot = (kk * 2 + u) * 2 + role;
                const int i0 = a.si[kk], jj = a.sj[kk];
                const int h = a.heads[i0], tt = a.tails[i0];
                const int hh = u ? (a.side[kk] ? h : jj) : h;
                const int th = u ? (a.side[kk] ? jj : tt) : tt;
                const int e = role ? th : hh;
                if (!transr_pair_dup(a, slot, r, e)) ent = e;
            }
        } else if (pq < npairs) {
            if (!transr_relpair_dup(a, r)) ent = r;  // entityVec_next_[relation] (transr/trainer.cpp:187)
            slot = -2;
        }
        if (pq < PP) {
            ent_of[pq] = ent;
            slot_of[pq] = slot;
            vio[pq] = 0;
        }
        wave_lds_sync();
        bool dup = false;
        for (int k = 0; k < PP; k += 4) {  // PP is a multiple of 16
            const int4 e4 = *(const int4*)(ent_of + k);
            dup |= (k < pq && e4.x == ent) | (k + 1 < pq && e4.y == ent) | (k + 2 < pq && e4.z == ent) |
                   (k + 3 < pq && e4.w == ent);
        }
        const bool live = ent >= 0 && !dup;
        const uint64_t m = __ballot(live);
        const int pos = __builtin_popcountll(m & ((1ull << l) - 1));
        if (live) rowmap[pos] = pq;
        if (pq < PP) posmap[pq] = live ? pos : -1;
        if (l == 0) misc[0] = __builtin_popcountll(m);
    } else {
        if (w == 1) {  // the zero rows of PG, PG2 and s0[PP]
            for (int i = l; i < L; i += kWave) {
                PG[PP * L + i] = T(0);
                PG2[PP * L + i] = T(0);
            }
            if (l == 0) s0[PP] = T(0);
        }
        const T* Wg = bf.W + (int64_t)r * n * ld;
#pragma unroll 8
        for (int idx = threadIdx.x - kWave; idx < NP * L; idx += blockDim.x - kWave) {
            const int j = idx / L, i = idx % L;
            Wl[idx] = (j < n && i < n) ? Wg[(int64_t)j * ld + i] : T(0);
        }
    }
    __syncthreads();
    const int nrows = misc[0];
    const int MR = rm_up16(nrows);
    for (int idx = threadIdx.x; idx < MR * L; idx += blockDim.x) {
        const int row = idx / L, i = idx % L;
        const int e = row < nrows ? ent_of[rowmap[row]] : -1;
        A0[idx] = (e >= 0 && i < n) ? bf.ent[(int64_t)e * ld + i] : T(0);
    }
    __syncthreads();
    const unsigned long long ck1 = bf.stats ? clock64() : 0ull;
    const T lr = (T)a.lr;
    // One wave per 16-row block (MR / 16 <= PP / 16 <= the block's waves):
    // P0 = A0 W0 and the check; only a tile with violators goes on to
    // K = W0^T W0, s0 = a0.a0 and the rounds.
    const int mb = w;
    const bool rows_here = mb < MR / 16;
    const int ar = mb * 16 + (l & 15), kq = l >> 4;
    typename M::acc_t pf[kConsNB];
    T nrm[4];
    bool live[4];
    auto rowsq = [&](T (&nr)[4]) {  // |p|^2 of the lane's four rows
#pragma unroll
        for (int q = 0; q < 4; ++q) nr[q] = T(0);
#pragma unroll
        for (int nb = 0; nb < kConsNB; ++nb) {
            if (nb >= NB) break;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                T v = pf[nb][q] * pf[nb][q];
                v += dpp_ror<8>(v);
                v += dpp_ror<4>(v);
                v += dpp_ror<2>(v);
                v += dpp_ror<1>(v);
                nr[q] += v;
            }
        }
    };
    // rows of Aop (this block) x Bop over k < rm_k4(n) (past it the images are zero)
    const int K4 = rm_k4(n);
    auto mul = [&](const T* Aop, const T* Bop, typename M::acc_t (&out)[kConsNB]) {
#pragma unroll
        for (int nb = 0; nb < kConsNB; ++nb) {
            if (nb >= NB) break;
            typename M::acc_t acc = {T(0), T(0), T(0), T(0)};
            const int bc = nb * 16 + (l & 15);
#pragma unroll
            for (int kb = 0; kb < NP; kb += 32) {
                T av[8], bv[8];
#pragma unroll
                for (int s8 = 0; s8 < 8; ++s8) {
                    const int k = kb + 4 * s8 + kq;
                    const bool ok = kb + 4 * s8 < NP;  // compile time; zeros past n in the images
                    av[s8] = ok ? Aop[ar * L + k] : T(0);
                    bv[s8] = ok ? Bop[k * L + bc] : T(0);
                }
#pragma unroll
                for (int s8 = 0; s8 < 8; ++s8)
                    if (kb + 4 * s8 < K4) acc = M::mma(av[s8], bv[s8], acc);
            }
            out[nb] = acc;
        }
    };
    if (rows_here) {
        mul(A0, Wl, pf);
        rowsq(nrm);
#pragma unroll
        for (int q = 0; q < 4; ++q) live[q] = mb * 16 + M::row(l, q) < nrows && nrm[q] > T(1);
        if ((l & 15) == 0) {
#pragma unroll
            for (int q = 0; q < 4; ++q)
                if (live[q]) vio[mb * 16 + M::row(l, q)] = 1;
        }
        const uint64_t anyv = __ballot(live[0] || live[1] || live[2] || live[3]);  // all lanes take part
        if (l == 0 && anyv) atomicAdd(&misc[1], 1);
#pragma unroll
        for (int nb = 0; nb < kConsNB; ++nb) {
            if (nb >= NB) break;
#pragma unroll
            for (int q = 0; q < 4; ++q) PG[(mb * 16 + M::row(l, q)) * L + nb * 16 + (l & 15)] = pf[nb][q];
        }
    }
    __syncthreads();
    if (misc[1] != 0) {
        // K = W0^T W0 (symmetric, zero past n) and s0 = a0.a0
        block_gemm_k<T, NP>(NB, NB, rm_k4(n), [&](int m, int k) { return Wl[k * L + m]; },
                      [&](int k, int c) { return Wl[k * L + c]; }, [&](int m, int c, T v) { K[m * L + c] = v; });
        for (int row = w; row < nrows; row += nw) {
            T ss = T(0);
            for (int i = l; i < L; i += kWave) ss += A0[row * L + i] * A0[row * L + i];
            ss = wave_sum(ss);
            if (l == 0) s0[row] = ss;
        }
        if (w == 0) {  // MR <= PP <= kWave
            const bool v = l < MR && vio[l] != 0;
            const uint64_t vm = __ballot(v);
            if (v) vrow[__builtin_popcountll(vm & ((1ull << l) - 1))] = l;
            if (l == 0) {
                const int nv = __builtin_popcountll(vm);
                misc[0] = nv;
                for (int b = 0; b < 3; ++b) misc[2 + b] = b * 16 < nv;  // every violator is live at round 0
            }
        }
        __syncthreads();
        const int nviol = misc[0];
        // The rounds on the violators' rows only (vrow: 16-row blocks of
        // them, usually one), all blocks in lockstep, one (row block, column
        // block) task per wave: a task keeps its 16 x 16 slice of p and G in
        // registers; PG holds the whole p of every row; |p|^2 is summed over
        // the column blocks' partials in column order.  A frozen row (its
        // first non-violation) keeps p, so it stays at <= 1, and a block with
        // no live row skips its MFMAs.
        constexpr int kTasks = (3 * kConsNB + 7) / 8;  // 3 row blocks x NB column blocks over 8 waves
        const int ntask = (rm_up16(nviol) / 16) * NB;
        auto vr_row = [&](int vr) { return vr < nviol ? vrow[vr] : PP; };  // PP: the zero row
        typename M::acc_t ps[kTasks], gs[kTasks];
        bool lv[kTasks][4];
        T cs[kTasks][4];
        int rounds[kTasks] = {};
        // loop invariants: each task's rows (A operand row of the lane, rows of
        // its four results) and, for the first task, its K fragment
        int arow[kTasks], orow[kTasks][4];
        constexpr int KS = NB <= 4 ? NP / 4 : 1;  // k-steps of a cached K fragment
        T kf[KS];
#pragma unroll
        for (int i = 0; i < kTasks; ++i) {
            const int task = w + i * nw;
            const int tm = task / NB, tn = task % NB;
            arow[i] = task < ntask ? vr_row(tm * 16 + (l & 15)) : PP;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int row = task < ntask ? vr_row(tm * 16 + M::row(l, q)) : PP;
                orow[i][q] = row;
                ps[i][q] = PG[row * L + tn * 16 + (l & 15)];
                gs[i][q] = T(0);
                lv[i][q] = row < PP;
                cs[i][q] = T(2) * lr * s0[row];
            }
            if (i == 0 && NB <= 4) {
#pragma unroll
                for (int s4 = 0; s4 < KS; ++s4) kf[s4] = K[(4 * s4 + kq) * L + tn * 16 + (l & 15)];
            }
        }
        unsigned long long ckr[6] = {0ull, 0ull, 0ull, 0ull, 0ull, 0ull};
        unsigned long long ckp = bf.stats ? clock64() : 0ull;
        auto rmark = [&](int k) {
            if (bf.stats) {
                const unsigned long long c = clock64();
                ckr[k] += c - ckp;
                ckp = c;
            }
        };
        // One barrier a round: p is double-buffered (PG, PG2) and so are the
        // partial norms, and every lane re-derives "some row still moves" from
        // the partials (a frozen row keeps |p|^2 <= 1, so live = |p|^2 > 1).
        for (int m = 0; m < kRParMaxIter; ++m) {
            T* Pc = (m & 1) ? PG2 : PG;   // p of this round
            T* Pn = (m & 1) ? PG : PG2;   // p of the next
            T* np = npart + (m & 1) * PP * NB;
            typename M::acc_t qs[kTasks];
            rmark(4);
#pragma unroll
            for (int i = 0; i < kTasks; ++i) {
                const int task = w + i * nw;
                if (task >= ntask) break;
                const int tn = task % NB;
#pragma unroll
                for (int q = 0; q < 4; ++q)
                    if (lv[i][q]) gs[i][q] += T(2) * ps[i][q];
                const uint64_t busy = __ballot(lv[i][0] || lv[i][1] || lv[i][2] || lv[i][3]);
                if (busy) ++rounds[i];
                if (i == 0) rmark(5);
                // (K p) for this slice: rows tm of P times columns tn of K
                typename M::acc_t acc = {T(0), T(0), T(0), T(0)};
                const int ar2 = arow[i], bc = tn * 16 + (l & 15);
#pragma unroll
                for (int kb = 0; kb < NP; kb += 32) {
                    if (!busy) break;
                    T av[8], bv[8];
#pragma unroll
                    for (int s8 = 0; s8 < 8; ++s8) {
                        const int k = kb + 4 * s8 + kq;
                        const bool ok = kb + 4 * s8 < NP;  // compile time
                        av[s8] = ok ? Pc[ar2 * L + k] : T(0);
                        if (i == 0 && NB <= 4) bv[s8] = ok ? kf[(kb / 4 + s8) % KS] : T(0);
                        else bv[s8] = ok ? K[k * L + bc] : T(0);
                    }
#pragma unroll
                    for (int s8 = 0; s8 < 8; ++s8)
                        if (kb + 4 * s8 < K4) acc = M::mma(av[s8], bv[s8], acc);
                }
                qs[i] = acc;
            }
            rmark(0);
#pragma unroll
            for (int i = 0; i < kTasks; ++i) {
                const int task = w + i * nw;
                if (task >= ntask) break;
                const int tm = task / NB, tn = task % NB;
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const int vr = tm * 16 + M::row(l, q), row = orow[i][q];
                    ps[i][q] = lv[i][q] ? ps[i][q] - T(2) * lr * qs[i][q] - cs[i][q] * ps[i][q] : ps[i][q];
                    Pn[row * L + tn * 16 + (l & 15)] = ps[i][q];  // the zero rows stay zero
                    T v = ps[i][q] * ps[i][q];
                    v += dpp_ror<8>(v);
                    v += dpp_ror<4>(v);
                    v += dpp_ror<2>(v);
                    v += dpp_ror<1>(v);
                    if ((l & 15) == 0) np[vr * NB + tn] = v;
                }
            }
            rmark(2);
            __syncthreads();  // p and the partial norms of this round
            rmark(1);
            ckr[3] += 1;
#pragma unroll
            for (int i = 0; i < kTasks; ++i) {
                const int task = w + i * nw;
                if (task >= ntask) break;
                const int tm = task / NB;
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const int vr = tm * 16 + M::row(l, q);
                    T pp[kConsNB];
#pragma unroll
                    for (int c = 0; c < NB; ++c) pp[c] = np[vr * NB + c];
                    T nr = T(0);
#pragma unroll
                    for (int c = 0; c < NB; ++c) nr += pp[c];
                    lv[i][q] = lv[i][q] && nr > T(1);
                }
            }
            bool more = false;  // lane v: violator row v (nviol <= PP <= kWave)
            if (l < nviol) {
                T pp[kConsNB];
#pragma unroll
                for (int c = 0; c < NB; ++c) pp[c] = np[l * NB + c];
                T nr = T(0);
#pragma unroll
                for (int c = 0; c < NB; ++c) nr += pp[c];
                more = nr > T(1);
            }
            if (!__ballot(more)) break;  // the same verdict in every wave
        }
        // G replaces P (every read of P is behind the last barrier): the
        // violators' slices, zeros on the other rows
#pragma unroll
        for (int i = 0; i < kTasks; ++i) {
            const int task = w + i * nw;
            if (task >= ntask) break;
            const int tn = task % NB;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                PG[orow[i][q] * L + tn * 16 + (l & 15)] = gs[i][q];
            }
        }
        for (int idx = threadIdx.x; idx < MR * L; idx += blockDim.x)
            if (!vio[idx / L]) PG[idx] = T(0);
        if (bf.stats && threadIdx.x == 0)
            for (int k = 0; k < 6; ++k) atomicAdd(&g_rpar_rounds[8 + k], ckr[k]);
        if (bf.stats) {
            for (int i = 0; i < kTasks; ++i) {
                const int task = w + i * nw;
                if (task < ntask && task % NB == 0 && l == 0 && rounds[i] > 0) {
                    atomicAdd(&g_rpar_rounds[0], (unsigned long long)rounds[i]);
                    atomicMax(&g_rpar_rounds[2], (unsigned long long)rounds[i]);
                }
            }
        }
    }
    __syncthreads();
    const unsigned long long ck2 = bf.stats ? clock64() : 0ull;
    if (w == 0) {  // pair flags and the tile's entry
        for (int pq = l; pq < 4 * cnt; pq += kWave) {
            const int slot = slot_of[pq];
            if (slot < 0) continue;
            const int pos = posmap[pq];
            bf.pflag[slot] = pos >= 0 && vio[pos] ? 1 : 0;
        }
        if (l == 0) {
            bf.cons_tile[blockIdx.x] = misc[1];
            if (misc[1] && bf.stats) atomicAdd(&g_rpar_rounds[1], 1ull);
        }
    }
    if (misc[1] == 0) {
        if (bf.stats && threadIdx.x == 0) {
            atomicAdd(&g_rpar_rounds[3], ck1 - ck0);
            atomicAdd(&g_rpar_rounds[4], ck2 - ck1);
            atomicMax(&g_rpar_rounds[6], clock64() - ck0);
            atomicAdd(&g_rpar_rounds[7], 1ull);
        }
        return;
    }
    // pair records da = -lr W0 G (B(k, c) = W0[c][k])
    block_gemm_k<T, NP>(MR / 16, NB, rm_k4(n), [&](int m, int k) { return PG[m * L + k]; },
                  [&](int k, int c) { return Wl[c * L + k]; }, [&](int m, int c, T v) {
                      if (m >= nrows || c >= n || !vio[m]) return;
                      const int sl = slot_of[rowmap[m]];
                      if (sl >= 0) bf.pair[(int64_t)sl * ld + c] = -lr * v;
                      else bf.relpair[(int64_t)r * ld + c] = -lr * v;
                  });
    for (int row = threadIdx.x; row < nrows; row += blockDim.x)
        if (vio[row] && slot_of[rowmap[row]] == -2) bf.relpair_stamp[r] = bf.stamp;
    // the tile's matrix partial  dW[j][i] = sum_p (-lr a0[p][j]) G[p][i]
    T* wp = bf.wpart + (int64_t)blockIdx.x * n * ld;
    block_gemm<T>(NB, NB, MR, [&](int j, int p) { return A0[p * L + j]; }, [&](int p, int i) { return PG[p * L + i]; },
                  [&](int j, int i, T v) {
                      if (j < n && i < n) wp[(int64_t)j * ld + i] = -lr * v;
                  });
    if (bf.stats) {
        __syncthreads();
        if (threadIdx.x == 0) {
            const unsigned long long ck3 = clock64();
            atomicAdd(&g_rpar_rounds[3], ck1 - ck0);
            atomicAdd(&g_rpar_rounds[4], ck2 - ck1);
            atomicAdd(&g_rpar_rounds[5], ck3 - ck2);
            atomicMax(&g_rpar_rounds[6], ck3 - ck0);
            atomicAdd(&g_rpar_rounds[7], 1ull);
        }
    }
}

}  // namespace kb2e
