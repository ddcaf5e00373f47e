// kernels_transr_widep.hpp -- the PARALLEL TransR schedule at 128 < n <= 512
// (kernels_transr_parallel.hpp has the model; this file its wide form).
//
// The n <= 128 kernels give a lane two elements of a row and keep the relation
// matrix W_r (n x n) in LDS; at n = 512 the matrix is 2 MiB (FP64), far past the
// 160 KiB of a CU.  Here a lane holds CP element pairs -- elements 128 c + 2 l,
// + 1 for c < CP (CP = ceil(n / 128), up to 4) -- and every matrix is read from
// global memory (L2 / HBM, rows coalesced), so the same steps run at any width
// the engine takes:
//   wide_tile_kernel      phase A per tile (projections, energies / compat
//                         projections, x, d = h - t, y = W x) and the tile's
//                         gradient partials dW, dr (transr/trainer.cpp:144-172);
//   wide_scan_energy      the compat work-vector scan's energies (transr/transr.cpp:
//                         20-35) in chunks small enough for the LDS;
//   wide_rel_rows_kernel  the relation rows: the tiles' partials in tile order,
//                         unit norm (transr/trainer.cpp:174-180);
//   wide_entity_kernel    the entity rows: summed -beta lr y and unit norm, or (after
//                         the chain) the transRNorm pair records with the pre / post
//                         split around the last update's norm;
//   wide_chain_kernel     transRNorm per relation, pair by pair in the reference's
//                         order (transr/trainer.cpp:35-64, :185-187; the chunk1
//                         model of oracle/parallel.py transr_constraint, the same as
//                         kernels_transr_chaing.hpp) with the working matrix W_c in a
//                         global scratch image (a workgroup's own), V = W'^T (W' p)
//                         from the relation's table row, the records at the end.
// Not the fast path of the headline widths: it exists so that every --size the
// reference takes (common/args.cpp:71-74) trains the same model on the GPU.
#pragma once

#include "kernels_transr_seq.hpp"

namespace kb2e {

constexpr int kWideMaxCP = 4;  // element pairs a lane: n <= 512

template <int CP, typename T>
__device__ __forceinline__ void lane_load(const T* row, int n, T (&v)[2 * CP]) {
    const int e0 = 2 * lane_id();
#pragma unroll
    for (int c = 0; c < CP; ++c) {
        const int e = 128 * c + e0;
        v[2 * c] = e < n ? row[e] : T(0);
        v[2 * c + 1] = e + 1 < n ? row[e + 1] : T(0);
    }
}

template <int CP, typename T>
__device__ __forceinline__ void lane_store(T* row, int n, const T (&v)[2 * CP]) {
    const int e0 = 2 * lane_id();
#pragma unroll
    for (int c = 0; c < CP; ++c) {
        const int e = 128 * c + e0;
        if (e < n) row[e] = v[2 * c];
        if (e + 1 < n) row[e + 1] = v[2 * c + 1];
    }
}

// the lane's element k of pair c
__device__ __forceinline__ int lane_elem(int c, int k) { return 128 * c + 2 * lane_id() + k; }

// LDS of the wide tile kernel (elements of T): per wave 4 x ld vectors | X [4 St + 1][ld] |
// D [4 St + 1][ld] | coef [4 St + 1]
template <typename T>
__host__ __device__ constexpr size_t wide_tile_lds(int ld, int St) {
    return sizeof(T) * (4 * 4 * (size_t)ld + 2 * (4 * (size_t)St + 1) * ld + 4 * (size_t)St + 1);
}

// Phase A of one tile (kernels_transr_parallel.hpp transr_tile_kernel), W_r from
// global memory: p_i = sum_j W[j][i] v_j with row j of W read coalesced (lane i),
// y_j = sum_i W[j][i] x_i with the lane's rows j read along i.
template <typename T, bool PROJ, bool GRAD, int CP>
__global__ __launch_bounds__(256) void wide_tile_kernel(RParArgs a, RParBufs<T> bf) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int t = a.tile_first[a.batch_seg[a.batch]] + blockIdx.x;
    if (t >= a.tile_first[a.batch_seg[a.batch + 1]]) return;
    int r, e0, cnt;
    tile_range(a, t, r, e0, cnt);
    const int n = a.n, ld = a.ld;
    constexpr int E = 2 * CP;
    T* vec = (T*)smem;                     // [4 waves][4][ld]
    T* Xl = vec + 16 * ld;                 // [2 cnt][ld] update directions
    T* Dl = Xl + (4 * a.St + 1) * ld;      // [2 cnt][ld] -lr beta (h - t), 0 if inactive
    T* coef = Dl + (4 * a.St + 1) * ld;    // [2 cnt] -lr beta, 0 if inactive
    const int w = threadIdx.x >> 6, l = lane_id();
    const T* Wg = bf.W + (int64_t)r * n * ld;
    T* v4 = vec + w * 4 * ld;
    for (int q = w; q < cnt; q += 4) {
        const int kk = a.kl.kk_of(a.keys[e0 + 2 * q]);
        if (PROJ) {
            const int i0 = a.si[kk], jj = a.sj[kk];
            const int h = a.heads[i0], tt = a.tails[i0];
            const int nh = a.side[kk] ? h : jj, nt = a.side[kk] ? jj : tt;
            T vh[E], vt[E], vnh[E], vnt[E], vr[E];
            lane_load<CP>(bf.ent + (int64_t)h * ld, n, vh);
            lane_load<CP>(bf.ent + (int64_t)tt * ld, n, vt);
            lane_load<CP>(bf.ent + (int64_t)nh * ld, n, vnh);
            lane_load<CP>(bf.ent + (int64_t)nt * ld, n, vnt);
            lane_load<CP>(bf.rel + (int64_t)r * ld, n, vr);
            lane_store<CP>(v4 + 0 * ld, n, vh);
            lane_store<CP>(v4 + 1 * ld, n, vt);
            lane_store<CP>(v4 + 2 * ld, n, vnh);
            lane_store<CP>(v4 + 3 * ld, n, vnt);
            wave_lds_sync();
            // W^T h, W^T t, W^T h', W^T t'
            T p[4][E];
#pragma unroll
            for (int s = 0; s < 4; ++s)
#pragma unroll
                for (int k = 0; k < E; ++k) p[s][k] = T(0);
            for (int j = 0; j < n; ++j) {
                T wv[E];
                lane_load<CP>(Wg + (int64_t)j * ld, n, wv);
#pragma unroll
                for (int s = 0; s < 4; ++s) {
                    const T vj = v4[s * ld + j];
#pragma unroll
                    for (int k = 0; k < E; ++k) p[s][k] += wv[k] * vj;
                }
            }
            T ep = T(0), en = T(0);
            T xp[E], xn[E];
#pragma unroll
            for (int k = 0; k < E; ++k) {
                const bool ok = lane_elem(k >> 1, k & 1) < n;
                const T dp = p[1][k] - p[0][k] - vr[k];
                const T dn = p[3][k] - p[2][k] - vr[k];
                ep += ok ? (a.l1 ? fabs(dp) : dp * dp) : T(0);
                en += ok ? (a.l1 ? fabs(dn) : dn * dn) : T(0);
                xp[k] = ok ? (a.l1 ? (dp > T(0) ? T(1) : T(-1)) : T(2) * dp) : T(0);
                xn[k] = ok ? (a.l1 ? (dn > T(0) ? T(1) : T(-1)) : T(2) * dn) : T(0);
            }
            T dpos[E], dneg[E];
#pragma unroll
            for (int k = 0; k < E; ++k) {
                dpos[k] = vh[k] - vt[k];
                dneg[k] = vnh[k] - vnt[k];
            }
            lane_store<CP>(bf.x + ((int64_t)kk * 2 + 0) * ld, n, xp);
            lane_store<CP>(bf.x + ((int64_t)kk * 2 + 1) * ld, n, xn);
            lane_store<CP>(bf.d + ((int64_t)kk * 2 + 0) * ld, n, dpos);
            lane_store<CP>(bf.d + ((int64_t)kk * 2 + 1) * ld, n, dneg);
            if (a.compat) {
                double* pr = a.proj + (int64_t)kk * 4 * ld;
#pragma unroll
                for (int k = 0; k < E; ++k) {
                    const int e = lane_elem(k >> 1, k & 1);
                    if (e >= n) continue;
                    pr[e] = (double)p[0][k];
                    pr[ld + e] = (double)p[1][k];
                    pr[2 * ld + e] = (double)p[2][k];
                    pr[3 * ld + e] = (double)p[3][k];
                }
            } else {
                ep = wave_sum(ep);
                en = wave_sum(en);
                const bool active = (double)ep + a.margin > (double)en;
                if (l == 0) {
                    a.act[kk] = active ? 1 : 0;
                    a.loss[kk] = active ? a.margin + (double)ep - (double)en : 0.0;
                }
                if (GRAD) {  // the tile's gradient rows, straight to LDS
#pragma unroll
                    for (int u = 0; u < 2; ++u) {
                        const T c = active ? (T)(-(u ? 1.0 : -1.0) * a.lr) : T(0);  // -lr beta
                        const T* dv = u ? dneg : dpos;
                        T dsc[E];
#pragma unroll
                        for (int k = 0; k < E; ++k) dsc[k] = c * dv[k];
                        lane_store<CP>(Xl + (2 * q + u) * ld, n, u ? xn : xp);
                        lane_store<CP>(Dl + (2 * q + u) * ld, n, dsc);
                        if (l == 0) coef[2 * q + u] = c;
                    }
                }
            }
            // y = W x for both updates: the lane's rows j along i, x through LDS
            wave_lds_sync();
            lane_store<CP>(v4 + 0 * ld, n, xp);
            lane_store<CP>(v4 + 1 * ld, n, xn);
            wave_lds_sync();
            T yp[E], yn[E];
#pragma unroll
            for (int k = 0; k < E; ++k) {
                const int j = lane_elem(k >> 1, k & 1);
                T sp = T(0), sn = T(0);
                if (j < n) {
                    const T* wr = Wg + (int64_t)j * ld;
                    for (int i = 0; i < n; ++i) {
                        const T wji = wr[i];
                        sp += wji * v4[i];
                        sn += wji * v4[ld + i];
                    }
                }
                yp[k] = sp;
                yn[k] = sn;
            }
            lane_store<CP>(bf.y + ((int64_t)kk * 2 + 0) * ld, n, yp);
            lane_store<CP>(bf.y + ((int64_t)kk * 2 + 1) * ld, n, yn);
            wave_lds_sync();
        }
    }
    if (!GRAD) return;
    if (!PROJ) {  // compat: directions from phase A, hinge from the work-vector scan
        for (int q = w; q < cnt; q += 4) {
            const int kk = a.kl.kk_of(a.keys[e0 + 2 * q]);
            const bool act = a.act[kk] != 0;
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const T c = act ? (T)(-(u ? 1.0 : -1.0) * a.lr) : T(0);  // -lr beta
                T xv[E], dv[E];
                lane_load<CP>(bf.x + ((int64_t)kk * 2 + u) * ld, n, xv);
                lane_load<CP>(bf.d + ((int64_t)kk * 2 + u) * ld, n, dv);
#pragma unroll
                for (int k = 0; k < E; ++k) dv[k] *= c;
                lane_store<CP>(Xl + (2 * q + u) * ld, n, xv);
                lane_store<CP>(Dl + (2 * q + u) * ld, n, dv);
                if (l == 0) coef[2 * q + u] = c;
            }
        }
    }
    __syncthreads();
    const int U = 2 * cnt;
    T* wp = bf.wpart + (int64_t)blockIdx.x * n * ld;  // partials are per batch: local tile index
    for (int j = w; j < n; j += 4) {  // dW = sum_u (-lr beta) (h - t) x^T
        T acc[E];
#pragma unroll
        for (int k = 0; k < E; ++k) acc[k] = T(0);
        for (int u = 0; u < U; ++u) {
            const T dj = Dl[u * ld + j];
#pragma unroll
            for (int k = 0; k < E; ++k) {
                const int i = lane_elem(k >> 1, k & 1);
                acc[k] += i < n ? dj * Xl[u * ld + i] : T(0);
            }
        }
        lane_store<CP>(wp + (int64_t)j * ld, n, acc);
    }
    if (w == 0) {  // dr = sum_u (-lr beta) x_u
        T acc[E];
#pragma unroll
        for (int k = 0; k < E; ++k) acc[k] = T(0);
        for (int u = 0; u < U; ++u) {
            const T c = coef[u];
#pragma unroll
            for (int k = 0; k < E; ++k) {
                const int i = lane_elem(k >> 1, k & 1);
                if (i < n) acc[k] += c * Xl[u * ld + i];
            }
        }
        lane_store<CP>(bf.rpart + (int64_t)blockIdx.x * ld, n, acc);
        if (l == 0) {
            int nact = 0;
            for (int u = 0; u < U; ++u) nact += coef[u] != T(0);
            a.tile_act[t] = nact;
        }
    }
}

// The compat energies of the chunk's samples from the scan (kernels_transr_parallel.hpp
// rpar_scan_energy_kernel with `chunk` calls a chunk, chosen so that the chunk's
// running vectors [chunk][2 n] fit the LDS), the hinge and the pair-dedupe inserts.
template <typename T, int CP>
__global__ __launch_bounds__(1024) void wide_scan_energy_kernel(RParArgs a, RParBufs<T> bf, const double* sums,
                                                                int32_t nchunks, int32_t chunk, const double* work_in,
                                                                double* work_out, const double* pre) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    double* run_l = (double*)smem;  // [chunk][2 n]
    const int c = blockIdx.x, n = a.n, ld = a.ld;
    const int64_t calls = 2 * (int64_t)a.B;
    const int64_t c0 = (int64_t)c * chunk, c1 = min<int64_t>(calls, c0 + chunk);
    __shared__ int act_l[32];
    const int nsamp = (int)(c1 - c0) / 2;
    int pent = -1, prel = -1;
    if ((int)threadIdx.x < 4 * nsamp) {
        const int64_t kk = c0 / 2 + (threadIdx.x >> 2);
        const int u = (threadIdx.x >> 1) & 1, role = threadIdx.x & 1;
        const int i0 = a.si[kk], jj = a.sj[kk];
        const int h = a.heads[i0], tt = a.tails[i0];
        const int hh = u ? (a.side[kk] ? h : jj) : h;
        const int th = u ? (a.side[kk] ? jj : tt) : tt;
        pent = role ? th : hh;
        prel = a.rels[i0];
    }
    const int E2 = 2 * n;
    for (int e = threadIdx.x; e < E2; e += blockDim.x) {
        double run;
        if (pre) {
            run = pre[(int64_t)c * E2 + e];
        } else {  // (few chunks: the earlier chunks' sums here)
            run = work_in[e];
            for (int q = 0; q < c; ++q) run += sums[(int64_t)q * E2 + e];
        }
        const int side = e / n, i = e % n;
        for (int64_t k = c0; k < c1; ++k) {
            run += a.proj[(k * 2 + side) * ld + i];
            run_l[(k - c0) * E2 + e] = run;
        }
        if (c == nchunks - 1) work_out[e] = run;
    }
    __syncthreads();
    const int w = threadIdx.x >> 6, nw = blockDim.x >> 6, l = lane_id();
    constexpr int E = 2 * CP;
    for (int64_t kk = c0 / 2 + w; kk < c1 / 2; kk += nw) {
        const int r = a.rels[a.si[kk]];
        T vr[E];
        lane_load<CP>(bf.rel + (int64_t)r * ld, n, vr);
        const double* pp = run_l + (kk * 2 - c0) * E2;  // [pos: head n, tail n][neg: head n, tail n]
        double ep = 0, en = 0;
#pragma unroll
        for (int k = 0; k < E; ++k) {
            const int i = lane_elem(k >> 1, k & 1);
            if (i >= n) continue;
            const double dp = pp[n + i] - pp[i] - (double)vr[k];
            const double dn = pp[3 * n + i] - pp[2 * n + i] - (double)vr[k];
            ep += a.l1 ? fabs(dp) : dp * dp;
            en += a.l1 ? fabs(dn) : dn * dn;
        }
        ep = wave_sum(ep);
        en = wave_sum(en);
        const bool active = ep + a.margin > en;
        if (l == 0) {
            a.act[kk] = active ? 1 : 0;
            a.loss[kk] = active ? a.margin + ep - en : 0.0;
            act_l[kk - c0 / 2] = active;
        }
    }
    ptab_clear_next(a, (int64_t)blockIdx.x * blockDim.x + threadIdx.x, (int64_t)gridDim.x * blockDim.x);
    __syncthreads();
    if (pent >= 0 && act_l[threadIdx.x >> 2])
        ptab_insert(a, prel, pent, (int)(c0 / 2) * 4 + (int)threadIdx.x);
}

// One wave per (relation segment, row j <= n): the tiles' partials in tile order
// added to row j of W_r (j < n) or the relation vector (j == n), then the unit
// norm (transr/trainer.cpp:174-180) -- kernels_transr_parallel.hpp
// transr_rel_rows_wave<NORM = true> with CP pairs a lane.
template <typename T, int CP>
__global__ __launch_bounds__(256) void wide_rel_rows_kernel(RParArgs a, RParBufs<T> bf) {
    const int gw = (int)((blockIdx.x * blockDim.x + threadIdx.x) >> 6);
    const int rows = a.n + 1;
    const int s = a.rel_begin[a.batch] + gw / rows;
    const int j = gw % rows;
    if (s >= a.batch_seg[a.batch + 1]) return;
    const int r = a.seg_row[s] - a.ne;
    const int t0 = a.tile_first[s], t1 = a.tile_first[s + 1];
    const int n = a.n, ld = a.ld;
    const int tb = a.tile_first[a.batch_seg[a.batch]];  // partials are indexed by tile within the batch
    constexpr int E = 2 * CP;
    bool any = false;
    for (int t = t0; t < t1 && !any; ++t) any = a.tile_act[t] != 0;
    if (!any) return;  // no active update: the reference leaves the relation alone
    T* row = j < n ? bf.W + ((int64_t)r * n + j) * ld : bf.rel + (int64_t)r * ld;
    T v[E];
    lane_load<CP>(row, n, v);
    for (int t = t0; t < t1; ++t) {
        if (!a.tile_act[t]) continue;  // (inactive tiles carry zero partials)
        const int64_t lt = t - tb;
        T p[E];
        lane_load<CP>(j < n ? bf.wpart + (lt * n + j) * ld : bf.rpart + lt * ld, n, p);
#pragma unroll
        for (int k = 0; k < E; ++k) v[k] += p[k];
    }
    T ss = T(0);
#pragma unroll
    for (int k = 0; k < E; ++k) ss += v[k] * v[k];
    const T len = sqrt(wave_sum(ss));
#pragma unroll
    for (int k = 0; k < E; ++k) v[k] = v[k] / len;
    lane_store<CP>(row, n, v);
}

// One wave per entity segment of the batch (kernels_transr_parallel.hpp
// transr_entity_block's short-segment form with CP pairs a lane): GRAD -- the
// summed -beta lr y of the row's updates, then the unit norm; !GRAD -- the
// transRNorm pair records of the row's moved pairs, split around the unit norm
// of its last update (bf.last_renorm), and (entity'[r], r) when stamped.
template <typename T, bool GRAD, int CP>
__global__ __launch_bounds__(256) void wide_entity_kernel(RParArgs a, RParBufs<T> bf) {
    constexpr int E = 2 * CP;
    const int s0 = a.batch_seg[a.batch], s1 = a.rel_begin[a.batch];  // entity segments sort first
    const int s = s0 + (int)((blockIdx.x * blockDim.x + threadIdx.x) >> 6);
    if (s >= s1) return;
    const int p0 = a.seg_start[s], p1 = a.seg_start[s + 1];
    const int row = a.seg_row[s];
    const int n = a.n, ld = a.ld, l = lane_id();
    const bool split = !GRAD && bf.last_renorm;
    const int last = split ? rpar_entity_last(a, p0, p1, 0, 1) : -1;
    T acc[E], acc2[E];
#pragma unroll
    for (int k = 0; k < E; ++k) acc[k] = acc2[k] = T(0);
    bool dirty = false, dirty2 = false, er_seen = false;
    for (int base = p0; base < p1; base += kWave) {
        const int p = base + l;
        int src = -1, src2 = -1;
        T c = T(0);
        bool nrm = false, er = false, post = false;
        if (p < p1) {
            const uint64_t key = a.keys[p];
            const int kk = a.kl.kk_of(key);
            if (a.act[kk]) {
                const int u = (int)((key >> 3) & 1);
                const uint32_t roles = (uint32_t)(key & 7);
                const bool hd = roles & kRoleHead, tl = roles & kRoleTail;
                er = roles & kRoleEntRel;
                if (GRAD) {
                    nrm = hd || tl;
                    if (hd != tl) {  // head and tail at once: -beta lr y + beta lr y
                        src = kk * 2 + u;
                        c = (T)((hd ? -1.0 : 1.0) * (u ? 1.0 : -1.0) * a.lr);
                    }
                } else {
                    const int s2 = (kk * 2 + u) * 2;
                    const bool ph = hd && (!bf.pflag || bf.pflag[s2]);
                    const bool pt = tl && (!bf.pflag || bf.pflag[s2 + 1]);
                    nrm = ph || pt;
                    post = split && kk * 2 + u == last;
                    if (ph) src = s2;
                    if (pt) {
                        if (src < 0) src = s2 + 1;
                        else src2 = s2 + 1;
                    }
                }
            }
        }
        if (__ballot(nrm && !post)) dirty = true;
        if (__ballot(nrm && post)) dirty2 = true;
        if (__ballot(er)) er_seen = true;
        const T* tab = GRAD ? bf.y : bf.pair;
        const uint64_t pm = __ballot(post);
        for (int pass = 0; pass < (GRAD ? 1 : 2); ++pass) {
            const int mine = pass ? src2 : src;
            for (uint64_t m = __ballot(mine >= 0); m; m &= m - 1) {  // in event order
                const int ev = __builtin_ctzll(m);
                T v[E];
                lane_load<CP>(tab + (int64_t)readlane_i32(mine, ev) * ld, n, v);
                const T cq = GRAD ? readlane_f(c, ev) : T(1);
                const bool to2 = (pm >> ev) & 1;
#pragma unroll
                for (int k = 0; k < E; ++k) {
                    if (to2) acc2[k] += cq * v[k];
                    else acc[k] += cq * v[k];
                }
            }
        }
    }
    if (!GRAD && er_seen && row < a.nr && bf.relpair_stamp[row] == bf.stamp) {
        T dv[E];
        lane_load<CP>(bf.relpair + (int64_t)row * ld, n, dv);
        if (split && last < 0) {  // no update renormalises the row: the delta stays
#pragma unroll
            for (int k = 0; k < E; ++k) acc2[k] += dv[k];
            dirty2 = true;
        } else {
#pragma unroll
            for (int k = 0; k < E; ++k) acc[k] += dv[k];
            dirty = true;
        }
    }
    if (!dirty && !dirty2) return;
    T* ptr = bf.ent + (int64_t)row * ld;
    T v[E];
    lane_load<CP>(ptr, n, v);
    if (dirty) {
#pragma unroll
        for (int k = 0; k < E; ++k) v[k] += acc[k];
    }
    if (GRAD || (split && dirty)) {
        T ss = T(0);
#pragma unroll
        for (int k = 0; k < E; ++k) ss += v[k] * v[k];
        const T len = sqrt(wave_sum(ss));
#pragma unroll
        for (int k = 0; k < E; ++k) v[k] = v[k] / len;
    }
    if (dirty2) {
#pragma unroll
        for (int k = 0; k < E; ++k) v[k] += acc2[k];
    }
    lane_store<CP>(ptr, n, v);
}

// ---- transRNorm, pair by pair (kernels_transr_chaing.hpp, wide) ---------------

constexpr int kWideThreads = 256;  // four waves
constexpr int kWideRows = 8;       // pairs a chunk
constexpr int kWideWin = 128;      // samples a window
constexpr int kWidePairs = 4 * kWideWin;

// LDS bytes: A [R][ld] | P [R][ld] | Gram [R][R] | u, V [2][ld] | qv [R] | red [8] (double)
// ; ints: pe, ps [kWidePairs] | wsum [4] | misc [8] ; vflag [kWidePairs]
__host__ __device__ constexpr size_t wide_chain_lds(int ld) {
    return sizeof(double) * (2 * (size_t)kWideRows * ld + kWideRows * kWideRows + 2 * (size_t)ld + kWideRows + 8) +
           sizeof(int) * (2 * (size_t)kWidePairs + 4 + 8) + (size_t)kWidePairs;
}

// One four-wave workgroup per relation of the batch, every step in double:
// W_c (n x ld) in the workgroup's global scratch image `wsc` (written back to the
// table at the end), the chunk's rows and projections in LDS.
template <typename T, int CP>
__global__ __launch_bounds__(kWideThreads) void wide_chain_kernel(RParArgs a, RParBufs<T> bf, double* wsc_all) {
    constexpr int R = kWideRows, NT = kWideThreads, NW = NT / 64, E = 2 * CP;
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
    const int tid = threadIdx.x, w = tid >> 6, l = lane_id();
    const double lr = a.lr, eps = 2.0 * a.lr;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    double* A = (double*)smem;              // [R][ld] the chunk's entity rows
    double* P = A + R * ld;                 // [R][ld] projections; the violators' rows then hold G
    double* Gm = P + R * ld;                // [R][R] a_j . a_k
    double* uv = Gm + R * R;                // [ld] W' p
    double* Vv = uv + ld;                   // [ld] V = W'^T (W' p)
    double* qv = Vv + ld;                   // [R] |p_j|^2
    int* pe = (int*)(qv + R + 8);           // [kWidePairs]
    int* ps = pe + kWidePairs;              // [kWidePairs]
    int* wsum = ps + kWidePairs;            // [NW]
    int* misc = wsum + 4;                   // [8]
    uint8_t* vflag = (uint8_t*)(misc + 8);  // [kWidePairs]
    const T* W0 = bf.W + (int64_t)r * n * ld;  // W' (the table row holds it until the write-back)
    double* Wc = wsc_all + (int64_t)blockIdx.x * n * ld;  // this workgroup's working matrix

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

    for (int64_t idx = tid; idx < (int64_t)n * ld; idx += NT) {
        const int i = (int)(idx % ld);
        Wc[idx] = i < n ? (double)W0[idx] : 0.0;
    }
    bool changed = false;
    __syncthreads();

    // one chunk: pairs [b, b + cc) of the LDS list; leaves W_c updated, vflag and the
    // records set
    auto chunk = [&](int b, int cc) {
        for (int idx = tid; idx < R * ld; idx += NT) {
            const int k = idx / ld, i = idx % ld;
            const int e = k < cc ? pe[b + k] : -1;
            A[idx] = e >= 0 && i < n ? (double)bf.ent[(int64_t)e * ld + i] : 0.0;
        }
        __syncthreads();
        // P = A W_c: wave w rows w, w + 4; lane l its element pairs; then |p|^2
        {
            double p[2][E];
#pragma unroll
            for (int h = 0; h < 2; ++h)
#pragma unroll
                for (int k = 0; k < E; ++k) p[h][k] = 0.0;
            for (int j = 0; j < n; ++j) {
                double wc[E];
                lane_load<CP>(Wc + (int64_t)j * ld, n, wc);
                const double a0 = A[w * ld + j], a1 = A[(w + 4) * ld + j];
#pragma unroll
                for (int k = 0; k < E; ++k) {
                    p[0][k] = fma(a0, wc[k], p[0][k]);
                    p[1][k] = fma(a1, wc[k], p[1][k]);
                }
            }
            double sq[2];
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int k = w + 4 * h;
                lane_store<CP>(P + k * ld, n, p[h]);
                double acc = 0.0;
#pragma unroll
                for (int q = 0; q < E; ++q) acc += p[h][q] * p[h][q];
                sq[h] = acc;
            }
            wave_sums<double, 2>(sq);
            if (l == 0) {
                qv[w] = w < cc ? sq[0] : 0.0;
                qv[w + 4] = w + 4 < cc ? sq[1] : 0.0;
            }
            if (w == 0) {  // the Gram matrix: lane (k1, k2)
                const int k1 = l >> 3, k2 = l & 7;
                double g = 0.0;
                for (int j = 0; j < n; ++j) g = fma(A[k1 * ld + j], A[k2 * ld + j], g);
                Gm[k1 * R + k2] = g;
            }
        }
        __syncthreads();
        uint32_t vmask = 0;
        for (int cursor = 0;;) {
            const double qq = l < R ? qv[l] : 0.0;
            const uint64_t cand = __ballot(l < cc && l >= cursor && qq > 1.0);
            if (!cand) break;
            const int v = __builtin_ctzll(cand);
            const double pp = readlane_f(qq, v);
            const double aa = Gm[v * R + v];
            // u = W' p_v: a wave a row j (rows tid >> 6, + NW, ...), the row's elements over the lanes
            for (int j = w; j < n; j += NW) {
                T wr[E];
                lane_load<CP>(W0 + (int64_t)j * ld, n, wr);
                double acc = 0.0;
#pragma unroll
                for (int k = 0; k < E; ++k) {
                    const int i = lane_elem(k >> 1, k & 1);
                    if (i < n) acc = fma((double)wr[k], P[v * ld + i], acc);
                }
                acc = wave_sum(acc);
                if (l == 0) uv[j] = acc;
            }
            __syncthreads();
            // V_i = sum_j W'[j][i] u_j: a thread a column i (strided), rows in order
            for (int i = tid; i < ld; i += NT) {
                double acc = 0.0;
                if (i < n)
                    for (int j = 0; j < n; ++j) acc = fma((double)W0[(int64_t)j * ld + i], uv[j], acc);
                Vv[i] = i < n ? acc : 0.0;
            }
            __syncthreads();
            // p.V, V.V (every wave the same sums), the rounds, g in the lane's elements
            double pv[E], vv[E];
            double s2[2] = {0.0, 0.0};
#pragma unroll
            for (int k = 0; k < E; ++k) {
                const int i = lane_elem(k >> 1, k & 1);
                pv[k] = i < n ? P[v * ld + i] : 0.0;
                vv[k] = i < n ? Vv[i] : 0.0;
                s2[0] += pv[k] * vv[k];
                s2[1] += vv[k] * vv[k];
            }
            wave_sums<double, 2>(s2);
            const double pV = s2[0], VV = s2[1];
            const double pvd = pV + aa * pp, vvd = VV + 2.0 * aa * pV + aa * aa * pp;
            const double kappa = pvd / pp;
            const double w2t = vvd - kappa * pvd;
            const double w2 = w2t > 0.0 ? w2t : 0.0;
            const double rho = 1.0 - eps * kappa;
            double S0, S1;
            transr_rounds_violator4(pp, w2, eps, rho, S0, S1);
            const double cpf = 2.0 * (S0 + eps * S1 * kappa), cvf = 2.0 * eps * S1;
            double g[E];
#pragma unroll
            for (int k = 0; k < E; ++k) g[k] = cpf * pv[k] - cvf * (vv[k] + aa * pv[k]);
            __syncthreads();  // every wave has read P's row v
            // the later rows: P_k -= lr (a_k . a_v) g, |p_k|^2 afresh; row v holds G
            double sq[2] = {0.0, 0.0};
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int k = w + 4 * h;
                if (k == v) lane_store<CP>(P + k * ld, n, g);
                if (k > v && k < cc) {
                    const double gl = -lr * Gm[k * R + v];
                    double x[E];
                    lane_load<CP>(P + k * ld, n, x);
                    double acc = 0.0;
#pragma unroll
                    for (int q = 0; q < E; ++q) {
                        x[q] = fma(gl, g[q], x[q]);
                        acc += x[q] * x[q];
                    }
                    lane_store<CP>(P + k * ld, n, x);
                    sq[h] = acc;
                }
            }
            wave_sums<double, 2>(sq);
            if (l == 0) {
                if (w > v && w < cc) qv[w] = sq[0];
                if (w + 4 > v && w + 4 < cc) qv[w + 4] = sq[1];
            }
            vmask |= 1u << v;
            cursor = v + 1;
            __syncthreads();  // the new |p|^2 and the G row
        }
        if (!vmask) return;
        changed = true;
        // the records G, flags, and W_c[j][i] -= lr sum_v a_v[j] G_v[i]
        for (uint32_t mm = vmask; mm; mm &= mm - 1) {
            const int v = __builtin_ctz(mm);
            const int sl = ps[b + v];
            T* dst = sl >= 0 ? bf.pair + (int64_t)sl * ld : bf.relpair + (int64_t)r * ld;
            if (w == 0) {
#pragma unroll
                for (int k = 0; k < E; ++k) {
                    const int i = lane_elem(k >> 1, k & 1);
                    if (i < n) dst[i] = (T)P[v * ld + i];
                }
            }
            if (tid == 0) {
                vflag[b + v] = 1;
                if (sl < 0) bf.relpair_stamp[r] = bf.stamp;
            }
        }
        for (int j = w; j < n; j += NW) {
            double x[E];
            lane_load<CP>(Wc + (int64_t)j * ld, n, x);
            for (uint32_t mm = vmask; mm; mm &= mm - 1) {
                const int v = __builtin_ctz(mm);
                const double al = -lr * A[v * ld + j];
#pragma unroll
                for (int k = 0; k < E; ++k) {
                    const int i = lane_elem(k >> 1, k & 1);
                    x[k] = fma(al, i < n ? P[v * ld + i] : 0.0, x[k]);
                }
            }
            lane_store<CP>(Wc + (int64_t)j * ld, n, x);
        }
        __syncthreads();  // (W_c's rows, read by every wave at the next chunk)
    };

    // windows of kWideWin samples up to the last active one; the last update's slots wait for the tail
    for (int wq = 0; wq <= klq; wq += kWideWin) {
        const int q = wq + tid;
        int kk = -1, ents[4] = {-1, -1, -1, -1};
        uint32_t keep = 0;
        if (tid < kWideWin && q <= klq) {
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
        for (int b = 0; b < npw; b += R) {
            chunk(b, min(R, npw - b));
            __syncthreads();  // W_c, and A / P free for the next chunk
        }
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
        if (changed) {  // the last update's unit rows (transr/trainer.cpp:178-180): a wave a row
            for (int j = w; j < n; j += NW) {
                double x[E];
                lane_load<CP>(Wc + (int64_t)j * ld, n, x);
                double ss = 0.0;
#pragma unroll
                for (int k = 0; k < E; ++k) ss += x[k] * x[k];
                const double len = sqrt(wave_sum(ss));
#pragma unroll
                for (int k = 0; k < E; ++k) x[k] = x[k] / len;
                lane_store<CP>(Wc + (int64_t)j * ld, n, x);
            }
        }
        __syncthreads();  // the tail list and W_c
        chunk(0, ntail);
        __syncthreads();
    }
    if (tid == 0) {
        int pos = 0;
        for (int k = 0; k < 2; ++k) bf.pflag[kl * 4 + 2 + k] = ((tkeep >> k) & 1) ? vflag[pos++] : 0;
    }
    // the relation's matrix back to its table row
    for (int64_t idx = tid; idx < (int64_t)n * ld; idx += NT) {
        if ((int)(idx % ld) < n) bf.W[(int64_t)r * n * ld + idx] = (T)Wc[idx];
    }
    __syncthreads();
    // the pair records da = -lr W G with the final matrix: the relation's violator
    // slots (pflag) of its active samples and (entity'[r], r) when stamped; windows
    // of kWideWin samples, the list in pe; groups of up to R records: their G rows
    // staged in LDS (A and P, free now), W_c read once a group, a wave a row j of it
    // (coalesced), the group's dots by wave sums
    const bool relrec = r < a.ne && bf.relpair_stamp[r] == bf.stamp;
    double* gst = A;  // [2 R][ld] (A and P are contiguous)
    constexpr int G = 2 * R;
    for (int wq = 0; wq < ns; wq += kWideWin) {
        const int q = wq + tid;
        int kk = -1;
        uint32_t fl = 0;
        if (tid < kWideWin && q < ns) {
            kk = a.kl.kk_of(a.keys[p0 + 2 * q]);
            if (a.act[kk])
                for (int k = 0; k < 4; ++k) fl |= bf.pflag[kk * 4 + k] ? 1u << k : 0u;
        }
        const int cnt = __builtin_popcount(fl);
        int x = cnt;
#pragma unroll
        for (int sh = 1; sh < kWave; sh <<= 1) {
            const int y = __shfl_up(x, sh);
            if (l >= sh) x += y;
        }
        if (l == kWave - 1) wsum[w] = x;
        __syncthreads();
        int off = 0, tot = 0;
#pragma unroll
        for (int k = 0; k < NW; ++k) {
            const int ws = wsum[k];
            off += k < w ? ws : 0;
            tot += ws;
        }
        {
            int pos = off + x - cnt;
            for (int k = 0; k < 4; ++k)
                if ((fl >> k) & 1) pe[pos++] = kk * 4 + k;
        }
        if (wq == 0 && relrec) {
            if (tid == 0) pe[tot] = -2;
            ++tot;
        }
        __syncthreads();  // the list
        for (int m0 = 0; m0 < tot; m0 += G) {
            const int gc = min(G, tot - m0);
            auto rec_row = [&](int k) {
                const int sl = pe[m0 + k];
                return sl >= 0 ? bf.pair + (int64_t)sl * ld : bf.relpair + (int64_t)r * ld;
            };
            for (int idx = tid; idx < gc * ld; idx += NT) {
                const int k = idx / ld, i = idx % ld;
                gst[idx] = i < n ? (double)rec_row(k)[i] : 0.0;
            }
            __syncthreads();  // the group's G rows (read before they are overwritten below)
            for (int j = w; j < n; j += NW) {
                double wr[E];
                lane_load<CP>(Wc + (int64_t)j * ld, n, wr);
                double d[G];
#pragma unroll
                for (int k = 0; k < G; ++k) {
                    double acc = 0.0;
                    if (k < gc)
#pragma unroll
                        for (int e = 0; e < E; ++e) {
                            const int i = lane_elem(e >> 1, e & 1);
                            if (i < n) acc = fma(wr[e], gst[k * ld + i], acc);
                        }
                    d[k] = acc;
                }
                wave_sums<double, G>(d);
                double mine = 0.0;
#pragma unroll
                for (int k = 0; k < G; ++k) mine = k == l ? d[k] : mine;
                if (l < gc) rec_row(l)[j] = (T)(-lr * mine);
            }
            __syncthreads();  // (the staged rows are rewritten by the next group)
        }
    }
}

}  // namespace kb2e
