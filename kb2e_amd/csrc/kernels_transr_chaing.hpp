// kernels_transr_chaing.hpp -- transRNorm of the PARALLEL TransR schedule per
// relation, pair by pair, for the widths and precisions the matrix-core chains
// do not take: FP32 tables (any n <= 128) and FP64 at 112 < n <= 128.  The same
// model as the other chain kernels (oracle/parallel.py transr_constraint,
// cons="chunk1"; the reference's calls are transr/trainer.cpp:185-187 on the loop
// at :35-64): the relation's pairs (h', r), (t', r) of its active updates in
// (sample, update, role) order, first occurrences per relation per batch, each
// checked against the matrix the earlier violators left; a violator's rounds in
// closed form along p and V = p K0 (transr_norm_rounds, K0 = W'^T W'), then
// W_c -= lr a^T g; the relation's last update's pairs and (entity'[r], r) after
// W_c's rows are renormalised; the pair records G become da = -lr W G with the
// relation's final matrix, and the entity pass splits pre / post deltas around
// the unit norm (bf.last_renorm).
//
// One four-wave workgroup per relation, every step in double whatever the table
// type (FP32 tables are widened on load and rounded on store).  W_c lives in LDS
// (n x LW doubles, up to 128 KiB at n = 128), so K0 does not fit beside it: V is
// W'^T (W' p) with W' read from the relation's table row (it is written back only
// at the end, so it still holds W' during the chain; L2-resident).  The chain is
// walked in lockstep, chunks of kGenRows pairs: P = A W_c and the chunk's Gram
// matrix, then per violator two barriers (W' p, then V) and one for the later
// rows' P_j -= lr (a_j . a_v) g and |p_j|^2.  Not the fast path: it exists so that
// these configurations train the same model as the FP64 kernels instead of the
// Jacobi form (whose loss departs from the reference's).
#pragma once

#include "kernels_transr_seq.hpp"

namespace kb2e {

constexpr int kGenThreads = 256;       // four waves
constexpr int kGenRows = 8;            // pairs a chunk
constexpr int kGenWin = 128;           // samples a window
constexpr int kGenPairs = 4 * kGenWin;
constexpr int kGenMaxN = 128;          // a lane holds the column pair 2 l, 2 l + 1

__host__ __device__ constexpr int gen_lw(int n) { return (n + 1) & ~1; }

// LDS bytes: W_c [n][LW] | A [R][LW] | P [R][LW] | Gram [R][R] | u, V [2][LW] | qv [R] | red [4][2]
// ; ints: pe, ps [kGenPairs] | wsum [4] | misc [8] ; vflag [kGenPairs]
__host__ __device__ constexpr size_t chaing_lds(int n) {
    return sizeof(double) * ((size_t)n * gen_lw(n) + 2 * (size_t)kGenRows * gen_lw(n) + kGenRows * kGenRows +
                             2 * (size_t)gen_lw(n) + kGenRows + 8) +
           sizeof(int) * (2 * (size_t)kGenPairs + 4 + 8) + (size_t)kGenPairs;
}

template <typename T>
__global__ __launch_bounds__(kGenThreads) void transr_cons_chain_gen_kernel(RParArgs a, RParBufs<T> bf) {
    constexpr int R = kGenRows, NT = kGenThreads, NW = NT / 64;
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
    const int n = a.n, ld = a.ld, LW = gen_lw(n);
    const int p0 = a.seg_start[s], ns = (a.seg_start[s + 1] - p0) / 2;
    const int tid = threadIdx.x, w = tid >> 6, l = lane_id();
    const int c0 = 2 * l;                  // the lane's column pair
    const bool cok0 = c0 < n, cok1 = c0 + 1 < n;
    const double lr = a.lr, eps = 2.0 * a.lr;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    double* Wc = (double*)smem;           // [n][LW] the working matrix
    double* A = Wc + n * LW;              // [R][LW] the chunk's entity rows
    double* P = A + R * LW;               // [R][LW] projections; the violators' rows then hold G
    double* Gm = P + R * LW;              // [R][R] a_j . a_k
    double* uv = Gm + R * R;              // [LW] W' p
    double* Vv = uv + LW;                 // [LW] V = W'^T (W' p)
    double* qv = Vv + LW;                 // [R] |p_j|^2
    double* red = qv + R;                 // [NW][2]
    int* pe = (int*)(red + 2 * NW);       // [kGenPairs]
    int* ps = pe + kGenPairs;             // [kGenPairs]
    int* wsum = ps + kGenPairs;           // [NW]
    int* misc = wsum + NW;                // [8]
    uint8_t* vflag = (uint8_t*)(misc + 8);  // [kGenPairs]
    const T* W0 = bf.W + (int64_t)r * n * ld;  // W' (the table row holds it until the write-back)

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

    for (int idx = tid; idx < n * LW; idx += NT) {
        const int j = idx / LW, i = idx % LW;
        Wc[idx] = i < n ? (double)W0[(int64_t)j * ld + i] : 0.0;
    }
    bool changed = false;
    __syncthreads();

    // one chunk: pairs [b, b + cc) of the LDS list; leaves W_c updated, vflag and the
    // records set
    auto chunk = [&](int b, int cc) {
        for (int idx = tid; idx < R * LW; idx += NT) {
            const int k = idx / LW, i = idx % LW;
            const int e = k < cc ? pe[b + k] : -1;
            A[idx] = e >= 0 && i < n ? (double)bf.ent[(int64_t)e * ld + i] : 0.0;
        }
        __syncthreads();
        // P = A W_c: wave w rows w, w + 4; lane l columns 2 l, 2 l + 1; then |p|^2
        {
            double p[2][2] = {{0.0, 0.0}, {0.0, 0.0}};
            if (cok0) {
                for (int j = 0; j < n; ++j) {
                    const double2 wc = *(const double2*)(Wc + j * LW + c0);
                    const double a0 = A[w * LW + j], a1 = A[(w + 4) * LW + j];
                    p[0][0] = fma(a0, wc.x, p[0][0]);
                    p[0][1] = fma(a0, wc.y, p[0][1]);
                    p[1][0] = fma(a1, wc.x, p[1][0]);
                    p[1][1] = fma(a1, wc.y, p[1][1]);
                }
            }
            double sq[2];
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                if (!cok1) p[h][1] = 0.0;
                const int k = w + 4 * h;
                if (cok0) *(double2*)(P + k * LW + c0) = double2{p[h][0], p[h][1]};
                sq[h] = p[h][0] * p[h][0] + p[h][1] * p[h][1];
            }
            wave_sums<double, 2>(sq);
            if (l == 0) {
                qv[w] = w < cc ? sq[0] : 0.0;
                qv[w + 4] = w + 4 < cc ? sq[1] : 0.0;
            }
            if (w == 0) {  // the Gram matrix: lane (k1, k2)
                const int k1 = l >> 3, k2 = l & 7;
                double g = 0.0;
                for (int j = 0; j < n; ++j) g = fma(A[k1 * LW + j], A[k2 * LW + j], g);
                Gm[k1 * R + k2] = g;
            }
        }
        __syncthreads();
        uint32_t vmask = 0;
        for (int cursor = 0;;) {
            // the next violator: every wave reads the same |p|^2 (uniform)
            const double qq = l < R ? qv[l] : 0.0;
            const uint64_t cand = __ballot(l < cc && l >= cursor && qq > 1.0);
            if (!cand) break;
            const int v = __builtin_ctzll(cand);
            const double pp = readlane_f(qq, v);
            const double aa = Gm[v * R + v];
            // u = W' p_v: a thread per half row (rows j = tid >> 1)
            {
                const int j = tid >> 1, hf = tid & 1, i0 = hf * (LW / 2), i1 = min(n, i0 + LW / 2);
                double acc = 0.0;
                if (j < n)
                    for (int i = i0; i < i1; ++i) acc = fma((double)W0[(int64_t)j * ld + i], P[v * LW + i], acc);
                acc += dpp_mov<0xB1>(acc);  // the two halves (quad_perm [1,0,3,2])
                if (j < n && hf == 0) uv[j] = acc;
            }
            __syncthreads();
            // V_i = sum_j W'[j][i] u_j: a thread per (column, half of the rows)
            {
                const int i = tid >> 1, hf = tid & 1, j0 = hf * (n / 2), j1 = hf ? n : n / 2;
                double acc = 0.0;
                if (i < n)
                    for (int j = j0; j < j1; ++j) acc = fma((double)W0[(int64_t)j * ld + i], uv[j], acc);
                acc += dpp_mov<0xB1>(acc);
                if (i < LW && hf == 0) Vv[i] = i < n ? acc : 0.0;
            }
            __syncthreads();
            // p.V, V.V (every wave the same sums), the rounds, g in the lane's columns
            const double2 pv2 = cok0 ? *(const double2*)(P + v * LW + c0) : double2{0.0, 0.0};
            const double2 vv2 = cok0 ? *(const double2*)(Vv + c0) : double2{0.0, 0.0};
            double s2[2] = {pv2.x * vv2.x + pv2.y * vv2.y, vv2.x * vv2.x + vv2.y * vv2.y};
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
            const double g0 = cok0 ? cpf * pv2.x - cvf * (vv2.x + aa * pv2.x) : 0.0;
            const double g1 = cok1 ? cpf * pv2.y - cvf * (vv2.y + aa * pv2.y) : 0.0;
            __syncthreads();  // every wave has read P's row v
            // the later rows: P_k -= lr (a_k . a_v) g, |p_k|^2 afresh; row v holds G
            double sq[2] = {0.0, 0.0};
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int k = w + 4 * h;
                if (k == v && cok0) *(double2*)(P + k * LW + c0) = double2{g0, g1};
                if (k > v && k < cc && cok0) {
                    const double gl = -lr * Gm[k * R + v];
                    double2 x = *(const double2*)(P + k * LW + c0);
                    x.x = fma(gl, g0, x.x);
                    x.y = fma(gl, g1, x.y);
                    *(double2*)(P + k * LW + c0) = x;
                    sq[h] = x.x * x.x + x.y * x.y;
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
                if (cok0) dst[c0] = (T)P[v * LW + c0];
                if (cok1) dst[c0 + 1] = (T)P[v * LW + c0 + 1];
            }
            if (tid == 0) {
                vflag[b + v] = 1;
                if (sl < 0) bf.relpair_stamp[r] = bf.stamp;
            }
        }
        if (cok0) {
            for (int j = w; j < n; j += NW) {
                double2 x = *(const double2*)(Wc + j * LW + c0);
                for (uint32_t mm = vmask; mm; mm &= mm - 1) {
                    const int v = __builtin_ctz(mm);
                    const double al = -lr * A[v * LW + j];
                    const double2 g = *(const double2*)(P + v * LW + c0);
                    x.x = fma(al, g.x, x.x);
                    x.y = fma(al, g.y, x.y);
                }
                *(double2*)(Wc + j * LW + c0) = x;
            }
        }
    };

    // windows of kGenWin samples up to the last active one; the last update's slots wait for the tail
    for (int wq = 0; wq <= klq; wq += kGenWin) {
        const int q = wq + tid;
        int kk = -1, ents[4] = {-1, -1, -1, -1};
        uint32_t keep = 0;
        if (tid < kGenWin && q <= klq) {
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
                const double2 x = cok0 ? *(const double2*)(Wc + j * LW + c0) : double2{0.0, 0.0};
                const double len = sqrt(wave_sum(x.x * x.x + x.y * x.y));
                if (cok0) *(double2*)(Wc + j * LW + c0) = double2{x.x / len, x.y / len};
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
    // the relation's matrix back, then transposed in place (Wt[i][j] = W[j][i]: the
    // records' lanes own rows j and read Wt's rows i, consecutive lanes consecutive j)
    for (int idx = tid; idx < n * n; idx += NT) {
        const int j = idx / n, i = idx % n;
        bf.W[((int64_t)r * n + j) * ld + i] = (T)Wc[j * LW + i];
    }
    __syncthreads();
    for (int idx = tid; idx < n * n; idx += NT) {
        const int j = idx / n, i = idx % n;
        if (j < i) {
            const double x = Wc[j * LW + i];
            Wc[j * LW + i] = Wc[i * LW + j];
            Wc[i * LW + j] = x;
        }
    }
    __syncthreads();
    // the pair records da = -lr W G with the final matrix: the relation's violator
    // slots (pflag) of its active samples and (entity'[r], r) when stamped; a wave a
    // record, lane l the rows 2 l, 2 l + 1 (G through the wave's LDS row); windows of
    // kGenWin samples, the list in pe / ps (4 kGenWin + 1 <= 2 kGenPairs entries)
    const bool relrec = r < a.ne && bf.relpair_stamp[r] == bf.stamp;
    double* gw = A + w * LW;  // (A is free: a G row a wave)
    for (int wq = 0; wq < ns; wq += kGenWin) {
        const int q = wq + tid;
        int kk = -1;
        uint32_t fl = 0;
        if (tid < kGenWin && q < ns) {
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
        for (int m = w; m < tot; m += NW) {
            const int sl = pe[m];
            T* row = sl >= 0 ? bf.pair + (int64_t)sl * ld : bf.relpair + (int64_t)r * ld;
            if (cok0) gw[c0] = (double)row[c0];
            if (cok1) gw[c0 + 1] = (double)row[c0 + 1];
            wave_lds_sync();
            double d0 = 0.0, d1 = 0.0;
            if (cok0) {
                for (int i = 0; i < n; ++i) {
                    const double2 wt = *(const double2*)(Wc + i * LW + c0);  // W[c0][i], W[c0 + 1][i]
                    const double gi = gw[i];
                    d0 = fma(wt.x, gi, d0);
                    d1 = fma(wt.y, gi, d1);
                }
            }
            wave_lds_sync();
            if (cok0) row[c0] = (T)(-lr * d0);
            if (cok1) row[c0 + 1] = (T)(-lr * d1);
        }
        __syncthreads();  // the list is rebuilt by the next window
    }
}

}  // namespace kb2e
