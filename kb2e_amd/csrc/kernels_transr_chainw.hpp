// kernels_transr_chainw.hpp -- transRNorm of the PARALLEL TransR schedule per
// relation, pair by pair, for every width up to 112 (FP64; the n <= 64
// matrix-core path keeps kernels_transr_seq.hpp / kernels_transr_pipe.hpp).
// The same model as those kernels (oracle/parallel.py transr_constraint,
// cons="chunk1"; the reference's calls are transr/trainer.cpp:185-187 on the
// loop at :35-64): the relation's pairs (h', r), (t', r) of its active updates
// in (sample, update, role) order, first occurrences per relation per batch,
// each checked against the matrix the earlier violators left; per violator v
// (|p_v|^2 > 1, p_v = a_v W_c) the rounds of the loop in closed form along p
// and V = p K0 (K0 = W'^T W', made at the relation's first violator;
// transr_norm_rounds) give g, and W_c -= lr a_v^T g.  The pairs of the
// relation's last update and (entity'[r], r) come last, after W_c's rows are
// renormalised when anything moved; pair records G become da = -lr W G with the
// final matrix (transr_cons_da_wide_kernel); the entity pass splits pre / post
// deltas around the unit norm (bf.last_renorm).
//
// Why a second kernel.  The n <= 64 kernels keep K0's column c in lane c of one
// wave (4 KS registers) and take their pair lists from the matrix-core gradient
// kernel.  At n = 100 (K5, BASELINE configs[4]) a column of K0 is 100 doubles,
// W_c alone is 100 KB of LDS, and the VALU tile path has no compacted pair lists.
// Here, eight waves a workgroup (one workgroup a CU: the LDS):
//  * the workgroup is one relation of the batch, the most frequent relations
//    first; it finds the relation's last active sample, then builds its pair list
//    in windows of 512 samples (a thread a sample: its four slots, first
//    occurrences by the per-batch (relation, entity) table, a block scan for the
//    positions); the last update's slots are held back for the tail, so the tail
//    is exact however many windows the relation spans;
//  * K0 lives in registers spread over the waves: thread t < 4 NP holds rows
//    [h NP/4, (h + 1) NP/4) of column c = t >> 2 (h = t & 3), so V = p K0 is NP/4
//    FMAs a thread (p broadcast from LDS) and two quad DPP adds; the W_c update
//    of a violator is the same layout (NP/4 rows of one column a thread, in
//    registers, eight rows at a time);
//  * per chunk of 16 pairs P = A W_c (NB column tiles) and the Gram matrix A A^T
//    (one tile) on the matrix cores, a tile a wave (NB + 1 <= 8), NP / 4 k-steps
//    over zero padding; the walk is workgroup-wide, three barriers a violator
//    (the p.V / V.V partial sums, g, then the later pairs'
//    P_j -= lr (a_j . a_v) g and |p_j|^2 afresh);
//  * the next chunk's entity rows are loaded into registers while the current
//    chunk is walked.
#pragma once

#include "kernels_transr_seq.hpp"

namespace kb2e {

constexpr int kWideThreads = 512;     // eight waves
constexpr int kWideWaves = kWideThreads / 64;
constexpr int kWideRows = 16;         // pairs a chunk: one MFMA row tile
constexpr int kWideWin = kWideThreads;  // samples a window (a thread each)
constexpr int kWidePairs = 4 * kWideWin;

__host__ __device__ constexpr int wide_nb(int n) { return (n + 15) / 16; }

// LDS bytes: W_c [NP][LW] | A [R][LW] | P [R][LW] | Gram [R][R + 1] | qpart [NB][R] |
// red [8][2] ; ints: pair entities, slots [kWidePairs] | wave sums [8] | misc [8] ; vio flags [kWidePairs]
// (W_c and A zero padded to NP x NP and R x NP: the MFMA k-loop runs NP / 4 steps, no guards)
__host__ __device__ constexpr size_t chainw_lds(int n) {
    return sizeof(double) * ((size_t)(16 * wide_nb(n)) * (16 * wide_nb(n) + 2) +
                             2 * (size_t)kWideRows * (16 * wide_nb(n) + 2) + (size_t)kWideRows * (kWideRows + 1) +
                             (size_t)wide_nb(n) * kWideRows + 2 * kWideWaves) +
           sizeof(int) * (2 * (size_t)kWidePairs + kWideWaves + 8) + (size_t)kWidePairs;
}

// the sum over the four lanes of a quad (lanes 4q .. 4q + 3), in every lane of it
__device__ __forceinline__ double quad_sum(double x) {
    x += dpp_mov<0xB1>(x);  // quad_perm [1,0,3,2]
    return x + dpp_mov<0x4E>(x);  // quad_perm [2,3,0,1]
}

template <int NB>
__global__ __launch_bounds__(kWideThreads) void transr_cons_chain_wide_kernel(RParArgs a, RParBufs<double> bf) {
    using T = double;
    using M = Mfma16<T>;
    constexpr int NP = 16 * NB, LW = NP + 2, R = kWideRows, LG = R + 1, KQ = NP / 4;
    constexpr int NT = kWideThreads, NW = kWideWaves;
    static_assert(NB + 1 <= NW, "a tile a wave");
    // block b takes the b-th most frequent relation, so the long chains of the hot
    // relations start first (a hot relation dispatched late would add its wait to the
    // batch); its segment in this batch's index by binary search over the batch's
    // relation segments (sorted by row), none: nothing to do
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
    const int tid = threadIdx.x, w = tid >> 6, l = lane_id(), kq = l >> 4, l16 = l & 15;
    const int c = tid >> 2, h = tid & 3;  // K0 / V / W-update layout: column c, quarter h of the rows
    const bool colt = c < NP;             // (4 NP <= 512 threads)
    const T lr = (T)a.lr;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    T* Wc = (T*)smem;            // [NP][LW] W'_r as the chain found it, then K0 = W'^T W' (the working matrix is in registers)
    T* A = Wc + NP * LW;         // [R][LW] the chunk's entity rows
    T* P = A + R * LW;           // [R][LW] projections; the violators' rows then hold G
    T* Gm = P + R * LW;          // [R][LG]
    T* qpart = Gm + R * LG;      // [NB][R]
    T* red = qpart + NB * R;     // [NW][2]
    int* pe = (int*)(red + 2 * NW);  // [kWidePairs]
    int* ps = pe + kWidePairs;   // [kWidePairs]
    int* wsum = ps + kWidePairs; // [NW]
    int* misc = wsum + NW;       // [8]
    uint8_t* vflag = (uint8_t*)(misc + 8);  // [kWidePairs]
    const long long ck0 = clock64();
    unsigned long long n_chunks = 0, n_vio = 0, n_rounds = 0, max_m = 0;
    // KB2E_RPAR_STATS: cycles of the phases on thread 0 (g_seq_stats 8..23; relations of
    // >= 200 chunks also 24..39, their chunks / count / violators 40..42): 0 prologue,
    // 1 window list, 2 rows + A barrier, 3 P / Gram MFMA + B1, 4 |p|^2 + K0, 5 V + sums,
    // 6 barrier (1), 7 rounds + g, 8 barrier (2), 9 later pairs, 10 barrier (3), 11 records +
    // W update, 12 end-of-chunk barrier, 13 window flags, 14 tail, 15 write-back
    __shared__ unsigned long long ph[16];  // (in LDS: sixteen 64-bit registers are too dear here)
    if (tid < 16) ph[tid] = 0;
    long long tq = ck0;
    auto tick = [&](int k) {
        if (bf.stats && tid == 0) {
            const long long t = clock64();
            ph[k] += (unsigned long long)(t - tq);
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
        __syncthreads();  // (read by every thread before the next round's atomics)
        if (found >= 0 || qb <= 0) break;
    }
    const int klq = misc[0];
    if (klq < 0) return;  // no active update: the gradient step left the relation alone
    const int kl = a.kl.kk_of(a.keys[p0 + 2 * klq]);
    const bool has_rel = r < a.ne && ptab_first(a, r, r) < 0;  // (entity'[r], r), transr/trainer.cpp:187

    // W'_r, zero padded to NP x NP
    for (int idx = tid; idx < NP * NP; idx += NT) {
        const int j = idx / NP, i = idx % NP;
        Wc[j * LW + i] = (j < n && i < n) ? bf.W[((int64_t)r * n + j) * ld + i] : T(0);
    }
    bool have_k0 = false, changed = false;
    // The working matrix W_c in registers, as the MFMA B fragments of the projection
    // tiles: wave w < NB, lane (kq, l16) holds W_c[4 s + kq][16 w + l16], s < NP / 4.
    // The P tiles read no B operand from LDS, and a violator's W_c -= lr a^T g is
    // register FMAs (its a and g rows broadcast from LDS) instead of an LDS
    // read-modify-write of the whole matrix.
    const bool wown = w < NB;
    const int wcol = 16 * w + l16;
    __syncthreads();  // (W' in LDS)
    T bW[NP / 4];
#pragma unroll
    for (int q = 0; q < NP / 4; ++q) bW[q] = wown ? Wc[(4 * q + kq) * LW + wcol] : T(0);
    tick(0);

    // the chunk's rows: R x NP elements, RPT a thread, into registers (every load is
    // issued, padding zeroed when stored: no register written under a branch while a
    // load into it is in flight)
    constexpr int RPT = (R * NP + NT - 1) / NT;
    T rows[RPT];
    uint32_t rows_ok = 0;
    auto load_rows = [&](int b, int e) {
        int ent[RPT];
#pragma unroll
        for (int q = 0; q < RPT; ++q) {
            const int idx = tid + q * NT;
            const int f = b + idx / NP;
            ent[q] = idx < R * NP && f < e ? pe[f] : -1;
        }
        rows_ok = 0;
#pragma unroll
        for (int q = 0; q < RPT; ++q) {
            const int j = (tid + q * NT) % NP;
            const bool ok = ent[q] >= 0 && j < n;
            rows[q] = bf.ent[ok ? (uint32_t)ent[q] * (uint32_t)ld + (uint32_t)j : 0u];
            rows_ok |= (ok ? 1u : 0u) << q;
        }
    };
    auto store_rows = [&]() {
#pragma unroll
        for (int q = 0; q < RPT; ++q) {
            const int idx = tid + q * NT;
            if (idx < R * NP) A[(idx / NP) * LW + idx % NP] = ((rows_ok >> q) & 1) ? rows[q] : T(0);
        }
    };

    // One chunk: pairs [b, b + cc) of the LDS list, rows already in `rows`; the rows of
    // [nb, ne) are loaded while it is walked.  Leaves W_c updated and vflag set.
    auto chunk = [&](int b, int cc, int nb, int ne) {
        ++n_chunks;
        store_rows();
        __syncthreads();  // A (and W_c) ready
        if (nb < ne) load_rows(nb, ne);
        tick(2);
        // P = A W_c (NB column tiles, B from the registers) and the Gram tile A A^T
        // (its B operand is the A operand itself), a tile a wave, NP / 4 k-steps over
        // the zero padding: straight-line code, no per-step guards
        if (w <= NB) {
            const bool gram = w == NB;
            const T* ap = A + l16 * LW + kq;
            typename M::acc_t acc = {T(0), T(0), T(0), T(0)};
            T av[NP / 4];
#pragma unroll
            for (int q = 0; q < NP / 4; ++q) av[q] = ap[4 * q];
            if (gram) {
#pragma unroll
                for (int q = 0; q < NP / 4; ++q) acc = M::mma(av[q], av[q], acc);
            } else {
#pragma unroll
                for (int q = 0; q < NP / 4; ++q) acc = M::mma(av[q], bW[q], acc);
            }
            if (gram) {
#pragma unroll
                for (int q = 0; q < 4; ++q) Gm[(kq + 4 * q) * LG + l16] = acc[q];
            } else {
                T sp[4];
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    P[(kq + 4 * q) * LW + w * 16 + l16] = acc[q];
                    sp[q] = acc[q] * acc[q];
                }
                row16_sums<T, 4>(sp);
                if (l16 == 0) {
#pragma unroll
                    for (int q = 0; q < 4; ++q) qpart[w * R + kq + 4 * q] = sp[q];
                }
            }
        }
        __syncthreads();  // P, Gram, |p|^2 partials
        tick(3);
        const int j = l16;  // |p_j|^2 of pair j in lanes j, j + 16, ... of every wave
        T qj = T(0);
        {
            T qv[NB];
#pragma unroll
            for (int v = 0; v < NB; ++v) qv[v] = qpart[v * R + j];
#pragma unroll
            for (int v = 0; v < NB; ++v) qj += qv[v];
            if (j >= cc) qj = T(0);
        }
        uint32_t cand = (uint32_t)__ballot(l < R && j < cc && qj > T(1));
        if (!cand) {
            tick(4);
            return;
        }
        if (!have_k0) {  // K0 = W'^T W' in place of W' (LDS): thread (c, h) rows of quarter h of column c
            have_k0 = true;
            T k0[KQ];
#pragma unroll
            for (int i = 0; i < KQ; ++i) k0[i] = T(0);
            if (colt) {
                for (int jr = 0; jr < n; ++jr) {
                    const T wc = Wc[jr * LW + c];
                    const double2* wrow = (const double2*)(Wc + jr * LW + h * KQ);
#pragma unroll
                    for (int i2 = 0; i2 < KQ / 2; ++i2) {
                        const double2 x = wrow[i2];
                        k0[2 * i2] = fma(x.x, wc, k0[2 * i2]);
                        k0[2 * i2 + 1] = fma(x.y, wc, k0[2 * i2 + 1]);
                    }
                }
            }
            __syncthreads();  // every thread done with W'
            if (colt) {
#pragma unroll
                for (int i = 0; i < KQ; ++i) Wc[(h * KQ + i) * LW + c] = k0[i];
            }
            __syncthreads();
        }
        tick(4);
        const T eps = T(2) * lr;
        uint32_t vmask = 0;
        for (int cursor = 0;;) {
            cand &= ~((1u << cursor) - 1);
            if (!cand) break;
            const int v = __builtin_ctz(cand);
            // V_c = sum_i p_v[i] K0[i][c] (K0 in LDS), the quarters of the rows in the lanes of a quad
            T V = T(0), pv = T(0);
            if (colt) {
                T acc4[4] = {T(0), T(0), T(0), T(0)};
                const double2* prow = (const double2*)(P + v * LW + h * KQ);
                const T* kcol = Wc + h * KQ * LW + c;
                pv = P[v * LW + c];
#pragma unroll
                for (int i0 = 0; i0 < KQ / 2; i0 += NB) {  // NB double2 + 2 NB K0 loads in flight a block
                    double2 pr[NB];
                    T kk[2 * NB];
#pragma unroll
                    for (int i2 = 0; i2 < NB; ++i2) {
                        pr[i2] = prow[i0 + i2];
                        kk[2 * i2] = kcol[(2 * (i0 + i2)) * LW];
                        kk[2 * i2 + 1] = kcol[(2 * (i0 + i2) + 1) * LW];
                    }
#pragma unroll
                    for (int i2 = 0; i2 < NB; ++i2) {
                        const int i = 2 * (i0 + i2);
                        acc4[i & 3] = fma(pr[i2].x, kk[2 * i2], acc4[i & 3]);
                        acc4[(i + 1) & 3] = fma(pr[i2].y, kk[2 * i2 + 1], acc4[(i + 1) & 3]);
                    }
                }
                V = (acc4[0] + acc4[1]) + (acc4[2] + acc4[3]);
            }
            V = quad_sum(V);
            T s2[2] = {colt && h == 0 ? pv * V : T(0), colt && h == 0 ? V * V : T(0)};
            wave_sums<T, 2>(s2);
            if (l == 0) {
                red[2 * w] = s2[0];
                red[2 * w + 1] = s2[1];
            }
            tick(5);
            __syncthreads();  // (1) the partial sums
            tick(6);
            T pV = T(0), VV = T(0);
            {
                T rr[2 * NW];
#pragma unroll
                for (int k = 0; k < 2 * NW; ++k) rr[k] = red[k];
#pragma unroll
                for (int k = 0; k < NW; ++k) {
                    pV += rr[2 * k];
                    VV += rr[2 * k + 1];
                }
            }
            const T pp = readlane_f(qj, v);
            const T aa = Gm[v * LG + v];  // |a_v|^2
            const T pvd = pV + aa * pp, vvd = VV + T(2) * aa * pV + aa * aa * pp;
            const T kappa = pvd / pp;
            const T w2t = vvd - kappa * pvd;
            const T w2 = w2t > T(0) ? w2t : T(0);
            const T rho = T(1) - eps * kappa;
            T S0, S1;
            const int m = transr_rounds_violator(pp, w2, eps, rho, S0, S1);
            n_rounds += (unsigned long long)m;
            max_m = max_m > (unsigned long long)m ? max_m : (unsigned long long)m;
            const T cpf = T(2) * (S0 + eps * S1 * kappa), cvf = T(2) * eps * S1;
            if (colt && h == 0) P[v * LW + c] = c < n ? cpf * pv - cvf * (V + aa * pv) : T(0);
            tick(7);
            __syncthreads();  // (2) g in P's row v
            tick(8);
            if (tid < 16 * R) {  // the later pairs: P[jr] -= lr (a_jr . a_v) g, |p_jr|^2 afresh (16 lanes a row)
                const int jr = tid >> 4, s16 = tid & 15;
                const bool later = jr > v && jr < cc;
                if (later) {
                    const T gl = -lr * Gm[jr * LG + v];
                    T x[NB], g[NB];
#pragma unroll
                    for (int k = 0; k < NB; ++k) {
                        x[k] = P[jr * LW + s16 + 16 * k];
                        g[k] = P[v * LW + s16 + 16 * k];
                    }
                    T sq = T(0);
#pragma unroll
                    for (int k = 0; k < NB; ++k) {
                        x[k] = fma(gl, g[k], x[k]);
                        P[jr * LW + s16 + 16 * k] = x[k];
                        sq = fma(x[k], x[k], sq);
                    }
                    T sv[1] = {sq};
                    row16_sums<T, 1>(sv);
                    if (s16 == 0) qpart[jr] = sv[0];  // (qpart row 0 is free once read)
                }
            }
            tick(9);
            __syncthreads();  // (3) the new |p_j|^2
            if (j > v && j < cc) qj = qpart[j];
            cand = (uint32_t)__ballot(l < R && j < cc && j > v && qj > T(1));
            vmask |= 1u << v;
            cursor = v + 1;
            ++n_vio;
            tick(10);
        }
        // the violators' records G, flags, and W_c[k][c] -= lr sum_v a_v[k] G_v[c]
        changed = true;
        for (uint32_t mm = vmask; mm; mm &= mm - 1) {
            const int v = __builtin_ctz(mm);
            const int sl = ps[b + v];
            if (colt && h == 0 && c < n) {
                T* dst = sl >= 0 ? bf.pair + (int64_t)sl * ld : bf.relpair + (int64_t)r * ld;
                dst[c] = P[v * LW + c];
            }
            if (tid == 0) {
                vflag[b + v] = 1;
                if (sl < 0) bf.relpair_stamp[r] = bf.stamp;
            }
        }
        if (wown) {  // W_c[4 s + kq][wcol] -= lr a_v[4 s + kq] g_v[wcol], in the fragments
            for (uint32_t mm = vmask; mm; mm &= mm - 1) {
                const int v = __builtin_ctz(mm);
                const T gl = -lr * P[v * LW + wcol];
                const T* av = A + v * LW + kq;
#pragma unroll
                for (int q = 0; q < NP / 4; ++q) bW[q] = fma(av[4 * q], gl, bW[q]);
            }
        }
        tick(11);
    };

    // windows of NT samples up to the last active one; the last update's slots wait for the tail
    for (int wq = 0; wq <= klq; wq += kWideWin) {
        const int q = wq + tid;
        int kk = -1, ents[4] = {-1, -1, -1, -1};
        uint32_t keep = 0;
        if (q <= klq) {
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
        tick(1);
        if (npw > 0) {
            load_rows(0, min(R, npw));
            for (int b = 0; b < npw; b += R) {
                const int e = min(b + R, npw);
                chunk(b, e - b, e, min(e + R, npw));
                __syncthreads();  // W_c, and A / P free for the next chunk
                tick(12);
            }
        }
        // the flags of the window's slots (the tail's wait)
        if (kk >= 0) {
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
        tick(13);
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
        if (changed) {  // the last update's unit rows (transr/trainer.cpp:178-180)
            // row 4 s + kq: its 16 columns of tile w summed in the DPP row, the tiles in
            // LDS (qpart's and red's space is free here: P [R][LW] >= NB x NP)
            T* rs = P;  // [NB][NP] row partials
#pragma unroll
            for (int q = 0; q < NP / 4; ++q) {
                T x[1] = {bW[q] * bW[q]};
                row16_sums<T, 1>(x);
                if (wown && l16 == 0) rs[w * NP + 4 * q + kq] = x[0];
            }
            __syncthreads();
            if (wown) {
#pragma unroll
                for (int q = 0; q < NP / 4; ++q) {
                    const int jr = 4 * q + kq;
                    T ss = rs[jr];
                    for (int v = 1; v < NB; ++v) ss += rs[v * NP + jr];
                    if (jr < n) bW[q] = bW[q] / sqrt(ss);
                }
            }
        }
        __syncthreads();  // the tail list and W_c
        load_rows(0, ntail);
        chunk(0, ntail, ntail, ntail);
        __syncthreads();
    }
    if (tid == 0) {
        int pos = 0;
        for (int k = 0; k < 2; ++k) bf.pflag[kl * 4 + 2 + k] = ((tkeep >> k) & 1) ? vflag[pos++] : 0;
    }
    tick(14);
    // the relation's matrix back, from the fragments
    if (wown && wcol < n) {
#pragma unroll
        for (int q = 0; q < NP / 4; ++q)
            if (4 * q + kq < n) bf.W[((int64_t)r * n + 4 * q + kq) * ld + wcol] = bW[q];
    }
    if (bf.stats && tid == 0) {
        const unsigned long long cyc = (unsigned long long)(clock64() - ck0);
        atomicAdd(&g_seq_stats[0], 1ull);
        atomicAdd(&g_seq_stats[1], n_chunks);
        atomicAdd(&g_seq_stats[2], n_vio);
        atomicAdd(&g_seq_stats[3], n_rounds);
        atomicAdd(&g_seq_stats[4], cyc);
        atomicMax(&g_seq_stats[5], cyc);
        atomicMax(&g_seq_stats[6], n_chunks);
        atomicMax(&g_seq_stats[7], max_m);
        tick(15);
        for (int k = 0; k < 16; ++k) atomicAdd(&g_seq_stats[8 + k], ph[k]);
        if (n_chunks >= 200) {  // the hot relations alone
            for (int k = 0; k < 16; ++k) atomicAdd(&g_seq_stats[24 + k], ph[k]);
            atomicAdd(&g_seq_stats[40], n_chunks);
            atomicAdd(&g_seq_stats[41], 1ull);
            atomicAdd(&g_seq_stats[42], n_vio);
        }
    }
}

// The pair records per relation (n <= 128): a workgroup per relation of the batch
// stages its final matrix once, transposed, in LDS (Wt[i][j] = W[j][i]) and turns
// every record of the relation into da = -lr W G -- the violators' slots (pflag)
// of its active samples, found by a thread a sample, and (entity'[r], r) when
// stamped.  transr_cons_da_wide_kernel below reads the whole matrix from L2 for
// every record instead (K5: ~88k records a batch x 80 KB).  A wave a record, two
// elements j = 2l, 2l + 1 a lane: 16-byte row-pair reads of Wt, G_i as broadcasts.
constexpr int kDaRelThreads = 1024;

// The records of relation r (its samples [p0, p0 + 2 ns) of the batch's keys) with
// its final matrix transposed in LDS (Wt [n][LT], LT even >= n, columns past n
// never read into results); gb: [NT / 64][LT] doubles, list: [4 NT + 1] ints (the
// window's slots and the relation record), wsum: [NT / 64] ints.  Ends with a barrier.
template <int NT>
__device__ __forceinline__ void relation_records(const RParArgs& a, const RParBufs<double>& bf, int r, int p0,
                                                 int ns, const double* Wt, int LT, double* gb, int* list,
                                                 int* wsum) {
    using T = double;
    constexpr int NW = NT / 64;
    const int n = a.n, ld = a.ld;
    const int tid = threadIdx.x, w = tid >> 6, l = lane_id();
    const bool relrec = r < a.ne && bf.relpair_stamp[r] == bf.stamp;
    const T lr = (T)a.lr;
    for (int wq = 0; wq < ns; wq += NT) {
        const int q = wq + tid;
        int kk = -1;
        uint32_t keep = 0;
        if (q < ns) {
            kk = a.kl.kk_of(a.keys[p0 + 2 * q]);
            if (a.act[kk]) {
                const uchar4 f = *(const uchar4*)(bf.pflag + (int64_t)kk * 4);
                keep = (f.x ? 1u : 0u) | (f.y ? 2u : 0u) | (f.z ? 4u : 0u) | (f.w ? 8u : 0u);
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
        int off = 0, tot = 0;
#pragma unroll
        for (int k = 0; k < NW; ++k) {
            const int ws = wsum[k];
            off += k < w ? ws : 0;
            tot += ws;
        }
        {
            int pos = off + x - cnt;
#pragma unroll
            for (int k = 0; k < 4; ++k)
                if ((keep >> k) & 1) list[pos++] = kk * 4 + k;
        }
        if (wq == 0 && relrec) {
            if (tid == 0) list[tot] = -2;
            ++tot;
        }
        __syncthreads();  // the list
        // a wave's records one after another, the next one's G row loaded while the
        // current one is made (a hot relation holds hundreds a batch)
        auto rec_row = [&](int m) {
            const int sl = list[m];
            return sl >= 0 ? bf.pair + (int64_t)sl * ld : bf.relpair + (int64_t)r * ld;
        };
        T gn[2] = {T(0), T(0)};
        if (w < tot) lane_pair_load(rec_row(w), n, gn);
        for (int m = w; m < tot; m += NW) {
            T* row = rec_row(m);
            T g[2] = {gn[0], gn[1]};
            if (m + NW < tot) lane_pair_load(rec_row(m + NW), n, gn);
            T* gw = gb + w * LT;
            lane_pair_store(gw, n, g);  // (this wave's row: in-order LDS, no barrier)
            T d0[4] = {T(0), T(0), T(0), T(0)}, d1[4] = {T(0), T(0), T(0), T(0)};
            const int jl = 2 * l < n ? 2 * l : 0;
            int i = 0;
            for (; i + 4 <= n; i += 4) {
                double2 wv[4];
                T gi[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    wv[u] = *(const double2*)(Wt + (i + u) * LT + jl);
                    gi[u] = gw[i + u];
                }
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    d0[u] = fma(wv[u].x, gi[u], d0[u]);
                    d1[u] = fma(wv[u].y, gi[u], d1[u]);
                }
            }
            for (; i < n; ++i) {
                const double2 wv = *(const double2*)(Wt + i * LT + jl);
                d0[0] = fma(wv.x, gw[i], d0[0]);
                d1[0] = fma(wv.y, gw[i], d1[0]);
            }
            const T out[2] = {-lr * ((d0[0] + d0[1]) + (d0[2] + d0[3])), -lr * ((d1[0] + d1[1]) + (d1[2] + d1[3]))};
            lane_pair_store(row, n, out);
        }
        __syncthreads();  // the list is rebuilt by the next window
    }
}

__host__ __device__ constexpr size_t da_rel_lds(int n) {
    return sizeof(double) * ((size_t)n * ((n + 1) & ~1) + (size_t)(kDaRelThreads / 64) * ((n + 1) & ~1)) +
           sizeof(int) * ((size_t)4 * kDaRelThreads + 1 + kDaRelThreads / 64 + 8);
}

// A workgroup per relation segment of the batch (no search: the grid runs over the
// batch's segments), the final matrix staged once, transposed.
static __attribute__((unused)) __global__ __launch_bounds__(kDaRelThreads) void transr_cons_da_rel_kernel(
    RParArgs a, RParBufs<double> bf) {
    using T = double;
    const int s = a.rel_begin[a.batch] + blockIdx.x;
    if (s >= a.batch_seg[a.batch + 1]) return;
    const int r = a.seg_row[s] - a.ne;
    const int n = a.n, ld = a.ld, LT = (n + 1) & ~1;
    const int p0 = a.seg_start[s], ns = (a.seg_start[s + 1] - p0) / 2;
    constexpr int NW = kDaRelThreads / 64;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    T* Wt = (T*)smem;                  // [n][LT]
    T* gb = Wt + n * LT;               // [NW][LT] a wave's G row
    int* list = (int*)(gb + NW * LT);  // [4 kDaRelThreads + 1]
    int* wsum = list + 4 * kDaRelThreads + 1;
    const T* Wg = bf.W + (int64_t)r * n * ld;
#pragma unroll 4
    for (int idx = threadIdx.x; idx < n * n; idx += kDaRelThreads) {
        const int j = idx / n, i = idx % n;
        Wt[i * LT + j] = Wg[(int64_t)j * ld + i];
    }
    __syncthreads();
    relation_records<kDaRelThreads>(a, bf, r, p0, ns, Wt, LT, gb, list, wsum);
}

}  // namespace kb2e
