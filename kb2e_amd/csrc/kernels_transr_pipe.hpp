// kernels_transr_pipe.hpp -- the per-relation sequential transRNorm of the
// PARALLEL TransR schedule (kernels_transr_seq.hpp explains the semantics:
// every pair against the matrix the relation's earlier pairs left,
// transr/trainer.cpp:35-64, :185-187; CPU model oracle/parallel.py
// transr_constraint, cons="chunk1"), software-pipelined across chunks.
//
// transr_cons_chain_kernel spends a chunk of 32 pairs as: all four waves make
// P = A W_c and the Gram matrix (MFMA), barrier, wave 0 walks the violators,
// barrier, all waves fold the violators into W_c, barrier -- the projections
// of a chunk wait for the previous chunk's walk.  Here the three other waves
// make the NEXT chunk's projections while wave 0 walks the current one:
//   X_{k+1} = A_{k+1} W_{k-1}                  (the matrix before chunk k's walk)
//   C       = A_{k+1} A_k^T                    (cross Gram, next x current)
//   P_{k+1} = X_{k+1} - lr C[:, vio_k] G_k     (chunk k's shrinks, W_k = W_{k-1} - lr A_k^T G_k)
// so after the walk only a rank-|vio_k| correction and the next chunk's |p|^2
// sit between two walks.  The working matrix W_c lives in registers of waves
// 1-3 as the MFMA B fragments of their column slices (slice cb on wave
// 1 + cb % 3), so X's tiles read no B operand from LDS, and chunk k's update
// W_c -= lr A_k^T G_k is made by waves 1-3 at the start of chunk k+1, while wave
// 0 walks chunk k+1, instead of between the two walks (a wave touches only its
// own slices' columns of the P buffers, so reading G_k and writing X_{k+2} into
// the same buffer need no barrier); the walker writes each violator's pair record
// G to global memory as it publishes it, off the helpers' per-chunk work.  The walk keeps the chunk's projection
// rows in registers (lane j: half l >> 5 of row j & 31), so a violator's
// rank-1 move of the later rows is FMAs on registers with the violator's G row
// read as LDS broadcasts.  The relation's last-update chunk starts after W_c's
// rows are renormalised: its projections are then made afresh (all waves).
#pragma once

#include "kernels_transr_cons.hpp"  // pair_sum32
#include "kernels_transr_seq.hpp"

namespace kb2e {

constexpr int kPipeList = 1536;  // pairs of one relation a window (entity and slot lists in LDS)

// LDS (elements of T): W_c [NP][L] (W' for K0; the final matrix for the records) |
// A [3][R][L] | P [2][R][L] (K0 [NP][L] in the prologue) | Gram [2][R][LG] | cross
// Gram [R][LG] | |p|^2 partials [4][R] | row partials [4][NP]; ints: pair entities,
// slots [kPipeList] each | pre [kSeqMaxTiles + 1] | misc [8] | the violators of the
// last two chunks [2][R]
template <typename T>
__host__ __device__ constexpr size_t pipe_lds(int n) {
    return sizeof(T) * ((size_t)rm_np(n) * rm_ld(n) + 5 * (size_t)kChainRows * rm_ld(n) +
                        3 * (size_t)kChainRows * (kChainRows + 1) + 4 * kChainRows + 4 * (size_t)rm_np(n)) +
           sizeof(int) * (size_t)(2 * kPipeList + kSeqMaxTiles + 1 + 8 + 2 * kChainRows);
}

template <typename T, int KS>
__global__ __launch_bounds__(kChainThreads) void transr_cons_pipe_kernel(RParArgs a, RParBufs<T> bf) {
    using M = Mfma16<T>;
    static_assert(sizeof(T) == 8, "the D-row / k-step identity below is the FP64 fragment layout");
    constexpr int NB = (4 * KS + 15) / 16;  // column slices of 16
    constexpr int NP = 16 * NB, L = NP + 2, R = kChainRows, LG = R + 1;
    constexpr int NH = 2 * KS;              // columns of a row half (walk registers; 4 KS >= n, the rest zero)
    constexpr int NSW = (NB + 2) / 3;       // column slices a helper wave owns (slice cb: wave 1 + cb % 3)
    static_assert(2 * R * L >= NP * L, "the K0 image borrows the two P buffers");
    static_assert(NSW * KS <= 4 * KS, "the helpers' slices share the walk's K0 registers");
    const int t0 = a.batch_t0[a.batch], t1 = a.batch_t0[a.batch + 1];
    int g0, r;  // the relation's first tile within the batch
    if (!chain_first_tile(a, t0, t1, g0, r)) return;
    const int n = a.n, ld = a.ld;
    const int w = threadIdx.x >> 6, l = lane_id(), kq = l >> 4, l16 = l & 15;
    const bool mine = w < NB;  // this wave computes a column slice of K0
    const int col = 16 * w + l16;
    const int hw = w - 1;      // helper wave index (waves 1-3)
    const T lr = (T)a.lr;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    T* Wc = (T*)smem;
    T* Abuf = Wc + NP * L;      // [3][R][L] entity rows of chunks k, k+1, k+2
    T* Pbuf = Abuf + 3 * R * L;  // [2][R][L] projections (then the violators' G rows) of chunks k, k+1
    T* Gbuf = Pbuf + 2 * R * L;  // [2][R][LG] Gram matrices A A^T of chunks k, k+1
    T* Cx = Gbuf + 2 * R * LG;   // [R][LG] A_{k+1} A_k^T
    T* qpart = Cx + R * LG;      // [4][R] |p_j|^2 partials of the column slices (next chunk)
    T* rp = qpart + 4 * R;       // [4][NP] row partials of the tail renorm
    int* pe = (int*)(rp + 4 * NP);
    int* ps = pe + kPipeList;
    int* pre = ps + kPipeList;
    int* misc = pre + kSeqMaxTiles + 1;
    int* vlist = misc + 8;  // [2][R] the chunks' violators in order, by chunk parity (misc[2]: the count)
    const long long ck0 = clock64();
    unsigned long long n_chunks = 0, n_vio = 0, n_rounds = 0, max_m = 0;
    __shared__ unsigned long long ph[16];  // (LDS, not sixteen 64-bit registers)
    if (threadIdx.x < 16) ph[threadIdx.x] = 0;
    long long tq = ck0;
    // (phases 12..15 on thread 64, helper wave 1: debt, tiles, helper_sync wait, rows +
    // corrections incl. the wait for the walk's end)
    auto tick = [&](int k) {
        if (bf.stats && threadIdx.x == (k >= 12 || k == 5 ? 64u : 0u)) {
            const long long t = clock64();
            ph[k] += (unsigned long long)(t - tq);
            tq = t;
        }
    };

    // W'_r, zero padded to NP x NP
    for (int idx = threadIdx.x; idx < NP * NP; idx += kChainThreads) {
        const int j = idx / NP, i = idx % NP;
        Wc[j * L + i] = (j < n && i < n) ? bf.W[((int64_t)r * n + j) * ld + i] : T(0);
    }
    // the relation's run of tiles, its last active sample's tile and how many of
    // that tile's pairs belong to the sample's corrupted-triple update (the tail)
    if (w == 0) {
        int run = 0;
        for (int m0 = 0;; m0 += kWave) {
            const int g = g0 + m0 + l;
            const uint64_t b = __ballot(t0 + g < t1 && a.td_r[t0 + g] == r);
            const int k = b == ~0ull ? kWave : __builtin_ctzll(~b);
            run += k;
            if (k < kWave) break;
        }
        const int c0 = bf.cnrows[g0] & 127;
        const int rel = c0 > 0 && bf.cpairs[(int64_t)g0 * 2 * kCPairs + kCPairs + c0 - 1] == -2;
        int kl = -1, gt = -1;
        for (int g = g0 + run - 1; g >= g0 && kl < 0; --g) {
            const int cs = a.td_cnt[t0 + g] & 255;
            const int kk = l < cs ? a.td_kk[(t0 + g) * 8 + l] : -1;
            const uint64_t b = __ballot(kk >= 0 && a.act[kk]);
            if (b) {
                kl = __shfl(kk, 63 - __builtin_clzll(b));
                gt = g;
            }
        }
        int ntail = 0;
        if (gt >= 0) {
            const int cp = bf.cnrows[gt] & 127;
            const int sl = l < cp ? bf.cpairs[(int64_t)gt * 2 * kCPairs + kCPairs + l] : -3;
            ntail = __builtin_popcountll(__ballot(sl >= 0 && (sl >> 1) == kl * 2 + 1));
        }
        if (l == 0) {
            misc[3] = rel;
            misc[4] = gt;
            misc[5] = run;
            misc[6] = ntail;
        }
    }
    __syncthreads();
    const int run = misc[5], has_rel = misc[3], g_tail = misc[4], n_tail = misc[6];
    // K0 = W'^T W' (four waves, MFMA) into the P buffers; wave 0 keeps column l of it,
    // the helper waves their slices of W' (the working matrix) -- in the same registers
    T reg[4 * KS];
    {
        T* K0 = Pbuf;
        if (mine) {
#pragma unroll
            for (int ib = 0; ib < NB; ++ib) {
                typename M::acc_t acc = {T(0), T(0), T(0), T(0)};
                T av[KS], bv[KS];
#pragma unroll
                for (int s = 0; s < KS; ++s) {
                    av[s] = Wc[(4 * s + kq) * L + ib * 16 + l16];
                    bv[s] = Wc[(4 * s + kq) * L + col];
                }
#pragma unroll
                for (int s = 0; s < KS; ++s) acc = M::mma(av[s], bv[s], acc);
#pragma unroll
                for (int qq = 0; qq < 4; ++qq) K0[(ib * 16 + kq + 4 * qq) * L + col] = acc[qq];
            }
        }
        __syncthreads();
        if (w == 0) {
            const int cK = l < NP ? l : 0;
#pragma unroll
            for (int i = 0; i < 4 * KS; ++i) reg[i] = K0[i * L + cK];
        } else {
#pragma unroll
            for (int i = 0; i < 4 * KS; ++i) reg[i] = T(0);
#pragma unroll
            for (int si = 0; si < NSW; ++si) {
                const int cb = hw + 3 * si;
                if (cb < NB) {
#pragma unroll
                    for (int s = 0; s < KS; ++s) reg[si * KS + s] = Wc[(4 * s + kq) * L + cb * 16 + l16];
                }
            }
        }
        if (threadIdx.x == 0) {  // (every thread has read misc[3..6] above)
            misc[5] = 0;   // helper-wave arrivals (helper_sync)
            misc[6] = -1;  // the chunk whose walk is complete
            misc[7] = -1;  // (chunk << 6) | violators published so far
        }
        __syncthreads();  // the P buffers are free again
    }
    bool changed = false;
    int32_t* const vio = bf.vio + (int64_t)g0 * kCPairs;  // the relation's violators (run * kCPairs >= its pairs)
    int nvt = 0;
    // the chunk whose W_c update the helper waves still owe (nv 0: none)
    int pend_nv = 0, pend_par = 0, pend_pc = 0, pend_ka = 0;
    tick(0);

    // one 16 x 16 MFMA tile: rows rt of A (Ar) against rows cb of B (a Gram tile);
    // out[(rt 16 + d) * ldo + cb 16 + l16]
    auto gram_tile = [&](const T* Ar, const T* Bm, int rt, int cb, T* out, int ldo) {
        typename M::acc_t acc = {T(0), T(0), T(0), T(0)};
        T av[KS], bv[KS];
#pragma unroll
        for (int s = 0; s < KS; ++s) {
            av[s] = Ar[(rt * 16 + l16) * L + 4 * s + kq];
            bv[s] = Bm[(cb * 16 + l16) * L + 4 * s + kq];
        }
#pragma unroll
        for (int s = 0; s < KS; ++s) acc = M::mma(av[s], bv[s], acc);
#pragma unroll
        for (int q = 0; q < 4; ++q) out[(rt * 16 + kq + 4 * q) * ldo + cb * 16 + l16] = acc[q];
    };
    // rows rt of A against the helper's column slice si (its W_c fragments)
    auto proj_tile = [&](const T* Ar, int rt, int si, T* out) {
        const int cb = hw + 3 * si;
        typename M::acc_t acc = {T(0), T(0), T(0), T(0)};
        T av[KS];
#pragma unroll
        for (int s = 0; s < KS; ++s) av[s] = Ar[(rt * 16 + l16) * L + 4 * s + kq];
#pragma unroll
        for (int s = 0; s < KS; ++s) acc = M::mma(av[s], reg[si * KS + s], acc);
#pragma unroll
        for (int q = 0; q < 4; ++q) out[(rt * 16 + kq + 4 * q) * L + cb * 16 + l16] = acc[q];
    };
    // rows of chunk [b, e) of the window: the helper waves stage them (R NP / 192
    // elements a thread, in registers), so the walker never waits on them
    constexpr int kHT = kChainThreads - kWave;
    constexpr int kRowsPer = (R * NP + kHT - 1) / kHT;
    static_assert(kRowsPer <= 32, "rows_ok bits");
    const int ht = (int)threadIdx.x - kWave;  // helper thread (w > 0)
    T rows[kRowsPer];
    uint32_t rows_ok = 0;
    auto load_rows = [&](int b, int e) {
        if (w == 0) return;
        int ent[kRowsPer];
#pragma unroll
        for (int q = 0; q < kRowsPer; ++q) {
            const int f = b + (ht + q * kHT) / NP;
            ent[q] = pe[f < kPipeList ? f : kPipeList - 1];
        }
        rows_ok = 0;
#pragma unroll
        for (int q = 0; q < kRowsPer; ++q) {
            const int idx = ht + q * kHT;
            const int k = idx / NP, j = idx % NP;
            const bool ok = idx < R * NP && b + k < e && ent[q] >= 0 && j < n;
            rows[q] = bf.ent[ok ? (uint32_t)ent[q] * (uint32_t)ld + (uint32_t)j : 0u];
            rows_ok |= (ok ? 1u : 0u) << q;
        }
    };
    auto store_rows = [&](int slot) {
        if (w == 0) return;
#pragma unroll
        for (int q = 0; q < kRowsPer; ++q) {
            const int idx = ht + q * kHT;
            if (idx < R * NP) Abuf[slot * R * L + (idx / NP) * L + idx % NP] = ((rows_ok >> q) & 1) ? rows[q] : T(0);
        }
    };
    // The helper waves meet (no s_barrier: the walker runs on): every helper has paid
    // its debt and written its projection / Gram tiles.  Bounded; a timeout sets
    // *bf.err (the host fails loudly) and gives up.
    int hsync_target = 0;
    auto helper_sync = [&]() {
        hsync_target += kChainThreads / kWave - 1;
        // (dbg 32, tests: helper wave 1 never arrives, so the others' waits time out)
        if (l == 0 && !((bf.dbg & 32) && hw == 0))
            __hip_atomic_fetch_add(&misc[5], 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        for (uint32_t sp = 0;
             __hip_atomic_load(&misc[5], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < hsync_target; ++sp) {
            if (sp > (1u << 22)) {
                if (l == 0) __hip_atomic_store(bf.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
    };
    // The next chunk's corrections P_n -= lr C[:, v] g_v, by the helper waves while
    // the walker walks: each violator as soon as the walker publishes it (misc[7]:
    // (chunk << 6) | count, after its G row and vl entry; misc[6] = chunk when the
    // walk ends), so after the walk only its last violators remain.  Then the
    // |p_j|^2 partials (qpart[0], the other slices' partials zero).  Sixteen threads a
    // row (one DPP row), NP / 16 columns each, rows rs, rs + 12, rs + 24.  The same
    // FMAs per element in the same order as correct_q.
    auto correct_inc = [&](T* Pn, int cn, const T* Pc, const T* An, const T* Ac, const int* vl, int ck) {
        constexpr int NE = NP / 16, NPS = (R + 11) / 12;
        const int rs = ht >> 4, cb = (ht & 15) * NE;
        T x[NPS][NE];
#pragma unroll
        for (int p = 0; p < NPS; ++p) {
            const int j = rs + 12 * p;
#pragma unroll
            for (int u = 0; u < NE; ++u) x[p][u] = j < cn ? Pn[j * L + cb + u] : T(0);
        }
        int used = 0;
        for (uint32_t sp = 0;; ++sp) {
            const bool done = __hip_atomic_load(&misc[6], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) == ck;
            const int pw = __hip_atomic_load(&misc[7], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
            const int avail = (pw >> 6) == ck ? (pw & 63) : 0;
            for (; used < avail; ++used) {
                const int v = vl[used];
                T gv[NE], av[NE], d[NPS];
#pragma unroll
                for (int u = 0; u < NE; ++u) {
                    gv[u] = Pc[v * L + cb + u];
                    av[u] = Ac[v * L + cb + u];
                }
#pragma unroll
                for (int p = 0; p < NPS; ++p) {  // a_{k+1}[j] . a_v, this thread's columns
                    const int j = rs + 12 * p;
                    d[p] = T(0);
#pragma unroll
                    for (int u = 0; u < NE; ++u) d[p] = fma(j < R ? An[j * L + cb + u] : T(0), av[u], d[p]);
                }
                row16_sums<T, NPS>(d);
#pragma unroll
                for (int p = 0; p < NPS; ++p) {
                    const int j = rs + 12 * p;
                    if (j < cn) {
                        const T gl = -lr * d[p];
#pragma unroll
                        for (int u = 0; u < NE; ++u) x[p][u] = fma(gl, gv[u], x[p][u]);
                    }
                }
            }
            if (done) break;
            if (sp > (1u << 22)) {
                if (l == 0) __hip_atomic_store(bf.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
        T sq[NPS];
#pragma unroll
        for (int p = 0; p < NPS; ++p) {
            const int j = rs + 12 * p;
            sq[p] = T(0);
            if (j < cn) {
#pragma unroll
                for (int u = 0; u < NE; ++u) {
                    if (used) Pn[j * L + cb + u] = x[p][u];
                    sq[p] = fma(x[p][u], x[p][u], sq[p]);
                }
            }
        }
        row16_sums<T, NPS>(sq);
        if ((ht & 15) == 0) {
#pragma unroll
            for (int p = 0; p < NPS; ++p) {
                const int j = rs + 12 * p;
                if (j < R) {
                    qpart[j] = j < cn ? sq[p] : T(0);
                    for (int v = 1; v < NB; ++v) qpart[v * R + j] = T(0);
                }
            }
        }
    };
    // P_n -= lr C[:, vio] G over the chunk's nv violators (vl; G: their rows of
    // Pc) and the |p_j|^2 partials of the cn rows (qpart[0]; the other slices'
    // partials zero), eight threads a row, NP / 8 columns each (on the VALU: the
    // few violators of a chunk make an MFMA form latency-bound)
    auto correct_q = [&](T* Pn, int cn, int nv, const T* Pc, const int* vl) {
        constexpr int NE = NP / 8;
        const int j = threadIdx.x >> 3, cb = (threadIdx.x & 7) * NE;
        T sq = T(0);
        if (j < cn) {
            T x[NE];
#pragma unroll
            for (int u = 0; u < NE; ++u) x[u] = Pn[j * L + cb + u];
            for (int k = 0; k < nv; ++k) {
                const int v = vl[k];
                const T gl = -lr * Cx[j * LG + v];
#pragma unroll
                for (int u = 0; u < NE; ++u) x[u] = fma(gl, Pc[v * L + cb + u], x[u]);
            }
#pragma unroll
            for (int u = 0; u < NE; ++u) {
                if (nv) Pn[j * L + cb + u] = x[u];
                sq = fma(x[u], x[u], sq);
            }
        }
        // the row's eight lanes: quad perms, then the half-row mirror (DPP, no LDS
        // round trips; the same sums as xor 1, 2, 4)
        sq += dpp_mov<0xB1>(sq);
        sq += dpp_mov<0x4E>(sq);
        sq += dpp_mov<0x141>(sq);
        if ((threadIdx.x & 7) == 0) {
            qpart[j] = j < cn ? sq : T(0);
            for (int v = 1; v < NB; ++v) qpart[v * R + j] = T(0);
        }
    };
    // the helper waves' debt: the pending chunk's W_c -= lr A^T G on their slices
    // (its G rows in P buffer pend_pc, its rows in A slot pend_ka)
    auto apply_pending = [&]() {
        if (w == 0 || pend_nv == 0) return;
        const T* Pp = Pbuf + pend_pc * R * L;
        const T* Ap = Abuf + pend_ka * R * L;
        const int* vl = vlist + pend_par * R;
        // the violators' rows as wave-uniform values (one LDS read for all of them); a
        // violator's a row serves every slice, and the next violator's reads are in flight
        // while this one's FMAs run (per element the same order of updates)
        const int vmine = l < pend_nv ? vl[l] : 0;
        T an[KS], gn[NSW];
        auto ldv = [&](int k) {
            const int v = __builtin_amdgcn_readlane(vmine, k);
#pragma unroll
            for (int s = 0; s < KS; ++s) an[s] = Ap[v * L + 4 * s + kq];
#pragma unroll
            for (int si = 0; si < NSW; ++si) {
                const int cb = hw + 3 * si;
                gn[si] = cb < NB ? -lr * Pp[v * L + cb * 16 + l16] : T(0);
            }
        };
        const int nvu = (bf.dbg & 16) ? 0 : pend_nv;  // (dbg 16, 8: timing experiments)
        if (nvu > 0) ldv(0);
        for (int k = 0; k < nvu; ++k) {
            T ac[KS], gc[NSW];
#pragma unroll
            for (int s = 0; s < KS; ++s) ac[s] = an[s];
#pragma unroll
            for (int si = 0; si < NSW; ++si) gc[si] = gn[si];
            if (k + 1 < nvu) ldv(k + 1);
#pragma unroll
            for (int si = 0; si < NSW; ++si)
                if (hw + 3 * si < NB) {
#pragma unroll
                    for (int s = 0; s < KS; ++s) reg[si * KS + s] = fma(ac[s], gc[si], reg[si * KS + s]);
                }
        }
        // (the pair records G were written by the walker as it published each violator)
    };
    // the relation's last update renormalises W_c's rows before its own pairs'
    // shrinks (transr/trainer.cpp:178-180): row sums of the slices in DPP rows, then
    // LDS; ends with a barrier.  The pending update must be applied first.
    auto renorm = [&] {
        if (w > 0) {
#pragma unroll
            for (int si = 0; si < NSW; ++si) {
                const int cb = hw + 3 * si;
#pragma unroll
                for (int s = 0; s < KS; ++s) {
                    T x[1] = {reg[si * KS + s] * reg[si * KS + s]};
                    row16_sums<T, 1>(x);
                    if (cb < NB && l16 == 0) rp[cb * NP + 4 * s + kq] = x[0];
                }
            }
        }
        __syncthreads();
        if (w > 0) {
#pragma unroll
            for (int si = 0; si < NSW; ++si) {
                if (hw + 3 * si >= NB) continue;
#pragma unroll
                for (int s = 0; s < KS; ++s) {
                    const int jr = 4 * s + kq;
                    T ss = rp[jr];
                    for (int v = 1; v < NB; ++v) ss += rp[v * NP + jr];
                    if (jr < n) reg[si * KS + s] = reg[si * KS + s] / sqrt(ss);
                }
            }
        }
        __syncthreads();
    };
    // projections and Gram matrix of a chunk afresh (the helpers their slices, wave 0
    // the Gram tiles), then the |p|^2 partials (two barriers; the chunk's rows in LDS)
    auto fresh = [&](const T* A, int cc, T* P, T* G) {
        const int nrt = cc > 16 ? 2 : 1;
        if (w > 0) {
#pragma unroll
            for (int si = 0; si < NSW; ++si)
                if (hw + 3 * si < NB)
                    for (int rt = 0; rt < nrt; ++rt) proj_tile(A, rt, si, P);
        } else {
            for (int gi = 0; gi < (nrt == 2 ? 3 : 1); ++gi) gram_tile(A, A, gi == 0 ? 0 : 1, gi == 2 ? 1 : 0, G, LG);
        }
        __syncthreads();
        correct_q(P, cc, 0, nullptr, vlist);
        __syncthreads();
    };

    // pairs a window: the LDS lists, or fewer (bf.chain_list >= 64 > a tile's
    // pairs, so every window takes at least one tile)
    // tiles a window: the prefix table, or fewer (bf.chain_tiles >= 1: tests force
    // windows that end before the relation's trailing inactive tiles)
    const int tile_cap = bf.chain_tiles >= 1 && bf.chain_tiles < kSeqMaxTiles ? bf.chain_tiles : kSeqMaxTiles;
    const int list_cap = bf.chain_list >= 64 && bf.chain_list < kPipeList ? bf.chain_list : kPipeList;
    int pc = 0;  // P / Gram buffer of the current chunk
    int par = 0;  // vlist parity of the current chunk
    for (int gw = g0; gw < g0 + run || gw == g0;) {
        if (w == 0) {  // exclusive prefix of the window's tile pair counts (the relation pair left out)
            const int nt = g0 + run - gw < tile_cap ? g0 + run - gw : tile_cap;
            int carry = 0, fit = 0;
            for (int m0 = 0; m0 < nt; m0 += kWave) {
                const int g = m0 + l;
                int c = g < nt ? (bf.cnrows[gw + g] & 127) : 0;
                if (gw + g == g0 && has_rel) c -= 1;
                int x = c;
#pragma unroll
                for (int s = 1; s < kWave; s <<= 1) {
                    const int y = __shfl_up(x, s);
                    if (l >= s) x += y;
                }
                if (g < nt) pre[g] = carry + x - c;
                fit += __builtin_popcountll(__ballot(g < nt && carry + x <= list_cap - 1));
                carry += __shfl(x, kWave - 1);
            }
            if (l == 0) {
                if (fit == nt) pre[nt] = carry;
                misc[0] = fit;
            }
        }
        __syncthreads();
        const int ntile = misc[0];
        // the window holding the relation's last active sample is its last: the
        // tiles after it hold no pairs (only inactive samples), so a window cut by
        // the tile cap after it would otherwise lose the tail's renorm
        const bool last = gw + ntile == g0 + run || (g_tail >= 0 && gw + ntile > g_tail);
        const int ntp = pre[ntile];
        const int npairs = ntp + (last && has_rel ? 1 : 0);
        const int tail_start = last && g_tail >= gw ? ntp - n_tail : npairs;
        for (int f = threadIdx.x; f < npairs; f += kChainThreads) {
            int e = r, sl = -2;
            if (f < ntp) {
                int lo = 0, hi = ntile - 1;
                while (lo < hi) {
                    const int mid = (lo + hi + 1) >> 1;
                    if (pre[mid] <= f) lo = mid;
                    else hi = mid - 1;
                }
                const int32_t* cp = bf.cpairs + (int64_t)(gw + lo) * 2 * kCPairs;
                e = cp[f - pre[lo]];
                sl = cp[kCPairs + f - pre[lo]];
            }
            pe[f] = e;
            ps[f] = sl;
        }
        // chunks of R pairs; the relation's last update's pairs (and (entity'[r], r)) alone
        auto chunk_end = [&](int b) {
            return b < tail_start ? (b + R < tail_start ? b + R : tail_start) : npairs;
        };
        __syncthreads();
        if (npairs > 0) {
            // prologue: rows of chunks 0 and 1 into A slots 0 and 1, chunk 2's in flight,
            // chunk 0's projections afresh
            const int e0 = chunk_end(0);
            const int e1 = e0 < npairs ? chunk_end(e0) : e0;
            load_rows(0, e0);
            store_rows(0);
            load_rows(e0, e1);
            store_rows(1);
            load_rows(e1, e1 < npairs ? chunk_end(e1) : e1);
            if (tail_start == 0 && changed) renorm();  // (barriers: the row stores are then visible)
            __syncthreads();
            pc = 0;
            fresh(Abuf, e0, Pbuf, Gbuf);
        }
        int ka = 0;  // A slot of the current chunk
        for (int base = 0; base < npairs;) {
            const int nbase = chunk_end(base);
            const int cc = nbase - base;
            const int nb2 = nbase < npairs ? chunk_end(nbase) : nbase;
            const int cn = nb2 - nbase;  // pairs of the next chunk (0: none)
            const T* A = Abuf + ka * R * L;
            const T* An = Abuf + (ka == 2 ? 0 : ka + 1) * R * L;
            T* P = Pbuf + pc * R * L;
            T* Pn = Pbuf + (pc ^ 1) * R * L;
            T* Gm = Gbuf + pc * R * LG;
            T* Gn = Gbuf + (pc ^ 1) * R * LG;
            int* vl = vlist + par * R;
            const int ck = (int)n_chunks;  // the chunk's tag in the publish words (misc[6], misc[7])
            ++n_chunks;
            tick(1);
            if (w == 0) {
                // Walk: the pairs in order, each against the matrix the earlier ones left
                // (transr/trainer.cpp:35-64 per pair).  A violator v's shrink
                // W_c -= lr a_v^T g_v moves every later projection by -lr (a_j . a_v) g_v.
                const int j = l & (R - 1);
                T q = T(0);
                if (j < cc) {
                    q = qpart[j];
                    for (int v = 1; v < NB; ++v) q += qpart[v * R + j];
                }
                uint32_t vmask = 0;
                int npub = 0;  // violators published to the helper waves (correct_inc)
                if (__ballot(j < cc && q > T(1)) != 0) {
                    const T aaj = Gm[j * LG + j];  // |a_j|^2 (the Gram diagonal), off the violators' path
                    const int c0 = (l >> 5) * NH;
                    T x[NH];  // row j, columns c0 .. c0 + NH - 1
#pragma unroll
                    for (int u = 0; u < NH; ++u) x[u] = P[j * L + c0 + u];
                    int cursor = 0;
                    const T eps = T(2) * lr;
                    for (;;) {
                        const uint64_t cand = __ballot(l < R && j < cc && j >= cursor && q > T(1));
                        if (!cand) break;
                        const int v = __builtin_ctzll(cand);
                        const int c = l;  // column
                        // the scalars known at the pick, ahead of V: |p_v|^2, 1 / |p_v|^2, |a_v|^2
                        const T pp = readlane_f(q, v);
                        const T aa = readlane_f(aaj, v);
                        const T cjv = Gm[j * LG + v];  // a_j . a_v for the later rows' update
                        const int slv = ps[base + v];  // the violator's record slot (-2: (entity'[r], r))
                        // the violator's current row to LDS for the column-lane layout
                        if (j == v) {
#pragma unroll
                            for (int u = 0; u < NH; ++u) P[v * L + c0 + u] = x[u];
                        }
                        tick(4);
                        const T pv = c < NP ? P[v * L + c] : T(0);
                        T vv4[4] = {T(0), T(0), T(0), T(0)};
#pragma unroll
                        for (int t = 0; t < KS; ++t)
#pragma unroll
                            for (int u = 0; u < 4; ++u) vv4[u] = fma(P[v * L + 4 * t + u], reg[4 * t + u], vv4[u]);
                        const T Vc = c < n ? (vv4[0] + vv4[1]) + (vv4[2] + vv4[3]) : T(0);
                        tick(7);
                        T s2[2] = {pv * Vc, Vc * Vc};
                        // 1 / |p_v|^2: v_rcp_f64 and two Newton steps, as LLVM's own f64 division
                        // before its final correction (the reciprocal to within an ulp; kappa =
                        // pvd / pp then differs from the quotient by at most an ulp or so, which
                        // moves rho = 1 - 2 lr kappa by ~1e-3 ulp: no round test flips on it),
                        // issued beside the wave sums, off the violator's critical path
                        T rpp = __builtin_amdgcn_rcp(pp);
                        rpp = fma(fma(-pp, rpp, T(1)), rpp, rpp);
                        rpp = fma(fma(-pp, rpp, T(1)), rpp, rpp);
                        wave_sums<T, 2>(s2);
                        tick(8);
                        const T pV = s2[0], VV = s2[1];
                        const T pvd = pV + aa * pp, vvd = VV + T(2) * aa * pV + aa * aa * pp;
                        const T kappa = pvd * rpp;
                        const T w2t = vvd - kappa * pvd;
                        const T w2 = w2t > T(0) ? w2t : T(0);
                        const T rho = T(1) - eps * kappa;
                        T S0, S1;
                        const int m = transr_rounds_violator4(pp, w2, eps, rho, S0, S1);
                        n_rounds += (unsigned long long)m;
                        max_m = max_m > (unsigned long long)m ? max_m : (unsigned long long)m;
                        const T cpf = T(2) * (S0 + eps * S1 * kappa), cvf = T(2) * eps * S1;
                        const T g = c < n ? cpf * pv - cvf * (Vc + aa * pv) : T(0);
                        tick(9);
                        if (c < NP) P[v * L + c] = g;  // the violator's row now holds G
                        {  // its pair record G (da = -lr W G with the final matrix: chain_records)
                            T* dst = slv >= 0 ? bf.pair + (int64_t)slv * ld : bf.relpair + (int64_t)r * ld;
                            if (c < n) dst[c] = g;
                            if (l == 0) vio[nvt + npub] = slv;
                        }
                        tick(10);
                        const bool upd = j > v && j < cc;
                        T qh = T(0);  // this lane's half of |p_j|^2
                        if (upd) {
                            const T gl = -lr * cjv;
                            T s4[4] = {T(0), T(0), T(0), T(0)};
#pragma unroll
                            for (int u = 0; u < NH; ++u) {
                                x[u] = fma(gl, P[v * L + c0 + u], x[u]);
                                s4[u & 3] = fma(x[u], x[u], s4[u & 3]);
                            }
                            qh = (s4[0] + s4[1]) + (s4[2] + s4[3]);
                        }
                        {
                            const T tot = pair_sum32(qh);  // lanes j and j + 32: the same bits
                            if (upd) q = tot;
                        }
                        // publish v to the helper waves: its G row (above) and vl entry first
                        if (l == 0) {
                            vl[npub] = v;
                            __hip_atomic_store(&misc[7], (ck << 6) | (npub + 1), __ATOMIC_RELEASE,
                                               __HIP_MEMORY_SCOPE_WORKGROUP);
                        }
                        ++npub;
                        vmask |= 1u << v;
                        cursor = v + 1;
                        ++n_vio;
                        tick(11);
                    }
                }
                if (l < cc) {  // the chunk's pair flags; (entity'[r], r) marks the relation
                    const int sl = ps[base + l];
                    const bool vio_l = (vmask >> l) & 1;
                    if (sl >= 0) bf.pflag[sl] = vio_l ? 1 : 0;
                    else if (vio_l) bf.relpair_stamp[r] = bf.stamp;
                }
                if (l == 0) {
                    misc[1 + 2 * par] = (int)vmask;
                    misc[2 + 2 * par] = npub;
                    __hip_atomic_store(&misc[6], ck, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
                }
                tick(2);
            } else {
                // chunk k-1's W_c update and records, then the next chunk against W_{k-1}:
                // X = A_{k+1} W_c (each helper its own slices), its Gram matrix and the cross
                // Gram A_{k+1} A_k^T (waves 2 and 3)
                apply_pending();
                tick(12);
                if (cn > 0) {
                    const int nrt = cn > 16 ? 2 : 1, crt = cc > 16 ? 2 : 1;
#pragma unroll
                    for (int si = 0; si < NSW; ++si)
                        if (hw + 3 * si < NB)
                            for (int rt = 0; rt < nrt; ++rt) proj_tile(An, rt, si, Pn);
                    // the Gram tiles to the helpers with the fewest projection tiles (the
                    // same greedy choice on every helper); no cross Gram: correct_inc takes
                    // the few violators' dots a_{k+1}[j] . a_v on the fly
                    const int ng = nrt == 2 ? 3 : 1;
                    int load[3];
#pragma unroll
                    for (int h = 0; h < 3; ++h) load[h] = nrt * ((NB - h + 2) / 3);  // slices h, h + 3, ...
                    for (int tl = 0; tl < ng; ++tl) {
                        int best = 0;
#pragma unroll
                        for (int h = 1; h < 3; ++h) best = load[h] < load[best] ? h : best;
                        ++load[best];
                        if (best == hw) gram_tile(An, An, tl == 0 ? 0 : 1, tl == 2 ? 1 : 0, Gn, LG);
                    }
                    (void)crt;
                }
                // every helper past its debt (chunk k-1's A slot and G rows are free) and its
                // tiles (P_n, the Gram matrices complete)
                tick(13);
                helper_sync();
                tick(14);
                // chunk k+2's rows into the slot chunk k-1 left, chunk k+3's in flight
                if (nb2 < npairs || cn > 0) {
                    store_rows(ka == 0 ? 2 : ka - 1);
                    const int n3 = nb2 < npairs ? chunk_end(nb2) : nb2;
                    load_rows(n3, n3 < npairs ? chunk_end(n3) : n3);
                }
                // chunk k's violators into P_{k+1} as the walker publishes them, then |p|^2
                if (cn > 0) correct_inc(Pn, cn, P, An, A, vl, ck);
                tick(15);
            }
            __syncthreads();  // B1: the walk, the next chunk's corrected projections and |p|^2
            tick(w == 0 ? 3 : 5);
            const uint32_t vmask = (uint32_t)misc[1 + 2 * par];
            const int nv = misc[2 + 2 * par];
            // chunk k's debt passes to the helpers (paid at the next chunk, or below)
            pend_nv = nv;
            pend_par = par;
            pend_pc = pc;
            pend_ka = ka;
            nvt += nv;
            if (vmask) changed = true;
            const bool restart = nbase == tail_start && changed && cn > 0;  // the tail: afresh
            tick(6);
            if (restart) {
                apply_pending();  // the matrix up to date before the rows' renorm
                pend_nv = 0;
                __syncthreads();
                renorm();
                fresh(An, cn, Pn, Gn);
            }
            pc ^= 1;
            par ^= 1;
            ka = ka == 2 ? 0 : ka + 1;
            base = nbase;
        }
        // the window's last debt before its lists are rebuilt
        apply_pending();
        pend_nv = 0;
        __syncthreads();
        gw += ntile;
        if (last || gw >= g0 + run) break;
    }
    // the relation's matrix back: the helpers' slices into LDS (the records' matrix), then HBM
    if (w > 0) {
#pragma unroll
        for (int si = 0; si < NSW; ++si) {
            const int cb = hw + 3 * si;
            if (cb < NB) {
#pragma unroll
                for (int s = 0; s < KS; ++s) Wc[(4 * s + kq) * L + cb * 16 + l16] = reg[si * KS + s];
            }
        }
    }
    __syncthreads();
    if (mine && col < n)
        for (int jj = 0; jj < n; ++jj) bf.W[((int64_t)r * n + jj) * ld + col] = Wc[jj * L + col];
    chain_records<T, NP, L>(a, bf, r, vio, nvt, Wc, Pbuf, 2 * R * L);
    if (bf.stats) {
        if (threadIdx.x == 0) {
            const unsigned long long cyc = (unsigned long long)(clock64() - ck0);
            atomicAdd(&g_seq_stats[0], 1ull);
            atomicAdd(&g_seq_stats[1], n_chunks);
            atomicAdd(&g_seq_stats[2], n_vio);
            atomicAdd(&g_seq_stats[3], n_rounds);
            atomicAdd(&g_seq_stats[4], cyc);
            atomicMax(&g_seq_stats[5], cyc);
            atomicMax(&g_seq_stats[6], n_chunks);
            atomicMax(&g_seq_stats[7], max_m);
            for (int k = 0; k < 16; ++k) atomicAdd(&g_seq_stats[8 + k], ph[k]);
            if (n_chunks >= 20) {
                for (int k = 0; k < 16; ++k) atomicAdd(&g_seq_stats[24 + k], ph[k]);
                atomicAdd(&g_seq_stats[40], n_chunks);
                atomicAdd(&g_seq_stats[41], 1ull);
                atomicAdd(&g_seq_stats[42], n_vio);
            }
        }
    }
}

}  // namespace kb2e
