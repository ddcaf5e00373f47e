// kernels_transr_seq.hpp -- transRNorm of the PARALLEL TransR schedule per
// relation, in chunks of the relation's pairs: Jacobi inside a chunk,
// Gauss-Seidel across chunks (transr/trainer.cpp:35-64, :185-187; CPU model:
// oracle/parallel.py transr_constraint, renorm="jc<C>").
//
// Why per relation.  The reference calls transRNorm(h', W'_r), transRNorm(t',
// W'_r) and transRNorm(entity'[r], W'_r) after every update of relation r, one
// after another, each on the matrix the previous calls left: a later pair only
// shrinks W'_r if it still violates |W^T a|^2 <= 1 after the earlier pairs'
// shrinks.  Computing every pair of the batch against the same W'_r and summing
// the corrections (the tile kernels' Jacobi form) over-shrinks W'_r along the
// directions the relation's entities share: on FB15k-shaped data the compat
// loss ends 20% below the reference's and outside its seed envelope
// (profiles/seed_envelope_r17_fb15k_R_compat.jsonl, tools/probe_compat_parallel.py).
// Walking the relation's pairs in order, C at a time, with W_r updated after
// every chunk keeps the coupling the reference has (loss within ~1% of the
// reference after each epoch in the CPU model, against -5% for the sum).
//
// Per chunk of <= C pairs (the (h', r), (t', r) pairs of the active updates in
// (sample, update, role) order and (entity'[r], r) once, first occurrences per
// relation per batch -- the gradient kernel's compacted lists bf.cpairs):
//   P = A W_c                      (A: the pairs' entity rows after the unit norms)
//   violators: |p|^2 > 1
//   V = P_v K0 + |a|^2 P_v         (K0 = W^T W of the relation's matrix, made once)
//   m = first round with |p - 2 lr m v|^2 <= 1   (the loop p <- p - 2 lr (K0 + |a|^2) p
//                                                 to first order in lr)
//   G = 2 m p - 2 lr m (m - 1) v   (sum of 2 p over the m rounds)
//   da = -lr W_c G  -> pair records (pass 2 adds them to the entity rows)
//   W_c <- W_c - lr A_v^T G        (the chunk's matrix corrections)
// and the relation's matrix is written back once, so the transRNorm pass needs
// no matrix partials.  All four products are matrix-core GEMMs
// (v_mfma_f64_16x16x4_f64 / f32) over LDS images.
#pragma once

#include "kernels_transr_mfma.hpp"

namespace kb2e {

constexpr int kSeqThreads = 256;
constexpr int kSeqMaxTiles = 256;  // tiles of one relation handled per window of the prefix table

// LDS row stride of the images: n rounded up to even (16-byte rows of FP64 pairs)
__host__ __device__ constexpr int seq_ld(int n) { return (n + 1) & ~1; }

// LDS bytes: Wc [n][L] | K0 [n][L] | A [C][L] | P [C][L] | V [C][L] | |p|^2 [C] | ints
template <typename T>
__host__ __device__ constexpr size_t seq_lds(int n, int C) {
    return sizeof(T) * ((size_t)seq_ld(n) * (2 * (size_t)n + 3 * (size_t)C) + (size_t)C) +
           sizeof(int) * (size_t)(5 * C + kSeqMaxTiles + 1 + 8);
}

// KB2E_RPAR_STATS: relations, chunks, violators, rounds, cycles (sum, max) of the blocks
static __device__ unsigned long long g_seq_stats[8];

template <typename T, int NP, int C>
__global__ __launch_bounds__(kSeqThreads) void transr_cons_seq_kernel(RParArgs a, RParBufs<T> bf) {
    static_assert(C % 16 == 0 && C <= 64, "chunk: multiple of 16, one wave of lanes");
    constexpr int kPre = (C * NP + kSeqThreads - 1) / kSeqThreads;  // prefetched row elements a thread
    const int t0 = a.batch_t0[a.batch], t1 = a.batch_t0[a.batch + 1];
    const int g0 = blockIdx.x;  // tile index within the batch
    if (t0 + g0 >= t1) return;
    const int r = a.td_r[t0 + g0];
    if (g0 > 0 && a.td_r[t0 + g0 - 1] == r) return;  // not the relation's first tile
    const int n = a.n, ld = a.ld, L = seq_ld(n);
    const int w = threadIdx.x >> 6, l = lane_id();
    const T lr = (T)a.lr;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    T* Wc = (T*)smem;
    T* K0 = Wc + n * L;
    T* A = K0 + n * L;
    T* P = A + C * L;
    T* V = P + C * L;
    T* qv = V + C * L;                // [C] |p|^2 of the chunk's pairs
    int* ents = (int*)(qv + C);       // [C] this chunk's pairs: entity, slot (-2: (entity[r], r))
    int* slots = ents + C;
    int* nents = slots + C;           // [C] the next chunk's
    int* nslots = nents + C;
    int* vio = nslots + C;            // [C] this chunk's violators (chunk positions)
    int* pre = vio + C;               // [kSeqMaxTiles + 1] exclusive prefix of the window's tile pair counts
    int* misc = pre + kSeqMaxTiles + 1;  // 1 violators, 2 K0 made, 3 relation pair, 4 last sample, 5 tiles, 6 tail
    const long long ck0 = clock64();
    unsigned long long n_chunks = 0, n_vio = 0, n_rounds = 0;

    // the relation's matrix W'_r (after the gradient step's unit row norms)
    for (int idx = threadIdx.x; idx < n * n; idx += kSeqThreads) {
        const int j = idx / n, i = idx % n;
        Wc[j * L + i] = bf.W[((int64_t)r * n + j) * ld + i];
    }
    if (threadIdx.x == 0) misc[2] = 0;

    // The relation's pairs in order: its tiles' compacted lists, except that the
    // (entity'[r], r) pair, which the gradient kernel appends to the relation's
    // first tile, goes last (as the reference's last call of the batch; the
    // order, and so the result, does not depend on the tile size).  Windows of
    // up to kSeqMaxTiles tiles hold the prefix table.
    if (w == 0) {
        int run = 0;  // the relation's tiles: a run of equal td_r from g0
        for (int m0 = 0;; m0 += kWave) {
            const int g = g0 + m0 + l;
            const uint64_t b = __ballot(t0 + g < t1 && a.td_r[t0 + g] == r);
            const int k = b == ~0ull ? kWave : __builtin_ctzll(~b);
            run += k;
            if (k < kWave) break;
        }
        const int c0 = bf.cnrows[g0] & 127;
        const int rel = c0 > 0 && bf.cpairs[(int64_t)g0 * 2 * kCPairs + kCPairs + c0 - 1] == -2;
        // the relation's last active sample kl (its last update: the corrupted triple,
        // kl 2 + 1) and how many of the pairs (first occurrences) belong to that update
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
    for (int gw = g0; gw < g0 + run || gw == g0; gw += kSeqMaxTiles) {
        const int ntile = g0 + run - gw < kSeqMaxTiles ? g0 + run - gw : kSeqMaxTiles;
        const bool last = gw + ntile == g0 + run;
        if (w == 0) {  // exclusive prefix of the window's tile pair counts (the relation pair left out)
            int carry = 0;
            for (int m0 = 0; m0 < ntile; m0 += kWave) {
                const int g = m0 + l;
                int c = g < ntile ? (bf.cnrows[gw + g] & 127) : 0;
                if (gw + g == g0 && has_rel) c -= 1;
                int x = c;  // inclusive wave scan
#pragma unroll
                for (int s = 1; s < kWave; s <<= 1) {
                    const int y = __shfl_up(x, s);
                    if (l >= s) x += y;
                }
                if (g < ntile) pre[g] = carry + x - c;
                carry += __shfl(x, kWave - 1);
            }
            if (l == 0) pre[ntile] = carry;
        }
        __syncthreads();
        const int ntp = pre[ntile];                       // pairs from the window's tiles
        const int npairs = ntp + (last && has_rel ? 1 : 0);
        // the last update's pairs and (entity'[r], r) form the final chunk (in the last window)
        const int tail_start = last && g_tail >= gw ? ntp - n_tail : npairs;
        auto chunk_end = [&](int b) { return b < tail_start ? (b + C < tail_start ? b + C : tail_start) : npairs; };
        // pair `base + l` (wave 0, lane l < C): the tile holding that flat index
        // (binary search in pre), its entity and slot into registers
        auto fetch_ids = [&](int base, int& e, int& s) {
            e = -1;
            s = -3;
            const int f = base + l;
            if (w == 0 && l < C && f == ntp && f < npairs) {
                e = r;
                s = -2;
            } else if (w == 0 && l < C && f < ntp) {
                int lo = 0, hi = ntile - 1;
                while (lo < hi) {
                    const int mid = (lo + hi + 1) >> 1;
                    if (pre[mid] <= f) lo = mid;
                    else hi = mid - 1;
                }
                const int32_t* cp = bf.cpairs + (int64_t)(gw + lo) * 2 * kCPairs;
                e = cp[f - pre[lo]];
                s = cp[kCPairs + f - pre[lo]];
            }
        };
        // the chunk's entity rows into registers (issued early, stored after the chunk)
        T pre_rows[kPre];
        auto load_rows = [&](const int* e_in) {
#pragma unroll
            for (int q = 0; q < kPre; ++q) {
                const int idx = threadIdx.x + q * kSeqThreads;
                const int k = idx / NP, j = idx % NP;
                const int e = (k < C) ? e_in[k] : -1;
                pre_rows[q] = (e >= 0 && j < n) ? bf.ent[(int64_t)e * ld + j] : T(0);
            }
        };
        auto store_rows = [&]() {
#pragma unroll
            for (int q = 0; q < kPre; ++q) {
                const int idx = threadIdx.x + q * kSeqThreads;
                const int k = idx / NP, j = idx % NP;
                if (k < C && j < L) A[k * L + j] = j < n ? pre_rows[q] : T(0);
            }
        };
        {
            int e, s;
            fetch_ids(0, e, s);
            if (w == 0 && l < C) {
                ents[l] = e;
                slots[l] = s;
            }
        }
        __syncthreads();
        load_rows(ents);
        store_rows();
        __syncthreads();
        for (int base = 0; base < npairs; base = chunk_end(base)) {
            const int cc = chunk_end(base) - base;
            ++n_chunks;
            // the next chunk's ids (their loads overlap this chunk's projections)
            const int nbase = chunk_end(base);
            const bool more = nbase < npairs;
            int e_next = -1, s_next = -3;
            if (more) fetch_ids(nbase, e_next, s_next);
            if (base == tail_start && misc[2]) {
                // the relation's last update renormalises the rows before its own pairs'
                // shrinks (transr/trainer.cpp:178-180): a wave a row
                for (int j = w; j < n; j += kSeqThreads / kWave) {
                    const T x = l < n ? Wc[j * L + l] : T(0);
                    const T len = sqrt(wave_sum(x * x));
                    if (l < n) Wc[j * L + l] = x / len;
                }
                __syncthreads();
            }
            // P = A W_c
            block_gemm<T>(C / 16, NP / 16, rm_k4(n),
                          [&](int ar, int k) { return (ar < cc && k < n) ? A[ar * L + k] : T(0); },
                          [&](int k, int bc) { return (k < n && bc < n) ? Wc[k * L + bc] : T(0); },
                          [&](int m, int c, T v) {
                              if (m < C && c < n) P[m * L + c] = v;
                          });
            if (more && w == 0 && l < C) {
                nents[l] = e_next;
                nslots[l] = s_next;
            }
            __syncthreads();
            if (more) load_rows(nents);  // the next chunk's rows in flight during this one
            {  // |p|^2: kSeqThreads / C threads a pair
                constexpr int TPP = kSeqThreads / C;
                const int k = threadIdx.x / TPP, part = threadIdx.x % TPP;
                T q = T(0);
                if (k < cc)
                    for (int i = part; i < n; i += TPP) q += P[k * L + i] * P[k * L + i];
#pragma unroll
                for (int sft = 1; sft < TPP; sft <<= 1) q += __shfl_xor(q, sft);
                if (part == 0) qv[k] = q;
            }
            __syncthreads();
            // violators |p|^2 > 1 (wave 0, lane = pair)
            if (w == 0) {
                const bool v = l < cc && qv[l < C ? l : 0] > T(1);
                const uint64_t m = __ballot(v);
                if (v) vio[__builtin_popcountll(m & ((1ull << l) - 1))] = l;
                if (l == 0) misc[1] = __builtin_popcountll(m);
                const int s = l < cc ? slots[l] : -3;
                if (l < cc && !v && s >= 0) bf.pflag[s] = 0;
                if (v && s >= 0) bf.pflag[s] = 1;
                if (v && s == -2) bf.relpair_stamp[r] = bf.stamp;
            }
            __syncthreads();
            const int nv = misc[1];
            if (nv > 0) {
                n_vio += nv;
                if (!misc[2]) {  // K0 = W^T W once (W_c is still W'_r before the first violator)
                    block_gemm<T>(NP / 16, NP / 16, rm_k4(n),
                                  [&](int ar, int k) { return (ar < n && k < n) ? Wc[k * L + ar] : T(0); },
                                  [&](int k, int bc) { return (k < n && bc < n) ? Wc[k * L + bc] : T(0); },
                                  [&](int m, int c, T v) {
                                      if (m < n && c < n) K0[m * L + c] = v;
                                  });
                    __syncthreads();
                    if (threadIdx.x == 0) misc[2] = 1;
                }
                // V = P_v K0 (rows: the compacted violators)
                block_gemm<T>((nv + 15) / 16, NP / 16, rm_k4(n),
                              [&](int ar, int k) { return (ar < nv && k < n) ? P[vio[ar] * L + k] : T(0); },
                              [&](int k, int bc) { return (k < n && bc < n) ? K0[k * L + bc] : T(0); },
                              [&](int m, int c, T v) {
                                  if (m < nv && c < n) V[m * L + c] = v;
                              });
                __syncthreads();
                // per violator (a wave each): the rounds of transRNorm's loop in closed
                // form (oracle/parallel.py transr_norm_rounds): v = (K0 + |a|^2) p =
                // kappa p + w, rho = 1 - eps kappa, |p_t|^2 = rho^2t Q0 + eps^2 t^2
                // rho^(2t-2) |w|^2, G = 2 (S0 p - eps S1 w) -> V
                const T eps = T(2) * lr;
                for (int v = w; v < nv; v += kSeqThreads / kWave) {
                    const int k = vio[v];
                    const T ai = l < n ? A[k * L + l] : T(0);
                    const T pi = l < n ? P[k * L + l] : T(0);
                    const T s0 = wave_sum(ai * ai);
                    const T vi = l < n ? V[v * L + l] + s0 * pi : T(0);
                    const T q0 = wave_sum(pi * pi);
                    const T kappa = wave_sum(pi * vi) / q0;
                    const T wi = l < n ? vi - kappa * pi : T(0);
                    const T w2 = wave_sum(wi * wi);
                    const T rho = T(1) - eps * kappa;
                    int m = 0;
                    T S0 = T(0), S1 = T(0), rt = T(1), rtm1 = T(0);
                    while (m < kRParMaxIter) {
                        const T mm = (T)m;
                        if (!(rt * rt * q0 + eps * eps * mm * mm * rtm1 * rtm1 * w2 > T(1))) break;
                        S0 += rt;
                        S1 += mm * rtm1;
                        ++m;
                        rtm1 = rt;
                        rt *= rho;
                    }
                    if (l == 0) n_rounds += (unsigned long long)m;
                    if (l < n) V[v * L + l] = T(2) * (S0 * pi - eps * S1 * wi);
                }
                __syncthreads();
                // da = -lr W_c G -> the pair records
                block_gemm<T>((nv + 15) / 16, NP / 16, rm_k4(n),
                              [&](int ar, int k) { return (ar < nv && k < n) ? V[ar * L + k] : T(0); },
                              [&](int k, int bc) { return (k < n && bc < n) ? Wc[bc * L + k] : T(0); },
                              [&](int m, int j, T v) {
                                  if (m < nv && j < n) {
                                      const int s = slots[vio[m]];
                                      T* dst = s >= 0 ? bf.pair + (int64_t)s * ld : bf.relpair + (int64_t)r * ld;
                                      dst[j] = -lr * v;
                                  }
                              });
                __syncthreads();
                // W_c -= lr A_v^T G
                block_gemm<T>(NP / 16, NP / 16, rm_k4(nv),
                              [&](int ar, int k) { return (ar < n && k < nv) ? A[vio[k] * L + ar] : T(0); },
                              [&](int k, int bc) { return (k < nv && bc < n) ? V[k * L + bc] : T(0); },
                              [&](int j, int i, T v) {
                                  if (j < n && i < n) Wc[j * L + i] -= lr * v;
                              });
                __syncthreads();
            }
            if (more) {  // the next chunk in place
                store_rows();
                if (w == 0 && l < C) {
                    ents[l] = nents[l];
                    slots[l] = nslots[l];
                }
                __syncthreads();
            }
        }
        __syncthreads();
    }
    // the relation's matrix back (the transRNorm pass adds no partials)
    for (int idx = threadIdx.x; idx < n * n; idx += kSeqThreads) {
        const int j = idx / n, i = idx % n;
        bf.W[((int64_t)r * n + j) * ld + i] = Wc[j * L + i];
    }
    if (bf.stats) {
        if (threadIdx.x == 0) {
            const unsigned long long cyc = (unsigned long long)(clock64() - ck0);
            atomicAdd(&g_seq_stats[0], 1ull);
            atomicAdd(&g_seq_stats[1], n_chunks);
            atomicAdd(&g_seq_stats[2], n_vio);
            atomicAdd(&g_seq_stats[4], cyc);
            atomicMax(&g_seq_stats[5], cyc);
            atomicMax(&g_seq_stats[6], n_chunks);
        }
        if (l == 0 && n_rounds) atomicAdd(&g_seq_stats[3], n_rounds);
    }
}

}  // namespace kb2e
