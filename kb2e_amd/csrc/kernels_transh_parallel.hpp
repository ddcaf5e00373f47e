// kernels_transh_parallel.hpp -- TransH under the PARALLEL schedule
// (KB2E_SCHEDULE_PARALLEL; kernels_parallel.hpp has the TransE form).
//
// The reference's TransH step (transh/trainer.cpp:11-59) for one update
// (h, t, r, beta), from the snapshot: hs = w.h, ts = w.t,
// x = sign(2((t - ts w) - (h - hs w) - r)), sum_x = x.w;
//   r' -= beta lr x,  h' -= beta lr x,  t' += beta lr x          (the TransE deltas)
//   w' += beta lr (hs - ts) x + beta lr sum_x (h - t)
//   norm(r'), norm(h'), norm(t') (<= 1), norm(w', false) (unit),
//   normOrth(r', w'), normOrth(h', w'), normOrth(t', w')       (common/utils.cpp:79-111)
// Here: the h/t/r rows take the TransE apply (summed sign counts, one norm);
// every relation's w gets its summed delta and one unit norm (one workgroup per
// relation, waves over chunks of its updates); then every (row, w') pair of an
// active update is checked (w'.a > 0.1), and the few violating pairs run the
// reference's normOrth loop in sample order on one wave, exactly as written
// (including its never-reset `sum`).
#pragma once

#include "kernels_relowner.hpp"

namespace kb2e {

template <typename T>
struct HParArgs {
    const int32_t* heads;
    const int32_t* tails;
    const int32_t* rels;
    const int32_t* si;
    const int32_t* sj;
    const uint8_t* side;
    int32_t B, n, ld, nw, ne, nr;
    int32_t batch;
    double lr;
    const uint64_t* keys;
    const int32_t* seg_start;
    const int32_t* batch_seg;
    const int32_t* seg_row;
    const int32_t* rel_begin;
    const uint8_t* act;
    const int32_t* meta;      // event records (kernels_transe.hpp EventRecs)
    const uint64_t* words;
    const T* scal;            // [B][2][4] hs, ts, sum_x
    const T* snap;            // [B][2][ld] each update's w delta (transh_score_kernel, EMIT)
    T* ent;
    T* rel;
    T* w;
    uint8_t* orth_mask;       // [B] violating (update, row) pairs of each sample, bits u * 3 + {r, h, t}
};

// One NWV-wave workgroup per relation segment of the batch: waves sum chunks
// of its events, partial sums combined in wave order, wave 0 applies.  The
// hottest relation (~1100 events on FB15k-shaped batches) sets the time, so
// the default is 16 waves (8 and 4 measured 16% and 50% slower).
template <typename T, int CH, int NWV>
__global__ __launch_bounds__(NWV * kWave) void transh_w_apply_kernel(HParArgs<T> a) {
    __shared__ T part[NWV][CH * kVec][kWave];
    __shared__ int any;
    const int s = a.rel_begin[a.batch] + blockIdx.x;
    if (s >= a.batch_seg[a.batch + 1]) return;
    const int w = threadIdx.x >> 6, l = lane_id();
    const int p0 = a.seg_start[s], p1 = a.seg_start[s + 1];
    const int r = a.seg_row[s] - a.ne;
    if (threadIdx.x == 0) any = 0;
    __syncthreads();
    T acc[CH][kVec] = {};
    bool act_any = false;
    for (int base = p0 + w * kWave; base < p1; base += NWV * kWave) {
        const int p = base + l;
        int xrow = -1;
        if (p < p1) {
            const int32_t meta = a.meta[p];
            if (((meta & 3) - 1) != 0) xrow = meta >> 4;  // active update: kk * 2 + u
        }
        uint64_t m = __ballot(xrow >= 0);
        if (m) act_any = true;
        while (m) {  // G updates' delta rows (score kernel) in flight together, summed in event order
            constexpr int G = 16 / CH;
            int ev[G], xr[G];
            int ne4 = 0;
            for (; ne4 < G && m; ++ne4) {
                ev[ne4] = __builtin_ctzll(m);
                m &= m - 1;
                xr[ne4] = readlane_i32(xrow, ev[ne4]);
            }
            T dv[G][CH][kVec];
#pragma unroll
            for (int q = 0; q < G; ++q) {
                if (q >= ne4) continue;
                const T* drow = a.snap + (int64_t)xr[q] * a.ld;
#pragma unroll
                for (int cc = 0; cc < CH; ++cc)
#pragma unroll
                    for (int k = 0; k < kVec; ++k) {
                        const int el = cc * (kWave * kVec) + l * kVec + k;
                        dv[q][cc][k] = el < a.n ? drow[el] : T(0);
                    }
            }
#pragma unroll
            for (int q = 0; q < G; ++q) {
                if (q >= ne4) continue;
#pragma unroll
                for (int cc = 0; cc < CH; ++cc)
#pragma unroll
                    for (int k = 0; k < kVec; ++k)
                        if (elem_valid(cc, k, a.n)) acc[cc][k] += dv[q][cc][k];
            }
        }
    }
#pragma unroll
    for (int cc = 0; cc < CH; ++cc)
#pragma unroll
        for (int k = 0; k < kVec; ++k) part[w][cc * kVec + k][l] = acc[cc][k];
    if (act_any && l == 0) atomicOr(&any, 1);
    __syncthreads();
    if (w != 0 || !any) return;
    RowReg<T, CH> W;
    T* wrow = a.w + (int64_t)r * a.ld;
    W.load(wrow, a.n);
#pragma unroll
    for (int cc = 0; cc < CH; ++cc)
#pragma unroll
        for (int k = 0; k < kVec; ++k) {
            T sum = part[0][cc * kVec + k][l];
            for (int v = 1; v < NWV; ++v) sum += part[v][cc * kVec + k][l];
            if (elem_valid(cc, k, a.n)) W.v[cc][k] = W.v[cc][k] + sum;
        }
    W.norm(a.n, false);
    W.store(wrow, a.n);
}

// One wave per active sample: w'.a for the rows r', h', t' of both updates
// (after every norm); bit set where the reference's loop would move them.
template <typename T, int CH>
__global__ __launch_bounds__(256) void transh_orth_check_kernel(HParArgs<T> a) {
    const int kk = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (kk >= a.B) return;
    const int l = lane_id();
    if (!a.act[kk]) {
        if (l == 0) a.orth_mask[kk] = 0;
        return;
    }
    const int i0 = a.si[kk], j = a.sj[kk];
    const int h = a.heads[i0], t = a.tails[i0], r = a.rels[i0];
    const int nh = a.side[kk] ? h : j, nt = a.side[kk] ? j : t;
    RowReg<T, CH> W;
    W.load(a.w + (int64_t)r * a.ld, a.n);
    const T* rows[6] = {a.rel + (int64_t)r * a.ld, a.ent + (int64_t)h * a.ld, a.ent + (int64_t)t * a.ld,
                        a.rel + (int64_t)r * a.ld, a.ent + (int64_t)nh * a.ld, a.ent + (int64_t)nt * a.ld};
    uint32_t mask = 0;
#pragma unroll
    for (int q = 0; q < 6; ++q) {
        if (q == 3) continue;  // the relation row is checked once: its second check sees the same rows
        RowReg<T, CH> A;
        A.load(rows[q], a.n);
        T x = T(0);
#pragma unroll
        for (int cc = 0; cc < CH; ++cc)
#pragma unroll
            for (int k = 0; k < kVec; ++k) x += W.v[cc][k] * A.v[cc][k];
        if (wave_sum(x) > T(0.1)) mask |= 1u << q;
    }
    if (l == 0) a.orth_mask[kk] = (uint8_t)mask;
}

// One wave, samples in order: the reference's normOrth (common/utils.cpp:79-111,
// orth_norm) on every flagged pair, in place on the live rows.  Per pass the
// flag words of 2048 samples are loaded at once and the flagged samples listed
// in sample order in LDS; their ids (r, h, t, h', t') are fetched for 64 list
// entries at a time, so the serial part is only the rows' load / normOrth /
// store.  w_r stays in registers while consecutive flagged samples share the
// relation (the reference reloads what it just stored), and a store is drained
// only before a later load of the same row (PendingRows).
constexpr int kOrthWords = 4;  // 8-byte flag words per lane per pass

// Rows stored by this wave and not yet drained: a load of one of them waits
// for the stores first (s_waitcnt vmcnt(0)); everything else loads at once.
struct PendingRows {
    static constexpr int kCap = 8;
    int id[kCap];
    int cnt = 0;
    __device__ void drain() {
        drain_stores();
        cnt = 0;
    }
    __device__ void before_load(int key) {
        bool hit = false;
        for (int i = 0; i < cnt; ++i) hit |= id[i] == key;
        if (hit) drain();
    }
    __device__ void add(int key) {
        if (cnt == kCap) drain();
        id[cnt++] = key;
    }
};

// common/utils.cpp:79-111 norm(a, b, rate) with the loop carried on scalars.
// After the leading unit norm of b (a vector operation, as written), every
// iterate is a combination a = p a0 + q b0, b = u a0 + v b0 of the rows that
// entered the loop, so |b|^2 and x = a.b follow from the three Gram products
// a0.a0, a0.b0, b0.b0 (one wave reduction for the three): an iteration is a
// dozen dependent scalar operations instead of two wave reductions, a sqrt
// and 2n divisions.  The reference's running `sum` (never reset) is kept.
// The rows are formed once at the end, then the trailing unit norm of b.
// Values agree with the element-wise loop to rounding (~1e-15 relative;
// PARALLEL-schedule tolerance, tests/test_gpu_parallel.py); every decision
// x > 0.1 is the same unless x lies within that rounding of 0.1.
template <typename T, int CH>
__device__ __forceinline__ void orth_norm_gram(RowReg<T, CH>& A, RowReg<T, CH>& Bv, int n, T rate, bool unit) {
    // unit: Bv is the previous call's output (just scaled to unit length): the
    // leading norm would divide by 1 +- ulp, skipped
    if (!unit) Bv.norm(n, false);
    T g[3] = {T(0), T(0), T(0)};
#pragma unroll
    for (int c = 0; c < CH; ++c)
#pragma unroll
        for (int k = 0; k < kVec; ++k) {
            g[0] += A.v[c][k] * A.v[c][k];
            g[1] += A.v[c][k] * Bv.v[c][k];
            g[2] += Bv.v[c][k] * Bv.v[c][k];
        }
#pragma unroll
    for (int i = 0; i < 3; ++i) g[i] = wave_sum(g[i]);
    const T aa = g[0], ab = g[1], bb = g[2];
    T p = T(1), q = T(0), u = T(0), v = T(1), sum = T(0);
    bool moved = false;
    for (int it = 0; it < 1 << 20; ++it) {
        sum = sqrt(sum + ((u * u) * aa + T(2) * (u * v) * ab + (v * v) * bb));
        const T rs = T(1) / sum;
        u = u * rs;
        v = v * rs;
        const T x = (p * u) * aa + (p * v + q * u) * ab + (q * v) * bb;
        if (!(x > T(0.1))) break;
        moved = true;
        p = p - rate * u;  // a -= rate b
        q = q - rate * v;
        u = u - rate * p;  // b -= rate a
        v = v - rate * q;
    }
#pragma unroll
    for (int c = 0; c < CH; ++c)
#pragma unroll
        for (int k = 0; k < kVec; ++k) {
            if (!elem_valid(c, k, n)) continue;
            const T a0 = A.v[c][k], b0 = Bv.v[c][k];
            if (moved) A.v[c][k] = p * a0 + q * b0;
            Bv.v[c][k] = u * a0 + v * b0;
        }
    Bv.norm(n, false);
}

// The rows of the flagged pairs are prefetched kOrthAhead tasks ahead (a task =
// one flagged (row, w) pair, in sample order); a row that one of the last
// kOrthAhead tasks stored is taken from those tasks' register copies instead
// of the (possibly stale) prefetch, and a prefetch of a row stored earlier and
// not yet drained waits for the stores first (PendingRows) -- so the serial
// part per task is normOrth itself, not a memory round trip.
constexpr int kOrthAhead = 4;
#ifdef KB2E_OWNER_PROF
__device__ unsigned long long g_orth_prof[16];  // tasks, w switches, chunks, passes, cycles: all, pass setup, task build, w loads, normOrth
#define ORTH_PROF(k, v) (l == 0 ? (void)atomicAdd(&g_orth_prof[k], (unsigned long long)(v)) : (void)0)
#else
#define ORTH_PROF(k, v) ((void)0)
#endif

template <typename T, int CH>
__global__ __launch_bounds__(64) void transh_orth_fix_kernel(HParArgs<T> a) {
    __shared__ int list[8 * kWave * kOrthWords];
    __shared__ int tkey[6 * kWave], trel[6 * kWave];  // the chunk's tasks: row key, relation
    const int l = lane_id();
    RowReg<T, CH> W;
    int wid = -1;
    bool wunit = false;  // W holds the last normOrth's unit output
    PendingRows pend;
    // ids: relations [0, nr), w rows [nr, 2 nr), entities from 2 nr
    auto row_of = [&](int key) -> T* {
        return key < a.nr ? a.rel + (int64_t)key * a.ld : a.ent + (int64_t)(key - 2 * a.nr) * a.ld;
    };
#ifdef KB2E_OWNER_PROF
    const unsigned long long ckA = clock64();
    unsigned long long ck = ckA;
#else
    unsigned long long ck = 0;
#endif
    auto mark = [&](int k) {
#ifdef KB2E_OWNER_PROF
        const unsigned long long c2 = clock64();
        ORTH_PROF(k, c2 - ck);
        ck = c2;
#else
        (void)k;
        (void)ck;
#endif
    };
    for (int base = 0; base < a.B; base += 8 * kWave * kOrthWords) {
        ORTH_PROF(3, 1);
        mark(15);
        uint64_t word[kOrthWords];
#pragma unroll
        for (int wi = 0; wi < kOrthWords; ++wi) {  // orth_mask is zero past B up to a multiple of 512
            const int off = base + 8 * (wi * kWave + l);
            word[wi] = off < a.B ? *reinterpret_cast<const uint64_t*>(a.orth_mask + off) : 0ull;
        }
        int count = 0;
#pragma unroll
        for (int wi = 0; wi < kOrthWords; ++wi) {  // sample order: word, lane, byte
            int mine = 0;
#pragma unroll
            for (int by = 0; by < 8; ++by) mine += ((word[wi] >> (8 * by)) & 0xffu) != 0;
            int pre = mine;  // inclusive scan over the lanes
#pragma unroll
            for (int d = 1; d < kWave; d <<= 1) {
                const int v = __shfl_up(pre, d);
                if (l >= d) pre += v;
            }
            int pos = count + pre - mine;
#pragma unroll
            for (int by = 0; by < 8; ++by)
                if (((word[wi] >> (8 * by)) & 0xffu) != 0) list[pos++] = base + 8 * (wi * kWave + l) + by;
            count += __shfl(pre, kWave - 1);
        }
        wave_lds_sync();
        mark(5);
        for (int g = 0; g < count; g += kWave) {
            ORTH_PROF(2, 1);
            // this lane's list entry: its flagged rows become tasks, in (sample, q) order
            int ntask;
            {
                int bits = 0, ids[6] = {0, 0, 0, 0, 0, 0}, r = 0;
                if (g + l < count) {
                    const int k2 = list[g + l];
                    const int i0 = a.si[k2], j = a.sj[k2];
                    const bool sd = a.side[k2];
                    bits = a.orth_mask[k2];
                    const int h = a.heads[i0], t = a.tails[i0];
                    r = a.rels[i0];
                    ids[0] = r;
                    ids[1] = 2 * a.nr + h;
                    ids[2] = 2 * a.nr + t;
                    ids[3] = r;
                    ids[4] = 2 * a.nr + (sd ? h : j);
                    ids[5] = 2 * a.nr + (sd ? j : t);
                }
                const int mine = __builtin_popcount(bits & 63);
                int pre = mine;
#pragma unroll
                for (int d = 1; d < kWave; d <<= 1) {
                    const int v = __shfl_up(pre, d);
                    if (l >= d) pre += v;
                }
                int pos = pre - mine;
#pragma unroll
                for (int q = 0; q < 6; ++q)
                    if ((bits >> q) & 1) {
                        tkey[pos] = ids[q];
                        trel[pos] = r;
                        ++pos;
                    }
                ntask = __shfl(pre, kWave - 1);
            }
            wave_lds_sync();
            mark(6);
            ORTH_PROF(0, ntask);
            // prefetch ring: slot j holds task t0 + j's row (t0 a multiple of kOrthAhead)
            RowReg<T, CH> ring[kOrthAhead], done[kOrthAhead];
            int dkey[kOrthAhead];
#pragma unroll
            for (int j = 0; j < kOrthAhead; ++j) {
                dkey[j] = -1;
                if (j < ntask) {
                    const int key = tkey[j];
                    pend.before_load(key);
                    row_load_sc1(ring[j], row_of(key), a.n);
                }
            }
            for (int t0 = 0; t0 < ntask; t0 += kOrthAhead) {
#pragma unroll
                for (int j = 0; j < kOrthAhead; ++j) {
                    const int t = t0 + j;
                    if (t >= ntask) break;
                    const int key = tkey[t], er = trel[t];
                    if (er != wid) {  // w_r: kept in registers while consecutive tasks share the relation
                        mark(14);
                        ORTH_PROF(1, 1);
                        if (wid >= 0) {
                            row_store_sc1(W, a.w + (int64_t)wid * a.ld, a.n);
                            pend.add(a.nr + wid);
                        }
                        pend.before_load(a.nr + er);
                        row_load_sc1(W, a.w + (int64_t)er * a.ld, a.n);
                        wid = er;
                        wunit = false;
#ifdef KB2E_OWNER_PROF
                        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
                        mark(7);
                    }
                    // the row: the newest copy among the last kOrthAhead tasks' stores, else the prefetch
                    RowReg<T, CH> A = ring[j];
#pragma unroll
                    for (int d = 1; d <= kOrthAhead; ++d) {  // slot (j - d) mod kOrthAhead: task t - d
                        const int sd = (j - d + kOrthAhead) % kOrthAhead;
                        if (dkey[sd] == key && t - d >= 0) {
                            A = done[sd];
                            break;
                        }
                    }
#ifdef KB2E_OWNER_PROF
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
                    mark(14);
                    orth_norm_gram<T, CH>(A, W, a.n, (T)a.lr, wunit);
                    wunit = true;
                    mark(8);
                    row_store_sc1(A, row_of(key), a.n);
                    pend.add(key);
                    done[j] = A;
                    dkey[j] = key;
                    if (t + kOrthAhead < ntask) {  // the prefetch of task t + kOrthAhead into the freed slot
                        const int k2 = tkey[t + kOrthAhead];
                        pend.before_load(k2);
                        row_load_sc1(ring[j], row_of(k2), a.n);
                    }
                }
            }
            wave_lds_sync();
        }
        wave_lds_sync();
    }
    if (wid >= 0) row_store_sc1(W, a.w + (int64_t)wid * a.ld, a.n);
    drain_stores();
#ifdef KB2E_OWNER_PROF
    ORTH_PROF(4, clock64() - ckA);
#endif
}

}  // namespace kb2e
