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
    int32_t* orth_ids;        // [B][8] a flagged sample's r, h, t, h', t' (check kernel; the one-wave pass)
    unsigned long long* ent_tag;  // [ne] stamp << 32 | multi << 31 | relation of the entity's flagged pairs
    uint32_t stamp;           // this batch's tag stamp (never 0)
    // normOrth's relation pass runs when the previous batch's normOrth work (its loop
    // iterations over both passes, a wave-serial step each) was >= orth_rel_min (little
    // work: the one-wave pass alone is cheaper than a launch over the relations); the
    // work counts alternate by batch
    uint32_t* orth_work_cur;    // this batch's iterations (relation and one-wave passes)
    uint32_t* orth_work_prev;   // the previous batch's (read by the relation pass, then zeroed)
    uint32_t orth_rel_min;
    uint32_t* orth_rel_runs;    // batches whose relation pass ran (kb2e_counter "transh_orth_rel_batches")
    int32_t orth_q;             // second-sweep queue capacity (kOrthQ; KB2E_HPAR_ORTH_Q for the tests)
    unsigned long long* clk;    // KB2E_HPAR_CLK (diagnostic): per w-apply workgroup start, after its small
                                // segments, end (wall clock), large segments << 32 | their events
};

// The flagged entity rows' relations this batch: the first relation a row is
// flagged under, and a mark once a second one shows up (one CAS loop).
template <typename T>
__device__ __forceinline__ void orth_tag_entity(HParArgs<T> a, int e, int r) {
    unsigned long long* p = a.ent_tag + e;
    const unsigned long long mine = ((unsigned long long)a.stamp << 32) | (unsigned)r;
    unsigned long long old = *p;
    for (;;) {
        unsigned long long nv;
        if ((uint32_t)(old >> 32) != a.stamp) nv = mine;
        else if ((old & 0x80000000ull) || (uint32_t)(old & 0x7fffffffu) == (uint32_t)r) return;
        else nv = old | 0x80000000ull;
        const unsigned long long prev = atomicCAS(p, old, nv);
        if (prev == old) return;
        old = prev;
    }
}

// an entity row flagged under more than one relation this batch (its tag was set by this batch)
template <typename T>
__device__ __forceinline__ bool orth_shared(HParArgs<T> a, int e) {
    return (a.ent_tag[e] & 0x80000000ull) != 0;
}

// One NWV-wave workgroup per NWV relation segments of the batch (most relations
// have a few events: a 16-wave workgroup each was 1,345 workgroups a batch, bound
// by dispatch, ~30 us).  A segment of at most kWSmall events is one wave's: its sum
// in event order, the unit norm, the store.  The larger ones (the hot relations)
// take the whole workgroup one after another: each wave sums a contiguous slice of
// the segment's events, the partial sums are combined in wave order, wave 0 applies.
// The kernel is a chain of dependent memory round trips on few waves (r23 PMC,
// 1.3 waves a SIMD, 2 LDS instructions a wave, no bank conflicts,
// SQ_WAIT_INST_ANY / SQ_ACTIVE_INST_ANY = 0.56), so every step keeps its loads
// together: the w row is loaded with the segment's first event records, a wave's
// event records (up to 64) in one load, their delta rows 16 at a time.
constexpr int kWSmall = 32;

template <typename T, int CH, int NWV>
__device__ __forceinline__ void transh_w_apply_body(HParArgs<T> a, int bid) {
    __shared__ T part[NWV][CH * kVec][kWave];
    __shared__ int any;
    const int sb = a.rel_begin[a.batch] + bid * NWV;
    const int se = min(sb + NWV, a.batch_seg[a.batch + 1]);
    if (sb >= se) return;
    const int w = threadIdx.x >> 6, l = lane_id();
    const unsigned long long t_start = a.clk ? wall_clock64() : 0ull;
    unsigned long long n_large = 0;
    constexpr int G = 16 / CH;
    // the active events of [q0, q1) (at most 64: one record a lane) added to acc in
    // event order, G delta rows (score kernel) in flight at a time
    auto add_events = [&](int q0, int q1, T (&acc)[CH][kVec]) {
        const int p = q0 + l;
        int xrow = -1;
        if (p < q1) {
            const int32_t meta = a.meta[p];
            if (((meta & 3) - 1) != 0) xrow = meta >> 4;  // active update: kk * 2 + u
        }
        uint64_t m = __ballot(xrow >= 0);
        const bool act = m != 0;
        while (m) {
            // G rows a round, every load unconditional (a missing event reads the round's
            // first row again and adds nothing): the loads issue back to back -- loads
            // behind a per-row condition were each waited for before the next one went
            // out, a memory round trip per event (KB2E_HPAR_CLK: the hot relation's
            // 1,140 events took 25 us)
            int xr[G];
#pragma unroll
            for (int q = 0; q < G; ++q) {
                xr[q] = m ? readlane_i32(xrow, __builtin_ctzll(m)) : -1;
                m &= m - 1;
            }
            T dv[G][CH][kVec];
#pragma unroll
            for (int q = 0; q < G; ++q) {
                const T* drow = a.snap + (int64_t)(xr[q] >= 0 ? xr[q] : xr[0]) * a.ld;
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
                if (xr[q] < 0) continue;
#pragma unroll
                for (int cc = 0; cc < CH; ++cc)
#pragma unroll
                    for (int k = 0; k < kVec; ++k)
                        if (elem_valid(cc, k, a.n)) acc[cc][k] += dv[q][cc][k];
            }
        }
        return act;
    };
    // w_r += the sum, unit norm (a relation is touched only through an active update);
    // W holds the row, loaded ahead
    auto apply = [&](RowReg<T, CH>& W, T* wrow, const T (&sum)[CH][kVec]) {
#pragma unroll
        for (int cc = 0; cc < CH; ++cc)
#pragma unroll
            for (int k = 0; k < kVec; ++k)
                if (elem_valid(cc, k, a.n)) W.v[cc][k] = W.v[cc][k] + sum[cc][k];
        W.norm(a.n, false);
        W.store(wrow, a.n);
    };
    {  // the small segments, a wave each
        const int s = sb + w;
        if (s < se) {
            const int p0 = a.seg_start[s], p1 = a.seg_start[s + 1];
            if (p1 - p0 <= kWSmall) {
                T* wrow = a.w + (int64_t)(a.seg_row[s] - a.ne) * a.ld;
                RowReg<T, CH> W;
                W.load(wrow, a.n);  // (beside the event records)
                T acc[CH][kVec] = {};
                const bool act = add_events(p0, p1, acc);
                if (act) apply(W, wrow, acc);
            }
        }
    }
    if (a.clk && threadIdx.x == 0) {
        a.clk[4 * bid] = t_start;
        a.clk[4 * bid + 1] = wall_clock64();
    }
    for (int s = sb; s < se; ++s) {  // the large ones, all waves (uniform: every wave sees the sizes)
        const int p0 = a.seg_start[s], p1 = a.seg_start[s + 1];
        if (p1 - p0 <= kWSmall) continue;
        n_large += (1ull << 32) | (unsigned long long)(p1 - p0);
        if (threadIdx.x == 0) any = 0;
        __syncthreads();
        T* wrow = a.w + (int64_t)(a.seg_row[s] - a.ne) * a.ld;
        RowReg<T, CH> W;
        if (w == 0) W.load(wrow, a.n);
        // wave w: events [p0 + w S, p0 + (w + 1) S), 64 records a load
        const int S = (p1 - p0 + NWV - 1) / NWV;
        const int q0 = p0 + w * S, q1 = min(p1, q0 + S);
        T acc[CH][kVec] = {};
        bool act = false;
        for (int q = q0; q < q1; q += kWave) act |= add_events(q, min(q1, q + kWave), acc);
#pragma unroll
        for (int cc = 0; cc < CH; ++cc)
#pragma unroll
            for (int k = 0; k < kVec; ++k) part[w][cc * kVec + k][l] = acc[cc][k];
        if (act && l == 0) atomicOr(&any, 1);
        __syncthreads();
        if (w == 0 && any) {
            T sum[CH][kVec];
#pragma unroll
            for (int cc = 0; cc < CH; ++cc)
#pragma unroll
                for (int k = 0; k < kVec; ++k) {
                    sum[cc][k] = part[0][cc * kVec + k][l];
                    for (int v = 1; v < NWV; ++v) sum[cc][k] += part[v][cc * kVec + k][l];
                }
            apply(W, wrow, sum);
        }
        __syncthreads();  // (part and any: the next large segment's)
    }
    if (a.clk && threadIdx.x == 0) {
        a.clk[4 * bid + 2] = wall_clock64();
        a.clk[4 * bid + 3] = n_large;
    }
}

template <typename T, int CH, int NWV>
__global__ __launch_bounds__(NWV * kWave) void transh_w_apply_kernel(HParArgs<T> a) {
    transh_w_apply_body<T, CH, NWV>(a, blockIdx.x);
}

// Phase B's two sums in one launch (they touch disjoint tables): workgroups
// [0, wgrid) the relation normals (16 segments each), the rest the TransE apply of the h/t/r rows,
// so the hottest relation's normal overlaps the row sums instead of preceding them.
template <typename T, int CH>
__global__ __launch_bounds__(1024) void transh_phase_b_kernel(HParArgs<T> h, FoldArgs<T> fa, EventRecs er,
                                                             const int32_t* long_list, const int32_t* long_count,
                                                             int32_t cap, int32_t wgrid) {
    if ((int)blockIdx.x < wgrid) transh_w_apply_body<T, CH, 16>(h, blockIdx.x);
    else transe_apply_body<T, CH, true>(fa, er, long_list, long_count, cap, blockIdx.x - wgrid, gridDim.x - wgrid);
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
    if (l == 0) {
        a.orth_mask[kk] = (uint8_t)mask;
        if (mask) {  // the one-wave pass reads the ids here, one load level instead of three
            *reinterpret_cast<int4*>(a.orth_ids + (int64_t)kk * 8) = make_int4(r, h, t, nh);
            a.orth_ids[(int64_t)kk * 8 + 4] = nt;
        }
        const int ids[6] = {r, h, t, r, nh, nt};
        for (int q = 1; q < 6; ++q)
            if (q != 3 && ((mask >> q) & 1u)) orth_tag_entity(a, ids[q], r);
    }
}

// One wave, samples in order: the reference's normOrth (common/utils.cpp:79-111,
// orth_norm) on every flagged pair, in place on the live rows.  Per pass the
// flag words of 2048 samples are loaded at once and the flagged samples listed
// in sample order in LDS; their ids (r, h, t, h', t') are fetched for 64 list
// entries at a time, so the serial part is only the rows' load / normOrth /
// store.  w_r stays in registers while consecutive flagged samples share the
// relation (the reference reloads what it just stored), and a store is drained
// only before a later load of the same row (PendingRows).
constexpr int kOrthWords = 10;  // 8-byte flag words per lane per pass (5,120 samples: one pass on FB15k)
// normOrth iterations of the previous batch from which normOrth takes the relation pass
// (KB2E_HPAR_ORTH_MIN; a schedule choice only, the result is the same either way)
constexpr uint32_t kOrthRelMin = 64;

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

// Two sweeps in the order of the two-pass model: first the pairs only their own
// relation touches (the relation row, entity rows flagged under it alone), then
// the entity rows several relations flagged.  When transh_orth_rel_kernel ran, it
// has done the first sweep's pairs and cleared their bits; when the gate skipped
// it, this wave does them, in sample order -- the same result bit for bit, since
// the relations' own pairs touch disjoint rows and normals (their interleaving
// does not matter, only each relation's sample order).  So the gate on the
// previous batch's normOrth work (kOrthRelMin) is a schedule choice only.
//
// The first sweep queues the samples with shared rows (their ids and those rows'
// bits, in sample order) in LDS, so the second runs from the queue without
// listing the flags and fetching the ids again; past kOrthQ queued samples it
// lists them again.  Each group of samples runs pair by pair with the next pair's
// rows loaded ahead (process_group).
constexpr int kOrthQ = 512;

template <typename T, int CH>
__global__ __launch_bounds__(64) void transh_orth_fix_kernel(HParArgs<T> a) {
    __shared__ int list[8 * kWave * kOrthWords];
    __shared__ int queue[6][kOrthQ];  // second sweep: bits, r, h, t, h', t'
    __shared__ int plist[kWave * 5];  // a group's (row, w_r) pairs in order: entry << 3 | row
    const int l = lane_id();
    RowReg<T, CH> W;
    int wid = -1;
    PendingRows pend;
    uint32_t work = 0;  // normOrth iterations (the next batch's gate)
    int nq = 0;         // samples queued for the second sweep (> orth_q: list them again)
    // A group of up to 64 samples (lane e: its rows' bits over r, h, t, -, h', t' and their
    // ids), pair by pair in order: the next pair's row (and its w_r when the relation
    // changes) is loaded while this pair's normOrth runs, so the wave waits for a load
    // only when a pair re-reads the row just stored (then it keeps it in registers)
    auto process_group = [&](int ng, uint32_t bits, const int (&eid)[6]) {
        const uint32_t mb = l < ng ? bits & 0x37u : 0u;
        const int cnt = __builtin_popcount(mb);
        int pre = cnt;
#pragma unroll
        for (int d = 1; d < kWave; d <<= 1) {
            const int v = __shfl_up(pre, d);
            if (l >= d) pre += v;
        }
        {
            int pos = pre - cnt;
#pragma unroll
            for (int q = 0; q < 6; ++q)
                if ((mb >> q) & 1u) plist[pos++] = (l << 3) | q;
        }
        const int np = __shfl(pre, kWave - 1);
        wave_lds_sync();
        struct Pair {
            int er, q, key;
            T* row;
        };
        auto pair_at = [&](int p) {
            const int info = __builtin_amdgcn_readfirstlane(plist[p]);
            const int e = info >> 3, q = info & 7;
            Pair P;
            P.er = readlane_i32(eid[0], e);
            const int id = q == 0 ? P.er : readlane_i32(q == 1 ? eid[1] : q == 2 ? eid[2] : q == 4 ? eid[4] : eid[5], e);
            P.q = q;
            // keys: relations [0, nr), w rows [nr, 2 nr), entities from 2 nr
            P.key = q == 0 ? id : 2 * a.nr + id;
            P.row = (q == 0 ? a.rel : a.ent) + (int64_t)id * a.ld;
            return P;
        };
        if (np == 0) return;
        Pair cur = pair_at(0);
        RowReg<T, CH> A, An, Wn;
        pend.before_load(cur.key);
        row_load_sc1(A, cur.row, a.n);
        for (int p = 0; p < np; ++p) {
            if (cur.er != wid) {  // w_r: kept in registers while consecutive pairs share the relation
                if (wid >= 0) {
                    row_store_sc1(W, a.w + (int64_t)wid * a.ld, a.n);
                    pend.add(a.nr + wid);
                }
                pend.before_load(a.nr + cur.er);
                row_load_sc1(W, a.w + (int64_t)cur.er * a.ld, a.n);
                wid = cur.er;
            }
            const bool more = p + 1 < np;
            Pair nx{};
            bool pre_a = false, pre_w = false;
            if (more) {  // the next pair's rows in flight
                nx = pair_at(p + 1);
                pre_a = nx.key != cur.key;
                if (pre_a) {
                    pend.before_load(nx.key);
                    row_load_sc1(An, nx.row, a.n);
                }
                pre_w = nx.er != cur.er;
                if (pre_w) {
                    pend.before_load(a.nr + nx.er);
                    row_load_sc1(Wn, a.w + (int64_t)nx.er * a.ld, a.n);
                }
            }
            work += (uint32_t)orth_norm<T, CH>(A, W, a.n, (T)a.lr);
            row_store_sc1(A, cur.row, a.n);
            pend.add(cur.key);
            if (!more) break;
            if (pre_a) A = An;  // (else the same row: A holds what was just stored)
            if (pre_w) {
                row_store_sc1(W, a.w + (int64_t)wid * a.ld, a.n);
                pend.add(a.nr + wid);
                W = Wn;
                wid = nx.er;
            }
            cur = nx;
        }
        wave_lds_sync();  // (plist is rebuilt by the next group)
    };
    // a sweep over the flag words, samples in order (sweep 1 only when the queue overflowed)
    auto sweep_flags = [&](int sweep) {
        for (int base = 0; base < a.B; base += 8 * kWave * kOrthWords) {
            uint64_t word[kOrthWords];
#pragma unroll
            for (int wi = 0; wi < kOrthWords; ++wi) {  // (an 8-byte word at off < B: orth_mask is zero up to a multiple of 512)
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
            for (int g = 0; g < count; g += kWave) {
                int bits = 0;
                int eid[6] = {0, 0, 0, 0, 0, 0};
                uint32_t sh = 0;  // the entity rows several relations flagged (second sweep)
                if (g + l < count) {  // this lane's list entry: ids as the check kernel left them
                    const int k2 = list[g + l];
                    const int4 i4 = *reinterpret_cast<const int4*>(a.orth_ids + (int64_t)k2 * 8);
                    bits = a.orth_mask[k2];
                    eid[0] = i4.x;
                    eid[1] = i4.y;
                    eid[2] = i4.z;
                    eid[3] = i4.x;
                    eid[4] = i4.w;
                    eid[5] = a.orth_ids[(int64_t)k2 * 8 + 4];
#pragma unroll
                    for (int q = 1; q < 6; ++q)
                        if (q != 3 && ((bits >> q) & 1) && orth_shared(a, eid[q])) sh |= 1u << q;
                    bits = sweep == 0 ? bits & (int)~sh : (int)sh;
                }
                if (sweep == 0) {  // the shared rows' samples queued for the second sweep, in order
                    const uint64_t qm = __ballot(sh != 0);
                    const int qp = nq + __builtin_popcountll(qm & ((1ull << l) - 1ull));
                    if (sh != 0 && qp < a.orth_q) {
                        queue[0][qp] = (int)sh;
                        queue[1][qp] = eid[0];
                        queue[2][qp] = eid[1];
                        queue[3][qp] = eid[2];
                        queue[4][qp] = eid[4];
                        queue[5][qp] = eid[5];
                    }
                    nq += __builtin_popcountll(qm);
                }
                process_group(min(kWave, count - g), (uint32_t)bits, eid);
            }
            wave_lds_sync();
        }
    };
    sweep_flags(0);
    if (nq <= a.orth_q) {
        wave_lds_sync();
        for (int g = 0; g < nq; g += kWave) {  // the queue, 64 samples a group
            uint32_t bits = 0;
            int eid[6] = {0, 0, 0, 0, 0, 0};
            if (g + l < nq) {
                bits = (uint32_t)queue[0][g + l];
                eid[0] = eid[3] = queue[1][g + l];
                eid[1] = queue[2][g + l];
                eid[2] = queue[3][g + l];
                eid[4] = queue[4][g + l];
                eid[5] = queue[5][g + l];
            }
            process_group(min(kWave, nq - g), bits, eid);
        }
    } else {
        sweep_flags(1);
    }
    if (wid >= 0) row_store_sc1(W, a.w + (int64_t)wid * a.ld, a.n);
    drain_stores();
    if (l == 0) {
        atomicAdd(a.orth_work_cur, work);
        *a.orth_work_prev = 0;  // read by this batch's relation pass; the next batch counts into it
    }
}

// normOrth, first pass (oracle/parallel.py transh_parallel_batches): one wave per
// relation segment of the batch, its samples in order, on the pairs only this
// relation touches -- the relation row r' and the entity rows flagged under r
// alone -- with w_r in registers; those bits are cleared, so the one-wave
// serial pass (transh_orth_fix_kernel) then runs only the entity rows that
// several relations flagged.  The relations' passes touch disjoint rows.
template <typename T, int CH>
__global__ __launch_bounds__(256) void transh_orth_rel_kernel(HParArgs<T> a) {
    // little normOrth work in the previous batch: leave every pair to the one-wave pass
    if (*a.orth_work_prev < a.orth_rel_min) return;
    if (blockIdx.x == 0 && threadIdx.x == 0) atomicAdd(a.orth_rel_runs, 1u);  // (kb2e_counter)
    const int s = a.rel_begin[a.batch] + (int)blockIdx.x * 4 + (int)(threadIdx.x >> 6);
    if (s >= a.batch_seg[a.batch + 1]) return;
    const int l = lane_id();
    const int p0 = a.seg_start[s], p1 = a.seg_start[s + 1];
    const int r = a.seg_row[s] - a.ne;
    RowReg<T, CH> W;
    bool have_w = false;
    uint32_t work = 0;  // normOrth iterations (the next batch's gate)
    PendingRows pend;  // a row stored earlier is drained before it is loaded again
    for (int base = p0; base < p1; base += kWave) {
        // lane-parallel: this lane's sample (an active sample's first update event),
        // its flagged rows' ids and which of them only this relation touches
        const int p = base + l;
        uint32_t mine = 0;
        int ids[6] = {r, 0, 0, r, 0, 0};
        if (p < p1) {
            const int32_t meta = a.meta[p];
            const int xrow = meta >> 4;
            if (((meta & 3) - 1) != 0 && (xrow & 1) == 0) {
                const int kk = xrow >> 1;
                const uint32_t bits = a.orth_mask[kk];
                if (bits) {
                    const int i0 = a.si[kk], j = a.sj[kk];
                    const bool sd = a.side[kk];
                    const int h = a.heads[i0], t = a.tails[i0];
                    ids[1] = h;
                    ids[2] = t;
                    ids[4] = sd ? h : j;
                    ids[5] = sd ? j : t;
                    uint32_t keep = 0;
#pragma unroll
                    for (int q = 1; q < 6; ++q)
                        if (q != 3 && ((bits >> q) & 1u) && orth_shared(a, ids[q])) keep |= 1u << q;
                    mine = bits & ~keep;
                    if (mine) a.orth_mask[kk] = (uint8_t)keep;
                }
            }
        }
        // serial, samples in order: normOrth on this relation's own rows, w_r in registers
        uint64_t m = __ballot(mine != 0);
        while (m) {
            const int e = __builtin_ctzll(m);
            m &= m - 1;
            const uint32_t eb = (uint32_t)readlane_i32((int)mine, e);
            int rid[6];
#pragma unroll
            for (int q = 0; q < 6; ++q) rid[q] = readlane_i32(ids[q], e);
            if (!have_w) {
                row_load_sc1(W, a.w + (int64_t)r * a.ld, a.n);
                have_w = true;
            }
            for (int q = 0; q < 6; ++q) {
                if (!((eb >> q) & 1u)) continue;
                T* row = (q == 0 ? a.rel : a.ent) + (int64_t)rid[q] * a.ld;
                const int key = q == 0 ? -1 : rid[q];
                RowReg<T, CH> A;
                pend.before_load(key);
                row_load_sc1(A, row, a.n);
                work += (uint32_t)orth_norm<T, CH>(A, W, a.n, (T)a.lr);
                row_store_sc1(A, row, a.n);
                pend.add(key);
            }
        }
    }
    if (have_w) row_store_sc1(W, a.w + (int64_t)r * a.ld, a.n);
    drain_stores();
    if (work && l == 0) atomicAdd(a.orth_work_cur, work);
}


}  // namespace kb2e
