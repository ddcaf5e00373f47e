// kernels_relowner.hpp -- exact TransH / TransR batches: relation-owner
// dataflow with per-entity tickets.
//
// In TransH and TransR the reference couples rows inside a batch: after every
// gradientUpdate it re-orthogonalises entity rows against the relation's
// normal (transh/trainer.cpp:56-58, common/utils.cpp:79-111) or re-projects
// them through the relation matrix (transRNorm, transr/trainer.cpp:35-64,
// 185-187), and those loops also modify the relation state.  The order of
// updates therefore matters across rows.  We replay it exactly:
//
//   * every relation belongs to one persistent "owner" workgroup (LPT-balanced
//     on relation frequency); an owner replays its relations' updates in
//     global sample order, holding the relation state (r, w / Mr) itself;
//   * every entity row touched in the batch carries a ticket counter; an
//     update may touch entity e only when e's counter equals the number of
//     earlier active updates on e (computed by ticket_kernel from the sorted
//     event index), and bumps it afterwards.
//
// Because each owner walks its list in increasing global order and every
// dependency points to an earlier update, the earliest unfinished update is
// always runnable: no deadlock with all owners resident (grid <= #CUs, one
// workgroup per CU).  Entity rows move between owners through write-through
// (sc1) stores drained by s_waitcnt vmcnt(0) before an agent-scope atomic
// flag, and sc1 loads after the poll (MI355X_MICROARCH.md "Valid forms").
//
// Phase A (score) exports everything the updates need from the start-of-batch
// snapshot, so phase B never reads a snapshot row another owner may have
// already advanced.
#pragma once

#include <algorithm>
#include <numeric>
#include <vector>

#include "host_data.hpp"
#include "kernels_common.hpp"
#include "kernels_transe.hpp"

namespace kb2e {

struct RelOwnerPlan {
    int num_owners = 0;
    std::vector<int32_t> owner;  // relation -> owner
};

inline void plan_owners(RelOwnerPlan& p, const TripleStore& ts, int num_relations, int max_owners) {
    p.num_owners = std::max(1, std::min(num_relations, max_owners));
    std::vector<int> order(num_relations);
    std::iota(order.begin(), order.end(), 0);
    std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return ts.rel_count[a] > ts.rel_count[b]; });
    std::vector<int64_t> load(p.num_owners, 0);
    p.owner.assign(num_relations, 0);
    for (int r : order) {
        int best = (int)(std::min_element(load.begin(), load.end()) - load.begin());
        p.owner[r] = best;
        load[best] += ts.rel_count[r] + 1;
    }
}

// ------------------------------------------------------------- coherence

using gu64 = __attribute__((address_space(1))) uint64_t;
using gu32 = __attribute__((address_space(1))) uint32_t;

template <typename T>
__device__ __forceinline__ T load_sc1(const T* p) {
    if constexpr (sizeof(T) == 8) {
        const uint64_t b = __hip_atomic_load((gu64*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return __builtin_bit_cast(T, b);
    } else {
        const uint32_t b = __hip_atomic_load((gu32*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return __builtin_bit_cast(T, b);
    }
}

template <typename T>
__device__ __forceinline__ void store_sc1(T* p, T v) {
    if constexpr (sizeof(T) == 8)
        __hip_atomic_store((gu64*)p, __builtin_bit_cast(uint64_t, v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else
        __hip_atomic_store((gu32*)p, __builtin_bit_cast(uint32_t, v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <typename T, int CH>
__device__ __forceinline__ void row_load_sc1(RowReg<T, CH>& R, const T* row, int n) {
    const int l = lane_id();
#pragma unroll
    for (int c = 0; c < CH; ++c) {
        const int e = c * (kWave * kVec) + l * kVec;
        R.v[c][0] = e < n ? load_sc1(row + e) : T(0);
        R.v[c][1] = e + 1 < n ? load_sc1(row + e + 1) : T(0);
    }
}

template <typename T, int CH>
__device__ __forceinline__ void row_store_sc1(const RowReg<T, CH>& R, T* row, int n) {
    const int l = lane_id();
#pragma unroll
    for (int c = 0; c < CH; ++c) {
        const int e = c * (kWave * kVec) + l * kVec;
        if (e < n) store_sc1(row + e, R.v[c][0]);
        if (e + 1 < n) store_sc1(row + e + 1, R.v[c][1]);
    }
}

// Wait until done[e] == ticket (bounded; a timeout sets *err and gives up).  The
// bound is wall-clock time (wall_clock64 ticks, OwnerArgs::wait_ticks): a wait
// lasts at most as long as the dependency chain in front of it, which at wide
// dims is seconds (ORDERED TransR at dim 512 on the L2-resident matrix), so a
// spin count would time out on a healthy batch.
__device__ __forceinline__ bool wait_expired(uint32_t& spins, long long t0, uint64_t ticks) {
    return (++spins & 255u) == 0 && (uint64_t)(wall_clock64() - t0) > ticks;
}

__device__ __forceinline__ void wait_ticket(const uint32_t* done, int e, uint32_t ticket, uint32_t* err,
                                            uint64_t ticks) {
    uint32_t spins = 0;
    const long long t0 = wall_clock64();
    while (__hip_atomic_load((gu32*)(done + e), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != ticket) {
        __builtin_amdgcn_s_sleep(1);
        if (wait_expired(spins, t0, ticks)) {
            __hip_atomic_store((gu32*)err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            return;
        }
    }
}

__device__ __forceinline__ void release_ticket(uint32_t* done, int e, uint32_t ticket) {
    if (lane_id() == 0)
        __hip_atomic_store((gu32*)(done + e), ticket + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ void drain_stores() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// ------------------------------------------------------------- tickets

struct TicketArgs {
    const uint64_t* keys;
    const int32_t* seg_start;
    const int32_t* batch_seg;
    int32_t batch;
    KeyLayout kl;
    int32_t ne;
    const uint8_t* act;  // [B]
    uint32_t* tickets;   // [B][2][3]
    uint32_t* done;      // [ne]
};

// One wave per entity segment: ticket = number of earlier active updates on
// the entity in this batch; resets the entity's counter.
__global__ __launch_bounds__(256) void ticket_kernel(TicketArgs a) {
    const int s0 = a.batch_seg[a.batch], s1 = a.batch_seg[a.batch + 1];
    const int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int nwaves = (gridDim.x * blockDim.x) >> 6;
    const int l = lane_id();
    for (int s = s0 + wave; s < s1; s += nwaves) {
        const int p0 = a.seg_start[s], p1 = a.seg_start[s + 1];
        const int row = a.kl.row_of(a.keys[p0]);
        if (row >= a.ne) continue;  // owner segments
        if (l == 0) a.done[row] = 0;
        uint32_t count = 0;
        for (int base = p0; base < p1; base += kWave) {
            const int p = base + l;
            uint64_t key = 0;
            bool active = false;
            if (p < p1) {
                key = a.keys[p];
                active = a.act[a.kl.kk_of(key)] != 0;
            }
            const uint64_t m = __ballot(active);
            const uint32_t before = (uint32_t)__popcll(m & ((1ull << l) - 1ull));
            if (active) {
                const int kk = a.kl.kk_of(key), u = (int)((key >> 3) & 1);
                const uint32_t roles = (uint32_t)(key & 7);
                uint32_t* t = a.tickets + ((int64_t)kk * 2 + u) * 3;
                if (roles & kRoleHead) t[0] = count + before;
                if (roles & kRoleTail) t[1] = count + before;
                if (roles & kRoleEntRel) t[2] = count + before;
            }
            count += (uint32_t)__popcll(m);
        }
    }
}

// owner_seg[b * owners + o] = segment of owner o in batch b (or -1).
__global__ __launch_bounds__(256) void owner_seg_kernel(const uint64_t* keys, const int32_t* seg_start,
                                                        const int32_t* nseg_p, KeyLayout kl, int32_t ne,
                                                        int32_t owners, int32_t* owner_seg) {
    const int nseg = *nseg_p;
    for (int s = blockIdx.x * blockDim.x + threadIdx.x; s < nseg; s += gridDim.x * blockDim.x) {
        const uint64_t k = keys[seg_start[s]];
        const int row = kl.row_of(k);
        if (row >= ne) owner_seg[(int64_t)kl.batch_of(k) * owners + (row - ne)] = s;
    }
}

// ---------------------------------------------------------- TransH phase A

template <typename T>
struct HScoreArgs {
    const int32_t* heads;
    const int32_t* tails;
    const int32_t* rels;
    const int32_t* si;
    const int32_t* sj;
    const uint8_t* side;
    int32_t B, n, ld, nw;
    const T* ent;
    const T* rel;
    const T* w;
    double margin;
    uint8_t* act;
    double* loss;
    uint64_t* xbits;  // [B][2][nw]
    T* scal;          // [B][2][4]: headSum, tailSum, sum_x
    T* snap;          // [B][2][2][ld]: snapshot head row, tail row; EMIT: [B][2][ld] w deltas
    double lr;        // EMIT: the w deltas' beta lr
};

// transh/transh.cpp:10-29 energies, transh/trainer.cpp:14-33 directions.
// EMIT (PARALLEL schedule): also the event records of the h/t/r updates, whose
// deltas are TransE's (transh/trainer.cpp:34-37; kernels_transe.hpp EventSlot).
template <typename T, int CH, bool EMIT = false>
__global__ __launch_bounds__(256) void transh_score_kernel(HScoreArgs<T> a, EventRecs er = {}, KeyLayout kl = {},
                                                           int64_t kbase = 0, int32_t ne = 0) {
    const int kk = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (kk >= a.B) return;
    const int l = lane_id();
    EventSlot slot;
    if (EMIT) slot.prefetch(er, kbase + kk);
    const int i = a.si[kk], j = a.sj[kk];
    const int h = a.heads[i], t = a.tails[i], r = a.rels[i];
    const int nh = a.side[kk] ? h : j, nt = a.side[kk] ? j : t;
    RowReg<T, CH> H, Tt, R, W, NH, NT;
    H.load(a.ent + (int64_t)h * a.ld, a.n);
    Tt.load(a.ent + (int64_t)t * a.ld, a.n);
    R.load(a.rel + (int64_t)r * a.ld, a.n);
    W.load(a.w + (int64_t)r * a.ld, a.n);
    NH.load(a.ent + (int64_t)nh * a.ld, a.n);
    NT.load(a.ent + (int64_t)nt * a.ld, a.n);
    T hs_p = T(0), ts_p = T(0), hs_n = T(0), ts_n = T(0);
#pragma unroll
    for (int c = 0; c < CH; ++c)
#pragma unroll
        for (int k = 0; k < kVec; ++k) {
            hs_p += W.v[c][k] * H.v[c][k];
            ts_p += W.v[c][k] * Tt.v[c][k];
            hs_n += W.v[c][k] * NH.v[c][k];
            ts_n += W.v[c][k] * NT.v[c][k];
        }
    hs_p = wave_sum(hs_p);
    ts_p = wave_sum(ts_p);
    hs_n = wave_sum(hs_n);
    ts_n = wave_sum(ts_n);
    T dp[CH][kVec], dn[CH][kVec];
    T ep = T(0), en = T(0);
#pragma unroll
    for (int c = 0; c < CH; ++c)
#pragma unroll
        for (int k = 0; k < kVec; ++k) {
            dp[c][k] = Tt.v[c][k] - ts_p * W.v[c][k] - (H.v[c][k] - hs_p * W.v[c][k]) - R.v[c][k];
            dn[c][k] = NT.v[c][k] - ts_n * W.v[c][k] - (NH.v[c][k] - hs_n * W.v[c][k]) - R.v[c][k];
            ep += fabs(dp[c][k]);
            en += fabs(dn[c][k]);
        }
    ep = wave_sum(ep);
    en = wave_sum(en);
    const double e_pos = (double)ep, e_neg = (double)en;
    const bool active = e_pos + a.margin > e_neg;
    if (l == 0) {
        a.act[kk] = active ? 1 : 0;
        a.loss[kk] = active ? a.margin + e_pos - e_neg : 0.0;
    }
    uint64_t bpw[CH * kVec], bnw[CH * kVec];
    if (!active) {
        if (EMIT) slot.write<CH * kVec>(er, kl, ne, kk, false, bpw, bnw, a.nw);
        return;
    }
    // sum_x = sum_i x_i w_i with x_i = +-1 (transh/trainer.cpp:33)
    T sx_p = T(0), sx_n = T(0);
#pragma unroll
    for (int c = 0; c < CH; ++c)
#pragma unroll
        for (int k = 0; k < kVec; ++k) {
            if (!elem_valid(c, k, a.n)) continue;
            sx_p += (dp[c][k] > T(0) ? T(1) : T(-1)) * W.v[c][k];
            sx_n += (dn[c][k] > T(0) ? T(1) : T(-1)) * W.v[c][k];
        }
    sx_p = wave_sum(sx_p);
    sx_n = wave_sum(sx_n);
#pragma unroll
    for (int c = 0; c < CH; ++c)
#pragma unroll
        for (int k = 0; k < kVec; ++k) {
            const bool valid = elem_valid(c, k, a.n);
            const uint64_t bp = __ballot(valid && dp[c][k] > T(0));
            const uint64_t bn = __ballot(valid && dn[c][k] > T(0));
            bpw[c * kVec + k] = bp;
            bnw[c * kVec + k] = bn;
            if (l == 0) {
                a.xbits[((int64_t)kk * 2 + 0) * a.nw + c * kVec + k] = bp;
                a.xbits[((int64_t)kk * 2 + 1) * a.nw + c * kVec + k] = bn;
            }
        }
    if (EMIT) slot.write<CH * kVec>(er, kl, ne, kk, true, bpw, bnw, a.nw);
    if (l == 0) {
        T* s0 = a.scal + ((int64_t)kk * 2 + 0) * 4;
        T* s1 = a.scal + ((int64_t)kk * 2 + 1) * 4;
        s0[0] = hs_p; s0[1] = ts_p; s0[2] = sx_p;
        s1[0] = hs_n; s1[1] = ts_n; s1[2] = sx_n;
    }
    if (EMIT) {
        // PARALLEL: each update's w delta  beta lr ((hs - ts) x + sum_x (h - t))
        // (transh/trainer.cpp:39-46), the expression transh_w_apply_kernel sums
        const T cp = (T)(-1.0 * a.lr), cn = (T)(1.0 * a.lr);
        RowReg<T, CH> Dp, Dn;
#pragma unroll
        for (int c = 0; c < CH; ++c)
#pragma unroll
            for (int k = 0; k < kVec; ++k) {
                const T xp = dp[c][k] > T(0) ? T(1) : T(-1), xn = dn[c][k] > T(0) ? T(1) : T(-1);
                Dp.v[c][k] = cp * ((hs_p - ts_p) * xp + sx_p * (H.v[c][k] - Tt.v[c][k]));
                Dn.v[c][k] = cn * ((hs_n - ts_n) * xn + sx_n * (NH.v[c][k] - NT.v[c][k]));
            }
        Dp.store(a.snap + ((int64_t)kk * 2 + 0) * a.ld, a.n);
        Dn.store(a.snap + ((int64_t)kk * 2 + 1) * a.ld, a.n);
        return;
    }
    H.store(a.snap + (((int64_t)kk * 2 + 0) * 2 + 0) * a.ld, a.n);
    Tt.store(a.snap + (((int64_t)kk * 2 + 0) * 2 + 1) * a.ld, a.n);
    NH.store(a.snap + (((int64_t)kk * 2 + 1) * 2 + 0) * a.ld, a.n);
    NT.store(a.snap + (((int64_t)kk * 2 + 1) * 2 + 1) * a.ld, a.n);
}

// common/utils.cpp:79-111 norm(a, b, rate) on registers, with the
// reference's running `sum` (never reset between iterations).  Returns the
// iterations run (the test included; wave-uniform).
template <typename T, int CH>
__device__ __forceinline__ int orth_norm(RowReg<T, CH>& A, RowReg<T, CH>& Bv, int n, T rate) {
    Bv.norm(n, false);
    T sum = T(0);
    int it = 0;
    for (; it < 1 << 20; ++it) {
        sum += Bv.sumsq();
        sum = sqrt(sum);
#pragma unroll
        for (int c = 0; c < CH; ++c)
#pragma unroll
            for (int k = 0; k < kVec; ++k)
                if (elem_valid(c, k, n)) Bv.v[c][k] = Bv.v[c][k] / sum;
        T x = T(0);
#pragma unroll
        for (int c = 0; c < CH; ++c)
#pragma unroll
            for (int k = 0; k < kVec; ++k) x += Bv.v[c][k] * A.v[c][k];
        x = wave_sum(x);
        if (!(x > T(0.1))) break;
#pragma unroll
        for (int c = 0; c < CH; ++c)
#pragma unroll
            for (int k = 0; k < kVec; ++k) {
                if (!elem_valid(c, k, n)) continue;
                A.v[c][k] = A.v[c][k] - rate * Bv.v[c][k];
                Bv.v[c][k] = Bv.v[c][k] - rate * A.v[c][k];
            }
    }
    Bv.norm(n, false);
    return it + 1;
}


// ---------------------------------------------------------- TransH phase B

template <typename T>
struct OwnerArgs {
    const uint64_t* keys;
    const int32_t* seg_start;
    const int32_t* owner_seg;  // [nb][owners]
    int32_t batch, owners;
    KeyLayout kl;
    int32_t n, ld, nw;
    const int32_t* heads;
    const int32_t* tails;
    const int32_t* rels;
    const int32_t* si;
    const int32_t* sj;
    const uint8_t* side;
    const uint8_t* act;
    const uint32_t* tickets;
    uint32_t* done;
    uint32_t* err;
    uint64_t wait_ticks;  // a ticket wait gives up after this many wall_clock64 ticks (the host: 600 s)
    T* ent;
    T* rel;
    T* w;        // TransH normals (live) / TransR matrices: next (W_B)
    const T* wsnap;  // TransR: matrices at batch start (W_A)
    uint32_t* wtouched;  // TransR: relation -> batch stamp
    double lr;
    const uint64_t* xbits;
    const T* xreal;
    const T* scal;
    const T* snap;
    const int32_t* batch_seg;
    uint4* desc;         // TransR: per-position update descriptors of this batch
};

struct UpdateIds {
    int kk, u, r;
    int ent[3];       // distinct entities (head first), -1 unused
    uint32_t roles[3];
    uint32_t tick[3];
    int count;
};

template <typename T>
__device__ __forceinline__ UpdateIds decode_update(const OwnerArgs<T>& a, uint64_t key, bool entrel) {
    UpdateIds d;
    d.kk = a.kl.kk_of(key);
    d.u = (int)((key >> 3) & 1);
    const int i = a.si[d.kk], j = a.sj[d.kk];
    const int h = a.heads[i], t = a.tails[i];
    d.r = a.rels[i];
    int eh = h, et = t;
    if (d.u == 1) {
        if (a.side[d.kk]) et = j;
        else eh = j;
    }
    const int ids[3] = {eh, et, entrel ? d.r : -1};
    const uint32_t rl[3] = {kRoleHead, kRoleTail, kRoleEntRel};
    const uint32_t* tk = a.tickets + ((int64_t)d.kk * 2 + d.u) * 3;
    d.count = 0;
    for (int q = 0; q < 3; ++q) {
        if (ids[q] < 0) continue;
        int found = -1;
        for (int p = 0; p < d.count; ++p)
            if (d.ent[p] == ids[q]) found = p;
        if (found >= 0) {
            d.roles[found] |= rl[q];
        } else {
            d.ent[d.count] = ids[q];
            d.roles[d.count] = rl[q];
            d.tick[d.count] = tk[q];
            ++d.count;
        }
    }
    return d;
}

// Descriptor of update (kk, u) at key position p: 3 x uint4
//   q0 = {kk, u | count << 2 | roles0 << 4 | roles1 << 8 | roles2 << 12, r, 0}
//   q1 = {ent0, ent1, ent2, 0}      q2 = {tick0, tick1, tick2, 0}
// count == 0 marks an inactive update.
template <typename T>
__global__ __launch_bounds__(256) void relowner_desc_kernel(OwnerArgs<T> a, int32_t ne, int32_t entrel) {
    const int pb0 = a.seg_start[a.batch_seg[a.batch]];
    const int pb1 = a.seg_start[a.batch_seg[a.batch + 1]];
    for (int p = pb0 + blockIdx.x * blockDim.x + threadIdx.x; p < pb1; p += gridDim.x * blockDim.x) {
        const uint64_t key = a.keys[p];
        if (a.kl.row_of(key) < ne) continue;  // entity events
        uint4* out = a.desc + (int64_t)(p - pb0) * 3;
        const int kk = a.kl.kk_of(key);
        if (!a.act[kk]) {
            out[0] = make_uint4((uint32_t)kk, 0u, 0u, 0u);
            continue;
        }
        const UpdateIds d = decode_update(a, key, entrel != 0);
        uint32_t packed = (uint32_t)d.u | ((uint32_t)d.count << 2);
        for (int q = 0; q < d.count; ++q) packed |= d.roles[q] << (4 + 4 * q);
        out[0] = make_uint4((uint32_t)kk, packed, (uint32_t)d.r, 0u);
        out[1] = make_uint4((uint32_t)d.ent[0], d.count > 1 ? (uint32_t)d.ent[1] : 0u,
                            d.count > 2 ? (uint32_t)d.ent[2] : 0u, 0u);
        out[2] = make_uint4(d.tick[0], d.count > 1 ? d.tick[1] : 0u, d.count > 2 ? d.tick[2] : 0u, 0u);
    }
}

// Per owner: the active descriptors of its segment, in order, packed to the
// front of the segment's slice (cdesc[(p0 - pb0) + i]), and their count.
__global__ __launch_bounds__(256) void relowner_compact_kernel(const int32_t* owner_seg, const int32_t* seg_start,
                                                             const int32_t* batch_seg, int32_t batch, int32_t owners,
                                                             const uint4* desc, uint4* cdesc, int32_t* ocount) {
    __shared__ int wave_tot[4];
    const int o = blockIdx.x;
    const int seg = owner_seg[(int64_t)batch * owners + o];
    if (seg < 0) {
        if (threadIdx.x == 0) ocount[o] = 0;
        return;
    }
    const int p0 = seg_start[seg], p1 = seg_start[seg + 1];
    const int pb0 = seg_start[batch_seg[batch]];
    const int base = p0 - pb0;
    const int wv = threadIdx.x >> 6, l = lane_id();
    int running = 0;
    for (int chunk = p0; chunk < p1; chunk += 256) {
        const int p = chunk + threadIdx.x;
        uint4 q0{}, q1{}, q2{};
        bool active = false;
        if (p < p1) {
            const uint4* d = desc + (int64_t)(p - pb0) * 3;
            q0 = d[0];
            active = ((q0.y >> 2) & 3u) != 0;
            if (active) {
                q1 = d[1];
                q2 = d[2];
            }
        }
        const uint64_t m = __ballot(active);
        if (l == 0) wave_tot[wv] = __popcll(m);
        __syncthreads();
        int before = __popcll(m & ((1ull << l) - 1ull));
        for (int k = 0; k < wv; ++k) before += wave_tot[k];
        const int total = wave_tot[0] + wave_tot[1] + wave_tot[2] + wave_tot[3];
        if (active) {
            uint4* out = cdesc + (int64_t)(base + running + before) * 3;
            out[0] = q0;
            out[1] = q1;
            out[2] = q2;
        }
        running += total;
        __syncthreads();
    }
    if (threadIdx.x == 0) ocount[o] = running;
}

__device__ __forceinline__ uint32_t uni(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); }

// Wait until done[e_q] == tick_q for every slot (polls issued together).
__device__ __forceinline__ void wait_tickets3(const uint32_t* done, int count, const uint32_t* e, const uint32_t* tk,
                                              uint32_t* err, uint64_t ticks) {
    uint32_t spins = 0;
    const long long t0 = wall_clock64();
    for (;;) {
        const uint32_t f0 = __hip_atomic_load((gu32*)(done + e[0]), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const uint32_t f1 = count > 1 ? __hip_atomic_load((gu32*)(done + e[1]), __ATOMIC_RELAXED,
                                                          __HIP_MEMORY_SCOPE_AGENT) : tk[1];
        const uint32_t f2 = count > 2 ? __hip_atomic_load((gu32*)(done + e[2]), __ATOMIC_RELAXED,
                                                          __HIP_MEMORY_SCOPE_AGENT) : tk[2];
        if (f0 == tk[0] && f1 == tk[1] && f2 == tk[2]) return;
        __builtin_amdgcn_s_sleep(1);
        if (wait_expired(spins, t0, ticks)) {
            __hip_atomic_store((gu32*)err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            return;
        }
    }
}

// common::norm on independent rows at once (the reductions overlap): the
// first rows with ignoreShort = true, the last one (w) with false.
template <typename T, int CH>
__device__ __forceinline__ void scale_row(RowReg<T, CH>& A, T len, bool apply, int n) {
    if (!apply) return;
    const T inv = T(1) / len;  // a / len exactly, via the correctly rounded reciprocal (div_markstein)
#pragma unroll
    for (int c = 0; c < CH; ++c)
#pragma unroll
        for (int k = 0; k < kVec; ++k)
            if (elem_valid(c, k, n)) A.v[c][k] = div_markstein(A.v[c][k], len, inv);
}
template <typename T, int CH>
__device__ __forceinline__ void norm_rows3(RowReg<T, CH>& A, RowReg<T, CH>& B, RowReg<T, CH>& Wn, int n) {
    T sa = T(0), sb = T(0), sw = T(0);
#pragma unroll
    for (int c = 0; c < CH; ++c)
#pragma unroll
        for (int k = 0; k < kVec; ++k) {
            sa += A.v[c][k] * A.v[c][k];
            sb += B.v[c][k] * B.v[c][k];
            sw += Wn.v[c][k] * Wn.v[c][k];
        }
    const T la = sqrt(wave_sum(sa)), lb = sqrt(wave_sum(sb)), lw = sqrt(wave_sum(sw));
    scale_row(A, la, la > T(1), n);
    scale_row(B, lb, lb > T(1), n);
    scale_row(Wn, lw, true, n);
}
template <typename T, int CH>
__device__ __forceinline__ void norm_rows4(RowReg<T, CH>& A, RowReg<T, CH>& B, RowReg<T, CH>& C,
                                           RowReg<T, CH>& Wn, int n) {
    T sa = T(0), sb = T(0), sc = T(0), sw = T(0);
#pragma unroll
    for (int c = 0; c < CH; ++c)
#pragma unroll
        for (int k = 0; k < kVec; ++k) {
            sa += A.v[c][k] * A.v[c][k];
            sb += B.v[c][k] * B.v[c][k];
            sc += C.v[c][k] * C.v[c][k];
            sw += Wn.v[c][k] * Wn.v[c][k];
        }
    const T la = sqrt(wave_sum(sa)), lb = sqrt(wave_sum(sb)), lc = sqrt(wave_sum(sc)), lw = sqrt(wave_sum(sw));
    scale_row(A, la, la > T(1), n);
    scale_row(B, lb, lb > T(1), n);
    scale_row(C, lc, lc > T(1), n);
    scale_row(Wn, lw, true, n);
}

// Per-update inputs of a TransH update exported by phase A.
template <typename T, int CH>
struct HUpdateIn {
    RowReg<T, CH> SH, ST;  // snapshot head / tail rows
    uint64_t words[2 * CH];
    T hs, ts, sumx;
    __device__ __forceinline__ void load(const OwnerArgs<T>& a, uint4 q0, int n) {
        const int kk = (int)uni(q0.x), u = (int)(uni(q0.y) & 1);
        const int64_t ku = (int64_t)kk * 2 + u;
        SH.load(a.snap + (ku * 2 + 0) * a.ld, n);
        ST.load(a.snap + (ku * 2 + 1) * a.ld, n);
        const uint64_t* xw = a.xbits + ku * a.nw;
#pragma unroll
        for (int q = 0; q < 2 * CH; ++q) words[q] = xw[q];
        const T* sc = a.scal + ku * 4;
        hs = sc[0];
        ts = sc[1];
        sumx = sc[2];
    }
};

// One persistent workgroup per owner walks its compacted update list; the
// relation state (r, w) stays in registers while consecutive updates share the
// relation, and the next update's descriptor and phase-A inputs are loaded
// during the current one.  Entity rows move through tickets as documented at
// the top of this file.
template <typename T, int CH>
__global__ __launch_bounds__(64) void transh_owner_kernel(OwnerArgs<T> a, const uint4* cdesc, const int32_t* ocount) {
    const int seg = a.owner_seg[(int64_t)a.batch * a.owners + blockIdx.x];
    if (seg < 0) return;
    const int m = ocount[blockIdx.x];
    const uint4* dl0 = cdesc + (int64_t)(a.seg_start[seg] - a.seg_start[a.batch_seg[a.batch]]) * 3;
    const int n = a.n;
    const T lr = (T)a.lr;
#ifdef KB2E_OWNER_PROF
    PhaseClock pc;
    pc.start();
#endif
    RowReg<T, CH> R, W;
    int cur = -1;
    // pipeline: descriptors run two updates ahead, phase-A inputs one ahead
    uint4 n0{}, n1{}, n2{}, f0{}, f1{}, f2{};
    HUpdateIn<T, CH> nin;
    if (m > 0) {
        n0 = dl0[0];
        n1 = dl0[1];
        n2 = dl0[2];
        nin.load(a, n0, n);
    }
    if (m > 1) {
        f0 = dl0[3];
        f1 = dl0[4];
        f2 = dl0[5];
    }
    for (int it = 0; it < m; ++it) {
        const uint4 q0 = n0, q1 = n1, q2 = n2;
        const HUpdateIn<T, CH> in = nin;
        n0 = f0;
        n1 = f1;
        n2 = f2;
        if (it + 2 < m) {
            const uint4* dn = dl0 + (int64_t)(it + 2) * 3;
            f0 = dn[0];
            f1 = dn[1];
            f2 = dn[2];
        }
        const uint32_t packed = uni(q0.y);
        const int count = (int)((packed >> 2) & 3);
        const int u = (int)(packed & 1), r = (int)uni(q0.z);
        const uint32_t ent[3] = {uni(q1.x), uni(q1.y), 0u};
        const uint32_t tk[3] = {uni(q2.x), uni(q2.y), 0u};
        if (r != cur) {
            if (cur >= 0) {
                R.store(a.rel + (int64_t)cur * a.ld, n);
                W.store(a.w + (int64_t)cur * a.ld, n);
            }
            drain_stores();  // a relation met again re-reads what this wave stored
            row_load_sc1(R, a.rel + (int64_t)r * a.ld, n);
            row_load_sc1(W, a.w + (int64_t)r * a.ld, n);
            cur = r;
        }
        if (it + 1 < m) nin.load(a, n0, n);
        OWNER_MARK(0);
        wait_tickets3(a.done, count, ent, tk, a.err, a.wait_ticks);
        OWNER_MARK(1);
        RowReg<T, CH> E0, E1;
        row_load_sc1(E0, a.ent + (int64_t)ent[0] * a.ld, n);
        if (count > 1) row_load_sc1(E1, a.ent + (int64_t)ent[1] * a.ld, n);
        else E1.load(nullptr, 0);  // zeros
        // head row = E0; tail row = E0 (h == t) or E1
        const bool same = count == 1;
        const T beta = u ? T(1) : T(-1);
        const T blr = beta * lr;  // beta * learningRate_
        OWNER_MARK(2);
        // transh/trainer.cpp:23-41
#pragma unroll
        for (int c = 0; c < CH; ++c)
#pragma unroll
            for (int k = 0; k < kVec; ++k) {
                if (!elem_valid(c, k, n)) continue;
                const T x = xbit(in.words, c, k) ? T(1) : T(-1);
                const T dlt = blr * x;
                R.v[c][k] = R.v[c][k] - dlt;
                E0.v[c][k] = E0.v[c][k] - dlt;
                if (same) E0.v[c][k] = E0.v[c][k] + dlt;
                else E1.v[c][k] = E1.v[c][k] + dlt;
                W.v[c][k] = W.v[c][k] + dlt * in.hs;
                W.v[c][k] = W.v[c][k] - dlt * in.ts;
            }
        // transh/trainer.cpp:43-46
        const T g = blr * in.sumx;
#pragma unroll
        for (int c = 0; c < CH; ++c)
#pragma unroll
            for (int k = 0; k < kVec; ++k) {
                if (!elem_valid(c, k, n)) continue;
                W.v[c][k] = W.v[c][k] + g * in.SH.v[c][k];
                W.v[c][k] = W.v[c][k] - g * in.ST.v[c][k];
            }
        OWNER_MARK(3);
        // transh/trainer.cpp:48-58: norm(r), norm(h), norm(t), norm(w, false),
        // then normOrth (common/utils.cpp:79-111) of r, h, t against w.
        // normOrth only moves a row when x = w.row > 0.1, which is rare; all
        // norms and the three x come from one round of raw sums, so the common
        // case costs one (7-way interleaved) reduction round.  There r', h', t'
        // get exactly the reference's single division by their length, and w'
        // is divided by its length once: the reference's further divisions of
        // w' by its (already unit) length inside normOrth are 1 +- ulp and are
        // the only difference.  Any x > 0.1 replays the reference's sequence
        // step by step on the untouched rows.
        T sR = T(0), s0 = T(0), s1 = T(0), sW = T(0), dR = T(0), d0 = T(0), d1 = T(0);
#pragma unroll
        for (int c = 0; c < CH; ++c)
#pragma unroll
            for (int k = 0; k < kVec; ++k) {
                sR += R.v[c][k] * R.v[c][k];
                s0 += E0.v[c][k] * E0.v[c][k];
                s1 += E1.v[c][k] * E1.v[c][k];
                sW += W.v[c][k] * W.v[c][k];
                dR += W.v[c][k] * R.v[c][k];
                d0 += W.v[c][k] * E0.v[c][k];
                d1 += W.v[c][k] * E1.v[c][k];
            }
        sR = wave_sum(sR);
        s0 = wave_sum(s0);
        s1 = wave_sum(s1);
        sW = wave_sum(sW);
        dR = wave_sum(dR);
        d0 = wave_sum(d0);
        d1 = wave_sum(d1);
        const T lR = sqrt(sR), l0 = sqrt(s0), l1 = sqrt(s1), lW = sqrt(sW);
        const T cR = lR > T(1) ? lR : T(1), c0 = l0 > T(1) ? l0 : T(1), c1 = l1 > T(1) ? l1 : T(1);
        // x = w.row / (|w| c) <= 0.1 (decisions only: compared by multiplication)
        const bool fast = dR <= T(0.1) * (lW * cR) && d0 <= T(0.1) * (lW * c0) &&
                          (same || d1 <= T(0.1) * (lW * c1));
        OWNER_MARK(4);
        if (fast) {
            scale_row(R, lR, lR > T(1), n);
            scale_row(E0, l0, l0 > T(1), n);
            if (same) E0.norm(n, true);
            else scale_row(E1, l1, l1 > T(1), n);
            scale_row(W, lW, true, n);
            OWNER_MARK(6);
        } else {
            if (same) {
                norm_rows3(R, E0, W, n);
                E0.norm(n, true);
            } else {
                norm_rows4(R, E0, E1, W, n);
            }
            orth_norm(R, W, n, lr);
            orth_norm(E0, W, n, lr);
            if (same) orth_norm(E0, W, n, lr);
            else orth_norm(E1, W, n, lr);
            OWNER_MARK(7);
        }
        row_store_sc1(E0, a.ent + (int64_t)ent[0] * a.ld, n);
        if (!same) row_store_sc1(E1, a.ent + (int64_t)ent[1] * a.ld, n);
        drain_stores();
        release_ticket(a.done, (int)ent[0], tk[0]);
        if (!same) release_ticket(a.done, (int)ent[1], tk[1]);
        OWNER_MARK(8);
        OWNER_COUNT(11);
    }
    if (cur >= 0) {
        R.store(a.rel + (int64_t)cur * a.ld, n);
        W.store(a.w + (int64_t)cur * a.ld, n);
    }
#ifdef KB2E_OWNER_PROF
    pc.flush(blockIdx.x < kProfOwners ? g_owner_prof[blockIdx.x] : nullptr);
#endif
}


// ---------------------------------------------------------- TransR phase A

template <typename T>
struct RScoreArgs {
    const int32_t* heads;
    const int32_t* tails;
    const int32_t* rels;
    const int32_t* si;
    const int32_t* sj;
    const uint8_t* side;
    int32_t B, n, ld;
    const T* ent;
    const T* rel;
    const T* W;       // matrices at batch start, rows [r * n + j] of length ld
    double margin;
    int32_t compat, l1;
    uint8_t* act;
    double* loss;
    T* x;             // [B][2][ld] update directions (+-1 for L1)
    T* d;             // [B][2][ld] snapshot head - tail
    double* proj;     // [B][2][2][ld] W^T head, W^T tail per energy call (compat)
};

// transr/transr.cpp:13-37 (projections summed over j in the reference's order)
// and transr/trainer.cpp:147-164 (x from fresh projections).
template <typename T, int CH>
__global__ __launch_bounds__(256) void transr_project_kernel(RScoreArgs<T> a) {
    const int kk = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (kk >= a.B) return;
    const int l = lane_id();
    const int n = a.n;
    const int i0 = a.si[kk], jj = a.sj[kk];
    const int h = a.heads[i0], t = a.tails[i0], r = a.rels[i0];
    const int nh = a.side[kk] ? h : jj, nt = a.side[kk] ? jj : t;
    const T* eh = a.ent + (int64_t)h * a.ld;
    const T* et = a.ent + (int64_t)t * a.ld;
    const T* enh = a.ent + (int64_t)nh * a.ld;
    const T* ent_ = a.ent + (int64_t)nt * a.ld;
    const T* Wr = a.W + (int64_t)r * n * a.ld;
    T ph[CH][kVec], pt[CH][kVec], pnh[CH][kVec], pnt[CH][kVec];
#pragma unroll
    for (int c = 0; c < CH; ++c)
#pragma unroll
        for (int k = 0; k < kVec; ++k) ph[c][k] = pt[c][k] = pnh[c][k] = pnt[c][k] = T(0);
    for (int j = 0; j < n; ++j) {
        const T hj = eh[j], tj = et[j], nhj = enh[j], ntj = ent_[j];
        const T* wrow = Wr + (int64_t)j * a.ld;
#pragma unroll
        for (int c = 0; c < CH; ++c) {
            const int e = c * (kWave * kVec) + l * kVec;
            if (e >= n) continue;
            const T w0 = wrow[e], w1 = wrow[e + 1];  // ld even: pair stays in the row
            ph[c][0] += w0 * hj; ph[c][1] += w1 * hj;
            pt[c][0] += w0 * tj; pt[c][1] += w1 * tj;
            pnh[c][0] += w0 * nhj; pnh[c][1] += w1 * nhj;
            pnt[c][0] += w0 * ntj; pnt[c][1] += w1 * ntj;
        }
    }
    RowReg<T, CH> R;
    R.load(a.rel + (int64_t)r * a.ld, n);
    T ep = T(0), en = T(0);
#pragma unroll
    for (int c = 0; c < CH; ++c)
#pragma unroll
        for (int k = 0; k < kVec; ++k) {
            const int e = c * (kWave * kVec) + l * kVec + k;
            if (e >= n) continue;
            const T dp = pt[c][k] - ph[c][k] - R.v[c][k];
            const T dn = pnt[c][k] - pnh[c][k] - R.v[c][k];
            ep += a.l1 ? fabs(dp) : dp * dp;
            en += a.l1 ? fabs(dn) : dn * dn;
            T xp = T(2.0) * dp, xn = T(2.0) * dn;
            if (a.l1) {
                xp = xp > T(0) ? T(1) : T(-1);
                xn = xn > T(0) ? T(1) : T(-1);
            }
            a.x[((int64_t)kk * 2 + 0) * a.ld + e] = xp;
            a.x[((int64_t)kk * 2 + 1) * a.ld + e] = xn;
            a.d[((int64_t)kk * 2 + 0) * a.ld + e] = eh[e] - et[e];
            a.d[((int64_t)kk * 2 + 1) * a.ld + e] = enh[e] - ent_[e];
            if (a.compat) {
                double* pr = a.proj + ((int64_t)kk * 2 + 0) * 2 * a.ld;
                pr[e] = (double)ph[c][k];
                pr[a.ld + e] = (double)pt[c][k];
                pr[2 * a.ld + e] = (double)pnh[c][k];
                pr[3 * a.ld + e] = (double)pnt[c][k];
            }
        }
    if (a.compat) return;  // energies come from the scanned work vectors
    ep = wave_sum(ep);
    en = wave_sum(en);
    const double e_pos = (double)ep, e_neg = (double)en;
    const bool active = e_pos + a.margin > e_neg;
    if (l == 0) {
        a.act[kk] = active ? 1 : 0;
        a.loss[kk] = active ? a.margin + e_pos - e_neg : 0.0;
    }
}

// Compat mode: the reference's work vectors accumulate every energy call's
// projection and are never zeroed (transr/transr.cpp:20-25, trainer.h:28-29),
// so call c sees hv = hv0 + sum_{c' <= c} W^T h_c'.  One wave per element i
// scans the batch's 2B calls in order (pos before neg) and carries the
// process-lifetime state in `work` ([2][n]: head, tail).
__global__ __launch_bounds__(64) void transr_compat_scan_kernel(double* proj, int32_t B, int32_t ld, int32_t n,
                                                                double* work) {
    const int i = blockIdx.x;
    if (i >= n) return;
    const int l = lane_id();
    const int64_t calls = 2ll * B;
    const int64_t per = (calls + kWave - 1) / kWave;
    const int64_t c0 = l * per, c1 = min<int64_t>(calls, c0 + per);
    double sh = 0, st = 0;
    for (int64_t c = c0; c < c1; ++c) {
        sh += proj[c * 2 * ld + i];
        st += proj[(c * 2 + 1) * ld + i];
    }
    // exclusive scan of the lane sums (in lane order)
    double eh = sh, et = st;
#pragma unroll
    for (int off = 1; off < kWave; off <<= 1) {
        const double yh = __shfl_up(eh, off, 64), yt = __shfl_up(et, off, 64);
        if (l >= off) {
            eh += yh;
            et += yt;
        }
    }
    double rh = work[i] + (eh - sh), rt = work[n + i] + (et - st);
    for (int64_t c = c0; c < c1; ++c) {
        rh += proj[c * 2 * ld + i];
        rt += proj[(c * 2 + 1) * ld + i];
        proj[c * 2 * ld + i] = rh;
        proj[(c * 2 + 1) * ld + i] = rt;
    }
    if (l == kWave - 1) {
        work[i] = rh;
        work[n + i] = rt;
    }
}

template <typename T, int CH>
__global__ __launch_bounds__(256) void transr_compat_energy_kernel(RScoreArgs<T> a) {
    const int kk = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (kk >= a.B) return;
    const int l = lane_id();
    const int r = a.rels[a.si[kk]];
    RowReg<T, CH> R;
    R.load(a.rel + (int64_t)r * a.ld, a.n);
    const double* pp = a.proj + ((int64_t)kk * 2 + 0) * 2 * a.ld;
    double ep = 0, en = 0;
#pragma unroll
    for (int c = 0; c < CH; ++c)
#pragma unroll
        for (int k = 0; k < kVec; ++k) {
            const int e = c * (kWave * kVec) + l * kVec + k;
            if (e >= a.n) continue;
            const double dp = pp[a.ld + e] - pp[e] - (double)R.v[c][k];
            const double dn = pp[3 * a.ld + e] - pp[2 * a.ld + e] - (double)R.v[c][k];
            ep += a.l1 ? fabs(dp) : dp * dp;
            en += a.l1 ? fabs(dn) : dn * dn;
        }
    ep = wave_sum(ep);
    en = wave_sum(en);
    const bool active = ep + a.margin > en;
    if (l == 0) {
        a.act[kk] = active ? 1 : 0;
        a.loss[kk] = active ? a.margin + ep - en : 0.0;
    }
}

// ---------------------------------------------------------- TransR phase B


// transRNorm (transr/trainer.cpp:35-64) on an entity row held in registers,
// with the relation matrix W (n x ldl) in LDS and `abuf` (n) as broadcast
// scratch.  Sums over j run in the reference's order for the check; the
// per-column dot products of the iteration use the wave reduction.
// The owner's matrix W' in LDS, or (WG: dim too wide for the LDS, kb2e_upload_triples)
// the relation's next-matrix row in global memory itself: one wave owns it, its
// own stores are drained before a barrier and re-read past the L1 (sc1), the
// convention of the entity rows handed between owners.
template <bool WG, typename T>
__device__ __forceinline__ T wld(const T* p) {
    if constexpr (WG) return load_sc1(p);
    else return *p;
}
template <bool WG, typename T>
__device__ __forceinline__ void wst(T* p, T v) {
    if constexpr (WG) store_sc1(p, v);
    else *p = v;
}
template <bool WG>
__device__ __forceinline__ void wsync() {
    if constexpr (WG) drain_stores();
    __syncthreads();
}

template <typename T, int CH, bool WG = false>
__device__ void transr_norm(RowReg<T, CH>& A, T* Wl, int ldl, T* abuf, int n, T lr OWNER_PC_PARAM) {
    const int l = lane_id();
    for (int iter = 0; iter < 100000; ++iter) {
        A.store(abuf, n);
        wsync<WG>();
        T xx = T(0);
#pragma unroll
        for (int c = 0; c < CH; ++c)
#pragma unroll
            for (int k = 0; k < kVec; ++k) {
                const int i = c * (kWave * kVec) + l * kVec + k;
                if (i >= n) continue;
                T tmp = T(0);
                for (int j = 0; j < n; ++j) tmp += wld<WG>(Wl + (int64_t)j * ldl + i) * abuf[j];
                xx += tmp * tmp;
            }
        xx = wave_sum(xx);
        __syncthreads();
        OWNER_MARK(6);
        if (xx <= T(1)) break;
        OWNER_COUNT(10);
        const T lambda = T(1);
        for (int i = 0; i < n; ++i) {
            T part = T(0);
#pragma unroll
            for (int c = 0; c < CH; ++c)
#pragma unroll
                for (int k = 0; k < kVec; ++k) {
                    const int j = c * (kWave * kVec) + l * kVec + k;
                    if (j < n) part += wld<WG>(Wl + (int64_t)j * ldl + i) * A.v[c][k];
                }
            T tmp = wave_sum(part);
            tmp *= T(2);
            const T coef = lr * lambda * tmp;
#pragma unroll
            for (int c = 0; c < CH; ++c)
#pragma unroll
                for (int k = 0; k < kVec; ++k) {
                    const int j = c * (kWave * kVec) + l * kVec + k;
                    if (j >= n) continue;
                    const T wn = wld<WG>(Wl + (int64_t)j * ldl + i) - coef * A.v[c][k];
                    wst<WG>(Wl + (int64_t)j * ldl + i, wn);
                    A.v[c][k] = A.v[c][k] - coef * wn;
                }
            wsync<WG>();
        }
        OWNER_MARK(7);
    }
}

template <typename T>
__device__ void w_spill(const T* Wl, int ldl, T* Wg, int n, int ld) {
    for (int idx = lane_id(); idx < n * n; idx += kWave) {
        const int j = idx / n, i = idx % n;
        Wg[(int64_t)j * ld + i] = Wl[j * ldl + i];
    }
}

template <typename T>
__device__ void w_fill(T* Wl, int ldl, const T* Wg, int n, int ld) {
    for (int idx = lane_id(); idx < n * n; idx += kWave) {
        const int j = idx / n, i = idx % n;
        Wl[j * ldl + i] = Wg[(int64_t)j * ld + i];
    }
}

template <typename T, int CH, bool WG = false>
__global__ __launch_bounds__(64) void transr_owner_kernel(OwnerArgs<T> a, uint32_t stamp) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int seg = a.owner_seg[(int64_t)a.batch * a.owners + blockIdx.x];
    if (seg < 0) return;
    const int p0 = a.seg_start[seg], p1 = a.seg_start[seg + 1];
    const int n = a.n;
    const int ldl = WG ? a.ld : n + 1;
    // n x ldl: the owner's relation matrix (next): in LDS, or (WG) the table row itself
    T* Wl = WG ? nullptr : (T*)smem;
    T* abuf = (T*)smem + (WG ? 0 : n * ldl);  // n: broadcast scratch
    T* xb = abuf + n;                    // n: update direction
    T* db = xb + n;                      // n: snapshot head - tail
    const int l = lane_id();
    const T lr = (T)a.lr;
    int cur = -1;
#ifdef KB2E_OWNER_PROF
    PhaseClock pc;
    pc.start();
#endif
    for (int p = p0; p < p1; ++p) {
        const uint64_t key = a.keys[p];
        const int kk = a.kl.kk_of(key);
        if (!a.act[kk]) continue;
        const UpdateIds d = decode_update(a, key, true);
        if (d.r != cur) {
            wsync<WG>();
            if (cur >= 0) {
                if (!WG) w_spill(Wl, ldl, a.w + (int64_t)cur * n * a.ld, n, a.ld);
                if (l == 0) a.wtouched[cur] = stamp;
            }
            if (WG) Wl = a.w + (int64_t)d.r * n * a.ld;
            else w_fill(Wl, ldl, a.w + (int64_t)d.r * n * a.ld, n, a.ld);
            cur = d.r;
            __syncthreads();
        }
        OWNER_MARK(0);
        for (int q = 0; q < d.count; ++q) wait_ticket(a.done, d.ent[q], d.tick[q], a.err, a.wait_ticks);
        OWNER_MARK(1);
        // slots: head is slot 0; tail/entrel slots by identity
        int tslot = 0, eslot = 0;
        for (int q = 0; q < d.count; ++q) {
            if (d.roles[q] & kRoleTail) tslot = q;
            if (d.roles[q] & kRoleEntRel) eslot = q;
        }
        RowReg<T, CH> E[3];
        for (int q = 0; q < d.count; ++q) row_load_sc1(E[q], a.ent + (int64_t)d.ent[q] * a.ld, n);
        RowReg<T, CH> R;
        R.load(a.rel + (int64_t)d.r * a.ld, n);
        const T* xg = a.xreal + ((int64_t)kk * 2 + d.u) * a.ld;
        const T* dg = a.scal + ((int64_t)kk * 2 + d.u) * a.ld;
        for (int i = l; i < n; i += kWave) {
            xb[i] = xg[i];
            db[i] = dg[i];
        }
        __syncthreads();
        OWNER_MARK(2);
        const T beta = d.u ? T(1) : T(-1);
        const T blr = beta * lr;
        // rank-1 update of W' (transr/trainer.cpp:167): W'[j][i] -= (blr x_i) d_j
        for (int idx = l; idx < n * n; idx += kWave) {
            const int j = idx / n, i = idx % n;
            wst<WG>(Wl + (int64_t)j * ldl + i, wld<WG>(Wl + (int64_t)j * ldl + i) - (blr * xb[i]) * db[j]);
        }
        OWNER_MARK(3);
        // entity deltas with the snapshot matrix, summed over i in order (:168-169)
        const T* Ws = a.wsnap + (int64_t)d.r * n * a.ld;
        const bool same = tslot == 0;
#pragma unroll
        for (int c = 0; c < CH; ++c)
#pragma unroll
            for (int k = 0; k < kVec; ++k) {
                const int j = c * (kWave * kVec) + l * kVec + k;
                if (j >= n) continue;
                const T* wrow = Ws + (int64_t)j * a.ld;
                T hv = E[0].v[c][k];
                T tv = E[tslot].v[c][k];
                for (int i = 0; i < n; ++i) {
                    const T g = (blr * xb[i]) * wrow[i];
                    if (same) {
                        hv = hv - g;
                        hv = hv + g;
                    } else {
                        hv = hv - g;
                        tv = tv + g;
                    }
                }
                E[0].v[c][k] = hv;
                if (!same) E[tslot].v[c][k] = tv;
            }
        // relation (:171)
#pragma unroll
        for (int c = 0; c < CH; ++c)
#pragma unroll
            for (int k = 0; k < kVec; ++k) {
                const int i = c * (kWave * kVec) + l * kVec + k;
                if (i < n) R.v[c][k] = R.v[c][k] - blr * xb[i];
            }
        __syncthreads();
        OWNER_MARK(4);
        // unit norms (:174-180): r', h', t', then every row of W'
        R.norm(n, false);
        E[0].norm(n, false);
        E[tslot].norm(n, false);
        if constexpr (WG) wsync<WG>();  // the rank-1 update's stores before another lane's row reads
        for (int j = l; j < n; j += kWave) {  // one lane per row: the reference's serial sum
            T s = T(0);
            for (int i = 0; i < n; ++i) {
                const T x = wld<WG>(Wl + (int64_t)j * ldl + i);
                s += x * x;
            }
            const T len = sqrt(s);
            for (int i = 0; i < n; ++i) wst<WG>(Wl + (int64_t)j * ldl + i, wld<WG>(Wl + (int64_t)j * ldl + i) / len);
        }
        wsync<WG>();
        // transRNorm on head, tail and entity[relation] (:185-187)
        OWNER_MARK(5);
        transr_norm<T, CH, WG>(E[0], Wl, ldl, abuf, n, lr OWNER_PC_ARG);
        transr_norm<T, CH, WG>(E[tslot], Wl, ldl, abuf, n, lr OWNER_PC_ARG);
        transr_norm<T, CH, WG>(E[eslot], Wl, ldl, abuf, n, lr OWNER_PC_ARG);
        R.store(a.rel + (int64_t)d.r * a.ld, n);
        for (int q = 0; q < d.count; ++q) row_store_sc1(E[q], a.ent + (int64_t)d.ent[q] * a.ld, n);
        drain_stores();
        for (int q = 0; q < d.count; ++q) release_ticket(a.done, d.ent[q], d.tick[q]);
        OWNER_MARK(8);
        OWNER_COUNT(11);
    }
    wsync<WG>();
    if (cur >= 0) {
        if (!WG) w_spill(Wl, ldl, a.w + (int64_t)cur * n * a.ld, n, a.ld);
        if (l == 0) a.wtouched[cur] = stamp;
    }
#ifdef KB2E_OWNER_PROF
    pc.flush(blockIdx.x < kProfOwners ? g_owner_prof[blockIdx.x] : nullptr);
#endif
}

// ------------------------------------------- TransR phase B, register owner
//
// For dim <= 64 (one element per lane).  Lane j keeps row j of the owner's
// relation matrix W' in registers (w[]) and reads row j of the batch-start
// snapshot from LDS (Ws, transposed so lane j's reads are consecutive), so the
// rank-1 update, the deltas and the row norms are lane-local and fully
// unrolled.  An LDS copy of W' (Wt, rows of ldl) is
// refreshed only when transRNorm's check needs the column sums W'^T a.
// Descriptors of every update (ids, slots, tickets) are precomputed in
// parallel by transr_desc_kernel, so the serial owner loop does one uniform
// load per update.

// LDS row stride of the W' copy: = 1 (mod 16) doubles, so lane j writing row
// j and lane i reading column i are both (nearly) conflict-free.
__host__ __device__ constexpr int transr_ldl(int nm) { return ((nm + 14) / 16) * 16 + 1; }

template <typename T, int NM>
__host__ __device__ constexpr size_t transr_reg_lds_bytes() {
    return ((size_t)NM * transr_ldl(NM) + kWave + 2 * kWave + (size_t)NM * kWave) * sizeof(T);
}

// transRNorm (transr/trainer.cpp:35-64) on the entity element `al` of this
// lane, W' rows in registers.  Every loop runs over the NM register slots
// without per-element guards: slots >= n (and lanes >= n) hold exact zeros,
// so their terms add +0 and leave the sums unchanged.  The check's column
// sums (four interleaved partial sums over j, from the LDS copy) decide the
// loop and seed column 0 of an iteration; later columns use the wave
// reduction.  Every element update is the reference's operation.
template <typename T, int NM>
__device__ __forceinline__ T transr_norm_reg(T al, T (&w)[NM], T* Wt, T* abuf, int n, T lr2, bool& dirty
                                             OWNER_PC_PARAM) {
    constexpr int ldl = transr_ldl(NM);
    const int l = lane_id();
    for (int iter = 0; iter < 100000; ++iter) {
        if (dirty) {
            if (l < NM) {
#pragma unroll
                for (int i = 0; i < NM; ++i) Wt[l * ldl + i] = w[i];
            }
            dirty = false;
        }
        abuf[l] = al;
        wave_lds_sync();
        // four interleaved partial sums (the value only decides x <= 1 and
        // seeds column 0, like the reduced sums of the later columns).  The
        // LDS reads are staged in double-buffered chunks so a chunk's reads
        // are in flight while the previous chunk is multiplied.
        constexpr int CK = 10;
        constexpr int NCK = (NM + CK - 1) / CK;
        T y4[4] = {T(0), T(0), T(0), T(0)};
        T wc[2][CK], ab[2][CK];
#pragma unroll
        for (int q = 0; q < CK; ++q) {
            wc[0][q] = q < NM ? Wt[q * ldl + l] : T(0);
            ab[0][q] = q < NM ? abuf[q] : T(0);
        }
#pragma unroll
        for (int c = 0; c < NCK; ++c) {
            if (c + 1 < NCK) {
#pragma unroll
                for (int q = 0; q < CK; ++q) {
                    const int j = (c + 1) * CK + q;
                    wc[(c + 1) & 1][q] = j < NM ? Wt[j * ldl + l] : T(0);
                    ab[(c + 1) & 1][q] = j < NM ? abuf[j] : T(0);
                }
            }
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int q = 0; q < CK; ++q) {
                const int j = c * CK + q;
                if (j < NM) y4[j & 3] += wc[c & 1][q] * ab[c & 1][q];
            }
            __builtin_amdgcn_sched_barrier(0);
        }
        const T y = (y4[0] + y4[1]) + (y4[2] + y4[3]);
        const T xx = wave_sum(l < n ? y * y : T(0));
        OWNER_MARK(6);
        if (xx <= T(1)) break;
        OWNER_COUNT(10);
        const T tmp0 = readlane_f(y, 0);
        // Column i's sum needs a after column i-1; its per-lane product is
        // prepared from values known before column i-1's coefficient c:
        //   w_{i} . a_new = P1 - c (P2 - c P1),  P1 = w_i a,  P2 = w_i w_{i-1}
        // (w_{i-1} before its update), two FMAs after c instead of five
        // dependent operations.  The element updates themselves are the
        // reference's operations, off the serial path.
        T prod = T(0);
#pragma unroll
        for (int i = 0; i < NM; ++i) {
            const T tmp = i == 0 ? tmp0 : wave_sum(prod);
            // learningRate_ * lambda * (2 tmp), lambda = 1: the doubling is exact,
            // so (2 lr) * tmp rounds the same real number once, as the reference
            const T coef = lr2 * tmp;
            if (i + 1 < NM) {
                const T P1 = w[i + 1] * al, P2 = w[i + 1] * w[i];
                prod = fma(-coef, fma(-coef, P1, P2), P1);
            }
            w[i] = w[i] - coef * al;
            al = al - coef * w[i];
        }
        dirty = true;
        OWNER_MARK(7);
    }
    return al;
}

// NM >= n register slots per lane (NM == n for the instantiated common dims).
template <typename T, int NM>
__global__ __launch_bounds__(64) void transr_owner_reg_kernel(OwnerArgs<T> a, const uint4* cdesc, const int32_t* ocount,
                                                              uint32_t stamp) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    constexpr int ldl = transr_ldl(NM);
    const int seg = a.owner_seg[(int64_t)a.batch * a.owners + blockIdx.x];
    if (seg < 0) return;
    const int m = ocount[blockIdx.x];
    const uint4* dl0 = cdesc + (int64_t)(a.seg_start[seg] - a.seg_start[a.batch_seg[a.batch]]) * 3;
    const int n = a.n, ld = a.ld;
    T* Wt = (T*)smem;               // NM rows of ldl (+ slack: lanes >= NM read past the last row)
    T* abuf = Wt + NM * ldl + kWave;  // [64] transRNorm broadcast
    T* xs = abuf + kWave;           // [64] beta * lr * x_i, zero past n
    T* Ws = xs + kWave;             // [NM][64]: Ws[i * 64 + j] = snapshot W[j][i], zero past n
    const int l = lane_id();
    const bool row_lane = l < n;
    const T lr = (T)a.lr;
    const T lr2 = T(2) * lr;        // lr * (2 tmp) == (2 lr) * tmp exactly
    T w[NM];
#pragma unroll
    for (int i = 0; i < NM; ++i) w[i] = T(0);
    int cur = -1;
    T rl = T(0);
    bool dirty = true;
#ifdef KB2E_OWNER_PROF
    PhaseClock pc;
    pc.start();
#endif
    // software pipeline: descriptors run two updates ahead, the x / d
    // elements of update it+1 are loaded during update it.
    uint4 n0{}, n1{}, n2{}, f0{}, f1{}, f2{};
    T nxl = T(0), ndl = T(0);
    if (m > 0) {
        n0 = dl0[0];
        n1 = dl0[1];
        n2 = dl0[2];
        const int64_t xo = ((int64_t)uni(n0.x) * 2 + (uni(n0.y) & 1)) * ld;
        nxl = row_lane ? a.xreal[xo + l] : T(0);
        ndl = row_lane ? a.scal[xo + l] : T(0);
    }
    if (m > 1) {
        f0 = dl0[3];
        f1 = dl0[4];
        f2 = dl0[5];
    }
    for (int it = 0; it < m; ++it) {
        const uint4 q0 = n0, q1 = n1, q2 = n2;
        const T xl = nxl, dl = ndl;
        n0 = f0;
        n1 = f1;
        n2 = f2;
        if (it + 2 < m) {
            const uint4* dn = dl0 + (int64_t)(it + 2) * 3;
            f0 = dn[0];
            f1 = dn[1];
            f2 = dn[2];
        }
        const uint32_t packed = uni(q0.y);
        const int count = (int)((packed >> 2) & 3);
        const int kk = (int)uni(q0.x), u = (int)(packed & 1), r = (int)uni(q0.z);
        (void)kk;
        const uint32_t ent[3] = {uni(q1.x), uni(q1.y), uni(q1.z)};
        const uint32_t tk[3] = {uni(q2.x), uni(q2.y), uni(q2.z)};
        const int ts = ((packed >> 8) & kRoleTail) ? 1 : 0;  // tail is slot 0 or 1
        const int es = ((packed >> 4) & kRoleEntRel) ? 0 : (((packed >> 8) & kRoleEntRel) ? 1 : 2);
        (void)count;
        if (r != cur) {
            if (cur >= 0 && row_lane) {
                T* dst = a.w + ((int64_t)cur * n + l) * ld;
#pragma unroll
                for (int i = 0; i < NM; ++i)
                    if (i < n) dst[i] = w[i];
            }
            if (cur >= 0 && l == 0) a.wtouched[cur] = stamp;
            drain_stores();  // a relation met again re-reads what this wave stored
            const T* src = a.w + ((int64_t)r * n + l) * ld;
            const T* srs = a.wsnap + ((int64_t)r * n + l) * ld;
#pragma unroll
            for (int i = 0; i < NM; ++i) {
                w[i] = (row_lane && i < n) ? load_sc1(src + i) : T(0);
                Ws[i * kWave + l] = (row_lane && i < n) ? srs[i] : T(0);
            }
            rl = row_lane ? load_sc1(a.rel + (int64_t)r * ld + l) : T(0);
            cur = r;
        }
        if (it + 1 < m) {  // x / d of the next update
            const int64_t xo = ((int64_t)uni(n0.x) * 2 + (uni(n0.y) & 1)) * ld;
            nxl = row_lane ? a.xreal[xo + l] : T(0);
            ndl = row_lane ? a.scal[xo + l] : T(0);
        }
        OWNER_MARK(0);
        // ---- relation state: transr/trainer.cpp:147-171 (W', r') and :174-180 (norms)
        const T blr = (u ? T(1) : T(-1)) * lr;  // beta * learningRate_
        xs[l] = blr * xl;  // dl: snapshot head - tail, element l
        wave_lds_sync();
        // W'[j][i] -= (blr x_i) d_j ; lane j owns row j
#pragma unroll
        for (int i = 0; i < NM; ++i) w[i] = w[i] - xs[i] * dl;
        rl = rl - xs[l];
        {
            const T len = sqrt(wave_sum(rl * rl));
            if (row_lane) rl = rl / len;
        }
        if (row_lane) {
            T sq = T(0);
#pragma unroll
            for (int i = 0; i < NM; ++i) sq += w[i] * w[i];
            const T len = sqrt(sq);
            const T inv = T(1) / len;
#pragma unroll
            for (int i = 0; i < NM; ++i) w[i] = div_markstein(w[i], len, inv);
            a.rel[(int64_t)r * ld + l] = rl;
        }
        dirty = true;
        OWNER_MARK(3);
        // ---- entity rows
        wait_tickets3(a.done, count, ent, tk, a.err, a.wait_ticks);
        OWNER_MARK(1);
        T v0 = row_lane ? load_sc1(a.ent + (int64_t)ent[0] * ld + l) : T(0);
        T v1 = (count > 1 && row_lane) ? load_sc1(a.ent + (int64_t)ent[1] * ld + l) : T(0);
        T v2 = (count > 2 && row_lane) ? load_sc1(a.ent + (int64_t)ent[2] * ld + l) : T(0);
        OWNER_MARK(2);
        // deltas with the snapshot matrix, subtracted in order of i (:168-169)
        if (ts == 0) {
#pragma unroll
            for (int i = 0; i < NM; ++i) {
                const T g = xs[i] * Ws[i * kWave + l];
                v0 = v0 - g;
                v0 = v0 + g;
            }
        } else {
#pragma unroll
            for (int i = 0; i < NM; ++i) {
                const T g = xs[i] * Ws[i * kWave + l];
                v0 = v0 - g;
                v1 = v1 + g;
            }
        }
        // common::norm(head), common::norm(tail) (:175-176)
        {
            const T len = sqrt(wave_sum(v0 * v0));
            if (row_lane) v0 = v0 / len;
        }
        {
            T tv = ts == 0 ? v0 : v1;
            const T len = sqrt(wave_sum(tv * tv));
            if (row_lane) tv = tv / len;
            if (ts == 0) v0 = tv;
            else v1 = tv;
        }
        OWNER_MARK(4);
        // transRNorm on head, tail, entity[relation] (:185-187); a slot is
        // published as soon as no later call touches it.
#pragma unroll 1
        for (int call = 0; call < 3; ++call) {
            const int s = call == 0 ? 0 : (call == 1 ? ts : es);
            T al = s == 0 ? v0 : (s == 1 ? v1 : v2);
            al = transr_norm_reg<T, NM>(al, w, Wt, abuf, n, lr2, dirty OWNER_PC_ARG);
            if (s == 0) v0 = al;
            else if (s == 1) v1 = al;
            else v2 = al;
            const bool later = (call == 0 && (ts == s || es == s)) || (call == 1 && es == s);
            if (!later) {
                if (row_lane) store_sc1(a.ent + (int64_t)ent[s] * ld + l, al);
                drain_stores();
                release_ticket(a.done, (int)ent[s], tk[s]);
            }
        }
        OWNER_MARK(8);
        OWNER_COUNT(11);
    }
    if (cur >= 0) {
        if (row_lane) {
            T* dst = a.w + ((int64_t)cur * n + l) * ld;
#pragma unroll
            for (int i = 0; i < NM; ++i)
                if (i < n) dst[i] = w[i];
        }
        if (l == 0) a.wtouched[cur] = stamp;
    }
#ifdef KB2E_OWNER_PROF
    pc.flush(blockIdx.x < kProfOwners ? g_owner_prof[blockIdx.x] : nullptr);
#endif
}

// After phase B: the committed matrices (snapshot table) take the new values
// of every relation touched in this batch.
template <typename T>
__global__ __launch_bounds__(256) void transr_commit_kernel(const T* wnext, T* wsnap, const uint32_t* touched,
                                                            uint32_t stamp, int32_t nr, int32_t n, int32_t ld) {
    const int64_t rows = (int64_t)nr * n;
    for (int64_t row = blockIdx.x; row < rows; row += gridDim.x) {
        if (touched[row / n] != stamp) continue;
        for (int i = threadIdx.x; i < n; i += blockDim.x) wsnap[row * ld + i] = wnext[row * ld + i];
    }
}
}  // namespace kb2e
