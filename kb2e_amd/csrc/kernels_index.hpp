// kernels_index.hpp -- per-epoch event index.
//
// The reference applies each batch's gradient updates to the *_next_ tables in
// sample order, renormalising after every update (common/trainer.cpp:75-99,
// transe/trainer.cpp:25-56).  Which rows an update touches depends only on the
// sample stream, never on embedding values, so the whole
// epoch's (row, sample, update) events are known before the epoch starts.  We
// emit one 64-bit key per event, radix-sort the epoch's keys once, and cut the
// sorted array into per-(batch, row) segments that the fold kernels replay in
// order.  Keys: [batch | row | kk | u | roles]; `row` is an entity id, or
// |E| + relation id (TransE per-row folds), or |E| + owner workgroup
// (TransH/TransR relation-owner schedules).
#pragma once

#include "kernels_common.hpp"

namespace kb2e {

struct KeyArgs {
    const int32_t* heads;
    const int32_t* tails;
    const int32_t* rels;
    const int32_t* si;
    const int32_t* sj;
    const uint8_t* side;
    const int32_t* owner;  // relation -> owner (relation-owner schedules), else null
    int64_t nsamples;      // samples in the epoch buffer
    int32_t B;             // batch size
    int32_t ne;
    KeyLayout kl;
    uint64_t* keys;        // slots * nsamples
};

__device__ __forceinline__ void put_entity_keys(const KeyArgs& a, uint64_t* out, int b, int kk, int u,
                                                int eh, int et, int er, int& w) {
    // Distinct entities of one update with OR'ed roles (head, tail, entity[r]).
    int ids[3] = {eh, et, er};
    uint32_t roles[3] = {kRoleHead, kRoleTail, kRoleEntRel};
    const int nid = er >= 0 ? 3 : 2;
    for (int q = 0; q < nid; ++q) {
        bool first = true;
        for (int p = 0; p < q; ++p)
            if (ids[p] == ids[q]) first = false;
        if (!first) continue;
        uint32_t m = roles[q];
        for (int p = q + 1; p < nid; ++p)
            if (ids[p] == ids[q]) m |= roles[p];
        out[w++] = a.kl.make(b, ids[q], kk, u, m);
    }
}

template <int SLOTS, bool ENTREL>
__global__ __launch_bounds__(256) void emit_keys_kernel(KeyArgs a) {
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= a.nsamples) return;
    const int b = (int)(k / a.B), kk = (int)(k % a.B);
    const int i = a.si[k], j = a.sj[k];
    const int h = a.heads[i], t = a.tails[i], r = a.rels[i];
    const int nh = a.side[k] ? h : j, nt = a.side[k] ? j : t;
    uint64_t* out = a.keys + k * SLOTS;
    int w = 0;
    const int rrow = a.ne + (a.owner ? a.owner[r] : r);
    out[w++] = a.kl.make(b, rrow, kk, 0, 0);
    out[w++] = a.kl.make(b, rrow, kk, 1, 0);
    put_entity_keys(a, out, b, kk, 0, h, t, ENTREL ? r : -1, w);
    put_entity_keys(a, out, b, kk, 1, nh, nt, ENTREL ? r : -1, w);
    while (w < SLOTS) out[w++] = kSentinelKey;
}

// PARALLEL TransR transRNorm pairs, deduplicated per relation per batch: for
// every update slot s = (kk * 2 + u) * 2 + role (role 0 the update's head, 1 its
// tail) the batch-local slot of the previous occurrence of the same (relation,
// entity) in the relation's (sample, update, role) order, or -1; rlast[b][r] =
// the last slot whose entity is r itself (the (entity[r], r) pair's duplicate,
// transr/trainer.cpp:187).  From the sorted event index: an entity segment
// lists the entity's events of one batch in (sample, update) order, so the
// previous occurrence is the nearest earlier event of the segment whose sample
// has the same relation.  Whether a slot is a duplicate then depends on which
// samples are active (per batch): transr_pair_dup walks the chain.
struct PairPrevArgs {
    const uint64_t* keys;  // sorted
    const int32_t* nvalid;
    const int32_t* si;     // the epoch's sample stream
    const int32_t* rels;
    int32_t B, ne, nr;
    KeyLayout kl;
    int32_t* pprev;        // [S][2][2]
    int32_t* rlast;        // [nb][nr], -1 before
};

__global__ __launch_bounds__(256) void pair_prev_kernel(PairPrevArgs a) {
    const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= *a.nvalid) return;
    const uint64_t key = a.keys[p];
    const int row = a.kl.row_of(key);
    const uint32_t roles = (uint32_t)(key & 7);
    const bool hd = roles & kRoleHead, tl = roles & kRoleTail;
    if (row >= a.ne || !(hd || tl)) return;
    const int b = a.kl.batch_of(key), kk = a.kl.kk_of(key), u = (int)((key >> 3) & 1);
    const int64_t k0 = (int64_t)b * a.B;
    const int rel = a.rels[a.si[k0 + kk]];
    const uint64_t seg = a.kl.seg_part(key);
    int prev = -1;
    for (int64_t q = p - 1; q >= 0; --q) {
        const uint64_t kq = a.keys[q];
        if (a.kl.seg_part(kq) != seg) break;
        const uint32_t rq = (uint32_t)(kq & 7);
        if (!(rq & (kRoleHead | kRoleTail))) continue;
        const int kkq = a.kl.kk_of(kq);
        if (a.rels[a.si[k0 + kkq]] != rel) continue;
        prev = (kkq * 2 + (int)((kq >> 3) & 1)) * 2 + ((rq & kRoleTail) ? 1 : 0);
        break;
    }
    const int s0 = (kk * 2 + u) * 2;
    int32_t* pp = a.pprev + (k0 + kk) * 4 + u * 2;
    if (hd) pp[0] = prev;
    if (tl) pp[1] = hd ? s0 : prev;
    if (row == rel) atomicMax(a.rlast + (int64_t)b * a.nr + rel, s0 + (tl ? 1 : 0));
}

// flags[p] = 1 where a new (batch,row) segment starts; counts valid keys.
__global__ __launch_bounds__(256) void seg_flags_kernel(const uint64_t* keys, int64_t n, KeyLayout kl,
                                                        int32_t* flags, int32_t* nvalid) {
    const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n) return;
    const uint64_t k = keys[p];
    const bool valid = k != kSentinelKey;
    flags[p] = valid && (p == 0 || kl.seg_part(keys[p - 1]) != kl.seg_part(k)) ? 1 : 0;
    if (valid && (p == n - 1 || keys[p + 1] == kSentinelKey)) *nvalid = (int32_t)(p + 1);
    if (p == 0 && !valid) *nvalid = 0;
}

__global__ __launch_bounds__(256) void seg_scatter_kernel(const int32_t* flags, const int32_t* idx, int64_t n,
                                                          int32_t* seg_start, int32_t* nseg,
                                                          const int32_t* nvalid) {
    const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n) return;
    if (flags[p]) seg_start[idx[p]] = (int32_t)p;
    if (p == n - 1) {
        const int32_t total = idx[p] + flags[p];
        *nseg = total;
        seg_start[total] = *nvalid;
    }
}

// batch_seg[b] = first segment of batch b; batch_seg[nb] = total segments.
__global__ __launch_bounds__(256) void batch_begin_kernel(const uint64_t* keys, const int32_t* seg_start,
                                                          const int32_t* nseg_p, int nb, KeyLayout kl,
                                                          int32_t* batch_seg) {
    const int nseg = *nseg_p;
    for (int s = blockIdx.x * blockDim.x + threadIdx.x; s <= nseg; s += gridDim.x * blockDim.x) {
        const int b = s < nseg ? kl.batch_of(keys[seg_start[s]]) : nb;
        const int prev = s == 0 ? -1 : kl.batch_of(keys[seg_start[s - 1]]);
        for (int bb = prev + 1; bb <= b && bb <= nb; ++bb) batch_seg[bb] = s;
    }
}

}  // namespace kb2e
