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
    int32_t sub, Bs;       // index batches a batch, samples an index batch (the last one the rest; 1, B: one)
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
    // index batch (batch, sub-batch; kb2e_config.sub_batches) and the sample within it
    const int q = (int)(k % a.B), sb = q / a.Bs;
    const int b = (int)(k / a.B) * a.sub + sb, kk = q - sb * a.Bs;
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
