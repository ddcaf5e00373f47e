// kernels_transr_parallel.hpp -- TransR under the PARALLEL schedule
// (KB2E_SCHEDULE_PARALLEL, see kernels_parallel.hpp for the TransE form).
//
// The reference's TransR step (transr/trainer.cpp:144-188) for one update u =
// (h, t, r, beta) with snapshot W = weights_[r]:
//   x = sign / 2 (W^T t - W^T h - r)                (L1 / L2; :147-164)
//   W'  -= beta lr (h - t) x^T                        (:166-167)
//   h'  -= beta lr W x,  t' += beta lr W x,  r' -= beta lr x   (:168-172)
//   unit norms of r', h', t' and of every row of W'   (:174-180)
//   transRNorm(h'), transRNorm(t'), transRNorm(entity'[r]) against W'  (:185-187)
// The ORDERED schedule replays that per update (kernels_relowner.hpp).  Here a
// batch is processed as:
//   tile      per (relation, <= St samples): W_r staged in LDS; projections of
//             h, t, h', t' (energies + hinge, or the compat work-vector scan),
//             x, d = h - t, y = W x for both updates; the tile's partial sums
//             dW = -lr sum beta d x^T and dr = -lr sum beta x.
//   rel rows  one wave per (relation, row j of W or the relation vector): the
//             tiles' partials in tile order, then the unit norm.
//   entities  per entity segment of the event index: sum of -beta lr y (head
//             role) / +beta lr y (tail role), then the unit norm.
//   transRNorm one Jacobi step per batch: per tile, every (h', r), (t', r) pair
//             of an active update and (entity'[r], r) once per relation with
//             |W'^T a|^2 > 1 takes g = 2 W'^T a, dW -= lr a g^T, da = -lr W' g
//             (the first column sweep of transRNorm's loop with the whole
//             column set at once); then rel rows (no norm) and entities (no norm).
// Every sum runs in a fixed order: deterministic.
#pragma once

#include <type_traits>

#include "kernels_common.hpp"

namespace kb2e {

// One tile: samples [first, first + count) of relation segment `seg`.
struct RTile {
    int32_t seg, q;
};

struct RParArgs {
    // batch
    const int32_t* heads;
    const int32_t* tails;
    const int32_t* rels;
    const int32_t* si;  // this batch's sample stream
    const int32_t* sj;
    const uint8_t* side;
    int32_t B, n, ld, ne, nr, St;
    int32_t batch;
    int32_t tgroup;  // matrix-core tile kernels: tiles a workgroup runs (one partial per group; 0, 1: one)
    double lr, margin;
    int32_t compat, l1;
    // event index
    const uint64_t* keys;       // sorted
    const int32_t* seg_start;
    const int32_t* batch_seg;
    const int32_t* seg_row;     // row of every segment
    const int32_t* rel_begin;   // [nb] first relation segment of each batch
    const int32_t* tile_first;  // [nseg + 1] first tile of each segment (exclusive scan of tile counts)
    const RTile* tiles;
    KeyLayout kl;
    // per-sample exports
    uint8_t* act;        // [B] of this batch
    double* loss;        // [B]
    double* proj;        // [B][2][2][ld] compat projections
    int32_t* tile_act;   // [tiles] active updates per tile
    // transRNorm pairs are deduplicated per relation per batch (ptab_insert / transr_pair_dup)
    unsigned long long* ptab;       // [mask + 1] this batch's table: (relation, entity) << 22 | first active slot
    unsigned long long* ptab_next;  // the other one (the next batch's): cleared by the inserting kernel
    uint32_t ptab_mask;
    // per-epoch tile descriptors (rtile_desc_kernel; matrix-core wave kernels): the
    // tiles' relation, sample count, samples and rows without the index chain
    const int32_t* batch_t0;  // [nb + 1] first tile of each batch
    const int32_t* td_r;      // [tiles]
    const int32_t* td_cnt;    // [tiles] samples | 256 when the tile is its relation's only one
    const int32_t* td_kk;     // [tiles][8] batch-local sample of tile sample q
    const int32_t* td_ent;    // [tiles][8][4] entity of row (q, h / t / h' / t'), -1 past cnt
    const int32_t* brel;      // [nrel] this batch's relations, most frequent in training first (rel_list_kernel;
                              // the chain kernels' block order: the long chains start first)
    int32_t nrel;             // their count: the chain launches' grid
};

// Per batch b (a block each): the relations with a segment in the batch (segments
// [rel_begin[b], batch_seg[b + 1]), sorted by row), listed in training-frequency order
// (rel_order) -- the chain kernels' blocks, so that a launch covers exactly the
// batch's relations, hot ones first -- and their count.
static __attribute__((unused)) __global__ __launch_bounds__(1024) void rel_list_kernel(
    const int32_t* rel_begin, const int32_t* batch_seg, const int32_t* seg_row, int32_t ne, const int32_t* rel_order,
    int32_t nr, int64_t cap, int32_t* brel, int32_t* nrel) {
    __shared__ int32_t wsum[16];
    const int b = blockIdx.x, t = threadIdx.x, w = t >> 6, l = t & 63;
    const int s0 = rel_begin[b], s1 = batch_seg[b + 1];
    int32_t* out = brel + (int64_t)b * cap;
    int total = 0;
    for (int base = 0; base < nr; base += 1024) {
        const int q = base + t;
        const int r = q < nr ? rel_order[q] : -1;
        bool here = false;
        if (r >= 0 && s0 < s1) {
            int lo = s0, hi = s1 - 1;
            const int want = ne + r;
            while (lo < hi) {
                const int mid = (lo + hi) >> 1;
                if (seg_row[mid] < want) lo = mid + 1;
                else hi = mid;
            }
            here = seg_row[lo] == want;
        }
        const uint64_t m = __ballot(here);
        if (l == 0) wsum[w] = __popcll(m);
        __syncthreads();
        int off = total;
        for (int k = 0; k < w; ++k) off += wsum[k];
        int all = 0;
        for (int k = 0; k < 16; ++k) all += wsum[k];
        if (here) out[off + __popcll(m & ((1ull << l) - 1))] = r;
        total += all;
        __syncthreads();
    }
    if (t == 0) nrel[b] = total;
}

// The per-batch (relation, entity) -> first active update slot table.  A pair
// (h', r), (t', r) or (entity[r], r) is the reference's repeated transRNorm
// call on an already constrained row when an earlier active slot of the batch
// holds the same (relation, entity) (transr/trainer.cpp:183-188), whichever tile
// it falls in.  One word per entry, all ones = empty; two tables alternate by
// batch, the inserting kernel of batch b clearing batch b + 1's (whose last
// reader was batch b - 1's transRNorm step).
constexpr int kPtabEntBits = 24, kPtabRelBits = 18, kPtabSlotBits = 22;
constexpr unsigned long long kPtabEmpty = ~0ull;

__device__ __forceinline__ unsigned long long ptab_key(int r, int e) {
    return ((unsigned long long)r << kPtabEntBits) | (unsigned long long)e;
}
__device__ __forceinline__ uint32_t ptab_hash(int r, int e) {
    return ((uint32_t)e * 2654435761u) ^ ((uint32_t)r * 0x9E3779B1u + 0x7F4A7C15u);
}

// Records an active slot: the key's entry keeps the smallest slot (one CAS when
// the key is new, an atomicMin when it is already there).
__device__ __forceinline__ void ptab_insert(const RParArgs& a, int r, int e, int slot) {
    const unsigned long long key = ptab_key(r, e);
    const unsigned long long word = (key << kPtabSlotBits) | (unsigned long long)slot;
    uint32_t h = ptab_hash(r, e) & a.ptab_mask;
    while (true) {
        const unsigned long long old = atomicCAS(a.ptab + h, kPtabEmpty, word);
        if (old == kPtabEmpty) return;
        if ((old >> kPtabSlotBits) == key) {
            atomicMin(a.ptab + h, word);
            return;
        }
        h = (h + 1) & a.ptab_mask;
    }
}

// The first active slot holding (r, e) this batch, or -1.
__device__ __forceinline__ int ptab_first(const RParArgs& a, int r, int e) {
    const unsigned long long key = ptab_key(r, e);
    uint32_t h = ptab_hash(r, e) & a.ptab_mask;
    while (true) {
        const unsigned long long w = a.ptab[h];
        if (w == kPtabEmpty) return -1;
        if ((w >> kPtabSlotBits) == key) return (int)(w & ((1ull << kPtabSlotBits) - 1));
        h = (h + 1) & a.ptab_mask;
    }
}

// The next batch's table, cleared by the threads of the inserting kernel.
__device__ __forceinline__ void ptab_clear_next(const RParArgs& a, int64_t tid, int64_t nthreads) {
    for (int64_t q = tid; q <= (int64_t)a.ptab_mask; q += nthreads) a.ptab_next[q] = kPtabEmpty;
}

__device__ __forceinline__ bool transr_pair_dup(const RParArgs& a, int slot, int r, int e) {
    return ptab_first(a, r, e) < slot;
}
__device__ __forceinline__ bool transr_relpair_dup(const RParArgs& a, int r) {
    return ptab_first(a, r, r) >= 0;
}

// After the batch's hinge decisions: every (h', r), (t', r) slot of an active update.
static __attribute__((unused)) __global__ __launch_bounds__(256) void transr_pair_first_kernel(RParArgs a) {
    const int slot = blockIdx.x * blockDim.x + threadIdx.x;
    ptab_clear_next(a, slot, (int64_t)gridDim.x * blockDim.x);
    if (slot >= 4 * a.B) return;
    const int kk = slot >> 2, u = (slot >> 1) & 1, role = slot & 1;
    if (!a.act[kk]) return;
    const int i0 = a.si[kk], jj = a.sj[kk];
    const int h = a.heads[i0], tt = a.tails[i0];
    const int hh = u ? (a.side[kk] ? h : jj) : h;
    const int th = u ? (a.side[kk] ? jj : tt) : tt;
    ptab_insert(a, a.rels[i0], role ? th : hh, slot);
}

template <typename T>
struct RParBufs {
    T* ent;
    T* rel;
    T* W;        // live matrices [r][j][ld]
    T* x;        // [B][2][ld]
    T* d;        // [B][2][ld] snapshot h - t
    T* y;        // [B][2][ld] W x
    T* wpart;    // [tiles][n][ld]
    T* rpart;    // [tiles][ld]
    T* pair;     // [B][2][2][ld] transRNorm deltas of (h, r), (t, r) per update
    T* relpair;  // [R][ld] transRNorm delta of (entity[r], r)
    uint32_t* relpair_stamp;  // [R] batch stamp when relpair[r] is valid this batch
    uint32_t stamp;
    // matrix-core transRNorm (kernels_transr_mfma.hpp); null on the VALU path
    uint8_t* pflag;      // [B][2][2] the pair record of the slot is valid this batch
    int32_t* cons_tile;  // [tiles][cons_ppt] the transRNorm matrix partial is valid (0: none)
    int32_t cons_ppt;    // transRNorm matrix partials per tile (1, or one per row block)
    // register-fragment kernels (kernels_transr_wave.hpp): phase A's entity of every
    // (tile, V row) and the transRNorm pairs of every tile, compacted by the gradient
    // kernel: [tile][kCPairs] entities then [tile][kCPairs] slots, and the row count
    int32_t* cpairs;     // [tiles][2][kCPairs]
    int32_t* cnrows;     // [tiles]
    int32_t stats;       // count transRNorm rounds (tools)
    int32_t last_renorm; // transRNorm pass: entity rows renormalised between pre / post pair deltas (kernels_transr_seq.hpp)
    int32_t dbg;         // transRNorm wave kernel: phases skipped for timing experiments (tools; wrong results)
    int32_t chain_list;  // pipelined chain kernel: pairs a window (0: all that fit the LDS; tests force windows)
    int32_t chain_tiles; // chain kernels: tiles a window (0: the prefix table's 256; tests force windows)
    int32_t* vio;        // n <= 64 chain kernels: [tiles][kCPairs] the violators' slots of the relation whose
                         // first tile it is (-2: (entity[r], r)); its pair records are made in-kernel
    uint32_t* err;       // pipelined chain: a bounded in-workgroup wait timed out (the host fails loudly)
};

__host__ __device__ constexpr int rm_up16_host_dev(int v) { return (v + 15) & ~15; }
constexpr int kCPairs = 64;  // transRNorm pairs of a tile (4 St + 1 <= 64)

template <typename T>
__host__ __device__ constexpr int rpar_lds_w(int n, int ld) {
    return n * ld;  // elements of one staged matrix
}

// Tile geometry: which samples (kk) a tile holds.  Relation segments list two
// events (u = 0, 1) per sample in kk order.
__device__ __forceinline__ void tile_range(const RParArgs& a, int t, int& r, int& e0, int& cnt) {
    const RTile tl = a.tiles[t];
    const int p0 = a.seg_start[tl.seg], p1 = a.seg_start[tl.seg + 1];
    r = a.seg_row[tl.seg] - a.ne;
    const int ns = (p1 - p0) / 2;
    const int f = tl.q * a.St;
    e0 = p0 + 2 * f;
    cnt = min(a.St, ns - f);
}

template <typename T>
__device__ __forceinline__ void stage_matrix(T* Wl, const T* Wg, int n, int ld) {
    for (int idx = threadIdx.x; idx < n * ld; idx += blockDim.x) Wl[idx] = Wg[idx];
}

// p_i = sum_j W[j][i] v_j for four vectors at once, lane l owning i = 2l, 2l+1
// (n <= 128); the vectors are read as LDS broadcasts.
template <typename T>
__device__ __forceinline__ void project4(const T* Wl, int ld, int n, const T* v4 /* [4][ld] */, T (&p)[4][2]) {
    const int l = lane_id();
    const int i = 2 * l;
#pragma unroll
    for (int q = 0; q < 4; ++q) p[q][0] = p[q][1] = T(0);
    if (i >= n) return;
    for (int j = 0; j < n; ++j) {
        const T w0 = Wl[j * ld + i], w1 = Wl[j * ld + i + 1];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const T vj = v4[q * ld + j];
            p[q][0] += w0 * vj;
            p[q][1] += w1 * vj;
        }
    }
}

// y_j = sum_i W[j][i] x_i, lane l owning j = 2l, 2l+1 (x read as LDS broadcasts).
template <typename T>
__device__ __forceinline__ void matvec_rows(const T* Wl, int ld, int n, const T* xl, T (&y)[2]) {
    const int l = lane_id();
    const int j = 2 * l;
    y[0] = y[1] = T(0);
    if (j >= n) return;
    const T* r0 = Wl + j * ld;
    const T* r1 = Wl + (j + 1) * ld;
    const bool has1 = j + 1 < n;
    for (int i = 0; i < n; ++i) {
        const T xi = xl[i];
        y[0] += r0[i] * xi;
        if (has1) y[1] += r1[i] * xi;
    }
}

template <typename T>
__device__ __forceinline__ void lane_pair_load(const T* row, int n, T (&v)[2]) {
    const int e = 2 * lane_id();
    v[0] = e < n ? row[e] : T(0);
    v[1] = e + 1 < n ? row[e + 1] : T(0);
}
template <typename T>
__device__ __forceinline__ void lane_pair_store(T* row, int n, const T (&v)[2]) {
    const int e = 2 * lane_id();
    if (e < n) row[e] = v[0];
    if (e + 1 < n) row[e + 1] = v[1];
}

// rows [j0, j0 + rows) of the tile's partial  dW[j][i] = sum_u D[u][j] X[u][i]
// (D already scaled by -lr beta, zero for inactive updates); lane l owns
// columns i = 2l, 2l+1.
template <typename T>
__device__ __forceinline__ void rank_sum_rows(const T* Dl, const T* Xl, int U, int ld, int n, int j, T (&acc)[2]) {
    const int i = 2 * lane_id();
    acc[0] = acc[1] = T(0);
    if (i >= n) return;
    for (int u = 0; u < U; ++u) {
        const T dj = Dl[u * ld + j];
        acc[0] += dj * Xl[u * ld + i];
        acc[1] += dj * Xl[u * ld + i + 1];
    }
}

// LDS layout of the tile kernels (elements of T): W [n][ld] | per wave 4 x ld
// vectors | X [4 St + 1][ld] | D [4 St + 1][ld] | coef [4 St + 1] | int [4 St + 1]
template <typename T>
__host__ __device__ constexpr size_t rpar_tile_lds(int n, int ld, int St) {
    return sizeof(T) * ((size_t)n * ld + 4 * 4 * (size_t)ld + 2 * (4 * (size_t)St + 1) * ld + 4 * (size_t)St + 1) +
           sizeof(int) * (4 * (size_t)St + 1);
}

// Tile phase A + gradient partials (non-compat: energies here; compat: the
// energies come from the work-vector scan, so GRAD runs as its own launch).
template <typename T, bool PROJ, bool GRAD>
__global__ __launch_bounds__(256) void transr_tile_kernel(RParArgs a, RParBufs<T> bf) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int t = a.tile_first[a.batch_seg[a.batch]] + blockIdx.x;
    if (t >= a.tile_first[a.batch_seg[a.batch + 1]]) return;
    int r, e0, cnt;
    tile_range(a, t, r, e0, cnt);
    const int n = a.n, ld = a.ld;
    T* Wl = (T*)smem;
    T* vec = Wl + n * ld;                  // [4 waves][4][ld]
    T* Xl = vec + 16 * ld;                 // [2 cnt][ld] update directions
    T* Dl = Xl + (4 * a.St + 1) * ld;      // [2 cnt][ld] -lr beta (h - t), 0 if inactive
    T* coef = Dl + (4 * a.St + 1) * ld;    // [2 cnt] -lr beta, 0 if inactive
    const int w = threadIdx.x >> 6, l = lane_id();
    stage_matrix(Wl, bf.W + (int64_t)r * n * ld, n, ld);
    __syncthreads();
    T* v4 = vec + w * 4 * ld;
    for (int q = w; q < cnt; q += 4) {
        const int kk = a.kl.kk_of(a.keys[e0 + 2 * q]);
        if (PROJ) {
            const int i0 = a.si[kk], jj = a.sj[kk];
            const int h = a.heads[i0], tt = a.tails[i0];
            const int nh = a.side[kk] ? h : jj, nt = a.side[kk] ? jj : tt;
            T vh[2], vt[2], vnh[2], vnt[2], vr[2];
            lane_pair_load(bf.ent + (int64_t)h * ld, n, vh);
            lane_pair_load(bf.ent + (int64_t)tt * ld, n, vt);
            lane_pair_load(bf.ent + (int64_t)nh * ld, n, vnh);
            lane_pair_load(bf.ent + (int64_t)nt * ld, n, vnt);
            lane_pair_load(bf.rel + (int64_t)r * ld, n, vr);
            lane_pair_store(v4 + 0 * ld, n, vh);
            lane_pair_store(v4 + 1 * ld, n, vt);
            lane_pair_store(v4 + 2 * ld, n, vnh);
            lane_pair_store(v4 + 3 * ld, n, vnt);
            wave_lds_sync();
            T p[4][2];
            project4(Wl, ld, n, v4, p);  // W^T h, W^T t, W^T h', W^T t'
            T ep = T(0), en = T(0);
            T xp[2], xn[2];
#pragma unroll
            for (int k = 0; k < 2; ++k) {
                const bool ok = 2 * l + k < n;
                const T dp = p[1][k] - p[0][k] - vr[k];
                const T dn = p[3][k] - p[2][k] - vr[k];
                ep += ok ? (a.l1 ? fabs(dp) : dp * dp) : T(0);
                en += ok ? (a.l1 ? fabs(dn) : dn * dn) : T(0);
                xp[k] = ok ? (a.l1 ? (dp > T(0) ? T(1) : T(-1)) : T(2) * dp) : T(0);
                xn[k] = ok ? (a.l1 ? (dn > T(0) ? T(1) : T(-1)) : T(2) * dn) : T(0);
            }
            const T dpos[2] = {vh[0] - vt[0], vh[1] - vt[1]};
            const T dneg[2] = {vnh[0] - vnt[0], vnh[1] - vnt[1]};
            lane_pair_store(bf.x + ((int64_t)kk * 2 + 0) * ld, n, xp);
            lane_pair_store(bf.x + ((int64_t)kk * 2 + 1) * ld, n, xn);
            lane_pair_store(bf.d + ((int64_t)kk * 2 + 0) * ld, n, dpos);
            lane_pair_store(bf.d + ((int64_t)kk * 2 + 1) * ld, n, dneg);
            if (a.compat) {
                double* pr = a.proj + (int64_t)kk * 4 * ld;
#pragma unroll
                for (int k = 0; k < 2; ++k) {
                    const int e = 2 * l + k;
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
                        const T dsc[2] = {c * dv[0], c * dv[1]};
                        lane_pair_store(Xl + (2 * q + u) * ld, n, u ? xn : xp);
                        lane_pair_store(Dl + (2 * q + u) * ld, n, dsc);
                        if (l == 0) coef[2 * q + u] = c;
                    }
                }
            }
            // y = W x for both updates (x through LDS)
            wave_lds_sync();
            lane_pair_store(v4 + 0 * ld, n, xp);
            lane_pair_store(v4 + 1 * ld, n, xn);
            wave_lds_sync();
            T yp[2], yn[2];
            matvec_rows(Wl, ld, n, v4 + 0 * ld, yp);
            matvec_rows(Wl, ld, n, v4 + 1 * ld, yn);
            lane_pair_store(bf.y + ((int64_t)kk * 2 + 0) * ld, n, yp);
            lane_pair_store(bf.y + ((int64_t)kk * 2 + 1) * ld, n, yn);
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
                T xv[2], dv[2];
                lane_pair_load(bf.x + ((int64_t)kk * 2 + u) * ld, n, xv);
                lane_pair_load(bf.d + ((int64_t)kk * 2 + u) * ld, n, dv);
                dv[0] *= c;
                dv[1] *= c;
                lane_pair_store(Xl + (2 * q + u) * ld, n, xv);
                lane_pair_store(Dl + (2 * q + u) * ld, n, dv);
                if (l == 0) coef[2 * q + u] = c;
            }
        }
    }
    __syncthreads();
    const int U = 2 * cnt;
    T* wp = bf.wpart + (int64_t)blockIdx.x * n * ld;  // partials are per batch: local tile index
    for (int j = w; j < n; j += 4) {  // dW = sum_u (-lr beta) (h - t) x^T
        T acc[2];
        rank_sum_rows(Dl, Xl, U, ld, n, j, acc);
        lane_pair_store(wp + (int64_t)j * ld, n, acc);
    }
    if (w == 0) {  // dr = sum_u (-lr beta) x_u
        T acc[2] = {T(0), T(0)};
        const int i = 2 * l;
        for (int u = 0; u < U; ++u) {
            const T c = coef[u];
            if (i < n) acc[0] += c * Xl[u * ld + i];
            if (i + 1 < n) acc[1] += c * Xl[u * ld + i + 1];
        }
        lane_pair_store(bf.rpart + (int64_t)blockIdx.x * ld, n, acc);
        if (l == 0) {
            int nact = 0;
            for (int u = 0; u < U; ++u) nact += coef[u] != T(0);
            a.tile_act[t] = nact;
        }
    }
}
// One wave per (relation segment, row j <= n) of the batch: the tiles' partials
// in tile order added to row j of W_r (j < n) or to the relation vector (j == n),
// then the unit norm (common::norm(v, false), transr/trainer.cpp:174-180) when
// NORM.  Without NORM (the transRNorm step) only the matrix rows change.
template <typename T, bool NORM>
__device__ __forceinline__ void transr_rel_rows_wave(RParArgs a, RParBufs<T> bf, int gw) {  // by value: no scratch copy
    const int rows = a.n + 1;
    const int s = a.rel_begin[a.batch] + gw / rows;
    const int j = gw % rows;
    if (s >= a.batch_seg[a.batch + 1]) return;
    if (!NORM && j == a.n) return;
    const int r = a.seg_row[s] - a.ne;
    const int t0 = a.tile_first[s], t1 = a.tile_first[s + 1];
    const int n = a.n, ld = a.ld;
    const int tb = a.tile_first[a.batch_seg[a.batch]];  // partials are indexed by tile within the batch
    // GRAD step: the reference touches (and normalises) a relation only through
    // an active update; matrix-core transRNorm step: only the partials whose
    // pairs moved (cons_ppt per tile, in (tile, row block) order)
    const bool sel = !NORM && bf.cons_tile;
    // partial slots u in [u0, u1): tiles (GRAD, VALU transRNorm) or (tile, block) pairs
    const int ppt = sel ? bf.cons_ppt : 1;
    const int u0 = sel ? (t0 - tb) * ppt : t0, u1 = sel ? (t1 - tb) * ppt : t1;
    const int ub = sel ? 0 : tb;  // slot u's partial is number u - ub of the batch
    // the slots that carry a partial, 64 flags per load (lane-parallel, not a
    // serial scan: a hot relation has tens of tiles)
    // (captures by value: a reference to the argument structs would put them in scratch)
    const int32_t* const fl = sel ? bf.cons_tile : a.tile_act;
    auto flags = [fl, u1](int base) {
        const int u = base + lane_id();
        const int f = u < u1 ? fl[u] : 0;
        return (uint64_t)__ballot(f != 0);
    };
    uint64_t any = 0;
    for (int base = u0; base < u1 && !any; base += kWave) any = flags(base);
    if (!any) return;
    T* row = j < n ? bf.W + ((int64_t)r * n + j) * ld : bf.rel + (int64_t)r * ld;
    T v[2];
    lane_pair_load(row, n, v);
    for (int base = u0; base < u1; base += kWave) {
        // every tile's partial for the VALU transRNorm step (it writes one for each
        // tile); the flagged ones otherwise: the gradient step's inactive tiles carry
        // zeros and a matrix-core tile group's partial sits on its first tile alone
        uint64_t m = (NORM || sel) ? flags(base) : (uint64_t)__ballot(base + lane_id() < u1);
        while (m) {  // eight partial rows in flight, summed in slot order
            T p[8][2];
            bool use[8];
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                use[q] = m != 0;
                const int64_t lt = use[q] ? base + __builtin_ctzll(m) - ub : 0;
                m &= m - 1;
                if (use[q]) lane_pair_load(j < n ? bf.wpart + (lt * n + j) * ld : bf.rpart + lt * ld, n, p[q]);
            }
#pragma unroll
            for (int q = 0; q < 8; ++q)
                if (use[q]) {
                    v[0] += p[q][0];
                    v[1] += p[q][1];
                }
        }
    }
    if (NORM) {
        const T len = sqrt(wave_sum(v[0] * v[0] + v[1] * v[1]));
        v[0] = v[0] / len;
        v[1] = v[1] / len;
    }
    lane_pair_store(row, n, v);
}

// n <= 64: the same sums, four rows a wave -- one per 16-lane DPP row, lane
// l & 15 holding elements 4 (l & 15) .. + 3 -- so a relation takes ceil((n + 1) / 4)
// waves instead of n + 1 (the per-relation loads are shared, four times fewer
// latency chains).
// E = 8: the same for n <= 128 (eight elements a lane, four partial rows in flight).
template <typename T, bool NORM, int E = 4>
__device__ __forceinline__ void transr_rel_rows4_wave(RParArgs a, RParBufs<T> bf, int gw) {
    using T2 = typename std::conditional<sizeof(T) == 8, double2, float2>::type;
    constexpr int E2 = E / 2, NQ = E == 4 ? 8 : 4;  // element pairs a lane, partial rows in flight
    const int n = a.n, ld = a.ld;
    const int RW = (n + 4) >> 2;  // waves per relation segment (rows 0 .. n)
    const int s = a.rel_begin[a.batch] + gw / RW;
    if (s >= a.batch_seg[a.batch + 1]) return;
    const int l = lane_id(), e0 = E * (l & 15);
    const int j = (gw % RW) * 4 + (l >> 4);  // this DPP row's table row (j == n: the relation vector)
    const bool jok = NORM ? j <= n : j < n;
    const int r = a.seg_row[s] - a.ne;
    const int t0 = a.tile_first[s], t1 = a.tile_first[s + 1];
    const int tb = a.tile_first[a.batch_seg[a.batch]];
    const bool sel = !NORM && bf.cons_tile;
    const int ppt = sel ? bf.cons_ppt : 1;
    const int u0 = sel ? (t0 - tb) * ppt : t0, u1 = sel ? (t1 - tb) * ppt : t1;
    const int ub = sel ? 0 : tb;
    const int32_t* const fl = sel ? bf.cons_tile : a.tile_act;
    auto flags = [fl, u1, l](int base) {
        const int u = base + l;
        return (uint64_t)__ballot(u < u1 && fl[u] != 0);
    };
    uint64_t any = 0;
    for (int base = u0; base < u1 && !any; base += kWave) any = flags(base);
    if (!any) return;
    bool pk[E2];  // the element pairs of the lane
#pragma unroll
    for (int k = 0; k < E2; ++k) pk[k] = jok && e0 + 2 * k < ld;
    auto load4 = [&](const T* rp, T (&v)[E]) {
#pragma unroll
        for (int k = 0; k < E2; ++k) {
            const T2 x = pk[k] ? *(const T2*)(rp + e0 + 2 * k) : T2{T(0), T(0)};
            v[2 * k] = x.x;
            v[2 * k + 1] = x.y;
        }
    };
    const int jr = jok ? j : 0;
    T* row = jr < n ? bf.W + ((int64_t)r * n + jr) * ld : bf.rel + (int64_t)r * ld;
    T v[E];
    load4(row, v);
    for (int base = u0; base < u1; base += kWave) {
        // the GRAD step's zero partials (inactive tiles) and the matrix-core transRNorm
        // step's unflagged ones are skipped; the VALU transRNorm step writes one for
        // every tile (a relation's first tile carries (entity[r], r) even when inactive)
        uint64_t m = (NORM || sel) ? flags(base) : (uint64_t)__ballot(base + l < u1);
        while (m) {  // NQ partial rows in flight, summed in slot order
            T p[NQ][E];
            bool use[NQ];
#pragma unroll
            for (int q = 0; q < NQ; ++q) {
                use[q] = m != 0;
                const int64_t lt = use[q] ? base + __builtin_ctzll(m) - ub : 0;
                m &= m - 1;
                if (use[q]) load4(jr < n ? bf.wpart + (lt * n + jr) * ld : bf.rpart + lt * ld, p[q]);
            }
#pragma unroll
            for (int q = 0; q < NQ; ++q)
                if (use[q])
#pragma unroll
                    for (int k = 0; k < E; ++k) v[k] += p[q][k];
        }
    }
    if (NORM) {  // common::norm(v, false): unit length (padding elements are zero)
        T ss = (v[0] * v[0] + v[1] * v[1]) + (v[2] * v[2] + v[3] * v[3]);
#pragma unroll
        for (int k = 4; k < E; k += 4) ss += (v[k] * v[k] + v[k + 1] * v[k + 1]) + (v[k + 2] * v[k + 2] + v[k + 3] * v[k + 3]);
        ss += dpp_ror<8>(ss);
        ss += dpp_ror<4>(ss);
        ss += dpp_ror<2>(ss);
        ss += dpp_ror<1>(ss);
        const T len = sqrt(ss);
#pragma unroll
        for (int k = 0; k < E; ++k) v[k] = v[k] / len;
    }
#pragma unroll
    for (int k = 0; k < E2; ++k)
        if (pk[k]) *(T2*)(row + e0 + 2 * k) = T2{v[2 * k], v[2 * k + 1]};
}

template <typename T, bool NORM>
__global__ __launch_bounds__(256) void transr_rel_rows_kernel(RParArgs a, RParBufs<T> bf) {
    transr_rel_rows_wave<T, NORM>(a, bf, (blockIdx.x * blockDim.x + threadIdx.x) >> 6);
}

template <typename T, bool NORM, int E = 4>
__global__ __launch_bounds__(256) void transr_rel_rows4_kernel(RParArgs a, RParBufs<T> bf) {
    transr_rel_rows4_wave<T, NORM, E>(a, bf, (blockIdx.x * blockDim.x + threadIdx.x) >> 6);
}

// transRNorm (transr/trainer.cpp:35-64) per tile, on W'_r and the entity rows
// after the batch's gradient step.  Pairs: (h', r), (t', r) of the tile's
// active updates and (entity'[r], r) on the relation's first tile; a pair
// whose entity already occurs earlier in the tile is the reference's repeated
// call on an already constrained row, a no-op to first order, and is skipped.
// Per pair, with W0 = W'_r and the loop run in Jacobi form (all columns at
// once) while |p|^2 > 1 (p = W^T a):
//   g_m = 2 p_m,  a_{m+1} = a_m - lr W0 g_m,
//   p_{m+1} = W0^T a_{m+1} - lr (a0.a0) sum_{k<=m} g_k   (W's own shrink, to first order),
// then da = a_K - a0 (pair record) and the matrix step -lr a0 (sum_m g_m)^T
// (tile partial; exact to first order in lr).
constexpr int kRParMaxIter = 256;

template <typename T>
__global__ __launch_bounds__(256) void transr_constraint_kernel(RParArgs a, RParBufs<T> bf) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int t = a.tile_first[a.batch_seg[a.batch]] + blockIdx.x;
    if (t >= a.tile_first[a.batch_seg[a.batch + 1]]) return;
    int r, e0, cnt;
    tile_range(a, t, r, e0, cnt);
    const int n = a.n, ld = a.ld;
    T* Wl = (T*)smem;
    T* vec = Wl + n * ld;
    T* Xl = vec + 16 * ld;                // sum of g per pair   [4 cnt + 1][ld]
    T* Dl = Xl + (4 * a.St + 1) * ld;     // -lr a0 per pair     [4 cnt + 1][ld]
    int* ent_of = (int*)(Dl + (4 * a.St + 1) * ld + 4 * a.St + 1);  // [4 cnt + 1] entity of each pair slot
    const int w = threadIdx.x >> 6, l = lane_id();
    const RTile tl = a.tiles[t];
    bool relpair = false;  // the relation-level pair rides on the first tile
    if (tl.q == 0) {
        int any = 0;
        for (int q = a.tile_first[tl.seg]; q < a.tile_first[tl.seg + 1]; ++q) any |= a.tile_act[q];
        relpair = any != 0 && r < a.ne;
    }
    const int npairs = 4 * cnt + (relpair ? 1 : 0);  // slots (q, u, role), then entity[r]
    for (int pq = threadIdx.x; pq < npairs; pq += blockDim.x) {
        int ent = -1;
        if (pq < 4 * cnt) {
            const int q = pq >> 2, u = (pq >> 1) & 1, role = pq & 1;
            const int kk = a.kl.kk_of(a.keys[e0 + 2 * q]);
            if (a.act[kk]) {
                const int i0 = a.si[kk], jj = a.sj[kk];
                const int h = a.heads[i0], tt = a.tails[i0];
                const int hh = u ? (a.side[kk] ? h : jj) : h;
                const int th = u ? (a.side[kk] ? jj : tt) : tt;
                const int e = role ? th : hh;
                if (!transr_pair_dup(a, (kk * 2 + u) * 2 + role, r, e)) ent = e;
            }
        } else if (!transr_relpair_dup(a, r)) {
            ent = r;  // entityVec_next_[relation] (transr/trainer.cpp:187)
        }
        ent_of[pq] = ent;
    }
    stage_matrix(Wl, bf.W + (int64_t)r * n * ld, n, ld);
    __syncthreads();
    T* v4 = vec + w * 4 * ld;
    const int i = 2 * l;
    for (int pq = w; pq < npairs; pq += 4) {
        const int ent = ent_of[pq];
        bool live = ent >= 0;
        for (int k = 0; live && k < pq; ++k) live = ent_of[k] != ent;  // first occurrence only
        T a0[2] = {T(0), T(0)}, G[2] = {T(0), T(0)}, da[2] = {T(0), T(0)};
        if (live) {
            lane_pair_load(bf.ent + (int64_t)ent * ld, n, a0);
            const T s0 = wave_sum(a0[0] * a0[0] + a0[1] * a0[1]);
            lane_pair_store(v4, n, a0);
            wave_lds_sync();
            T p[2] = {T(0), T(0)};  // p = W'^T a0
            if (i < n)
                for (int j = 0; j < n; ++j) {
                    const T aj = v4[j];
                    p[0] += Wl[j * ld + i] * aj;
                    p[1] += Wl[j * ld + i + 1] * aj;
                }
            if (i + 1 >= n) p[1] = T(0);
            if (i >= n) p[0] = T(0);
            wave_lds_sync();
            for (int m = 0; m < kRParMaxIter; ++m) {
                const T xx = wave_sum(p[0] * p[0] + p[1] * p[1]);
                if (!(xx > T(1))) break;
                G[0] += T(2) * p[0];
                G[1] += T(2) * p[1];
                lane_pair_store(v4, n, p);
                wave_lds_sync();
                T v[2];
                matvec_rows(Wl, ld, n, v4, v);  // W p
                lane_pair_store(v4 + ld, n, v);
                wave_lds_sync();
                T q[2] = {T(0), T(0)};  // W^T (W p)
                if (i < n)
                    for (int j = 0; j < n; ++j) {
                        const T vj = v4[ld + j];
                        q[0] += Wl[j * ld + i] * vj;
                        q[1] += Wl[j * ld + i + 1] * vj;
                    }
                wave_lds_sync();
                const T c = T(2) * T(a.lr) * s0;
#pragma unroll
                for (int k = 0; k < 2; ++k) p[k] = i + k < n ? p[k] - T(2) * T(a.lr) * q[k] - c * p[k] : T(0);
            }
            lane_pair_store(v4, n, G);
            wave_lds_sync();
            matvec_rows(Wl, ld, n, v4, da);  // da = -lr W G
            da[0] *= T(-a.lr);
            da[1] *= T(-a.lr);
            wave_lds_sync();
        }
        if (pq < 4 * cnt) {
            const int q = pq >> 2, u = (pq >> 1) & 1, role = pq & 1;
            const int kk = a.kl.kk_of(a.keys[e0 + 2 * q]);
            if (a.act[kk]) lane_pair_store(bf.pair + (((int64_t)kk * 2 + u) * 2 + role) * ld, n, da);
        } else {
            lane_pair_store(bf.relpair + (int64_t)r * ld, n, da);
            if (l == 0) bf.relpair_stamp[r] = bf.stamp;
        }
        const T dv[2] = {T(-a.lr) * a0[0], T(-a.lr) * a0[1]};
        lane_pair_store(Xl + pq * ld, n, G);
        lane_pair_store(Dl + pq * ld, n, dv);
    }
    __syncthreads();
    T* wp = bf.wpart + (int64_t)blockIdx.x * n * ld;
    for (int j = w; j < n; j += 4) {
        T acc[2];
        rank_sum_rows(Dl, Xl, npairs, ld, n, j, acc);
        lane_pair_store(wp + (int64_t)j * ld, n, acc);
    }
}

// Entity rows, per entity segment of the batch (one wave; long segments a
// 1024-thread workgroup).  GRAD: head role -beta lr y, tail role +beta lr y
// (transr/trainer.cpp:168-169), then the unit norm (:175-176) if an active
// update used the row as head or tail.  !GRAD: the transRNorm pair deltas
// (and the (entity[r], r) delta once), no norm -- or, with bf.last_renorm (the
// per-relation chunk kernel, kernels_transr_seq.hpp), the deltas of pairs made
// before the row's last update of the batch ("pre": the reference's unit norm
// at that update follows them), a unit norm, then the deltas of the last
// update's own pairs ("post"; the (entity[r], r) delta is post when no update
// touches the row as head or tail, pre otherwise).
constexpr int kRParWaves = 16;

// The row's last active update in the batch, kk 2 + u (-1: none), over the
// events [p0 + 64 first, ...) of its segment in strides of 64 stride; the
// maximum in every lane.
__device__ __forceinline__ int rpar_entity_last(const RParArgs& a, int p0, int p1, int first, int stride) {
    const int l = lane_id();
    int last = -1;
    for (int base = p0 + first * kWave; base < p1; base += stride * kWave) {
        const int p = base + l;
        if (p < p1) {
            const uint64_t key = a.keys[p];
            const int kk = a.kl.kk_of(key);
            if (a.act[kk] && (key & (kRoleHead | kRoleTail))) last = max(last, kk * 2 + (int)((key >> 3) & 1));
        }
    }
#pragma unroll
    for (int s = 32; s >= 1; s >>= 1) last = max(last, __shfl_xor(last, s));
    return last;
}

// Events [p0 + 64 first, ...) of an entity segment in chunks of 64 (lane q:
// event q); the rows the active ones add (y rows, or transRNorm pair deltas)
// are then fetched four at a time, so a long segment keeps several loads in
// flight instead of one dependent chain per event.  acc / dirty: the deltas
// (GRAD, and !GRAD without last_renorm: all of them; with it: the pre ones),
// acc2 / dirty2: the post ones of update `last`.
template <typename T, bool GRAD>
__device__ __forceinline__ void rpar_entity_events(const RParArgs& a, const RParBufs<T>& bf, int row, int p0, int p1,
                                                   int first, int stride, int last, T (&acc)[2], T (&acc2)[2],
                                                   bool& dirty, bool& dirty2, bool& er_seen) {
    const int n = a.n, ld = a.ld, l = lane_id();
    const bool split = !GRAD && bf.last_renorm;
    for (int base = p0 + first * kWave; base < p1; base += stride * kWave) {
        const int p = base + l;
        int src = -1;     // row of the y / pair table this lane's event adds (GRAD: its y row)
        int src2 = -1;    // !GRAD: second pair row (the row is head and tail of the update)
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
                } else {  // pair records; with flags only those whose pair moved
                    const int s0 = (kk * 2 + u) * 2;
                    const bool ph = hd && (!bf.pflag || bf.pflag[s0]);
                    const bool pt = tl && (!bf.pflag || bf.pflag[s0 + 1]);
                    nrm = ph || pt;
                    post = split && kk * 2 + u == last;
                    if (ph) src = s0;
                    if (pt) {
                        if (src < 0) src = s0 + 1;
                        else src2 = s0 + 1;
                    }
                }
            }
        }
        if (__ballot(nrm && !post)) dirty = true;
        if (__ballot(nrm && post)) dirty2 = true;
        if (__ballot(er)) er_seen = true;
        const T* tab = GRAD ? bf.y : bf.pair;
        for (int pass = 0; pass < (GRAD ? 1 : 2); ++pass) {
            const int mine = pass ? src2 : src;
            uint64_t m = __ballot(mine >= 0);
            const uint64_t pm = __ballot(post);
            while (m) {
                int ev[4];
                int k = 0;
                for (; k < 4 && m; ++k) {
                    ev[k] = __builtin_ctzll(m);
                    m &= m - 1;
                }
                T v[4][2];
#pragma unroll
                for (int q = 0; q < 4; ++q)
                    if (q < k) lane_pair_load(tab + (int64_t)readlane_i32(mine, ev[q]) * ld, n, v[q]);
#pragma unroll
                for (int q = 0; q < 4; ++q)
                    if (q < k) {
                        const T cq = GRAD ? readlane_f(c, ev[q]) : T(1);
                        T(&dst)[2] = ((pm >> ev[q]) & 1) ? acc2 : acc;
                        dst[0] += cq * v[q][0];
                        dst[1] += cq * v[q][1];
                    }
            }
        }
    }
}

template <typename T, bool GRAD>
__device__ __forceinline__ void rpar_entity_finish(const RParArgs& a, const RParBufs<T>& bf, int row, T (&acc)[2],
                                                   T (&acc2)[2], bool dirty, bool dirty2, bool er_seen, int last) {
    const int n = a.n, ld = a.ld;
    const bool split = !GRAD && bf.last_renorm;
    if (!GRAD && er_seen && row < a.nr && bf.relpair_stamp[row] == bf.stamp) {
        T dv[2];
        lane_pair_load(bf.relpair + (int64_t)row * ld, n, dv);
        if (split && last < 0) {  // no update renormalises the row: the delta stays
            acc2[0] += dv[0];
            acc2[1] += dv[1];
            dirty2 = true;
        } else {
            acc[0] += dv[0];
            acc[1] += dv[1];
            dirty = true;
        }
    }
    if (!dirty && !dirty2) return;
    T* ptr = bf.ent + (int64_t)row * ld;
    T v[2];
    lane_pair_load(ptr, n, v);
    if (dirty) {
        v[0] += acc[0];
        v[1] += acc[1];
    }
    if (GRAD || (split && dirty)) {
        const T len = sqrt(wave_sum(v[0] * v[0] + v[1] * v[1]));
        v[0] = v[0] / len;
        v[1] = v[1] / len;
    }
    if (dirty2) {
        v[0] += acc2[0];
        v[1] += acc2[1];
    }
    lane_pair_store(ptr, n, v);
}

// the entity rows of workgroup `bid` of G (1024 threads)
template <typename T, bool GRAD>
__device__ __forceinline__ void transr_entity_block(RParArgs a, RParBufs<T> bf, int32_t long_min, int bid, int G) {
    __shared__ T part[kRParWaves][4][kWave];
    __shared__ int flags[4];
    __shared__ int longs[1024], nlong;
    const int w = threadIdx.x >> 6, l = lane_id();
    const bool split = !GRAD && bf.last_renorm;
    const int s0 = a.batch_seg[a.batch], s1 = a.rel_begin[a.batch];  // entity segments sort first
    const int blockIdx_x = bid;
    // long segments: whole workgroup, segments s0 + blockIdx_x, s0 + blockIdx_x + G, ... that are
    // long, found by one thread each (blockDim.x candidates per pass; the order between
    // segments is immaterial, each is a different row)
    for (int c0 = s0 + blockIdx_x; c0 < s1; c0 += G * (int)blockDim.x) {
        if (threadIdx.x == 0) nlong = 0;
        __syncthreads();
        const int cs = c0 + G * (int)threadIdx.x;
        if (cs < s1 && a.seg_start[cs + 1] - a.seg_start[cs] >= long_min) longs[atomicAdd(&nlong, 1)] = cs;
        __syncthreads();
        const int nl = nlong;
        for (int li = 0; li < nl; ++li) {
        const int s = longs[li];
        const int p0 = a.seg_start[s], p1 = a.seg_start[s + 1];
        const int row = a.seg_row[s];
        if (threadIdx.x < 4) flags[threadIdx.x] = threadIdx.x == 3 ? -1 : 0;
        __syncthreads();
        int last = -1;
        if (split) {  // the row's last update over the whole segment (chunks w, w + 16, ...)
            last = rpar_entity_last(a, p0, p1, w, kRParWaves);
            if (l == 0) atomicMax(&flags[3], last);
            __syncthreads();
            last = flags[3];
        }
        T acc[2] = {T(0), T(0)}, acc2[2] = {T(0), T(0)};
        bool dirty = false, dirty2 = false, er = false;
        rpar_entity_events<T, GRAD>(a, bf, row, p0, p1, w, kRParWaves, last, acc, acc2, dirty, dirty2,
                                    er);  // chunks w, w + 16, ...
        part[w][0][l] = acc[0];
        part[w][1][l] = acc[1];
        part[w][2][l] = acc2[0];
        part[w][3][l] = acc2[1];
        if (l == 0 && dirty) atomicOr(&flags[0], 1);
        if (l == 0 && er) atomicOr(&flags[1], 1);
        if (l == 0 && dirty2) atomicOr(&flags[2], 1);
        __syncthreads();
        if (w == 0) {
            acc[0] = part[0][0][l];
            acc[1] = part[0][1][l];
            acc2[0] = part[0][2][l];
            acc2[1] = part[0][3][l];
            for (int v = 1; v < kRParWaves; ++v) {
                acc[0] += part[v][0][l];
                acc[1] += part[v][1][l];
                acc2[0] += part[v][2][l];
                acc2[1] += part[v][3][l];
            }
            rpar_entity_finish<T, GRAD>(a, bf, row, acc, acc2, flags[0] != 0, flags[2] != 0, flags[1] != 0, last);
        }
        __syncthreads();
        }
    }
    // short segments: one wave each
    for (int s = s0 + blockIdx_x * kRParWaves + w; s < s1; s += G * kRParWaves) {
        const int p0 = a.seg_start[s], p1 = a.seg_start[s + 1];
        if (p1 - p0 >= long_min) continue;
        const int row = a.seg_row[s];
        const int last = split ? rpar_entity_last(a, p0, p1, 0, 1) : -1;
        T acc[2] = {T(0), T(0)}, acc2[2] = {T(0), T(0)};
        bool dirty = false, dirty2 = false, er = false;
        rpar_entity_events<T, GRAD>(a, bf, row, p0, p1, 0, 1, last, acc, acc2, dirty, dirty2, er);
        rpar_entity_finish<T, GRAD>(a, bf, row, acc, acc2, dirty, dirty2, er, last);
    }
}

template <typename T, bool GRAD>
__global__ __launch_bounds__(1024) void transr_entity_kernel(RParArgs a, RParBufs<T> bf, int32_t long_min) {
    transr_entity_block<T, GRAD>(a, bf, long_min, blockIdx.x, gridDim.x);
}

// Both row passes of one step in one launch (they touch disjoint tables):
// workgroups [0, egrid) the entity rows, the rest one wave per (relation, row).
// RM: the relation-row layout -- 0 a row a wave, 4 / 8 four rows a wave with 4 / 8
// elements a lane (n <= 64 / n <= 128)
template <typename T, bool PASS1, int RM>
__global__ __launch_bounds__(1024) void transr_rows_kernel(RParArgs a, RParBufs<T> bf, int32_t long_min,
                                                           int32_t egrid) {
    const int gw = (((int)blockIdx.x - egrid) * (int)blockDim.x + (int)threadIdx.x) >> 6;
    if ((int)blockIdx.x < egrid) transr_entity_block<T, PASS1>(a, bf, long_min, blockIdx.x, egrid);
    else if (RM == 4) transr_rel_rows4_wave<T, PASS1, 4>(a, bf, gw);
    else if (RM == 8) transr_rel_rows4_wave<T, PASS1, 8>(a, bf, gw);
    else transr_rel_rows_wave<T, PASS1>(a, bf, gw);
}

// ---- compat energy: the work-vector prefix scan over the batch's calls -------
//
// transr/transr.cpp:20-25 never zeroes the work vectors, so call c of the
// batch (pos, neg of sample 0, then of sample 1, ...) sees work + the sum of
// the projections of calls 0..c.  Two passes over chunks of kScanChunk calls
// (chunk sums; then per chunk its prefix, the inclusive scan inside it and the
// energies), one thread per (head/tail, element), coalesced rows.
constexpr int kScanChunk = 64;

static __attribute__((unused)) __global__ __launch_bounds__(256) void rpar_scan_sums_kernel(const double* proj, int64_t calls, int32_t ld,
                                                             int32_t n, double* sums) {
    const int c = blockIdx.x;
    const int64_t c0 = (int64_t)c * kScanChunk, c1 = min<int64_t>(calls, c0 + kScanChunk);
    for (int e = threadIdx.x; e < 2 * n; e += blockDim.x) {
        const int side = e / n, i = e % n;
        // four interleaved partial sums: 16 independent loads in flight per step
        double s[4] = {0, 0, 0, 0};
        for (int64_t k = c0; k < c1; k += 16) {
            double v[16];
#pragma unroll
            for (int q = 0; q < 16; ++q) v[q] = k + q < c1 ? proj[((k + q) * 2 + side) * ld + i] : 0.0;
#pragma unroll
            for (int q = 0; q < 16; ++q) s[q & 3] += v[q];
        }
        sums[(int64_t)c * 2 * n + e] = (s[0] + s[1]) + (s[2] + s[3]);
    }
}

// Many chunks (K5: 5,000 a batch): the exclusive prefix over the chunks once for
// all, pre[c][e] = work_in[e] + sum_{c' < c} sums[c'][e], instead of every block
// summing all earlier chunks (quadratic in the chunks: ~20 GB of L2 reads a K5
// batch).  A block takes 32 elements, 32 threads an element each over a
// contiguous run of chunks: run totals, their exclusive scan, then the prefix
// written along each run (rows of 32 consecutive elements: 256-byte accesses).
constexpr int kScanDirectMax = 256;  // chunks up to which every block sums its own prefix

static __attribute__((unused)) __global__ __launch_bounds__(1024) void rpar_scan_prefix_kernel(
    const double* sums, int32_t nchunks, int32_t E2, const double* work_in, double* pre) {
    __shared__ double tot[32][33];
    const int el = threadIdx.x & 31, part = threadIdx.x >> 5;
    const int e = blockIdx.x * 32 + el;
    const int per = (nchunks + 31) / 32;
    const int c0 = part * per, c1 = min(nchunks, c0 + per);
    double s = 0.0;
    if (e < E2) {
        for (int c = c0; c < c1; c += 8) {
            double v[8];
#pragma unroll
            for (int q = 0; q < 8; ++q) v[q] = c + q < c1 ? sums[(int64_t)(c + q) * E2 + e] : 0.0;
#pragma unroll
            for (int q = 0; q < 8; ++q) s += v[q];
        }
    }
    tot[part][el] = s;
    __syncthreads();
    double run = e < E2 ? work_in[e] : 0.0;
    for (int p = 0; p < part; ++p) run += tot[p][el];
    if (e >= E2) return;
    for (int c = c0; c < c1; c += 8) {
        double v[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) v[q] = c + q < c1 ? sums[(int64_t)(c + q) * E2 + e] : 0.0;
#pragma unroll
        for (int q = 0; q < 8; ++q)
            if (c + q < c1) {
                pre[(int64_t)(c + q) * E2 + e] = run;
                run += v[q];
            }
    }
}

// The chunk's exclusive prefix (work_in + the sums of all earlier chunks, each
// block summing them itself: no serial pass over the chunks; or pre[c] from
// rpar_scan_prefix_kernel when there are many chunks), the inclusive
// scan inside the chunk (LDS), then the compat energies of the chunk's
// kScanChunk / 2 samples (transr/transr.cpp:26-35 on the accumulated vectors)
// and the hinge (common/trainer.cpp:138-141).  The last chunk leaves the work
// vectors after the batch in work_out (ping-pong with work_in across batches).
template <typename T>
__global__ __launch_bounds__(1024) void rpar_scan_energy_kernel(RParArgs a, RParBufs<T> bf, const double* sums,
                                                                int32_t nchunks, const double* work_in,
                                                                double* work_out, const double* pre) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    double* run_l = (double*)smem;  // [kScanChunk][2 n]
    const int c = blockIdx.x, n = a.n, ld = a.ld;
    const int64_t calls = 2 * (int64_t)a.B;
    const int64_t c0 = (int64_t)c * kScanChunk, c1 = min<int64_t>(calls, c0 + kScanChunk);
    // the pair-dedupe slots of the chunk's samples (thread 4 q + slot): entity and
    // relation loaded now, recorded once the hinge is known
    __shared__ int act_l[kScanChunk / 2];
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
    // the sums of all earlier chunks: G thread groups per element, group g over chunks
    // g*16.., (g+G)*16.., sixteen loads in flight (one round trip for FB15k's ~150
    // chunks instead of ten), combined in group order
    const int E2 = 2 * n, G = max(1, (int)blockDim.x / E2);
    double* part = run_l + kScanChunk * E2;  // [G][2 n]
    if (!pre && (int)threadIdx.x < G * E2) {
        const int g = threadIdx.x / E2, e = threadIdx.x % E2;
        double s[4] = {0, 0, 0, 0};
        for (int q0 = g * 16; q0 < c; q0 += G * 16) {
            double v[16];
#pragma unroll
            for (int q = 0; q < 16; ++q) v[q] = q0 + q < c ? sums[(int64_t)(q0 + q) * E2 + e] : 0.0;
#pragma unroll
            for (int q = 0; q < 16; ++q) s[q & 3] += v[q];
        }
        part[g * E2 + e] = (s[0] + s[1]) + (s[2] + s[3]);
    }
    __syncthreads();
    for (int e = threadIdx.x; e < 2 * n; e += blockDim.x) {
        double run;
        if (pre) {
            run = pre[(int64_t)c * E2 + e];
        } else {
            double p = 0.0;
            for (int g = 0; g < G; ++g) p += part[g * E2 + e];
            run = work_in[e] + p;
        }
        const int side = e / n, i = e % n;
        for (int64_t k = c0; k < c1; k += 16) {
            double v[16];
#pragma unroll
            for (int q = 0; q < 16; ++q) v[q] = k + q < c1 ? a.proj[((k + q) * 2 + side) * ld + i] : 0.0;
#pragma unroll
            for (int q = 0; q < 16; ++q)
                if (k + q < c1) {
                    run += v[q];
                    run_l[(k + q - c0) * 2 * n + e] = run;
                }
        }
        if (c == nchunks - 1) work_out[e] = run;
    }
    __syncthreads();
    const int w = threadIdx.x >> 6, nw = blockDim.x >> 6, l = lane_id();
    for (int64_t kk = c0 / 2 + w; kk < c1 / 2; kk += nw) {
        const int r = a.rels[a.si[kk]];
        T vr[2];
        lane_pair_load(bf.rel + (int64_t)r * ld, n, vr);
        const double* pp = run_l + (kk * 2 - c0) * 2 * n;  // [pos: head n, tail n][neg: head n, tail n]
        double ep = 0, en = 0;
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            const int i = 2 * l + k;
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

// ---- per-epoch tile index --------------------------------------------------

// Tiles per segment (relation segments: ceil(samples / St); entity segments 0),
// and the first relation segment of every batch.
static __attribute__((unused)) __global__ __launch_bounds__(256) void rtile_count_kernel(const uint64_t* keys, const int32_t* seg_start,
                                                          const int32_t* nseg_p, int64_t cap, KeyLayout kl,
                                                          int32_t ne, int32_t St, int32_t* ntiles,
                                                          int32_t* rel_begin) {
    const int nseg = *nseg_p;
    for (int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; s < cap; s += (int64_t)gridDim.x * blockDim.x) {
        if (s >= nseg) {
            ntiles[s] = 0;
            continue;
        }
        const uint64_t k = keys[seg_start[s]];
        const int row = kl.row_of(k);
        const bool isrel = row >= ne;
        const int ns = (seg_start[s + 1] - seg_start[s]) / 2;
        ntiles[s] = isrel ? (ns + St - 1) / St : 0;
        if (isrel) {
            const bool first = s == 0 || kl.batch_of(keys[seg_start[s - 1]]) != kl.batch_of(k) ||
                               kl.row_of(keys[seg_start[s - 1]]) < ne;
            if (first) rel_begin[kl.batch_of(k)] = (int32_t)s;
        }
    }
}

static __attribute__((unused)) __global__ __launch_bounds__(256) void rtile_scatter_kernel(const int32_t* ntiles, const int32_t* tile_first,
                                                            const int32_t* nseg_p, RTile* tiles) {
    const int nseg = *nseg_p;
    for (int s = blockIdx.x * blockDim.x + threadIdx.x; s < nseg; s += gridDim.x * blockDim.x)
        for (int q = 0; q < ntiles[s]; ++q) tiles[tile_first[s] + q] = RTile{s, q};
}

// Per epoch, after the tiles: each tile's relation, count, samples and the
// entities of its rows (sample q: h, t, h', t'), and the first tile of each batch.
struct RTileDescArgs {
    const uint64_t* keys;
    const int32_t* seg_start;
    const int32_t* seg_row;
    const RTile* tiles;
    const int32_t* tile_first;
    const int32_t* nseg;
    const int32_t* batch_seg;
    int32_t nb, St, ne, B;
    int32_t sub, Bs;    // index batches a batch, samples an index batch (kb2e_config.sub_batches)
    KeyLayout kl;
    const int32_t* si;  // the epoch's sample stream
    const int32_t* sj;
    const uint8_t* side;
    const int32_t* heads;
    const int32_t* tails;
    int32_t* batch_t0;
    int32_t* td_r;
    int32_t* td_cnt;
    int32_t* td_kk;
    int32_t* td_ent;
};

static __attribute__((unused)) __global__ __launch_bounds__(256) void rtile_desc_kernel(RTileDescArgs a) {
    const int ntiles = a.tile_first[*a.nseg];
    const int gid = blockIdx.x * blockDim.x + threadIdx.x;
    if (gid <= a.nb) a.batch_t0[gid] = a.tile_first[a.batch_seg[gid]];
    for (int64_t x = gid; x < (int64_t)ntiles * 8; x += (int64_t)gridDim.x * blockDim.x) {
        const int t = (int)(x >> 3), q = (int)(x & 7);
        const RTile tl = a.tiles[t];
        const int p0 = a.seg_start[tl.seg], p1 = a.seg_start[tl.seg + 1];
        const int f = tl.q * a.St, cnt = min(a.St, (p1 - p0) / 2 - f);
        if (q == 0) {
            a.td_r[t] = a.seg_row[tl.seg] - a.ne;
            const bool single = a.tile_first[tl.seg + 1] - a.tile_first[tl.seg] == 1;
            a.td_cnt[t] = cnt | (single ? 256 : 0);
        }
        int kk = 0, e4[4] = {-1, -1, -1, -1};
        if (q < cnt) {
            const uint64_t key = a.keys[p0 + 2 * (f + q)];
            kk = a.kl.kk_of(key);
            const int ib = a.kl.batch_of(key);
            const int64_t k = (int64_t)(ib / a.sub) * a.B + (int64_t)(ib % a.sub) * a.Bs + kk;
            const int i0 = a.si[k], jj = a.sj[k];
            const int h = a.heads[i0], tt = a.tails[i0];
            const bool sd = a.side[k] != 0;
            e4[0] = h;
            e4[1] = tt;
            e4[2] = sd ? h : jj;
            e4[3] = sd ? jj : tt;
        }
        a.td_kk[x] = kk;
        *(int4*)(a.td_ent + 4 * x) = make_int4(e4[0], e4[1], e4[2], e4[3]);
    }
}

}  // namespace kb2e
