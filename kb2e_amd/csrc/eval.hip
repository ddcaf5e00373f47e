// eval.hip -- link-prediction evaluation on the device (EmbeddingEvaluation::run,
// common/evaluation.cpp:107-251).  Part of libkb2e.so (kb2e_evaluate,
// kb2e_evaluate_transr_compat in engine.hip call in here).
//
// For every test triple and both corruption sides the reference scores all |E|
// candidate triples, sorts them and reads off the raw rank (position of the
// true triple) and the filtered rank (1 + candidates ranked above it that are
// not known triples).  Ties with the true triple's energy are ranked after it
// (std::sort leaves their order unspecified; the oracle uses the same rule).
//
// * Stateless energies (evaluate_fixed): eval_project_kernel writes each
//   entity's model projection for one relation into a TRANSPOSED table
//   PT[k][i] (TransE: the row; TransH: e - (w.e) w, transh/transh.cpp:18-26;
//   TransR: W^T e with zeroed work vectors), then eval_rank_kernel gives one
//   thread per candidate and a tile of kQ queries in LDS; each energy is summed
//   over k in the reference's serial order, bit-identical to its FP64 value.
//
// * TransR compat (evaluate_transr_compat): the reference never zeroes the
//   energy work vectors (transr/transr.cpp:20-25, transr/evaluation.cpp:22-23),
//   so each computed energy depends on every energy computed before it, in the
//   order of its cached relation-major loop (common/evaluation.cpp:107-121,
//   213-238).  That order is a single dependency chain per vector element; it
//   is replayed exactly (same operations, same order, FP64) by one wave of
//   compat_chain_kernel while a loader wave stages the next candidates' rows
//   and a summing wave turns finished calls into energies; which pairs the
//   reference computes (and which it reads back from its per-relation cache)
//   is decided from first-occurrence indices (host, compat_plan).  Ranking is
//   then parallel (compat_rank_kernel) over the cached or per-pass energies.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <cstdlib>
#include <cmath>
#include <stdexcept>
#include <vector>

#include "eval.hpp"
#include "hip_util.hpp"
#include "host_data.hpp"
#include "kernels_common.hpp"

namespace kb2e {
namespace {

constexpr int kQ = 16;                   // queries per rank tile
constexpr int kMaxCacheEntities = 40000;  // common/evaluation.h:11
constexpr size_t kLdsMax = 160 * 1024;

// host_data.hpp mix64 on the device: the FilterSet slot of a key
__device__ __forceinline__ uint64_t eval_mix64(uint64_t x) {
    x ^= x >> 31;
    x *= 0x7fb5d329728ea185ull;
    x ^= x >> 27;
    x *= 0x81dadef4bc2dd44dull;
    x ^= x >> 33;
    return x;
}

struct FilterView {
    const uint64_t* slots;
    uint64_t mask, nr64, ne64;
    __device__ __forceinline__ bool has(int64_t h, int64_t r, int64_t t) const {
        const uint64_t k = ((uint64_t)h * nr64 + (uint64_t)r) * ne64 + (uint64_t)t;
        uint64_t p = eval_mix64(k) & mask;
        while (true) {
            const uint64_t s = slots[p];
            if (s == k) return true;
            if (s == ~0ull) return false;
            p = (p + 1) & mask;
        }
    }
};

// ------------------------------------------------------------ fixed energies

template <typename T>
struct ProjArgs {
    int32_t model, n, ld, ne, r;
    const T* ent;
    const T* rel;
    const T* w;
    double* PT;    // [n][ne]
    double* relv;  // [n] relation r in FP64
};

// One thread per entity: its projection for relation r, in FP64, summed in the
// reference's order.
template <typename T>
__global__ __launch_bounds__(256) void eval_project_kernel(ProjArgs<T> a) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    for (int k = i; k < a.n; k += (int)(gridDim.x * blockDim.x)) a.relv[k] = (double)a.rel[(int64_t)a.r * a.ld + k];
    if (i >= a.ne) return;
    const T* e = a.ent + (int64_t)i * a.ld;
    if (a.model == 0) {
        for (int k = 0; k < a.n; ++k) a.PT[(int64_t)k * a.ne + i] = (double)e[k];
    } else if (a.model == 1) {
        const T* w = a.w + (int64_t)a.r * a.ld;
        double s = 0;
        for (int k = 0; k < a.n; ++k) s += (double)w[k] * (double)e[k];
        for (int k = 0; k < a.n; ++k) a.PT[(int64_t)k * a.ne + i] = (double)e[k] - s * (double)w[k];
    } else {
        const T* W = a.w + (int64_t)a.r * a.n * a.ld;
        for (int k = 0; k < a.n; ++k) {
            double s = 0;
            for (int j = 0; j < a.n; ++j) s += (double)W[(int64_t)j * a.ld + k] * (double)e[j];
            a.PT[(int64_t)k * a.ne + i] = s;
        }
    }
}

struct RankArgs {
    const double* PT;    // [n][ne]
    const double* relv;  // [n]
    int32_t n, ne, l1, r;
    const int32_t* qh;  // queries of this relation
    const int32_t* qt;
    int32_t nq;
    FilterView filt;
    unsigned long long* counts;  // [nq][4]: head raw, head filtered, tail raw, tail filtered
    double* target;              // [nq] true energies
};

__device__ __forceinline__ double eval_energy(const RankArgs& a, int h, int t) {
    double e = 0;
    for (int k = 0; k < a.n; ++k) {
        const double d = a.PT[(int64_t)k * a.ne + t] - a.PT[(int64_t)k * a.ne + h] - a.relv[k];
        e += a.l1 ? fabs(d) : d * d;
    }
    return e;
}

__global__ __launch_bounds__(256) void eval_target_kernel(RankArgs a) {
    const int q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q < a.nq) a.target[q] = eval_energy(a, a.qh[q], a.qt[q]);
}

// grid.x: entity blocks of 256; grid.y: query tiles of kQ.  Dynamic LDS:
// P(true head), P(true tail) of the tile's queries [kQ][n] each + r [n]; when
// that does not fit (n > 600, kRowsInLds false) the query rows are read from the
// projection table itself (every thread of a block the same address: L1/L2
// broadcasts), so any --size ranks, as in the reference.
template <bool kRowsInLds>
__global__ __launch_bounds__(256) void eval_rank_kernel(RankArgs a) {
    extern __shared__ __attribute__((aligned(16))) double lds[];
    double* th = lds;
    double* tt = th + kQ * a.n;
    double* rv = tt + kQ * a.n;
    __shared__ unsigned int cnt[kQ][4];
    const int q0 = blockIdx.y * kQ;
    const int nq = min(kQ, a.nq - q0);
    if constexpr (kRowsInLds) {
        for (int x = threadIdx.x; x < kQ * a.n; x += blockDim.x) {
            const int q = x / a.n, k = x % a.n;
            if (q < nq) {
                th[x] = a.PT[(int64_t)k * a.ne + a.qh[q0 + q]];
                tt[x] = a.PT[(int64_t)k * a.ne + a.qt[q0 + q]];
            }
        }
        for (int k = threadIdx.x; k < a.n; k += blockDim.x) rv[k] = a.relv[k];
    }
    int qhv[kQ], qtv[kQ];  // the tile's query entities (kRowsInLds false)
#pragma unroll
    for (int q = 0; q < kQ; ++q) {
        qhv[q] = q < nq ? a.qh[q0 + q] : 0;
        qtv[q] = q < nq ? a.qt[q0 + q] : 0;
    }
    if (threadIdx.x < kQ * 4) cnt[threadIdx.x / 4][threadIdx.x % 4] = 0;
    __syncthreads();
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < a.ne) {
        double eh[kQ], et[kQ];  // head replaced by i / tail replaced by i
#pragma unroll
        for (int q = 0; q < kQ; ++q) eh[q] = et[q] = 0;
        for (int k = 0; k < a.n; ++k) {
            const double* col = a.PT + (int64_t)k * a.ne;
            const double v = col[i];
            const double r = kRowsInLds ? rv[k] : a.relv[k];
#pragma unroll
            for (int q = 0; q < kQ; ++q) {
                const double pt = kRowsInLds ? tt[q * a.n + k] : col[qtv[q]];
                const double ph = kRowsInLds ? th[q * a.n + k] : col[qhv[q]];
                const double dh = pt - v - r;  // (P(t) - P(i)) - r
                const double dt = v - ph - r;  // (P(i) - P(h)) - r
                eh[q] += a.l1 ? fabs(dh) : dh * dh;
                et[q] += a.l1 ? fabs(dt) : dt * dt;
            }
        }
#pragma unroll
        for (int q = 0; q < kQ; ++q) {
            if (q >= nq) continue;
            const int h = a.qh[q0 + q], t = a.qt[q0 + q];
            const double target = a.target[q0 + q];
            if (i != h && eh[q] < target) {
                atomicAdd(&cnt[q][0], 1u);
                if (!a.filt.has(i, a.r, t)) atomicAdd(&cnt[q][1], 1u);
            }
            if (i != t && et[q] < target) {
                atomicAdd(&cnt[q][2], 1u);
                if (!a.filt.has(h, a.r, i)) atomicAdd(&cnt[q][3], 1u);
            }
        }
    }
    __syncthreads();
    if (threadIdx.x < nq * 4) {
        const int q = threadIdx.x / 4, c = threadIdx.x % 4;
        if (cnt[q][c]) atomicAdd(&a.counts[(int64_t)(q0 + q) * 4 + c], (unsigned long long)cnt[q][c]);
    }
}

// ------------------------------------------------------------ TransR compat

// One evalCorruption pass (common/evaluation.cpp:124-179).
struct CompatPass {
    int32_t rel, h, t;
    int32_t side;     // 0: corrupt the head (calls (i, t)); 1: corrupt the tail (calls (h, x))
    int64_t ftime;    // offset of the first-occurrence array deciding which candidates are
                      // computed (not cached): candidate c iff ftime[c] >= thr; -1: all
    int32_t thr;
    int32_t out_row;  // no cache: row of the per-pass energy buffer
};

template <typename T>
struct CompatChainArgs {
    const T* ent;
    const T* rel;
    const T* W;  // [nr][n][ld]
    int32_t n, ld, ne, l1, G;
    int32_t wglob;  // W read from global memory (L2) instead of an LDS image: dims whose n x n image does not fit
    const CompatPass* passes;
    int32_t npass;
    const int32_t* ftime;
    double* work;   // [2][n] head, tail work vectors (persist across launches)
    double* cache;  // [ne][ne] (head-major) or nullptr
    double* pbuf;   // [rows][ne] when no cache
};

constexpr int kChainThreads = 192;  // wave 0: chain, wave 1: energies, wave 2: loader

__host__ __device__ constexpr size_t chain_lds_bytes(int n, int G, bool wglob = false) {
    return 8 * ((wglob ? 0 : (size_t)n * n) + 3 * (size_t)G * n + 3 * (size_t)n) + 4 * (3 * (size_t)G + 8);
}

// The calls of `npass` passes in the reference's order.  Each step: the loader
// fills buffer s%3 with the next <= G computed candidates of one pass (ids +
// FP64 rows + the pass's fixed row), the chain wave replays buffer (s-1)%3 --
// per call, per element i in lane i, headVec[i] += W[j][i] h[j] and
// tailVec[i] += W[j][i] t[j] for j = 0..n-1 (transr/transr.cpp:20-25), then
// |tailVec[i] - headVec[i] - r[i]| (or its square) into the call's slot --
// and the summing wave adds buffer (s-2)%3's terms over i in order
// (transr/transr.cpp:27-34) and stores the energies.
template <typename T, int CH>
__global__ __launch_bounds__(kChainThreads) void compat_chain_kernel(CompatChainArgs<T> a) {
    extern __shared__ __attribute__((aligned(16))) double lds[];
    const int n = a.n, G = a.G;
    double* Wl = lds;                        // [n][n]: W[j][i] of the current relation (LDS image)
    double* slots = Wl + (a.wglob ? 0 : (size_t)n * n);  // [3][G][n]: candidate rows, then the call's terms
    double* bvec = slots + (size_t)3 * G * n;  // [3][n]: the pass's fixed entity row
    int* ids = (int*)(bvec + 3 * n);         // [3][G]
    int* cnt = ids + 3 * G;                  // [3]
    int* gpass = cnt + 3;                    // [3]
    int* exh = gpass + 3;                    // [1]: step at which the loader ran dry
    const int wv = threadIdx.x >> 6, l = lane_id();
    if (threadIdx.x == 0) *exh = -1;
    // chain-wave state
    double hv[CH], tv[CH], rv[CH];
    int cur_rel = -1;
    if (wv == 0) {
#pragma unroll
        for (int c = 0; c < CH; ++c) {
            const int i = l + 64 * c;
            hv[c] = i < n ? a.work[i] : 0.0;
            tv[c] = i < n ? a.work[n + i] : 0.0;
            rv[c] = 0.0;
        }
    }
    // loader state (wave-uniform)
    int lp = 0, lcur = 0;
    __syncthreads();
    for (int s = 0;; ++s) {
        if (wv == 2) {
            const int L = s % 3;
            int got = 0, gp = -1;
            while (lp < a.npass && got < G) {
                const CompatPass ps = a.passes[lp];
                const int c = lcur + l;
                const bool ok = c < a.ne && (ps.ftime < 0 || a.ftime[ps.ftime + c] >= ps.thr);
                const uint64_t m = __ballot(ok);
                const int avail = __popcll(m);
                const int take = min(avail, G - got);
                const int pos = __popcll(m & ((1ull << l) - 1));
                if (ok && pos < take) ids[L * G + got + pos] = c;
                gp = lp;
                got += take;
                if (take < avail) {  // group full inside this chunk: resume at the first candidate not taken
                    const uint64_t nxt = __ballot(ok && pos == take);
                    lcur += __ffsll((long long)nxt) - 1;
                    break;
                }
                lcur += 64;
                if (lcur >= a.ne) {  // pass done: a group never spans two passes
                    ++lp;
                    lcur = 0;
                    if (got > 0) break;
                }
            }
            if (got > 0) {
                const CompatPass ps = a.passes[gp];
                for (int q = 0; q < got; ++q) {
                    const T* row = a.ent + (int64_t)ids[L * G + q] * a.ld;
                    for (int i = l; i < n; i += 64) slots[((size_t)L * G + q) * n + i] = (double)row[i];
                }
                const T* fr = a.ent + (int64_t)(ps.side == 0 ? ps.t : ps.h) * a.ld;
                for (int i = l; i < n; i += 64) bvec[L * n + i] = (double)fr[i];
            }
            if (l == 0) {
                cnt[L] = got > 0 ? got : -1;
                gpass[L] = gp;
                if (got == 0 && *exh < 0) *exh = s;
            }
        } else if (wv == 0 && s >= 1) {
            const int C = (s + 2) % 3;
            const int k = cnt[C];
            if (k > 0) {
                const CompatPass ps = a.passes[gpass[C]];
                if (ps.rel != cur_rel) {
                    cur_rel = ps.rel;
                    const T* Wg = a.W + (int64_t)cur_rel * n * a.ld;
                    if (!a.wglob)
                        for (int idx = l; idx < n * n; idx += 64) Wl[idx] = (double)Wg[(int64_t)(idx / n) * a.ld + idx % n];
#pragma unroll
                    for (int c = 0; c < CH; ++c) {
                        const int i = l + 64 * c;
                        rv[c] = i < n ? (double)a.rel[(int64_t)cur_rel * a.ld + i] : 0.0;
                    }
                    wave_lds_sync();
                }
                const double* y = bvec + C * n;
                // the candidate is the head (side 0) or the tail (side 1) of each call
                double va[CH], fa[CH];
#pragma unroll
                for (int c = 0; c < CH; ++c) {
                    va[c] = ps.side == 0 ? hv[c] : tv[c];
                    fa[c] = ps.side == 0 ? tv[c] : hv[c];
                }
                const T* Wg = a.W + (int64_t)cur_rel * n * a.ld;  // (the wglob form: rows of ld, from L2)
                for (int q = 0; q < k; ++q) {
                    double* x = slots + ((size_t)C * G + q) * n;
#pragma unroll
                    for (int c = 0; c < CH; ++c) {
                        const int i = l + 64 * c;
                        if (i < n) {
                            double v = va[c], f = fa[c];
                            if (a.wglob) {
                                for (int j = 0; j < n; ++j) {
                                    const double w = (double)Wg[(int64_t)j * a.ld + i];
                                    v += w * x[j];
                                    f += w * y[j];
                                }
                            } else {
                                for (int j = 0; j < n; ++j) {
                                    const double w = Wl[j * n + i];
                                    v += w * x[j];
                                    f += w * y[j];
                                }
                            }
                            va[c] = v;
                            fa[c] = f;
                        }
                    }
                    wave_lds_sync();  // every lane has read x before its slot is overwritten
#pragma unroll
                    for (int c = 0; c < CH; ++c) {
                        const int i = l + 64 * c;
                        if (i < n) {
                            const double hh = ps.side == 0 ? va[c] : fa[c];
                            const double tt = ps.side == 0 ? fa[c] : va[c];
                            const double d = tt - hh - rv[c];
                            x[i] = a.l1 ? fabs(d) : d * d;
                        }
                    }
                    wave_lds_sync();
                }
#pragma unroll
                for (int c = 0; c < CH; ++c) {
                    hv[c] = ps.side == 0 ? va[c] : fa[c];
                    tv[c] = ps.side == 0 ? fa[c] : va[c];
                }
            }
        } else if (wv == 1 && s >= 2) {
            const int S = (s + 1) % 3;
            const int k = cnt[S];
            if (k > 0 && l < k) {
                const CompatPass ps = a.passes[gpass[S]];
                const double* x = slots + ((size_t)S * G + l) * n;
                double e = 0;
                for (int i = 0; i < n; ++i) e += x[i];
                const int c = ids[S * G + l];
                if (a.cache) {
                    const int64_t hh = ps.side == 0 ? c : ps.h, tt = ps.side == 0 ? ps.t : c;
                    a.cache[hh * a.ne + tt] = e;
                } else {
                    a.pbuf[(int64_t)ps.out_row * a.ne + c] = e;
                }
            }
        }
        __syncthreads();
        const int ex = *exh;
        if (ex >= 0 && s >= ex + 2) break;
    }
    if (wv == 0) {
#pragma unroll
        for (int c = 0; c < CH; ++c) {
            const int i = l + 64 * c;
            if (i < n) {
                a.work[i] = hv[c];
                a.work[n + i] = tv[c];
            }
        }
    }
}

struct CompatRankArgs {
    const CompatPass* passes;
    int32_t npass, ne;
    const double* cache;
    const double* pbuf;
    FilterView filt;
    unsigned long long* counts;  // [npass][3]: raw, filtered, ties
};

// grid.x: candidate blocks of 256, grid.y: passes.
__global__ __launch_bounds__(256) void compat_rank_kernel(CompatRankArgs a) {
    __shared__ unsigned int cnt[3];
    const CompatPass ps = a.passes[blockIdx.y];
    if (threadIdx.x < 3) cnt[threadIdx.x] = 0;
    __syncthreads();
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const int truth = ps.side == 0 ? ps.h : ps.t;
    if (i < a.ne && i != truth) {
        double e, target;
        if (a.cache) {
            e = ps.side == 0 ? a.cache[(int64_t)i * a.ne + ps.t] : a.cache[(int64_t)ps.h * a.ne + i];
            target = a.cache[(int64_t)ps.h * a.ne + ps.t];
        } else {
            e = a.pbuf[(int64_t)ps.out_row * a.ne + i];
            target = a.pbuf[(int64_t)ps.out_row * a.ne + truth];
        }
        if (e < target) {
            atomicAdd(&cnt[0], 1u);
            const bool known = ps.side == 0 ? a.filt.has(i, ps.rel, ps.t) : a.filt.has(ps.h, ps.rel, i);
            if (!known) atomicAdd(&cnt[1], 1u);
        } else if (e == target) {
            atomicAdd(&cnt[2], 1u);
        }
    }
    __syncthreads();
    if (threadIdx.x < 3 && cnt[threadIdx.x])
        atomicAdd(&a.counts[(int64_t)blockIdx.y * 3 + threadIdx.x], (unsigned long long)cnt[threadIdx.x]);
}

// ------------------------------------------------------------ host side

struct Grouped {
    std::vector<std::vector<int64_t>> byrel;  // test triple indices per relation, file order
};

Grouped group_tests(const EvalTables& t, const EvalQuery& q) {
    Grouped g;
    g.byrel.resize(t.nr);
    for (int64_t k = 0; k < q.ntest; ++k) {
        if (q.th[k] < 0 || q.th[k] >= t.ne || q.tt[k] < 0 || q.tt[k] >= t.ne || q.tr[k] < 0 || q.tr[k] >= t.nr)
            throw std::invalid_argument("test triple out of range");
        g.byrel[q.tr[k]].push_back(k);
    }
    return g;
}

struct DeviceFilter {
    FilterSet fs;
    DevBuf slots;
    FilterView view(int64_t ne, int64_t nr) const {
        return FilterView{slots.as<uint64_t>(), fs.mask, (uint64_t)nr, (uint64_t)ne};
    }
};

void build_filter(const EvalTables& t, const EvalQuery& q, DeviceFilter& df) {
    std::vector<int32_t> H(q.fh, q.fh + q.nfilter), T(q.ft, q.ft + q.nfilter), R(q.fr, q.fr + q.nfilter);
    for (int64_t k = 0; k < q.nfilter; ++k)
        if (H[k] < 0 || H[k] >= t.ne || T[k] < 0 || T[k] >= t.ne || R[k] < 0 || R[k] >= t.nr)
            throw std::invalid_argument("filter triple out of range");
    df.fs.build(H, T, R, t.ne, t.nr);
    df.slots.alloc(df.fs.slots.size() * 8);
    HIPCHK(hipMemcpyAsync(df.slots.p, df.fs.slots.data(), df.fs.slots.size() * 8, hipMemcpyHostToDevice, t.stream));
}

template <typename K>
void allow_lds(K kernel, size_t bytes) {
    HIPCHK(hipFuncSetAttribute((const void*)kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes));
}

void finish(long long rawSum, long long filtSum, long long rawHits, long long filtHits, int64_t ntest, double* out) {
    const double nc = (double)ntest * 2.0;  // common/evaluation.cpp:246-250
    out[0] = rawSum / nc;
    out[1] = rawHits / nc;
    out[2] = filtSum / nc;
    out[3] = filtHits / nc;
}

template <typename T>
void project(const EvalTables& t, int r, double* PT, double* relv) {
    ProjArgs<T> a{t.model, t.n, t.ld, t.ne, r, (const T*)t.ent, (const T*)t.rel, (const T*)t.w, PT, relv};
    eval_project_kernel<T><<<(std::max(t.ne, t.n) + 255) / 256, 256, 0, t.stream>>>(a);
    HIPCHK(hipGetLastError());
}

template <typename T, int CH>
void launch_chain(const EvalTables& t, const CompatChainArgs<T>& a, size_t lds) {
    allow_lds(compat_chain_kernel<T, CH>, lds);
    compat_chain_kernel<T, CH><<<1, kChainThreads, lds, t.stream>>>(a);
    HIPCHK(hipGetLastError());
}

template <typename T>
void run_chain(const EvalTables& t, CompatChainArgs<T> a) {
    if (a.npass == 0) return;
    const size_t lds = chain_lds_bytes(t.n, a.G, a.wglob != 0);
    switch ((t.n + 63) / 64) {
        case 1: launch_chain<T, 1>(t, a, lds); break;
        case 2: launch_chain<T, 2>(t, a, lds); break;
        case 3: launch_chain<T, 3>(t, a, lds); break;
        case 4: launch_chain<T, 4>(t, a, lds); break;
        case 5: launch_chain<T, 5>(t, a, lds); break;
        case 6: launch_chain<T, 6>(t, a, lds); break;
        case 7: launch_chain<T, 7>(t, a, lds); break;
        case 8: launch_chain<T, 8>(t, a, lds); break;
        default: throw std::invalid_argument("TransR compat evaluation supports dim <= 512");
    }
}

}  // namespace

void evaluate_fixed(const EvalTables& t, const EvalQuery& q, double out[4]) {
    if (q.ntest < 1) throw std::invalid_argument("empty test set");
    const int ne = t.ne, n = t.n;
    // n <= 600; KB2E_EVAL_ROWS_L2=1 forces the L2 form (tests)
    const char* l2 = getenv("KB2E_EVAL_ROWS_L2");
    const bool rows_lds = (size_t)(2 * kQ + 1) * n * 8 <= kLdsMax && !(l2 && l2[0] == '1');
    const size_t rank_lds = rows_lds ? (size_t)(2 * kQ + 1) * n * 8 : 0;
    Grouped g = group_tests(t, q);
    DeviceFilter df;
    build_filter(t, q, df);
    std::vector<int32_t> qh, qt;
    std::vector<int64_t> qoff(t.nr + 1, 0);
    for (int r = 0; r < t.nr; ++r) {
        for (int64_t k : g.byrel[r]) {
            qh.push_back(q.th[k]);
            qt.push_back(q.tt[k]);
        }
        qoff[r + 1] = (int64_t)qh.size();
    }
    DevBuf d_qh, d_qt, d_counts, d_target, d_PT, d_relv;
    d_qh.alloc(qh.size() * 4);
    d_qt.alloc(qt.size() * 4);
    HIPCHK(hipMemcpyAsync(d_qh.p, qh.data(), qh.size() * 4, hipMemcpyHostToDevice, t.stream));
    HIPCHK(hipMemcpyAsync(d_qt.p, qt.data(), qt.size() * 4, hipMemcpyHostToDevice, t.stream));
    d_counts.alloc(qh.size() * 4 * 8);
    HIPCHK(hipMemsetAsync(d_counts.p, 0, d_counts.bytes, t.stream));
    d_target.alloc(qh.size() * 8);
    d_PT.alloc((size_t)n * ne * 8);
    d_relv.alloc((size_t)n * 8);
    if (rows_lds) allow_lds(eval_rank_kernel<true>, rank_lds);
    for (int r = 0; r < t.nr; ++r) {
        const int64_t nq = qoff[r + 1] - qoff[r];
        if (nq == 0) continue;
        if (t.f64) project<double>(t, r, d_PT.as<double>(), d_relv.as<double>());
        else project<float>(t, r, d_PT.as<double>(), d_relv.as<double>());
        RankArgs ra{};
        ra.PT = d_PT.as<double>();
        ra.relv = d_relv.as<double>();
        ra.n = n;
        ra.ne = ne;
        ra.l1 = t.l1;
        ra.r = r;
        ra.qh = d_qh.as<int32_t>() + qoff[r];
        ra.qt = d_qt.as<int32_t>() + qoff[r];
        ra.nq = (int32_t)nq;
        ra.filt = df.view(ne, t.nr);
        ra.counts = d_counts.as<unsigned long long>() + qoff[r] * 4;
        ra.target = d_target.as<double>() + qoff[r];
        eval_target_kernel<<<(int)((nq + 255) / 256), 256, 0, t.stream>>>(ra);
        HIPCHK(hipGetLastError());
        dim3 grid((ne + 255) / 256, (unsigned)((nq + kQ - 1) / kQ));
        if (rows_lds) eval_rank_kernel<true><<<grid, 256, rank_lds, t.stream>>>(ra);
        else eval_rank_kernel<false><<<grid, 256, 0, t.stream>>>(ra);
        HIPCHK(hipGetLastError());
    }
    std::vector<unsigned long long> counts(qh.size() * 4);
    HIPCHK(hipMemcpyAsync(counts.data(), d_counts.p, counts.size() * 8, hipMemcpyDeviceToHost, t.stream));
    HIPCHK(hipStreamSynchronize(t.stream));
    long long rawSum = 0, filtSum = 0, rawHits = 0, filtHits = 0;
    for (size_t x = 0; x < qh.size(); ++x) {
        for (int side = 0; side < 2; ++side) {
            const long long raw = 1 + (long long)counts[x * 4 + 2 * side];
            const long long filt = 1 + (long long)counts[x * 4 + 2 * side + 1];
            rawSum += raw;
            filtSum += filt;
            rawHits += raw <= 10;
            filtHits += filt <= 10;
        }
    }
    finish(rawSum, filtSum, rawHits, filtHits, q.ntest, out);
}

void evaluate_transr_compat(const EvalTables& t, const EvalQuery& q, double* work, double out[5],
                            void (*progress)(double, void*), void* ud) {
    if (t.model != 2) throw std::invalid_argument("compat evaluation is TransR's");
    if (q.ntest < 1) throw std::invalid_argument("empty test set");
    const int ne = t.ne, n = t.n;
    // W's n x n image in LDS up to dim 140; above it the chain wave reads W from L2
    // (every dim a context takes; KB2E_EVAL_W_L2=1 forces that form in the tests)
    const char* wl2 = getenv("KB2E_EVAL_W_L2");
    int G = 0;
    bool wglob = false;
    for (int pass = 0; pass < 2 && G == 0; ++pass) {
        wglob = pass == 1 || (wl2 && wl2[0] == '1');
        for (int g : {64, 32, 16, 8, 4})
            if (chain_lds_bytes(n, g, wglob) <= kLdsMax) {
                G = g;
                break;
            }
    }
    if (G == 0 || n > 512) throw std::invalid_argument("TransR compat evaluation supports dim <= 512");
    Grouped g = group_tests(t, q);
    DeviceFilter df;
    build_filter(t, q, df);
    const bool cache_on = ne <= kMaxCacheEntities;  // common/evaluation.cpp:195-198
    DevBuf d_work, d_cache, d_pbuf, d_ftime, d_chain, d_rank, d_counts;
    d_work.alloc((size_t)2 * n * 8);
    std::vector<double> w0(2 * (size_t)n, 0.0);
    if (work) w0.assign(work, work + 2 * (size_t)n);
    HIPCHK(hipMemcpyAsync(d_work.p, w0.data(), w0.size() * 8, hipMemcpyHostToDevice, t.stream));
    // per-pass energies when there is no cache: bounded chunks of passes
    const int64_t rows_cap = cache_on ? 0 : std::max<int64_t>(2, ((int64_t)1 << 30) / ((int64_t)ne * 8));
    if (cache_on) d_cache.alloc((size_t)ne * ne * 8);
    else d_pbuf.alloc((size_t)rows_cap * ne * 8);

    long long rawSum = 0, filtSum = 0, rawHits = 0, filtHits = 0, ties = 0;
    std::vector<CompatPass> chain, rank;
    std::vector<int32_t> ftime;
    int64_t done = 0;
    // one chunk = the passes of one relation (cache: the cache belongs to one
    // relation, common/evaluation.cpp:213-218) or <= rows_cap passes (no cache)
    auto flush = [&]() {
        if (rank.empty()) return;
        if (!ftime.empty()) {
            d_ftime.alloc(ftime.size() * 4);
            HIPCHK(hipMemcpyAsync(d_ftime.p, ftime.data(), ftime.size() * 4, hipMemcpyHostToDevice, t.stream));
        }
        d_chain.alloc(std::max<size_t>(1, chain.size()) * sizeof(CompatPass));
        d_rank.alloc(rank.size() * sizeof(CompatPass));
        if (!chain.empty())
            HIPCHK(hipMemcpyAsync(d_chain.p, chain.data(), chain.size() * sizeof(CompatPass), hipMemcpyHostToDevice,
                                  t.stream));
        HIPCHK(hipMemcpyAsync(d_rank.p, rank.data(), rank.size() * sizeof(CompatPass), hipMemcpyHostToDevice,
                              t.stream));
        if (t.f64) {
            CompatChainArgs<double> a{(const double*)t.ent, (const double*)t.rel, (const double*)t.w, n, t.ld, ne, t.l1, G,
                                wglob, d_chain.as<CompatPass>(), (int32_t)chain.size(), d_ftime.as<int32_t>(),
                                d_work.as<double>(), cache_on ? d_cache.as<double>() : nullptr, d_pbuf.as<double>()};
            run_chain<double>(t, a);
        } else {
            CompatChainArgs<float> a{(const float*)t.ent, (const float*)t.rel, (const float*)t.w, n, t.ld, ne, t.l1, G,
                               wglob, d_chain.as<CompatPass>(), (int32_t)chain.size(), d_ftime.as<int32_t>(),
                               d_work.as<double>(), cache_on ? d_cache.as<double>() : nullptr, d_pbuf.as<double>()};
            run_chain<float>(t, a);
        }
        d_counts.alloc(rank.size() * 3 * 8);
        HIPCHK(hipMemsetAsync(d_counts.p, 0, d_counts.bytes, t.stream));
        CompatRankArgs ra{d_rank.as<CompatPass>(), (int32_t)rank.size(), ne,
                          cache_on ? d_cache.as<double>() : nullptr, d_pbuf.as<double>(), df.view(ne, t.nr),
                          d_counts.as<unsigned long long>()};
        dim3 grid((ne + 255) / 256, (unsigned)rank.size());
        compat_rank_kernel<<<grid, 256, 0, t.stream>>>(ra);
        HIPCHK(hipGetLastError());
        std::vector<unsigned long long> c(rank.size() * 3);
        HIPCHK(hipMemcpyAsync(c.data(), d_counts.p, c.size() * 8, hipMemcpyDeviceToHost, t.stream));
        HIPCHK(hipStreamSynchronize(t.stream));
        for (size_t p = 0; p < rank.size(); ++p) {
            const long long raw = 1 + (long long)c[3 * p], filt = 1 + (long long)c[3 * p + 1];
            rawSum += raw;
            filtSum += filt;
            rawHits += raw <= 10;
            filtHits += filt <= 10;
            ties += (long long)c[3 * p + 2];
        }
        chain.clear();
        rank.clear();
        ftime.clear();
    };
    std::vector<int32_t> fh, ft;
    for (int r = 0; r < t.nr; ++r) {
        const auto& ks = g.byrel[r];
        if (ks.empty()) continue;
        if (cache_on) {
            // first test-triple index (within relation r) with each head / tail: a pair
            // (i, x) is computed by whichever of "tail pass of i's first triple" and
            // "head pass of x's first triple" comes first, and read from the cache after
            fh.assign(ne, INT_MAX);
            ft.assign(ne, INT_MAX);
            for (int32_t k = 0; k < (int32_t)ks.size(); ++k) {
                fh[q.th[ks[k]]] = std::min(fh[q.th[ks[k]]], k);
                ft[q.tt[ks[k]]] = std::min(ft[q.tt[ks[k]]], k);
            }
            ftime.insert(ftime.end(), fh.begin(), fh.end());
            ftime.insert(ftime.end(), ft.begin(), ft.end());
            const int64_t off_h = 0, off_t = ne;
            for (int32_t k = 0; k < (int32_t)ks.size(); ++k) {
                const int32_t h = q.th[ks[k]], tt = q.tt[ks[k]];
                // head pass: (i, tt) computed iff i is not the head of an earlier triple
                CompatPass hp{r, h, tt, 0, off_h, k, 0};
                if (ft[tt] == k) chain.push_back(hp);  // else the whole column is cached
                rank.push_back(hp);
                // tail pass: (h, x) computed iff x was not a tail at or before k
                CompatPass tp{r, h, tt, 1, off_t, k + 1, 0};
                if (fh[h] == k) chain.push_back(tp);
                rank.push_back(tp);
            }
            flush();
        } else {
            for (int64_t k : ks) {
                for (int side = 0; side < 2; ++side) {
                    CompatPass p{r, q.th[k], q.tt[k], side, -1, 0, (int32_t)rank.size()};
                    chain.push_back(p);
                    rank.push_back(p);
                    if ((int64_t)rank.size() >= rows_cap) flush();
                }
            }
        }
        done += (int64_t)ks.size();
        if (progress) progress((double)done / (double)q.ntest, ud);
    }
    flush();
    HIPCHK(hipMemcpyAsync(w0.data(), d_work.p, w0.size() * 8, hipMemcpyDeviceToHost, t.stream));
    HIPCHK(hipStreamSynchronize(t.stream));
    if (work) std::copy(w0.begin(), w0.end(), work);
    finish(rawSum, filtSum, rawHits, filtHits, q.ntest, out);
    out[4] = (double)ties;
}

}  // namespace kb2e
