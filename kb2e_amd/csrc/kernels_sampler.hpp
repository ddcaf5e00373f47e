// kernels_sampler.hpp -- the reference's sample stream, drawn on the device.
//
// The reference draws each sample from the glibc rand() stream in sequence
// (common/trainer.cpp:79-98): i = randMax(|train|) (2 words), j = randMax(|E|)
// (2 words), rand() % 1000 against the Bernoulli threshold (1 word), then 2
// more words per rejected j while the corrupted triple is a training triple.
// A sample starting at word p therefore occupies len(p) = 5 + 2 * rejections
// words, and the epoch's samples start at 0, next(0), next(next(0)), ... with
// next(p) = p + len(p).  Whether a sample is rejected depends only on the words
// and the filter, never on embeddings, so:
//   1. sample_len: every word position p computes the sample that would start
//      there (filter probes included) -> next[p], j[p], side[p]   (parallel);
//   2. pointer doubling: level k holds next^(2^k)                  (log S passes);
//   3. sample_chain: sample s starts at next^s(0), composed from the levels;
//   4. sample_emit: (i, j, side) of every sample + the words consumed.
// The host supplies the raw words (glibc TYPE_3 outputs) of the epoch and
// advances its own generator by exactly the number consumed.
#pragma once

#include "kernels_common.hpp"
#include "kernels_glibc.hpp"

namespace kb2e {

struct SamplerArgs {
    const int32_t* words;   // rand() outputs, [nraw]
    int64_t nraw;
    const int32_t* heads;
    const int32_t* tails;
    const int32_t* rels;
    int32_t ntrain, ne;
    const double* pr;       // per relation: 1000*tailMean/(tailMean+headMean), or 500 (unif)
    const uint64_t* slots;  // filter hash table
    uint64_t mask;
    uint64_t nr64, ne64;
    int32_t* next;          // [nraw + 1]
    int32_t* jfin;          // [nraw]
    uint8_t* sidefin;       // [nraw]
};

__device__ __forceinline__ uint64_t dev_mix64(uint64_t x) {
    x ^= x >> 31;
    x *= 0x7fb5d329728ea185ull;
    x ^= x >> 27;
    x *= 0x81dadef4bc2dd44dull;
    x ^= x >> 33;
    return x;
}

__device__ __forceinline__ bool filter_has(const SamplerArgs& a, int64_t h, int64_t r, int64_t t) {
    const uint64_t k = ((uint64_t)h * a.nr64 + (uint64_t)r) * a.ne64 + (uint64_t)t;
    uint64_t p = dev_mix64(k) & a.mask;
    while (true) {
        const uint64_t s = a.slots[p];
        if (s == k) return true;
        if (s == ~0ull) return false;
        p = (p + 1) & a.mask;
    }
}

// common/utils.cpp:113-120 on two consumed words.
__device__ __forceinline__ int32_t dev_rand_max(int32_t a, int32_t b, int32_t x) {
    int32_t res = (int32_t)((uint32_t)a * (uint32_t)b) % x;
    while (res < 0) res += x;
    return res;
}

__global__ __launch_bounds__(256) void sample_len_kernel(SamplerArgs a) {
    const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p > a.nraw) return;
    if (p == a.nraw) {
        a.next[p] = (int32_t)a.nraw;  // sink
        return;
    }
    if (p + 5 > a.nraw) {  // not enough words left for a sample: invalid
        a.next[p] = (int32_t)a.nraw;
        a.jfin[p] = 0;
        a.sidefin[p] = 2;
        return;
    }
    const int32_t* w = a.words;
    const int32_t i = dev_rand_max(w[p], w[p + 1], a.ntrain);
    int32_t j = dev_rand_max(w[p + 2], w[p + 3], a.ne);
    const int32_t r = a.rels[i];
    const bool tail = (double)(w[p + 4] % 1000) < a.pr[r];
    int64_t q = p + 5;
    const int32_t h = a.heads[i], t = a.tails[i];
    uint8_t valid = 1;
    while (tail ? filter_has(a, h, r, j) : filter_has(a, j, r, t)) {
        if (q + 2 > a.nraw) {  // words ran out inside the rejection loop
            q = a.nraw;
            valid = 0;
            break;
        }
        j = dev_rand_max(w[q], w[q + 1], a.ne);
        q += 2;
    }
    a.next[p] = (int32_t)q;
    a.jfin[p] = j;
    a.sidefin[p] = valid ? (tail ? 1 : 0) : 2;
}

// dst[p] = src[src[p]]  (next^(2^k) from next^(2^(k-1)))
__global__ __launch_bounds__(256) void sample_double_kernel(const int32_t* src, int32_t* dst, int64_t n1) {
    const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n1) return;
    dst[p] = src[src[p]];
}

struct ChainArgs {
    const int32_t* levels;  // [K][nraw + 1]
    int32_t K;
    int64_t stride;         // nraw + 1
    int64_t nsamples;
    int64_t nraw;
    const int32_t* words;
    const int32_t* jfin;
    const uint8_t* sidefin;
    const int32_t* next;
    int32_t ntrain;
    int32_t* si;
    int32_t* sj;
    uint8_t* side;
    int64_t* consumed;      // words used by the epoch, or -1 if the buffer ran out
};

__global__ __launch_bounds__(256) void sample_chain_kernel(ChainArgs a) {
    const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= a.nsamples) return;
    int64_t p = 0;
    for (int k = 0; k < a.K && p < a.nraw; ++k)
        if ((s >> k) & 1) p = a.levels[(int64_t)k * a.stride + p];
    const bool ok = p < a.nraw && a.sidefin[p] != 2;
    a.si[s] = ok ? dev_rand_max(a.words[p], a.words[p + 1], a.ntrain) : 0;
    a.sj[s] = ok ? a.jfin[p] : 0;
    a.side[s] = ok ? a.sidefin[p] : 0;
    // Chain positions increase, so the last sample is valid iff all are.
    if (s == a.nsamples - 1) *a.consumed = ok ? (int64_t)a.next[p] : -1;
}

}  // namespace kb2e
