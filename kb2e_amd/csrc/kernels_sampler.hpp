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
//   2. the chain by chunks (chain_*): the stream is cut into chunks of kChainW
//      words; a sample chain enters a chunk at an offset below the previous
//      sample's length, so each chunk tabulates, per entry offset < kChainEmax,
//      where the chain leaves it and how many samples it starts there; the
//      tables compose (superchunks of kChainG chunks, then one walk over the
//      superchunks) into every chunk's true entry and first sample index, and
//      each chunk emits its samples.  A sample longer than kChainEmax words at a
//      chunk edge flags overflow (consumed = -2) and the host redraws the epoch
//      with the general form:
//   2'. pointer doubling: level k holds next^(2^k) (log S passes), sample s
//      starts at next^s(0), composed from the levels (sample_chain).
// The device makes the raw words (glibc TYPE_3 outputs) of the epoch from the
// generator's window; the host advances its generator by exactly the number
// consumed.
#pragma once

#include "kernels_common.hpp"
#include "kernels_glibc.hpp"

namespace kb2e {

struct SamplerArgs {
    const int32_t* words;   // rand() outputs, [nraw]
    int64_t nraw;
    const int4* trip;       // per training triple: head, tail, relation, Bernoulli threshold
                            // (#k in [0,1000) with k < pr[r], pr = 1000*tailMean/(tailMean+headMean) or 500)
    const uint64_t* trip8;  // the same packed in 8 bytes when it fits (null: trip): head | tail << eb |
    int32_t eb, rb;         //   relation << 2 eb | threshold << (2 eb + rb); eb / rb bits of an entity / relation id
    int32_t ntrain, ne;
    const uint64_t* slots;  // filter hash table
    uint64_t mask;
    const uint64_t* bloom;  // FilterSet::bloom (host_data.hpp): two bits a key in one word
    uint64_t bloom_mask;
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
    const uint64_t b = dev_mix64(k ^ 0x9e3779b97f4a7c15ull);  // FilterSet::kBloomSalt
    const uint64_t bits = (1ull << ((b >> 52) & 63)) | (1ull << (b >> 58));
    if ((a.bloom[b & a.bloom_mask] & bits) != bits) return false;
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

__device__ __forceinline__ void sample_len_at(const SamplerArgs& a, int64_t p);

// Grid-stride: the launch may use fewer workgroups than positions, so that
// beside the batches (side stream) it holds a bounded share of the machine.
__global__ __launch_bounds__(256) void sample_len_kernel(SamplerArgs a) {
    for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p <= a.nraw;
         p += (int64_t)gridDim.x * blockDim.x)
        sample_len_at(a, p);
}

__device__ __forceinline__ void sample_len_at(const SamplerArgs& a, int64_t p) {
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
    int32_t h, t, r, thr;  // one random read for the triple and its threshold
    if (a.trip8) {  // (8 bytes: half the table, most of it in L2)
        const uint64_t v = a.trip8[i];
        const uint64_t em = (1ull << a.eb) - 1ull, rm = (1ull << a.rb) - 1ull;
        h = (int32_t)(v & em);
        t = (int32_t)((v >> a.eb) & em);
        r = (int32_t)((v >> (2 * a.eb)) & rm);
        thr = (int32_t)(v >> (2 * a.eb + a.rb));
    } else {
        const int4 tr = a.trip[i];
        h = tr.x;
        t = tr.y;
        r = tr.z;
        thr = tr.w;
    }
    const bool tail = w[p + 4] % 1000 < thr;  // == (double)(rand() % 1000) < pr[r]
    int64_t q = p + 5;
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

// ---------------------------------------------------------------- the chain by chunks
constexpr int kChainW = 1024;           // words per chunk
constexpr int kChainEmax = 64;          // entry offsets tabulated per chunk
constexpr int kChainG = 64;             // chunks per superchunk
constexpr int kChainMaxSamples = kChainW / 5 + 2;  // samples are >= 5 words long
constexpr uint32_t kChainTerm = 255;    // the chain has ended (reached nraw)

struct ChunkArgs {
    const int32_t* next;    // sample_len's next[], [nraw + 1]
    int64_t nraw;
    int32_t nchunks, nsuper;
    int32_t emax;           // entry offsets allowed (<= kChainEmax; lower only to test the overflow path)
    uint32_t* table;        // [nchunks][64]: exit offset | samples << 8
    uint2* super;           // [nsuper][64]: (exit offset, samples)
    uint2* sc_state;        // [nsuper]: (entry offset, first sample)
    uint2* ch_state;        // [nchunks]
    int32_t* overflow;      // cleared by glibc_starts_pow_kernel
    // emission, as sample_chain
    int64_t nsamples;
    const int32_t* words;
    const int32_t* jfin;
    const uint8_t* sidefin;
    int32_t ntrain;
    int32_t* si;
    int32_t* sj;
    uint8_t* side;
    int64_t* consumed;
};

// Per chunk and entry offset e (one lane each): walk next[] in LDS from the
// chunk's word e to the first chain position past the chunk.
__global__ __launch_bounds__(64) void chain_table_kernel(ChunkArgs a) {
    __shared__ int32_t nx[kChainW];
    const int c = blockIdx.x, l = threadIdx.x;
    const int64_t base = (int64_t)c * kChainW;
    const int64_t end = min(base + kChainW, a.nraw);
    for (int q = l; q < kChainW; q += 64) {
        const int64_t p = base + q;
        nx[q] = p < a.nraw ? a.next[p] : (int32_t)a.nraw;
    }
    __syncthreads();
    int64_t p = base + l;
    uint32_t cnt = 0;
    while (p < end) {  // next[p] > p: the walk ends
        ++cnt;
        p = nx[p - base];
    }
    uint32_t ex = kChainTerm;
    if (p < a.nraw) {
        const int64_t e = p - (base + kChainW);
        if (e < a.emax) ex = (uint32_t)e;
        else a.overflow[0] = 1;
    }
    a.table[(size_t)c * 64 + l] = ex | cnt << 8;
}

// Per superchunk: the composed table of its kChainG chunks, every entry offset a lane.
__global__ __launch_bounds__(64) void chain_super_kernel(ChunkArgs a) {
    __shared__ uint32_t T[kChainG][64];
    const int sc = blockIdx.x, l = threadIdx.x;
    const int c0 = sc * kChainG, ng = min(kChainG, a.nchunks - c0);
    for (int g = 0; g < ng; ++g) T[g][l] = a.table[(size_t)(c0 + g) * 64 + l];
    __syncthreads();
    uint32_t cur = l, tot = 0;
    for (int g = 0; g < ng && cur != kChainTerm; ++g) {
        const uint32_t v = T[g][cur];
        tot += v >> 8;
        cur = v & 255;
    }
    a.super[(size_t)sc * 64 + l] = make_uint2(cur, tot);
}

// One workgroup: the chain through the superchunks from word 0 (tiles of 64
// superchunk tables in LDS, one lane walking); the error words of consumed.
__global__ __launch_bounds__(64) void chain_top_kernel(ChunkArgs a) {
    __shared__ uint2 T[64][64];
    __shared__ uint32_t s_cur, s_base;
    const int l = threadIdx.x;
    if (l == 0) {
        s_cur = 0;
        s_base = 0;
    }
    for (int t0 = 0; t0 < a.nsuper; t0 += 64) {
        const int nt = min(64, a.nsuper - t0);
        __syncthreads();
        for (int g = 0; g < nt; ++g) T[g][l] = a.super[(size_t)(t0 + g) * 64 + l];
        __syncthreads();
        if (l == 0) {
            uint32_t cur = s_cur, base = s_base;
            for (int g = 0; g < nt; ++g) {
                a.sc_state[t0 + g] = make_uint2(cur, base);
                if (cur != kChainTerm) {
                    const uint2 v = T[g][cur];
                    base += v.y;
                    cur = v.x;
                }
            }
            s_cur = cur;
            s_base = base;
        }
    }
    __syncthreads();
    if (l == 0) {
        if (a.overflow[0]) *a.consumed = -2;                       // redraw with pointer doubling
        else if ((int64_t)s_base < a.nsamples) *a.consumed = -1;  // the word buffer ran out
    }
}

// Per superchunk: each chunk's entry offset and first sample, from the superchunk's.
__global__ __launch_bounds__(64) void chain_entries_kernel(ChunkArgs a) {
    __shared__ uint32_t T[kChainG][64];
    const int sc = blockIdx.x, l = threadIdx.x;
    const int c0 = sc * kChainG, ng = min(kChainG, a.nchunks - c0);
    for (int g = 0; g < ng; ++g) T[g][l] = a.table[(size_t)(c0 + g) * 64 + l];
    __syncthreads();
    if (l == 0) {
        const uint2 st = a.sc_state[sc];
        uint32_t cur = st.x, base = st.y;
        for (int g = 0; g < ng; ++g) {
            a.ch_state[c0 + g] = make_uint2(cur, base);
            if (cur != kChainTerm) {
                const uint32_t v = T[g][cur];
                base += v >> 8;
                cur = v & 255;
            }
        }
    }
}

// Per chunk: the chain's positions in it (one lane walks LDS), then every
// sample written by its own lane (as sample_chain_kernel).
__global__ __launch_bounds__(256) void chain_emit_kernel(ChunkArgs a) {
    __shared__ int32_t nx[kChainW];
    __shared__ int32_t pos[kChainMaxSamples];
    __shared__ int32_t s_cnt;
    const int c = blockIdx.x, l = threadIdx.x;
    const uint2 st = a.ch_state[c];
    if (a.overflow[0] || st.x == kChainTerm || (int64_t)st.y >= a.nsamples) return;
    const int64_t base = (int64_t)c * kChainW;
    const int64_t end = min(base + kChainW, a.nraw);
    for (int q = l; q < kChainW; q += 256) {
        const int64_t p = base + q;
        nx[q] = p < a.nraw ? a.next[p] : (int32_t)a.nraw;
    }
    __syncthreads();
    if (l == 0) {
        int64_t p = base + st.x;
        int k = 0;
        while (p < end) {
            pos[k++] = (int32_t)p;
            p = nx[p - base];
        }
        s_cnt = k;
    }
    __syncthreads();
    const int cnt = s_cnt;
    for (int k = l; k < cnt; k += 256) {
        const int64_t s = (int64_t)st.y + k;
        if (s >= a.nsamples) break;
        const int32_t p = pos[k];
        const bool ok = a.sidefin[p] != 2;
        a.si[s] = ok ? dev_rand_max(a.words[p], a.words[p + 1], a.ntrain) : 0;
        a.sj[s] = ok ? a.jfin[p] : 0;
        a.side[s] = ok ? a.sidefin[p] : 0;
        if (s == a.nsamples - 1) *a.consumed = ok ? (int64_t)a.next[p] : -1;
    }
}

}  // namespace kb2e
