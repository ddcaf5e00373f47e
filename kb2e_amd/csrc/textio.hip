// textio.hip -- device init and the reference's text table formats on the
// device (textio.hpp).  HBM-bound byte / integer work: one pass counts per
// 4096-item block, a device scan places the blocks, a second pass re-derives
// its items and writes them at their final positions -- no per-item index
// arrays, no atomics on the data path.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <vector>

#include "hip_util.hpp"
#include "kernels_glibc.hpp"
#include "textio.hpp"

namespace kb2e {
namespace {

constexpr int kThreads = 256;
constexpr int kItems = 16;  // items per thread
constexpr int kBlockItems = kThreads * kItems;

using BlockScan = hipcub::BlockScan<int, kThreads>;
using BlockReduce = hipcub::BlockReduce<int, kThreads>;

// Exclusive scan of per-block counts (int64, device) into offsets; returns the
// total (synchronises the stream).
struct Scanner {
    DevBuf tmp, off, total;
    size_t tmp_bytes = 0;
    int64_t run(const int64_t* counts, int64_t nblk, hipStream_t st) {
        size_t need = 0;
        HIPCHK(hipcub::DeviceScan::InclusiveSum(nullptr, need, counts, (int64_t*)nullptr, (int)nblk, st));
        if (need > tmp_bytes) {
            tmp.alloc(need);
            tmp_bytes = need;
        }
        if (off.bytes < (size_t)(nblk + 1) * 8) off.alloc((size_t)(nblk + 1) * 8);
        HIPCHK(hipMemsetAsync(off.p, 0, 8, st));
        HIPCHK(hipcub::DeviceScan::InclusiveSum(tmp.p, need, counts, off.as<int64_t>() + 1, (int)nblk, st));
        int64_t t = 0;
        HIPCHK(hipMemcpyAsync(&t, off.as<int64_t>() + nblk, 8, hipMemcpyDeviceToHost, st));
        HIPCHK(hipStreamSynchronize(st));
        return t;  // off[b] = items before block b
    }
    const int64_t* offsets() const { return off.as<int64_t>(); }
};

// ------------------------------------------------------------ randn (A13)

struct RandnArgs {
    const int32_t* words;  // rand() outputs of the chunk; attempt a uses words 2a, 2a+1
    int64_t attempts;
    double lo, span;       // rand(lo, hi): lo + (hi - lo) * rand() / (RAND_MAX + 1.0)
    double miu, c, den;    // normal(): c = 1 / sqrt(2 PI) / sigma, den = 2 sigma^2
    double peak;           // normal(miu, miu, sigma)
};

// One attempt of common::randn's loop (common/utils.cpp:26-38), in the
// reference's operation order: accept unless dScope > y.
__device__ __forceinline__ bool randn_attempt(const RandnArgs& a, int64_t t, double& x, bool& near) {
    x = a.lo + a.span * (double)a.words[2 * t] / 2147483648.0;
    const double d = x - a.miu;
    const double y = a.c * exp(-1 * (d * d) / a.den);
    const double scope = 0.0 + (a.peak - 0.0) * (double)a.words[2 * t + 1] / 2147483648.0;
    near = fabs(scope - y) <= y * 0x1p-49;
    return !(scope > y);
}

__global__ __launch_bounds__(kThreads) void randn_count_kernel(RandnArgs a, int64_t* blk_count) {
    __shared__ typename BlockReduce::TempStorage tmp;
    const int64_t first = (int64_t)blockIdx.x * kBlockItems + (int64_t)threadIdx.x * kItems;
    int acc = 0;
    for (int k = 0; k < kItems; ++k) {
        const int64_t t = first + k;
        if (t >= a.attempts) break;
        double x;
        bool near;
        acc += randn_attempt(a, t, x, near);
    }
    const int total = BlockReduce(tmp).Sum(acc);
    if (threadIdx.x == 0) blk_count[blockIdx.x] = total;
}

// Values in draw order; the near-ties counted are those of attempts the
// request consumes (every attempt up to the need-th acceptance).
__global__ __launch_bounds__(kThreads) void randn_emit_kernel(RandnArgs a, const int64_t* blk_off, double* out,
                                                              int64_t need, int64_t* last_attempt,
                                                              unsigned long long* near_ties) {
    __shared__ typename BlockScan::TempStorage tmp;
    const int64_t first = (int64_t)blockIdx.x * kBlockItems + (int64_t)threadIdx.x * kItems;
    if (blk_off[blockIdx.x] >= need) return;  // every value of this block is past the request
    bool acc[kItems], near[kItems];
    double xs[kItems];
    int cnt = 0;
    for (int k = 0; k < kItems; ++k) {
        const int64_t t = first + k;
        near[k] = false;
        acc[k] = t < a.attempts && randn_attempt(a, t, xs[k], near[k]);
        cnt += acc[k];
    }
    int pre;
    BlockScan(tmp).ExclusiveSum(cnt, pre);
    int64_t rank = blk_off[blockIdx.x] + pre;
    int nt = 0;
    for (int k = 0; k < kItems; ++k) {
        nt += near[k] && rank < need;
        if (!acc[k]) continue;
        if (rank < need) out[rank] = xs[k];
        if (rank == need - 1) *last_attempt = first + k;
        ++rank;
    }
    if (nt) atomicAdd(near_ties, (unsigned long long)nt);
}

// ------------------------------------------------------------ table rows

template <typename T>
__global__ __launch_bounds__(256) void place_rows_kernel(const double* vals, int64_t rows, int n, int ld, T* dst,
                                                         bool norm, bool ignore_short) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= rows) return;
    const double* a = vals + r * n;
    double len = 1;
    bool scale = false;
    if (norm) {  // common/utils.cpp:45-52, 70-77: sequential sum, sqrt, divide
        double res = 0;
        for (int i = 0; i < n; ++i) res += a[i] * a[i];
        len = sqrt(res);
        scale = !ignore_short || len > 1;
    }
    T* d = dst + r * ld;
    for (int i = 0; i < n; ++i) d[i] = (T)(scale ? a[i] / len : a[i]);
}

template <typename T>
__global__ __launch_bounds__(256) void identity_kernel(T* w, int64_t rows, int n, int ld) {
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= rows * ld) return;
    const int64_t row = k / ld;
    const int i = (int)(k - row * ld);
    const int j = (int)(row % n);
    w[k] = (T)(i < n && i == j ? 1.0 : 0.0);
}

// ------------------------------------------------------------ %.6lf writer

template <typename T>
struct FmtArgs {
    const T* table;
    int64_t row0, elems;  // the chunk: elements [0, elems) from row row0
    int n, ld;
};

template <typename T>
__device__ __forceinline__ int fmt_len(const FmtArgs<T>& a, int64_t k, double& v) {
    const int64_t r = k / a.n;
    const int i = (int)(k - r * a.n);
    v = (double)a.table[(a.row0 + r) * a.ld + i];
    return fmt_fixed6(v, nullptr) + 1 + (i == a.n - 1);  // "\t", and "\n" after a row
}

template <typename T>
__global__ __launch_bounds__(kThreads) void fmt_count_kernel(FmtArgs<T> a, int64_t* blk_bytes) {
    __shared__ typename BlockReduce::TempStorage tmp;
    const int64_t first = (int64_t)blockIdx.x * kBlockItems + (int64_t)threadIdx.x * kItems;
    int acc = 0;
    for (int k = 0; k < kItems && first + k < a.elems; ++k) {
        double v;
        acc += fmt_len(a, first + k, v);
    }
    const int total = BlockReduce(tmp).Sum(acc);
    if (threadIdx.x == 0) blk_bytes[blockIdx.x] = total;
}

template <typename T>
__global__ __launch_bounds__(kThreads) void fmt_write_kernel(FmtArgs<T> a, const int64_t* blk_off, char* out) {
    __shared__ typename BlockScan::TempStorage tmp;
    const int64_t first = (int64_t)blockIdx.x * kBlockItems + (int64_t)threadIdx.x * kItems;
    int acc = 0;
    for (int k = 0; k < kItems && first + k < a.elems; ++k) {
        double v;
        acc += fmt_len(a, first + k, v);
    }
    int pre;
    BlockScan(tmp).ExclusiveSum(acc, pre);
    char* o = out + blk_off[blockIdx.x] + pre;
    for (int k = 0; k < kItems && first + k < a.elems; ++k) {
        const int64_t e = first + k;
        const int i = (int)(e % a.n);
        double v = (double)a.table[(a.row0 + e / a.n) * a.ld + i];
        o += fmt_fixed6(v, o);
        *o++ = '\t';
        if (i == a.n - 1) *o++ = '\n';
    }
}

// ------------------------------------------------------------ %lf reader

__device__ __forceinline__ bool is_ws(char ch) {
    return ch == ' ' || ch == '\t' || ch == '\n' || ch == '\v' || ch == '\f' || ch == '\r';
}

struct ParseArgs {
    const char* text;  // the chunk; it starts after whitespace (or at the file start)
    int64_t len;
    int64_t tok0;      // tokens before the chunk
    int64_t count;     // tokens wanted
    double* out;
    unsigned long long* nslow; // slow-path tokens: index and byte offset appended
    int64_t* slow;             // [cap][2]
    int64_t slow_cap;
};

__device__ __forceinline__ bool tok_start(const ParseArgs& a, int64_t i) {
    return !is_ws(a.text[i]) && (i == 0 || is_ws(a.text[i - 1]));
}

__global__ __launch_bounds__(kThreads) void parse_count_kernel(ParseArgs a, int64_t* blk_count) {
    __shared__ typename BlockReduce::TempStorage tmp;
    const int64_t first = (int64_t)blockIdx.x * kBlockItems + (int64_t)threadIdx.x * kItems;
    int acc = 0;
    for (int k = 0; k < kItems && first + k < a.len; ++k) acc += tok_start(a, first + k);
    const int total = BlockReduce(tmp).Sum(acc);
    if (threadIdx.x == 0) blk_count[blockIdx.x] = total;
}

__global__ __launch_bounds__(kThreads) void parse_emit_kernel(ParseArgs a, const int64_t* blk_off) {
    __shared__ typename BlockScan::TempStorage tmp;
    const int64_t first = (int64_t)blockIdx.x * kBlockItems + (int64_t)threadIdx.x * kItems;
    uint32_t starts = 0;
    int acc = 0;
    for (int k = 0; k < kItems && first + k < a.len; ++k)
        if (tok_start(a, first + k)) {
            starts |= 1u << k;
            ++acc;
        }
    int pre;
    BlockScan(tmp).ExclusiveSum(acc, pre);
    int64_t tok = a.tok0 + blk_off[blockIdx.x] + pre;
    for (int k = 0; k < kItems; ++k) {
        if (!(starts >> k & 1)) continue;
        if (tok < a.count) {
            const int64_t s = first + k;
            int64_t e = s;
            while (e < a.len && !is_ws(a.text[e])) ++e;
            double v = 0;
            const int st = parse_fast(a.text + s, e - s, &v);
            if (st == 0) {
                a.out[tok] = v;
            } else {
                const unsigned long long q = atomicAdd(a.nslow, 1ull);
                if ((int64_t)q < a.slow_cap) {
                    a.slow[2 * q] = tok;
                    a.slow[2 * q + 1] = s;
                }
            }
        }
        ++tok;
    }
}

int64_t blocks_for(int64_t items) { return (items + kBlockItems - 1) / kBlockItems; }

}  // namespace

// ---------------------------------------------------------------- host side

int64_t device_randn(GlibcRand& rng, const uint32_t* jump, int L, double miu, double sigma, double lo, double hi,
                     int64_t count, double* out, hipStream_t st) {
    if (count <= 0) return 0;
    constexpr double kPi = 3.1415926535897932384626433832795;  // common/constants.h:4
    RandnArgs a{};
    a.lo = lo;
    a.span = hi - lo;
    a.miu = miu;
    a.c = 1.0 / std::sqrt(2 * kPi) / sigma;
    a.den = 2 * (sigma * sigma);
    a.peak = a.c * std::exp(-1 * ((miu - miu) * (miu - miu)) / a.den);  // normal(miu, miu, sigma)
    // Chunks of W words (2 per attempt); the expected need is count / acceptance.
    const double accept = std::max(1e-4, 1.0 / (a.span * a.peak));
    const int64_t want = (int64_t)(2.2 * (double)count / accept) + 4 * kBlockItems;
    const int64_t W = std::min<int64_t>((int64_t)1 << 28, (want + 2 * L - 1) / (2 * L) * (2 * L));
    const int64_t nblocks_gen = W / L;
    DevBuf raw, words, starts, counts, tie, last, win;
    raw.alloc((size_t)(W + 31) * 4);
    words.alloc((size_t)W * 4);
    starts.alloc((size_t)nblocks_gen * 31 * 4);
    const int64_t attempts = W / 2;
    const int64_t nblk = blocks_for(attempts);
    counts.alloc((size_t)nblk * 8);
    tie.alloc(8);
    last.alloc(8);
    win.alloc(32 * 4);
    HIPCHK(hipMemsetAsync(tie.p, 0, 8, st));
    Scanner scan;
    GlibcWindow gw;
    rng.window(gw.w);
    int64_t done = 0;
    a.words = words.as<int32_t>();
    a.attempts = attempts;
    while (true) {
        glibc_starts_kernel<<<1, 64, 0, st>>>(gw, jump, L, (int32_t)nblocks_gen, starts.as<uint32_t>(),
                                               raw.as<uint32_t>());
        HIPCHK(hipGetLastError());
        glibc_words_kernel<<<(int)((W + 255) / 256), 256, 0, st>>>(jump, L, starts.as<uint32_t>(), W,
                                                                     raw.as<uint32_t>(), words.as<int32_t>());
        HIPCHK(hipGetLastError());
        randn_count_kernel<<<(int)nblk, kThreads, 0, st>>>(a, counts.as<int64_t>());
        HIPCHK(hipGetLastError());
        const int64_t got = scan.run(counts.as<int64_t>(), nblk, st);
        const int64_t need = count - done;
        randn_emit_kernel<<<(int)nblk, kThreads, 0, st>>>(a, scan.offsets(), out + done, need,
                                                            last.as<int64_t>(), tie.as<unsigned long long>());
        HIPCHK(hipGetLastError());
        int64_t used = W;  // words of this chunk consumed
        if (got >= need) {
            int64_t t = 0;
            HIPCHK(hipMemcpyAsync(&t, last.p, 8, hipMemcpyDeviceToHost, st));
            HIPCHK(hipStreamSynchronize(st));
            used = 2 * t + 2;
        }
        // the generator window after `used` words of the chunk: raw[used .. used + 31)
        HIPCHK(hipMemcpyAsync(gw.w, raw.as<uint32_t>() + used, 31 * 4, hipMemcpyDeviceToHost, st));
        HIPCHK(hipStreamSynchronize(st));
        if (got >= need) break;
        done += got;
    }
    rng.set_window(gw.w);
    unsigned long long ties = 0;
    HIPCHK(hipMemcpy(&ties, tie.p, 8, hipMemcpyDeviceToHost));
    return (int64_t)ties;
}

void place_rows(const double* vals, int64_t rows, int n, int ld, void* dst, bool f64, bool norm, bool ignore_short,
                hipStream_t st) {
    if (rows <= 0) return;
    const int grid = (int)((rows + 255) / 256);
    if (f64) place_rows_kernel<double><<<grid, 256, 0, st>>>(vals, rows, n, ld, (double*)dst, norm, ignore_short);
    else place_rows_kernel<float><<<grid, 256, 0, st>>>(vals, rows, n, ld, (float*)dst, norm, ignore_short);
    HIPCHK(hipGetLastError());
}

void identity_weights(void* w, int64_t nr, int n, int ld, bool f64, hipStream_t st) {
    const int64_t rows = nr * n;
    const int64_t grid = (rows * ld + 255) / 256;
    if (f64) identity_kernel<double><<<(int)grid, 256, 0, st>>>((double*)w, rows, n, ld);
    else identity_kernel<float><<<(int)grid, 256, 0, st>>>((float*)w, rows, n, ld);
    HIPCHK(hipGetLastError());
}

int64_t format_table(const void* table, bool f64, int64_t rows, int n, int ld, hipStream_t st,
                     const std::function<void(const char*, size_t)>& sink) {
    if (rows <= 0 || n <= 0) return 0;
    const int64_t rows_per_chunk = std::max<int64_t>(1, ((int64_t)1 << 24) / n);
    DevBuf counts, dev_out;
    counts.alloc((size_t)blocks_for(rows_per_chunk * n) * 8);
    Scanner scan;
    std::vector<char> host;
    int64_t total = 0;
    for (int64_t r0 = 0; r0 < rows; r0 += rows_per_chunk) {
        const int64_t nr = std::min(rows_per_chunk, rows - r0);
        const int64_t elems = nr * n;
        const int64_t nblk = blocks_for(elems);
        int64_t bytes = 0;
        auto run = [&](auto tag) {
            using T = decltype(tag);
            FmtArgs<T> a{(const T*)table, r0, elems, n, ld};
            fmt_count_kernel<T><<<(int)nblk, kThreads, 0, st>>>(a, counts.as<int64_t>());
            HIPCHK(hipGetLastError());
            bytes = scan.run(counts.as<int64_t>(), nblk, st);
            if (dev_out.bytes < (size_t)bytes) dev_out.alloc((size_t)bytes);
            fmt_write_kernel<T><<<(int)nblk, kThreads, 0, st>>>(a, scan.offsets(), dev_out.as<char>());
            HIPCHK(hipGetLastError());
        };
        if (f64) run(double());
        else run(float());
        host.resize((size_t)bytes);
        HIPCHK(hipMemcpyAsync(host.data(), dev_out.p, (size_t)bytes, hipMemcpyDeviceToHost, st));
        HIPCHK(hipStreamSynchronize(st));
        sink(host.data(), (size_t)bytes);
        total += bytes;
    }
    return total;
}

int64_t parse_doubles(const char* text, int64_t len, int64_t count, double* out, hipStream_t st, int64_t* bad,
                      int64_t* slow_out) {
    *bad = -1;
    *slow_out = 0;
    if (count <= 0) return 0;
    auto ws = [](char ch) {
        return ch == ' ' || ch == '\t' || ch == '\n' || ch == '\v' || ch == '\f' || ch == '\r';
    };
    const int64_t kChunk = (int64_t)1 << 30;
    const int64_t slow_cap = 1 << 16;
    DevBuf dtext, counts, flags, slow;
    dtext.alloc((size_t)std::min(len, kChunk) + 1);
    counts.alloc((size_t)blocks_for(std::min(len, kChunk)) * 8);
    flags.alloc(16);
    slow.alloc((size_t)slow_cap * 16);
    HIPCHK(hipMemsetAsync(flags.p, 0, 16, st));
    Scanner scan;
    int64_t tokens = 0;
    std::vector<int64_t> slow_host;
    for (int64_t pos = 0; pos < len && tokens < count;) {
        int64_t end = std::min(len, pos + kChunk);
        if (end < len) {  // split after whitespace so no token crosses chunks
            while (end > pos && !ws(text[end - 1])) --end;
            if (end == pos) throw std::invalid_argument("token longer than 1 GiB");
        }
        const int64_t clen = end - pos;
        HIPCHK(hipMemcpyAsync(dtext.p, text + pos, (size_t)clen, hipMemcpyHostToDevice, st));
        ParseArgs a{};
        a.text = dtext.as<char>();
        a.len = clen;
        a.tok0 = tokens;
        a.count = count;
        a.out = out;
        a.nslow = flags.as<unsigned long long>();
        a.slow = slow.as<int64_t>();
        a.slow_cap = slow_cap;
        const int64_t nblk = blocks_for(clen);
        parse_count_kernel<<<(int)nblk, kThreads, 0, st>>>(a, counts.as<int64_t>());
        HIPCHK(hipGetLastError());
        const int64_t ntok = scan.run(counts.as<int64_t>(), nblk, st);
        parse_emit_kernel<<<(int)nblk, kThreads, 0, st>>>(a, scan.offsets());
        HIPCHK(hipGetLastError());
        unsigned long long nslow = 0;
        HIPCHK(hipMemcpyAsync(&nslow, flags.p, 8, hipMemcpyDeviceToHost, st));
        HIPCHK(hipStreamSynchronize(st));
        if (nslow > (unsigned long long)slow_cap) throw std::invalid_argument("too many tokens outside the exact parser");
        if (nslow) {  // rare: tokens strtod converts (never produced by "%.6lf")
            std::vector<int64_t> sl(2 * nslow);
            HIPCHK(hipMemcpy(sl.data(), slow.p, sl.size() * 8, hipMemcpyDeviceToHost));
            for (size_t q = 0; q < nslow; ++q) {
                const int64_t s = pos + sl[2 * q + 1];
                int64_t e = s;
                while (e < len && !ws(text[e])) ++e;
                const std::string tok(text + s, text + e);
                char* stop = nullptr;
                const double v = std::strtod(tok.c_str(), &stop);
                if (stop != tok.c_str() + tok.size()) {  // fscanf("%lf") would fail here
                    *bad = *bad < 0 ? sl[2 * q] : std::min(*bad, sl[2 * q]);
                    continue;
                }
                HIPCHK(hipMemcpy(out + sl[2 * q], &v, 8, hipMemcpyHostToDevice));
            }
            *slow_out += (int64_t)nslow;
            memset_sync(flags.p, 0, 8);
        }
        tokens += ntok;
        pos = end;
    }
    int64_t parsed = std::min(tokens, count);
    if (*bad >= 0 && *bad < parsed) parsed = *bad;
    return parsed;
}

}  // namespace kb2e
