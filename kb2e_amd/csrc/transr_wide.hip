// transr_wide.hip -- host side of the PARALLEL TransR kernels at 128 < n <= 512
// (kernels_transr_widep.hpp), in their own translation unit: CP = ceil(n / 128)
// element pairs a lane, FP64 and FP32 tables.
#include <algorithm>
#include <stdexcept>

#include "hip_util.hpp"
#include "kernels_transr_widep.hpp"
#include "transr_cons.hpp"

namespace kb2e {

namespace {

// the compat scan's chunk sums with `chunk` calls a chunk (rpar_scan_sums_kernel's form)
__global__ __launch_bounds__(256) void wide_scan_sums_kernel(const double* proj, int64_t calls, int32_t ld, int32_t n,
                                                             int32_t chunk, double* sums) {
    const int c = blockIdx.x;
    const int64_t c0 = (int64_t)c * chunk, c1 = min<int64_t>(calls, c0 + chunk);
    for (int e = threadIdx.x; e < 2 * n; e += blockDim.x) {
        const int side = e / n, i = e % n;
        double s = 0.0;
        for (int64_t k = c0; k < c1; ++k) s += proj[(k * 2 + side) * ld + i];
        sums[(int64_t)c * 2 * n + e] = s;
    }
}

template <typename T, int CP>
struct WideK {
    static const void* tile(bool p, bool g) {
        return p && g ? (const void*)wide_tile_kernel<T, true, true, CP>
               : p    ? (const void*)wide_tile_kernel<T, true, false, CP>
                      : (const void*)wide_tile_kernel<T, false, true, CP>;
    }
};

template <typename T, typename F>
void by_cp(int n, F&& f) {
    switch ((n + 127) / 128) {
        case 2: f(std::integral_constant<int, 2>()); return;
        case 3: f(std::integral_constant<int, 3>()); return;
        case 4: f(std::integral_constant<int, 4>()); return;
    }
    throw std::runtime_error("wide PARALLEL TransR kernels: 128 < n <= 512");
}

}  // namespace

bool wide_par_supported(int n) { return n > 128 && n <= kWideParMaxN; }

WideGeom wide_setup(int n, int ld, int esize) {
    WideGeom g{};
    constexpr size_t kBudget = 150 * 1024;
    g.St = 1;
    for (int St = 8; St >= 1; St >>= 1) {
        const size_t b = esize == 8 ? wide_tile_lds<double>(ld, St) : wide_tile_lds<float>(ld, St);
        if (b <= kBudget) {
            g.St = St;
            break;
        }
    }
    g.tile_lds = esize == 8 ? wide_tile_lds<double>(ld, g.St) : wide_tile_lds<float>(ld, g.St);
    // compat scan: the chunk's running vectors [chunk][2 n] doubles within 96 KiB (even)
    g.chunk = std::max(2, std::min(64, (int)((96 * 1024) / (2 * (size_t)n * 8)) & ~1));
    g.scan_lds = (size_t)g.chunk * 2 * n * 8;
    g.chain_lds = wide_chain_lds(ld);
    auto allow = [](const void* k, size_t b) {
        HIPCHK(hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)b));
    };
    auto each = [&](auto tag) {
        using T = decltype(tag);
        by_cp<T>(n, [&](auto cpc) {
            constexpr int CP = decltype(cpc)::value;
            for (int v = 0; v < 3; ++v) allow(WideK<T, CP>::tile(v != 2, v != 1), g.tile_lds);
            allow((const void*)wide_scan_energy_kernel<T, CP>, g.scan_lds);
            allow((const void*)wide_chain_kernel<T, CP>, g.chain_lds);
        });
    };
    if (esize == 8) each(double());
    else each(float());
    return g;
}

template <typename T>
void wide_phase_a(const RParArgs& a, const RParBufs<T>& bf, const WideGeom& g, int tgrid, double* scan,
                  double* scan_pre, const double* work_in, double* work_out, hipStream_t st) {
    RParArgs aa = a;
    RParBufs<T> bb = bf;
    void* args[] = {&aa, &bb};
    by_cp<T>(a.n, [&](auto cpc) {
        constexpr int CP = decltype(cpc)::value;
        if (!a.compat) {
            HIPCHK(hipLaunchKernel(WideK<T, CP>::tile(true, true), dim3(tgrid), dim3(256), args, g.tile_lds, st));
            transr_pair_first_kernel<<<(int)((4 * a.B + 255) / 256), 256, 0, st>>>(a);
            HIPCHK(hipGetLastError());
            return;
        }
        HIPCHK(hipLaunchKernel(WideK<T, CP>::tile(true, false), dim3(tgrid), dim3(256), args, g.tile_lds, st));
        const int64_t calls = 2 * (int64_t)a.B;
        const int nchunks = (int)((calls + g.chunk - 1) / g.chunk);
        wide_scan_sums_kernel<<<nchunks, 256, 0, st>>>(a.proj, calls, a.ld, a.n, g.chunk, scan);
        const double* pre = nullptr;
        // (the chunks' prefix once; a few: every block sums its own; KB2E_RPAR_SCAN_PREFIX=1 / 0
        // forces one form, tests)
        const char* sp = getenv("KB2E_RPAR_SCAN_PREFIX");
        if (sp ? sp[0] == '1' : nchunks > 8) {
            rpar_scan_prefix_kernel<<<(2 * a.n + 31) / 32, 1024, 0, st>>>(scan, nchunks, 2 * a.n, work_in, scan_pre);
            pre = scan_pre;
        }
        wide_scan_energy_kernel<T, CP><<<nchunks, 1024, g.scan_lds, st>>>(a, bf, scan, nchunks, g.chunk, work_in,
                                                                          work_out, pre);
        HIPCHK(hipGetLastError());
        HIPCHK(hipLaunchKernel(WideK<T, CP>::tile(false, true), dim3(tgrid), dim3(256), args, g.tile_lds, st));
    });
}

template <typename T>
void wide_phase_b(const RParArgs& a, const RParBufs<T>& bf, const WideGeom& g, double* wsc, bool constraint,
                  int rel_segs_max, hipStream_t st) {
    by_cp<T>(a.n, [&](auto cpc) {
        constexpr int CP = decltype(cpc)::value;
        const int rw = rel_segs_max * (a.n + 1);             // a wave per (relation segment, row)
        wide_rel_rows_kernel<T, CP><<<(rw + 3) / 4, 256, 0, st>>>(a, bf);
        const int ew = 5 * a.B;                               // entity segments of the batch, at most
        wide_entity_kernel<T, true, CP><<<(ew + 3) / 4, 256, 0, st>>>(a, bf);
        HIPCHK(hipGetLastError());
        if (!constraint) return;
        wide_chain_kernel<T, CP><<<std::max(1, a.nrel), kWideThreads, g.chain_lds, st>>>(a, bf, wsc);
        wide_entity_kernel<T, false, CP><<<(ew + 3) / 4, 256, 0, st>>>(a, bf);
        HIPCHK(hipGetLastError());
    });
}

template void wide_phase_a<double>(const RParArgs&, const RParBufs<double>&, const WideGeom&, int, double*, double*,
                                   const double*, double*, hipStream_t);
template void wide_phase_a<float>(const RParArgs&, const RParBufs<float>&, const WideGeom&, int, double*, double*,
                                  const double*, double*, hipStream_t);
template void wide_phase_b<double>(const RParArgs&, const RParBufs<double>&, const WideGeom&, double*, bool, int,
                                   hipStream_t);
template void wide_phase_b<float>(const RParArgs&, const RParBufs<float>&, const WideGeom&, double*, bool, int,
                                  hipStream_t);

}  // namespace kb2e
