// transr_cons.hip -- the register-resident transRNorm kernel of the PARALLEL
// TransR schedule (kernels_transr_cons.hpp), instantiated for every live
// k-step count 1..16 (n <= 64) in FP64 and FP32.
#include "transr_cons.hpp"

#include <algorithm>
#include <cstring>
#include <stdexcept>
#include <string>
#include <utility>

#include "hip_util.hpp"
#include "kernels_transr_cons.hpp"
#include "kernels_transr_seq.hpp"
#include "kernels_transr_chainw.hpp"
#include "kernels_transr_chainwp.hpp"
#include "kernels_transr_chaing.hpp"
#include "kernels_transr_pipe.hpp"
#include "kernels_transr_wave.hpp"

namespace kb2e {

namespace {

enum Kind { kCons, kGrad, kProj };

// the chain kernels' grid: a workgroup per relation of the batch (a.brel)
int chain_grid(const RParArgs& a) { return a.nrel > 0 ? a.nrel : 1; }

template <typename T, int KS>
const void* fn_at(Kind k) {
    return k == kCons ? (const void*)transr_cons_wave_kernel<T, KS>
           : k == kGrad ? (const void*)transr_grad_wave_kernel<T, KS>
                        : (const void*)transr_proj_wave_kernel<T, KS>;
}

template <typename T, int... KS>
const void* fn_table(Kind k, int ks, std::integer_sequence<int, KS...>) {
    const void* tab[] = {fn_at<T, KS + 1>(k)...};
    return tab[ks - 1];
}

template <typename T>
const void* kernel_fn(Kind k, int n) {
    if (!cons_wave_supported(n)) throw std::runtime_error("TransR wave kernels: n > 64");
    return fn_table<T>(k, cons_live_steps<T>(n), std::make_integer_sequence<int, 16>{});
}

template <typename T>
const void* cons_fn(int n) {
    return kernel_fn<T>(kCons, n);
}

template <int... KS>
const void* pipe_table(int ks, std::integer_sequence<int, KS...>) {
    const void* tab[] = {(const void*)transr_cons_pipe_kernel<double, KS + 1>...};
    return tab[ks - 1];
}

const void* pipe_fn(int n) {
    if (!cons_wave_supported(n)) throw std::runtime_error("transRNorm pipelined chain kernel: n > 64");
    return pipe_table((n + 3) / 4, std::make_integer_sequence<int, 16>{});
}

const void* chainw_fn(int n) {
    switch (wide_nb(n)) {
        case 1: return (const void*)transr_cons_chain_wide_kernel<1>;
        case 2: return (const void*)transr_cons_chain_wide_kernel<2>;
        case 3: return (const void*)transr_cons_chain_wide_kernel<3>;
        case 4: return (const void*)transr_cons_chain_wide_kernel<4>;
        case 5: return (const void*)transr_cons_chain_wide_kernel<5>;
        case 6: return (const void*)transr_cons_chain_wide_kernel<6>;
        case 7: return (const void*)transr_cons_chain_wide_kernel<7>;
    }
    throw std::runtime_error("transRNorm wide chain kernel: n > 112");
}

const void* chainwp_fn(int n) {
    switch (wp_ks(n)) {
        case 18: return (const void*)transr_cons_chain_wpipe_kernel<18>;
        case 20: return (const void*)transr_cons_chain_wpipe_kernel<20>;
        case 22: return (const void*)transr_cons_chain_wpipe_kernel<22>;
        case 24: return (const void*)transr_cons_chain_wpipe_kernel<24>;
        case 25: return (const void*)transr_cons_chain_wpipe_kernel<25>;
    }
    throw std::runtime_error("transRNorm pipelined wide chain kernel: no instantiation");
}

// 64 < n <= 100: the pipelined wide chain (kernels_transr_chainwp.hpp);
// KB2E_RPAR_CHAIN=lockstep runs the eight-wave lockstep kernel there too (A/B)
bool use_wpipe(int n) {
    const char* e = getenv("KB2E_RPAR_CHAIN");
    return n > 64 && n <= kWPMaxN && !(e && std::string(e) == "lockstep");
}

}  // namespace

size_t cons_seq_setup(int n) {
    const size_t lds = pipe_lds<double>(n);
    HIPCHK(hipFuncSetAttribute(pipe_fn(n), hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    return lds;
}

void cons_seq_launch(const RParArgs& a, const RParBufs<double>& bf, size_t lds, hipStream_t stream) {
    RParArgs aa = a;
    RParBufs<double> bb = bf;
    void* args[] = {&aa, &bb};
    // one workgroup per relation of the batch, most frequent first (chain_first_tile);
    // the pair records are made at the end of each relation's chain (chain_records)
    HIPCHK(hipLaunchKernel(pipe_fn(a.n), dim3(chain_grid(a)), dim3(kChainThreads), args, lds, stream));
}

bool cons_chainw_supported(int n) { return n >= 1 && n <= kWideMaxN; }

size_t cons_chainw_setup(int n) {
    HIPCHK(hipFuncSetAttribute((const void*)transr_cons_da_rel_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)da_rel_lds(n)));
    const bool wp = use_wpipe(n);
    const size_t lds = wp ? chainwp_lds(n) : chainw_lds(n);
    HIPCHK(hipFuncSetAttribute(wp ? chainwp_fn(n) : chainw_fn(n), hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)lds));
    return lds;
}

bool cons_chainw_pipelined(int n) { return use_wpipe(n); }

void cons_chainw_launch(const RParArgs& a, const RParBufs<double>& bf, size_t lds, hipStream_t stream) {
    RParArgs aa = a;
    RParBufs<double> bb = bf;
    void* args[] = {&aa, &bb};
    // one workgroup per relation of the batch, most frequent first
    const int grid = chain_grid(a);
    // (the LDS size was chosen by cons_chainw_setup under the same switch)
    if (use_wpipe(a.n)) {
        // (the pipelined chain makes its relation's pair records itself)
        HIPCHK(hipLaunchKernel(chainwp_fn(a.n), dim3(grid), dim3(kWPThreads), args, lds, stream));
    } else {
        HIPCHK(hipLaunchKernel(chainw_fn(a.n), dim3(grid), dim3(kWideThreads), args, lds, stream));
        // the pair records: a workgroup per relation, its final matrix staged once
        HIPCHK(hipLaunchKernel((const void*)transr_cons_da_rel_kernel, dim3(grid), dim3(kDaRelThreads), args,
                               da_rel_lds(a.n), stream));
    }
}

bool cons_wave_supported(int n) { return n >= 1 && n <= 64; }

size_t cons_wave_setup(int n, int St, int esize) {
    const size_t lds = esize == 8 ? rcons_lds<double>(n, St) : rcons_lds<float>(n, St);
    HIPCHK(hipFuncSetAttribute(esize == 8 ? cons_fn<double>(n) : cons_fn<float>(n),
                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    return lds;
}

template <typename T>
void cons_wave_launch(const RParArgs& a, const RParBufs<T>& bf, int grid, size_t lds, hipStream_t stream) {
    RParArgs aa = a;
    RParBufs<T> bb = bf;
    void* args[] = {&aa, &bb};
    HIPCHK(hipLaunchKernel(cons_fn<T>(a.n), dim3(grid), dim3(kConsWaves * kWave), args, lds, stream));
}

template <typename T>
void grad_wave_launch(const RParArgs& a, const RParBufs<T>& bf, int grid, hipStream_t stream) {
    RParArgs aa = a;
    RParBufs<T> bb = bf;
    void* args[] = {&aa, &bb};
    HIPCHK(hipLaunchKernel(kernel_fn<T>(kGrad, a.n), dim3(grid), dim3(kConsWaves * kWave), args, 0, stream));
}

template <typename T>
void proj_wave_launch(const RParArgs& a, const RParBufs<T>& bf, int grid, hipStream_t stream) {
    RParArgs aa = a;
    RParBufs<T> bb = bf;
    void* args[] = {&aa, &bb};
    const size_t lds = sizeof(T) * (size_t)proj_wave_rows<T>(cons_live_steps<T>(a.n)) * rm_ld(a.n);
    HIPCHK(hipLaunchKernel(kernel_fn<T>(kProj, a.n), dim3(grid), dim3(kProjWaves * kWave), args, lds, stream));
}

bool cons_chaing_supported(int n) { return n >= 1 && n <= kGenMaxN; }

size_t cons_chaing_setup(int n, int esize) {
    const size_t lds = chaing_lds(n);
    HIPCHK(hipFuncSetAttribute(esize == 8 ? (const void*)transr_cons_chain_gen_kernel<double>
                                          : (const void*)transr_cons_chain_gen_kernel<float>,
                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    return lds;
}

template <typename T>
void cons_chaing_launch(const RParArgs& a, const RParBufs<T>& bf, size_t lds, hipStream_t stream) {
    RParArgs aa = a;
    RParBufs<T> bb = bf;
    void* args[] = {&aa, &bb};
    // one workgroup per relation of the batch, most frequent first
    HIPCHK(hipLaunchKernel((const void*)transr_cons_chain_gen_kernel<T>, dim3(chain_grid(a)), dim3(kGenThreads), args,
                           lds, stream));
}
template void cons_chaing_launch<double>(const RParArgs&, const RParBufs<double>&, size_t, hipStream_t);
template void cons_chaing_launch<float>(const RParArgs&, const RParBufs<float>&, size_t, hipStream_t);

template void proj_wave_launch<double>(const RParArgs&, const RParBufs<double>&, int, hipStream_t);
template void proj_wave_launch<float>(const RParArgs&, const RParBufs<float>&, int, hipStream_t);

template void grad_wave_launch<double>(const RParArgs&, const RParBufs<double>&, int, hipStream_t);
template void grad_wave_launch<float>(const RParArgs&, const RParBufs<float>&, int, hipStream_t);

template void cons_wave_launch<double>(const RParArgs&, const RParBufs<double>&, int, size_t, hipStream_t);
template void cons_wave_launch<float>(const RParArgs&, const RParBufs<float>&, int, size_t, hipStream_t);

void cons_seq_take_stats(unsigned long long (&st)[64]) {
    HIPCHK(hipMemcpyFromSymbol(st, HIP_SYMBOL(g_seq_stats), sizeof(st)));
    unsigned long long z[64] = {};
    HIPCHK(hipMemcpyToSymbol(HIP_SYMBOL(g_seq_stats), z, sizeof(z)));
}

void cons_wave_take_stats(unsigned long long (&st)[16]) {
    unsigned long long mine[16];
    HIPCHK(hipMemcpyFromSymbol(mine, HIP_SYMBOL(g_cons_stats), sizeof(mine)));
    for (int k = 0; k < 16; ++k) st[k] = (k == 2 || k == 6) ? std::max(st[k], mine[k]) : st[k] + mine[k];
    std::memset(mine, 0, sizeof(mine));
    HIPCHK(hipMemcpyToSymbol(HIP_SYMBOL(g_cons_stats), mine, sizeof(mine)));
}

}  // namespace kb2e
