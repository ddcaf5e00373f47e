// Micro-benchmark of one transRNorm VALU round (kernels_transr_cons.hpp) on
// gfx950: cycles (clock64) per round for R rows, two matvecs (W0 then W0^T)
// or one (K), one wave per workgroup, `wgs` workgroups.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#include "../../kb2e_amd/csrc/kernels_transr_cons.hpp"

using namespace kb2e;

template <int R, int NP, int KN, bool TWO>
__global__ void round_bench(double* out, int iters) {
    constexpr int L = NP + 1;
    __shared__ double Wl[NP * L];
    __shared__ double SP[2 * kValuRows * NP];
    const int l = threadIdx.x;
    for (int idx = l; idx < NP * L; idx += 64) Wl[idx] = ((idx * 7919) % 101) * 1e-4;
    for (int idx = l; idx < 2 * kValuRows * NP; idx += 64) SP[idx] = ((idx * 31) % 17) * 1e-3;
    __syncthreads();
    const int i = l < NP ? l : 0;
    double pv[R];
    for (int j = 0; j < R; ++j) pv[j] = SP[j * NP + i];
    const unsigned long long t0 = clock64();
    for (int it = 0; it < iters; ++it) {
        double tv[R], q[R];
        if (TWO) {
            valu_matvec<double, R, L, NP, KN, true>(Wl, SP, i, tv);
#pragma unroll
            for (int j = 0; j < R; ++j) SP[(kValuRows + j) * NP + i] = tv[j];
            wave_lds_sync();
            valu_matvec<double, R, L, NP, KN, false>(Wl, SP + kValuRows * NP, i, q);
        } else {
            valu_matvec<double, R, L, NP, KN, false>(Wl, SP, i, q);
        }
        double nr[R];
#pragma unroll
        for (int j = 0; j < R; ++j) {
            pv[j] = pv[j] - 2e-3 * q[j] - 1e-3 * pv[j];
            nr[j] = wave_sum(pv[j] * pv[j]);
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
        for (int j = 0; j < R; ++j) SP[j * NP + i] = pv[j] + (nr[j] > 1e30 ? 1.0 : 0.0);
        wave_lds_sync();
    }
    const unsigned long long t1 = clock64();
    if (l == 0) out[blockIdx.x] = (double)(t1 - t0) / iters;
}

// K column of lane i in registers, p_k as LDS broadcasts
template <int R, int NP, int KN>
__global__ void round_bench_kreg(double* out, int iters) {
    constexpr int L = NP + 1;
    __shared__ double Wl[NP * L];
    __shared__ double SP[2 * kValuRows * NP];
    const int l = threadIdx.x;
    for (int idx = l; idx < NP * L; idx += 64) Wl[idx] = ((idx * 7919) % 101) * 1e-4;
    for (int idx = l; idx < 2 * kValuRows * NP; idx += 64) SP[idx] = ((idx * 31) % 17) * 1e-3;
    __syncthreads();
    const int i = l < NP ? l : 0;
    double kr[KN];
#pragma unroll
    for (int k = 0; k < KN; ++k) kr[k] = Wl[k * L + i];
    double pv[R];
    for (int j = 0; j < R; ++j) pv[j] = SP[j * NP + i];
    const unsigned long long t0 = clock64();
    for (int it = 0; it < iters; ++it) {
        double acc[R][4];
#pragma unroll
        for (int j = 0; j < R; ++j) acc[j][0] = acc[j][1] = acc[j][2] = acc[j][3] = 0.0;
#pragma unroll
        for (int k = 0; k < KN; k += 4)
#pragma unroll
            for (int j = 0; j < R; ++j)
#pragma unroll
                for (int u = 0; u < 4; ++u) acc[j][u] += kr[k + u] * SP[j * NP + k + u];
        double nr[R];
#pragma unroll
        for (int j = 0; j < R; ++j) {
            const double q = (acc[j][0] + acc[j][1]) + (acc[j][2] + acc[j][3]);
            pv[j] = pv[j] - 2e-3 * q - 1e-3 * pv[j];
            nr[j] = wave_sum(pv[j] * pv[j]);
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
        for (int j = 0; j < R; ++j) SP[j * NP + i] = pv[j] + (nr[j] > 1e30 ? 1.0 : 0.0);
        wave_lds_sync();
    }
    const unsigned long long t1 = clock64();
    if (l == 0) out[blockIdx.x] = (double)(t1 - t0) / iters;
}

// p loaded into registers first (all LDS broadcasts in flight), then FMAs;
// K from LDS (KREG false) or from registers (true)
template <int R, int NP, int KN, bool KREG>
__global__ void round_bench_pre(double* out, int iters) {
    constexpr int L = NP + 1;
    __shared__ double Wl[NP * L];
    __shared__ double SP[2 * kValuRows * NP];
    const int l = threadIdx.x;
    for (int idx = l; idx < NP * L; idx += 64) Wl[idx] = ((idx * 7919) % 101) * 1e-4;
    for (int idx = l; idx < 2 * kValuRows * NP; idx += 64) SP[idx] = ((idx * 31) % 17) * 1e-3;
    __syncthreads();
    const int i = l < NP ? l : 0;
    double kr[KREG ? KN : 1];
    if (KREG) {
#pragma unroll
        for (int k = 0; k < KN; ++k) kr[k] = Wl[k * L + i];
    }
    double pv[R];
    for (int j = 0; j < R; ++j) pv[j] = SP[j * NP + i];
    const unsigned long long t0 = clock64();
    for (int it = 0; it < iters; ++it) {
        double acc[R][4];
#pragma unroll
        for (int j = 0; j < R; ++j) acc[j][0] = acc[j][1] = acc[j][2] = acc[j][3] = 0.0;
#pragma unroll
        for (int k0 = 0; k0 < KN; k0 += 16) {  // 16 k at a time: loads in flight, then FMAs
            double pk[R][16], kk[16];
#pragma unroll
            for (int k = 0; k < 16; ++k) {
                if (k0 + k >= KN) break;
                if (!KREG) kk[k] = Wl[(k0 + k) * L + i];
#pragma unroll
                for (int j = 0; j < R; ++j) pk[j][k] = SP[j * NP + k0 + k];
            }
#pragma unroll
            for (int k = 0; k < 16; ++k) {
                if (k0 + k >= KN) break;
                if (!KREG) pin(kk[k]);
#pragma unroll
                for (int j = 0; j < R; ++j) pin(pk[j][k]);
            }
#pragma unroll
            for (int k = 0; k < 16; ++k) {
                if (k0 + k >= KN) break;
                const double w = KREG ? kr[k0 + k] : kk[k];
#pragma unroll
                for (int j = 0; j < R; ++j) acc[j][k & 3] = fma(w, pk[j][k], acc[j][k & 3]);
            }
        }
        double nr[R];
#pragma unroll
        for (int j = 0; j < R; ++j) {
            const double q = (acc[j][0] + acc[j][1]) + (acc[j][2] + acc[j][3]);
            pv[j] = pv[j] - 2e-3 * q - 1e-3 * pv[j];
            nr[j] = wave_sum(pv[j] * pv[j]);
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
        for (int j = 0; j < R; ++j) SP[j * NP + i] = pv[j] + (nr[j] > 1e30 ? 1.0 : 0.0);
        wave_lds_sync();
    }
    const unsigned long long t1 = clock64();
    if (l == 0) out[blockIdx.x] = (double)(t1 - t0) / iters;
}

template <int R, bool KREG>
void run_pre(int wgs, double* d) {
    const int iters = 200;
    round_bench_pre<R, 64, 52, KREG><<<wgs, 64>>>(d, iters);
    (void)hipDeviceSynchronize();
    round_bench_pre<R, 64, 52, KREG><<<wgs, 64>>>(d, iters);
    (void)hipDeviceSynchronize();
    std::vector<double> h(wgs);
    (void)hipMemcpy(h.data(), d, wgs * sizeof(double), hipMemcpyDeviceToHost);
    double s = 0;
    for (double v : h) s += v;
    printf("%-28s R=%d wgs=%5d: %8.0f cycles/round (clock64)\n", KREG ? "p preloaded, K regs" : "p preloaded, K LDS",
           R, wgs, s / wgs);
}

template <int R>
void run_kreg(int wgs, double* d) {
    const int iters = 200;
    round_bench_kreg<R, 64, 52><<<wgs, 64>>>(d, iters);
    (void)hipDeviceSynchronize();
    round_bench_kreg<R, 64, 52><<<wgs, 64>>>(d, iters);
    (void)hipDeviceSynchronize();
    std::vector<double> h(wgs);
    (void)hipMemcpy(h.data(), d, wgs * sizeof(double), hipMemcpyDeviceToHost);
    double s = 0;
    for (double v : h) s += v;
    printf("%-28s R=%d wgs=%5d: %8.0f cycles/round (clock64)\n", "K column in registers", R, wgs, s / wgs);
}

template <int R, bool TWO>
void run(int wgs, double* d, const char* name) {
    const int iters = 200;
    round_bench<R, 64, 52, TWO><<<wgs, 64>>>(d, iters);
    (void)hipDeviceSynchronize();
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    (void)hipEventRecord(a);
    round_bench<R, 64, 52, TWO><<<wgs, 64>>>(d, iters);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    std::vector<double> h(wgs);
    (void)hipMemcpy(h.data(), d, wgs * sizeof(double), hipMemcpyDeviceToHost);
    double s = 0;
    for (double v : h) s += v;
    printf("%-28s R=%d wgs=%5d: %8.0f cycles/round (clock64), %7.3f us/round (events)\n", name, R, wgs, s / wgs,
           ms * 1e3 / iters);
}

int main() {
    double* d;
    (void)hipMalloc(&d, 8192 * sizeof(double));
    for (int wgs : {1, 1024}) {
        run<1, true>(wgs, d, "two matvecs (W0, W0^T)");
        run<1, false>(wgs, d, "one matvec (K)");
        run<2, true>(wgs, d, "two matvecs (W0, W0^T)");
        run<4, true>(wgs, d, "two matvecs (W0, W0^T)");
        run_kreg<1>(wgs, d);
        run_pre<1, false>(wgs, d);
        run_pre<1, true>(wgs, d);
        run_pre<2, false>(wgs, d);
        run_pre<4, false>(wgs, d);
    }
    int clk = 0;
    (void)hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, 0);
    printf("clock rate %d kHz\n", clk);
    return 0;
}
