// One-wave cycle counts (clock64) for v_mfma_f64_16x16x4_f64: a dependent
// accumulation chain, four interleaved chains, and v_fma_f64 for comparison.
// hipcc --offload-arch=gfx950 -O3 tools/diag/mfma_f64.hip -o /tmp/mfma_f64 && /tmp/mfma_f64
#include <hip/hip_runtime.h>
#include <cstdio>

typedef double d4 __attribute__((ext_vector_type(4)));
constexpr int N = 256;

__global__ void bench(double* out, double seed) {
    const int l = threadIdx.x;
    double a = seed + l * 1e-9, b = 1.0 - l * 1e-9;
    d4 c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
    unsigned long long t0 = clock64();
#pragma unroll
    for (int q = 0; q < N; ++q) asm volatile("v_mfma_f64_16x16x4_f64 %0, %1, %2, %0" : "+v"(c0) : "v"(a), "v"(b));
    asm volatile("s_nop 7\n s_nop 7\n v_mov_b64 %0, %0" : "+v"(a) : "v"(c0));
    unsigned long long t1 = clock64();
#pragma unroll
    for (int q = 0; q < N / 4; ++q) {
        asm volatile("v_mfma_f64_16x16x4_f64 %0, %1, %2, %0" : "+v"(c0) : "v"(a), "v"(b));
        asm volatile("v_mfma_f64_16x16x4_f64 %0, %1, %2, %0" : "+v"(c1) : "v"(a), "v"(b));
        asm volatile("v_mfma_f64_16x16x4_f64 %0, %1, %2, %0" : "+v"(c2) : "v"(a), "v"(b));
        asm volatile("v_mfma_f64_16x16x4_f64 %0, %1, %2, %0" : "+v"(c3) : "v"(a), "v"(b));
    }
    unsigned long long t2 = clock64();
    double r[8];
    for (int q = 0; q < 8; ++q) r[q] = a + q;
#pragma unroll
    for (int q = 0; q < N / 8; ++q)
#pragma unroll
        for (int k = 0; k < 8; ++k) asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(r[k]) : "v"(b), "v"(a));
    unsigned long long t3 = clock64();
    float fa = (float)a, fb = (float)b;
    typedef float f4 __attribute__((ext_vector_type(4)));
    f4 g0 = {0, 0, 0, 0};
#pragma unroll
    for (int q = 0; q < N; ++q) asm volatile("v_mfma_f32_16x16x4_f32 %0, %1, %2, %0" : "+v"(g0) : "v"(fa), "v"(fb));
    unsigned long long t4 = clock64();
    if (l == 0) {
        out[0] = (double)(t1 - t0) / N;
        out[1] = (double)(t2 - t1) / N;
        out[2] = (double)(t3 - t2) / N;
        out[3] = (double)(t4 - t3) / N;
    }
    double s = 0;
    for (int k = 0; k < 8; ++k) s += r[k];
    out[8 + l] = c0[0] + c1[1] + c2[2] + c3[3] + s + g0[0];
}

int main() {
    double* d;
    (void)hipMalloc(&d, 128 * sizeof(double));
    for (int rep = 0; rep < 3; ++rep) {
        bench<<<1, 64>>>(d, 1.0);
        (void)hipDeviceSynchronize();
    }
    double h[4];
    (void)hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    printf("mfma_f64_16x16x4 dependent chain: %.1f cyc/op\n", h[0]);
    printf("mfma_f64_16x16x4 4 chains interleaved: %.1f cyc/op\n", h[1]);
    printf("v_fma_f64 8 independent chains: %.1f cyc/op\n", h[2]);
    printf("mfma_f32_16x16x4 dependent chain: %.1f cyc/op\n", h[3]);
    return 0;
}
