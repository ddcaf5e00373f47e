// Single-wave latency / issue micro-benchmark for the instruction mix of the
// serial chains (fold, owners): cycles (clock64) per operation.
#include <hip/hip_runtime.h>
#include <cstdio>

#define REP 256

__global__ void bench(double* out, double seed, int iters) {
    const int l = threadIdx.x;
    double a = seed + l * 1e-9, b = 1.0000001, c = 0.9999999;
    double r[8];
    for (int q = 0; q < 8; ++q) r[q] = a + q;
    unsigned long long t0, t1;
    int k = 0;
    // 1. dependent v_mul_f64 chain
    t0 = clock64();
    for (int it = 0; it < iters; ++it)
#pragma unroll
        for (int q = 0; q < REP; ++q) asm volatile("v_mul_f64 %0, %0, %1" : "+v"(a) : "v"(b));
    t1 = clock64();
    if (l == 0) out[k] = (double)(t1 - t0) / (iters * REP);
    ++k;
    // 2. eight independent v_mul_f64 chains
    t0 = clock64();
    for (int it = 0; it < iters; ++it)
#pragma unroll
        for (int q = 0; q < REP / 8; ++q) {
            asm volatile("v_mul_f64 %0, %0, %1" : "+v"(r[0]) : "v"(b));
            asm volatile("v_mul_f64 %0, %0, %1" : "+v"(r[1]) : "v"(b));
            asm volatile("v_mul_f64 %0, %0, %1" : "+v"(r[2]) : "v"(b));
            asm volatile("v_mul_f64 %0, %0, %1" : "+v"(r[3]) : "v"(b));
            asm volatile("v_mul_f64 %0, %0, %1" : "+v"(r[4]) : "v"(b));
            asm volatile("v_mul_f64 %0, %0, %1" : "+v"(r[5]) : "v"(b));
            asm volatile("v_mul_f64 %0, %0, %1" : "+v"(r[6]) : "v"(b));
            asm volatile("v_mul_f64 %0, %0, %1" : "+v"(r[7]) : "v"(b));
        }
    t1 = clock64();
    if (l == 0) out[k] = (double)(t1 - t0) / (iters * REP);
    ++k;
    // 3. dependent v_fma_f64 chain
    t0 = clock64();
    for (int it = 0; it < iters; ++it)
#pragma unroll
        for (int q = 0; q < REP; ++q) asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(a) : "v"(b), "v"(c));
    t1 = clock64();
    if (l == 0) out[k] = (double)(t1 - t0) / (iters * REP);
    ++k;
    // 4. dependent v_rsq_f64 chain
    t0 = clock64();
    for (int it = 0; it < iters; ++it)
#pragma unroll
        for (int q = 0; q < REP; ++q) asm volatile("v_rsq_f64 %0, %0" : "+v"(a));
    t1 = clock64();
    if (l == 0) out[k] = (double)(t1 - t0) / (iters * REP);
    ++k;
    // 5. dependent v_add_f32 chain and 6. independent v_add_f32
    float fa = (float)a, fb = 1.0f;
    float fr[8];
    for (int q = 0; q < 8; ++q) fr[q] = fa + q;
    t0 = clock64();
    for (int it = 0; it < iters; ++it)
#pragma unroll
        for (int q = 0; q < REP; ++q) asm volatile("v_add_f32 %0, %0, %1" : "+v"(fa) : "v"(fb));
    t1 = clock64();
    if (l == 0) out[k] = (double)(t1 - t0) / (iters * REP);
    ++k;
    t0 = clock64();
    for (int it = 0; it < iters; ++it)
#pragma unroll
        for (int q = 0; q < REP / 8; ++q) {
            asm volatile("v_add_f32 %0, %0, %1" : "+v"(fr[0]) : "v"(fb));
            asm volatile("v_add_f32 %0, %0, %1" : "+v"(fr[1]) : "v"(fb));
            asm volatile("v_add_f32 %0, %0, %1" : "+v"(fr[2]) : "v"(fb));
            asm volatile("v_add_f32 %0, %0, %1" : "+v"(fr[3]) : "v"(fb));
            asm volatile("v_add_f32 %0, %0, %1" : "+v"(fr[4]) : "v"(fb));
            asm volatile("v_add_f32 %0, %0, %1" : "+v"(fr[5]) : "v"(fb));
            asm volatile("v_add_f32 %0, %0, %1" : "+v"(fr[6]) : "v"(fb));
            asm volatile("v_add_f32 %0, %0, %1" : "+v"(fr[7]) : "v"(fb));
        }
    t1 = clock64();
    if (l == 0) out[k] = (double)(t1 - t0) / (iters * REP);
    ++k;
    // 7. readlane -> VALU use round trip (f32 add of a readlane'd value, dependent)
    t0 = clock64();
    for (int it = 0; it < iters; ++it)
#pragma unroll
        for (int q = 0; q < REP; ++q) {
            int sv;
            asm volatile("v_readlane_b32 %0, %1, 5" : "=s"(sv) : "v"(fa));
            asm volatile("s_nop 0\n\tv_add_f32 %0, %1, %0" : "+v"(fa) : "s"(sv));
        }
    t1 = clock64();
    if (l == 0) out[k] = (double)(t1 - t0) / (iters * REP);
    ++k;
    // 8. dependent DPP row_ror + v_add_f32
    t0 = clock64();
    for (int it = 0; it < iters; ++it)
#pragma unroll
        for (int q = 0; q < REP; ++q) asm volatile("s_nop 1\n\tv_add_f32_dpp %0, %0, %0 row_ror:1 row_mask:0xf bank_mask:0xf" : "+v"(fa));
    t1 = clock64();
    if (l == 0) out[k] = (double)(t1 - t0) / (iters * REP);
    ++k;
    // 9. s_nop 0 cost
    t0 = clock64();
    for (int it = 0; it < iters; ++it)
#pragma unroll
        for (int q = 0; q < REP; ++q) asm volatile("s_nop 0");
    t1 = clock64();
    if (l == 0) out[k] = (double)(t1 - t0) / (iters * REP);
    ++k;
    // 10. wall clock rate vs clock64 (s_memrealtime is 100 MHz)
    unsigned long long w0 = wall_clock64();
    t0 = clock64();
    for (int it = 0; it < iters * 16; ++it)
#pragma unroll
        for (int q = 0; q < REP; ++q) asm volatile("v_mul_f64 %0, %0, %1" : "+v"(a) : "v"(b));
    t1 = clock64();
    unsigned long long w1 = wall_clock64();
    if (l == 0) out[k] = (double)(t1 - t0) / ((double)(w1 - w0) / 100.0);  // clock64 ticks per microsecond
    ++k;
    double sink = a + fa;
    for (int q = 0; q < 8; ++q) sink += r[q] + fr[q];
    if (sink == 12345.678) out[15] = sink;
}

int main() {
    double* d;
    (void)hipMalloc(&d, 16 * sizeof(double));
    (void)hipMemset(d, 0, 16 * sizeof(double));
    bench<<<1, 64>>>(d, 1.0, 64);
    (void)hipDeviceSynchronize();
    bench<<<1, 64>>>(d, 1.0, 64);
    double h[16];
    (void)hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    const char* names[] = {"dep v_mul_f64", "8x indep v_mul_f64", "dep v_fma_f64", "dep v_rsq_f64", "dep v_add_f32",
                           "8x indep v_add_f32", "readlane->v_add_f32 round trip", "dep DPP v_add_f32",
                           "s_nop 0", "clock64 ticks per us"};
    for (int k = 0; k < 10; ++k) printf("%-34s %8.2f\n", names[k], h[k]);
    return 0;
}
