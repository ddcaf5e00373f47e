// kappa = pvd * (1 / pp) with 1 / pp from v_rcp_f64 plus one or two Newton steps,
// against the IEEE quotient pvd / pp (the CPU model's), over pp in (1, 64) and
// pvd in (-64, 64): the largest difference in ulps of the quotient, and how often
// the two differ at all (kernels_transr_pipe.hpp / _chainwp.hpp).
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdint>

__device__ double ulps(double a, double b) {
    const double u = fabs(b) > 0 ? ldexp(1.0, ilogb(b) - 52) : 4.9e-324;
    return fabs(a - b) / u;
}

__global__ void probe(double* out, unsigned long long* cnt, int n) {
    double m1 = 0, m2 = 0;
    unsigned long long d1 = 0, d2 = 0;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        uint64_t s = 0x9E3779B97F4A7C15ull * (uint64_t)(i + 1);
        s ^= s >> 29; s *= 0xBF58476D1CE4E5B9ull; s ^= s >> 32;
        const double u0 = (double)(s >> 11) * 0x1p-53;
        s *= 0x94D049BB133111EBull; s ^= s >> 31;
        const double u1 = (double)(s >> 11) * 0x1p-53;
        const double pp = 1.0 + 63.0 * u0, pvd = -64.0 + 128.0 * u1;
        const double q = pvd / pp;
        double r = __builtin_amdgcn_rcp(pp);
        r = fma(fma(-pp, r, 1.0), r, r);
        const double k1 = pvd * r;
        r = fma(fma(-pp, r, 1.0), r, r);
        const double k2 = pvd * r;
        m1 = fmax(m1, ulps(k1, q));
        m2 = fmax(m2, ulps(k2, q));
        d1 += k1 != q;
        d2 += k2 != q;
    }
    atomicMax((unsigned long long*)&out[0], __double_as_longlong(m1));
    atomicMax((unsigned long long*)&out[1], __double_as_longlong(m2));
    atomicAdd(&cnt[0], d1);
    atomicAdd(&cnt[1], d2);
}

int main() {
    double* d;
    unsigned long long* c;
    hipMalloc(&d, 2 * sizeof(double));
    hipMalloc(&c, 2 * sizeof(unsigned long long));
    hipMemset(d, 0, 2 * sizeof(double));
    hipMemset(c, 0, 2 * sizeof(unsigned long long));
    const int n = 1 << 26;
    probe<<<1024, 256>>>(d, c, n);
    double h[2];
    unsigned long long hc[2];
    hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    hipMemcpy(hc, c, sizeof(hc), hipMemcpyDeviceToHost);
    printf("kappa vs pvd/pp over %d draws: 1 newton max %.2f ulp (%llu differ), 2 newton max %.2f ulp (%llu differ)\n",
           n, h[0], hc[0], h[1], hc[1]);
    return 0;
}
