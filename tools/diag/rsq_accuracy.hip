// Max relative error of the hardware v_rsq_f64 estimate (and after one and two
// Newton steps) against 1/sqrt(x) computed with IEEE sqrt and division.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>

__global__ void probe(double* out, int n) {
    double e0 = 0, e1 = 0, e2 = 0;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const double x = 0.25 + 3.75 * ((double)i / n);
        const double ref = 1.0 / sqrt(x);
        double y = __builtin_amdgcn_rsq(x);
        e0 = fmax(e0, fabs(y - ref) / ref);
        y = y * (1.5 - 0.5 * x * y * y);
        e1 = fmax(e1, fabs(y - ref) / ref);
        y = y * (1.5 - 0.5 * x * y * y);
        e2 = fmax(e2, fabs(y - ref) / ref);
    }
    atomicMax((unsigned long long*)&out[0], __double_as_longlong(e0));
    atomicMax((unsigned long long*)&out[1], __double_as_longlong(e1));
    atomicMax((unsigned long long*)&out[2], __double_as_longlong(e2));
}

int main() {
    double* d;
    hipMalloc(&d, 3 * sizeof(double));
    hipMemset(d, 0, 3 * sizeof(double));
    probe<<<1024, 256>>>(d, 1 << 26);
    double h[3];
    hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    printf("max rel err: rsq %.3e  1 newton %.3e  2 newton %.3e (2^-52 = %.3e)\n", h[0], h[1], h[2], std::ldexp(1.0, -52));
    return 0;
}
