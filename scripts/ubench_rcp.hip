// Accuracy of the gfx950 fp64 reciprocal / reciprocal square root instructions (v_rcp_f64, v_rsq_f64)
// and of one Newton step on v_rcp_f64, against the host (the evidence for how many Newton steps the
// interior point's reciprocals need).  hipcc --offload-arch=gfx950 -O2 scripts/ubench_rcp.hip -o scripts/ubench_rcp
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cmath>
#include <cstdlib>
__global__ void k(const double* x, double* r0, double* r1, double* s0, int n) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    double v = x[i];
    double y = __builtin_amdgcn_rcp(v);
    r0[i] = y;
    double e = fma(-v, y, 1.0);
    r1[i] = fma(y, e, y);
    s0[i] = __builtin_amdgcn_rsq(v);
}
int main() {
    const int n = 1 << 20;
    double *x, *a, *b, *c;
    hipMallocManaged(&x, n * 8); hipMallocManaged(&a, n * 8); hipMallocManaged(&b, n * 8); hipMallocManaged(&c, n * 8);
    srand(1);
    for (int i = 0; i < n; ++i) x[i] = std::ldexp(1.0 + rand() / (double)RAND_MAX, (rand() % 80) - 40);
    hipLaunchKernelGGL(k, dim3(n / 256), dim3(256), 0, 0, x, a, b, c, n);
    hipDeviceSynchronize();
    double m0 = 0, m1 = 0, ms = 0;
    for (int i = 0; i < n; ++i) {
        double r = 1.0 / x[i], q = 1.0 / std::sqrt(x[i]);
        m0 = fmax(m0, fabs(a[i] - r) / r); m1 = fmax(m1, fabs(b[i] - r) / r); ms = fmax(ms, fabs(c[i] - q) / q);
    }
    printf("rel err: rcp %.3e, rcp+1 newton %.3e, rsq %.3e (ulp %.3e)\n", m0, m1, ms, 2.220446e-16);
    return 0;
}
