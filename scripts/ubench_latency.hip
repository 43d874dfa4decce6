// Latency micro-benchmark for the SQP kernel's critical-path operations on gfx950
// (one wave, s_memtime around dependent chains).  Diagnostic only, not part of
// the product.  Build + run:
//   hipcc --offload-arch=gfx950 -O3 scripts/ubench_latency.hip -o /tmp/ubench && /tmp/ubench
#include <hip/hip_runtime.h>

#include <cstdio>

#define REPS 256

__global__ void ubench(double* out, unsigned long long* cyc, double seed) {
    __shared__ double sh[256];
    const int lane = threadIdx.x;
    double x = seed + lane * 1e-3, y = 1.0000001;
    unsigned long long t0, t1;
    // 1) dependent fp64 FMA chain
    t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 16
    for (int i = 0; i < REPS; ++i) x = fma(x, y, 1e-9);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) cyc[0] = t1 - t0;
    // 2) independent fp64 FMAs (5 chains interleaved, issue rate)
    double a0 = x, a1 = x + 1, a2 = x + 2, a3 = x + 3, a4 = x + 4;
    t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 16
    for (int i = 0; i < REPS; ++i) {
        a0 = fma(a0, y, 1e-9); a1 = fma(a1, y, 1e-9); a2 = fma(a2, y, 1e-9);
        a3 = fma(a3, y, 1e-9); a4 = fma(a4, y, 1e-9);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) cyc[1] = t1 - t0;
    x = a0 + a1 + a2 + a3 + a4;
    // 3) dependent v_rsq_f64 chain
    double r = 1.5 + lane * 1e-6;
    t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 16
    for (int i = 0; i < REPS; ++i) r = __builtin_amdgcn_rsq(r) + 0.5;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) cyc[2] = t1 - t0;  // rsq + add per step
    x += r;
    // 4) readlane round trip: VALU result -> v_readlane (2 x b32) -> VALU consumer
    double z = x;
    t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 16
    for (int i = 0; i < REPS; ++i) {
        const int lo = __builtin_amdgcn_readlane(__double2loint(z), 5);
        const int hi = __builtin_amdgcn_readlane(__double2hiint(z), 5);
        z = fma(__hiloint2double(hi, lo), y, 1e-9);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) cyc[3] = t1 - t0;  // readlane pair + fma per step
    x += z;
    // 5) LDS round trip: ds_write -> ds_read (another lane's slot) -> VALU consumer
    double w = x;
    t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 16
    for (int i = 0; i < REPS; ++i) {
        sh[lane] = w;
        asm volatile("" ::: "memory");
        w = fma(sh[(lane + 1) & 63], y, 1e-9);
        asm volatile("" ::: "memory");
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) cyc[4] = t1 - t0;  // write + read + fma per step
    x += w;
    out[lane] = x;
}

int main() {
    double* d_out;
    unsigned long long* d_cyc;
    hipMalloc(&d_out, 64 * sizeof(double));
    hipMalloc(&d_cyc, 8 * sizeof(unsigned long long));
    unsigned long long cyc[8];
    const char* names[5] = {"dependent v_fma_f64", "5 independent v_fma_f64 (per fma)", "dependent v_rsq_f64 + v_add_f64",
                            "v_readlane x2 -> v_fma_f64", "ds_write_b64 -> ds_read_b64 -> v_fma_f64"};
    const double div[5] = {REPS, 5.0 * REPS, REPS, REPS, REPS};
    for (int rep = 0; rep < 3; ++rep) {
        hipLaunchKernelGGL(ubench, dim3(1), dim3(64), 0, 0, d_out, d_cyc, 1.0 + rep);
        hipDeviceSynchronize();
    }
    hipMemcpy(cyc, d_cyc, sizeof(cyc), hipMemcpyDeviceToHost);
    for (int i = 0; i < 5; ++i) printf("%-44s %7.1f cycles per step\n", names[i], cyc[i] / div[i]);
    hipFree(d_out);
    hipFree(d_cyc);
    return 0;
}
