// mpcg_kernels.hip — MI355X (gfx950) kernels of the batched T-MPC++ SQP solve.
//
// One wavefront (64 lanes, one workgroup) solves one (scene, guess) pair:
// the body of one `Solver::solve()` call of the OpenMP fan-out in
// GuidanceConstraints::optimize (guidance_constraints.cpp:304-421), i.e.
// `sqp_iters` acados SQP-RTI iterations (acados_solver_interface.cpp:311-429).
//
// Lane roles inside the wave
//   * stage lanes   lane k in [0, N]: linearisation of shooting stage k (cost,
//                   ERK4 sensitivities + exact Hessian, constraints, MIRROR),
//                   and every per-inequality interior-point operation of stage k
//   * element lanes lane e < 49: one entry (i, j) of the 7x7 Riccati stage
//                   block during the backward factorisation
//   * all lanes     redundant scalar recursions (vector pass, forward pass),
//                   so no LDS round trip sits on those sequential chains
// All QP data of one solve lives in LDS (struct Lds below); stage-indexed
// arrays are stage-minor so stage lanes access consecutive 8-byte words.
// Reductions (max residual, complementarity sum, step length) are xor
// butterflies: bit-identical in every lane, deterministic.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>
#include <string>

#include "mpcg.h"
#include "mpcg_device.h"
#include "mpcg_sqp.h"

namespace mpcg {

// ---- planner selection per scene (guidance_constraints.cpp:372-420, 572-590)
__global__ void select_best_kernel(int n_scenes, int G, int N, const double* __restrict__ xtraj,
                                   const double* __restrict__ pobj, const int* __restrict__ exit_code,
                                   const double* __restrict__ prev, double w_cons,
                                   const unsigned char* __restrict__ cons_en,
                                   const unsigned char* __restrict__ prev_sel, double sel_w,
                                   const unsigned char* __restrict__ disabled, int* __restrict__ best,
                                   double* __restrict__ objective) {
    const int sc = blockIdx.x * blockDim.x + threadIdx.x;
    if (sc >= n_scenes) return;
    double best_obj = 1e10;
    int best_i = -1;
    for (int g = 0; g < G; ++g) {
        const int s = sc * G + g;
        double obj = pobj[s];
        if (prev && cons_en && cons_en[s]) {
            // calculateConsistencyCostForSolver (guidance_constraints.cpp:1025-1050)
            double acc = 0.0;
            for (int k = 1; k <= N - 2; ++k) {
                const double dx = xtraj[((size_t)s * (N + 1) + k) * NX + 0] - prev[((size_t)sc * N + k) * 2 + 0];
                const double dy = xtraj[((size_t)s * (N + 1) + k) * NX + 1] - prev[((size_t)sc * N + k) * 2 + 1];
                acc += dx * dx + dy * dy;
            }
            obj -= w_cons * acc;
        }
        if (prev_sel && prev_sel[s]) obj *= sel_w;
        if (objective) objective[s] = obj;
        const bool dis = disabled && disabled[s];
        if (!dis && exit_code[s] == 1 && obj < best_obj) {
            best_obj = obj;
            best_i = g;
        }
    }
    best[sc] = best_i;
}

// ---- dispatch over compiled instances ------------------------------------
static thread_local std::string g_err;
static unsigned long long* g_stamps = nullptr;  // diagnostic stamp buffer (MPCG_STAMPS builds only)

template <class C>
static int launch(const mpcg_problem& pr, int batch, const double* params, const double* warm,
                  const double* xinit, double* xtraj, double* utraj, double* pobj, int* exit_code,
                  int* info, hipStream_t stream) {
    hipLaunchKernelGGL((sqp_kernel<C>), dim3(batch), dim3(64), 0, stream, pr, batch, params, warm, xinit,
                       xtraj, utraj, pobj, exit_code, info, g_stamps);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        g_err = std::string("sqp_kernel launch: ") + hipGetErrorString(e);
        return -1;
    }
    return 0;
}

using Fn = int (*)(const mpcg_problem&, int, const double*, const double*, const double*, double*, double*,
                   double*, int*, int*, hipStream_t);

static Fn find_instance(const mpcg_problem& pr) {
    if (pr.rk_steps < 1 || pr.n_seg < 1 || pr.n_seg > 16) return nullptr;
#define MPCG_INST(N_, L_, E_) \
    if (pr.N == N_ && pr.n_lin == L_ && pr.n_ell == E_) return &launch<Cfg<N_, L_, E_>>;
    MPCG_INST(20, 4, 4)    // C1
    MPCG_INST(20, 8, 8)    // C2 (north star)
    MPCG_INST(30, 12, 12)  // C4
    MPCG_INST(10, 2, 2)    // small test instance
#undef MPCG_INST
    return nullptr;
}

}  // namespace mpcg

extern "C" {

int mpcg_abi_version(void) { return MPCG_ABI_VERSION; }

/* diagnostic builds only: device buffer of batch x 10 u64 phase-cycle sums */
void mpcg_debug_set_stamp_buffer(unsigned long long* dev_ptr) { mpcg::g_stamps = dev_ptr; }

const char* mpcg_last_error(void) { return mpcg::g_err.c_str(); }

int mpcg_supported(const mpcg_problem* pr) { return (pr && mpcg::find_instance(*pr)) ? 0 : -1; }

int mpcg_solve_batch_device(const mpcg_problem* pr, int batch, const double* params, const double* warm,
                            const double* xinit, double* xtraj, double* utraj, double* pobj, int* exit_code,
                            int* info, void* stream) {
    if (!pr || batch < 0) { mpcg::g_err = "invalid arguments"; return -1; }
    if (batch == 0) return 0;
    mpcg::Fn fn = mpcg::find_instance(*pr);
    if (!fn) {
        mpcg::g_err = "no compiled instance for N=" + std::to_string(pr->N) + " n_lin=" + std::to_string(pr->n_lin) +
                      " n_ell=" + std::to_string(pr->n_ell);
        return -2;
    }
    return fn(*pr, batch, params, warm, xinit, xtraj, utraj, pobj, exit_code, info, (hipStream_t)stream);
}

int mpcg_solve_batch_host(const mpcg_problem* pr, int batch, const double* params, const double* warm,
                          const double* xinit, double* xtraj, double* utraj, double* pobj, int* exit_code,
                          int* info) {
    if (!pr || batch < 0) { mpcg::g_err = "invalid arguments"; return -1; }
    if (batch == 0) return 0;
    const size_t N = pr->N, np = pr->npar;
    const size_t s_par = batch * N * np, s_warm = batch * (N + 1) * MPCG_NVAR, s_xi = (size_t)batch * MPCG_NX;
    const size_t s_xt = batch * (N + 1) * MPCG_NX, s_ut = batch * N * MPCG_NU;
    double *dpar, *dwarm, *dxi, *dxt, *dut, *dpo;
    int *dex, *dinfo;
    size_t dbl = s_par + s_warm + s_xi + s_xt + s_ut + batch;
    if (hipMalloc(&dpar, dbl * sizeof(double)) != hipSuccess) { mpcg::g_err = "hipMalloc failed"; return -3; }
    if (hipMalloc(&dex, (size_t)batch * (1 + MPCG_INFO_STRIDE) * sizeof(int)) != hipSuccess) {
        (void)hipFree(dpar);
        mpcg::g_err = "hipMalloc failed";
        return -3;
    }
    dwarm = dpar + s_par; dxi = dwarm + s_warm; dxt = dxi + s_xi; dut = dxt + s_xt; dpo = dut + s_ut;
    dinfo = dex + batch;
    bool ok = hipMemcpy(dpar, params, s_par * sizeof(double), hipMemcpyHostToDevice) == hipSuccess &&
              hipMemcpy(dwarm, warm, s_warm * sizeof(double), hipMemcpyHostToDevice) == hipSuccess &&
              hipMemcpy(dxi, xinit, s_xi * sizeof(double), hipMemcpyHostToDevice) == hipSuccess;
    int rc = ok ? mpcg_solve_batch_device(pr, batch, dpar, dwarm, dxi, dxt, dut, dpo, dex, dinfo, nullptr) : -5;
    if (!ok) mpcg::g_err = "host to device copy failed";
    if (rc == 0) {
        hipError_t e = hipDeviceSynchronize();
        if (e != hipSuccess) { mpcg::g_err = std::string("solve: ") + hipGetErrorString(e); rc = -4; }
    }
    if (rc == 0) {
        ok = hipMemcpy(xtraj, dxt, s_xt * sizeof(double), hipMemcpyDeviceToHost) == hipSuccess &&
             hipMemcpy(utraj, dut, s_ut * sizeof(double), hipMemcpyDeviceToHost) == hipSuccess &&
             hipMemcpy(pobj, dpo, batch * sizeof(double), hipMemcpyDeviceToHost) == hipSuccess &&
             hipMemcpy(exit_code, dex, batch * sizeof(int), hipMemcpyDeviceToHost) == hipSuccess &&
             (!info || hipMemcpy(info, dinfo, (size_t)batch * MPCG_INFO_STRIDE * sizeof(int),
                                 hipMemcpyDeviceToHost) == hipSuccess);
        if (!ok) { mpcg::g_err = "device to host copy failed"; rc = -5; }
    }
    (void)hipFree(dpar);
    (void)hipFree(dex);
    return rc;
}

int mpcg_select_best_device(int n_scenes, int n_guesses, int N, const double* xtraj, const double* pobj,
                            const int* exit_code, const double* prev_traj, double w_cons,
                            const unsigned char* consistency_enabled, const unsigned char* previously_selected,
                            double selection_weight, const unsigned char* disabled, int* best, double* objective,
                            void* stream) {
    if (n_scenes <= 0) return 0;
    const int T = 64;
    hipLaunchKernelGGL(mpcg::select_best_kernel, dim3((n_scenes + T - 1) / T), dim3(T), 0, (hipStream_t)stream,
                       n_scenes, n_guesses, N, xtraj, pobj, exit_code, prev_traj, w_cons, consistency_enabled,
                       previously_selected, selection_weight, disabled, best, objective);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        mpcg::g_err = std::string("select_best launch: ") + hipGetErrorString(e);
        return -1;
    }
    return 0;
}

}  // extern "C"
