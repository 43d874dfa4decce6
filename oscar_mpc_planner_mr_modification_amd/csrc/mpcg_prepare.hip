// mpcg_prepare.hip — entry point of the per-guess input producers
// (mpcg_prepare, include/mpcg.h).  Compiled on its own with
// -ffp-contract=off: the producers must agree bit for bit with the host
// restatement (producers.py), so no multiply-add may be fused here, while the
// solve kernels in mpcg_kernels.hip keep contraction on.
#include <hip/hip_runtime.h>

#include <string>

#include "mpcg.h"
#include "mpcg_prepare.h"

namespace mpcg {
extern thread_local std::string g_err;  // defined in mpcg_kernels.hip
}

extern "C" {

int mpcg_prepare(const mpcg_problem* pr, int n_scenes, int n_guesses, const mpcg_scene_io* in, double* params,
                 double* warm, double* xinit, double* prev_interp, unsigned char* consistency_active, void* stream) {
    if (!pr || !in || n_scenes < 0 || n_guesses < 1 || !params || !warm || !xinit || !in->stage_params ||
        !in->state || (pr->n_ell > 0 && (!in->obst || !in->obst_meta)) || !in->guidance) {
        mpcg::g_err = "mpcg_prepare: invalid arguments";
        return -1;
    }
    if (pr->nx != MPCG_NX || pr->n_scen != 0) {
        mpcg::g_err = "mpcg_prepare: the T-MPC producers need the 5-state model without scenario rows";
        return -2;
    }
    const int n_obs = pr->n_lin < pr->n_ell ? pr->n_lin : pr->n_ell;
    if (pr->N > mpcg::PREP_MAX_N || n_obs > mpcg::PREP_MAX_OBS || pr->N < 2) {
        mpcg::g_err = "mpcg_prepare: N or the obstacle count exceeds the kernel's limits";
        return -2;
    }
    if (n_scenes == 0) return 0;
    hipLaunchKernelGGL(mpcg::prepare_kernel, dim3(n_scenes * n_guesses), dim3(64), 0, (hipStream_t)stream, *pr,
                       n_scenes, n_guesses, *in, params, warm, xinit, prev_interp, consistency_active);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        mpcg::g_err = std::string("prepare launch: ") + hipGetErrorString(e);
        return -1;
    }
    return 0;
}

int mpcg_advance(const mpcg_problem* pr, int n_scenes, int n_guesses, const mpcg_step_io* io, double* main_warm_next,
                 double* prev_traj_next, double* prev_elapsed_next, unsigned char* consistency_on_next,
                 unsigned char* previously_selected_next, double* lam_next, void* stream) {
    if (!pr || !io || n_scenes < 0 || n_guesses < 1 || !io->best || !io->exit_code || !io->xtraj || !io->utraj ||
        !io->warm || !io->state_next || !main_warm_next || !prev_traj_next || !prev_elapsed_next ||
        !consistency_on_next || !previously_selected_next) {
        mpcg::g_err = "mpcg_advance: invalid arguments";
        return -1;
    }
    if (pr->nx != MPCG_NX) {
        mpcg::g_err = "mpcg_advance: the T-MPC step bookkeeping needs the 5-state model";
        return -2;
    }
    if (n_scenes == 0) return 0;
    hipLaunchKernelGGL(mpcg::advance_kernel, dim3(n_scenes), dim3(64), 0, (hipStream_t)stream, *pr, n_scenes,
                       n_guesses, *io, main_warm_next, prev_traj_next, prev_elapsed_next, consistency_on_next,
                       previously_selected_next, lam_next);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        mpcg::g_err = std::string("advance launch: ") + hipGetErrorString(e);
        return -1;
    }
    return 0;
}

int mpcg_prepare_scenario(const mpcg_problem* pr, int n_scenes, int n_solvers, const mpcg_scenario_io* in,
                          double* params, double* warm, double* xinit, void* stream) {
    if (!pr || !in || n_scenes < 0 || n_solvers < 1 || !params || !warm || !xinit || !in->stage_params ||
        !in->state || !in->samples) {
        mpcg::g_err = "mpcg_prepare_scenario: invalid arguments";
        return -1;
    }
    if (pr->n_scen < 1 || pr->i_scen0 < 0 || pr->nx < 5 || pr->nx > MPCG_MAX_NX || pr->N < 2 ||
        pr->N > mpcg::SCEN_MAX_N || pr->n_scen > mpcg::SCEN_MAX_ROWS || in->n_samples < 1 ||
        in->n_samples > 64 * mpcg::SCEN_PER_LANE) {
        mpcg::g_err = "mpcg_prepare_scenario: needs scenario rows, N <= 32, n_scen <= 32 and 1..2048 samples";
        return -2;
    }
    if (n_scenes == 0) return 0;
    const int M = in->n_samples;
    auto kern = M <= 64 * 8 ? mpcg::scenario_prepare_kernel<8>
                            : (M <= 64 * 20 ? mpcg::scenario_prepare_kernel<20> : mpcg::scenario_prepare_kernel<32>);
    hipLaunchKernelGGL(kern, dim3(n_scenes * n_solvers), dim3(256), 0, (hipStream_t)stream, *pr, n_scenes, n_solvers,
                       *in, params, warm, xinit);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        mpcg::g_err = std::string("scenario prepare launch: ") + hipGetErrorString(e);
        return -1;
    }
    return 0;
}

}  // extern "C"
