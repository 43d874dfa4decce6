// mpcg_prepare.h — per-guess solver inputs of one control step on the GPU
// (SURVEY §8f rows 1-3): the host-side module steps that run before every
// Solver::solve() in GuidanceConstraints::optimize, for all scenes x planners
// at once.  Host restatement and semantics: producers.py; ABI: include/mpcg.h
// (mpcg_prepare).
//
// One workgroup (64 lanes) per (scene, planner):
//   warm start   main warm start (or the braking plan, acados_solver_interface.cpp:303-342),
//                guided planners: x, y, psi, v from the guidance trajectory at k dt, k = 1..N-1
//                (initializeSolverWithGuidance, guidance_constraints.cpp:546-570)
//   halfspaces   lane k-1 runs LinearizedConstraints::update for stage k: 3 Douglas-Rachford
//                rounds over all obstacles (linearized_constraints.cpp:130-148), then
//                a = (o - p) / |o - p|, b = a.o - (1e-3 + r_robot) (:84-105);
//                non-guided planner: dummies (a1 = 1, a2 = 0, b = x + 100)
//   ellipsoids   stage 0 dummies, stage k prediction k-1 (ellipsoid_constraints.cpp:34-86)
//   consistency  interpolated previous plan (guidance_constraints.cpp:1073-1133) on stages
//                1..N-2 of the planners with the consistency cost (:986-1023)
// then all lanes stream the N x npar parameter block out with coalesced stores.
// Compiled only into mpcg_prepare.hip, with -ffp-contract=off (no fused
// multiply-adds), and written in the host restatement's operation order, so
// the halfspace, ellipsoid and consistency values agree bit for bit with
// producers.py / the test oracle.
#pragma once
#include <hip/hip_runtime.h>

#include "mpcg.h"

namespace mpcg {

constexpr int PREP_MAX_N = 32;
constexpr int PREP_MAX_OBS = 24;

__device__ __forceinline__ double norm2_rn(double dx, double dy) {
    return __dsqrt_rn(__dadd_rn(__dmul_rn(dx, dx), __dmul_rn(dy, dy)));
}

// ros_tools DouglasRachford: project onto the outside of the disc (c, r) along c -> start
__device__ __forceinline__ void dr_project_disc(double px, double py, double cx, double cy, double r, double sx,
                                                double sy, double& ox, double& oy) {
    if (norm2_rn(__dsub_rn(px, cx), __dsub_rn(py, cy)) < r) {
        const double dx = __dsub_rn(sx, cx), dy = __dsub_rn(sy, cy);
        const double n = norm2_rn(dx, dy);
        ox = __dadd_rn(cx, __dmul_rn(__ddiv_rn(dx, n), r));
        oy = __dadd_rn(cy, __dmul_rn(__ddiv_rn(dy, n), r));
    } else {
        ox = px;
        oy = py;
    }
}

__device__ __forceinline__ void dr_reflect(double px, double py, double cx, double cy, double r, double sx,
                                           double sy, double& ox, double& oy) {
    double qx, qy;
    dr_project_disc(px, py, cx, cy, r, sx, sy, qx, qy);
    ox = __dsub_rn(__dmul_rn(2.0, qx), px);
    oy = __dsub_rn(__dmul_rn(2.0, qy), py);
}

struct PrepLds {
    double warm[PREP_MAX_N + 1][MPCG_NVAR];
    double prev[PREP_MAX_N][2];
    int prev_ok;
};

__global__ __launch_bounds__(64) void prepare_kernel(mpcg_problem pr, int n_scenes, int G, mpcg_scene_io in,
                                                     double* __restrict__ params, double* __restrict__ warm,
                                                     double* __restrict__ xinit, double* __restrict__ prev_out,
                                                     unsigned char* __restrict__ cons_active) {
    __shared__ PrepLds L;
    const int sol = blockIdx.x;
    const int sc = sol / G, g = sol - sc * G;
    if (sc >= n_scenes) return;
    const int lane = threadIdx.x;
    const int N = pr.N, npar = pr.npar, NL = pr.n_lin, NE = pr.n_ell;
    const double dt = pr.dt;
    const double* st = in.state + (size_t)sc * MPCG_NX;
    const bool guided = in.guided && in.guided[(size_t)sc * G + g];
    const double x0 = st[0], y0 = st[1];

    // ---- main warm start (copied into every planner: *solver = *_solver)
    if (in.main_warm) {
        const double* mw = in.main_warm + (size_t)sc * (N + 1) * MPCG_NVAR;
        for (int e = lane; e < (N + 1) * MPCG_NVAR; e += 64) (&L.warm[0][0])[e] = mw[e];
    } else if (lane == 0) {
        // Solver::initializeWithBraking
        double x = st[0], y = st[1], psi = st[2], v = st[3], s = st[4];
        const double a = -fabs(in.deceleration);
        const double c = cos(psi), sn = sin(psi);
        double* w = L.warm[0];
        w[0] = a; w[1] = 0.0; w[2] = x; w[3] = y; w[4] = psi; w[5] = v; w[6] = s;
        for (int k = 1; k <= N; ++k) {
            x = __dadd_rn(x, __dmul_rn(__dmul_rn(v, dt), c));
            y = __dadd_rn(y, __dmul_rn(__dmul_rn(v, dt), sn));
            s = __dadd_rn(s, __dmul_rn(v, dt));
            v = fmax(__dadd_rn(v, __dmul_rn(a, dt)), 0.0);
            w = L.warm[k];
            w[0] = a; w[1] = 0.0; w[2] = x; w[3] = y; w[4] = psi; w[5] = v; w[6] = s;
        }
    }
    __syncthreads();
    // t-mpc.warmstart_with_mpc_solution (guidance_constraints.cpp:335-338): a guided planner whose
    // guidance already existed starts from its own previous output (Solver::initializeWarmstart,
    // acados_solver_interface.cpp:344-376) on top of the copied main warm start
    const bool own_warm = guided && in.warmstart_with_mpc_solution && in.existing_guidance && in.planner_xtraj &&
                          in.planner_utraj && in.existing_guidance[(size_t)sc * G + g];
    if (own_warm) {
        const double* xt = in.planner_xtraj + (size_t)sol * (N + 1) * MPCG_NX;
        const double* ut = in.planner_utraj + (size_t)sol * N * MPCG_NU;
        for (int e = lane; e < (N + 1) * MPCG_NVAR; e += 64) {
            const int k = e / MPCG_NVAR, i = e - k * MPCG_NVAR;
            if (!in.shift_forward) {
                // [out_0 .. out_{N-1}]; x0[N] stays the copied main warm start
                if (k < N) (&L.warm[0][0])[e] = i < MPCG_NU ? ut[k * MPCG_NU + i] : xt[k * MPCG_NX + i - MPCG_NU];
            } else {
                // [state, out_2, ..., out_{N-1}, out_{N-1}, out_{N-1}]; stage 0's inputs: out_1's (the
                // reference reads them out of State's range, as in advance_kernel)
                const int src = k == 0 ? 1 : (k >= N - 1 ? N - 1 : k + 1);
                (&L.warm[0][0])[e] = i < MPCG_NU ? ut[src * MPCG_NU + i]
                                                 : (k == 0 ? st[i - MPCG_NU] : xt[src * MPCG_NX + i - MPCG_NU]);
            }
        }
    }
    __syncthreads();
    // ---- initializeSolverWithGuidance (k = 1..N-1)
    if (guided && !own_warm && lane >= 1 && lane < N) {
        const double* gk = in.guidance + (((size_t)sc * G + g) * (N + 1) + lane) * 4;
        L.warm[lane][2] = gk[0];
        L.warm[lane][3] = gk[1];
        L.warm[lane][4] = atan2(gk[3], gk[2]);
        L.warm[lane][5] = norm2_rn(gk[2], gk[3]);
    }
    __syncthreads();
    // ---- topology halfspaces, lane k-1 <-> stage k
    const int n_obs = NL < NE ? NL : NE;
    const double rr = __dadd_rn(1e-3, in.robot_radius);
    if (guided && lane < N - 1 && n_obs > 0) {
        const int k = lane + 1;
        const double* ob = in.obst + (size_t)sc * NE * N * 5;  // [i][j][5]
        auto opos = [&](int i, double& ox, double& oy) {
            const double* o = ob + ((size_t)i * N + (k - 1)) * 5;
            ox = o[0];
            oy = o[1];
        };
        double px = L.warm[k][2], py = L.warm[k][3];
        double ax, ay;
        opos(0, ax, ay);
        for (int it = 0; it < 3; ++it)
            for (int i = 0; i < n_obs; ++i) {
                double cx, cy, fx, fy, rx, ry;
                opos(i, cx, cy);
                dr_reflect(px, py, ax, ay, rr, px, py, fx, fy);
                dr_reflect(fx, fy, cx, cy, rr, px, py, rx, ry);
                px = __dmul_rn(0.5, __dadd_rn(px, rx));
                py = __dmul_rn(0.5, __dadd_rn(py, ry));
            }
        // straight into the stage's parameter row (the stream below skips these entries): no
        // [N][obstacles] staging array in LDS, whose 18 KB held the kernel at 7 workgroups per CU
        double* Pl = params + ((size_t)sol * N + k) * npar + pr.i_lin0;
        for (int i = 0; i < n_obs; ++i) {
            double ox, oy;
            opos(i, ox, oy);
            const double dx = __dsub_rn(ox, px), dy = __dsub_rn(oy, py);
            const double dist = norm2_rn(dx, dy);
            const double a1 = __ddiv_rn(dx, dist), a2 = __ddiv_rn(dy, dist);
            Pl[3 * i + 0] = a1;
            Pl[3 * i + 1] = a2;
            Pl[3 * i + 2] = __dsub_rn(__dadd_rn(__dmul_rn(a1, ox), __dmul_rn(a2, oy)), rr);
        }
    }
    // ---- previous plan interpolated by the elapsed time
    if (lane == 0) {
        int ok = 0;
        if (in.prev_traj && in.prev_elapsed) {
            const double el = in.prev_elapsed[sc];
            if (isfinite(el)) {
                const int k_shift = (int)floor(__ddiv_rn(el, dt));
                ok = k_shift < N - 1;
            }
        }
        L.prev_ok = ok;
    }
    __syncthreads();
    const bool prev_ok = L.prev_ok != 0;
    if (prev_ok && lane < N) {
        const double* pv = in.prev_traj + (size_t)sc * N * 2;
        const double el = in.prev_elapsed[sc];
        const int k_shift = (int)floor(__ddiv_rn(el, dt));
        const double alpha = __ddiv_rn(__dsub_rn(el, __dmul_rn((double)k_shift, dt)), dt);
        const int src = lane + k_shift;
        for (int c = 0; c < 2; ++c) {
            double v;
            if (src < N - 1) {
                v = __dadd_rn(__dmul_rn(__dsub_rn(1.0, alpha), pv[src * 2 + c]), __dmul_rn(alpha, pv[(src + 1) * 2 + c]));
            } else if (src == N - 1) {
                v = pv[(N - 1) * 2 + c];
            } else {
                const double vel = __ddiv_rn(__dsub_rn(pv[(N - 1) * 2 + c], pv[(N - 2) * 2 + c]), dt);
                const double extra = __dadd_rn(__dmul_rn((double)(src - (N - 1)), dt), __dmul_rn(alpha, dt));
                v = __dadd_rn(pv[(N - 1) * 2 + c], __dmul_rn(vel, extra));
            }
            L.prev[lane][c] = v;
        }
    } else if (lane < N) {
        L.prev[lane][0] = 0.0;
        L.prev[lane][1] = 0.0;
    }
    __syncthreads();
    const bool cons = prev_ok && in.consistency_on && in.consistency_on[(size_t)sc * G + g] && pr.i_cons_w >= 0;

    // ---- stream out the parameter block [N][npar]
    const double* base = in.stage_params + (size_t)sc * npar;
    double* P = params + (size_t)sol * N * npar;
    const int lin0 = pr.i_lin0, ell0 = pr.i_ell0;
    // lane <-> parameter index idx = c0 + lane of every stage: the scene's base row is read once per
    // chunk and each stage's row is one coalesced store (no dependent global load per element)
    for (int c0 = 0; c0 < npar; c0 += 64) {
        const int idx = c0 + lane;
        if (idx >= npar) break;
        const double bv = base[idx];
        const bool is_lin = NL > 0 && idx >= lin0 && idx < lin0 + 3 * NL;
        const bool is_ell = !is_lin && NE > 0 && idx >= ell0 && idx < ell0 + 7 * NE;
        const bool is_cons = !is_lin && !is_ell && pr.i_cons_w >= 0 &&
                             (idx == pr.i_cons_w || idx == pr.i_prev_x || idx == pr.i_prev_y);
        const int li = is_lin ? (idx - lin0) / 3 : 0, lc = is_lin ? (idx - lin0) - 3 * li : 0;
        const int ej = is_ell ? (idx - ell0) / 7 : 0, ec = is_ell ? (idx - ell0) - 7 * ej : 0;
#pragma unroll 4
        for (int k = 0; k < N; ++k) {
            double v = bv;
            if (is_lin) {
                if (guided && k >= 1 && li < n_obs) continue;  // written by the stage's DR lane
                v = lc == 0 ? 1.0 : (lc == 1 ? 0.0 : __dadd_rn(x0, 100.0));
            } else if (is_ell) {
                if (k == 0) {
                    const double dummy[7] = {__dadd_rn(x0, 50.0), __dadd_rn(y0, 50.0), 0.0, 0.0, 0.0, 1.0, 0.1};
                    v = dummy[ec];
                } else {
                    const double* o = in.obst + (((size_t)sc * NE + ej) * N + (k - 1)) * 5;
                    const double* m = in.obst_meta + ((size_t)sc * NE + ej) * 2;
                    v = ec < 5 ? o[ec] : (ec == 5 ? m[1] : m[0]);  // x y psi major minor | chi r
                }
            } else if (is_cons) {
                const bool on = cons && k >= 1 && k <= N - 2;
                v = !on ? 0.0 : (idx == pr.i_cons_w ? in.w_consistency : L.prev[k][idx == pr.i_prev_x ? 0 : 1]);
            }
            P[(size_t)k * npar + idx] = v;
        }
    }
    double* W = warm + (size_t)sol * (N + 1) * MPCG_NVAR;
    for (int e = lane; e < (N + 1) * MPCG_NVAR; e += 64) W[e] = (&L.warm[0][0])[e];
    if (lane < MPCG_NX) xinit[(size_t)sol * MPCG_NX + lane] = st[lane];
    if (g == 0 && prev_out && lane < N) {
        prev_out[((size_t)sc * N + lane) * 2 + 0] = L.prev[lane][0];
        prev_out[((size_t)sc * N + lane) * 2 + 1] = L.prev[lane][1];
    }
    if (cons_active && lane == 0) cons_active[sol] = cons ? 1 : 0;
}

}  // namespace mpcg

namespace mpcg {

// Between two control steps (include/mpcg.h, mpcg_advance); one workgroup per scene.
__global__ __launch_bounds__(64) void advance_kernel(mpcg_problem pr, int n_scenes, int G, mpcg_step_io io,
                                                     double* __restrict__ main_warm, double* __restrict__ prev_traj,
                                                     double* __restrict__ prev_elapsed,
                                                     unsigned char* __restrict__ cons_on,
                                                     unsigned char* __restrict__ prev_sel,
                                                     double* __restrict__ lam_next) {
    const int sc = blockIdx.x;
    if (sc >= n_scenes) return;
    const int lane = threadIdx.x;
    const int N = pr.N, NV = MPCG_NVAR, NXs = MPCG_NX, NUs = MPCG_NU;
    const double dt = pr.dt;
    const int best = io.best[sc];
    const bool feasible = best >= 0;
    const int b = sc * G + (feasible ? best : 0);
    const double* st = io.state_next + (size_t)sc * NXs;
    double* W = main_warm + (size_t)sc * (N + 1) * NV;
    if (feasible) {
        const double* xt = io.xtraj + (size_t)b * (N + 1) * NXs;
        const double* ut = io.utraj + (size_t)b * N * NUs;
        const double* wb = io.warm + (size_t)b * (N + 1) * NV;
        for (int e = lane; e < (N + 1) * NV; e += 64) {
            const int k = e / NV, i = e - k * NV;
            double v;
            if (!io.shift_forward) {
                // [x_0 .. x_{N-1}] of the winner; x0[N] stays the winner's own warm start
                v = k < N ? (i < NUs ? ut[k * NUs + i] : xt[k * NXs + i - NUs]) : wb[N * NV + i];
            } else {
                // [state, out_2, ..., out_{N-1}, out_{N-1}, out_{N-1}] (acados_solver_interface.cpp:346-368);
                // the reference reads the inputs of stage 0 out of State's range: here out_1's inputs
                const int src = k == 0 ? 1 : (k >= N - 1 ? N - 1 : k + 1);
                v = i < NUs ? ut[src * NUs + i] : (k == 0 ? st[i - NUs] : xt[src * NXs + i - NUs]);
            }
            W[e] = v;
        }
        if (lane < N) {
            prev_traj[((size_t)sc * N + lane) * 2 + 0] = xt[lane * NXs + 0];
            prev_traj[((size_t)sc * N + lane) * 2 + 1] = xt[lane * NXs + 1];
        }
    } else {
        if (lane == 0) {
            // Solver::initializeWithBraking(state)
            double x = st[0], y = st[1], psi = st[2], v = st[3], s = st[4];
            const double a = -fabs(io.deceleration);
            const double c = cos(psi), sn = sin(psi);
            for (int k = 0; k <= N; ++k) {
                if (k > 0) {
                    x = __dadd_rn(x, __dmul_rn(__dmul_rn(v, dt), c));
                    y = __dadd_rn(y, __dmul_rn(__dmul_rn(v, dt), sn));
                    s = __dadd_rn(s, __dmul_rn(v, dt));
                    v = fmax(__dadd_rn(v, __dmul_rn(a, dt)), 0.0);
                }
                double* w = W + k * NV;
                w[0] = a; w[1] = 0.0; w[2] = x; w[3] = y; w[4] = psi; w[5] = v; w[6] = s;
            }
        }
        if (lane < N) {
            prev_traj[((size_t)sc * N + lane) * 2 + 0] = 0.0;
            prev_traj[((size_t)sc * N + lane) * 2 + 1] = 0.0;
        }
    }
    if (lane == 0) prev_elapsed[sc] = feasible ? io.elapsed : __longlong_as_double(0x7ff8000000000000LL);
    // consistency / selection flags of the next step
    const bool best_original = feasible && !(io.guided && io.guided[(size_t)sc * G + best]);
    const int sel_topo = feasible ? (io.topology ? io.topology[(size_t)sc * G + best] : best) : -1;
    for (int g = lane; g < G; g += 64) {
        const size_t i = (size_t)sc * G + g;
        const bool guided = io.guided && io.guided[i];
        const int topo = io.topology_next ? io.topology_next[i] : g;
        bool on = false, ps;
        if (feasible) {
            on = guided ? (!best_original && topo == sel_topo) : (io.consistency_on_non_guided && best_original);
            ps = guided && !best_original && topo == sel_topo;
        } else {
            ps = io.previously_selected ? io.previously_selected[i] != 0 : false;
        }
        cons_on[i] = on ? 1 : 0;
        prev_sel[i] = ps ? 1 : 0;
    }
    // carried multipliers of every planner (Solver_acados_reset zeroes them after a failure)
    if (lam_next) {
        const int L = N * (NXs + pr.n_lin + pr.n_ell);
        for (int g = 0; g < G; ++g) {
            const size_t i = (size_t)sc * G + g;
            const bool ok = io.exit_code[i] == 1 && io.lam_out;
            double* dst = lam_next + i * L;
            const double* src = ok ? io.lam_out + i * L : nullptr;
            for (int e = lane; e < L; e += 64) dst[e] = ok ? src[e] : 0.0;
        }
    }
}

}  // namespace mpcg

namespace mpcg {

// ---------------------------------------------------------------------------
// SH-MPC inputs of one control step (include/mpcg.h, mpcg_prepare_scenario):
// ScenarioConstraints::optimize copies the main solver into every parallel
// solver and writes each copy's scenario halfspaces before its solve
// (scenario_constraints.cpp:58-84).  Host restatement and semantics:
// scenario.py (prepare_scenario_host); the reduction of samples to halfspaces
// restates the external scenario_module (parity unpinned there).
//
// One workgroup of 4 wavefronts per (scene, parallel solver):
//   warm start   main warm start or the braking plan (acados_solver_interface.cpp:303-342)
//   halfspaces   wave w reduces stages k = 1 + w, 5 + w, ...: each lane holds the distances
//                of samples lane, lane + 64, ... to the warm-start position p_k in registers
//                and a sorted list of its 4 closest; n_scen DPP wave arg-min rounds over the
//                list heads (distance, then sample index: the stable order of the host's
//                argsort) pick the closest samples, the winning lane pops its head and a
//                lane whose list runs dry rebuilds it from the samples after its last pick; row
//                n = (q - p_k) / max(|q - p_k|, 1e-9), b = n . q - radius
//   stage 0      inactive rows (0, 0, 100)
// then the N x npar parameter block is streamed out with coalesced stores.
// Memory bound: every sample is read once (N-1 stages x M x 16 B per solve).
// ---------------------------------------------------------------------------
constexpr int SCEN_MAX_N = 32, SCEN_MAX_ROWS = 32, SCEN_PER_LANE = 32;  // M <= 64 * 32
constexpr int SCEN_TOPK = 4;  // per-lane candidate list of the arg-min rounds
constexpr double SCEN_DUMMY_B = 100.0;

__device__ __forceinline__ double readlane_dbl(double v, int lane) {
    const int lo = __builtin_amdgcn_readlane(__double2loint(v), lane);
    const int hi = __builtin_amdgcn_readlane(__double2hiint(v), lane);
    return __hiloint2double(hi, lo);
}

// one DPP step of a wave arg-min over (distance, index): lanes outside the
// row mask compare with themselves
template <int CTRL, int ROWS>
__device__ __forceinline__ void dpp_argmin_step(double& d, int& i) {
    const int lo = __builtin_amdgcn_update_dpp(__double2loint(d), __double2loint(d), CTRL, ROWS, 0xf, false);
    const int hi = __builtin_amdgcn_update_dpp(__double2hiint(d), __double2hiint(d), CTRL, ROWS, 0xf, false);
    const int oi = __builtin_amdgcn_update_dpp(i, i, CTRL, ROWS, 0xf, false);
    const double od = __hiloint2double(hi, lo);
    if (od < d || (od == d && oi < i)) {
        d = od;
        i = oi;
    }
}

struct ScenLds {
    double warm[SCEN_MAX_N + 1][MPCG_NU + MPCG_MAX_NX];
    double rows[SCEN_MAX_N][SCEN_MAX_ROWS][3];
};

// PL: samples per lane held in registers (M <= 64 PL); instances 8 / 20 / 32
template <int PL>
__global__ __launch_bounds__(256) void scenario_prepare_kernel(mpcg_problem pr, int n_scenes, int P,
                                                               mpcg_scenario_io in, double* __restrict__ params,
                                                               double* __restrict__ warm,
                                                               double* __restrict__ xinit) {
    __shared__ ScenLds L;
    const int sol = blockIdx.x;
    const int sc = sol / P;
    if (sc >= n_scenes) return;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int N = pr.N, npar = pr.npar, nx = pr.nx, NV = MPCG_NU + nx, NS = pr.n_scen, M = in.n_samples;
    const double dt = pr.dt;
    const double* st = in.state + (size_t)sc * nx;

    // ---- warm start: the main solver's, or Solver::initializeWithBraking (other entries 0)
    if (in.main_warm) {
        const double* mw = in.main_warm + (size_t)sc * (N + 1) * NV;
        for (int e = tid; e < (N + 1) * NV; e += 256) L.warm[e / NV][e % NV] = mw[e];
    } else if (tid == 0) {
        double x = st[0], y = st[1], psi = st[2], v = st[3], s = st[4];
        const double a = -fabs(in.deceleration);
        const double c = cos(psi), sn = sin(psi);
        for (int k = 0; k <= N; ++k) {
            if (k > 0) {
                x = __dadd_rn(x, __dmul_rn(__dmul_rn(v, dt), c));
                y = __dadd_rn(y, __dmul_rn(__dmul_rn(v, dt), sn));
                s = __dadd_rn(s, __dmul_rn(v, dt));
                v = fmax(__dadd_rn(v, __dmul_rn(a, dt)), 0.0);
            }
            double* w = L.warm[k];
            w[0] = a; w[1] = 0.0; w[2] = x; w[3] = y; w[4] = psi; w[5] = v; w[6] = s;
            for (int i = 7; i < NV; ++i) w[i] = 0.0;
        }
    }
    __syncthreads();

    // ---- sample -> halfspace reduction, one stage per wave at a time
    const double INF = __longlong_as_double(0x7ff0000000000000LL);
    constexpr int BIG = 0x7fffffff;
    for (int k = 1 + wave; k < N; k += 4) {
        const double* q = in.samples + ((size_t)sol * N + k) * (size_t)M * 2;
        const double rx = L.warm[k][2], ry = L.warm[k][3];
        double dist[PL];
        int left = 0;  // samples of this lane not picked yet
#pragma unroll
        for (int j = 0; j < PL; ++j) {
            const int i = lane + 64 * j;
            double d = INF;
            if (i < M) {
                d = norm2_rn(__dsub_rn(q[2 * i], rx), __dsub_rn(q[2 * i + 1], ry));
                ++left;
            }
            dist[j] = d;
        }
        // each lane keeps its SCEN_TOPK closest samples sorted by (distance, index); the
        // list is rebuilt from the samples after the last pick when it runs dry
        double td[SCEN_TOPK];
        int ti[SCEN_TOPK];
        double lastd = -1.0;
        int lasti = -1;
        auto rebuild = [&]() {
#pragma unroll
            for (int t = 0; t < SCEN_TOPK; ++t) { td[t] = INF; ti[t] = BIG; }
#pragma unroll
            for (int j = 0; j < PL; ++j) {
                double x = dist[j];
                int xi = lane + 64 * j;
                if (!(x > lastd || (x == lastd && xi > lasti))) continue;
#pragma unroll
                for (int t = 0; t < SCEN_TOPK; ++t)
                    if (x < td[t]) {  // strict: equal distances keep the lower index first
                        const double y = td[t];
                        const int yi = ti[t];
                        td[t] = x; ti[t] = xi;
                        x = y; xi = yi;
                    }
            }
        };
        rebuild();
        // lane r keeps round r's pick; the rows are formed after the rounds, one per lane (the
        // same operations as forming each in lane 0 inside its round)
        double pick_d = 0.0;
        int pick_i = BIG;
        for (int r = 0; r < NS; ++r) {
            // wave arg-min of the list heads over (distance, index) through DPP
            double bd = td[0];
            int bi = ti[0];
            dpp_argmin_step<0xB1, 0xf>(bd, bi);   // quad_perm [1,0,3,2]
            dpp_argmin_step<0x4E, 0xf>(bd, bi);   // quad_perm [2,3,0,1]
            dpp_argmin_step<0x124, 0xf>(bd, bi);  // row_ror:4
            dpp_argmin_step<0x128, 0xf>(bd, bi);  // row_ror:8
            dpp_argmin_step<0x142, 0xa>(bd, bi);  // row_bcast:15
            dpp_argmin_step<0x143, 0xc>(bd, bi);  // row_bcast:31
            bd = readlane_dbl(bd, 63);
            bi = __builtin_amdgcn_readlane(bi, 63);
            const bool found = bi < M;
            if (found && lane == (bi & 63)) {
                lastd = td[0];
                lasti = ti[0];
                --left;
#pragma unroll
                for (int t = 0; t + 1 < SCEN_TOPK; ++t) { td[t] = td[t + 1]; ti[t] = ti[t + 1]; }
                td[SCEN_TOPK - 1] = INF;
                ti[SCEN_TOPK - 1] = BIG;
            }
            if (__any(left > 0 && ti[0] == BIG)) {
                if (left > 0 && ti[0] == BIG) rebuild();
            }
            if (lane == r) {
                pick_d = bd;
                pick_i = bi;
            }
        }
        if (lane < NS) {
            double a1 = 0.0, a2 = 0.0, b = 0.0;
            if (pick_i < M) {
                const double qx = q[2 * pick_i], qy = q[2 * pick_i + 1];
                const double dn = fmax(pick_d, 1e-9);
                a1 = __ddiv_rn(__dsub_rn(qx, rx), dn);
                a2 = __ddiv_rn(__dsub_rn(qy, ry), dn);
                b = __dsub_rn(__dadd_rn(__dmul_rn(a1, qx), __dmul_rn(a2, qy)), in.radius);
            }
            L.rows[k][lane][0] = a1;
            L.rows[k][lane][1] = a2;
            L.rows[k][lane][2] = b;
        }
    }
    __syncthreads();

    // ---- stream out the parameter block, warm start and xinit
    const double* base = in.stage_params + (size_t)sc * npar;
    double* Pp = params + (size_t)sol * N * npar;
    const int s0 = pr.i_scen0;
    for (int e = tid; e < N * npar; e += 256) {
        const int k = e / npar, idx = e - k * npar;
        double v = base[idx];
        if (idx >= s0 && idx < s0 + 3 * NS) {
            const int i = (idx - s0) / 3, c = (idx - s0) - 3 * i;
            v = k == 0 ? (c == 2 ? SCEN_DUMMY_B : 0.0) : L.rows[k][i][c];
        }
        Pp[e] = v;
    }
    double* W = warm + (size_t)sol * (N + 1) * NV;
    for (int e = tid; e < (N + 1) * NV; e += 256) W[e] = L.warm[e / NV][e % NV];
    if (tid < nx) xinit[(size_t)sol * nx + tid] = st[tid];
}

}  // namespace mpcg
