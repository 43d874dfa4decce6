"""Host-side description of the C ABI (include/mpcg.h): the `mpcg_problem`
struct, the solver options restated from the reference's acados generator
and the unicycle bounds.  Importable without a GPU and without loading
libmpcg.so (the CPU tests use it)."""
from __future__ import annotations

import ctypes as C

import numpy as np

from .layouts import Layout

NX, NU, NVAR = 5, 2, 7   # the T-MPC unicycle; the SH-MPC slack model has nx 6, the C3 bicycle nu 3 / nx 6
MAX_NX, MAX_NU = 6, 3
INFO_STRIDE = 4
STATS_STRIDE = 4   # NLP residuals: stationarity, res_eq, inequality violation, complementarity


class MpcgProblem(C.Structure):
    """Mirror of `mpcg_problem` (include/mpcg.h)."""
    _fields_ = [
        ("N", C.c_int), ("npar", C.c_int),
        ("n_lin", C.c_int), ("n_ell", C.c_int), ("n_seg", C.c_int),
        ("i_w_acc", C.c_int), ("i_w_ang", C.c_int), ("i_w_vel", C.c_int), ("i_v_ref", C.c_int),
        ("i_w_contour", C.c_int), ("i_w_lag", C.c_int),
        ("i_spline0", C.c_int),
        ("i_cons_w", C.c_int), ("i_prev_x", C.c_int), ("i_prev_y", C.c_int),
        ("i_lin0", C.c_int),
        ("i_disc_r", C.c_int), ("i_disc_off", C.c_int),
        ("i_ell0", C.c_int),
        ("n_scen", C.c_int), ("i_scen0", C.c_int), ("i_w_slack", C.c_int), ("nx", C.c_int),
        ("dt", C.c_double), ("rk_steps", C.c_int),
        ("lbu", C.c_double * MAX_NU), ("ubu", C.c_double * MAX_NU),
        ("lbx", C.c_double * MAX_NX), ("ubx", C.c_double * MAX_NX),
        ("sqp_iters", C.c_int), ("qp_tol", C.c_double), ("qp_iter_max", C.c_int),
        ("reg_eps", C.c_double), ("qp_mu0", C.c_double), ("qp_thr0", C.c_double),
        ("res_eq_fail", C.c_double),
        ("nu", C.c_int), ("model", C.c_int), ("i_w_tangle", C.c_int), ("i_w_tcont", C.c_int),
        ("qp_warm_start", C.c_int), ("qp_ws_thr", C.c_double),
        # ABI 6
        ("nlp_solver", C.c_int), ("nlp_max_iter", C.c_int), ("nlp_tol", C.c_double), ("qp_warm_first", C.c_int),
        # ABI 7
        ("qp_t_min", C.c_double), ("qp_mu_max", C.c_double),
        # ABI 8: the interior point's profile
        ("qp_profile", C.c_int), ("qp_init_move", C.c_int), ("qp_cond_pred_corr", C.c_int),
        ("qp_itref_corr_max", C.c_int), ("qp_sigma_clip", C.c_int), ("qp_maxit_first", C.c_int),
        # ABI 9: BLASFEO's rule for a non-positive Cholesky pivot
        ("qp_pivot_zero", C.c_int),
    ]


# acados options restated (generate_acados_solver.py:88-173: qp_tol, qp_solver_iter_max, MIRROR
# epsilon, tol) + the IPM's cold start; qp_warm_start=2 (the reference's qp_solver_warm_start, :173)
# with acados' warm_start_first_qp off (qp_warm_first=0) starts every SQP-RTI QP cold and the
# later QPs of a full SQP call (solver_type="SQP") warm (DESIGN.md §2 "QP start")
DEFAULT_OPTIONS = dict(qp_tol=1e-5, qp_iter_max=50, reg_eps=1e-4, res_eq_fail=1e-2,
                       qp_warm_start=2, qp_ws_thr=0.1, qp_warm_first=0, solver_type="SQP_RTI", nlp_max_iter=100,
                       nlp_tol=1e-2, qp_profile="hpipm")
# The interior point's profiles (mpcg_problem_set_qp_profile in libmpcg.so writes the
# same values): "hpipm", the default, restates HPIPM's BALANCE mode as acados configures it (the
# reference sets four QP options and leaves the rest at acados' defaults, generate_acados_solver.py:162-173);
# "robust" is round 4's interior point.  Any field can be overridden by name.
QP_PROFILES = {
    "hpipm": dict(qp_profile_id=0, qp_mu0=10.0, qp_thr0=0.1, qp_t_min=1e-16, qp_mu_max=0.0, qp_init_move=1,
                  qp_cond_pred_corr=1, qp_itref_corr_max=2, qp_sigma_clip=0, qp_maxit_first=1, qp_pivot_zero=1),
    "robust": dict(qp_profile_id=1, qp_mu0=1.0, qp_thr0=1.0, qp_t_min=1e-12, qp_mu_max=1e8, qp_init_move=0,
                   qp_cond_pred_corr=0, qp_itref_corr_max=0, qp_sigma_clip=1, qp_maxit_first=0, qp_pivot_zero=0),
}
QP_FIELDS = ("qp_mu0", "qp_thr0", "qp_t_min", "qp_mu_max", "qp_init_move", "qp_cond_pred_corr", "qp_itref_corr_max",
             "qp_sigma_clip", "qp_maxit_first", "qp_pivot_zero")
NLP_SOLVER = {"SQP_RTI": 0, "SQP": 1}
# ContouringSecondOrderUnicycleModel bounds (solver_model.py:204-205), z = [a, w, x, y, psi, v, s]
UNICYCLE_LB = (-2.0, -0.8, -2000.0, -2000.0, -4 * np.pi, -0.01, -1.0)
UNICYCLE_UB = (2.0, 0.8, 2000.0, 2000.0, 4 * np.pi, 3.0, 10000.0)


def problem_from_layout(layout: Layout, **opts) -> MpcgProblem:
    o = dict(DEFAULT_OPTIONS)
    o.update(opts)
    pr = MpcgProblem()
    pr.N, pr.npar = layout.N, layout.npar
    pr.n_lin, pr.n_ell, pr.n_seg = layout.n_lin, layout.n_ell, layout.n_seg
    pr.n_scen = layout.n_scen
    pr.nx = nx = layout.nx
    pr.nu = nu = layout.nu
    pr.model = layout.model_id
    for k, v in layout.index_struct().items():
        setattr(pr, k, v)
    pr.dt = o.get("dt", layout.dt)
    pr.rk_steps = o.get("rk_steps", layout.rk_steps)
    lb, ub = o.get("lb", layout.lb), o.get("ub", layout.ub)
    for i in range(nu):
        pr.lbu[i], pr.ubu[i] = lb[i], ub[i]
    for i in range(nx):
        pr.lbx[i], pr.ubx[i] = lb[nu + i], ub[nu + i]
    pr.sqp_iters = o.get("sqp_iters", layout.sqp_iters)
    pr.qp_tol = o["qp_tol"]
    pr.qp_iter_max = o["qp_iter_max"]
    pr.reg_eps = o["reg_eps"]
    pr.res_eq_fail = o["res_eq_fail"]
    pr.qp_warm_start = o["qp_warm_start"]
    pr.qp_ws_thr = o["qp_ws_thr"]
    pr.qp_warm_first = o["qp_warm_first"]
    pr.nlp_solver = NLP_SOLVER[o["solver_type"]]
    pr.nlp_max_iter = o["nlp_max_iter"]
    pr.nlp_tol = o["nlp_tol"]
    prof = QP_PROFILES[o["qp_profile"]]
    pr.qp_profile = prof["qp_profile_id"]
    for f in QP_FIELDS:
        setattr(pr, f, o.get(f, prof[f]))
    return pr


def needs_full(pr: MpcgProblem) -> bool:
    """whether a launch of `pr` runs the FULL kernel variant whatever buffers it is given
    (mpcg_sqp.h needs_full: a full SQP call, or a first QP that starts warm); otherwise the
    lean variant runs unless the call passes QP memory or a stats buffer"""
    return pr.nlp_solver == NLP_SOLVER["SQP"] or (pr.qp_warm_start == 2 and bool(pr.qp_warm_first))


class MpcgIo(C.Structure):
    """Mirror of `mpcg_io` (include/mpcg.h)."""
    _fields_ = [("params", C.c_void_p), ("warm", C.c_void_p), ("xinit", C.c_void_p), ("lam_in", C.c_void_p),
                ("xtraj", C.c_void_p), ("utraj", C.c_void_p), ("pobj", C.c_void_p),
                ("exit_code", C.c_void_p), ("info", C.c_void_p), ("lam_out", C.c_void_p),
                ("qp_in", C.c_void_p), ("qp_out", C.c_void_p), ("stats", C.c_void_p)]


class MpcgSceneIo(C.Structure):
    """Mirror of `mpcg_scene_io` (include/mpcg.h)."""
    _fields_ = [("stage_params", C.c_void_p), ("state", C.c_void_p), ("obst", C.c_void_p),
                ("obst_meta", C.c_void_p), ("guidance", C.c_void_p), ("guided", C.c_void_p),
                ("main_warm", C.c_void_p), ("prev_traj", C.c_void_p), ("prev_elapsed", C.c_void_p),
                ("consistency_on", C.c_void_p), ("robot_radius", C.c_double), ("w_consistency", C.c_double),
                ("deceleration", C.c_double),
                # ABI 6: t-mpc.warmstart_with_mpc_solution
                ("planner_xtraj", C.c_void_p), ("planner_utraj", C.c_void_p), ("existing_guidance", C.c_void_p),
                ("warmstart_with_mpc_solution", C.c_int), ("shift_forward", C.c_int)]


class MpcgStepIo(C.Structure):
    """Mirror of `mpcg_step_io` (include/mpcg.h)."""
    _fields_ = [("best", C.c_void_p), ("exit_code", C.c_void_p), ("xtraj", C.c_void_p), ("utraj", C.c_void_p),
                ("warm", C.c_void_p), ("lam_out", C.c_void_p), ("state_next", C.c_void_p), ("guided", C.c_void_p),
                ("topology", C.c_void_p), ("topology_next", C.c_void_p), ("previously_selected", C.c_void_p),
                ("shift_forward", C.c_int), ("consistency_on_non_guided", C.c_int), ("elapsed", C.c_double),
                ("deceleration", C.c_double)]


class MpcgScenarioIo(C.Structure):
    """Mirror of `mpcg_scenario_io` (include/mpcg.h)."""
    _fields_ = [("stage_params", C.c_void_p), ("state", C.c_void_p), ("main_warm", C.c_void_p),
                ("samples", C.c_void_p), ("n_samples", C.c_int), ("radius", C.c_double),
                ("deceleration", C.c_double)]


ABI_VERSION = 9
EXPORTS = ("mpcg_abi_version", "mpcg_last_error", "mpcg_supported", "mpcg_num_h", "mpcg_lam_size", "mpcg_qp_mem_size",
           "mpcg_problem_from_map", "mpcg_problem_from_map_model", "mpcg_solve", "mpcg_context_create", "mpcg_context_destroy",
           "mpcg_context_solve", "mpcg_context_set_iterations", "mpcg_solve_batch_device", "mpcg_solve_batch_host", "mpcg_select_best_device", "mpcg_prepare", "mpcg_advance",
           "mpcg_prepare_scenario", "mpcg_select_lowest_cost_device", "mpcg_winner_records_device",
           "mpcg_release_stream_workspace",
           "mpcg_instance_traits", "mpcg_problem_set_qp_profile")


