"""ctypes binding of the CPU oracle (oracle/libmpcg_oracle.so, nx 5;
oracle/libmpcg_oracle_slack.so, nx 6 — the C5 slack model;
oracle/libmpcg_oracle_bicycle.so, nu 3 / nx 6 — the C3 curvature-aware bicycle).

TEST INFRASTRUCTURE ONLY — imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, never by the product package.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "libmpcg_oracle.so")
LIB_SLACK = os.path.join(HERE, "libmpcg_oracle_slack.so")
LIB_BICYCLE = os.path.join(HERE, "libmpcg_oracle_bicycle.so")
LIBS = {"unicycle": LIB, "unicycle_slack": LIB_SLACK, "bicycle_ca": LIB_BICYCLE}
MODEL_DIMS = {"unicycle": (5, 2), "unicycle_slack": (6, 2), "bicycle_ca": (6, 3)}
# arithmetic-form builds (mpcg_oracle.c "Arithmetic forms"): the default builds use HPIPM's /
# BLASFEO's forms; "_literal" (-DORC_LITERAL: divisions and row-order sums) is the second
# kernel-agnostic build of the rounding-sensitivity record; "_kernel" (-DORC_KERNEL_FORMS: the
# GPU kernel's forms and lane association) is diagnostic only
FORMS = ("hpipm", "literal", "kernel")
for _m, _stem in (("unicycle", "libmpcg_oracle"), ("unicycle_slack", "libmpcg_oracle_slack"),
                  ("bicycle_ca", "libmpcg_oracle_bicycle")):
    for _forms in FORMS[1:]:
        LIBS[_m + "_" + _forms] = os.path.join(HERE, f"{_stem}_{_forms}.so")
        MODEL_DIMS[_m + "_" + _forms] = MODEL_DIMS[_m]

ORC_MAX_NU, ORC_MAX_NX = 3, 6

# The interior point's profiles (the same values as the product's
# mpcg_problem_set_qp_profile): "hpipm" restates HPIPM's BALANCE mode as acados configures it
# (the reference leaves every QP option but four at acados' defaults,
# generate_acados_solver.py:162-173), "robust" is round 4's algorithm.
QP_PROFILES = {
    "hpipm": dict(qp_mu0=10.0, qp_thr0=0.1, qp_t_min=1e-16, qp_mu_max=0.0, qp_init_move=1, qp_cond_pred_corr=1,
                  qp_itref_corr_max=2, qp_sigma_clip=0, qp_maxit_first=1, qp_ric_alg=1, qp_pivot_zero=1,
                  qp_lq_fact=0),
    "robust": dict(qp_mu0=1.0, qp_thr0=1.0, qp_t_min=1e-12, qp_mu_max=1e8, qp_init_move=0, qp_cond_pred_corr=0,
                   qp_itref_corr_max=0, qp_sigma_clip=1, qp_maxit_first=0, qp_ric_alg=0, qp_pivot_zero=0,
                   qp_lq_fact=0),
}


class OrcProblem(C.Structure):
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
        ("lbu", C.c_double * ORC_MAX_NU), ("ubu", C.c_double * ORC_MAX_NU),
        ("lbx", C.c_double * ORC_MAX_NX), ("ubx", C.c_double * ORC_MAX_NX),
        ("sqp_iters", C.c_int), ("qp_tol", C.c_double), ("qp_iter_max", C.c_int),
        ("reg_eps", C.c_double), ("qp_mu0", C.c_double), ("qp_thr0", C.c_double),
        ("res_eq_fail", C.c_double),
        ("i_w_tangle", C.c_int), ("i_w_tcont", C.c_int), ("nu", C.c_int),
        ("qp_warm_start", C.c_int), ("qp_ws_thr", C.c_double),
        ("nlp_solver", C.c_int), ("nlp_max_iter", C.c_int), ("nlp_tol", C.c_double), ("qp_warm_first", C.c_int),
        ("qp_t_min", C.c_double), ("qp_mu_max", C.c_double),
        ("qp_init_move", C.c_int), ("qp_cond_pred_corr", C.c_int), ("qp_itref_corr_max", C.c_int),
        ("qp_sigma_clip", C.c_int), ("qp_maxit_first", C.c_int),
        ("qp_ric_alg", C.c_int), ("qp_pivot_zero", C.c_int), ("qp_lq_fact", C.c_int),
    ]


class OrcInfo(C.Structure):
    _fields_ = [("sqp_iter", C.c_int), ("qp_iter_total", C.c_int), ("qp_status", C.c_int),
                ("res_eq", C.c_double), ("pobj", C.c_double),
                ("res_stat", C.c_double), ("res_ineq", C.c_double), ("res_comp", C.c_double),
                ("qp_maxiter", C.c_int), ("qp_center", C.c_int), ("qp_itref", C.c_int), ("qp_lq", C.c_int)]


def build(force: bool = False) -> str:
    srcs = [os.path.join(HERE, f) for f in ("mpcg_oracle.c", "mpcg_oracle.h", "orc_bicycle_ca.inc", "Makefile")]
    newest = max(os.path.getmtime(f) for f in srcs)
    if force or any(not os.path.exists(x) or os.path.getmtime(x) < newest for x in LIBS.values()):
        subprocess.run(["make", "-C", HERE, "-s"], check=True)
    return LIB


_libs = {}


def lib(model: str = "unicycle"):
    if isinstance(model, int):  # legacy: nx 5 / 6 of the unicycle models
        model = "unicycle" if model == 5 else "unicycle_slack"
    if model not in _libs:
        path = LIBS[model]
        if not os.path.exists(path):
            build()
        L = C.CDLL(path)
        dp = np.ctypeslib.ndpointer(dtype=np.float64, flags="C_CONTIGUOUS")
        ip = np.ctypeslib.ndpointer(dtype=np.int32, flags="C_CONTIGUOUS")
        P = C.POINTER(OrcProblem)
        L.orc_stage_cost.argtypes = [P, dp, dp, dp, dp, dp]
        L.orc_num_h.argtypes = [P]
        L.orc_num_h.restype = C.c_int
        L.orc_stage_constraints.argtypes = [P, dp, dp, dp, dp, dp]
        L.orc_h_bounds.argtypes = [P, dp, dp]
        L.orc_dynamics.argtypes = [dp, dp, dp, dp]
        L.orc_erk4.argtypes = [P, dp, dp, dp, dp, C.c_void_p, C.c_void_p]
        L.orc_discrete.argtypes = [P, dp, C.c_void_p, dp, dp, dp, C.c_void_p, C.c_void_p]
        L.orc_stage_cost_k.argtypes = [P, C.c_int, dp, dp, dp, dp, dp]
        L.orc_ca_update.argtypes = [P, dp, dp, dp, dp, dp, dp]
        L.orc_mirror.argtypes = [C.c_int, dp, C.c_double]
        L.orc_solve.argtypes = [P, dp, dp, dp, dp, dp, C.POINTER(OrcInfo)]
        L.orc_solve.restype = C.c_int
        L.orc_solve_batch.argtypes = [P, C.c_int, dp, dp, dp, dp, dp, dp, ip, ip, C.c_int]
        vp = C.c_void_p
        L.orc_solve_batch_ex.argtypes = [P, C.c_int, dp, dp, dp, vp, dp, dp, dp, ip, ip, vp, C.c_int]
        L.orc_solve_batch_full.argtypes = [P, C.c_int, dp, dp, dp, vp, vp, dp, dp, ip, vp, vp, vp, C.c_int]
        L.orc_qp_mem_size.argtypes = [P]
        L.orc_qp_mem_size.restype = C.c_int
        L.orc_nx.restype = C.c_int
        L.orc_nu.restype = C.c_int
        if (L.orc_nx(), L.orc_nu()) != MODEL_DIMS[model]:
            raise RuntimeError(f"{path} is built for nx={L.orc_nx()} nu={L.orc_nu()}, expected {MODEL_DIMS[model]}")
        _libs[model] = L
    return _libs[model]


def problem_from_layout(layout, **opts) -> OrcProblem:
    from_idx = layout.index_struct()
    pr = OrcProblem()
    pr.N = layout.N
    pr.npar = layout.npar
    pr.n_lin, pr.n_ell, pr.n_seg = layout.n_lin, layout.n_ell, layout.n_seg
    for k, v in from_idx.items():
        setattr(pr, k, v)
    pr.dt = opts.get("dt", layout.dt)
    pr.rk_steps = opts.get("rk_steps", layout.rk_steps)
    pr.n_scen = getattr(layout, "n_scen", 0)
    pr.nx = nx = layout.nx
    pr.nu = nu = layout.nu
    lb = opts.get("lb", layout.lb)
    ub = opts.get("ub", layout.ub)
    for i in range(nu):
        pr.lbu[i], pr.ubu[i] = lb[i], ub[i]
    for i in range(nx):
        pr.lbx[i], pr.ubx[i] = lb[nu + i], ub[nu + i]
    pr.sqp_iters = opts.get("sqp_iters", layout.sqp_iters)
    pr.qp_tol = opts.get("qp_tol", 1e-5)
    pr.qp_iter_max = opts.get("qp_iter_max", 50)
    pr.reg_eps = opts.get("reg_eps", 1e-4)
    prof = QP_PROFILES[opts.get("qp_profile", "hpipm")]
    pr.qp_mu0 = opts.get("qp_mu0", prof["qp_mu0"])
    pr.qp_thr0 = opts.get("qp_thr0", prof["qp_thr0"])
    pr.res_eq_fail = opts.get("res_eq_fail", 1e-2)
    # QP start as the reference configures it: qp_solver_warm_start 2 (generate_acados_solver.py:173)
    # with warm_start_first_qp off -- every SQP-RTI QP starts cold; qp_warm_first=1 warm-starts the
    # first QP of each call too (DESIGN.md §2 "QP start")
    pr.qp_warm_start = opts.get("qp_warm_start", 2)
    pr.qp_ws_thr = opts.get("qp_ws_thr", 0.1)
    pr.qp_warm_first = opts.get("qp_warm_first", 0)
    # solver_type: "SQP_RTI" (default) or "SQP" (one acados SQP call, tol 1e-2, max_iter 100)
    pr.nlp_solver = {"SQP_RTI": 0, "SQP": 1}[opts.get("solver_type", "SQP_RTI")]
    pr.nlp_max_iter = opts.get("nlp_max_iter", 100)
    pr.nlp_tol = opts.get("nlp_tol", 1e-2)
    # floor of t and lambda after every interior-point step, the divergence test (<= 0: none) and
    # the structural switches of the profile
    for f in ("qp_t_min", "qp_mu_max", "qp_init_move", "qp_cond_pred_corr", "qp_itref_corr_max", "qp_sigma_clip",
              "qp_maxit_first", "qp_ric_alg", "qp_pivot_zero", "qp_lq_fact"):
        setattr(pr, f, opts.get(f, prof[f]))
    return pr


class Oracle:
    """Thin wrapper: stage functions and full solves on numpy arrays."""

    def __init__(self, layout, literal=False, forms="hpipm", **opts):
        """forms: "hpipm" (default: HPIPM's / BLASFEO's arithmetic forms), "literal" (the second
        kernel-agnostic build; literal=True is the same) or "kernel" (diagnostic: the GPU kernel's
        forms) -- rounding-sensitivity records only"""
        if literal:
            forms = "literal"
        assert forms in FORMS, forms
        self.forms = forms
        self.layout = layout
        self.pr = problem_from_layout(layout, **opts)
        self.nx = nx = layout.nx
        self.nu = layout.nu
        self.nz = nx + self.nu
        self.L = lib(layout.model + ("" if forms == "hpipm" else "_" + forms))

    @property
    def nh(self):
        return self.L.orc_num_h(C.byref(self.pr))

    def stage_cost(self, z, p):
        nz = self.nz
        out = np.zeros(1)
        g = np.zeros(nz)
        H = np.zeros(nz * nz)
        self.L.orc_stage_cost(C.byref(self.pr), np.ascontiguousarray(z, float), np.ascontiguousarray(p, float), out, g, H)
        return out[0], g, H.reshape(nz, nz)

    def stage_cost_k(self, k, z, p):
        nz = self.nz
        out, g, H = np.zeros(1), np.zeros(nz), np.zeros(nz * nz)
        self.L.orc_stage_cost_k(C.byref(self.pr), k, np.ascontiguousarray(z, float), np.ascontiguousarray(p, float),
                                out, g, H)
        return out[0], g, H.reshape(nz, nz)

    def ca_update(self, z, I, p):
        """C3 CA spline update g(z, I); gradient / Hessian over (z, I)."""
        n = self.nz + 5
        out, g, H = np.zeros(1), np.zeros(n), np.zeros(n * n)
        self.L.orc_ca_update(C.byref(self.pr), np.ascontiguousarray(z, float), np.ascontiguousarray(I, float),
                             np.ascontiguousarray(p, float), out, g, H)
        return out[0], g, H.reshape(n, n)

    def discrete(self, z, p, adj=None):
        """one shooting interval with the stage parameters: x+, A, B (and the adjoint Hessian)"""
        nx, nu, nz = self.nx, self.nu, self.nz
        xn, A, B, H = np.zeros(nx), np.zeros(nx * nx), np.zeros(nx * nu), np.zeros(nz * nz)
        p = np.ascontiguousarray(p, float)
        a = None if adj is None else np.ascontiguousarray(adj, float)
        self.L.orc_discrete(C.byref(self.pr), np.ascontiguousarray(z, float), p.ctypes.data_as(C.c_void_p), xn, A, B,
                            None if a is None else a.ctypes.data_as(C.c_void_p),
                            None if a is None else H.ctypes.data_as(C.c_void_p))
        if adj is None:
            return xn, A.reshape(nx, nx), B.reshape(nx, nu)
        return xn, A.reshape(nx, nx), B.reshape(nx, nu), H.reshape(nz, nz)

    def stage_constraints(self, z, p):
        nh, nz = self.nh, self.nz
        h = np.zeros(max(nh, 1))
        J = np.zeros(max(nh, 1) * nz)
        Hh = np.zeros(max(nh, 1) * nz * nz)
        self.L.orc_stage_constraints(C.byref(self.pr), np.ascontiguousarray(z, float), np.ascontiguousarray(p, float), h, J, Hh)
        return h[:nh], J[:nh * nz].reshape(nh, nz), Hh[:nh * nz * nz].reshape(nh, nz, nz)

    def h_bounds(self):
        nh = self.nh
        lh, uh = np.zeros(nh), np.zeros(nh)
        self.L.orc_h_bounds(C.byref(self.pr), lh, uh)
        return lh, uh

    def dynamics(self, z):
        """continuous model of the integrated states (C3: the 5 bicycle states)"""
        nxi, nz = (5 if self.layout.model == "bicycle_ca" else self.nx), self.nz
        f, J, H = np.zeros(nxi), np.zeros(nxi * nz), np.zeros(nxi * nz * nz)
        self.L.orc_dynamics(np.ascontiguousarray(z, float), f, J, H)
        return f, J.reshape(nxi, nz), H.reshape(nxi, nz, nz)

    def erk4(self, z, adj=None):
        nx, nz = self.nx, self.nz
        nu = self.nu
        xn, A, B = np.zeros(nx), np.zeros(nx * nx), np.zeros(nx * nu)
        H = np.zeros(nz * nz)
        if adj is None:
            self.L.orc_erk4(C.byref(self.pr), np.ascontiguousarray(z, float), xn, A, B, None, None)
            return xn, A.reshape(nx, nx), B.reshape(nx, nu)
        adj = np.ascontiguousarray(adj, float)
        self.L.orc_erk4(C.byref(self.pr), np.ascontiguousarray(z, float), xn, A, B,
                        adj.ctypes.data_as(C.c_void_p), H.ctypes.data_as(C.c_void_p))
        return xn, A.reshape(nx, nx), B.reshape(nx, nu), H.reshape(nz, nz)

    def mirror(self, H, eps=1e-4):
        n = H.shape[0]
        Hc = np.ascontiguousarray(H, float).copy().ravel()
        self.L.orc_mirror(n, Hc, eps)
        return Hc.reshape(n, n)

    def solve(self, params, warm, xinit):
        N, nx = self.layout.N, self.nx
        xt, ut = np.zeros((N + 1) * nx), np.zeros(N * self.nu)
        info = OrcInfo()
        code = self.L.orc_solve(C.byref(self.pr), np.ascontiguousarray(params, float).ravel(),
                                np.ascontiguousarray(warm, float).ravel(), np.ascontiguousarray(xinit, float).ravel(),
                                xt, ut, C.byref(info))
        return dict(exit=code, xtraj=xt.reshape(N + 1, nx), utraj=ut.reshape(N, self.nu), pobj=info.pobj,
                    sqp_iter=info.sqp_iter, qp_iter=info.qp_iter_total, qp_status=info.qp_status,
                    res_eq=info.res_eq)

    def lam_size(self):
        return self.layout.N * (self.nx + self.layout.nh)

    def qp_mem_size(self):
        return self.L.orc_qp_mem_size(C.byref(self.pr))

    def solve_batch(self, params, warm, xinit, nthreads=0, lam_in=None, return_lam=False, qp_in=None,
                    return_qp=False):
        """lam_in / returned lam: [B, N, nx + nh] NLP multipliers (include/mpcg.h, mpcg_io);
        qp_in / returned qp: [B, qp_mem_size] the capsule's QP memory (oracle layout).
        Returns trajectories, pobj, status and the per-solve info arrays (sqp_iter,
        qp_iter, qp_status, res_eq, res_stat, res_ineq, res_comp)."""
        N, nx = self.layout.N, self.nx
        B = params.shape[0]
        xt, ut = np.zeros((B, N + 1, nx)), np.zeros((B, N, self.nu))
        st = np.zeros(B, np.int32)
        infos = (OrcInfo * max(B, 1))()
        li = None if lam_in is None else np.ascontiguousarray(lam_in, float).reshape(B, -1)
        lo = np.zeros((B, N, nx + self.layout.nh)) if return_lam else None
        qs = self.qp_mem_size()
        qi_ = None if qp_in is None else np.ascontiguousarray(qp_in, float).reshape(B, qs)
        qo = np.zeros((B, qs)) if return_qp else None
        vp = lambda a: None if a is None else a.ctypes.data_as(C.c_void_p)  # noqa: E731
        self.L.orc_solve_batch_full(C.byref(self.pr), B, np.ascontiguousarray(params, float).reshape(-1),
                                    np.ascontiguousarray(warm, float).reshape(-1),
                                    np.ascontiguousarray(xinit, float).reshape(-1), vp(li), vp(qi_),
                                    xt.reshape(-1), ut.reshape(-1), st, vp(lo), vp(qo),
                                    C.cast(infos, C.c_void_p), nthreads)
        get = lambda f, dt: np.array([getattr(infos[b], f) for b in range(B)], dt)  # noqa: E731
        out = dict(xtraj=xt, utraj=ut, pobj=get("pobj", float), status=st, qp_iter=get("qp_iter_total", np.int32),
                   sqp_iter=get("sqp_iter", np.int32), qp_status=get("qp_status", np.int32),
                   res_eq=get("res_eq", float), res_stat=get("res_stat", float),
                   res_ineq=get("res_ineq", float), res_comp=get("res_comp", float),
                   qp_maxiter=get("qp_maxiter", np.int32), qp_center=get("qp_center", np.int32),
                   qp_itref=get("qp_itref", np.int32), qp_lq=get("qp_lq", np.int32))
        if return_lam:
            out["lam"] = lo
        if return_qp:
            out["qp"] = qo
        return out
