"""ctypes binding of the CPU oracle (oracle/libmpcg_oracle.so).

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

ORC_NX, ORC_NU, ORC_NZ = 5, 2, 7


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
        ("dt", C.c_double), ("rk_steps", C.c_int),
        ("lbu", C.c_double * 2), ("ubu", C.c_double * 2), ("lbx", C.c_double * 5), ("ubx", C.c_double * 5),
        ("sqp_iters", C.c_int), ("qp_tol", C.c_double), ("qp_iter_max", C.c_int),
        ("reg_eps", C.c_double), ("qp_mu0", C.c_double), ("qp_thr0", C.c_double),
        ("res_eq_fail", C.c_double),
    ]


class OrcInfo(C.Structure):
    _fields_ = [("sqp_iter", C.c_int), ("qp_iter_total", C.c_int), ("qp_status", C.c_int),
                ("res_eq", C.c_double), ("pobj", C.c_double)]


def build(force: bool = False) -> str:
    src = os.path.join(HERE, "mpcg_oracle.c")
    if force or not os.path.exists(LIB) or os.path.getmtime(LIB) < os.path.getmtime(src):
        subprocess.run(["make", "-C", HERE, "-s"], check=True)
    return LIB


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        L = C.CDLL(LIB)
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
        L.orc_mirror.argtypes = [C.c_int, dp, C.c_double]
        L.orc_solve.argtypes = [P, dp, dp, dp, dp, dp, C.POINTER(OrcInfo)]
        L.orc_solve.restype = C.c_int
        L.orc_solve_batch.argtypes = [P, C.c_int, dp, dp, dp, dp, dp, dp, ip, ip, C.c_int]
        vp = C.c_void_p
        L.orc_solve_batch_ex.argtypes = [P, C.c_int, dp, dp, dp, vp, dp, dp, dp, ip, ip, vp, C.c_int]
        _lib = L
    return _lib


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
    lb = opts.get("lb", (-2.0, -0.8, -2000.0, -2000.0, -4 * np.pi, -0.01, -1.0))
    ub = opts.get("ub", (2.0, 0.8, 2000.0, 2000.0, 4 * np.pi, 3.0, 10000.0))
    for i in range(2):
        pr.lbu[i], pr.ubu[i] = lb[i], ub[i]
    for i in range(5):
        pr.lbx[i], pr.ubx[i] = lb[2 + i], ub[2 + i]
    pr.sqp_iters = opts.get("sqp_iters", layout.sqp_iters)
    pr.qp_tol = opts.get("qp_tol", 1e-5)
    pr.qp_iter_max = opts.get("qp_iter_max", 50)
    pr.reg_eps = opts.get("reg_eps", 1e-4)
    pr.qp_mu0 = opts.get("qp_mu0", 1.0)
    pr.qp_thr0 = opts.get("qp_thr0", 1.0)
    pr.res_eq_fail = opts.get("res_eq_fail", 1e-2)
    return pr


class Oracle:
    """Thin wrapper: stage functions and full solves on numpy arrays."""

    def __init__(self, layout, **opts):
        self.layout = layout
        self.pr = problem_from_layout(layout, **opts)
        self.L = lib()

    @property
    def nh(self):
        return self.L.orc_num_h(C.byref(self.pr))

    def stage_cost(self, z, p):
        out = np.zeros(1)
        g = np.zeros(7)
        H = np.zeros(49)
        self.L.orc_stage_cost(C.byref(self.pr), np.ascontiguousarray(z, float), np.ascontiguousarray(p, float), out, g, H)
        return out[0], g, H.reshape(7, 7)

    def stage_constraints(self, z, p):
        nh = self.nh
        h = np.zeros(nh)
        J = np.zeros(nh * 7)
        Hh = np.zeros(nh * 49)
        self.L.orc_stage_constraints(C.byref(self.pr), np.ascontiguousarray(z, float), np.ascontiguousarray(p, float), h, J, Hh)
        return h, J.reshape(nh, 7), Hh.reshape(nh, 7, 7)

    def h_bounds(self):
        nh = self.nh
        lh, uh = np.zeros(nh), np.zeros(nh)
        self.L.orc_h_bounds(C.byref(self.pr), lh, uh)
        return lh, uh

    def dynamics(self, z):
        f, J, H = np.zeros(5), np.zeros(35), np.zeros(245)
        self.L.orc_dynamics(np.ascontiguousarray(z, float), f, J, H)
        return f, J.reshape(5, 7), H.reshape(5, 7, 7)

    def erk4(self, z, adj=None):
        xn, A, B = np.zeros(5), np.zeros(25), np.zeros(10)
        H = np.zeros(49)
        if adj is None:
            self.L.orc_erk4(C.byref(self.pr), np.ascontiguousarray(z, float), xn, A, B, None, None)
            return xn, A.reshape(5, 5), B.reshape(5, 2)
        adj = np.ascontiguousarray(adj, float)
        self.L.orc_erk4(C.byref(self.pr), np.ascontiguousarray(z, float), xn, A, B,
                        adj.ctypes.data_as(C.c_void_p), H.ctypes.data_as(C.c_void_p))
        return xn, A.reshape(5, 5), B.reshape(5, 2), H.reshape(7, 7)

    def mirror(self, H, eps=1e-4):
        n = H.shape[0]
        Hc = np.ascontiguousarray(H, float).copy().ravel()
        self.L.orc_mirror(n, Hc, eps)
        return Hc.reshape(n, n)

    def solve(self, params, warm, xinit):
        N = self.layout.N
        xt, ut = np.zeros((N + 1) * 5), np.zeros(N * 2)
        info = OrcInfo()
        code = self.L.orc_solve(C.byref(self.pr), np.ascontiguousarray(params, float).ravel(),
                                np.ascontiguousarray(warm, float).ravel(), np.ascontiguousarray(xinit, float).ravel(),
                                xt, ut, C.byref(info))
        return dict(exit=code, xtraj=xt.reshape(N + 1, 5), utraj=ut.reshape(N, 2), pobj=info.pobj,
                    sqp_iter=info.sqp_iter, qp_iter=info.qp_iter_total, qp_status=info.qp_status,
                    res_eq=info.res_eq)

    def lam_size(self):
        return self.layout.N * (5 + self.layout.nh)

    def solve_batch(self, params, warm, xinit, nthreads=0, lam_in=None, return_lam=False):
        """lam_in / returned lam: [B, N, 5 + nh] NLP multipliers (include/mpcg.h, mpcg_io)."""
        N = self.layout.N
        B = params.shape[0]
        if lam_in is not None or return_lam:
            xt, ut = np.zeros((B, N + 1, 5)), np.zeros((B, N, 2))
            pobj, st, qi = np.zeros(B), np.zeros(B, np.int32), np.zeros(B, np.int32)
            li = None if lam_in is None else np.ascontiguousarray(lam_in, float).reshape(B, -1)
            lo = np.zeros((B, N, 5 + self.layout.nh))
            self.L.orc_solve_batch_ex(C.byref(self.pr), B, np.ascontiguousarray(params, float).reshape(-1),
                                      np.ascontiguousarray(warm, float).reshape(-1),
                                      np.ascontiguousarray(xinit, float).reshape(-1),
                                      None if li is None else li.ctypes.data_as(C.c_void_p),
                                      xt.reshape(-1), ut.reshape(-1), pobj, st, qi,
                                      lo.ctypes.data_as(C.c_void_p), nthreads)
            return dict(xtraj=xt, utraj=ut, pobj=pobj, status=st, qp_iter=qi, lam=lo)
        xt = np.zeros((B, N + 1, 5))
        ut = np.zeros((B, N, 2))
        pobj = np.zeros(B)
        st = np.zeros(B, np.int32)
        qi = np.zeros(B, np.int32)
        self.L.orc_solve_batch(C.byref(self.pr), B, np.ascontiguousarray(params, float).reshape(-1),
                               np.ascontiguousarray(warm, float).reshape(-1),
                               np.ascontiguousarray(xinit, float).reshape(-1),
                               xt.reshape(-1), ut.reshape(-1), pobj, st, qi, nthreads)
        return dict(xtraj=xt, utraj=ut, pobj=pobj, status=st, qp_iter=qi)
