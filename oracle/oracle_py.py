"""ctypes binding of the CPU oracle (oracle/libmpcg_oracle.so, nx 5;
oracle/libmpcg_oracle_slack.so, nx 6 — the C5 slack model).

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
LIBS = {5: LIB, 6: LIB_SLACK}

ORC_NU, ORC_MAX_NX = 2, 6


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
        ("lbu", C.c_double * 2), ("ubu", C.c_double * 2),
        ("lbx", C.c_double * ORC_MAX_NX), ("ubx", C.c_double * ORC_MAX_NX),
        ("sqp_iters", C.c_int), ("qp_tol", C.c_double), ("qp_iter_max", C.c_int),
        ("reg_eps", C.c_double), ("qp_mu0", C.c_double), ("qp_thr0", C.c_double),
        ("res_eq_fail", C.c_double),
    ]


class OrcInfo(C.Structure):
    _fields_ = [("sqp_iter", C.c_int), ("qp_iter_total", C.c_int), ("qp_status", C.c_int),
                ("res_eq", C.c_double), ("pobj", C.c_double)]


def build(force: bool = False) -> str:
    srcs = [os.path.join(HERE, f) for f in ("mpcg_oracle.c", "mpcg_oracle.h")]
    newest = max(os.path.getmtime(f) for f in srcs)
    if force or any(not os.path.exists(x) or os.path.getmtime(x) < newest for x in LIBS.values()):
        subprocess.run(["make", "-C", HERE, "-s"], check=True)
    return LIB


_libs = {}


def lib(nx: int = 5):
    if nx not in _libs:
        path = LIBS[nx]
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
        L.orc_mirror.argtypes = [C.c_int, dp, C.c_double]
        L.orc_solve.argtypes = [P, dp, dp, dp, dp, dp, C.POINTER(OrcInfo)]
        L.orc_solve.restype = C.c_int
        L.orc_solve_batch.argtypes = [P, C.c_int, dp, dp, dp, dp, dp, dp, ip, ip, C.c_int]
        vp = C.c_void_p
        L.orc_solve_batch_ex.argtypes = [P, C.c_int, dp, dp, dp, vp, dp, dp, dp, ip, ip, vp, C.c_int]
        L.orc_nx.restype = C.c_int
        if L.orc_nx() != nx:
            raise RuntimeError(f"{path} is built for nx={L.orc_nx()}, expected {nx}")
        _libs[nx] = L
    return _libs[nx]


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
    lb = opts.get("lb", layout.lb)
    ub = opts.get("ub", layout.ub)
    for i in range(2):
        pr.lbu[i], pr.ubu[i] = lb[i], ub[i]
    for i in range(nx):
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
        self.nx = nx = layout.nx
        self.nz = nx + ORC_NU
        self.L = lib(nx)

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
        nx, nz = self.nx, self.nz
        f, J, H = np.zeros(nx), np.zeros(nx * nz), np.zeros(nx * nz * nz)
        self.L.orc_dynamics(np.ascontiguousarray(z, float), f, J, H)
        return f, J.reshape(nx, nz), H.reshape(nx, nz, nz)

    def erk4(self, z, adj=None):
        nx, nz = self.nx, self.nz
        xn, A, B = np.zeros(nx), np.zeros(nx * nx), np.zeros(nx * 2)
        H = np.zeros(nz * nz)
        if adj is None:
            self.L.orc_erk4(C.byref(self.pr), np.ascontiguousarray(z, float), xn, A, B, None, None)
            return xn, A.reshape(nx, nx), B.reshape(nx, 2)
        adj = np.ascontiguousarray(adj, float)
        self.L.orc_erk4(C.byref(self.pr), np.ascontiguousarray(z, float), xn, A, B,
                        adj.ctypes.data_as(C.c_void_p), H.ctypes.data_as(C.c_void_p))
        return xn, A.reshape(nx, nx), B.reshape(nx, 2), H.reshape(nz, nz)

    def mirror(self, H, eps=1e-4):
        n = H.shape[0]
        Hc = np.ascontiguousarray(H, float).copy().ravel()
        self.L.orc_mirror(n, Hc, eps)
        return Hc.reshape(n, n)

    def solve(self, params, warm, xinit):
        N, nx = self.layout.N, self.nx
        xt, ut = np.zeros((N + 1) * nx), np.zeros(N * 2)
        info = OrcInfo()
        code = self.L.orc_solve(C.byref(self.pr), np.ascontiguousarray(params, float).ravel(),
                                np.ascontiguousarray(warm, float).ravel(), np.ascontiguousarray(xinit, float).ravel(),
                                xt, ut, C.byref(info))
        return dict(exit=code, xtraj=xt.reshape(N + 1, nx), utraj=ut.reshape(N, 2), pobj=info.pobj,
                    sqp_iter=info.sqp_iter, qp_iter=info.qp_iter_total, qp_status=info.qp_status,
                    res_eq=info.res_eq)

    def lam_size(self):
        return self.layout.N * (self.nx + self.layout.nh)

    def solve_batch(self, params, warm, xinit, nthreads=0, lam_in=None, return_lam=False):
        """lam_in / returned lam: [B, N, nx + nh] NLP multipliers (include/mpcg.h, mpcg_io)."""
        N, nx = self.layout.N, self.nx
        B = params.shape[0]
        if lam_in is not None or return_lam:
            xt, ut = np.zeros((B, N + 1, nx)), np.zeros((B, N, 2))
            pobj, st, qi = np.zeros(B), np.zeros(B, np.int32), np.zeros(B, np.int32)
            li = None if lam_in is None else np.ascontiguousarray(lam_in, float).reshape(B, -1)
            lo = np.zeros((B, N, nx + self.layout.nh))
            self.L.orc_solve_batch_ex(C.byref(self.pr), B, np.ascontiguousarray(params, float).reshape(-1),
                                      np.ascontiguousarray(warm, float).reshape(-1),
                                      np.ascontiguousarray(xinit, float).reshape(-1),
                                      None if li is None else li.ctypes.data_as(C.c_void_p),
                                      xt.reshape(-1), ut.reshape(-1), pobj, st, qi,
                                      lo.ctypes.data_as(C.c_void_p), nthreads)
            return dict(xtraj=xt, utraj=ut, pobj=pobj, status=st, qp_iter=qi, lam=lo)
        xt = np.zeros((B, N + 1, nx))
        ut = np.zeros((B, N, 2))
        pobj = np.zeros(B)
        st = np.zeros(B, np.int32)
        qi = np.zeros(B, np.int32)
        self.L.orc_solve_batch(C.byref(self.pr), B, np.ascontiguousarray(params, float).reshape(-1),
                               np.ascontiguousarray(warm, float).reshape(-1),
                               np.ascontiguousarray(xinit, float).reshape(-1),
                               xt.reshape(-1), ut.reshape(-1), pobj, st, qi, nthreads)
        return dict(xtraj=xt, utraj=ut, pobj=pobj, status=st, qp_iter=qi)
