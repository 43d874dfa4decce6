"""ctypes binding of the C ABI (include/mpcg.h) implemented by libmpcg.so.

The product path: no fallback.  If libmpcg.so is missing or cannot be loaded
the import of this module raises, and every solve fails loudly.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

from .layouts import Layout

PKG = os.path.dirname(os.path.abspath(__file__))
# MPCG_LIB selects a diagnostic build (e.g. libmpcg_stamps.so); default the production library
LIB_PATH = os.environ.get("MPCG_LIB") or os.path.join(PKG, "libmpcg.so")

NX, NU, NVAR = 5, 2, 7
INFO_STRIDE = 4


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
        ("dt", C.c_double), ("rk_steps", C.c_int),
        ("lbu", C.c_double * 2), ("ubu", C.c_double * 2), ("lbx", C.c_double * 5), ("ubx", C.c_double * 5),
        ("sqp_iters", C.c_int), ("qp_tol", C.c_double), ("qp_iter_max", C.c_int),
        ("reg_eps", C.c_double), ("qp_mu0", C.c_double), ("qp_thr0", C.c_double),
        ("res_eq_fail", C.c_double),
    ]


# acados options restated (generate_acados_solver.py:88-173) + our IPM cold start
DEFAULT_OPTIONS = dict(qp_tol=1e-5, qp_iter_max=50, reg_eps=1e-4, qp_mu0=1.0, qp_thr0=1.0, res_eq_fail=1e-2)
# ContouringSecondOrderUnicycleModel bounds (solver_model.py:204-205), z = [a, w, x, y, psi, v, s]
UNICYCLE_LB = (-2.0, -0.8, -2000.0, -2000.0, -4 * np.pi, -0.01, -1.0)
UNICYCLE_UB = (2.0, 0.8, 2000.0, 2000.0, 4 * np.pi, 3.0, 10000.0)


def problem_from_layout(layout: Layout, **opts) -> MpcgProblem:
    o = dict(DEFAULT_OPTIONS)
    o.update(opts)
    pr = MpcgProblem()
    pr.N, pr.npar = layout.N, layout.npar
    pr.n_lin, pr.n_ell, pr.n_seg = layout.n_lin, layout.n_ell, layout.n_seg
    for k, v in layout.index_struct().items():
        setattr(pr, k, v)
    pr.dt = o.get("dt", layout.dt)
    pr.rk_steps = o.get("rk_steps", layout.rk_steps)
    lb, ub = o.get("lb", UNICYCLE_LB), o.get("ub", UNICYCLE_UB)
    for i in range(NU):
        pr.lbu[i], pr.ubu[i] = lb[i], ub[i]
    for i in range(NX):
        pr.lbx[i], pr.ubx[i] = lb[NU + i], ub[NU + i]
    pr.sqp_iters = o.get("sqp_iters", layout.sqp_iters)
    pr.qp_tol = o["qp_tol"]
    pr.qp_iter_max = o["qp_iter_max"]
    pr.reg_eps = o["reg_eps"]
    pr.qp_mu0 = o["qp_mu0"]
    pr.qp_thr0 = o["qp_thr0"]
    pr.res_eq_fail = o["res_eq_fail"]
    return pr


EXPORTS = ("mpcg_abi_version", "mpcg_last_error", "mpcg_supported", "mpcg_solve_batch_device",
           "mpcg_solve_batch_host", "mpcg_select_best_device")


def _load():
    # Load torch's HIP runtime first: libmpcg.so's libamdhip64.so.7 /
    # libhsa-runtime64.so.1 then resolve (by SONAME) to the copies torch already
    # mapped, so the process holds exactly one HIP runtime and device pointers
    # from torch tensors are valid in our kernels.
    import torch  # noqa: F401

    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} not built: run `python -c 'import __graft_entry__ as g; g.build()'` "
                          "(hipcc --offload-arch=gfx950); there is no CPU fallback")
    lib = C.CDLL(LIB_PATH)
    P = C.POINTER(MpcgProblem)
    vp = C.c_void_p
    lib.mpcg_abi_version.restype = C.c_int
    lib.mpcg_last_error.restype = C.c_char_p
    lib.mpcg_supported.argtypes = [P]
    lib.mpcg_supported.restype = C.c_int
    lib.mpcg_solve_batch_device.argtypes = [P, C.c_int, vp, vp, vp, vp, vp, vp, vp, vp, vp]
    lib.mpcg_solve_batch_device.restype = C.c_int
    lib.mpcg_solve_batch_host.argtypes = [P, C.c_int, vp, vp, vp, vp, vp, vp, vp, vp]
    lib.mpcg_solve_batch_host.restype = C.c_int
    lib.mpcg_select_best_device.argtypes = [C.c_int, C.c_int, C.c_int, vp, vp, vp, vp, C.c_double, vp, vp,
                                            C.c_double, vp, vp, vp, vp]
    lib.mpcg_select_best_device.restype = C.c_int
    return lib


lib = _load()


def last_error() -> str:
    return lib.mpcg_last_error().decode()


def _ptr(t):
    return None if t is None else C.c_void_p(t.data_ptr())


def _check(rc, what):
    if rc != 0:
        raise RuntimeError(f"{what} failed ({rc}): {last_error()}")


def solve_batch_device(pr: MpcgProblem, params, warm, xinit, out=None, stream=None):
    """Batched solve on device tensors (torch, float64, on the current HIP device).
    params (B, N, npar), warm (B, N+1, 7), xinit (B, 5).  Returns a dict of
    device tensors; asynchronous on `stream` (torch.cuda stream or None = current)."""
    import torch

    B = params.shape[0]
    N = pr.N
    assert params.dtype == torch.float64 and params.is_cuda and params.is_contiguous()
    assert tuple(params.shape) == (B, N, pr.npar), (tuple(params.shape), (B, N, pr.npar))
    assert tuple(warm.shape) == (B, N + 1, NVAR) and warm.is_contiguous() and warm.dtype == torch.float64
    assert tuple(xinit.shape) == (B, NX) and xinit.is_contiguous() and xinit.dtype == torch.float64
    dev = params.device
    if out is None:
        out = dict(xtraj=torch.empty((B, N + 1, NX), dtype=torch.float64, device=dev),
                   utraj=torch.empty((B, N, NU), dtype=torch.float64, device=dev),
                   pobj=torch.empty((B,), dtype=torch.float64, device=dev),
                   exit=torch.empty((B,), dtype=torch.int32, device=dev),
                   info=torch.empty((B, INFO_STRIDE), dtype=torch.int32, device=dev))
    s = stream if stream is not None else torch.cuda.current_stream(dev)
    rc = lib.mpcg_solve_batch_device(C.byref(pr), B, _ptr(params), _ptr(warm), _ptr(xinit), _ptr(out["xtraj"]),
                                     _ptr(out["utraj"]), _ptr(out["pobj"]), _ptr(out["exit"]), _ptr(out["info"]),
                                     C.c_void_p(s.cuda_stream))
    _check(rc, "mpcg_solve_batch_device")
    return out


def solve_batch_host(pr: MpcgProblem, params: np.ndarray, warm: np.ndarray, xinit: np.ndarray):
    """Host-buffer solve through the same kernels (copies in/out, synchronous)."""
    B = params.shape[0]
    N = pr.N
    params = np.ascontiguousarray(params, np.float64)
    warm = np.ascontiguousarray(warm, np.float64)
    xinit = np.ascontiguousarray(xinit, np.float64)
    assert params.shape == (B, N, pr.npar) and warm.shape == (B, N + 1, NVAR) and xinit.shape == (B, NX)
    xt = np.zeros((B, N + 1, NX))
    ut = np.zeros((B, N, NU))
    po = np.zeros(B)
    ex = np.zeros(B, np.int32)
    info = np.zeros((B, INFO_STRIDE), np.int32)
    vp = lambda a: a.ctypes.data_as(C.c_void_p)  # noqa: E731
    rc = lib.mpcg_solve_batch_host(C.byref(pr), B, vp(params), vp(warm), vp(xinit), vp(xt), vp(ut), vp(po),
                                   vp(ex), vp(info))
    _check(rc, "mpcg_solve_batch_host")
    return dict(xtraj=xt, utraj=ut, pobj=po, exit=ex, info=info)


def select_best_device(n_scenes, n_guesses, N, xtraj, pobj, exit_code, prev_traj=None, w_cons=0.0,
                       consistency_enabled=None, previously_selected=None, selection_weight=1.0,
                       disabled=None, stream=None):
    import torch

    dev = pobj.device
    best = torch.empty((n_scenes,), dtype=torch.int32, device=dev)
    objective = torch.empty((n_scenes * n_guesses,), dtype=torch.float64, device=dev)
    s = stream if stream is not None else torch.cuda.current_stream(dev)
    rc = lib.mpcg_select_best_device(n_scenes, n_guesses, N, _ptr(xtraj), _ptr(pobj), _ptr(exit_code),
                                     _ptr(prev_traj), float(w_cons), _ptr(consistency_enabled),
                                     _ptr(previously_selected), float(selection_weight), _ptr(disabled),
                                     _ptr(best), _ptr(objective), C.c_void_p(s.cuda_stream))
    _check(rc, "mpcg_select_best_device")
    return best, objective
