"""ctypes binding of the C ABI (include/mpcg.h) implemented by libmpcg.so.

The product path: no fallback.  If libmpcg.so is missing or cannot be loaded
the import of this module raises, and every solve fails loudly.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

from .native_spec import (DEFAULT_OPTIONS, EXPORTS, INFO_STRIDE, NU, NVAR, NX, UNICYCLE_LB,  # noqa: F401
                          UNICYCLE_UB, MpcgProblem, problem_from_layout)

PKG = os.path.dirname(os.path.abspath(__file__))
# MPCG_LIB selects a diagnostic build (e.g. libmpcg_stamps.so); default the production library
LIB_PATH = os.environ.get("MPCG_LIB") or os.path.join(PKG, "libmpcg.so")

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
