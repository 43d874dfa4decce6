#!/usr/bin/env python3
"""Golden stage-function vectors of the C3 problem from the
reference's own Python problem definition (TEST INFRASTRUCTURE — run once in
the build container; outputs committed under tests/golden/).

C3 = BicycleModel2ndOrderCurvatureAware (solver_model.py:355-437) +
MPCBase(a, w, slack) + CurvatureAwareContouring (curvature_aware_contouring.py:15-105)
+ DecompConstraints(12 halfspaces with slack, decomp_constraints.py:16-98),
built through the same sympy casadi stand-in as gen_golden.py.  The
reference generates this model only with Forces (forces_discrete_dynamics,
solver_model.py:11-36, then model_discrete_dynamics): Forces is licensed and
absent, so the discretisation is pinned in two pieces — the reference's
continuous_model and its CA spline update model_discrete_dynamics(z, I)
(integrated states I as free symbols) — and composed with one explicit RK4
step (forcespro.nlp.integrators.RK4, stepsize = integrator_step, the
published RK4 tableau) here, symbolically, for the composed map.

Output: tests/golden/stage_C3.npz and tests/golden/parameter_maps_c3.json.
"""
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import gen_golden as G  # noqa: E402,F401  (sets up the stub and the reference paths)

import sympy as sp  # noqa: E402

from control_modules import ModuleManager  # noqa: E402
from util.parameters import Parameters  # noqa: E402
from solver_definition import (define_parameters, objective, constraints,  # noqa: E402
                               constraint_lower_bounds, constraint_upper_bounds)
from solver_model import BicycleModel2ndOrderCurvatureAware  # noqa: E402
from mpc_base import MPCBaseModule  # noqa: E402
from curvature_aware_contouring import CurvatureAwareContouringModule  # noqa: E402
from decomp_constraints import DecompConstraintModule  # noqa: E402

N_C3 = 30
DT = 0.2


def settings_c3(N=N_C3):
    return {"N": N, "n_discs": 1, "integrator_step": DT,
            "decomp": {"max_constraints": 12},
            "contouring": {"num_segments": 5, "dynamic_velocity_reference": False}}


def ca_decomp_stack(settings):
    modules = ModuleManager()
    model = BicycleModel2ndOrderCurvatureAware()
    base = modules.add_module(MPCBaseModule(settings))
    base.weigh_variable(var_name="a", weight_names="acceleration")
    base.weigh_variable(var_name="w", weight_names="angular_velocity")
    base.weigh_variable(var_name="slack", weight_names="slack")
    modules.add_module(CurvatureAwareContouringModule(settings))
    modules.add_module(DecompConstraintModule(settings))
    return model, modules


def _scalar(e):
    if isinstance(e, sp.MatrixBase):
        assert e.shape == (1, 1)
        return e[0, 0]
    return sp.sympify(e)


def rk4(f, x, u, h):
    """One classical RK4 step of x' = f(x, u) (u held constant)."""
    k1 = [sp.sympify(e) for e in f(x, u)]
    k2 = [sp.sympify(e) for e in f([xi + h / 2 * ki for xi, ki in zip(x, k1)], u)]
    k3 = [sp.sympify(e) for e in f([xi + h / 2 * ki for xi, ki in zip(x, k2)], u)]
    k4 = [sp.sympify(e) for e in f([xi + h * ki for xi, ki in zip(x, k3)], u)]
    return [xi + h / 6 * (a + 2 * b + 2 * c + d) for xi, a, b, c, d in zip(x, k1, k2, k3, k4)]


def synthetic_point(rng, pmap, npar, nz, straight=False):
    p = np.zeros(npar)
    w = {"acceleration": 0.34, "angular_velocity": 0.85, "slack": 10000.0, "velocity": 0.55,
         "reference_velocity": 2.0, "contour": 0.05, "lag": 0.75,
         "terminal_angle": 100.0, "terminal_contouring": 10.0}
    for k, v in w.items():
        p[pmap[k]] = v * rng.uniform(0.5, 1.5)
    s0 = 0.0
    px, py, th = rng.uniform(-5, 5), rng.uniform(-5, 5), rng.uniform(-np.pi, np.pi)
    for j in range(5):
        L = rng.uniform(3.0, 6.0)
        # near-straight paths put 1 / curvature above the 1e5 floor of
        # solver_model.py:429 (the other branch of fmax)
        dth = rng.uniform(-1e-6, 1e-6) if straight else rng.uniform(-0.6, 0.6)
        c = np.array([np.cos(th), np.sin(th)])
        th1 = th + dth
        c1 = np.array([np.cos(th1), np.sin(th1)])
        p0 = np.array([px, py])
        p1 = p0 + L * 0.5 * (c + c1)
        for ax, name in enumerate(["x", "y"]):
            A = np.array([[L ** 3, L ** 2], [3 * L ** 2, 2 * L]])
            rhs = np.array([p1[ax] - p0[ax] - c[ax] * L, c1[ax] - c[ax]])
            a_, b_ = np.linalg.solve(A, rhs)
            p[pmap[f"spline_{name}{j}_a"]] = a_
            p[pmap[f"spline_{name}{j}_b"]] = b_
            p[pmap[f"spline_{name}{j}_c"]] = c[ax]
            p[pmap[f"spline_{name}{j}_d"]] = p0[ax]
        p[pmap[f"spline{j}_start"]] = s0
        s0 += L
        px, py, th = p1[0], p1[1], th1
    p[pmap["ego_disc_0_offset"]] = rng.uniform(-0.5, 1.5)
    z = np.zeros(nz)
    z[0] = rng.uniform(-3, 3)          # a
    z[1] = rng.uniform(-1.5, 1.5)      # w (steering rate)
    z[2] = rng.uniform(0, 2)           # slack
    z[3] = rng.uniform(-10, 10)        # x
    z[4] = rng.uniform(-10, 10)        # y
    z[5] = rng.uniform(-np.pi, np.pi)  # psi
    z[6] = rng.uniform(0, 6)           # v
    z[7] = rng.uniform(-0.55, 0.55)    # delta
    z[8] = rng.uniform(0.5, s0 - 0.5)  # spline
    for i in range(12):
        th = rng.uniform(-np.pi, np.pi)
        p[pmap[f"disc_0_decomp_{i}_a1"]] = np.cos(th)
        p[pmap[f"disc_0_decomp_{i}_a2"]] = np.sin(th)
        p[pmap[f"disc_0_decomp_{i}_b"]] = rng.uniform(-5, 5)
    return z, p


def main(npts=24, seed=20251215):
    t0 = time.time()
    settings = settings_c3()
    model, modules = ca_decomp_stack(settings)
    params = Parameters()
    define_parameters(modules, params, settings)
    npar = params.length()
    settings["params"] = params
    pmap = dict(params._params)
    nz = model.get_nvar()
    nu, nx = model.nu, model.nx
    zs = [sp.Symbol(f"z{i}", real=True) for i in range(nz)]
    ps = [sp.Symbol(f"p{i}", real=True) for i in range(npar)]
    Is = [sp.Symbol(f"I{i}", real=True) for i in range(nx - 1)]
    # stage_idx 1 (path stages) and N - 1 (the terminal terms, curvature_aware_contouring.py:91-103)
    L1 = _scalar(objective(modules, zs, ps, model, settings, 1))
    print(f"[C3] L1 {time.time() - t0:.1f}s")
    LN = _scalar(objective(modules, zs, ps, model, settings, settings["N"] - 1))
    print(f"[C3] LN {time.time() - t0:.1f}s")
    h = [_scalar(c) for c in constraints(modules, zs, ps, model, settings, 1)]
    lb = constraint_lower_bounds(modules)
    ub = constraint_upper_bounds(modules)
    f = [sp.sympify(e) for e in model.continuous_model(zs[nu:], zs[:nu])]
    # CA spline update with the integrated states as free symbols
    params.load(ps)
    model.load(zs)
    model.load_settings(settings)
    g = [sp.sympify(e) for e in model.model_discrete_dynamics(zs, sp.Matrix(Is))]
    print(f"[C3] g {time.time() - t0:.1f}s")
    # composed discrete map: one RK4 step of the integrated states, then the CA update
    xi = rk4(lambda x, u: model.continuous_model(x, u), zs[nu:nu + nx - 1], zs[:nu], DT)
    model.load(zs)
    Fd = [e.subs(dict(zip(Is, xi))) for e in g]
    print(f"[C3] symbolic build {time.time() - t0:.1f}s npar={npar} nh={len(h)} nz={nz}")

    def jet(exprs, vars_):
        d1 = [[sp.diff(e, v) for v in vars_] for e in exprs]
        d2 = [[[sp.diff(d1[r][i], vars_[j]) for j in range(len(vars_))] for i in range(len(vars_))]
              for r in range(len(exprs))]
        return d1, d2

    dL1 = [sp.diff(L1, v) for v in zs]
    d2L1 = [[sp.diff(dL1[i], zs[j]) for j in range(nz)] for i in range(nz)]
    dLN = [sp.diff(LN, v) for v in zs]
    d2LN = [[sp.diff(dLN[i], zs[j]) for j in range(nz)] for i in range(nz)]
    dh, d2h = jet(h, zs)
    df, d2f = jet(f, zs)
    zi = zs + Is
    dg, d2g = jet(g, zi)
    dF = [[sp.diff(e, v) for v in zs] for e in Fd]  # the composed Hessian is checked by differences
    print(f"[C3] derivatives {time.time() - t0:.1f}s")
    mods = [{"Heaviside": lambda x, h0=0.5: np.heaviside(x, h0), "fmod": np.fmod, "DiracDelta": lambda x, *a: 0.0 * x}, "numpy"]
    fL1 = sp.lambdify((zs, ps), [L1, dL1, d2L1], mods, cse=True)
    fLN = sp.lambdify((zs, ps), [LN, dLN, d2LN], mods, cse=True)
    fh = sp.lambdify((zs, ps), [h, dh, d2h], mods, cse=True)
    ff = sp.lambdify((zs, ps), [f, df, d2f], mods, cse=True)
    fg = sp.lambdify((zs, Is, ps), [g, dg, d2g], mods, cse=True)
    fF = sp.lambdify((zs, ps), [Fd, dF, 0], mods, cse=True)
    print(f"[C3] lambdify {time.time() - t0:.1f}s")
    rng = np.random.default_rng(seed)
    keys = ["L1", "dL1", "d2L1", "LN", "dLN", "d2LN", "h", "dh", "d2h", "f", "df", "d2f",
            "g", "dg", "d2g", "F", "dF"]
    out = {k: [] for k in keys}
    Z, P, IV = [], [], []
    for n in range(npts):
        z, p = synthetic_point(rng, pmap, npar, nz, straight=(n % 6 == 5))
        iv = z[3:8] + rng.uniform(-0.5, 0.5, nx - 1)
        Z.append(z); P.append(p); IV.append(iv)
        for key, fn, args in (("L1", fL1, (z, p)), ("LN", fLN, (z, p)), ("h", fh, (z, p)),
                              ("f", ff, (z, p)), ("g", fg, (z, iv, p)), ("F", fF, (z, p))):
            a, b, c = fn(*[list(x) for x in args])
            out[key].append(np.array(a, float))
            out["d" + key].append(np.array(b, float))
            if key != "F":
                out["d2" + key].append(np.array(c, float))
    np.savez_compressed(os.path.join(HERE, "stage_C3.npz"), z=np.array(Z), p=np.array(P), I=np.array(IV),
                        lh=np.array([float(v) for v in lb]), uh=np.array([float(v) for v in ub]),
                        model_lb=np.array(model.lower_bound, float), model_ub=np.array(model.upper_bound, float),
                        dt=DT, N=settings["N"], **{k: np.array(v) for k, v in out.items()})
    with open(os.path.join(HERE, "parameter_maps_c3.json"), "w") as fh_:
        json.dump({"C3": pmap}, fh_, indent=1, sort_keys=True)
    print(f"[C3] {npts} points in {time.time() - t0:.1f}s; npar {npar}")


if __name__ == "__main__":
    main()
