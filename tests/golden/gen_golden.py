#!/usr/bin/env python3
"""Generate golden stage-function vectors from the reference's OWN Python
problem definition (TEST INFRASTRUCTURE — run once in the build container,
outputs committed under tests/golden/).

What it does
------------
* Puts `tests/golden/_casadi_stub` (a sympy stand-in for casadi 3.5.5, which
  is not installable offline) in front of sys.path and imports the
  reference's `solver_generator` and `mpc_planner_modules/scripts` from
  /root/reference (read-only; never copied, never shipped to the GPU box).
* Re-creates the module stack of the north-star problem exactly as
  `configuration_tmpc_consistency_cost` builds it
  (mpc_planner_jackalsimulator/scripts/generate_jackalsimulator_solver.py:37-116):
  MPCBase(a, w, v) + Contouring + Consistency + GuidanceConstraints(Ellipsoid).
* Calls the reference's `define_parameters` / `objective(..., stage_idx=1)` /
  `constraints(..., 1)` / `constraint_{lower,upper}_bounds`
  (solver_generator/solver_definition.py:5-67) and
  `ContouringSecondOrderUnicycleModel.continuous_model`
  (solver_generator/solver_model.py:207-214) on sympy symbols — the same call
  sequence `create_acados_model` makes (generate_acados_solver.py:27-65).
* Differentiates with sympy and evaluates at seeded random (z, p):
  L, dL/dz, d2L/dz2, h, dh/dz, d2h_i/dz2, f, df/dz, d2f_i/dz2.
* Dumps the parameter index maps of configs C1/C2/C4 and of the
  reference's known-answer module tests.

Outputs: tests/golden/stage_<cfg>.npz, tests/golden/parameter_maps.json
"""
import json
import os
import sys
import time

import numpy as np

REF = os.environ.get("MPCG_REFERENCE", "/root/reference")
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "_casadi_stub"))
sys.path.insert(1, os.path.join(REF, "solver_generator"))
sys.path.insert(2, os.path.join(REF, "mpc_planner_modules", "scripts"))

import sympy as sp  # noqa: E402

from control_modules import ModuleManager  # noqa: E402
from util.parameters import Parameters  # noqa: E402
from solver_definition import (define_parameters, objective, constraints,  # noqa: E402
                               constraint_lower_bounds, constraint_upper_bounds)
from solver_model import ContouringSecondOrderUnicycleModel  # noqa: E402
from mpc_base import MPCBaseModule  # noqa: E402
from contouring import ContouringModule  # noqa: E402
from consistency_module import ConsistencyModule  # noqa: E402
from guidance_constraints import GuidanceConstraintModule  # noqa: E402
from ellipsoid_constraints import EllipsoidConstraintModule  # noqa: E402
from path_reference_velocity import PathReferenceVelocityModule  # noqa: E402


def settings_for(N, max_obstacles, consistency=True):
    return {
        "N": N,
        "n_discs": 1,
        "max_obstacles": max_obstacles,
        "contouring": {"num_segments": 5, "dynamic_velocity_reference": False},
        "linearized_constraints": {"add_halfspaces": 0},
        "JULES": {"consistency_enabled": consistency},
    }


def tmpc_consistency_stack(settings):
    """The module stack of configuration_tmpc_consistency_cost
    (generate_jackalsimulator_solver.py:37-59, 107-116)."""
    modules = ModuleManager()
    model = ContouringSecondOrderUnicycleModel()
    base = modules.add_module(MPCBaseModule(settings))
    base.weigh_variable(var_name="a", weight_names="acceleration")
    base.weigh_variable(var_name="w", weight_names="angular_velocity")
    base.weigh_variable(var_name="v", weight_names=["velocity", "reference_velocity"],
                        cost_function=lambda x, w: w[0] * (x - w[1]) ** 2)
    modules.add_module(ContouringModule(settings))
    if settings["JULES"]["consistency_enabled"]:
        modules.add_module(ConsistencyModule(settings))
    modules.add_module(GuidanceConstraintModule(settings, constraint_submodule=EllipsoidConstraintModule))
    return model, modules


def parameter_map(settings):
    model, modules = tmpc_consistency_stack(settings)
    params = Parameters()
    define_parameters(modules, params, settings)
    return dict(params._params), params.length()


def _scalar(e):
    if isinstance(e, sp.MatrixBase):
        assert e.shape == (1, 1)
        return e[0, 0]
    return sp.sympify(e)


def symbolic_stage(settings):
    model, modules = tmpc_consistency_stack(settings)
    params = Parameters()
    define_parameters(modules, params, settings)
    npar = params.length()
    settings["params"] = params
    nz = model.get_nvar()
    zs = [sp.Symbol(f"z{i}", real=True) for i in range(nz)]
    ps = [sp.Symbol(f"p{i}", real=True) for i in range(npar)]
    L = _scalar(objective(modules, zs, ps, model, settings, 1))
    h = [_scalar(c) for c in constraints(modules, zs, ps, model, settings, 1)]
    f = [sp.sympify(e) for e in model.continuous_model(zs[model.nu:], zs[:model.nu])]
    lb = constraint_lower_bounds(modules)
    ub = constraint_upper_bounds(modules)
    return dict(model=model, params=params, zs=zs, ps=ps, L=L, h=h, f=f, lb=lb, ub=ub,
                npar=npar, nz=nz)


def synthetic_point(rng, pmap, npar, n_obs, nz):
    """A random but realistic (z, p): a smooth 5-segment path, weights near
    settings.yaml:78-92, obstacles near the ego, non-zero disc offset so the
    psi-dependence of the ellipsoid constraint is exercised."""
    p = np.zeros(npar)
    w = {"acceleration": 0.34, "angular_velocity": 0.85, "velocity": 0.55,
         "reference_velocity": 2.0, "contour": 0.05, "lag": 0.75,
         "terminal_angle": 100.0, "terminal_contouring": 10.0}
    for k, v in w.items():
        p[pmap[k]] = v * rng.uniform(0.5, 1.5)
    # path: 5 cubic segments x(t)=a t^3+b t^2+c t+d, t = s - s_start
    s0 = 0.0
    px, py, th = rng.uniform(-5, 5), rng.uniform(-5, 5), rng.uniform(-np.pi, np.pi)
    for j in range(5):
        L = rng.uniform(3.0, 6.0)
        dth = rng.uniform(-0.6, 0.6)
        c = np.array([np.cos(th), np.sin(th)])
        th1 = th + dth
        c1 = np.array([np.cos(th1), np.sin(th1)])
        # Hermite cubic between (p0, c) and (p0 + L*(c+c1)/2, c1)
        p0 = np.array([px, py])
        p1 = p0 + L * 0.5 * (c + c1)
        for ax, name in enumerate(["x", "y"]):
            d_, c_ = p0[ax], c[ax]
            # solve a L^3 + b L^2 = p1 - d - c L ; 3a L^2 + 2 b L = c1 - c
            A = np.array([[L ** 3, L ** 2], [3 * L ** 2, 2 * L]])
            rhs = np.array([p1[ax] - d_ - c_ * L, c1[ax] - c_])
            a_, b_ = np.linalg.solve(A, rhs)
            p[pmap[f"spline_{name}{j}_a"]] = a_
            p[pmap[f"spline_{name}{j}_b"]] = b_
            p[pmap[f"spline_{name}{j}_c"]] = c_
            p[pmap[f"spline_{name}{j}_d"]] = d_
        p[pmap[f"spline{j}_start"]] = s0
        s0 += L
        px, py, th = p1[0], p1[1], th1
    s_tot = s0
    if "consistency_weight" in pmap:
        p[pmap["consistency_weight"]] = rng.uniform(0.0, 0.1)
        p[pmap["prev_traj_x"]] = rng.uniform(-10, 10)
        p[pmap["prev_traj_y"]] = rng.uniform(-10, 10)
    for i in range(n_obs):
        th = rng.uniform(-np.pi, np.pi)
        p[pmap[f"lin_constraint_{i}_a1"]] = np.cos(th)
        p[pmap[f"lin_constraint_{i}_a2"]] = np.sin(th)
        p[pmap[f"lin_constraint_{i}_b"]] = rng.uniform(-5, 5)
    p[pmap["ego_disc_radius"]] = 0.325
    p[pmap["ego_disc_0_offset"]] = rng.uniform(-0.3, 0.3)
    z = np.zeros(nz)
    z[0] = rng.uniform(-2, 2)      # a
    z[1] = rng.uniform(-0.8, 0.8)  # w
    z[2] = rng.uniform(-10, 10)    # x
    z[3] = rng.uniform(-10, 10)    # y
    z[4] = rng.uniform(-np.pi, np.pi)  # psi
    z[5] = rng.uniform(0, 2.5)     # v
    z[6] = rng.uniform(0, s_tot)   # spline
    for j in range(n_obs):
        p[pmap[f"ellipsoid_obst_{j}_x"]] = z[2] + rng.uniform(-6, 6)
        p[pmap[f"ellipsoid_obst_{j}_y"]] = z[3] + rng.uniform(-6, 6)
        p[pmap[f"ellipsoid_obst_{j}_psi"]] = rng.uniform(-np.pi, np.pi)
        p[pmap[f"ellipsoid_obst_{j}_major"]] = rng.uniform(0.0, 0.6)
        p[pmap[f"ellipsoid_obst_{j}_minor"]] = rng.uniform(0.0, 0.6)
        p[pmap[f"ellipsoid_obst_{j}_chi"]] = rng.uniform(0.5, 2.0)
        p[pmap[f"ellipsoid_obst_{j}_r"]] = 0.325
    return z, p


def gen_stage_fixture(name, N, n_obs, npts, seed):
    t0 = time.time()
    S = symbolic_stage(settings_for(N, n_obs))
    zs, ps = S["zs"], S["ps"]
    nz = S["nz"]
    L = S["L"]
    dL = [sp.diff(L, v) for v in zs]
    d2L = [[sp.diff(dL[i], zs[j]) for j in range(nz)] for i in range(nz)]
    h = S["h"]
    dh = [[sp.diff(e, v) for v in zs] for e in h]
    d2h = [[[sp.diff(dh[r][i], zs[j]) for j in range(nz)] for i in range(nz)] for r in range(len(h))]
    f = S["f"]
    nu = S["model"].nu
    xs = zs[nu:] + zs[:nu]  # f is a function of (x, u); derivatives taken w.r.t. z = [u; x]
    df = [[sp.diff(e, v) for v in zs] for e in f]
    d2f = [[[sp.diff(df[r][i], zs[j]) for j in range(nz)] for i in range(nz)] for r in range(len(f))]
    args = (zs, ps)
    fL = sp.lambdify(args, [L, dL, d2L], "numpy", cse=True)
    fh = sp.lambdify(args, [h, dh, d2h], "numpy", cse=True)
    ff = sp.lambdify(args, [f, df, d2f], "numpy", cse=True)
    print(f"[{name}] symbolic build {time.time() - t0:.1f}s  npar={S['npar']} nh={len(h)}")
    pmap = dict(S["params"]._params)
    rng = np.random.default_rng(seed)
    Z, P = [], []
    out = {k: [] for k in ["L", "dL", "d2L", "h", "dh", "d2h", "f", "df", "d2f"]}
    for _ in range(npts):
        z, p = synthetic_point(rng, pmap, S["npar"], n_obs, nz)
        Z.append(z)
        P.append(p)
        a, b, c = fL(list(z), list(p))
        out["L"].append(float(a)); out["dL"].append(np.array(b, float)); out["d2L"].append(np.array(c, float))
        a, b, c = fh(list(z), list(p))
        out["h"].append(np.array(a, float)); out["dh"].append(np.array(b, float)); out["d2h"].append(np.array(c, float))
        a, b, c = ff(list(z), list(p))
        out["f"].append(np.array(a, float)); out["df"].append(np.array(b, float)); out["d2f"].append(np.array(c, float))
    lb = np.array([float(v) for v in S["lb"]])
    ub = np.array([float(v) for v in S["ub"]])
    np.savez_compressed(os.path.join(HERE, f"stage_{name}.npz"), z=np.array(Z), p=np.array(P),
                        lh=lb, uh=ub,
                        model_lb=np.array(S["model"].lower_bound, float),
                        model_ub=np.array(S["model"].upper_bound, float),
                        **{k: np.array(v) for k, v in out.items()})
    print(f"[{name}] {npts} points in {time.time() - t0:.1f}s")
    return pmap


def known_answer_maps():
    """The parameter counts the reference's own tests assert
    (solver_generator/test/test_control_modules.py:53-54, 86-87)."""
    s = {"contouring": {"num_segments": 10, "dynamic_velocity_reference": False}, "N": 20}
    m = ModuleManager()
    m.add_module(ContouringModule(s))
    m.add_module(PathReferenceVelocityModule(s))
    p = Parameters()
    define_parameters(m, p, s)
    s2 = {"n_discs": 1, "max_obstacles": 1}
    m2 = ModuleManager()
    m2.add_module(EllipsoidConstraintModule(s2))
    p2 = Parameters()
    define_parameters(m2, p2, s2)
    return {"contouring10_pathrefvel": dict(p._params), "ellipsoid1": dict(p2._params)}


def main():
    maps = {}
    maps["C2"] = gen_stage_fixture("C2", 20, 8, npts=48, seed=20251212)
    maps["C1"] = gen_stage_fixture("C1", 20, 4, npts=24, seed=20251213)
    maps["C4"], _ = parameter_map(settings_for(30, 12))
    maps["C1_no_consistency"], _ = parameter_map(settings_for(20, 4, consistency=False))
    maps.update(known_answer_maps())
    with open(os.path.join(HERE, "parameter_maps.json"), "w") as fh:
        json.dump(maps, fh, indent=1, sort_keys=True)
    print("wrote parameter_maps.json:", {k: len(v) for k, v in maps.items()})


if __name__ == "__main__":
    main()
