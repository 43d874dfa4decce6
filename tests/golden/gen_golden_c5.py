#!/usr/bin/env python3
"""Golden stage-function vectors of the SH-MPC problem from
the reference's own Python problem definition (TEST INFRASTRUCTURE — run once
in the build container; outputs committed under tests/golden/).

Builds `configuration_safe_horizon`
(mpc_planner_jackalsimulator/scripts/generate_jackalsimulator_solver.py:69-89):
ContouringSecondOrderUnicycleModelWithSlack (solver_model.py:274-298) +
MPCBase(a, w, slack, v) + Contouring + ScenarioConstraints(24 halfspaces with
slack, scenario_constraints.py:24-94), through the same sympy casadi stand-in
as gen_golden.py.  Output: tests/golden/stage_C5.npz and the C5 entry of
tests/golden/parameter_maps_c5.json.
"""
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import gen_golden as G  # noqa: E402  (sets up the stub and the reference paths)

import sympy as sp  # noqa: E402

from control_modules import ModuleManager  # noqa: E402
from util.parameters import Parameters  # noqa: E402
from solver_definition import (define_parameters, objective, constraints,  # noqa: E402
                               constraint_lower_bounds, constraint_upper_bounds)
from solver_model import ContouringSecondOrderUnicycleModelWithSlack  # noqa: E402
from mpc_base import MPCBaseModule  # noqa: E402
from contouring import ContouringModule  # noqa: E402
from scenario_constraints import ScenarioConstraintModule  # noqa: E402


def settings_c5(N=20):
    return {"N": N, "n_discs": 1, "max_obstacles": 12,
            "contouring": {"num_segments": 5, "dynamic_velocity_reference": False}}


def safe_horizon_stack(settings):
    modules = ModuleManager()
    model = ContouringSecondOrderUnicycleModelWithSlack()
    base = modules.add_module(MPCBaseModule(settings))
    base.weigh_variable(var_name="a", weight_names="acceleration")
    base.weigh_variable(var_name="w", weight_names="angular_velocity")
    base.weigh_variable(var_name="slack", weight_names="slack", rqt_max_value=10000.0)
    base.weigh_variable(var_name="v", weight_names=["velocity", "reference_velocity"],
                        cost_function=lambda x, w: w[0] * (x - w[1]) ** 2)
    modules.add_module(ContouringModule(settings))
    modules.add_module(ScenarioConstraintModule(settings))
    return model, modules


def main(npts=24, seed=20251214):
    t0 = time.time()
    settings = settings_c5()
    model, modules = safe_horizon_stack(settings)
    params = Parameters()
    define_parameters(modules, params, settings)
    settings["params"] = params
    npar, nz, nu = params.length(), model.get_nvar(), model.nu
    zs = [sp.Symbol(f"z{i}", real=True) for i in range(nz)]
    ps = [sp.Symbol(f"p{i}", real=True) for i in range(npar)]
    L = G._scalar(objective(modules, zs, ps, model, settings, 1))
    h = [G._scalar(c) for c in constraints(modules, zs, ps, model, settings, 1)]
    f = [sp.sympify(e) for e in model.continuous_model(zs[nu:], zs[:nu])]
    dL = [sp.diff(L, v) for v in zs]
    d2L = [[sp.diff(dL[i], zs[j]) for j in range(nz)] for i in range(nz)]
    dh = [[sp.diff(e, v) for v in zs] for e in h]
    d2h = [[[sp.diff(dh[r][i], zs[j]) for j in range(nz)] for i in range(nz)] for r in range(len(h))]
    df = [[sp.diff(e, v) for v in zs] for e in f]
    d2f = [[[sp.diff(df[r][i], zs[j]) for j in range(nz)] for i in range(nz)] for r in range(len(f))]
    fL = sp.lambdify((zs, ps), [L, dL, d2L], "numpy", cse=True)
    fh = sp.lambdify((zs, ps), [h, dh, d2h], "numpy", cse=True)
    ff = sp.lambdify((zs, ps), [f, df, d2f], "numpy", cse=True)
    pmap = dict(params._params)
    print(f"[C5] symbolic build {time.time() - t0:.1f}s npar={npar} nh={len(h)} nz={nz}")
    rng = np.random.default_rng(seed)
    Z, P = [], []
    out = {k: [] for k in ["L", "dL", "d2L", "h", "dh", "d2h", "f", "df", "d2f"]}
    for _ in range(npts):
        p = np.zeros(npar)
        for k, v in {"acceleration": 0.34, "angular_velocity": 0.85, "velocity": 0.55,
                     "reference_velocity": 2.0, "contour": 0.05, "lag": 0.75, "terminal_angle": 100.0,
                     "terminal_contouring": 10.0, "slack": 10000.0}.items():
            p[pmap[k]] = v * rng.uniform(0.5, 1.5)
        s0 = 0.0
        px, py, th = rng.uniform(-5, 5), rng.uniform(-5, 5), rng.uniform(-np.pi, np.pi)
        for j in range(5):
            Ls = rng.uniform(3.0, 6.0)
            th1 = th + rng.uniform(-0.6, 0.6)
            c0 = np.array([np.cos(th), np.sin(th)])
            c1 = np.array([np.cos(th1), np.sin(th1)])
            p0 = np.array([px, py])
            p1 = p0 + Ls * 0.5 * (c0 + c1)
            A = np.array([[Ls ** 3, Ls ** 2], [3 * Ls ** 2, 2 * Ls]])
            for ax, name in enumerate("xy"):
                a_, b_ = np.linalg.solve(A, [p1[ax] - p0[ax] - c0[ax] * Ls, c1[ax] - c0[ax]])
                p[pmap[f"spline_{name}{j}_a"]] = a_
                p[pmap[f"spline_{name}{j}_b"]] = b_
                p[pmap[f"spline_{name}{j}_c"]] = c0[ax]
                p[pmap[f"spline_{name}{j}_d"]] = p0[ax]
            p[pmap[f"spline{j}_start"]] = s0
            s0 += Ls
            px, py, th = p1[0], p1[1], th1
        p[pmap["ego_disc_0_offset"]] = rng.uniform(-0.3, 0.3)
        for i in range(24):
            tha = rng.uniform(-np.pi, np.pi)
            p[pmap[f"disc_0_scenario_constraint_{i}_a1"]] = np.cos(tha)
            p[pmap[f"disc_0_scenario_constraint_{i}_a2"]] = np.sin(tha)
            p[pmap[f"disc_0_scenario_constraint_{i}_b"]] = rng.uniform(-5, 5)
        z = np.array([rng.uniform(-2, 2), rng.uniform(-0.8, 0.8), rng.uniform(-10, 10), rng.uniform(-10, 10),
                      rng.uniform(-np.pi, np.pi), rng.uniform(0, 2.5), rng.uniform(0, s0), rng.uniform(0, 2)])
        Z.append(z)
        P.append(p)
        a, b, c = fL(list(z), list(p))
        out["L"].append(float(a)); out["dL"].append(np.array(b, float)); out["d2L"].append(np.array(c, float))
        a, b, c = fh(list(z), list(p))
        out["h"].append(np.array(a, float)); out["dh"].append(np.array(b, float)); out["d2h"].append(np.array(c, float))
        a, b, c = ff(list(z), list(p))
        out["f"].append(np.array(a, float)); out["df"].append(np.array(b, float)); out["d2f"].append(np.array(c, float))
    lb = np.array([float(v) for v in constraint_lower_bounds(modules)])
    ub = np.array([float(v) for v in constraint_upper_bounds(modules)])
    np.savez_compressed(os.path.join(HERE, "stage_C5.npz"), z=np.array(Z), p=np.array(P), lh=lb, uh=ub,
                        model_lb=np.array(model.lower_bound, float), model_ub=np.array(model.upper_bound, float),
                        **{k: np.array(v) for k, v in out.items()})
    bundles = {k: list(v) for k, v in params.parameter_bundles.items()}
    mm = {}
    for i, st in enumerate(model.states):
        lo, hi = model.get_bounds(st)[:2]
        mm[st] = ["x", i + model.nu, float(lo), float(hi)]
    for i, u in enumerate(model.inputs):
        lo, hi = model.get_bounds(u)[:2]
        mm[u] = ["u", i, float(lo), float(hi)]
    with open(os.path.join(HERE, "parameter_maps_c5.json"), "w") as fh_:
        json.dump({"C5": pmap, "C5_bundles": bundles, "C5_model_map": mm,
                   "C5_solver_settings": {"N": 20, "nx": model.nx, "nu": model.nu, "nvar": nz, "npar": npar}},
                  fh_, indent=1, sort_keys=True)
    print(f"[C5] {npts} points in {time.time() - t0:.1f}s")


if __name__ == "__main__":
    main()
