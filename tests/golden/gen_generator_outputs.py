#!/usr/bin/env python3
"""Golden generator outputs (TEST INFRASTRUCTURE — run once in the build
container, output committed as tests/golden/generator_outputs.json).

Builds the reference's own module stacks (via gen_golden.py's imports of
/root/reference through the sympy casadi stand-in) and records what the
reference's generator would write for them, read straight from the
reference's objects — without calling the file writers, which would write
into the reference tree:

* parameter bundles (util/parameters.py:25-61; they name the generated
  setSolverParameter<Bundle> functions, generate_cpp_files.py:235-254),
* the model map rows (solver_model.py:118-128: state -> ["x", nu + i, lb, ub],
  input -> ["u", i, lb, ub]),
* solver_settings (generate_solver.py:37-46: N, nx, nu, nvar, npar).
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

import gen_golden as G  # noqa: E402
from util.parameters import Parameters  # noqa: E402
from solver_definition import define_parameters  # noqa: E402


def outputs(N, n_obs, consistency=True):
    settings = G.settings_for(N, n_obs, consistency)
    model, modules = G.tmpc_consistency_stack(settings)
    params = Parameters()
    define_parameters(modules, params, settings)
    mm = {}
    for i, st in enumerate(model.states):
        lb, ub = model.get_bounds(st)[:2]
        mm[st] = ["x", i + model.nu, float(lb), float(ub)]
    for i, u in enumerate(model.inputs):
        lb, ub = model.get_bounds(u)[:2]
        mm[u] = ["u", i, float(lb), float(ub)]
    return {
        "bundles": {k: list(v) for k, v in params.parameter_bundles.items()},
        "model_map": mm,
        "solver_settings": {"N": N, "nx": model.nx, "nu": model.nu, "nvar": model.get_nvar(),
                            "npar": params.length()},
    }


def main():
    out = {"C1": outputs(20, 4), "C2": outputs(20, 8), "C4": outputs(30, 12)}
    with open(os.path.join(HERE, "generator_outputs.json"), "w") as fh:
        json.dump(out, fh, indent=1)
    print({k: (v["solver_settings"], len(v["bundles"])) for k, v in out.items()})


if __name__ == "__main__":
    main()
