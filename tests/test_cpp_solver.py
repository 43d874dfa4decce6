"""The drop-in C++ `MPCPlanner::Solver` (include/mpc_planner_solver/,
csrc/host/) and the solver-directory generator (codegen.py).

CPU: generated files against the reference's own generator outputs
(tests/golden/generator_outputs.json, parameter_maps.json) and the C++
plumbing test (tests/cpp/test_solver.cpp, mirroring what the reference's
mpc_planner_solver/test/test_solver.cpp checks).
GPU: Solver::solve(), carried multipliers across two control steps,
SolverBatch and the one-iteration interface against the oracle.
"""
import json
import os
import subprocess

import numpy as np
import pytest
import yaml

from oscar_mpc_planner_mr_modification_amd import codegen
from oscar_mpc_planner_mr_modification_amd.layouts import config_layout

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


@pytest.fixture(scope="module")
def gen_out():
    with open(os.path.join(GOLDEN, "generator_outputs.json")) as fh:
        return json.load(fh)


@pytest.fixture(scope="module")
def cpp_build():
    from oscar_mpc_planner_mr_modification_amd import _build
    return _build.build_cpp("C2")


@pytest.fixture(scope="module")
def cpp_build_c5():
    from oscar_mpc_planner_mr_modification_amd import _build
    return _build.build_cpp("C5")


@pytest.fixture(scope="module")
def cpp_build_c3():
    from oscar_mpc_planner_mr_modification_amd import _build
    return _build.build_cpp("C3")


@pytest.fixture(scope="module")
def cpp_build_js():
    from oscar_mpc_planner_mr_modification_amd import _build
    return _build.build_cpp("JS")


def _env(d):
    env = dict(os.environ)
    env["MPCG_SOLVER_DIR"] = d
    env["MPCG_SETTINGS"] = os.path.join(d, "settings.yaml")
    return env


@pytest.mark.parametrize("cfg", ["C1", "C2", "C4"])
def test_generated_maps_match_reference_generator(tmp_path, gen_out, cfg):
    lay = config_layout(cfg)
    codegen.generate(lay, str(tmp_path))
    pm = yaml.safe_load(open(tmp_path / "parameter_map.yaml"))
    maps = json.load(open(os.path.join(GOLDEN, "parameter_maps.json")))
    assert pm.pop("num parameters") == lay.npar
    assert pm == maps[cfg]
    assert yaml.safe_load(open(tmp_path / "model_map.yaml")) == gen_out[cfg]["model_map"]
    assert yaml.safe_load(open(tmp_path / "solver_settings.yaml")) == gen_out[cfg]["solver_settings"]
    assert lay.bundles == gen_out[cfg]["bundles"]


def test_generated_setters_cover_every_bundle(tmp_path, gen_out):
    lay = config_layout("C2")
    codegen.generate(lay, str(tmp_path))
    hdr = open(tmp_path / "include" / "mpc_planner_solver" / "mpc_planner_parameters.h").read()
    src = open(tmp_path / "mpc_planner_parameters.cpp").read()
    for bundle, idx in gen_out["C2"]["bundles"].items():
        fn = "setSolverParameter" + bundle.replace("_", " ").title().replace(" ", "")
        assert f"void {fn}(int k, AcadosParameters& params, const double value, int index" in hdr
        assert f"void {fn}(" in src
    assert "setSolverParameterSplineXA" in hdr and "setSolverParameterEllipsoidObstPsi" in hdr


def test_cpp_solver_plumbing(cpp_build):
    r = subprocess.run([cpp_build["test"], "plumbing"], env=_env(cpp_build["dir"]), capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "OK plumbing" in r.stdout


def test_cpp_solver_plumbing_slack_model(cpp_build_c5):
    """The same drop-in compiled for the SH-MPC solver (nx 6, scenario rows)."""
    r = subprocess.run([cpp_build_c5["test"], "plumbing"], env=_env(cpp_build_c5["dir"]), capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "OK plumbing" in r.stdout


def test_cpp_solver_plumbing_bicycle_model(cpp_build_c3):
    """The same drop-in compiled for the C3 solver (curvature-aware bicycle, nu 3,
    decomp halfspaces): generated decomp setters, slack input, model_map inputs."""
    r = subprocess.run([cpp_build_c3["test"], "plumbing"], env=_env(cpp_build_c3["dir"]), capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "OK plumbing" in r.stdout


def test_cpp_solver_rejects_mismatched_settings(cpp_build, tmp_path):
    """A solver directory whose dimensions differ from the compiled ones is
    refused at construction (the reference exits when its capsule cannot be
    created, acados_solver_interface.cpp:35-39)."""
    codegen.generate(config_layout("C1"), str(tmp_path))
    r = subprocess.run([cpp_build["test"], "plumbing"], env=_env(str(tmp_path)), capture_output=True, text=True,
                       timeout=120)
    assert r.returncode != 0
    assert "does not match the compiled dimensions" in r.stderr


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", ["C2", "C5", "C3", "JS"])
def test_cpp_solver_on_gpu_matches_oracle(cpp_build, cpp_build_c5, cpp_build_c3, cpp_build_js, oracle_mod, tmp_path,
                                          cfg):
    from oscar_mpc_planner_mr_modification_amd.bicycle import make_c3_batch
    from oscar_mpc_planner_mr_modification_amd.scenario import make_shmpc_batch
    from oscar_mpc_planner_mr_modification_amd.synthetic import make_batch
    lay = config_layout(cfg)
    if cfg == "C2":
        b = make_batch(lay, 3, 8, seed=8080)
    elif cfg == "JS":
        # the shipped jackalsimulator solver: 4 guided planners + the non-guided one
        b, cpp_build = make_batch(lay, 3, 5, seed=8080), cpp_build_js
    elif cfg == "C5":
        b, cpp_build = make_shmpc_batch(lay, 6, seed=8080), cpp_build_c5
    else:
        b, cpp_build = make_c3_batch(lay, 6, seed=8080), cpp_build_c3
    B, N, nx, nu = b.params.shape[0], lay.N, lay.nx, lay.nu
    fin = tmp_path / "in.bin"
    with open(fin, "wb") as fh:
        np.array([B, N, lay.npar, 10], np.int32).tofile(fh)
        for a in (b.params, b.warm, b.xinit):
            np.ascontiguousarray(a, np.float64).tofile(fh)
    fout = tmp_path / "out.bin"
    r = subprocess.run([cpp_build["test"], "solve", str(fin), str(fout)], env=_env(cpp_build["dir"]),
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    NE = 9  # pobj, exit, sqp_iter, qp_status, nlp_res, kkt_norm_inf, elapsed_time, solvetime, min_time
    rec = (N + 1) * nx + N * nu + NE
    raw = np.fromfile(fout, np.float64).reshape(-1, B, rec)
    assert raw.shape[0] == 5  # solve x2, batch x2, one-iteration

    def split(a):
        x0 = (N + 1) * nx + N * nu
        e = a[:, x0:]
        return dict(xtraj=a[:, :(N + 1) * nx].reshape(B, N + 1, nx), utraj=a[:, (N + 1) * nx:x0].reshape(B, N, nu),
                    pobj=e[:, 0], exit=e[:, 1].astype(np.int32), sqp_iter=e[:, 2].astype(np.int32),
                    qp_status=e[:, 3].astype(np.int32), nlp_res=e[:, 4], kkt=e[:, 5], elapsed=e[:, 6],
                    solvetime=e[:, 7], min_time=e[:, 8])

    step1, step2, batch1, batch2, oneit = (split(raw[i]) for i in range(5))
    orc = oracle_mod.Oracle(lay)
    ref1 = orc.solve_batch(b.params, b.warm, b.xinit, return_lam=True)
    lam = np.where((ref1["status"] == 1)[:, None, None], ref1["lam"], 0.0)
    ref2 = orc.solve_batch(b.params, b.warm, b.xinit, lam_in=lam)
    for got, ref, label in ((step1, ref1, "solve step 1"), (step2, ref2, "solve step 2")):
        np.testing.assert_array_equal(got["exit"], ref["status"], err_msg=label)
        ok = got["exit"] == 1
        assert ok.any()
        assert np.abs(got["xtraj"][ok] - ref["xtraj"][ok]).max() <= 1e-4, label
        # AcadosInfo: executed RTI iterations, the acados QP status, and nlp_res = kkt_norm_inf =
        # max of the NLP residuals at the last linearisation point
        np.testing.assert_array_equal(got["sqp_iter"], ref["sqp_iter"], err_msg=label)
        np.testing.assert_array_equal(got["qp_status"], ref["qp_status"], err_msg=label)
        nres = np.max(np.stack([ref["res_stat"], ref["res_eq"], ref["res_ineq"], ref["res_comp"]]), 0)
        np.testing.assert_allclose(got["nlp_res"], nres, rtol=1e-6, atol=1e-9, err_msg=label)
        np.testing.assert_array_equal(got["kkt"], got["nlp_res"])
        assert (got["elapsed"] > 0).all() and (got["min_time"] <= got["elapsed"]).all()
        assert (got["solvetime"] >= got["elapsed"]).all()
    # one launch for all planners == one solve() per planner (bit-identical)
    timing = ("elapsed", "solvetime", "min_time")
    for a, c in ((batch1, step1), (batch2, step2)):
        for k in a:
            if k not in timing:
                np.testing.assert_array_equal(a[k], c[k], err_msg=k)
    # solveOneIteration x iterations == solve()
    for k in oneit:
        if k not in timing:
            np.testing.assert_array_equal(oneit[k], step1[k], err_msg=k)


def test_module_call_sites_compile_and_land(cpp_build):
    """Boundary test: the reference modules' setParameters / glue call shapes
    (mpc_base.cpp, contouring.cpp, linearized_constraints.cpp, ellipsoid_constraints.cpp,
    guidance_constraints.cpp; restated in tests/cpp/test_module_callsites.cpp since the
    module TUs need ROS / ros_tools / Eigen / yaml-cpp) compile against the drop-in headers
    and write the slots the generated parameter map names.  CPU only."""
    from oscar_mpc_planner_mr_modification_amd import _build
    src = os.path.join(os.path.dirname(__file__), "cpp", "test_module_callsites.cpp")
    exe = os.path.join(cpp_build["dir"], "test_module_callsites")
    inc = [f"-I{os.path.join(cpp_build['dir'], 'include')}", f"-I{_build.INCLUDE}"]
    subprocess.run(["g++", "-std=c++17", "-O1", "-Wall", "-Wextra", "-Werror"] + inc +
                   [src, "-o", exe, f"-L{cpp_build['dir']}", "-lmpc_planner_solver", f"-L{_build.PKG}", "-lmpcg",
                    f"-Wl,-rpath,{cpp_build['dir']}:{_build.PKG}"], check=True, timeout=300)
    r = subprocess.run([exe], env=_env(cpp_build["dir"]), capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "OK module call sites" in r.stdout
