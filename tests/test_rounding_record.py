"""Rounding-sensitivity record of the C5 SH-MPC QPs and the t / lambda floor that settles it
(DESIGN.md §2.2, §3.2), CPU only.  The record is of the robust QP profile (round 4's interior
point, qp_profile="robust"), whose floor was chosen on it.

Copy 7799 of the C5 bench batch (scene 1949, parallel solver 3) reaches, in its fifth QP, the
dual-degenerate drift of the pinned slack rows: the multipliers of the slack's lower bound grow
10x every two interior-point iterations while their slacks fall towards 1e-17, and after ~45
iterations the stationarity residual is the rounding of cancelling terms of 1e20.

* Without a floor (qp_t_min = 0, the round-3 algorithm) the two kernel-agnostic oracle builds
  (HPIPM's forms, the default; the literal forms) part there: one build's residual cancels and
  its QP converges (10 RTI / 120 IPM iterations), the other's QP stops at the 50-iteration cap,
  which ends the reference's RTI loop (acados_solver_interface.cpp:105) after 5 of 10
  iterations -- 1.5e-3 apart in x.  The divergence is in the problem, not in one build.
* With the floor t, lambda >= 1e-12 after every step (qp_t_min, the default) the walk is
  bounded and all three builds (HPIPM forms, literal, the kernel's forms) take the same path to
  rounding."""
import numpy as np
import pytest


@pytest.fixture(scope="module")
def scene1949():
    from oscar_mpc_planner_mr_modification_amd.layouts import config_layout
    from oscar_mpc_planner_mr_modification_amd.scenario import make_shmpc_batch
    lay = config_layout("C5")
    return lay, make_shmpc_batch(lay, 1, first_scene=1949)


def _path(r, i):
    return int(r["status"][i]), int(r["sqp_iter"][i]), int(r["qp_iter"][i]), int(r["qp_maxiter"][i])


def test_without_the_floor_the_builds_part_on_the_dual_degenerate_copy(oracle_mod, scene1949):
    lay, b = scene1949
    a = oracle_mod.Oracle(lay, qp_profile="robust", qp_t_min=0.0).solve_batch(b.params, b.warm, b.xinit)
    c = oracle_mod.Oracle(lay, literal=True, qp_profile="robust", qp_t_min=0.0).solve_batch(b.params, b.warm, b.xinit)
    dx = np.abs(a["xtraj"] - c["xtraj"]).reshape(4, -1).max(1)
    # copies 0-2: the same result to rounding
    assert dx[:3].max() < 1e-12
    # copy 3 (= 7799): both succeed, on different paths, 1.5e-3 apart
    assert _path(a, 3) == (1, 10, 120, 0)
    assert _path(c, 3) == (1, 5, 83, 1)
    assert 1e-4 < dx[3] < 1e-2


def test_with_the_floor_every_build_takes_one_path(oracle_mod, scene1949):
    lay, b = scene1949
    runs = [oracle_mod.Oracle(lay, forms=f, qp_profile="robust").solve_batch(b.params, b.warm, b.xinit) for f in ("hpipm", "literal", "kernel")]
    for r in runs[1:]:
        np.testing.assert_array_equal(r["status"], runs[0]["status"])
        np.testing.assert_array_equal(r["qp_iter"], runs[0]["qp_iter"])
        assert np.abs(r["xtraj"] - runs[0]["xtraj"]).max() < 1e-12
    assert _path(runs[0], 3) == (1, 5, 83, 1)


def test_literal_build_agrees_elsewhere(oracle_mod):
    """away from those copies the builds agree to rounding (C2 batch)"""
    from oscar_mpc_planner_mr_modification_amd.layouts import config_layout
    from oscar_mpc_planner_mr_modification_amd.synthetic import make_batch
    lay = config_layout("C2")
    b = make_batch(lay, 4, 8, seed=20251212)
    a = oracle_mod.Oracle(lay).solve_batch(b.params, b.warm, b.xinit)
    for forms in ("literal", "kernel"):
        c = oracle_mod.Oracle(lay, forms=forms).solve_batch(b.params, b.warm, b.xinit)
        np.testing.assert_array_equal(a["status"], c["status"])
        ok = a["status"] == 1
        assert np.abs(a["xtraj"][ok] - c["xtraj"][ok]).max() < 1e-9
