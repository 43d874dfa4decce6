"""The interior point's two profiles in the oracle (CPU, small slices of the bench
batches).  Each feature HPIPM's profile restates does what the full-size record says
(profiles/r05_qp_profile.txt, scripts/qp_profile.py): the conditional predictor-corrector fires and
keeps QPs off the iteration cap, the corrector's refinement runs and changes no outcome on the
unicycle batches, the primal box move changes the slack model's starts, and the robust profile has
none of them.  The oracle is test infrastructure; the GPU kernel is held to it by the parity tests."""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "scripts")]


def _solve(lay, b, **opts):
    import oracle_py
    return oracle_py.Oracle(lay, **opts).solve_batch(b.params, b.warm, b.xinit, nthreads=8)


def _parted(a, c):
    B = len(a["status"])
    dx = np.abs(a["xtraj"] - c["xtraj"]).reshape(B, -1).max(1)
    return (a["status"] != c["status"]) | ((a["status"] == 1) & (c["status"] == 1) & (dx > 1e-4))


@pytest.fixture(scope="module")
def c2():
    from parity_full import inputs
    return inputs("C2", 24)  # 24 scenes x 8 guesses of the bench batch


@pytest.fixture(scope="module")
def c2_hpipm(c2):
    return _solve(*c2)


def test_hpipm_is_the_default_profile(c2, c2_hpipm):
    r = _solve(*c2, qp_profile="hpipm")
    for k in ("status", "qp_iter", "sqp_iter", "qp_center", "qp_itref"):
        assert np.array_equal(r[k], c2_hpipm[k]), k
    assert np.array_equal(r["xtraj"], c2_hpipm["xtraj"])


def test_conditional_corrector_fires_and_keeps_qps_off_the_cap(c2, c2_hpipm):
    off = _solve(*c2, qp_cond_pred_corr=0)
    assert c2_hpipm["qp_center"].sum() > 0
    assert off["qp_center"].sum() == 0
    # bench batch: 4 solves with a capped QP with it, 150 without
    assert (off["qp_maxiter"] > 0).sum() > (c2_hpipm["qp_maxiter"] > 0).sum()


def test_refinement_runs_and_changes_no_outcome_on_the_unicycle(c2, c2_hpipm):
    off = _solve(*c2, qp_itref_corr_max=0)
    assert c2_hpipm["qp_itref"].sum() > 0
    assert off["qp_itref"].sum() == 0
    assert not _parted(c2_hpipm, off).any()


def test_box_move_changes_the_slack_models_starts():
    from parity_full import inputs
    lay, b = inputs("C5", 8)  # 8 scenes x 4 parallel solvers
    on = _solve(lay, b)
    off = _solve(lay, b, qp_init_move=0)
    # the slack's lower-bound gap is 0 at every stage: every start moves, and the interior point's
    # path with it (bench batch: 1,676 of 8,192 solves part)
    assert not np.array_equal(on["qp_iter"], off["qp_iter"])


def test_robust_profile_has_none_of_the_features(c2, c2_hpipm):
    r = _solve(*c2, qp_profile="robust")
    assert r["qp_center"].sum() == 0 and r["qp_itref"].sum() == 0
    # mu0 1 and thr0 1: fewer IPM iterations than HPIPM's mu0 10 / thr0 0.1 (bench batch 44.3 vs 53.7)
    assert r["qp_iter"].mean() < c2_hpipm["qp_iter"].mean()
