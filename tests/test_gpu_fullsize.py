"""Full-size GPU-vs-oracle parity on the bench batches (BASELINE.json configs):
C2 1024 scenes x 8 guesses, C4 2048 x 8 (one GPU's shard of 16384), C5 2048 x 4
parallel scenario solvers, C3 4096 bicycle solves, JS (the shipped jackalsimulator
solver) 4096 x 5, C1 1024 scenes.  Exit codes identical on every solve, trajectories of
successful solves within 1e-4, and failed solves that took the same path (same
RTI and interior-point iteration counts on both sides) also within 1e-4.

C5 exception: the SH-MPC slack state is pinned at 0 by the x0
bound and its zero dynamics (generate_acados_solver.py:95, solver_model.py:289-292),
so its lower-bound rows have zero gap at every stage and the QP is dual-degenerate
(the pinned rows' multipliers and the slack's dynamics multipliers trade along an
unbounded ray).  On a few QPs the interior point drifts along that ray until the
multipliers reach 1e13-1e15 and the residuals' rounding floor (one ulp of them) passes
the tolerance; whether it converges first is decided by rounding, and the solve then
ends in a QP NaN status on one side.  The test bounds their number and checks that
every disagreement is of that kind; with the previous-plan warm start (round 2) the exit
codes agree on the full batch and the same drift shows as a successful copy whose interior
point took a different path on the two sides."""
import os
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.timeout(900)
@pytest.mark.parametrize("cfg", ["C2", "C4", "C5", "C3", "JS", "C1"])
def test_fullsize_exit_agreement(cfg):
    sys.path.insert(0, os.path.join(ROOT, "scripts"))
    from parity_full import DEFAULT_SCENES, compare

    r = compare(cfg, DEFAULT_SCENES[cfg], 0)
    print(r)
    assert r["same_path_failed_dx"] is None or r["same_path_failed_dx"] <= 1e-4
    assert r["max_abs_dx_success_same_path"] <= 1e-4
    if cfg != "C5":
        assert r["max_abs_dx_success"] <= 1e-4
        assert r["exit_agreement"] == 1.0
        assert r["success_frac"] >= 0.9, r["success_frac"]
        assert r["rti_iters_per_solve"] >= 9.0
    else:
        # rounding decides the interior-point path of the dual-degenerate slack QPs: a few
        # copies end differently or, both succeeding, on different paths; bounded, and each
        # one of that kind
        assert r["exit_agreement"] >= 0.999
        for d in r["disagreeing"]:
            assert d["gpu_info"][2] == 1 or d["oracle_qp_status"] == 1, d
        assert len(r["success_dx_over_1e-4"]) <= 8, r["success_dx_over_1e-4"]
        for d in r["success_dx_over_1e-4"]:
            assert not d["same_path"], d
        assert r["success_frac"] >= 0.85, r["success_frac"]
