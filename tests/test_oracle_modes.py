"""The acados solver options the oracle restates beyond the default SQP-RTI loop (CPU):
the QP start (qp_solver_warm_start 2 with warm_start_first_qp off, the reference's
setting, generate_acados_solver.py:173) and solver_type SQP (one full acados SQP call,
acados_solver_interface.cpp:27-29, tol 1e-2, generate_acados_solver.py:144)."""
import numpy as np


def _batch(cfg, S, G, seed):
    from oscar_mpc_planner_mr_modification_amd.layouts import config_layout
    from oscar_mpc_planner_mr_modification_amd.synthetic import make_batch
    lay = config_layout(cfg)
    return lay, make_batch(lay, S, G, seed=seed)


def test_reference_qp_start_is_cold_in_sqp_rti(oracle_mod):
    """Every SQP-RTI QP is the first QP of its acados call, so qp_solver_warm_start 2 without
    warm_start_first_qp is the cold start bit for bit; with it the QPs start warm."""
    lay, b = _batch("C2", 3, 8, 11)
    ref = oracle_mod.Oracle(lay).solve_batch(b.params, b.warm, b.xinit)            # 2, first cold
    cold = oracle_mod.Oracle(lay, qp_warm_start=0).solve_batch(b.params, b.warm, b.xinit)
    warm = oracle_mod.Oracle(lay, qp_warm_start=2, qp_warm_first=1).solve_batch(b.params, b.warm, b.xinit)
    np.testing.assert_array_equal(ref["xtraj"], cold["xtraj"])
    np.testing.assert_array_equal(ref["qp_iter"], cold["qp_iter"])
    assert not np.array_equal(warm["qp_iter"], cold["qp_iter"])


def test_full_sqp_terminates_on_the_nlp_residuals(oracle_mod):
    lay, b = _batch("C2", 4, 8, 4711)
    orc = oracle_mod.Oracle(lay, solver_type="SQP")
    r = orc.solve_batch(b.params, b.warm, b.xinit)
    ok = r["status"] == 1
    assert ok.mean() > 0.5
    # converged: every residual of the final iterate below tol (strict, acados' test)
    for k in ("res_stat", "res_eq", "res_ineq", "res_comp"):
        assert (r[k][ok] < 1e-2).all(), k
    # more than one iteration where the RTI loop would stop at ten regardless
    assert r["sqp_iter"].max() > 1 and (r["sqp_iter"] <= 100).all()


def test_full_sqp_max_iter_status(oracle_mod):
    """nlp_solver_max_iter reached without convergence: acados' MAXITER status (2), which
    completeOneIteration passes through unchanged; with max_iter 0 nothing is solved."""
    lay, b = _batch("C2", 2, 8, 4711)
    full = oracle_mod.Oracle(lay, solver_type="SQP").solve_batch(b.params, b.warm, b.xinit)
    short = oracle_mod.Oracle(lay, solver_type="SQP", nlp_max_iter=1).solve_batch(b.params, b.warm, b.xinit)
    slow = full["sqp_iter"] > 1
    assert slow.any()
    assert (short["status"][slow & (full["status"] == 1)] == 2).all()
    assert (short["sqp_iter"] <= 1).all()
    none = oracle_mod.Oracle(lay, solver_type="SQP", nlp_max_iter=0).solve_batch(b.params, b.warm, b.xinit)
    assert (none["sqp_iter"] == 0).all() and (none["qp_iter"] == 0).all()
    np.testing.assert_array_equal(none["xtraj"], b.warm[:, :, 2:])


def _bench_scenes(first, count):
    """scenes [first, first + count) of the C2 bench batch (scripts/parity_full.py inputs)"""
    from oscar_mpc_planner_mr_modification_amd.layouts import config_layout
    from oscar_mpc_planner_mr_modification_amd.synthetic import make_batch
    lay = config_layout("C2")
    return lay, make_batch(lay, count, 8, first_scene=first)


def test_square_root_riccati_matches_the_classical_form(oracle_mod):
    """HPIPM's square-root Riccati (qp_ric_alg 1, acados' default; the oracle's default build on HPIPM's
    profile) and the classical form the kernel runs are the same recursion: same exit codes and IPM
    iterations, successful trajectories within rounding"""
    lay, b = _batch("C2", 8, 8, 5)
    sq = oracle_mod.Oracle(lay).solve_batch(b.params, b.warm, b.xinit)
    cl = oracle_mod.Oracle(lay, qp_ric_alg=0).solve_batch(b.params, b.warm, b.xinit)
    np.testing.assert_array_equal(sq["status"], cl["status"])
    ok = sq["status"] == 1
    assert ok.mean() > 0.8
    assert np.abs(sq["xtraj"] - cl["xtraj"])[ok].max() < 1e-9


def test_lq_factorisation_matches_the_cholesky_one(oracle_mod):
    """HPIPM's LQ factorisation of a stage (qp_lq_fact 2: LQ only) gives the Cholesky factor of the same
    block without forming it: on well-conditioned QPs the solves agree to rounding"""
    lay, b = _batch("C2", 8, 8, 5)
    ch = oracle_mod.Oracle(lay).solve_batch(b.params, b.warm, b.xinit)
    lq = oracle_mod.Oracle(lay, qp_lq_fact=2).solve_batch(b.params, b.warm, b.xinit)
    np.testing.assert_array_equal(ch["status"], lq["status"])
    np.testing.assert_array_equal(ch["qp_iter"], lq["qp_iter"])
    ok = ch["status"] == 1
    assert np.abs(ch["xtraj"] - lq["xtraj"])[ok].max() < 1e-9


def test_blasfeo_pivot_rule_on_diverging_qps(oracle_mod):
    """Scenes 14 and 15 of the C2 bench batch hold two solves (scene 14 guess 4, scene 15 guess 2) whose
    first QP is infeasible and diverges until a Riccati pivot turns non-positive.  The robust profile's
    rule ends that QP with the NaN status; BLASFEO's (HPIPM's profile, qp_pivot_zero 1) continues with a
    zero inverse, and the QP ends on its step length (MINSTEP) -- a QP failure either way, so the exit
    codes agree; the lq_fact switch (an LQ factorisation after the inaccurate Cholesky one) fires on
    exactly these QPs and ends them the same way (scripts/lq_fact_effect.py: 1 exit code of 102,400
    bench solves changes)"""
    lay, b = _bench_scenes(14, 2)
    nan = oracle_mod.Oracle(lay, qp_pivot_zero=0).solve_batch(b.params, b.warm, b.xinit)
    bf = oracle_mod.Oracle(lay).solve_batch(b.params, b.warm, b.xinit)
    lq = oracle_mod.Oracle(lay, qp_lq_fact=1).solve_batch(b.params, b.warm, b.xinit)
    div = np.array([4, 10])
    assert (nan["qp_status"][div] == 1).all() and (nan["status"][div] == 4).all()
    assert (bf["qp_status"][div] == 3).all() and (bf["status"][div] == 4).all()
    np.testing.assert_array_equal(nan["status"], bf["status"])
    np.testing.assert_array_equal(bf["status"], lq["status"])
    assert (lq["qp_lq"][div] >= 1).all() and lq["qp_lq"].sum() == (bf["qp_status"] == 3).sum()
