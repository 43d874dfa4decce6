"""GPU parity of the restated HPIPM warm start (qp_solver_warm_start = 2,
generate_acados_solver.py:173), of the capsule's QP memory carried between
solves (mpcg_io.qp_in / qp_out; reset on failure, acados_solver_interface.cpp:186-190)
and of the NLP residuals the kernel returns for AcadosInfo (mpcg_io.stats;
nlp_res / kkt_norm_inf, acados_solver_interface.cpp:151,164).  HIP path through
the C ABI against the C oracle on the same seeded inputs."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

X_TOL = 1e-4


@pytest.fixture(scope="module")
def dev():
    import torch
    assert torch.cuda.is_available(), "gpu test on a box without a GPU"
    return torch.device("cuda:0")


@pytest.fixture(scope="module")
def native():
    from oscar_mpc_planner_mr_modification_amd import native as nat
    return nat


def _t(dev):
    import torch
    return lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)


def _batch(cfg, S, seed):
    from oscar_mpc_planner_mr_modification_amd.layouts import config_layout
    lay = config_layout(cfg)
    if cfg == "C5":
        from oscar_mpc_planner_mr_modification_amd.scenario import make_shmpc_batch
        return lay, make_shmpc_batch(lay, S, seed=seed)
    from oscar_mpc_planner_mr_modification_amd.synthetic import make_batch
    return lay, make_batch(lay, S, 8, seed=seed)


def _check(ref, got, label):
    same = got["exit"] == ref["status"]
    ok = same & (got["exit"] == 1)
    dx = np.abs(got["xtraj"] - ref["xtraj"]).reshape(len(same), -1).max(1)
    print(f"{label}: {len(same)} solves, exit agreement {same.mean():.3f}, success {ok.mean():.2f}, "
          f"max|dx| {dx[ok].max() if ok.any() else 0:.2e}, qp iters gpu {got['info'][:, 1].mean():.1f} "
          f"oracle {ref['qp_iter'].mean():.1f}")
    assert same.all(), np.flatnonzero(~same)
    assert ok.any()
    assert dx[ok].max() <= X_TOL, dx[ok].max()
    np.testing.assert_array_equal(got["info"][:, 0], ref["sqp_iter"])


@pytest.mark.parametrize("cfg,S,seed", [("C2", 16, 20251212), ("C1", 8, 3)])
def test_warm_start_parity(native, dev, oracle_mod, cfg, S, seed):
    """qp_warm_start = 2 with warm_start_first_qp (qp_warm_first): every QP after the first
    starts from its predecessor's solution with slacks and multipliers clipped at qp_ws_thr;
    GPU == oracle."""
    lay, b = _batch(cfg, S, seed)
    t = _t(dev)
    ref = oracle_mod.Oracle(lay, qp_warm_start=2, qp_warm_first=1).solve_batch(b.params, b.warm, b.xinit)
    out = native.solve_batch_device(native.problem_from_layout(lay, qp_warm_start=2, qp_warm_first=1), t(b.params),
                                    t(b.warm), t(b.xinit))
    got = {k: v.cpu().numpy() for k, v in out.items()}
    _check(ref, got, f"{cfg} warm start")
    cold = oracle_mod.Oracle(lay, qp_warm_start=0).solve_batch(b.params, b.warm, b.xinit)
    assert not np.array_equal(cold["qp_iter"], ref["qp_iter"])   # the start matters


def test_qp_memory_carried_between_solves(native, dev, oracle_mod):
    """Two solves of the same planners: the second one's first QP starts from the QP
    memory the first one left (each side in its own opaque layout), with the carried
    multipliers; a block marked absent (NaN) starts cold like a reset capsule."""
    import torch
    lay, b = _batch("C2", 8, 515)
    t = _t(dev)
    orc = oracle_mod.Oracle(lay, qp_warm_start=2, qp_warm_first=1)
    pr = native.problem_from_layout(lay, qp_warm_start=2, qp_warm_first=1)
    ref1 = orc.solve_batch(b.params, b.warm, b.xinit, return_lam=True, return_qp=True)
    out1 = native.solve_batch_device(pr, t(b.params), t(b.warm), t(b.xinit), lam_out=True, qp_out=True)
    got1 = {k: v.cpu().numpy() for k, v in out1.items()}
    _check(ref1, got1, "call 1")
    ok = ref1["status"] == 1
    lam = np.where(ok[:, None, None], ref1["lam"], 0.0)
    q_ref = ref1["qp"].copy()
    q_gpu = out1["qp"].clone()
    q_ref[~ok, 0] = np.nan                       # failed solves: QP memory reset
    q_gpu[torch.from_numpy(~ok).to(dev), 0] = float("nan")
    ref2 = orc.solve_batch(b.params, b.warm, b.xinit, lam_in=lam, qp_in=q_ref)
    out2 = native.solve_batch_device(pr, t(b.params), t(b.warm), t(b.xinit), lam_in=t(lam), qp_in=q_gpu)
    got2 = {k: v.cpu().numpy() for k, v in out2.items()}
    _check(ref2, got2, "call 2 (QP memory)")
    # without the QP memory the second call differs (its first QP starts cold)
    ref2c = orc.solve_batch(b.params, b.warm, b.xinit, lam_in=lam)
    assert not np.array_equal(ref2c["qp_iter"][ok], ref2["qp_iter"][ok])
    # the NaN-marked (reset) solves equal a solve without any QP memory
    out2c = native.solve_batch_device(pr, t(b.params), t(b.warm), t(b.xinit), lam_in=t(lam))
    np.testing.assert_array_equal(out2c["xtraj"].cpu().numpy()[~ok], got2["xtraj"][~ok])


@pytest.mark.parametrize("cfg,ws", [("C2", 0), ("C2", 2), ("C5", 0), ("C4", 0)])
def test_nlp_residual_stats(native, dev, oracle_mod, cfg, ws):
    """mpcg_io.stats == the oracle's NLP residuals at the last linearisation point
    (stationarity, dynamics, inequality violation, complementarity)."""
    lay, b = _batch(cfg, 4 if cfg != "C5" else 8, 77)
    t = _t(dev)
    ref = oracle_mod.Oracle(lay, qp_warm_start=ws, qp_warm_first=1).solve_batch(b.params, b.warm, b.xinit)
    out = native.solve_batch_device(native.problem_from_layout(lay, qp_warm_start=ws, qp_warm_first=1), t(b.params),
                                    t(b.warm), t(b.xinit), stats=True)
    st = out["stats"].cpu().numpy()
    ex = out["exit"].cpu().numpy()
    same = ex == ref["status"]
    assert same.all()
    want = np.stack([ref["res_stat"], ref["res_eq"], ref["res_ineq"], ref["res_comp"]], 1)
    np.testing.assert_allclose(st, want, rtol=1e-6, atol=1e-9)
    assert (st >= 0).all() and np.isfinite(st).all()
