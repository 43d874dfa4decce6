"""SH-MPC (configuration_safe_horizon) solver inputs.

The reference's ScenarioConstraints module (scenario_constraints.cpp:58-110)
runs `parallel_solvers` (4, settings.yaml:48-49) copies of the main solver.
Each copy draws its own obstacle prediction samples
(onDataReceived -> IntegrateAndTranslateToMeanAndVariance, :112-131), reduces
them to 24 halfspaces per stage in the external `scenario_module`, writes them
as `disc_0_scenario_constraint_<i>_{a1,a2,b}` and solves; the lowest-cost
successful copy wins (:86-103).  The solve itself is the same batched
SQP-RTI path on the slack model (ContouringSecondOrderUnicycleModelWithSlack,
solver_model.py:274-298): one batch element per (scene, parallel solver).

`scenario_module` is not part of the reference, so the sample -> halfspace
reduction here is a restatement of its published idea, PARITY UNPINNED:
  samples   per obstacle, a Gaussian random walk around the constant-velocity
            mean (velocity noise integrated over the stages, so sample paths
            are time-correlated like an integrated process-noise model);
  halfspace for a sample q at stage k and the ego reference position p_k (the
            warm start), n = (q - p_k) / |q - p_k|, n . p <= n . q - (r_robot + r_obs);
  reduction keep the `n_constraints` halfspaces of the closest samples
            (smallest |q - p_k|), closest first.
Stage 0 carries inactive dummies (it is not part of the QP).

Slack semantics on the reference's acados path: `ocp.constraints.x0` covers
all nx states (generate_acados_solver.py:95), Solver::setXinit(State) writes
the state's slack (0, state.cpp:20-23) and the slack has zero dynamics, so the
slack stays at its initial value over the horizon and the scenario rows act
as hard constraints; a copy whose halfspaces are contradictory ends in a QP
failure, and the pick below takes another copy.

Warm start: the main solver's previous plan, shifted (Solver::initializeWarmstart,
acados_solver_interface.cpp:286-301), which the copies inherit.  In steady operation
that plan satisfied the previous step's scenario rows, so it keeps clear of the
obstacles' sample clouds; the stand-in is a kinematically tracked trajectory pushed
PLAN_CLEAR from every obstacle's mean path (synthetic._guess_trajectory, the C2
generator's guidance stand-in), the best of PLAN_TRIES passing patterns.  With the
braking plan instead (`previous_plan=False`; the reference's start-up and
after-failure case) a plan through an obstacle's sample cloud gives halfspaces
pointing every way around it, an empty polygon and an infeasible first QP.

Seeds: scene i uses `seed + i`; parallel solver s draws its samples from
`seed + i` with stream s and the previous plan's passing patterns come from stream
0, so any sub-range regenerates bit-identically.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from .layouts import Layout
from .synthetic import (DECELERATION, OBSTACLE_RADIUS, ROBOT_RADIUS, SETTINGS_WEIGHTS, _guess_trajectory, _path,
                        _path_eval)

SEED0 = 20251212
SLACK_WEIGHT = 10000.0        # settings.yaml:89
PARALLEL_SOLVERS = 4          # settings.yaml:48-49
SAMPLE_VEL_STD = 0.3          # [m/s] per-axis velocity noise integrated over the horizon
DUMMY_B = 100.0               # inactive stage-0 rows
# previous plan: clearance from the obstacle means = robot + obstacle radius + ~2.5 sigma of
# the samples' spread at the last stage (SAMPLE_VEL_STD * dt * sqrt(N))
PLAN_CLEAR = ROBOT_RADIUS + OBSTACLE_RADIUS + 0.65
PLAN_TRIES = 8
SPAWN_AHEAD, SPAWN_LAT = 16.0, 4.0


@dataclass
class ScenarioScenes:
    """Scene-level SH-MPC inputs (the mpcg_scenario_io buffers, include/mpcg.h)."""
    stage_params: np.ndarray  # (S, npar)
    state: np.ndarray         # (S, nx)
    samples: np.ndarray       # (S*P, N, M, 2), M = obstacles x samples per obstacle
    n_solvers: int
    main_warm: np.ndarray | None = None  # (S, N+1, nu+nx) or None = braking plan


@dataclass
class ScenarioBatch:
    """Inputs of n_scenes * n_solvers independent solves, solve = scene * n_solvers + solver."""
    params: np.ndarray   # (B*P, N, npar)
    warm: np.ndarray     # (B*P, N+1, nu+nx)
    xinit: np.ndarray    # (B*P, nx)
    n_scenes: int
    n_solvers: int
    scenes: ScenarioScenes | None = None


def braking_warm(x0: np.ndarray, N: int, dt: float, nvar: int = 8, decel: float = DECELERATION) -> np.ndarray:
    """Solver::initializeWithBraking (acados_solver_interface.cpp:303-342); the
    entries it does not write (the slack state) stay 0."""
    warm = np.zeros((N + 1, nvar))
    x, y, psi, v, s = (float(t) for t in x0[:5])
    a = -abs(decel)
    c, sn = np.cos(psi), np.sin(psi)
    warm[0, :7] = (a, 0.0, x, y, psi, v, s)
    for k in range(1, N + 1):
        x = x + v * dt * c
        y = y + v * dt * sn
        s = s + v * dt
        v = max(v + a * dt, 0.0)
        warm[k, :7] = (a, 0.0, x, y, psi, v, s)
    return warm


def reduce_samples(samples: np.ndarray, ref: np.ndarray, n_constraints: int, radius: float) -> np.ndarray:
    """samples (M, 2) at one stage, ref (2,) ego reference position ->
    (n_constraints, 3) rows a1 a2 b of the closest samples, closest first
    (ties: lower sample index); rows past M stay 0."""
    d = samples - ref[None, :]
    dist = np.sqrt(d[:, 0] * d[:, 0] + d[:, 1] * d[:, 1])
    order = np.argsort(dist, kind="stable")[:n_constraints]
    dd, dn = d[order], dist[order]
    n = dd / np.maximum(dn, 1e-9)[:, None]
    b = n[:, 0] * samples[order, 0] + n[:, 1] * samples[order, 1] - radius
    out = np.zeros((n_constraints, 3))
    out[:len(order), 0:2] = n
    out[:len(order), 2] = b
    return out


def previous_plan(layout: Layout, x0: np.ndarray, path, obstacles, rng) -> np.ndarray:
    """(N+1, nu+nx) warm start [a w | x y psi v s slack] along a collision-free tracked
    trajectory from x0 (stage 0 = x0, inputs inside their bounds, slack 0)."""
    N, dt = layout.N, layout.dt
    n_obs = len(obstacles)
    best = None
    signs = [1 if (j % 2) == 0 else -1 for j in range(n_obs)]
    for _ in range(PLAN_TRIES):
        pos, vel, clear = _guess_trajectory(x0[:5], path, obstacles, signs, N, dt,
                                            SETTINGS_WEIGHTS["reference_velocity"], clear=PLAN_CLEAR)
        if best is None or clear > best[2]:
            best = (pos, vel, clear)
        if clear >= PLAN_CLEAR - 0.15:
            break
        signs = list(rng.choice([-1, 1], n_obs))
    pos, vel = best[0], best[1]
    speed = np.hypot(vel[:, 0], vel[:, 1])
    psi = np.unwrap(np.concatenate([[x0[2]], np.arctan2(vel[1:, 1], vel[1:, 0])]))
    seg = np.hypot(*np.diff(pos, axis=0).T)
    warm = np.zeros((N + 1, layout.nvar))
    warm[:, 2:4] = pos
    warm[:, 4] = psi
    warm[:, 5] = speed
    warm[:, 6] = x0[4] + np.concatenate([[0.0], np.cumsum(seg)])
    warm[0, 2:7] = x0[:5]
    warm[:N, 0] = np.clip(np.diff(warm[:, 5]) / dt, -2.0, 2.0)
    warm[:N, 1] = np.clip(np.diff(warm[:, 4]) / dt, -0.8, 0.8)
    warm[N, 0:2] = warm[N - 1, 0:2]
    return warm


def make_shmpc_scenes(layout: Layout, n_scenes: int, n_solvers: int = PARALLEL_SOLVERS, n_obs: int = 12,
                      n_samples: int = 100, seed: int = SEED0, first_scene: int = 0,
                      previous_plan_warm: bool = True) -> ScenarioScenes:
    assert layout.model == "unicycle_slack" and layout.n_scen > 0
    N, dt, npar, ix = layout.N, layout.dt, layout.npar, layout.idx
    S, P, M = n_scenes, n_solvers, n_obs * n_samples
    stage_params = np.zeros((S, npar))
    state = np.zeros((S, layout.nx))
    samples = np.zeros((S * P, N, M, 2))
    main_warm = np.zeros((S, N + 1, layout.nvar)) if previous_plan_warm else None
    tk = dt * np.arange(N)
    for sc in range(S):
        rng = np.random.default_rng(seed + first_scene + sc)
        coef, starts = _path(rng, layout.n_seg)
        s_ego = rng.uniform(0.0, 1.0)
        p_on, t_on = _path_eval(coef, starts, s_ego)
        n_on = np.array([-t_on[1], t_on[0]])
        ego_pos = p_on + rng.normal(0, 0.2) * n_on
        v0 = rng.uniform(0.0, 2.0)
        psi0 = np.arctan2(t_on[1], t_on[0]) + rng.normal(0.0, 0.1)
        state[sc, :5] = (ego_pos[0], ego_pos[1], psi0, v0, s_ego)
        means = np.zeros((n_obs, N, 2))
        for j in range(n_obs):
            ahead = rng.uniform(2.0, SPAWN_AHEAD)
            lat = rng.uniform(-SPAWN_LAT, SPAWN_LAT)
            pj, tj = _path_eval(coef, starts, s_ego + ahead)
            nj = np.array([-tj[1], tj[0]])
            vj = rng.normal(0.0, 0.7, size=2)
            means[j] = (pj + lat * nj)[None, :] + vj[None, :] * tk[:, None]
        base = stage_params[sc]
        for name in ("acceleration", "angular_velocity", "velocity", "reference_velocity", "contour", "lag",
                     "terminal_angle", "terminal_contouring"):
            base[ix(name)] = SETTINGS_WEIGHTS[name]
        base[ix("slack")] = SLACK_WEIGHT
        for j in range(layout.n_seg):
            for ax, axn in enumerate("xy"):
                for ci, cn in enumerate("abcd"):
                    base[ix(f"spline_{axn}{j}_{cn}")] = coef[j, ax, ci]
            base[ix(f"spline{j}_start")] = starts[j]
        base[ix("ego_disc_0_offset")] = 0.0
        for s in range(P):
            srng = np.random.default_rng([seed + first_scene + sc, s + 1])
            # (n_obs, n_samples, N, 2): integrated velocity noise, zero at stage 0
            vel = srng.normal(0.0, SAMPLE_VEL_STD, size=(n_obs, n_samples, N, 2))
            vel[:, :, 0] = 0.0
            walk = np.cumsum(vel * dt, axis=2)
            smp = means[:, None] + walk                      # (n_obs, n_samples, N, 2)
            samples[sc * P + s] = smp.transpose(2, 0, 1, 3).reshape(N, M, 2)
        if main_warm is not None:
            obstacles = [(means[j, 0], (means[j, 1] - means[j, 0]) / dt) for j in range(n_obs)]
            main_warm[sc] = previous_plan(layout, state[sc], (coef, starts, s_ego), obstacles,
                                          np.random.default_rng([seed + first_scene + sc, 0]))
    return ScenarioScenes(stage_params=stage_params, state=state, samples=samples, n_solvers=P, main_warm=main_warm)


def prepare_scenario_host(layout: Layout, sc: ScenarioScenes, radius: float = ROBOT_RADIUS + OBSTACLE_RADIUS,
                          deceleration: float = DECELERATION) -> ScenarioBatch:
    """Host restatement of mpcg_prepare_scenario (include/mpcg.h): what
    ScenarioConstraints::optimize writes into each parallel solver before its
    solve (scenario_constraints.cpp:58-84)."""
    N, npar, nc, nx = layout.N, layout.npar, layout.n_scen, layout.nx
    S, P = sc.stage_params.shape[0], sc.n_solvers
    nv = layout.nvar
    i_scen = layout.idx("disc_0_scenario_constraint_0_a1")
    params = np.repeat(np.repeat(sc.stage_params[:, None, None, :], P, 1), N, 2).reshape(S * P, N, npar)
    warm = np.zeros((S * P, N + 1, nv))
    xinit = np.repeat(sc.state, P, 0).copy()
    for s_ in range(S):
        w = sc.main_warm[s_] if sc.main_warm is not None else braking_warm(sc.state[s_], N, layout.dt, nv,
                                                                             deceleration)
        for p_ in range(P):
            b = s_ * P + p_
            warm[b] = w
            rows = np.zeros((N, nc, 3))
            rows[0] = (0.0, 0.0, DUMMY_B)
            for k in range(1, N):
                rows[k] = reduce_samples(sc.samples[b, k], w[k, 2:4], nc, radius)
            params[b, :, i_scen:i_scen + 3 * nc] = rows.reshape(N, 3 * nc)
    return ScenarioBatch(params=params, warm=warm, xinit=xinit, n_scenes=S, n_solvers=P, scenes=sc)


def make_shmpc_batch(layout: Layout, n_scenes: int, n_solvers: int = PARALLEL_SOLVERS, n_obs: int = 12,
                     n_samples: int = 100, seed: int = SEED0, first_scene: int = 0,
                     previous_plan_warm: bool = True) -> ScenarioBatch:
    sc = make_shmpc_scenes(layout, n_scenes, n_solvers, n_obs, n_samples, seed, first_scene, previous_plan_warm)
    return prepare_scenario_host(layout, sc)


def select_lowest_cost(pobj: np.ndarray, exit_code: np.ndarray, n_solvers: int) -> np.ndarray:
    """ScenarioConstraints::optimize's pick (scenario_constraints.cpp:86-103):
    the successful copy with the lowest pobj below 1e9; -1 when none."""
    po = pobj.reshape(-1, n_solvers)
    ok = (exit_code.reshape(-1, n_solvers) == 1) & (po < 1e9)
    masked = np.where(ok, po, np.inf)
    best = np.argmin(masked, axis=1)
    return np.where(ok.any(axis=1), best, -1).astype(np.int32)
