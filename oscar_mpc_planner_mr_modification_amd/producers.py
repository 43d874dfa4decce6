"""Per-guess solver inputs of one control step, built from scene data (SURVEY
§8f rows 1-3).  These are the host-side module steps that run before each
`Solver::solve()` inside GuidanceConstraints::optimize.  The GPU does the
same work for a whole batch (`native.prepare_device` ->
`mpcg_prepare_device`); this module is the CPU restatement of those steps.

For every (scene, planner) pair:

* warm start     the main solver's x0 is copied to every planner
                 (`*solver = *_solver`, guidance_constraints.cpp:319-320).
                 Without a previous solution it is the braking plan
                 (acados_solver_interface.cpp:303-342).  Guided planners then
                 get x, y, psi, v at k*dt of their guidance trajectory for
                 k = 1..N-1 (initializeSolverWithGuidance, guidance_constraints.cpp:546-570)
* halfspaces     LinearizedConstraints::update / setParameters
                 (linearized_constraints.cpp:49-128, 150-189), topology mode:
                 one disc at the robot centre, radius 1e-3 + robot_radius.
                 The guess position is first projected to safety: 3 rounds of
                 Douglas-Rachford over all obstacles, anchored at obstacle 0
                 (:130-148).  The non-guided planner is updated with empty
                 data, so all its halfspaces are dummies (a1=1, a2=0,
                 b = x + 100, linearized_constraints.h:28, .cpp:54)
* ellipsoids     EllipsoidConstraints::setParameters (ellipsoid_constraints.cpp:34-86):
                 stage 0 dummies, stage k prediction k-1
* consistency    interpolatePrevTrajectoryByElapsedTime (guidance_constraints.cpp:1073-1133)
                 + setConsistencyParametersForPlanner (:986-1023), stages 1..N-2
* xinit          the ego state (Planner: setXinit(state))

The Douglas-Rachford projection lives in the external ros_tools package
(not in the reference tree).  `dr_project` restates the textbook iteration
z <- (z + R_B(R_A(z))) / 2 with the reflections ros_tools uses (projection
onto the outside of a disc along the ray towards a start pose); parity for
that step is unpinned.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional

import numpy as np

from .layouts import Layout

TOPOLOGY_RADIUS = 1e-3  # linearized_constraints.cpp:97 (`_use_guidance`)


@dataclass
class Scenes:
    """Scene-level inputs of one control step for S scenes x G planners.

    stage_params   (S, npar)  the stage-invariant parameters the other modules
                              write identically on every stage (MPCBase weights,
                              contouring spline segments, ego disc radius/offset)
    state          (S, 5)     ego state x, y, psi, v, spline
    obst           (S, n_ell, N, 5)  mode-0 prediction j of each obstacle (x, y, angle,
                              major, minor); the list is padded to max_obstacles with
                              dummies at (x+100, y+100), radius 0 (data_preparation.cpp:49-55, 147-160)
    obst_meta      (S, n_ell, 2)     radius, chi (1 for deterministic predictions)
    guidance       (S, G, N+1, 4)    guidance trajectory sampled at t = k dt: x, y, vx, vy
                                     (RosTools::Spline2D getPoint / getVelocity)
    guided         (S, G) bool       False for the non-guided T-MPC++ planner
    main_warm      (S, N+1, 7) or None  the main solver's warm start; None = braking
    prev_traj      (S, N, 2)  stored previous plan (storePreviousTrajectoryFromSolver)
    prev_elapsed   (S,)       seconds since it was stored; NaN = no previous plan
    consistency_on (S, G) bool   shouldEnableConsistencyForPlanner
    previously_selected (S, G) bool  guidance previously selected (selection weight)
    """
    stage_params: np.ndarray
    state: np.ndarray
    obst: np.ndarray
    obst_meta: np.ndarray
    guidance: np.ndarray
    guided: np.ndarray
    prev_traj: np.ndarray
    prev_elapsed: np.ndarray
    consistency_on: np.ndarray
    previously_selected: np.ndarray
    main_warm: Optional[np.ndarray] = None
    # t-mpc.warmstart_with_mpc_solution (guidance_constraints.cpp:335-338): each planner's own
    # previous output and whether its guidance existed in the previous step
    planner_xtraj: Optional[np.ndarray] = None      # (S*G, N+1, 5)
    planner_utraj: Optional[np.ndarray] = None      # (S*G, N, 2)
    existing_guidance: Optional[np.ndarray] = None  # (S, G) bool

    @property
    def n_scenes(self) -> int:
        return self.state.shape[0]

    @property
    def n_guesses(self) -> int:
        return self.guided.shape[1]


@dataclass
class Prepared:
    params: np.ndarray        # (S*G, N, npar)
    warm: np.ndarray          # (S*G, N+1, 7)
    xinit: np.ndarray         # (S*G, 5)
    prev_interp: np.ndarray   # (S, N, 2) interpolated previous plan (consistency reference)
    prev_valid: np.ndarray    # (S,) bool


def braking(state: np.ndarray, N: int, dt: float, deceleration: float) -> np.ndarray:
    """Solver::initializeWithBraking for a batch of states (S, 5) -> (S, N+1, 7)."""
    S = state.shape[0]
    warm = np.zeros((S, N + 1, 7))
    x, y, psi, v, s = (state[:, i].copy() for i in range(5))
    a = -abs(deceleration)
    warm[:, 0] = np.stack([np.full(S, a), np.zeros(S), x, y, psi, v, s], 1)
    for k in range(1, N + 1):
        x = x + v * dt * np.cos(psi)
        y = y + v * dt * np.sin(psi)
        s = s + v * dt
        v = np.maximum(v + a * dt, 0.0)
        warm[:, k] = np.stack([np.full(S, a), np.zeros(S), x, y, psi, v, s], 1)
    return warm


def _norm(d):
    # sqrt(dx*dx + dy*dy) with one rounding per operation: the device code
    # (csrc/mpcg_prepare.h) evaluates the same sequence without contraction,
    # so the inside/outside decisions and the halfspaces agree bit for bit
    return np.sqrt(d[..., 0] * d[..., 0] + d[..., 1] * d[..., 1])


def _dr_project_disc(p, c, r, start):
    """ros_tools DouglasRachford project: a point strictly inside the circle
    (c, r) goes to the circle along the ray from c towards `start`."""
    inside = _norm(p - c) < r
    sd = start - c
    out = c + sd / _norm(sd)[..., None] * r
    return np.where(inside[..., None], out, p)


def _dr_reflect(p, c, r, start):
    return 2.0 * _dr_project_disc(p, c, r, start) - p


def dr_project(pos, delta, anchor, r):
    """One Douglas-Rachford step of ros_tools douglasRachfordProjection(pos,
    delta, anchor, r, start = pos), as linearized_constraints.cpp:142-145
    calls it: pos <- (pos + R_delta(R_anchor(pos; start = pos); start = pos)) / 2,
    R = 2 P - I with P the projection onto the outside of the disc."""
    with np.errstate(invalid="ignore", divide="ignore"):
        first = _dr_reflect(pos, anchor, r, pos)
        return 0.5 * (pos + _dr_reflect(first, delta, r, pos))


def interpolate_prev(prev: np.ndarray, elapsed: np.ndarray, dt: float):
    """GuidanceConstraints::interpolatePrevTrajectoryByElapsedTime (:1073-1133)
    for a batch: prev (S, N, 2), elapsed (S,) -> (S, N, 2), valid (S,)."""
    S, N, _ = prev.shape
    out = np.zeros_like(prev)
    valid = np.isfinite(elapsed)
    for s in range(S):
        if not valid[s]:
            continue
        k_shift = int(np.floor(elapsed[s] / dt))
        alpha = (elapsed[s] - k_shift * dt) / dt
        if k_shift >= N - 1:  # critically stale: consistency disabled this step
            valid[s] = False
            continue
        for k in range(N):
            src = k + k_shift
            if src < N - 1:
                out[s, k] = (1.0 - alpha) * prev[s, src] + alpha * prev[s, src + 1]
            elif src == N - 1:
                out[s, k] = prev[s, N - 1]
            else:
                vel = (prev[s, N - 1] - prev[s, N - 2]) / dt
                extra = (src - (N - 1)) * dt + alpha * dt
                out[s, k] = prev[s, N - 1] + vel * extra
    return out, valid


def initialize_warmstart(warm, xtraj, utraj, state, shift_forward: bool):
    """Solver::initializeWarmstart(state, shift) (acados_solver_interface.cpp:344-376) on a
    copied warm start `warm` (N+1, 7) from the solver's own previous output: keep ->
    [out_0 .. out_{N-1}] with x0[N] unchanged; shift -> [state, out_2, .., out_{N-1},
    out_{N-1}, out_{N-1}] (stage 0's inputs: out_1's, the reference reads them out of
    State's range)"""
    N = utraj.shape[0]
    w = np.array(warm, float)
    for k in range(N + 1):
        if not shift_forward:
            if k < N:
                w[k, :2], w[k, 2:] = utraj[k], xtraj[k]
        else:
            src = 1 if k == 0 else (N - 1 if k >= N - 1 else k + 1)
            w[k, :2] = utraj[src]
            w[k, 2:] = state if k == 0 else xtraj[src]
    return w


def prepare_host(layout: Layout, sc: Scenes, robot_radius: float, w_consistency: float,
                 deceleration: float = 3.0, warmstart_with_mpc_solution: bool = False,
                 shift_forward: bool = False) -> Prepared:
    N, npar, dt = layout.N, layout.npar, layout.dt
    S, G = sc.n_scenes, sc.n_guesses
    ix = layout.idx
    main = braking(sc.state, N, dt, deceleration) if sc.main_warm is None else np.array(sc.main_warm, float)
    params = np.repeat(np.repeat(sc.stage_params[:, None, None, :], G, 1), N, 2)  # (S, G, N, npar)
    warm = np.repeat(main[:, None], G, 1).copy()                                    # (S, G, N+1, 7)
    # t-mpc.warmstart_with_mpc_solution: guided planners with existing guidance start from their
    # own previous output (guidance_constraints.cpp:335-338)
    own = np.zeros((S, G), bool)
    if warmstart_with_mpc_solution and sc.existing_guidance is not None and sc.planner_xtraj is not None:
        own = np.asarray(sc.guided, bool) & np.asarray(sc.existing_guidance, bool)
        for s_ in range(S):
            for g_ in range(G):
                if own[s_, g_]:
                    b = s_ * G + g_
                    warm[s_, g_] = initialize_warmstart(warm[s_, g_], sc.planner_xtraj[b], sc.planner_utraj[b],
                                                        sc.state[s_], shift_forward)
    # initializeSolverWithGuidance: k = 1..N-1
    gd = sc.guidance
    for k in range(1, N):
        g = sc.guided & ~own
        warm[:, :, k, 2] = np.where(g, gd[:, :, k, 0], warm[:, :, k, 2])
        warm[:, :, k, 3] = np.where(g, gd[:, :, k, 1], warm[:, :, k, 3])
        warm[:, :, k, 4] = np.where(g, np.arctan2(gd[:, :, k, 3], gd[:, :, k, 2]), warm[:, :, k, 4])
        warm[:, :, k, 5] = np.where(g, _norm(gd[:, :, k, 2:4]), warm[:, :, k, 5])
    # ellipsoids (EllipsoidConstraints::setParameters); disc radius/offset are in stage_params
    ne = layout.n_ell
    if ne:
        e0 = ix("ellipsoid_obst_0_x")
        blk = params[..., e0:e0 + 7 * ne].reshape(S, G, N, ne, 7)
        x0 = sc.state[:, 0][:, None, None]
        y0 = sc.state[:, 1][:, None, None]
        blk[:, :, 0, :, 0] = x0 + 50.0
        blk[:, :, 0, :, 1] = y0 + 50.0
        blk[:, :, 0, :, 2:7] = (0.0, 0.0, 0.0, 1.0, 0.1)
        pred = sc.obst[:, :, :N - 1]                       # (S, ne, N-1, 5), prediction k-1 for stage k
        stage_vals = np.concatenate([pred[..., 0:5], np.repeat(sc.obst_meta[:, :, None, 1:2], N - 1, 2),
                                     np.repeat(sc.obst_meta[:, :, None, 0:1], N - 1, 2)], -1)
        # order x y psi major minor chi r
        blk[:, :, 1:] = np.transpose(stage_vals, (0, 2, 1, 3))[:, None]
        params[..., e0:e0 + 7 * ne] = blk.reshape(S, G, N, 7 * ne)
    # topology halfspaces (LinearizedConstraints, topology mode)
    nl = layout.n_lin
    if nl:
        l0 = ix("lin_constraint_0_a1")
        blk = params[..., l0:l0 + 3 * nl].reshape(S, G, N, nl, 3)
        blk[..., 0] = 1.0
        blk[..., 1] = 0.0
        blk[..., 2] = sc.state[:, 0][:, None, None, None] + 100.0
        n_obs = min(ne, nl)
        if n_obs:
            r = TOPOLOGY_RADIUS + robot_radius
            for k in range(1, N):
                pos = warm[:, :, k, 2:4].copy()                         # (S, G, 2) ego prediction
                obs_k = sc.obst[:, :n_obs, k - 1, 0:2]                  # (S, n_obs, 2)
                anchor = obs_k[:, 0][:, None]                           # (S, 1, 2)
                for _ in range(3):
                    for i in range(n_obs):
                        pos = dr_project(pos, obs_k[:, i][:, None], anchor, r)
                diff = obs_k[:, None] - pos[:, :, None]                # (S, G, n_obs, 2)
                dist = _norm(diff)
                a1, a2 = diff[..., 0] / dist, diff[..., 1] / dist
                b = a1 * obs_k[:, None, :, 0] + a2 * obs_k[:, None, :, 1] - r
                g = sc.guided[:, :, None]
                blk[:, :, k, :n_obs, 0] = np.where(g, a1, blk[:, :, k, :n_obs, 0])
                blk[:, :, k, :n_obs, 1] = np.where(g, a2, blk[:, :, k, :n_obs, 1])
                blk[:, :, k, :n_obs, 2] = np.where(g, b, blk[:, :, k, :n_obs, 2])
        params[..., l0:l0 + 3 * nl] = blk.reshape(S, G, N, 3 * nl)
    # consistency parameters
    prev_i, valid = interpolate_prev(sc.prev_traj, sc.prev_elapsed, dt)
    if layout.consistency:
        on = sc.consistency_on & valid[:, None]
        ks = np.arange(N)
        stage_ok = (ks >= 1) & (ks <= N - 2)
        m = on[:, :, None] & stage_ok[None, None, :]
        params[..., ix("consistency_weight")] = np.where(m, w_consistency, 0.0)
        params[..., ix("prev_traj_x")] = np.where(m, prev_i[:, None, :, 0], 0.0)
        params[..., ix("prev_traj_y")] = np.where(m, prev_i[:, None, :, 1], 0.0)
    xinit = np.repeat(sc.state[:, None], G, 1)
    return Prepared(params=params.reshape(S * G, N, npar), warm=warm.reshape(S * G, N + 1, 7),
                    xinit=xinit.reshape(S * G, 5), prev_interp=prev_i, prev_valid=valid)


@dataclass
class Carried:
    """What one control step leaves for the next (mpcg_advance)."""
    main_warm: np.ndarray           # (S, N+1, 7)
    prev_traj: np.ndarray           # (S, N, 2)
    prev_elapsed: np.ndarray        # (S,)
    consistency_on: np.ndarray      # (S, G) bool
    previously_selected: np.ndarray  # (S, G) bool
    lam: Optional[np.ndarray]       # (S*G, N, nx + nh)


def advance_host(layout: Layout, best, exit_code, xtraj, utraj, warm, lam_out, state_next, guided,
                 elapsed: float, deceleration: float = 3.0, shift_forward: bool = False,
                 consistency_on_non_guided: bool = True, topology=None, topology_next=None,
                 previously_selected=None) -> Carried:
    """Bookkeeping between two control steps (include/mpcg.h, mpcg_advance):
    Planner::solveMPC warm start (planner.cpp:129-137, acados_solver_interface.cpp:344-376),
    storePreviousTrajectoryFromSolver / the selection flags (guidance_constraints.cpp:429-537, 951-984)
    and each planner's carried multipliers (reset after a failure, acados_solver_interface.cpp:186-190)."""
    N = layout.N
    S, G = guided.shape
    best = np.asarray(best)
    topo = np.tile(np.arange(G), (S, 1)) if topology is None else np.asarray(topology)
    topo_n = np.tile(np.arange(G), (S, 1)) if topology_next is None else np.asarray(topology_next)
    main = braking(state_next, N, layout.dt, deceleration)
    prev = np.zeros((S, N, 2))
    el = np.full(S, np.nan)
    cons = np.zeros((S, G), bool)
    psel = np.zeros((S, G), bool) if previously_selected is None else np.array(previously_selected, bool)
    for s in range(S):
        if best[s] < 0:
            continue
        b = s * G + int(best[s])
        xt, ut = xtraj[b], utraj[b]
        if not shift_forward:
            main[s, :N, :2] = ut
            main[s, :N, 2:] = xt[:N]
            main[s, N] = warm[b, N]
        else:
            for k in range(N + 1):
                src = 1 if k == 0 else (N - 1 if k >= N - 1 else k + 1)
                main[s, k, :2] = ut[src]
                main[s, k, 2:] = state_next[s] if k == 0 else xt[src]
        prev[s] = xt[:N, :2]
        el[s] = elapsed
        original = not guided[s, best[s]]
        sel_topo = topo[s, best[s]]
        for g in range(G):
            if guided[s, g]:
                cons[s, g] = (not original) and topo_n[s, g] == sel_topo
                psel[s, g] = (not original) and topo_n[s, g] == sel_topo
            else:
                cons[s, g] = consistency_on_non_guided and original
                psel[s, g] = False
    lam = None
    if lam_out is not None:
        lam = np.where((np.asarray(exit_code) == 1)[:, None, None], lam_out, 0.0)
    return Carried(main_warm=main, prev_traj=prev, prev_elapsed=el, consistency_on=cons,
                   previously_selected=psel, lam=lam)
