"""Seeded synthetic scenes for the batched T-MPC++ solve.

One scene = one control step of `Planner::solveMPC` on the jackal T-MPC
problem: a 5-segment reference path, the ego state, `n_obs` constant-velocity
obstacles (padded to max_obstacles with the planner's far-away dummies), the
previous plan, and G = n_guided + 1 planners (the guided ones plus the T-MPC++
non-guided one) with their guidance trajectories.  `make_scenes` returns the
scene-level data (producers.Scenes); `make_batch` turns it into per-planner
solver inputs with producers.prepare_host, i.e. exactly what the reference's
host-side modules write before `Solver::solve()`:

* weights + spline segments for every stage      (mpc_base.cpp:23-35, contouring.cpp:52-126)
* topology halfspaces from the guess trajectory    (linearized_constraints.cpp:49-189;
  radius 1e-3 + robot_radius because `_use_guidance`, robot centre, no disc,
  Douglas-Rachford projection to safety first)
* stage-0 dummies                                   (linearized_constraints.cpp:155-166,
                                                     ellipsoid_constraints.cpp:42-56)
* obstacle ellipsoids, stage k uses prediction k-1 (ellipsoid_constraints.cpp:61-86)
* consistency parameters on stages 1..N-2 of the planners whose topology
  was selected last step, from the previous plan interpolated by the elapsed
  time                                              (guidance_constraints.cpp:951-1133)
* warm start: braking for the non-guided planner    (acados_solver_interface.cpp:303-342)
  and guidance-initialised x, y, psi, v on k=1..N-1 for the guided ones
  (guidance_constraints.cpp:546-570), a/w/spline from the braking warm start.

Seeds: scene i uses `seed + i` (default seed 20251212), so any sub-range of a
batch (e.g. one GPU's shard) regenerates bit-identically.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import numpy as np

from .layouts import Layout
from .producers import Scenes, prepare_host

SETTINGS_WEIGHTS = {  # mpc_planner_jackalsimulator/config/settings.yaml:78-92
    "acceleration": 0.34, "angular_velocity": 0.85, "velocity": 0.55,
    "reference_velocity": 2.0, "contour": 0.05, "lag": 0.75,
    "terminal_angle": 100.0, "terminal_contouring": 10.0, "consistency": 0.05,
}
ROBOT_RADIUS = 0.325          # settings.yaml:38
OBSTACLE_RADIUS = 0.325       # settings.yaml:43
DECELERATION = 3.0            # settings.yaml:36 deceleration_at_infeasible
CONTROL_PERIOD = 0.05         # settings.yaml:8 control_frequency 20 Hz
SEED0 = 20251212
# clearance of the synthetic guidance trajectories from every obstacle centre: robot
# radius + obstacle radius (0.65, the ellipsoid rows' radius) + 0.25 m margin
GUIDE_CLEAR = ROBOT_RADIUS + OBSTACLE_RADIUS + 0.25
GUIDE_TRIES = 6
# initial path heading range.  guidance_constraints.cpp:564 sets psi = atan2(vy, vx) of
# the guidance velocity, which jumps by 2 pi where a guess crosses heading +-pi; the
# first QP linearised across that jump is infeasible (scripts/qp_feasibility.py), a
# reference behaviour the restated producer keeps.  The synthetic world frame is rotated
# so that scenes do not sit on that cut (pi restores uniform headings).
HEADING_SPAN = 0.5 * np.pi
IMMINENT_S, IMMINENT_R = 1.0, 1.5   # obstacles reaching the robot's position this soon are redrawn


@dataclass
class Batch:
    """Inputs of B*G independent solves, solve index = scene*G + guess."""
    params: np.ndarray   # (B*G, N, npar)   horizon-major all_parameters
    warm: np.ndarray     # (B*G, N+1, 7)    [u x] per stage (AcadosParameters::x0)
    xinit: np.ndarray    # (B*G, 5)
    guided: np.ndarray   # (B*G,) bool, False for the non-guided (T-MPC++) planner
    n_scenes: int
    n_guesses: int
    prev_traj: np.ndarray  # (B, N, 2) interpolated previous trajectory (consistency reference)
    consistency_on: np.ndarray = None       # (B*G,) bool, planners with the consistency cost
    previously_selected: np.ndarray = None  # (B*G,) bool, guidance selected in the previous step
    scenes: Scenes = None


def _path(rng, n_seg):
    """Cubic Hermite segments through a random smooth curve: segment length
    U[3,6] m, heading change U[-0.6, 0.6] rad per segment."""
    coef = np.zeros((n_seg, 2, 4))
    starts = np.zeros(n_seg)
    px, py = rng.uniform(-5, 5), rng.uniform(-5, 5)
    # world frame: paths start heading within +-pi/2 of the x axis, away from the branch
    # cut of the atan2 that initializeSolverWithGuidance uses for psi (see HEADING_SPAN)
    th = rng.uniform(-HEADING_SPAN, HEADING_SPAN)
    s0 = 0.0
    for j in range(n_seg):
        L = rng.uniform(3.0, 6.0)
        th1 = th + rng.uniform(-0.6, 0.6)
        c0 = np.array([np.cos(th), np.sin(th)])
        c1 = np.array([np.cos(th1), np.sin(th1)])
        p0 = np.array([px, py])
        p1 = p0 + L * 0.5 * (c0 + c1)
        A = np.array([[L ** 3, L ** 2], [3 * L ** 2, 2 * L]])
        for ax in range(2):
            a_, b_ = np.linalg.solve(A, [p1[ax] - p0[ax] - c0[ax] * L, c1[ax] - c0[ax]])
            coef[j, ax] = (a_, b_, c0[ax], p0[ax])
        starts[j] = s0
        s0 += L
        px, py, th = p1[0], p1[1], th1
    return coef, starts


def _path_eval(coef, starts, s):
    """Plain (un-glued) piecewise evaluation used only to place scene objects;
    `s` scalar or array."""
    s = np.asarray(s, dtype=float)
    j = np.clip(np.searchsorted(starts, s, side="right") - 1, 0, len(starts) - 1)
    t = (s - starts[j])[..., None]
    a, b, c, d = coef[j, :, 0], coef[j, :, 1], coef[j, :, 2], coef[j, :, 3]
    pos = ((a * t + b) * t + c) * t + d
    der = (3 * a * t + 2 * b) * t + c
    return pos, der / np.linalg.norm(der, axis=-1, keepdims=True)


def _braking(x0, N, dt):
    """Solver::initializeWithBraking (acados_solver_interface.cpp:303-342)."""
    warm = np.zeros((N + 1, 7))
    x, y, psi, v, s = x0
    a = -abs(DECELERATION)
    warm[0] = (a, 0.0, x, y, psi, v, s)
    for k in range(1, N + 1):
        x += v * dt * np.cos(psi)
        y += v * dt * np.sin(psi)
        s += v * dt
        v = max(v + a * dt, 0.0)
        warm[k] = (a, 0.0, x, y, psi, v, s)
    return warm


def _clear_path(pts, times, opos, ovel, dt, clear, sweeps=6):
    """Push every sample of `pts` (at `times`) out to `clear` metres from each obstacle's
    position at that time and one stage earlier (the prediction the solver's
    constraints use at a stage, ellipsoid_constraints.cpp:66-70)."""
    pts = pts.copy()
    for _ in range(sweeps):
        moved = False
        for tk in (times - dt, times):
            ob = opos[None, :, :] + ovel[None, :, :] * np.maximum(tk, 0.0)[:, None, None]  # (T, J, 2)
            d = pts[:, None, :] - ob
            dist = np.sqrt((d * d).sum(-1))
            j = np.argmin(dist, 1)
            dm = dist[np.arange(len(pts)), j]
            bad = dm < clear
            if bad.any():
                moved = True
                dv = d[np.arange(len(pts)), j] / np.maximum(dm, 1e-9)[:, None]
                pts[bad] = ob[np.arange(len(pts)), j][bad] + dv[bad] * clear
        if not moved:
            break
    return pts


def _min_clearance(pos, opos, ovel, dt):
    """smallest distance of the stage samples k = 1..N to the obstacles at t = (k-1) dt and k dt"""
    N = len(pos) - 1
    m = np.inf
    for off in (1, 0):
        t = (np.arange(1, N + 1) - off) * dt
        ob = opos[None] + ovel[None] * t[:, None, None]
        d = pos[1:, None, :] - ob
        m = min(m, float(np.sqrt((d * d).sum(-1)).min()))
    return m


def _guess_trajectory(ego, tangent_path, obstacles, signs, N, dt, vref, clear=None):
    """A collision-free, kinematically consistent guidance trajectory (stand-in for the
    external guidance_planner's space-time PRM output): nominal progress along the
    path towards v_ref, a lateral offset that passes obstacle j on side signs[j]
    (+1 left, -1 right), the desired path pushed out to a clearance from every
    obstacle in space-time, then tracked by a pure-pursuit unicycle inside the input
    bounds from the current state (guidance_planner's search starts from the robot's
    state and only returns collision-free trajectories).
    Returns positions and velocities at t = k*dt, k = 0..N, and the smallest clearance
    of the stage samples from the obstacles (the constraints' and the physical time).
    `clear`: the clearance the desired path is pushed out to (default GUIDE_CLEAR + 0.3)."""
    coef, starts, s_ego = tangent_path
    CLEAR = 0.8
    fine = np.linspace(0, N * dt, 8 * N + 1)
    # progress: start at the ego speed, accelerate at 1 m/s^2 towards v_ref
    v0 = ego[3]
    vt = np.minimum(v0 + 1.0 * fine, max(vref, v0))
    s_nom = s_ego + np.concatenate([[0.0], np.cumsum(0.5 * (vt[1:] + vt[:-1]) * np.diff(fine))])
    nom, tan = _path_eval(coef, starts, s_nom)
    nrm = np.stack([-tan[:, 1], tan[:, 0]], 1)
    off = np.zeros(len(fine))
    for j, (op, ov) in enumerate(obstacles):
        ob = op[None, :] + ov[None, :] * fine[:, None]
        d = np.linalg.norm(nom - ob, axis=1)
        ic = int(np.argmin(d))
        lat = float(np.sum((ob[ic] - nom[ic]) * nrm[ic]))
        want = lat + signs[j] * (CLEAR + 0.4)
        if signs[j] * want < 0:  # already on the requested side with margin
            continue
        off += want * np.exp(-0.5 * ((fine - fine[ic]) / 1.2) ** 2) * (1.0 - np.exp(-fine / 0.8))
    desired = nom + off[:, None] * nrm
    desired = desired - desired[0] + ego[:2]
    if obstacles:
        opos = np.array([o[0] for o in obstacles])
        ovel = np.array([o[1] for o in obstacles])
        desired = _clear_path(desired, fine, opos, ovel, dt, GUIDE_CLEAR + 0.3 if clear is None else clear)
    # track the desired path with a pure-pursuit unicycle inside the input
    # bounds (|a| <= 2, |w| <= 0.8), so the guess is kinematically reachable
    # from the current state, as guidance_planner's start-state-aware search is
    h = float(fine[1] - fine[0])
    x, y, psi, v = float(ego[0]), float(ego[1]), float(ego[2]), float(ego[3])
    traj = np.zeros_like(desired)
    des = desired.tolist()
    vtl = vt.tolist()
    nf = len(fine)
    for i in range(nf):
        traj[i, 0] = x
        traj[i, 1] = y
        look = max(0.6, 0.6 * v)
        j = min(nf - 1, i + int(math.ceil(look / max(vtl[i], 0.3) / h - 1e-9)))
        tx, ty = des[j][0] - x, des[j][1] - y
        alpha = math.atan2(ty, tx) - psi
        alpha = (alpha + math.pi) % (2 * math.pi) - math.pi
        w = min(0.8, max(-0.8, 2.0 * max(v, 0.3) * math.sin(alpha) / max(math.hypot(tx, ty), 0.3)))
        a = min(2.0, max(-2.0, 2.0 * (vtl[i] - v)))
        x += h * v * math.cos(psi)
        y += h * v * math.sin(psi)
        psi += h * w
        v = max(v + h * a, 0.0)
    vel = np.gradient(traj, fine, axis=0)
    idx = np.searchsorted(fine, np.arange(N + 1) * dt - 1e-12)
    pos = traj[idx]
    clear = _min_clearance(pos, opos, ovel, dt) if obstacles else np.inf
    return pos, vel[idx], clear


def make_scenes(layout: Layout, n_scenes: int, n_guesses: int = 8, n_obs: int | None = None,
                seed: int = SEED0, first_scene: int = 0) -> Scenes:
    """Scene-level inputs (producers.Scenes) of scenes [first_scene, first_scene + n_scenes)."""
    N, dt = layout.N, layout.dt
    npar, ix = layout.npar, layout.idx
    ne = layout.n_ell
    n_obs = ne if n_obs is None else n_obs
    assert n_obs <= ne
    G = n_guesses
    S = n_scenes
    stage_params = np.zeros((S, npar))
    state = np.zeros((S, 5))
    obst = np.zeros((S, ne, N, 5))
    meta = np.zeros((S, ne, 2))
    guidance = np.zeros((S, G, N + 1, 4))
    guided = np.zeros((S, G), bool)
    guided[:, :G - 1] = True
    prev = np.zeros((S, N, 2))
    elapsed = np.full(S, np.nan)
    cons_on = np.zeros((S, G), bool)
    prev_sel = np.zeros((S, G), bool)
    for sc in range(S):
        rng = np.random.default_rng(seed + first_scene + sc)
        coef, starts = _path(rng, layout.n_seg)
        s_ego = rng.uniform(0.0, 1.0)
        p_on, t_on = _path_eval(coef, starts, s_ego)
        n_on = np.array([-t_on[1], t_on[0]])
        ego_pos = p_on + rng.normal(0, 0.2) * n_on
        v0 = rng.uniform(0.0, 2.0)
        psi0 = np.arctan2(t_on[1], t_on[0]) + rng.normal(0.0, 0.1)
        x0 = np.array([ego_pos[0], ego_pos[1], psi0, v0, s_ego])
        state[sc] = x0
        obstacles = []
        for j in range(n_obs):
            # an obstacle on a collision course with the robot's current position inside
            # the first second is redrawn (the scene would start in an unavoidable
            # collision, which the reference's planner never faces in steady operation)
            for _ in range(20):
                ahead = rng.uniform(2.0, 10.0)
                lat = rng.uniform(-3.0, 3.0)
                pj, tj = _path_eval(coef, starts, s_ego + ahead)
                nj = np.array([-tj[1], tj[0]])
                op, ov = pj + lat * nj, rng.normal(0.0, 0.7, size=2)
                tt = np.linspace(0.0, IMMINENT_S, 11)
                if np.min(np.linalg.norm(op[None] + ov[None] * tt[:, None] - ego_pos[None], axis=1)) >= IMMINENT_R:
                    break
            obstacles.append((op, ov))
        # stage-invariant module parameters (mpc_base.cpp:23-35, contouring.cpp:52-126,
        # ellipsoid_constraints.cpp:38-40)
        base = stage_params[sc]
        for name in ("acceleration", "angular_velocity", "velocity", "reference_velocity", "contour", "lag",
                     "terminal_angle", "terminal_contouring"):
            base[ix(name)] = SETTINGS_WEIGHTS[name]
        for j in range(layout.n_seg):
            for ax, axn in enumerate("xy"):
                for ci, cn in enumerate("abcd"):
                    base[ix(f"spline_{axn}{j}_{cn}")] = coef[j, ax, ci]
            base[ix(f"spline{j}_start")] = starts[j]
        base[ix("ego_disc_radius")] = ROBOT_RADIUS
        base[ix("ego_disc_0_offset")] = 0.0
        # obstacles: constant-velocity deterministic predictions (data_preparation.cpp:60-81),
        # padded with dummies at (x + 100, y + 100), radius 0
        for j in range(ne):
            if j < n_obs:
                op, ov = obstacles[j]
                obst[sc, j, :, 0:2] = op[None, :] + ov[None, :] * dt * np.arange(N)[:, None]
                meta[sc, j] = (OBSTACLE_RADIUS, 1.0)
            else:
                obst[sc, j, :, 0:2] = (x0[0] + 100.0, x0[1] + 100.0)
                meta[sc, j] = (0.0, 1.0)
        # previous plan stored one control period ago: a constant-speed roll-out
        # along the heading; one scene in ten is a first step without one
        if rng.uniform() >= 0.1:
            vp = max(v0, 0.5)
            dirv = np.array([np.cos(psi0), np.sin(psi0)])
            for k in range(N):
                prev[sc, k] = ego_pos + vp * (k * dt - CONTROL_PERIOD) * dirv
            elapsed[sc] = CONTROL_PERIOD
            sel = int(rng.integers(0, G))
            if sel == G - 1:
                cons_on[sc, G - 1] = True       # consistency_on_non_guided_planner: true (settings.yaml)
            else:
                cons_on[sc, sel] = True         # the guided planner of the selected topology
                prev_sel[sc, sel] = True
        for g in range(G - 1):
            signs = [1 if (g >> (j % 3)) & 1 else -1 for j in range(n_obs)]
            grng = np.random.default_rng(seed + 7919 * ((first_scene + sc) * G + g))
            if g >= 8:
                signs = list(grng.choice([-1, 1], n_obs))
            # guidance_planner returns only collision-free homotopies: a passing pattern
            # whose tracked trajectory cannot keep the clearance is replaced by another
            # one (random side per obstacle), the best of GUIDE_TRIES kept otherwise
            best = None
            for _ in range(GUIDE_TRIES):
                pos, vel, clear = _guess_trajectory(x0, (coef, starts, s_ego), obstacles, signs, N, dt,
                                                    SETTINGS_WEIGHTS["reference_velocity"])
                if best is None or clear > best[2]:
                    best = (pos, vel, clear)
                if clear >= GUIDE_CLEAR:
                    break
                signs = list(grng.choice([-1, 1], n_obs))
            guidance[sc, g, :, 0:2] = best[0]
            guidance[sc, g, :, 2:4] = best[1]
    return Scenes(stage_params=stage_params, state=state, obst=obst, obst_meta=meta, guidance=guidance,
                  guided=guided, prev_traj=prev, prev_elapsed=elapsed, consistency_on=cons_on,
                  previously_selected=prev_sel, main_warm=None)


def concat_scenes(parts) -> Scenes:
    return Scenes(**{f: np.concatenate([getattr(p, f) for p in parts]) for f in
                     ("stage_params", "state", "obst", "obst_meta", "guidance", "guided", "prev_traj",
                      "prev_elapsed", "consistency_on", "previously_selected")}, main_warm=None)


def make_batch(layout: Layout, n_scenes: int, n_guesses: int = 8, n_obs: int | None = None,
               seed: int = SEED0, first_scene: int = 0, consistency: bool = True, workers: int = 1) -> Batch:
    """Scenes [first_scene, first_scene + n_scenes) x n_guesses planners, as
    per-planner solver inputs.  With workers > 1 the scenes are generated in a
    process pool; per-scene seeding makes the result identical to the serial one."""
    if workers > 1 and n_scenes >= 2 * workers:
        from concurrent.futures import ProcessPoolExecutor

        chunks = np.array_split(np.arange(n_scenes), workers)
        with ProcessPoolExecutor(max_workers=workers) as ex:
            futs = [ex.submit(make_scenes, layout, len(c), n_guesses, n_obs, seed, first_scene + int(c[0]))
                    for c in chunks if len(c)]
            sc = concat_scenes([f.result() for f in futs])
    else:
        sc = make_scenes(layout, n_scenes, n_guesses, n_obs, seed, first_scene)
    if not consistency:
        sc.consistency_on[:] = False
    p = prepare_host(layout, sc, ROBOT_RADIUS, SETTINGS_WEIGHTS["consistency"], DECELERATION)
    G = n_guesses
    return Batch(params=p.params, warm=p.warm, xinit=p.xinit, guided=sc.guided.reshape(-1), n_scenes=n_scenes,
                 n_guesses=G, prev_traj=p.prev_interp,
                 consistency_on=(sc.consistency_on & p.prev_valid[:, None]).reshape(-1),
                 previously_selected=sc.previously_selected.reshape(-1), scenes=sc)


def step_scenes(layout: Layout, sc: Scenes, state_next: np.ndarray, carried) -> Scenes:
    """The next control step of the synthetic scenes, one integrator step
    (dt) later: obstacle predictions and guidance trajectories move on by one
    sample (constant-velocity extrapolation at the end), the ego state is
    `state_next`, and the planner bookkeeping comes from `carried`
    (producers.Carried / the mpcg_advance outputs, host arrays)."""
    obst = np.concatenate([sc.obst[:, :, 1:], 2 * sc.obst[:, :, -1:] - sc.obst[:, :, -2:-1]], 2)
    obst[..., 2:5] = sc.obst[..., 2:5]
    gd = np.concatenate([sc.guidance[:, :, 1:], sc.guidance[:, :, -1:]], 2)
    gd[:, :, -1, 0:2] = sc.guidance[:, :, -1, 0:2] + layout.dt * sc.guidance[:, :, -1, 2:4]
    return Scenes(stage_params=sc.stage_params.copy(), state=np.array(state_next, float), obst=obst,
                  obst_meta=sc.obst_meta.copy(), guidance=gd, guided=sc.guided.copy(),
                  prev_traj=np.array(carried.prev_traj, float), prev_elapsed=np.array(carried.prev_elapsed, float),
                  consistency_on=np.array(carried.consistency_on, bool),
                  previously_selected=np.array(carried.previously_selected, bool),
                  main_warm=np.array(carried.main_warm, float))
