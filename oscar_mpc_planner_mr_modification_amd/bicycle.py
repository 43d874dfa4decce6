"""Seeded synthetic scenes of the C3 problem: the
curvature-aware bicycle (BicycleModel2ndOrderCurvatureAware) tracking a
reference path with CurvatureAwareContouring, inside static decomp halfspaces.

One scene = one control step: a 5-segment reference path, the ego state, a
set of static occupied points near the path (the costmap cells DecompUtil is
fed with, decomp_constraints.cpp:122-148) and the solver inputs the
reference's modules write before `Solver::solve()`:

* weights + spline segments for every stage         (mpc_base.cpp:23-35, contouring.cpp:52-126;
  values from mpc_planner_rosnavigation/config/settings.yaml)
* decomp halfspaces at stages 1..N-1 from the polyhedron around the path point
  of stage k-1 (decomp_constraints.cpp:52-120): stage 0 and unused rows hold
  the dummies a1 = 1, a2 = 0, b = x + 100 (decomp_constraints.h:35, .cpp:60,
  108-113).  DecompUtil's ellipsoid decomposition is external; the synthetic
  polyhedron is one separating halfspace per occupied point within range of the
  path segment of the stage, n = (o - q) / |o - q| with q the closest segment point,
  b = n . o - margin, the closest points first, at most max_constraints.
* warm start: the previous plan shifted forward (Solver::initializeWarmstart,
  acados_solver_interface.cpp:344-376), synthesised as the path followed at the
  current speed (x, y, psi on the path, a = w = delta = slack = 0).  The decomp
  polyhedra are built along the predicted speed of that plan.
  `braking_warm` (initializeWithBraking, :303-342) is the failure-recovery
  start; with it the decomp path points stop where the braking plan stops.

Seeds: scene i uses `seed + i`, so any sub-range regenerates bit-identically.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from .layouts import Layout
from .synthetic import _path, _path_eval

# mpc_planner_rosnavigation/config/settings.yaml:76-88 (weights) and :33-36
C3_WEIGHTS = {"acceleration": 0.34, "angular_velocity": 0.85, "slack": 10000.0, "velocity": 0.55,
              "reference_velocity": 2.0, "contour": 0.05, "lag": 0.75, "terminal_angle": 100.0,
              "terminal_contouring": 10.0}
DECELERATION = 3.0      # deceleration_at_infeasible
DECOMP_MARGIN = 0.5     # inflated-map margin of the synthetic occupied points
DECOMP_RANGE = 8.0      # local bounding box of DecompUtil (decomp.range)
SEED0 = 20251212


@dataclass
class C3Batch:
    params: np.ndarray   # (B, N, npar)
    warm: np.ndarray     # (B, N+1, 9) [a w slack | x y psi v delta s]
    xinit: np.ndarray    # (B, 6)


def braking_warm(x0, N, dt, decel=DECELERATION):
    """Solver::initializeWithBraking (acados_solver_interface.cpp:303-342) on the
    bicycle's variables: x, y, psi, v, spline rolled out at constant heading,
    a = -decel, w = 0; delta keeps the state value, slack 0 (initializeWithState)."""
    warm = np.zeros((N + 1, 9))
    x, y, psi, v, delta, s = x0
    a = -abs(decel)
    warm[0] = (a, 0.0, 0.0, x, y, psi, v, delta, s)
    for k in range(1, N + 1):
        x += v * dt * np.cos(psi)
        y += v * dt * np.sin(psi)
        s += v * dt
        v = max(v + a * dt, 0.0)
        warm[k] = (a, 0.0, 0.0, x, y, psi, v, delta, s)
    return warm


def path_warm(x0, coef, starts, N, dt):
    """The previous plan shifted forward: the path followed at the current speed."""
    warm = np.zeros((N + 1, 9))
    v, s0 = max(float(x0[3]), 0.0), float(x0[5])
    sk = s0 + v * dt * np.arange(N + 1)
    pos, tan = _path_eval(coef, starts, sk)
    psi = np.unwrap(np.arctan2(tan[:, 1], tan[:, 0]))
    psi += np.round((x0[2] - psi[0]) / (2 * np.pi)) * 2 * np.pi
    warm[:, 3:5] = pos
    warm[:, 5] = psi
    warm[:, 6] = v
    warm[:, 8] = sk
    warm[0, 3:9] = x0
    return warm


def make_c3_batch(layout: Layout, n_scenes: int, seed: int = SEED0, first_scene: int = 0) -> C3Batch:
    N, dt, npar, ix = layout.N, layout.dt, layout.npar, layout.idx
    nd = layout.n_scen
    params = np.zeros((n_scenes, N, npar))
    warm = np.zeros((n_scenes, N + 1, 9))
    xinit = np.zeros((n_scenes, 6))
    i_dec = ix("disc_0_decomp_0_a1")
    for sc in range(n_scenes):
        rng = np.random.default_rng(seed + first_scene + sc)
        coef, starts = _path(rng, layout.n_seg)
        s_ego = rng.uniform(0.0, 1.0)
        p_on, t_on = _path_eval(coef, starts, s_ego)
        n_on = np.array([-t_on[1], t_on[0]])
        pos = p_on + rng.normal(0, 0.2) * n_on
        v0 = rng.uniform(0.0, 3.0)
        psi0 = np.arctan2(t_on[1], t_on[0]) + rng.normal(0.0, 0.05)
        x0 = np.array([pos[0], pos[1], psi0, v0, rng.uniform(-0.1, 0.1), s_ego])
        xinit[sc] = x0
        base = np.zeros(npar)
        for name, v in C3_WEIGHTS.items():
            base[ix(name)] = v
        for j in range(layout.n_seg):
            for ax, axn in enumerate("xy"):
                for ci, cn in enumerate("abcd"):
                    base[ix(f"spline_{axn}{j}_{cn}")] = coef[j, ax, ci]
            base[ix(f"spline{j}_start")] = starts[j]
        base[ix("ego_disc_0_offset")] = 0.0
        # static occupied points: beside the path (1.2 - 4 m lateral), some ahead on it
        n_pts = int(rng.integers(10, 25))
        s_pts = s_ego + rng.uniform(-2.0, 18.0, n_pts)
        pp, tp = _path_eval(coef, starts, s_pts)
        npv = np.stack([-tp[:, 1], tp[:, 0]], 1)
        lat = rng.choice([-1.0, 1.0], n_pts) * rng.uniform(1.2, 4.0, n_pts)
        pts = pp + lat[:, None] * npv
        w = path_warm(x0, coef, starts, N, dt)
        warm[sc] = w
        params[sc] = base[None, :]
        dummy = (1.0, 0.0, x0[0] + 100.0)  # decomp_constraints.h:35, .cpp:60
        # DecompConstraints::update: path points at s advanced by the predicted speed
        # (decomp_constraints.cpp:68-82); the halfspaces of stage k come from the segment
        # between path points k-1 and k (decomp_constraints.cpp:90-106)
        s_pts_k = s_ego + dt * np.concatenate([[0.0], np.cumsum(w[:N - 1, 6])])
        cpts = _path_eval(coef, starts, s_pts_k)[0]
        for k in range(N):
            blk = np.tile(dummy, nd)
            if k >= 1:
                c0, c1 = cpts[k - 1], cpts[min(k, N - 1)]
                seg = c1 - c0
                L2 = float(seg @ seg)
                tq = np.clip(((pts - c0) @ seg) / L2, 0.0, 1.0) if L2 > 1e-12 else np.zeros(len(pts))
                q = c0[None, :] + tq[:, None] * seg[None, :]
                d = np.linalg.norm(pts - q, axis=1)
                order = np.argsort(d, kind="stable")
                rows = []
                for j in order:
                    if d[j] <= DECOMP_MARGIN + 0.05 or d[j] > DECOMP_RANGE:
                        continue
                    nrm = (pts[j] - q[j]) / d[j]
                    rows.append((nrm[0], nrm[1], float(nrm @ pts[j]) - DECOMP_MARGIN))
                    if len(rows) == nd:
                        break
                for r, row in enumerate(rows):
                    blk[3 * r:3 * r + 3] = row
            params[sc, k, i_dec:i_dec + 3 * nd] = blk
    return C3Batch(params=params, warm=warm, xinit=xinit)
