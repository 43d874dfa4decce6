"""TEST INFRASTRUCTURE — plain-loop restatement of the per-guess input
producers, the checker for producers.prepare_host and
for the device kernel mpcg_prepare.  Only tests/ may import it.

One (scene, planner, stage) at a time, following the reference sources:
  braking                acados_solver_interface.cpp:303-342
  guidance warm start    guidance_constraints.cpp:546-570
  own warm start         t-mpc.warmstart_with_mpc_solution, guidance_constraints.cpp:335-338 ->
                         Solver::initializeWarmstart, acados_solver_interface.cpp:344-376
  topology halfspaces    linearized_constraints.cpp:49-128 (update), 130-148
                         (projectToSafety), 150-189 (setParameters)
  Douglas-Rachford       ros_tools (external, not in /root/reference): the
                         textbook step z <- (z + R_B(R_A(z))) / 2, parity unpinned
  ellipsoids             ellipsoid_constraints.cpp:34-86
  consistency            guidance_constraints.cpp:986-1023, 1073-1133
"""
import math

import numpy as np


def _norm(dx, dy):
    return math.sqrt(dx * dx + dy * dy)


def _project(p, c, r, start):
    if _norm(p[0] - c[0], p[1] - c[1]) < r:
        dx, dy = start[0] - c[0], start[1] - c[1]
        n = _norm(dx, dy)
        return (c[0] + dx / n * r, c[1] + dy / n * r)
    return p


def _reflect(p, c, r, start):
    q = _project(p, c, r, start)
    return (2.0 * q[0] - p[0], 2.0 * q[1] - p[1])


def douglas_rachford(pos, delta, anchor, r):
    """douglasRachfordProjection(pos, delta, anchor, r, pos)."""
    ra = _reflect(pos, anchor, r, pos)
    rb = _reflect(ra, delta, r, pos)
    return (0.5 * (pos[0] + rb[0]), 0.5 * (pos[1] + rb[1]))


def prepare(layout, sc, robot_radius, w_consistency, deceleration=3.0, warmstart_with_mpc_solution=False,
            shift_forward=False):
    N, npar, dt = layout.N, layout.npar, layout.dt
    S, G = sc.state.shape[0], sc.guided.shape[1]
    ix = layout.idx
    params = np.zeros((S * G, N, npar))
    warm = np.zeros((S * G, N + 1, 7))
    xinit = np.zeros((S * G, 5))
    prev_i = np.zeros((S, N, 2))
    active = np.zeros(S * G, bool)
    for s in range(S):
        x0 = sc.state[s]
        # main warm start: braking
        if sc.main_warm is None:
            mw = np.zeros((N + 1, 7))
            x, y, psi, v, sp = x0
            a = -abs(deceleration)
            mw[0] = (a, 0, x, y, psi, v, sp)
            for k in range(1, N + 1):
                x = x + v * dt * math.cos(psi)
                y = y + v * dt * math.sin(psi)
                sp = sp + v * dt
                v = max(v + a * dt, 0.0)
                mw[k] = (a, 0, x, y, psi, v, sp)
        else:
            mw = np.array(sc.main_warm[s])
        # previous plan interpolation
        valid = bool(np.isfinite(sc.prev_elapsed[s]))
        if valid:
            el = sc.prev_elapsed[s]
            k_shift = int(math.floor(el / dt))
            alpha = (el - k_shift * dt) / dt
            if k_shift >= N - 1:
                valid = False
            else:
                P = sc.prev_traj[s]
                for k in range(N):
                    src = k + k_shift
                    for c in range(2):
                        if src < N - 1:
                            prev_i[s, k, c] = (1.0 - alpha) * P[src, c] + alpha * P[src + 1, c]
                        elif src == N - 1:
                            prev_i[s, k, c] = P[N - 1, c]
                        else:
                            vel = (P[N - 1, c] - P[N - 2, c]) / dt
                            extra = (src - (N - 1)) * dt + alpha * dt
                            prev_i[s, k, c] = P[N - 1, c] + vel * extra
        for g in range(G):
            b = s * G + g
            guided = bool(sc.guided[s, g])
            w = mw.copy()
            own = (guided and warmstart_with_mpc_solution and sc.existing_guidance is not None
                   and bool(sc.existing_guidance[s, g]))
            if own:
                # initializeWarmstart(state, shift) on the copied main solver, from this planner's
                # own previous output (getOutput reads the local solver's _output)
                xt, ut = sc.planner_xtraj[b], sc.planner_utraj[b]
                for k in range(N + 1):
                    if not shift_forward:
                        if k < N:
                            w[k, 0:2] = ut[k]
                            w[k, 2:7] = xt[k]
                    elif k == 0:
                        w[0, 0:2] = ut[1]      # the reference reads State out of range here
                        w[0, 2:7] = x0
                    else:
                        src = N - 1 if k >= N - 1 else k + 1
                        w[k, 0:2] = ut[src]
                        w[k, 2:7] = xt[src]
            elif guided:
                for k in range(1, N):
                    gx, gy, vx, vy = sc.guidance[s, g, k]
                    w[k, 2], w[k, 3] = gx, gy
                    w[k, 4] = math.atan2(vy, vx)
                    w[k, 5] = _norm(vx, vy)
            warm[b] = w
            xinit[b] = x0
            cons = valid and bool(sc.consistency_on[s, g]) and layout.consistency
            active[b] = cons
            for k in range(N):
                p = sc.stage_params[s].copy()
                # ellipsoids
                for j in range(layout.n_ell):
                    e0 = ix(f"ellipsoid_obst_{j}_x")
                    if k == 0:
                        p[e0:e0 + 7] = (x0[0] + 50.0, x0[1] + 50.0, 0.0, 0.0, 0.0, 1.0, 0.1)
                    else:
                        o = sc.obst[s, j, k - 1]
                        p[e0:e0 + 7] = (o[0], o[1], o[2], o[3], o[4], sc.obst_meta[s, j, 1], sc.obst_meta[s, j, 0])
                # halfspaces
                n_obs = min(layout.n_lin, layout.n_ell)
                for i in range(layout.n_lin):
                    l0 = ix(f"lin_constraint_{i}_a1")
                    p[l0:l0 + 3] = (1.0, 0.0, x0[0] + 100.0)
                if guided and k >= 1 and n_obs:
                    r = 1e-3 + robot_radius
                    pos = (w[k, 2], w[k, 3])
                    anchor = tuple(sc.obst[s, 0, k - 1, 0:2])
                    for _ in range(3):
                        for i in range(n_obs):
                            pos = douglas_rachford(pos, tuple(sc.obst[s, i, k - 1, 0:2]), anchor, r)
                    for i in range(n_obs):
                        ox, oy = sc.obst[s, i, k - 1, 0:2]
                        dx, dy = ox - pos[0], oy - pos[1]
                        dist = _norm(dx, dy)
                        a1, a2 = dx / dist, dy / dist
                        l0 = ix(f"lin_constraint_{i}_a1")
                        p[l0:l0 + 3] = (a1, a2, a1 * ox + a2 * oy - r)
                # consistency
                if layout.consistency:
                    on = cons and 1 <= k <= N - 2
                    p[ix("consistency_weight")] = w_consistency if on else 0.0
                    p[ix("prev_traj_x")] = prev_i[s, k, 0] if on else 0.0
                    p[ix("prev_traj_y")] = prev_i[s, k, 1] if on else 0.0
                params[b, k] = p
    return dict(params=params, warm=warm, xinit=xinit, prev_interp=prev_i, consistency_active=active)
