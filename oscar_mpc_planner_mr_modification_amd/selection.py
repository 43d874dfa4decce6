"""Planner selection of T-MPC++ — host mirror of the reference rule.

GuidanceConstraints::optimize computes per planner
    objective = pobj - consistency_cost          (guidance_constraints.cpp:386-416)
    objective *= selection_weight_consistency_   if the guidance was previously selected (:418-419)
with consistency_cost = w * sum_{k=1}^{N-2} |xy_k - prev_k|^2 (:1025-1050), then
FindBestPlanner (:572-590) takes the argmin over enabled, successful planners
(strict `<` against a 1e10 start, so the first index wins ties; -1 if none).

`find_best_planner_host` is the NumPy statement of that rule (used by the
C++-less callers and as the check of the device kernel
`mpcg_select_best_device`, which the batched path uses).
"""
from __future__ import annotations

import numpy as np


def consistency_cost(xtraj: np.ndarray, prev: np.ndarray, w: float) -> float:
    N = prev.shape[0]
    d = xtraj[1:N - 1, :2] - prev[1:N - 1]
    return w * float(np.sum(d[:, 0] * d[:, 0] + d[:, 1] * d[:, 1]))


def find_best_planner_host(n_scenes, G, N, xtraj, pobj, exit_code, prev_traj=None, w_cons=0.0,
                           consistency_enabled=None, previously_selected=None, selection_weight=1.0,
                           disabled=None):
    xtraj = np.asarray(xtraj).reshape(n_scenes * G, N + 1, 5)
    best = np.full(n_scenes, -1, np.int32)
    objective = np.zeros(n_scenes * G)
    for sc in range(n_scenes):
        best_obj = 1e10
        for g in range(G):
            s = sc * G + g
            obj = float(pobj[s])
            if prev_traj is not None and consistency_enabled is not None and consistency_enabled[s]:
                acc = 0.0
                for k in range(1, N - 1):
                    dx = xtraj[s, k, 0] - prev_traj[sc, k, 0]
                    dy = xtraj[s, k, 1] - prev_traj[sc, k, 1]
                    acc += dx * dx + dy * dy
                obj -= w_cons * acc
            if previously_selected is not None and previously_selected[s]:
                obj *= selection_weight
            objective[s] = obj
            dis = disabled is not None and disabled[s]
            if not dis and exit_code[s] == 1 and obj < best_obj:
                best_obj = obj
                best[sc] = g
    return best, objective
