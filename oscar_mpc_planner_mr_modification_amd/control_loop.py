"""Consecutive control steps of many scenes on one GPU: the work
GuidanceConstraints::optimize and Planner::solveMPC do per step, with every
per-step quantity device-resident.

    step():  mpcg_prepare (per-guess inputs) -> mpcg_solve (all guesses, carried
             multipliers) -> mpcg_select_best_device (FindBestPlanner with the
             consistency / selection-weight bookkeeping) -> mpcg_advance (warm
             start, previous plan, selection flags, multipliers of the next step)

The scene data of the next step (ego state, obstacle predictions, guidance
trajectories) comes from outside the planner (sensors, guidance_planner), so
`set_scene_data` replaces it between steps.
"""
from __future__ import annotations

from . import native
from .layouts import Layout


class ControlLoop:
    def __init__(self, layout: Layout, scenes, device, robot_radius: float, w_consistency: float,
                 selection_weight: float, deceleration: float = 3.0, shift_forward: bool = False,
                 consistency_on_non_guided: bool = True, elapsed: float | None = None,
                 warmstart_with_mpc_solution: bool = False):
        import torch

        self.lay = layout
        self.pr = native.problem_from_layout(layout)
        self.dev = device
        self.S, self.G = scenes.n_scenes, scenes.n_guesses
        self.rr, self.wc, self.sw, self.dec = robot_radius, w_consistency, selection_weight, deceleration
        self.shift, self.cong = shift_forward, consistency_on_non_guided
        # t-mpc.warmstart_with_mpc_solution (guidance_constraints.cpp:335-338): from the second step on,
        # guided planners (whose guidance then exists) start from their own previous output
        self.own_warm = warmstart_with_mpc_solution
        self.elapsed = layout.dt if elapsed is None else elapsed
        self.dsc = native.scenes_to_device(scenes, device)
        LS = 5 + layout.nh
        self.lam = torch.zeros((self.S * self.G, layout.N, LS), dtype=torch.float64, device=device)
        self.last = None
        self.existing = None

    def set_scene_data(self, state, obst, guidance, existing_guidance=None):
        """Replace the externally provided scene data (device tensors or arrays).

        existing_guidance (S, G) bool, optional: which guided planners' guidance existed in the
        previous step -- in the reference a planner keeps its guidance only when the homotopy
        class guidance_planner finds this step maps back to the same planner
        (guidance_constraints.cpp:211-257), so it comes from the guidance search, outside the
        planner.  Read by the next step() with warmstart_with_mpc_solution (such a planner
        starts from its own previous output, the others from their guidance); when not given,
        every guided planner's guidance is taken to have existed (each kept its class)."""
        import torch

        t = lambda a: torch.as_tensor(a, dtype=torch.float64, device=self.dev).contiguous()  # noqa: E731
        self.dsc["state"], self.dsc["obst"], self.dsc["guidance"] = t(state), t(obst), t(guidance)
        self.existing = None
        if existing_guidance is not None:
            ex = torch.as_tensor(existing_guidance, device=self.dev).reshape(self.S, self.G)
            self.existing = ex.to(torch.uint8).contiguous()

    def step(self, stream=None):
        """One control step of every scene.  Returns dict(best, exit, xtraj, utraj, pobj, objective, prepared)."""
        pr, S, G, N = self.pr, self.S, self.G, self.lay.N
        if self.own_warm and self.last is not None:
            self.dsc["planner_xtraj"], self.dsc["planner_utraj"] = self.last["xtraj"], self.last["utraj"]
            self.dsc["existing_guidance"] = self.dsc["guided"] if self.existing is None else self.existing
        prep = native.prepare_device(pr, self.dsc, self.rr, self.wc, self.dec, stream=stream,
                                     warmstart_with_mpc_solution=self.own_warm, shift_forward=self.shift)
        out = native.solve_batch_device(pr, prep["params"], prep["warm"], prep["xinit"], stream=stream,
                                        lam_in=self.lam, lam_out=True)
        best, objective = native.select_best_device(S, G, N, out["xtraj"], out["pobj"], out["exit"],
                                                    prev_traj=prep["prev_interp"], w_cons=self.wc,
                                                    consistency_enabled=prep["consistency_active"],
                                                    previously_selected=self.dsc["previously_selected"],
                                                    selection_weight=self.sw, stream=stream)
        self.last = dict(best=best, exit=out["exit"], xtraj=out["xtraj"], utraj=out["utraj"], pobj=out["pobj"],
                         objective=objective, prepared=prep, lam=out["lam"])
        return self.last

    def advance(self, state_next, stream=None):
        """Carry the planner state into the next step (call after step())."""
        import torch

        L = self.last
        sn = torch.as_tensor(state_next, dtype=torch.float64, device=self.dev).contiguous()
        c = native.advance_device(self.pr, self.S, self.G, L["best"], L["exit"], L["xtraj"], L["utraj"],
                                  L["prepared"]["warm"], L["lam"], sn, self.dsc["guided"], self.elapsed,
                                  self.dec, self.shift, self.cong,
                                  previously_selected=self.dsc["previously_selected"], stream=stream)
        self.dsc["main_warm"] = c["main_warm"]
        self.dsc["prev_traj"] = c["prev_traj"]
        self.dsc["prev_elapsed"] = c["prev_elapsed"]
        self.dsc["consistency_on"] = c["consistency_on"]
        self.dsc["previously_selected"] = c["previously_selected"]
        self.lam = c["lam"]
        self.dsc["state"] = sn
        return c
