"""Parameter layouts: the horizon-major `all_parameters[k*npar + idx]` map.

Mirrors the reference's `define_parameters` (solver_generator/solver_definition.py:5-16):
objective modules first, then constraint modules, each appending its
parameters in declaration order, duplicates skipped (util/parameters.py:187-217).
The module stacks are the ones the reference's generator scripts build:

* ``tmpc``     — configuration_tmpc_consistency_cost
                 (mpc_planner_jackalsimulator/scripts/generate_jackalsimulator_solver.py:37-59,107-116):
                 MPCBase(a, w, v) + Contouring [+ Consistency] + GuidanceConstraints(Ellipsoid)
* ``lmpcc``    — configuration_basic (same file :62-67): MPCBase + Contouring + Ellipsoid

The resulting maps are checked against the reference's own maps in
tests/golden/parameter_maps.json.
"""
from __future__ import annotations

from dataclasses import dataclass, field

# bounds of ContouringSecondOrderUnicycleModel (solver_model.py:204-205), z = [a, w, x, y, psi, v, s]
UNICYCLE_LB = (-2.0, -0.8, -2000.0, -2000.0, -12.566370614359172, -0.01, -1.0)
UNICYCLE_UB = (2.0, 0.8, 2000.0, 2000.0, 12.566370614359172, 3.0, 10000.0)
UNICYCLE_STATES = ("x", "y", "psi", "v", "spline")
UNICYCLE_INPUTS = ("a", "w")
# ContouringSecondOrderUnicycleModelWithSlack (solver_model.py:274-285): + slack state in [0, 5000]
SLACK_LB = UNICYCLE_LB + (0.0,)
SLACK_UB = UNICYCLE_UB + (5000.0,)
SLACK_STATES = UNICYCLE_STATES + ("slack",)
# BicycleModel2ndOrderCurvatureAware (solver_model.py:355-376), z = [a, w, slack, x, y, psi, v, delta, s]
BICYCLE_LB = (-3.0, -1.5, 0.0, -1.0e6, -1.0e6, -12.566370614359172, -0.01, -0.55, -1.0)
BICYCLE_UB = (3.0, 1.5, 1.0e2, 1.0e6, 1.0e6, 12.566370614359172, 8.0, 0.55, 5000.0)
BICYCLE_STATES = ("x", "y", "psi", "v", "delta", "spline")
BICYCLE_INPUTS = ("a", "w", "slack")


class _Params:
    """Same add() semantics as util/parameters.py:187-217 (name -> next index,
    bundle -> list of indices)."""

    def __init__(self):
        self.map: dict[str, int] = {}
        self.bundles: dict[str, list[int]] = {}

    def add(self, name: str, bundle: str | None = None):
        if name in self.map:
            return
        idx = len(self.map)
        self.map[name] = idx
        self.bundles.setdefault(bundle or name, []).append(idx)


def _mpc_base(p: _Params):
    # weigh_variable a/acceleration, w/angular_velocity, v/[velocity, reference_velocity]
    for n in ("acceleration", "angular_velocity", "velocity", "reference_velocity"):
        p.add(n)


def _contouring(p: _Params, num_segments: int):
    # contouring.py:114-138
    p.add("contour")
    p.add("lag")
    if "velocity" not in p.map:
        p.add("velocity")
        p.add("reference_velocity")
    p.add("terminal_angle")
    p.add("terminal_contouring")
    for i in range(num_segments):
        for ax in ("x", "y"):
            for c in ("a", "b", "c", "d"):
                p.add(f"spline_{ax}{i}_{c}", f"spline_{ax}_{c}")
        p.add(f"spline{i}_start", "spline_start")


def _consistency(p: _Params):
    # consistency_module.py:220-227
    p.add("consistency_weight")
    p.add("prev_traj_x")
    p.add("prev_traj_y")


def _guidance_linear(p: _Params, n: int):
    # guidance_constraints.py:333-338
    for i in range(n):
        p.add(f"lin_constraint_{i}_a1", "lin_constraint_a1")
        p.add(f"lin_constraint_{i}_a2", "lin_constraint_a2")
        p.add(f"lin_constraint_{i}_b", "lin_constraint_b")


def _scenario(p: _Params, n_discs: int, n_constraints: int):
    # scenario_constraints.py:41-50
    for d in range(n_discs):
        p.add(f"ego_disc_{d}_offset", "ego_disc_offset")
        for i in range(n_constraints * n_discs):
            for c in ("a1", "a2", "b"):
                p.add(f"disc_{d}_scenario_constraint_{i}_{c}")


def _decomp(p: _Params, n_discs: int, max_constraints: int):
    # decomp_constraints.py:46-54
    for d in range(n_discs):
        p.add(f"ego_disc_{d}_offset", "ego_disc_offset")
        for i in range(max_constraints):
            p.add(f"disc_{d}_decomp_{i}_a1", "decomp_a1")
            p.add(f"disc_{d}_decomp_{i}_a2", "decomp_a2")
            p.add(f"disc_{d}_decomp_{i}_b", "decomp_b")


def _ellipsoid(p: _Params, n_discs: int, n_obs: int):
    # ellipsoid_constraints.py:406-419
    p.add("ego_disc_radius")
    for d in range(n_discs):
        p.add(f"ego_disc_{d}_offset", "ego_disc_offset")
    for j in range(n_obs):
        for f in ("x", "y", "psi", "major", "minor", "chi", "r"):
            p.add(f"ellipsoid_obst_{j}_{f}", f"ellipsoid_obst_{f}")


@dataclass
class Layout:
    """Everything the kernels need to find a parameter by meaning."""
    name: str
    N: int
    max_obstacles: int
    n_lin: int
    n_ell: int
    n_seg: int = 5
    consistency: bool = True
    model: str = "unicycle"      # "unicycle_slack" (slack state last) or "bicycle_ca" (C3)
    n_scen: int = 0
    dt: float = 0.2
    rk_steps: int = 3
    sqp_iters: int = 10
    pmap: dict = field(default_factory=dict)
    bundles: dict = field(default_factory=dict)

    @property
    def npar(self) -> int:
        return len(self.pmap)

    @property
    def nx(self) -> int:
        return 5 if self.model == "unicycle" else 6

    @property
    def nu(self) -> int:
        return 3 if self.model == "bicycle_ca" else 2

    @property
    def model_id(self) -> int:
        """mpcg_problem.model (include/mpcg.h): 0 contouring unicycle, 1 curvature-aware bicycle"""
        return 1 if self.model == "bicycle_ca" else 0

    @property
    def nvar(self) -> int:
        return self.nx + self.nu

    @property
    def nh(self) -> int:
        return self.n_lin + self.n_ell + self.n_scen

    @property
    def states(self):
        return {"unicycle_slack": SLACK_STATES, "bicycle_ca": BICYCLE_STATES}.get(self.model, UNICYCLE_STATES)

    @property
    def inputs(self):
        return BICYCLE_INPUTS if self.model == "bicycle_ca" else UNICYCLE_INPUTS

    @property
    def lb(self):
        return {"unicycle_slack": SLACK_LB, "bicycle_ca": BICYCLE_LB}.get(self.model, UNICYCLE_LB)

    @property
    def ub(self):
        return {"unicycle_slack": SLACK_UB, "bicycle_ca": BICYCLE_UB}.get(self.model, UNICYCLE_UB)

    def idx(self, name: str) -> int:
        return self.pmap.get(name, -1)

    def index_struct(self) -> dict:
        """Base indices consumed by the C ABI (include/mpcg.h, mpcg_problem)."""
        g = self.idx
        return dict(
            i_w_acc=g("acceleration"), i_w_ang=g("angular_velocity"), i_w_vel=g("velocity"),
            i_v_ref=g("reference_velocity"), i_w_contour=g("contour"), i_w_lag=g("lag"),
            i_spline0=g("spline_x0_a"), i_cons_w=g("consistency_weight"),
            i_prev_x=g("prev_traj_x"), i_prev_y=g("prev_traj_y"),
            i_lin0=g("lin_constraint_0_a1") if self.n_lin else -1,
            i_disc_r=g("ego_disc_radius"), i_disc_off=g("ego_disc_0_offset"),
            i_ell0=g("ellipsoid_obst_0_x") if self.n_ell else -1,
            i_scen0=(g("disc_0_decomp_0_a1") if self.model == "bicycle_ca" else
                     g("disc_0_scenario_constraint_0_a1")) if self.n_scen else -1,
            i_w_slack=g("slack"),
            i_w_tangle=g("terminal_angle"), i_w_tcont=g("terminal_contouring"),
        )


def tmpc_layout(N: int = 20, max_obstacles: int = 8, consistency: bool = True,
                num_segments: int = 5, add_halfspaces: int = 0, name: str | None = None) -> Layout:
    p = _Params()
    _mpc_base(p)
    _contouring(p, num_segments)
    if consistency:
        _consistency(p)
    n_lin = max_obstacles + add_halfspaces
    _guidance_linear(p, n_lin)
    _ellipsoid(p, 1, max_obstacles)
    return Layout(name=name or f"tmpc_N{N}_obs{max_obstacles}", N=N, max_obstacles=max_obstacles,
                  n_lin=n_lin, n_ell=max_obstacles, n_seg=num_segments, consistency=consistency,
                  pmap=p.map, bundles=p.bundles)


def lmpcc_layout(N: int = 20, max_obstacles: int = 4, num_segments: int = 5) -> Layout:
    p = _Params()
    _mpc_base(p)
    _contouring(p, num_segments)
    _ellipsoid(p, 1, max_obstacles)
    return Layout(name=f"lmpcc_N{N}_obs{max_obstacles}", N=N, max_obstacles=max_obstacles,
                  n_lin=0, n_ell=max_obstacles, n_seg=num_segments, consistency=False,
                  pmap=p.map, bundles=p.bundles)


def safe_horizon_layout(N: int = 20, n_constraints: int = 24, num_segments: int = 5) -> Layout:
    """configuration_safe_horizon (generate_jackalsimulator_solver.py:69-89): MPCBase(a, w, slack, v) +
    Contouring + ScenarioConstraints on ContouringSecondOrderUnicycleModelWithSlack."""
    p = _Params()
    for n in ("acceleration", "angular_velocity", "slack", "velocity", "reference_velocity"):
        p.add(n)
    _contouring(p, num_segments)
    _scenario(p, 1, n_constraints)
    return Layout(name=f"shmpc_N{N}_scen{n_constraints}", N=N, max_obstacles=0, n_lin=0, n_ell=0,
                  n_seg=num_segments, consistency=False, model="unicycle_slack", n_scen=n_constraints,
                  pmap=p.map, bundles=p.bundles)


def ca_decomp_layout(N: int = 30, max_constraints: int = 12, num_segments: int = 5) -> Layout:
    """C3: BicycleModel2ndOrderCurvatureAware + MPCBase(a, w, slack) +
    CurvatureAwareContouring (curvature_aware_contouring.py:22-44, same parameter order as
    contouring) + DecompConstraints(max_constraints, decomp_constraints.py:46-54).  The
    decomp halfspaces are the slack rows of the kernel (n_scen).  The reference discretises
    this model with Forces only (solver_model.py:11-36): one RK4 step of integrator_step."""
    p = _Params()
    for n in ("acceleration", "angular_velocity", "slack"):
        p.add(n)
    _contouring(p, num_segments)
    _decomp(p, 1, max_constraints)
    return Layout(name=f"cadecomp_N{N}_dec{max_constraints}", N=N, max_obstacles=0, n_lin=0, n_ell=0,
                  n_seg=num_segments, consistency=False, model="bicycle_ca", n_scen=max_constraints,
                  rk_steps=1, pmap=p.map, bundles=p.bundles)


# BASELINE.json configs
def config_layout(cfg: str) -> Layout:
    cfg = cfg.upper()
    if cfg == "C1":
        return tmpc_layout(N=20, max_obstacles=4, name="C1")
    if cfg == "C2":
        return tmpc_layout(N=20, max_obstacles=8, name="C2")
    if cfg == "C4":
        return tmpc_layout(N=30, max_obstacles=12, name="C4")
    if cfg == "JS":
        # the reference's shipped jackalsimulator solver: configuration_tmpc_consistency_cost
        # (generate_jackalsimulator_solver.py:147) with N 30, max_obstacles 4
        # (mpc_planner_jackalsimulator/config/settings.yaml:3,37); n_paths 4 -> 5 planners (:104)
        return tmpc_layout(N=30, max_obstacles=4, name="JS")
    if cfg == "JD":
        # the reference's shipped jackal / dingo solver: configuration_tmpc
        # (generate_jackal_solver.py:54-75, consistency on: settings.yaml:110) with N 30,
        # max_obstacles 5 (mpc_planner_jackal/config/settings.yaml:3,38, mpc_planner_dingo :2,33),
        # n_paths 4 -> 5 planners (:102)
        return tmpc_layout(N=30, max_obstacles=5, name="JD")
    if cfg == "C5":
        lay = safe_horizon_layout(N=20, n_constraints=24)
        lay.name = "C5"
        return lay
    if cfg == "C3":
        lay = ca_decomp_layout(N=30, max_constraints=12)
        lay.name = "C3"
        return lay
    if cfg == "T10":
        # diagnostic shape (not a BASELINE config): N 10, 2 obstacles -- the built-in test instance
        # whose LDS block (17 KB) admits two waves per SIMD, for register-budget A/B runs
        return tmpc_layout(N=10, max_obstacles=2, name="T10")
    raise KeyError(f"config {cfg} has no layout")
