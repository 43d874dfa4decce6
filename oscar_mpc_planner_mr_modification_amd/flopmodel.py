"""Analytic fp64 operation counts of one SQP-RTI solve (the useful-work roofline).

The solve is fp64-latency bound, so its roofline is the fp64
vector peak, priced with the ALGORITHM's operations, not with the kernel's
issued instructions (those include masked lanes, redundant per-part copies and
bookkeeping).  The count follows the algorithm restated in
`oracle/mpcg_oracle.c` (acados SQP-RTI with the options of
`solver_generator/generate_acados_solver.py:88-173`), exploiting only the
structure every implementation exploits: symmetric blocks stored once, the
one-nonzero box rows, the few nonzeros of an h row (its gradient touches
`row_nnz` variables), x0 eliminated.  One add, multiply, fma-half, divide or
square root counts one operation (an fma counts 2).

Per IPM iteration and stage k < N (nz = nu + nx, m_k rows, row r touching c_r
variables):

* residuals: stationarity H dz + g + [B A]'pi_k - pi_{k-1} + sum_r c_r lam_r;
  dynamics A dx + B du + b - dx+; rows d - D dz - t; complementarity;
* barrier Hessian: H + sum_r D_r' (lam_r / t_r) D_r (symmetric outer products);
* Riccati factorisation: P F, F' P F (symmetric), Cholesky of the nu x nu pivot,
  Y = L^-1 M_ux, P = M_xx - Y'Y (symmetric);
* twice (predictor, corrector): Newton gradient, backward vector pass, forward
  pass with the new dynamics multipliers, row steps, step length;
* Mehrotra centring and the update of z, pi, t, lam.

Per SQP iteration and stage k < N (the linearisation): ERK4 with forward
sensitivities and the second-order adjoint of the dynamics (rk_steps x 4 stage
evaluations, dense nx x nz sensitivities), the stage cost's gradient and
Hessian (model-specific constant), the h rows' values, gradients and weighted
Hessians, and MIRROR: cyclic Jacobi on the nz x nz block (JACOBI_SWEEPS sweeps
of nz(nz-1)/2 rotations, symmetric update of two rows and of two eigenvector
columns) plus the reconstruction V f(D) V'.

The per-solve total uses the solve's EXECUTED counts (info[:,0] SQP
iterations, info[:,1] IPM iterations), so the figure follows the workload.
"""
from __future__ import annotations

import numpy as np

JACOBI_SWEEPS = 6        # cyclic Jacobi on a 7x7-9x9 symmetric block: quadratic convergence, 5-7 sweeps
# stage cost gradient + Hessian, excluding the rows and the dynamics: MPCBase weights, the
# 5-segment sigmoid-glued cubic spline in both axes with two derivatives, contouring / lag
# errors and their second-order terms, consistency (unicycle); CA contouring with the
# curvature, the terminal angle and the decomp-slack cost (bicycle)
COST_OPS = {"unicycle": 420, "unicycle_slack": 430, "bicycle_ca": 620}
ROW_OPS = {2: 8, 3: 48}  # value, gradient and weighted Hessian of an h row by its nnz (linear: 2, curved: 3)


def _row_nnz(lay):
    """nnz of each h row of a stage: topology halfspaces touch (x, y), ellipsoids (x, y, psi),
    scenario / decomp halfspaces (x, y, slack)."""
    return [2] * lay.n_lin + [3] * lay.n_ell + [3] * lay.n_scen


def ipm_iteration_ops(lay) -> int:
    """fp64 operations of one interior-point iteration over the whole horizon."""
    return int(sum(ipm_iteration_ops_by_part(lay).values()))


def ipm_iteration_ops_by_part(lay) -> dict:
    """ipm_iteration_ops split by the algorithm's parts: residuals, barrier-augmented Hessian,
    Riccati factorisation, the two Newton solves (gradient, vector passes, row steps) and the
    centring + update (scripts/phase_isa.py sets them beside the kernel's phases)."""
    N, nu, nx = lay.N, lay.nu, lay.nx
    nz = nu + nx
    h = _row_nnz(lay)
    parts = {"residuals": 0, "barrier": 0, "factorisation": 0, "newton_solves": 0, "update": 0}
    for k in range(N):
        rows = [1] * (2 * nu) + ([1] * (2 * nx) + h if k >= 1 else [])
        m = len(rows)
        sc = sum(rows)
        # residuals
        res = (nz * (nz + 1) + nz) + 2 * nx * nz + nx + 2 * sc  # stationarity (symmetric H dz)
        res += 2 * nx * nz + 2 * nx                              # dynamics residual
        res += 2 * sc + 2 * m                                    # row residuals
        res += 2 * m                                             # complementarity sum
        # barrier-augmented Hessian
        bar = sum(1 + c * (c + 1) for c in rows)
        # Riccati factorisation
        fac = 2 * nx * nx * nz + nx * nz * (nz + 1)              # P F, F' (P F) symmetric
        fac += nu * (nu + 1) * (nu + 2) // 3                     # Cholesky of the pivot block
        fac += nu * nu * nx                                      # Y = L^-1 M_ux
        fac += nu * nx * (nx + 1)                                # P = M_xx - Y'Y (symmetric)
        # one Newton solve
        sol = nz * (nz + 1) + nz + sum(2 * c + 3 for c in rows)  # gradient q
        sol += 2 * nx * nx + nx + 2 * nx * nz + nu * nu + 2 * nu * nx  # backward pass
        sol += 2 * nu * nx + nu * nu + 2 * nx * nz + nx + 2 * nx * nx + nx  # forward pass + pi
        sol += sum(2 * c + 5 for c in rows) + 2 * m              # row steps, step length
        # centring + update
        upd = 8 * m + 2 * nz + 3 * nx
        parts["residuals"] += res
        parts["barrier"] += bar
        parts["factorisation"] += fac
        parts["newton_solves"] += 2 * sol
        parts["update"] += upd
    # terminal stage: P_N = H_N, its part of the residuals and update
    parts["factorisation"] += nx * (nx + 1)
    parts["residuals"] += 2 * nx
    parts["update"] += 2 * nz
    return parts


def linearisation_ops(lay, rk_steps: int | None = None) -> int:
    """fp64 operations of one linearisation of the horizon (one SQP-RTI iteration's QP data)."""
    N, nu, nx = lay.N, lay.nu, lay.nx
    nz = nu + nx
    steps = rk_steps if rk_steps is not None else (1 if lay.model == "bicycle_ca" else 3)
    dyn = steps * 4 * (2 * nx * nx * nz + 2 * nz * nz * nx + 2 * nx * (nz + 1) + 12)
    rows = sum(ROW_OPS[c] for c in _row_nnz(lay))
    rot = 12 * nz + 12
    mirror = JACOBI_SWEEPS * (nz * (nz - 1) // 2 * rot + nz * (nz + 1)) + nz * nz * (nz + 1) * 3 // 2 + 2 * nz
    per_stage = dyn + COST_OPS[lay.model] + mirror + 2 * nz * nz  # + packing H, g, [B A]
    return int(N * per_stage + (N - 1) * rows)


def solve_ops(lay, info) -> np.ndarray:
    """Per-solve fp64 operations from the kernel's executed counts: info[:,0] SQP-RTI iterations
    (one linearisation each), info[:,1] interior-point iterations (summed over the QPs).  The base
    count: the Mehrotra iteration without HPIPM's extras (solve_ops_executed adds them)."""
    info = np.asarray(info)
    return info[:, 0].astype(np.float64) * linearisation_ops(lay) + info[:, 1].astype(np.float64) * ipm_iteration_ops(lay)


def _rows_of_stage(lay, k):
    return [1] * (2 * lay.nu) + ([1] * (2 * lay.nx) + _row_nnz(lay) if k >= 1 else [])


def refinement_test_ops(lay) -> int:
    """HPIPM's itref_corr_max > 0: after every corrector, the direction's linear KKT
    residual against its tolerance -- stationarity at the trial point (H (dz + ddz) + g + box and row
    multiplier sums + [B A]'pi_new - pi_new,prev), the dynamics rows at the trial point and per row
    the complementarity part l dt + t dl + rc; then one compare per component."""
    N, nu, nx = lay.N, lay.nu, lay.nx
    nz = nu + nx
    ops = 0
    for k in range(N):
        rows = _rows_of_stage(lay, k)
        m, sc = len(rows), sum(rows)
        ops += nz + (nz * (nz + 1) + nz) + 2 * nx * nz + nx + 2 * sc + nz  # trial point, stationarity
        ops += nz + 2 * nx * nz + 2 * nx + nx                              # dynamics at the trial point
        ops += 8 * m + 2 * m                                               # row steps, complementarity
    return int(ops)


def newton_solve_ops(lay) -> int:
    """one Newton solve with the factorisation at hand (a centring pass of the conditional
    predictor-corrector re-solves the corrector's system): the gradient, both vector passes, the
    feedback, the row steps and the step length (the `sol` term of ipm_iteration_ops_by_part)."""
    return int(ipm_iteration_ops_by_part(lay)["newton_solves"] // 2)


def refinement_solve_ops(lay) -> int:
    """one refinement step: the right-hand side from the linear residual (refinement_test_ops' terms
    with the Newton gradient formed from them) and one Newton solve"""
    return int(refinement_test_ops(lay) + sum(2 * c + 3 for k in range(lay.N) for c in _rows_of_stage(lay, k)) +
               newton_solve_ops(lay))


def solve_ops_executed(lay, info, profile="hpipm", center_per_ipm=0.0, itref_per_ipm=0.0) -> np.ndarray:
    """The operations of the interior point that actually runs: solve_ops plus,
    under HPIPM's profile, the refinement test of every IPM iteration, and the rare passes -- centring
    re-solves of the conditional predictor-corrector and refinement solves -- at the given rates per
    IPM iteration (the kernel does not count them; bench.py takes them from the oracle run on a sample
    of the same batch, whose IPM path the GPU's follows solve for solve)."""
    info = np.asarray(info)
    ipm = info[:, 1].astype(np.float64)
    ops = solve_ops(lay, info)
    if profile == "hpipm":
        ops = ops + ipm * (refinement_test_ops(lay) + center_per_ipm * newton_solve_ops(lay) +
                           itref_per_ipm * refinement_solve_ops(lay))
    return ops
