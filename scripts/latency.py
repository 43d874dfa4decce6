#!/usr/bin/env python3
"""Single-planner latency of the drop-in path (one Solver::solve()
with batch 1) and of one scene's guesses (batch G), through a persistent
mpcg_context (host buffers in, host buffers out, what MPCPlanner::Solver and
SolverBatch do), next to the CPU oracle on one core.

    python scripts/latency.py [--config C1] [--reps 200]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C1")
    ap.add_argument("--reps", type=int, default=200)
    ap.add_argument("--guesses", type=int, default=8)
    ap.add_argument("--solver-type", default="SQP_RTI", choices=("SQP_RTI", "SQP"))
    args = ap.parse_args()
    import torch  # noqa: F401  (HIP runtime before libmpcg.so)
    from oscar_mpc_planner_mr_modification_amd import native
    from oscar_mpc_planner_mr_modification_amd.layouts import config_layout
    from oscar_mpc_planner_mr_modification_amd.synthetic import make_batch

    lay = config_layout(args.config)
    b = make_batch(lay, 4, args.guesses, seed=99)
    pr = native.problem_from_layout(lay, solver_type=args.solver_type)
    out = {"config": args.config, "N": lay.N, "obstacles": lay.max_obstacles, "solver_type": args.solver_type}
    for batch in (1, args.guesses):
        ctx = native.Context(pr, batch)
        P, W, X = b.params[:batch], b.warm[:batch], b.xinit[:batch]
        for _ in range(5):
            ctx.solve(P, W, X)
        ts = []
        for _ in range(args.reps):
            t0 = time.perf_counter()
            ctx.solve(P, W, X)
            ts.append(time.perf_counter() - t0)
        ts = np.array(ts) * 1e3
        out[f"gpu_batch{batch}_ms"] = {"median": float(np.median(ts)), "p90": float(np.percentile(ts, 90))}
        ctx.close()
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle_py
    orc = oracle_py.Oracle(lay, solver_type=args.solver_type)
    ts = []
    for i in range(min(args.reps, 50)):
        t0 = time.perf_counter()
        orc.solve_batch(b.params[i % 4 * args.guesses:][:1], b.warm[i % 4 * args.guesses:][:1],
                        b.xinit[i % 4 * args.guesses:][:1], nthreads=1)
        ts.append(time.perf_counter() - t0)
    out["cpu_oracle_1core_ms"] = {"median": float(np.median(ts) * 1e3)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
