#!/usr/bin/env python3
"""Benchmark of the MI355X T-MPC++ per-guess SQP backend.

Workload (BASELINE.json configs[1], "C2"): jackal unicycle T-MPC++, N=20,
8 obstacles, 1024 synthetic scenes x 8 topology guesses per GPU (7 guided +
the non-guided T-MPC++ planner), 10 SQP-RTI iterations per solve, timeout
disabled.  One step = one control step of every scene, all on the GPU:
per-guess solver inputs from the scene data (mpcg_prepare: warm starts,
topology halfspaces with Douglas-Rachford projection, obstacles, consistency
references) + one batched solve of all scenes x guesses + per-scene planner
selection (FindBestPlanner with the consistency and selection-weight
bookkeeping) + one RCCL all-gather of the winning trajectories when
N_gpus > 1 (scenes are sharded, weak scaling).  Scene data is uploaded once
before the timed region (inputs resident in HBM).

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nproc-per-node N bench.py --gpus N ...

Rank 0 prints one JSON line.  `roofline` prices the solve kernel against HBM
with SURVEY.md §8(d)'s algorithmic bytes per solve (the path is fp64-VALU /
latency bound); `cpu_baseline` times the C oracle (same
algorithm, OpenMP over solves) on a bounded sample of the same batch, and
`parity` is max |x - x_ref| over that sample.

`--config C3` runs the curvature-aware bicycle workload:
4096 scenes per GPU, N=30, the bicycle with the CA spline update, CA
contouring and 12 decomp halfspaces per stage, one solver per scene.

`--config C5` runs the SH-MPC workload instead: 2048
scenes x 4 parallel scenario solvers per GPU on the slack model, 24 scenario
halfspaces per stage reduced on the GPU from 12 obstacles x 100 prediction
samples (mpcg_prepare_scenario), batched solve, lowest-cost pick
(ScenarioConstraints::optimize) and the winner gather.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "SQP solves/s (N=20, 8 obs, 8 guesses) at 1/2/4/8 MI355X; max |x−x_ref|"
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
FP64_VALU_PEAK_TFLOPS = 78.6   # MI355X fp64 vector (vendor spec)


def algorithmic_bytes_per_solve(lay):
    """B = 8*[N*npar + (N+1)*nvar + nx + (N+1)*nx + N*nu + 2]"""
    N = lay.N
    return 8 * (N * lay.npar + (N + 1) * lay.nvar + lay.nx + (N + 1) * lay.nx + N * lay.nu + 2)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="C2")
    ap.add_argument("--scenes", type=int, default=None, help="scenes per GPU (C2: 1024, C3: 4096, C4: 2048, C5: 2048)")
    ap.add_argument("--guesses", type=int, default=8)
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="bound of the CPU-baseline sample")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--traffic-json", default=None, help="PMC summary (default profiles/traffic_<config>.json)")
    args = ap.parse_args()
    if args.traffic_json is None:
        args.traffic_json = os.path.join(ROOT, "profiles", f"traffic_{args.config}.json")

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
    dev = torch.device("cuda", local_rank)
    torch.cuda.set_device(dev)

    from oscar_mpc_planner_mr_modification_amd import native
    from oscar_mpc_planner_mr_modification_amd.distributed import gather_winners, winner_records, winner_width
    from oscar_mpc_planner_mr_modification_amd.layouts import config_layout
    from oscar_mpc_planner_mr_modification_amd.producers import prepare_host
    from oscar_mpc_planner_mr_modification_amd.synthetic import (DECELERATION, ROBOT_RADIUS, SETTINGS_WEIGHTS,
                                                                 concat_scenes, make_scenes)

    lay = config_layout(args.config)
    if args.config == "C5":
        return run_shmpc(args, lay, world, rank, dev)
    if args.config == "C3":
        return run_c3(args, lay, world, rank, dev)
    # BASELINE.json configs[3]: 16384 scenes over 8 GPUs -> 2048 per GPU for C4
    S, G, N = args.scenes or (2048 if args.config == "C4" else 1024), args.guesses, lay.N
    B = S * G
    W_CONS, SEL_W = SETTINGS_WEIGHTS["consistency"], 0.75   # guidance_planner.yaml:37 selection weight
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or min(16, os.cpu_count() or 1)
    t0 = time.time()
    workers = min(threads, 16)
    if workers > 1 and S >= 2 * workers:
        from concurrent.futures import ProcessPoolExecutor
        chunks = np.array_split(np.arange(S), workers)
        with ProcessPoolExecutor(max_workers=workers) as ex:
            scenes = concat_scenes(list(ex.map(make_scenes, [lay] * len(chunks), [len(c) for c in chunks],
                                               [G] * len(chunks), [None] * len(chunks), [20251212] * len(chunks),
                                               [rank * S + int(c[0]) for c in chunks])))
    else:
        scenes = make_scenes(lay, S, G, first_scene=rank * S)
    gen_s = time.time() - t0
    dsc = native.scenes_to_device(scenes, dev)
    pr = native.problem_from_layout(lay)
    prep = dict(params=torch.empty((B, N, lay.npar), dtype=torch.float64, device=dev),
                warm=torch.empty((B, N + 1, 7), dtype=torch.float64, device=dev),
                xinit=torch.empty((B, 5), dtype=torch.float64, device=dev),
                prev_interp=torch.empty((S, N, 2), dtype=torch.float64, device=dev),
                consistency_active=torch.empty((B,), dtype=torch.uint8, device=dev))
    out = dict(xtraj=torch.empty((B, N + 1, 5), dtype=torch.float64, device=dev),
               utraj=torch.empty((B, N, 2), dtype=torch.float64, device=dev),
               pobj=torch.empty((B,), dtype=torch.float64, device=dev),
               exit=torch.empty((B,), dtype=torch.int32, device=dev),
               info=torch.empty((B, 4), dtype=torch.int32, device=dev))
    win_w = winner_width(N)
    winners = torch.empty((S, win_w), dtype=torch.float64, device=dev)
    gathered = torch.empty((S * world, win_w), dtype=torch.float64, device=dev) if world > 1 else None
    stream = torch.cuda.current_stream(dev)
    ev_s = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps)]
    ev_e = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps)]
    ev_p = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps)]

    def step(i=None):
        if i is not None:
            ev_p[i].record(stream)
        native.prepare_device(pr, dsc, ROBOT_RADIUS, W_CONS, DECELERATION, out=prep, stream=stream)
        if i is not None:
            ev_s[i].record(stream)
        native.solve_batch_device(pr, prep["params"], prep["warm"], prep["xinit"], out=out, stream=stream)
        if i is not None:
            ev_e[i].record(stream)
        best, _ = native.select_best_device(S, G, N, out["xtraj"], out["pobj"], out["exit"],
                                            prev_traj=prep["prev_interp"], w_cons=W_CONS,
                                            consistency_enabled=prep["consistency_active"],
                                            previously_selected=dsc["previously_selected"], selection_weight=SEL_W,
                                            stream=stream)
        winner_records(out["xtraj"], out["utraj"], out["pobj"], best, G, out=winners)
        if world > 1:
            gather_winners(winners, world, out=gathered)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t_start = time.perf_counter()
    for i in range(args.steps):
        step(i)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t_start
    kern_ms = float(np.mean([ev_s[i].elapsed_time(ev_e[i]) for i in range(args.steps)]))
    prep_ms = float(np.mean([ev_p[i].elapsed_time(ev_s[i]) for i in range(args.steps)]))
    if world > 1:
        te = torch.tensor([elapsed, kern_ms], dtype=torch.float64, device=dev)
        dist.all_reduce(te, op=dist.ReduceOp.MAX)
        elapsed, kern_ms = float(te[0]), float(te[1])

    total = args.steps * B * world
    value = total / elapsed
    exit_h = out["exit"].cpu().numpy()
    xt_h = out["xtraj"].cpu().numpy()
    info_h = out["info"].cpu().numpy()

    bps = algorithmic_bytes_per_solve(lay)
    achieved = bps * B / (kern_ms * 1e-3) / 1e9
    traffic, f64 = None, None
    if os.path.exists(args.traffic_json):
        try:
            tj = json.load(open(args.traffic_json))
            if tj.get("config") == args.config and tj.get("batch") == B:
                traffic = tj.get("hbm_bytes_per_launch")
                f64 = tj.get("fp64_issued_flop_per_launch")
        except Exception:
            traffic, f64 = None, None
    roofline = {"bound": "hbm", "achieved": round(achieved, 3), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                "kernel": "sqp_kernel", "kernel_ms": round(kern_ms, 4), "bytes_per_solve": bps}

    if f64:
        # the path is fp64-VALU / latency bound: issued fp64 FLOP/s of the
        # solve kernel (PMC SQ_INSTS_VALU_*_F64 x 64 lanes, profiles/) against the vector peak
        roofline["fp64_valu"] = {"achieved_tflops": round(f64 / (kern_ms * 1e-3) / 1e12, 3),
                                 "peak_tflops": FP64_VALU_PEAK_TFLOPS,
                                 "frac": f64 / (kern_ms * 1e-3) / 1e12 / FP64_VALU_PEAK_TFLOPS}
    result = {
        "metric": METRIC, "value": round(value, 2), "unit": "solves/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f64",
        "data": "synthetic (seeded scenes, SURVEY.md §8d)",
        "config": {"workload": f"{args.config}: jackal unicycle T-MPC++, N={N}, {lay.max_obstacles} obstacles, "
                               f"{S} scenes x {G} guesses per GPU, 10 SQP-RTI iterations",
                   "scenes_per_gpu": S, "guesses": G, "N": N, "obstacles": lay.max_obstacles,
                   "parallelism": f"scene-sharded x{world}" + (" + RCCL all-gather of winners" if world > 1 else "")},
        "roofline": roofline,
        "solver_stats": {"success_frac": float((exit_h == 1).mean()), "qp_iters_per_solve": float(info_h[:, 1].mean()),
                         "scene_gen_s": round(gen_s, 2)},
        "phases_ms": {"prepare": round(prep_ms, 4), "solve": round(kern_ms, 4)},
    }

    if rank == 0 and world == 1 and not args.no_cpu:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle_py

        oracle_py.build()
        orc = oracle_py.Oracle(lay)
        hb = prepare_host(lay, scenes, ROBOT_RADIUS, W_CONS, DECELERATION)

        class _B:  # host copy of the solver inputs the GPU prepared
            params, warm, xinit = hb.params, hb.warm, hb.xinit
        b = _B()
        # bounded sample: chunks of the same batch until ~cpu_seconds of CPU work
        done, t_cpu, chunk = 0, 0.0, 256
        max_abs_dx, agree, compared = 0.0, 0, 0
        while done < B and t_cpu < args.cpu_seconds:
            sl = slice(done, min(B, done + chunk))
            tc = time.perf_counter()
            ref = orc.solve_batch(b.params[sl], b.warm[sl], b.xinit[sl], nthreads=threads)
            t_cpu += time.perf_counter() - tc
            ok = (ref["status"] == 1) & (exit_h[sl] == 1)
            if ok.any():
                max_abs_dx = max(max_abs_dx, float(np.abs(xt_h[sl][ok] - ref["xtraj"][ok]).max()))
            agree += int((ref["status"] == exit_h[sl]).sum())
            compared += len(ref["status"])
            done = sl.stop
        # also 1 thread and 8 threads (the reference's num_threads(8))
        def rate(n, nthreads):
            tc = time.perf_counter()
            orc.solve_batch(b.params[:n], b.warm[:n], b.xinit[:n], nthreads=nthreads)
            return n / (time.perf_counter() - tc)

        r1 = rate(64, 1)
        r8 = rate(512, 8) if threads >= 8 else None
        result["cpu_baseline"] = {"value": round(done / t_cpu, 2), "unit": "solves/s", "cores": threads,
                                  "kind": "port",
                                  "sample": f"first {done} of the {B} solves of this batch, C oracle "
                                            f"(same algorithm), OpenMP {threads} threads",
                                  "single_thread_solves_per_s": round(r1, 2),
                                  "eight_thread_solves_per_s": None if r8 is None else round(r8, 2)}
        result["parity"] = {"max_abs_dx": max_abs_dx, "exit_agreement": agree / max(1, compared),
                            "solves_compared": compared, "tolerance": 1e-4}
        result["vs_cpu_baseline"] = round(value / (done / t_cpu), 2)
    if rank == 0:
        print(json.dumps(result))
    if world > 1:
        dist.destroy_process_group()


def run_c3(args, lay, world, rank, dev):
    """C3: one batched solve of every scene's bicycle CA-MPC problem + the gather of the results.
    The decomp halfspaces come from DecompUtil (external) on the host: the per-scene solver
    inputs are built once on the host and resident in HBM before the timed region."""
    import torch
    import torch.distributed as dist

    from oscar_mpc_planner_mr_modification_amd import native
    from oscar_mpc_planner_mr_modification_amd.bicycle import make_c3_batch
    from oscar_mpc_planner_mr_modification_amd.distributed import gather_winners, winner_records, winner_width

    S, N, nx, nu = args.scenes or 4096, lay.N, lay.nx, lay.nu
    B = S
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or min(16, os.cpu_count() or 1)
    t0 = time.time()
    b = make_c3_batch(lay, S, first_scene=rank * S)
    gen_s = time.time() - t0
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    d_par, d_warm, d_xi = t(b.params), t(b.warm), t(b.xinit)
    pr = native.problem_from_layout(lay)
    out = dict(xtraj=torch.empty((B, N + 1, nx), dtype=torch.float64, device=dev),
               utraj=torch.empty((B, N, nu), dtype=torch.float64, device=dev),
               pobj=torch.empty((B,), dtype=torch.float64, device=dev),
               exit=torch.empty((B,), dtype=torch.int32, device=dev),
               info=torch.empty((B, 4), dtype=torch.int32, device=dev))
    win_w = winner_width(N, nx, nu)
    winners = torch.empty((S, win_w), dtype=torch.float64, device=dev)
    gathered = torch.empty((S * world, win_w), dtype=torch.float64, device=dev) if world > 1 else None
    stream = torch.cuda.current_stream(dev)
    ev = [[torch.cuda.Event(enable_timing=True) for _ in range(2)] for _ in range(args.steps)]

    def step(i=None):
        if i is not None:
            ev[i][0].record(stream)
        native.solve_batch_device(pr, d_par, d_warm, d_xi, out=out, stream=stream)
        if i is not None:
            ev[i][1].record(stream)
        best = torch.where(out["exit"] == 1, 0, -1).to(torch.int32)
        winner_records(out["xtraj"], out["utraj"], out["pobj"], best, 1, out=winners)
        if world > 1:
            gather_winners(winners, world, out=gathered)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t_start = time.perf_counter()
    for i in range(args.steps):
        step(i)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t_start
    kern_ms = float(np.mean([e[0].elapsed_time(e[1]) for e in ev]))
    if world > 1:
        te = torch.tensor([elapsed, kern_ms], dtype=torch.float64, device=dev)
        dist.all_reduce(te, op=dist.ReduceOp.MAX)
        elapsed, kern_ms = float(te[0]), float(te[1])
    value = args.steps * B * world / elapsed
    exit_h, xt_h, info_h = out["exit"].cpu().numpy(), out["xtraj"].cpu().numpy(), out["info"].cpu().numpy()
    bps = algorithmic_bytes_per_solve(lay)
    achieved = bps * B / (kern_ms * 1e-3) / 1e9
    traffic = None
    if os.path.exists(args.traffic_json):
        try:
            tj = json.load(open(args.traffic_json))
            if tj.get("config") == args.config and tj.get("batch") == B:
                traffic = tj.get("hbm_bytes_per_launch")
        except Exception:
            traffic = None
    result = {
        "metric": METRIC, "value": round(value, 2), "unit": "solves/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f64",
        "data": "synthetic (seeded scenes, SURVEY.md §8d C3)",
        "config": {"workload": f"C3: BicycleModel2ndOrderCurvatureAware + CA-MPC contouring + {lay.n_scen} decomp "
                               f"halfspaces, N={N}, {S} scenes per GPU, 10 SQP-RTI iterations",
                   "scenes_per_gpu": S, "N": N,
                   "parallelism": f"scene-sharded x{world}" + (" + RCCL all-gather of results" if world > 1 else "")},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 3), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "kernel": "sqp_kernel",
                     "kernel_ms": round(kern_ms, 4), "bytes_per_solve": bps},
        "solver_stats": {"success_frac": float((exit_h == 1).mean()), "qp_iters_per_solve": float(info_h[:, 1].mean()),
                         "scene_gen_s": round(gen_s, 2)},
        "phases_ms": {"solve": round(kern_ms, 4)},
    }
    if rank == 0 and world == 1 and not args.no_cpu:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle_py

        oracle_py.build()
        orc = oracle_py.Oracle(lay)
        done, t_cpu, chunk = 0, 0.0, 256
        max_abs_dx, agree, compared = 0.0, 0, 0
        while done < B and t_cpu < args.cpu_seconds:
            sl = slice(done, min(B, done + chunk))
            tc = time.perf_counter()
            ref = orc.solve_batch(b.params[sl], b.warm[sl], b.xinit[sl], nthreads=threads)
            t_cpu += time.perf_counter() - tc
            ok = (ref["status"] == 1) & (exit_h[sl] == 1)
            if ok.any():
                max_abs_dx = max(max_abs_dx, float(np.abs(xt_h[sl][ok] - ref["xtraj"][ok]).max()))
            agree += int((ref["status"] == exit_h[sl]).sum())
            compared += len(ref["status"])
            done = sl.stop
        tc = time.perf_counter()
        orc.solve_batch(b.params[:64], b.warm[:64], b.xinit[:64], nthreads=1)
        r1 = 64 / (time.perf_counter() - tc)
        result["cpu_baseline"] = {"value": round(done / t_cpu, 2), "unit": "solves/s", "cores": threads,
                                  "kind": "port",
                                  "sample": f"first {done} of the {B} solves of this batch, C oracle (same algorithm), "
                                            f"OpenMP {threads} threads",
                                  "single_thread_solves_per_s": round(r1, 2)}
        result["parity"] = {"max_abs_dx": max_abs_dx, "exit_agreement": agree / max(1, compared),
                            "solves_compared": compared, "tolerance": 1e-4}
        result["vs_cpu_baseline"] = round(value / (done / t_cpu), 2)
    if rank == 0:
        print(json.dumps(result))
    if world > 1:
        dist.destroy_process_group()


def run_shmpc(args, lay, world, rank, dev):
    """C5: SH-MPC step = scenario producer (samples -> halfspaces) + solve + lowest-cost pick + gather."""
    import torch
    import torch.distributed as dist

    from oscar_mpc_planner_mr_modification_amd import native
    from oscar_mpc_planner_mr_modification_amd.distributed import gather_winners, winner_records, winner_width
    from oscar_mpc_planner_mr_modification_amd.scenario import (OBSTACLE_RADIUS, PARALLEL_SOLVERS, ROBOT_RADIUS,
                                                                ScenarioScenes, make_shmpc_scenes,
                                                                prepare_scenario_host)
    from oscar_mpc_planner_mr_modification_amd.synthetic import DECELERATION

    S, P, N, nx = args.scenes or 2048, PARALLEL_SOLVERS, lay.N, lay.nx
    B = S * P
    n_obs, n_samples = 12, 100
    radius = ROBOT_RADIUS + OBSTACLE_RADIUS
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or min(16, os.cpu_count() or 1)
    t0 = time.time()
    workers = min(threads, 16)
    first = rank * S
    if workers > 1 and S >= 2 * workers:
        from concurrent.futures import ProcessPoolExecutor
        chunks = [c for c in np.array_split(np.arange(S), workers) if len(c)]
        with ProcessPoolExecutor(max_workers=workers) as ex:
            parts = list(ex.map(make_shmpc_scenes, [lay] * len(chunks), [len(c) for c in chunks],
                                [P] * len(chunks), [n_obs] * len(chunks), [n_samples] * len(chunks),
                                [20251212] * len(chunks), [first + int(c[0]) for c in chunks]))
        scenes = ScenarioScenes(stage_params=np.concatenate([q.stage_params for q in parts]),
                                state=np.concatenate([q.state for q in parts]),
                                samples=np.concatenate([q.samples for q in parts]), n_solvers=P)
        del parts
    else:
        scenes = make_shmpc_scenes(lay, S, P, n_obs, n_samples, first_scene=first)
    gen_s = time.time() - t0
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    d_sp, d_st, d_smp = t(scenes.stage_params), t(scenes.state), t(scenes.samples)
    pr = native.problem_from_layout(lay)
    prep = dict(params=torch.empty((B, N, lay.npar), dtype=torch.float64, device=dev),
                warm=torch.empty((B, N + 1, lay.nvar), dtype=torch.float64, device=dev),
                xinit=torch.empty((B, nx), dtype=torch.float64, device=dev))
    out = dict(xtraj=torch.empty((B, N + 1, nx), dtype=torch.float64, device=dev),
               utraj=torch.empty((B, N, 2), dtype=torch.float64, device=dev),
               pobj=torch.empty((B,), dtype=torch.float64, device=dev),
               exit=torch.empty((B,), dtype=torch.int32, device=dev),
               info=torch.empty((B, 4), dtype=torch.int32, device=dev))
    best = torch.empty((S,), dtype=torch.int32, device=dev)
    win_w = winner_width(N, nx)
    winners = torch.empty((S, win_w), dtype=torch.float64, device=dev)
    gathered = torch.empty((S * world, win_w), dtype=torch.float64, device=dev) if world > 1 else None
    stream = torch.cuda.current_stream(dev)
    ev = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(args.steps)]

    def step(i=None):
        if i is not None:
            ev[i][0].record(stream)
        native.prepare_scenario_device(pr, P, d_sp, d_st, d_smp, radius, DECELERATION, out=prep, stream=stream)
        if i is not None:
            ev[i][1].record(stream)
        native.solve_batch_device(pr, prep["params"], prep["warm"], prep["xinit"], out=out, stream=stream)
        if i is not None:
            ev[i][2].record(stream)
        native.select_lowest_cost_device(S, P, out["pobj"], out["exit"], out=best, stream=stream)
        winner_records(out["xtraj"], out["utraj"], out["pobj"], best, P, out=winners)
        if world > 1:
            gather_winners(winners, world, out=gathered)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t_start = time.perf_counter()
    for i in range(args.steps):
        step(i)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t_start
    prep_ms = float(np.mean([e[0].elapsed_time(e[1]) for e in ev]))
    kern_ms = float(np.mean([e[1].elapsed_time(e[2]) for e in ev]))
    if world > 1:
        te = torch.tensor([elapsed, kern_ms], dtype=torch.float64, device=dev)
        dist.all_reduce(te, op=dist.ReduceOp.MAX)
        elapsed, kern_ms = float(te[0]), float(te[1])
    value = args.steps * B * world / elapsed
    exit_h, xt_h, info_h = out["exit"].cpu().numpy(), out["xtraj"].cpu().numpy(), out["info"].cpu().numpy()
    best_h = best.cpu().numpy()
    prep_h = {k: v.cpu().numpy() for k, v in prep.items()} if (rank == 0 and world == 1 and not args.no_cpu) else None
    bps = algorithmic_bytes_per_solve(lay)
    achieved = bps * B / (kern_ms * 1e-3) / 1e9
    # the producer is the HBM-heavy kernel: every sample read once
    prep_bytes = B * ((N - 1) * n_obs * n_samples * 16 + N * lay.npar * 8 + (N + 1) * lay.nvar * 8)
    traffic = None
    if os.path.exists(args.traffic_json):
        try:
            tj = json.load(open(args.traffic_json))
            if tj.get("config") == args.config and tj.get("batch") == B:
                traffic = tj.get("hbm_bytes_per_launch")
        except Exception:
            traffic = None
    result = {
        "metric": METRIC, "value": round(value, 2), "unit": "solves/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f64",
        "data": "synthetic (seeded scenes, SURVEY.md §8d C5)",
        "config": {"workload": f"C5: SH-MPC slack model, N={N}, {lay.n_scen} scenario halfspaces per stage from "
                               f"{n_obs} obstacles x {n_samples} samples, {S} scenes x {P} parallel solvers per GPU, "
                               f"10 SQP-RTI iterations",
                   "scenes_per_gpu": S, "parallel_solvers": P, "N": N,
                   "parallelism": f"scene-sharded x{world}" + (" + RCCL all-gather of winners" if world > 1 else "")},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 3), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "kernel": "sqp_kernel",
                     "kernel_ms": round(kern_ms, 4), "bytes_per_solve": bps,
                     "producer": {"kernel": "scenario_prepare_kernel", "kernel_ms": round(prep_ms, 4),
                                  "algorithmic_gbs": round(prep_bytes / (prep_ms * 1e-3) / 1e9, 2),
                                  "frac": prep_bytes / (prep_ms * 1e-3) / 1e9 / HBM_PEAK_GBS}},
        "solver_stats": {"success_frac": float((exit_h == 1).mean()), "scene_feasible_frac": float((best_h >= 0).mean()),
                         "qp_iters_per_solve": float(info_h[:, 1].mean()), "scene_gen_s": round(gen_s, 2)},
        "phases_ms": {"prepare": round(prep_ms, 4), "solve": round(kern_ms, 4)},
    }
    if rank == 0 and world == 1 and not args.no_cpu:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle_py

        oracle_py.build()
        orc = oracle_py.Oracle(lay)
        done_sc, t_cpu, chunk = 0, 0.0, 64
        max_abs_dx, agree, compared, prod_dev = 0.0, 0, 0, 0.0
        host_b = None
        while done_sc < S and t_cpu < args.cpu_seconds:
            sl = slice(done_sc, min(S, done_sc + chunk))
            bs = slice(sl.start * P, sl.stop * P)
            if done_sc < 4 * chunk:
                # producer check on the first chunks: host restatement vs the GPU's inputs
                sub = ScenarioScenes(stage_params=scenes.stage_params[sl], state=scenes.state[sl],
                                     samples=scenes.samples[bs], n_solvers=P)
                hb = prepare_scenario_host(lay, sub, radius, DECELERATION)
                prod_dev = max(prod_dev, float(np.abs(hb.params - prep_h["params"][bs]).max()),
                               float(np.abs(hb.warm - prep_h["warm"][bs]).max()))
            # the oracle solves the GPU producer's inputs, so parity isolates the solve
            prm, wrm, xin = prep_h["params"][bs], prep_h["warm"][bs], prep_h["xinit"][bs]
            host_b = (prm, wrm, xin) if host_b is None else host_b
            tc = time.perf_counter()
            ref = orc.solve_batch(prm, wrm, xin, nthreads=threads)
            t_cpu += time.perf_counter() - tc
            ok = (ref["status"] == 1) & (exit_h[bs] == 1)
            if ok.any():
                max_abs_dx = max(max_abs_dx, float(np.abs(xt_h[bs][ok] - ref["xtraj"][ok]).max()))
            agree += int((ref["status"] == exit_h[bs]).sum())
            compared += len(ref["status"])
            done_sc = sl.stop
        done = done_sc * P
        tc = time.perf_counter()
        n1 = min(64, len(host_b[0]))
        orc.solve_batch(host_b[0][:n1], host_b[1][:n1], host_b[2][:n1], nthreads=1)
        r1 = n1 / (time.perf_counter() - tc)
        result["cpu_baseline"] = {"value": round(done / t_cpu, 2), "unit": "solves/s", "cores": threads,
                                  "kind": "port",
                                  "sample": f"first {done} of the {B} solves of this batch (the GPU producer's "
                                            f"inputs), C oracle (same algorithm), OpenMP {threads} threads",
                                  "single_thread_solves_per_s": round(r1, 2)}
        result["parity"] = {"max_abs_dx": max_abs_dx, "exit_agreement": agree / max(1, compared),
                            "solves_compared": compared, "tolerance": 1e-4,
                            "producer_max_abs_diff": prod_dev}
        result["vs_cpu_baseline"] = round(value / (done / t_cpu), 2)
    if rank == 0:
        print(json.dumps(result))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
