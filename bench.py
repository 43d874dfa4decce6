#!/usr/bin/env python3
"""Benchmark of the MI355X T-MPC++ per-guess SQP backend.

Workload (BASELINE.json configs[1], "C2"): jackal unicycle T-MPC++, N=20,
8 obstacles, 1024 synthetic scenes x 8 topology guesses per GPU (7 guided +
the non-guided T-MPC++ planner), up to 10 SQP-RTI iterations per solve (the
reference's loop breaks on a failed QP; `solver_stats.rti_iters_per_solve` is
the executed count), timeout disabled.  One step = one control step of every
scene, all on the GPU: per-guess solver inputs from the scene data
(mpcg_prepare: warm starts, topology halfspaces with Douglas-Rachford
projection, obstacles, consistency references) + one batched solve of all
scenes x guesses + per-scene planner selection (FindBestPlanner with the
consistency and selection-weight bookkeeping) + one RCCL all-gather of the
winning trajectories when N_gpus > 1 (scenes are sharded, weak scaling).
Scene data is uploaded once before the timed region (inputs resident in HBM).

    python bench.py [--gpus N --steps K --warmup W] [--config C2|C3|C4|C5]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N ...

`--gpus N > 1` without a launcher (no WORLD_SIZE in the environment) starts the N
rank processes itself: torch.distributed.run as a CHILD process (one rank per GPU,
RCCL), before this process touches torch or the GPU, and exits with its code.

Rank 0 prints one JSON line.  `roofline` prices the solve kernel against the
fp64 vector peak with the algorithm's analytic operation count
(oscar_mpc_planner_mr_modification_amd/flopmodel.py, times the SQP and IPM
iterations each solve executed; the path is fp64-latency bound);
`roofline.hbm` prices it against HBM with SURVEY.md §8(d)'s algorithmic bytes
per solve; `roofline.traffic` comes from the rocprofv3 PMC
summary under profiles/ only when that summary was taken on the same kernel
sources (source hash), else it is null.  `cpu_baseline` times the C oracle
(same algorithm, OpenMP over solves) on a bounded sample of the same batch
(rank 0, N=1), and `parity` is the oracle check of that sample; at N>1 every
rank checks a sample of its own shard and the results are reduced over ranks.

`--config C3`: the curvature-aware bicycle workload, 4096
scenes per GPU, N=30, CA spline update, CA contouring and 12 decomp
halfspaces per stage, one solver per scene.
`--config C4`: N=30, 12 obstacles, 2048 scenes x 8 guesses per GPU (one GPU's
shard of BASELINE.json configs[3]).
`--config JS`: the reference's shipped jackalsimulator solver (N=30, 4 obstacles,
4 guided + 1 non-guided planners), 4096 scenes x 5 planners per GPU.
`--config C5`: SH-MPC, 2048 scenes x 4 parallel scenario solvers per GPU on the
slack model, 24 scenario halfspaces per stage reduced on the GPU from 12
obstacles x 100 prediction samples (mpcg_prepare_scenario), batched solve,
lowest-cost pick (ScenarioConstraints::optimize) and the winner gather.
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
DEFAULT_SCENES = {"C1": 1024, "C2": 1024, "C3": 4096, "C4": 2048, "C5": 2048, "JS": 4096, "JD": 4096,
                  "T10": 2048}  # T10: diagnostic shape for register-budget A/B runs, not a BASELINE config
# jackalsimulator / jackal / dingo as shipped: n_paths 4 + the non-guided planner
DEFAULT_GUESSES = {"JS": 5, "JD": 5}
CHECK_CHUNK = 256              # solves per oracle call in the check leg
RANK_SAMPLE = 256              # solves each rank checks at N > 1


def algorithmic_bytes_per_solve(lay):
    """B = 8*[N*npar + (N+1)*nvar + nx + (N+1)*nx + N*nu + 2]"""
    N = lay.N
    return 8 * (N * lay.npar + (N + 1) * lay.nvar + lay.nx + (N + 1) * lay.nx + N * lay.nu + 2)


def load_counters(path, config, batch):
    """PMC summary (scripts/summarize_profile.py) of the solve kernel, used only when it
    was collected on the same kernel sources and batch: returns (traffic, fp64, note)."""
    from oscar_mpc_planner_mr_modification_amd._build import source_hash

    if not os.path.exists(path):
        return None, None, "no PMC summary"
    try:
        tj = json.load(open(path))
    except Exception as e:  # noqa: BLE001
        return None, None, f"unreadable PMC summary: {e}"
    if tj.get("config") != config or tj.get("batch") != batch:
        return None, None, f"PMC summary {tj.get('tag')} is for {tj.get('config')} batch {tj.get('batch')}"
    if tj.get("source_sha256") != source_hash():
        return None, None, f"PMC summary {tj.get('tag')} was taken on other kernel sources (stale)"
    f64 = tj.get("fp64_issued_flop_per_launch")
    if f64:
        f64 = {"flop": f64, "lane_util": tj.get("valu_lane_util")}
    return tj.get("hbm_bytes_per_launch"), f64, f"profiles/{tj.get('tag')}"


def cpu_share():
    """CPUs this job may use on the host: nproc, the affinity mask, the cgroup CPU quota
    (cgroup v2 cpu.max or v1 cfs_quota_us / cfs_period_us) and OMP_NUM_THREADS if set.
    On the GPU box nproc counts the whole machine while the job's share is a slice of it
    (the pool sets OMP_NUM_THREADS to that share), so the CPU baseline's widest leg runs
    on `share` threads and reports nproc beside it."""
    nproc = os.cpu_count() or 1
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else nproc
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        quota = None if q == "max" else int(q) / int(per)
    except (OSError, ValueError):
        try:
            q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
            per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
            quota = q / per if q > 0 else None
        except (OSError, ValueError):
            pass
    share = aff if quota is None else max(1, min(aff, int(quota)))
    omp = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    if omp > 0:
        share = min(share, omp)
    return {"nproc": nproc, "affinity": aff, "cgroup_quota": quota, "omp_num_threads": omp or None,
            "share": share}


def spawn_ranks(n, argv):
    """`bench.py --gpus N` without a launcher: run torch.distributed.run as a child process
    (one rank per GPU, rendezvous on 127.0.0.1, a free port) and return its exit code.  The
    parent has not imported torch nor touched the GPU; it never re-execs itself."""
    import socket
    import subprocess

    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + list(argv)
    return subprocess.call(cmd, env=dict(os.environ))


def spawn_check(world, config="C4", per_rank=None):
    """--spawn-check (CPU test of the rank spawning and of the step's collective): every rank joins a
    gloo group and counts the ranks, then runs the winner all-gather the timed step runs at this
    world size on host tensors: the weak-scaling shards of `config` (per_rank scenes each, the
    bench's default per GPU: C4 2048, i.e. BASELINE config 4's 16,384 scenes over 8 ranks) into the
    preallocated result buffer, and an uneven sharding of the same total plus 3 scenes (ranks with
    one scene fewer; distributed.gather_winners(total=...)).  Each record holds its global scene
    index, so rank 0 checks both gathers exactly; it prints one JSON line."""
    import torch
    import torch.distributed as dist

    from oscar_mpc_planner_mr_modification_amd.distributed import gather_winners, shard, winner_width
    from oscar_mpc_planner_mr_modification_amd.layouts import config_layout

    rank = int(os.environ.get("RANK", "0"))
    if world > 1:
        dist.init_process_group("gloo")
    t = torch.ones(1)
    if world > 1:
        dist.all_reduce(t)
    lay = config_layout(config)
    S = per_rank or DEFAULT_SCENES[config]
    w = winner_width(lay.N, lay.nx, lay.nu)

    def records(first, count):
        # scene s: column j holds s + j / w (distinct per scene and column, exact in f64)
        s = torch.arange(first, first + count, dtype=torch.float64)[:, None]
        return s + torch.arange(w, dtype=torch.float64)[None, :] / w

    even = torch.empty((S * world, w), dtype=torch.float64)
    got_even = gather_winners(records(rank * S, S), world, out=even)
    total = S * world + 3
    first, count = shard(total, world, rank)
    got_uneven = gather_winners(records(first, count), world, total=total)
    ok = bool(torch.equal(got_even, records(0, S * world)) and torch.equal(got_uneven, records(0, total)))
    if world > 1:
        flag = torch.tensor([1.0 if ok else 0.0])
        dist.all_reduce(flag, op=dist.ReduceOp.MIN)
        ok = bool(flag.item() == 1.0)
    if rank == 0:
        print(json.dumps({"spawn_check": True, "n_gpus": world, "ranks_seen": int(t.item()),
                          "local_ranks": world, "config": config, "scenes_per_rank": S,
                          "gather_even_scenes": S * world, "gather_uneven_scenes": total, "gather_ok": ok}))
    if world > 1:
        dist.destroy_process_group()


# ----------------------------------------------------------------- workloads
class Workload:
    """One config's GPU step: `step(timed)` enqueues one control step of every scene
    on `stream`; phase events are recorded when timed."""
    phases = ("solve",)

    def __init__(self, args, lay, rank, world, dev):
        self.args, self.lay, self.rank, self.world, self.dev = args, lay, rank, world, dev
        self.S = args.scenes or DEFAULT_SCENES[args.config]
        self.threads = cpu_share()["share"]

    def host_inputs(self, lo, hi):
        """host copies (params, warm, xinit) of solves [lo, hi) for the oracle check"""
        raise NotImplementedError

    def gather(self, winners):
        from oscar_mpc_planner_mr_modification_amd.distributed import gather_winners
        if self.world > 1:
            gather_winners(winners, self.world, out=self.gathered)


class TmpcWorkload(Workload):
    """C1 / C2 / C4 / JS: T-MPC++ control step (prepare -> solve -> select -> winner records)."""
    phases = ("prepare", "solve")

    def __init__(self, args, lay, rank, world, dev):
        super().__init__(args, lay, rank, world, dev)
        import torch

        from oscar_mpc_planner_mr_modification_amd import native
        from oscar_mpc_planner_mr_modification_amd.distributed import winner_width
        from oscar_mpc_planner_mr_modification_amd.synthetic import make_batch

        S, G, N = self.S, args.guesses, lay.N
        self.G, self.B = G, S * G
        t0 = time.time()
        self.batch = make_batch(lay, S, G, first_scene=rank * S, workers=min(self.threads, 16))
        self.gen_s = time.time() - t0
        self.scenes = self.batch.scenes
        self.dsc = native.scenes_to_device(self.scenes, dev)
        self.pr = native.problem_from_layout(lay, qp_warm_start=args.qp_warm_start, qp_warm_first=args.qp_warm_first,
                                             solver_type=args.solver_type, qp_profile=args.qp_profile)
        B = self.B
        f64 = dict(dtype=torch.float64, device=dev)
        self.prep = dict(params=torch.empty((B, N, lay.npar), **f64), warm=torch.empty((B, N + 1, 7), **f64),
                         xinit=torch.empty((B, 5), **f64), prev_interp=torch.empty((S, N, 2), **f64),
                         consistency_active=torch.empty((B,), dtype=torch.uint8, device=dev))
        self.out = dict(xtraj=torch.empty((B, N + 1, 5), **f64), utraj=torch.empty((B, N, 2), **f64),
                        pobj=torch.empty((B,), **f64), exit=torch.empty((B,), dtype=torch.int32, device=dev),
                        info=torch.empty((B, 4), dtype=torch.int32, device=dev))
        self.winners = torch.empty((S, winner_width(N)), **f64)
        self.gathered = torch.empty((S * world, winner_width(N)), **f64) if world > 1 else None
        self.workload = (f"{args.config}: jackal unicycle T-MPC++, N={N}, {lay.max_obstacles} obstacles, {S} scenes x "
                         f"{G} guesses per GPU, up to {lay.sqp_iters} SQP-RTI iterations per solve")
        self.config = {"scenes_per_gpu": S, "guesses": G, "N": N, "obstacles": lay.max_obstacles}

    def step(self, ev=None):
        from oscar_mpc_planner_mr_modification_amd import native
        from oscar_mpc_planner_mr_modification_amd.synthetic import DECELERATION, ROBOT_RADIUS, SETTINGS_WEIGHTS

        s = self.stream
        if ev:
            ev[0].record(s)
        native.prepare_device(self.pr, self.dsc, ROBOT_RADIUS, SETTINGS_WEIGHTS["consistency"], DECELERATION,
                              out=self.prep, stream=s)
        if ev:
            ev[1].record(s)
        native.solve_batch_device(self.pr, self.prep["params"], self.prep["warm"], self.prep["xinit"], out=self.out,
                                  stream=s)
        if ev:
            ev[2].record(s)
        best, _ = native.select_best_device(self.S, self.G, self.lay.N, self.out["xtraj"], self.out["pobj"],
                                            self.out["exit"], prev_traj=self.prep["prev_interp"],
                                            w_cons=SETTINGS_WEIGHTS["consistency"],
                                            consistency_enabled=self.prep["consistency_active"],
                                            previously_selected=self.dsc["previously_selected"],
                                            selection_weight=0.75, stream=s)   # guidance_planner.yaml:37
        native.winner_records_device(self.out["xtraj"], self.out["utraj"], self.out["pobj"], best, self.G, self.winners,
                                     stream=s)
        self.gather(self.winners)

    def host_inputs(self, lo, hi):
        # the GPU producer is bit-identical to the host restatement (tests/test_producers.py)
        b = self.batch
        return b.params[lo:hi], b.warm[lo:hi], b.xinit[lo:hi]


class C3Workload(Workload):
    """C3: one batched solve of every scene's bicycle CA-MPC problem + the result gather
    (the decomp halfspaces come from DecompUtil, external, so the per-scene solver inputs
    are built on the host once, resident in HBM before the timed region)."""

    def __init__(self, args, lay, rank, world, dev):
        super().__init__(args, lay, rank, world, dev)
        import torch

        from oscar_mpc_planner_mr_modification_amd import native
        from oscar_mpc_planner_mr_modification_amd.bicycle import make_c3_batch
        from oscar_mpc_planner_mr_modification_amd.distributed import winner_width

        S, N, nx, nu = self.S, lay.N, lay.nx, lay.nu
        self.B = S
        t0 = time.time()
        self.b = make_c3_batch(lay, S, first_scene=rank * S)
        self.gen_s = time.time() - t0
        t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
        self.d_par, self.d_warm, self.d_xi = t(self.b.params), t(self.b.warm), t(self.b.xinit)
        self.pr = native.problem_from_layout(lay, qp_warm_start=args.qp_warm_start, qp_warm_first=args.qp_warm_first,
                                             solver_type=args.solver_type, qp_profile=args.qp_profile)
        f64 = dict(dtype=torch.float64, device=dev)
        self.out = dict(xtraj=torch.empty((S, N + 1, nx), **f64), utraj=torch.empty((S, N, nu), **f64),
                        pobj=torch.empty((S,), **f64), exit=torch.empty((S,), dtype=torch.int32, device=dev),
                        info=torch.empty((S, 4), dtype=torch.int32, device=dev))
        self.winners = torch.empty((S, winner_width(N, nx, nu)), **f64)
        self.gathered = torch.empty((S * world, winner_width(N, nx, nu)), **f64) if world > 1 else None
        self.workload = (f"C3: BicycleModel2ndOrderCurvatureAware + CA-MPC contouring + {lay.n_scen} decomp "
                         f"halfspaces, N={N}, {S} scenes per GPU, up to {lay.sqp_iters} SQP-RTI iterations per solve")
        self.config = {"scenes_per_gpu": S, "N": N}

    def step(self, ev=None):
        import torch

        from oscar_mpc_planner_mr_modification_amd import native

        s = self.stream
        if ev:
            ev[0].record(s)
        native.solve_batch_device(self.pr, self.d_par, self.d_warm, self.d_xi, out=self.out, stream=s)
        if ev:
            ev[1].record(s)
        best = torch.where(self.out["exit"] == 1, 0, -1).to(torch.int32)
        native.winner_records_device(self.out["xtraj"], self.out["utraj"], self.out["pobj"], best, 1, self.winners, stream=s)
        self.gather(self.winners)

    def host_inputs(self, lo, hi):
        b = self.b
        return b.params[lo:hi], b.warm[lo:hi], b.xinit[lo:hi]


class ShmpcWorkload(Workload):
    """C5: SH-MPC step = scenario producer (samples -> halfspaces) + solve + lowest-cost pick + gather."""
    phases = ("prepare", "solve")

    def __init__(self, args, lay, rank, world, dev):
        super().__init__(args, lay, rank, world, dev)
        import torch

        from oscar_mpc_planner_mr_modification_amd import native
        from oscar_mpc_planner_mr_modification_amd.distributed import winner_width
        from oscar_mpc_planner_mr_modification_amd.scenario import (OBSTACLE_RADIUS, PARALLEL_SOLVERS, ROBOT_RADIUS,
                                                                    ScenarioScenes, make_shmpc_scenes)

        S, P, N, nx = self.S, PARALLEL_SOLVERS, lay.N, lay.nx
        self.P, self.B = P, S * P
        self.n_obs, self.n_samples = 12, 100
        self.radius = ROBOT_RADIUS + OBSTACLE_RADIUS
        t0 = time.time()
        workers, first = min(self.threads, 16), rank * S
        if workers > 1 and S >= 2 * workers:
            from concurrent.futures import ProcessPoolExecutor
            chunks = [c for c in np.array_split(np.arange(S), workers) if len(c)]
            with ProcessPoolExecutor(max_workers=workers) as ex:
                parts = list(ex.map(make_shmpc_scenes, [lay] * len(chunks), [len(c) for c in chunks],
                                    [P] * len(chunks), [self.n_obs] * len(chunks), [self.n_samples] * len(chunks),
                                    [20251212] * len(chunks), [first + int(c[0]) for c in chunks]))
            self.scenes = ScenarioScenes(stage_params=np.concatenate([q.stage_params for q in parts]),
                                         state=np.concatenate([q.state for q in parts]),
                                         samples=np.concatenate([q.samples for q in parts]), n_solvers=P,
                                         main_warm=np.concatenate([q.main_warm for q in parts]))
            del parts
        else:
            self.scenes = make_shmpc_scenes(lay, S, P, self.n_obs, self.n_samples, first_scene=first)
        self.gen_s = time.time() - t0
        t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
        self.d_sp, self.d_st, self.d_smp = t(self.scenes.stage_params), t(self.scenes.state), t(self.scenes.samples)
        self.d_mw = t(self.scenes.main_warm)   # the main solver's previous plan (scenario.previous_plan)
        self.pr = native.problem_from_layout(lay, qp_warm_start=args.qp_warm_start, qp_warm_first=args.qp_warm_first,
                                             solver_type=args.solver_type, qp_profile=args.qp_profile)
        B = self.B
        f64 = dict(dtype=torch.float64, device=dev)
        self.prep = dict(params=torch.empty((B, N, lay.npar), **f64), warm=torch.empty((B, N + 1, lay.nvar), **f64),
                         xinit=torch.empty((B, nx), **f64))
        self.out = dict(xtraj=torch.empty((B, N + 1, nx), **f64), utraj=torch.empty((B, N, 2), **f64),
                        pobj=torch.empty((B,), **f64), exit=torch.empty((B,), dtype=torch.int32, device=dev),
                        info=torch.empty((B, 4), dtype=torch.int32, device=dev))
        self.best = torch.empty((S,), dtype=torch.int32, device=dev)
        self.winners = torch.empty((S, winner_width(N, nx)), **f64)
        self.gathered = torch.empty((S * world, winner_width(N, nx)), **f64) if world > 1 else None
        self.workload = (f"C5: SH-MPC slack model, N={N}, {lay.n_scen} scenario halfspaces per stage from "
                         f"{self.n_obs} obstacles x {self.n_samples} samples, {S} scenes x {P} parallel solvers "
                         f"per GPU, up to {lay.sqp_iters} SQP-RTI iterations per solve")
        self.config = {"scenes_per_gpu": S, "parallel_solvers": P, "N": N}
        self._host = None

    def step(self, ev=None):
        from oscar_mpc_planner_mr_modification_amd import native
        from oscar_mpc_planner_mr_modification_amd.synthetic import DECELERATION

        s = self.stream
        if ev:
            ev[0].record(s)
        native.prepare_scenario_device(self.pr, self.P, self.d_sp, self.d_st, self.d_smp, self.radius, DECELERATION,
                                       main_warm=self.d_mw, out=self.prep, stream=s)
        if ev:
            ev[1].record(s)
        native.solve_batch_device(self.pr, self.prep["params"], self.prep["warm"], self.prep["xinit"], out=self.out,
                                  stream=s)
        if ev:
            ev[2].record(s)
        native.select_lowest_cost_device(self.S, self.P, self.out["pobj"], self.out["exit"], out=self.best, stream=s)
        native.winner_records_device(self.out["xtraj"], self.out["utraj"], self.out["pobj"], self.best, self.P,
                                     self.winners, stream=s)
        self.gather(self.winners)

    def host_inputs(self, lo, hi):
        # the oracle solves the GPU producer's inputs, so parity isolates the solve; the
        # producer itself is checked against the host restatement on the first scenes
        if self._host is None:
            self._host = {k: v.cpu().numpy() for k, v in self.prep.items()}
        h = self._host
        return h["params"][lo:hi], h["warm"][lo:hi], h["xinit"][lo:hi]

    def producer_check(self, n_scenes=64):
        from oscar_mpc_planner_mr_modification_amd.scenario import ScenarioScenes, prepare_scenario_host
        from oscar_mpc_planner_mr_modification_amd.synthetic import DECELERATION

        n = min(n_scenes, self.S)
        sub = ScenarioScenes(stage_params=self.scenes.stage_params[:n], state=self.scenes.state[:n],
                             samples=self.scenes.samples[:n * self.P], n_solvers=self.P,
                             main_warm=self.scenes.main_warm[:n])
        hb = prepare_scenario_host(self.lay, sub, self.radius, DECELERATION)
        prm, wrm, _ = self.host_inputs(0, n * self.P)
        return max(float(np.abs(hb.params - prm).max()), float(np.abs(hb.warm - wrm).max()))

    def producer_roofline(self, prep_ms):
        lay, N = self.lay, self.lay.N
        # the producer reads every sample and the previous plan once and streams the solver inputs out
        prep_bytes = self.B * ((N - 1) * self.n_obs * self.n_samples * 16 + N * lay.npar * 8 + (N + 1) * lay.nvar * 8)
        prep_bytes += self.S * (N + 1) * lay.nvar * 8
        gbs = prep_bytes / (prep_ms * 1e-3) / 1e9
        return {"kernel": "scenario_prepare_kernel", "kernel_ms": round(prep_ms, 4), "algorithmic_gbs": round(gbs, 2),
                "frac": gbs / HBM_PEAK_GBS}


# ----------------------------------------------------------------- check leg
def oracle_check(wl, orc, lo, hi, exit_h, xt_h, info_h, nthreads):
    """oracle on solves [lo, hi): (seconds, max dx over successful solves, max dx over failed solves
    that took the same path on both sides, agreeing exit codes, compared)"""
    prm, wrm, xin = wl.host_inputs(lo, hi)
    tc = time.perf_counter()
    ref = orc.solve_batch(prm, wrm, xin, nthreads=nthreads)
    sec = time.perf_counter() - tc
    ex, xt, inf = exit_h[lo:hi], xt_h[lo:hi], info_h[lo:hi]
    same = ref["status"] == ex
    dx = np.abs(xt - ref["xtraj"]).reshape(len(ex), -1).max(1)
    ok = same & (ex == 1)
    # failed solves that took the same path on both sides with every accepted step from a
    # converged QP (no max-iter QP): their last iterates must agree like successful ones
    path = (same & (ex != 1) & (inf[:, 0] == ref["sqp_iter"]) & (inf[:, 1] == ref["qp_iter"]) &
            (inf[:, 3] == 0) & (ref["qp_maxiter"] == 0))
    # the oracle's rare interior-point passes on these solves (centring re-solves, refinement solves)
    # and its IPM iterations: the rates the executed-work flop count uses (flopmodel.solve_ops_executed)
    rare = np.array([ref["qp_iter"].sum(), ref["qp_center"].sum(), ref["qp_itref"].sum()], dtype=np.float64)
    return (sec, float(dx[ok].max()) if ok.any() else 0.0, float(dx[path].max()) if path.any() else 0.0,
            int(same.sum()), len(ex), rare)


def native_problem(lay, args, profile):
    from oscar_mpc_planner_mr_modification_amd import native

    return native.problem_from_layout(lay, qp_warm_start=args.qp_warm_start, qp_warm_first=args.qp_warm_first,
                                      solver_type=args.solver_type, qp_profile=profile)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="C2", choices=sorted(DEFAULT_SCENES))
    ap.add_argument("--scenes", type=int, default=None, help="scenes per GPU (C2: 1024, C3: 4096, C4: 2048, C5: 2048)")
    ap.add_argument("--guesses", type=int, default=None, help="planners per scene (8; JS: 5)")
    ap.add_argument("--qp-warm-start", type=int, default=2, choices=(0, 2),
                    help="qp_solver_warm_start: 2 (the reference's, generate_acados_solver.py:173) or 0 cold")
    ap.add_argument("--solver-type", default="SQP_RTI", choices=("SQP_RTI", "SQP"),
                    help="solver_settings.acados.solver_type: SQP_RTI (default, every shipped config) or SQP "
                         "(one full acados SQP call per solve, DESIGN.md §2)")
    ap.add_argument("--qp-warm-first", type=int, default=0, choices=(0, 1),
                    help="acados warm_start_first_qp: 0 (default: every SQP-RTI QP starts cold), 1 warm-start "
                         "the first QP of each call too (DESIGN.md §2 'QP start')")
    ap.add_argument("--qp-profile", default="hpipm", choices=("hpipm", "robust"),
                    help="the interior point (DESIGN.md §2.2): hpipm = HPIPM's BALANCE mode as acados configures "
                         "it (the reference's configuration, default), robust = round 4's constants")
    ap.add_argument("--alt-steps", type=int, default=10,
                    help="N=1: also time this many steps with the other QP profile (0: skip)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="bound of the CPU-baseline sample")
    ap.add_argument("--no-cpu", action="store_true", help="skip the oracle (CPU baseline and parity)")
    ap.add_argument("--traffic-json", default=None, help="PMC summary (default profiles/traffic_<config>.json)")
    ap.add_argument("--spawn-check", action="store_true", help=argparse.SUPPRESS)
    args = ap.parse_args()
    if args.guesses is None:
        args.guesses = DEFAULT_GUESSES.get(args.config, 8)
    if args.traffic_json is None:
        args.traffic_json = os.path.join(ROOT, "profiles", f"traffic_{args.config}.json")

    # one process per GPU.  Without a launcher, --gpus N > 1 starts the N ranks as a child
    # torch.distributed.run (before any torch / GPU call here); under a launcher --gpus must
    # match its world size (checked before any GPU call)
    backend = os.environ.get("MPCG_BENCH_BACKEND", "nccl")
    if backend not in ("nccl", "gloo"):
        sys.exit(f"bench.py: MPCG_BENCH_BACKEND={backend}: expected nccl or gloo")
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(spawn_ranks(args.gpus, sys.argv[1:]))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if args.gpus != world:
        sys.exit(f"bench.py: --gpus {args.gpus} but the launcher's WORLD_SIZE={world} (one rank per GPU: "
                 f"`python -m torch.distributed.run --nnodes=1 --nproc-per-node {args.gpus} --master-addr "
                 f"127.0.0.1 bench.py --gpus {args.gpus} ...`, or plain `bench.py --gpus {args.gpus}`)")
    if args.spawn_check:
        return spawn_check(world, args.config, args.scenes)

    import torch
    import torch.distributed as dist

    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    # RCCL (one rank per GPU) is the product path; MPCG_BENCH_BACKEND=gloo is a rehearsal of the
    # multi-rank code on fewer GPUs (ranks share devices round-robin, collectives staged through
    # the host) and is labelled as such in the line
    n_dev = torch.cuda.device_count()  # (does not initialise the GPU)
    if backend == "gloo":
        local_rank = local_rank % max(1, n_dev)
    elif world > n_dev:
        sys.exit(f"bench.py: --gpus {world} with RCCL needs {world} GPUs, {n_dev} visible "
                 "(MPCG_BENCH_BACKEND=gloo rehearses the multi-rank path on fewer GPUs)")
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local_rank)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
        else:
            dist.init_process_group("gloo")
    dev = torch.device("cuda", local_rank)
    torch.cuda.set_device(dev)
    from oscar_mpc_planner_mr_modification_amd.distributed import all_reduce_

    from oscar_mpc_planner_mr_modification_amd.layouts import config_layout

    lay = config_layout(args.config)
    cls = {"C3": C3Workload, "C5": ShmpcWorkload}.get(args.config, TmpcWorkload)
    wl = cls(args, lay, rank, world, dev)
    wl.stream = torch.cuda.current_stream(dev)
    n_ev = len(wl.phases) + 1
    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(n_ev)] for _ in range(args.steps)]

    for _ in range(args.warmup):
        wl.step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t_start = time.perf_counter()
    for i in range(args.steps):
        wl.step(evs[i])
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t_start
    # per-phase kernel times from HIP events on the launch stream
    phase_ms = {p: float(np.mean([e[j].elapsed_time(e[j + 1]) for e in evs])) for j, p in enumerate(wl.phases)}
    if world > 1:
        te = torch.tensor([elapsed] + [phase_ms[p] for p in wl.phases], dtype=torch.float64, device=dev)
        all_reduce_(te, dist.ReduceOp.MAX)
        elapsed = float(te[0])
        phase_ms = {p: float(te[1 + j]) for j, p in enumerate(wl.phases)}
    kern_ms = phase_ms["solve"]
    # the other QP profile on the same batch (N = 1, after the timed region): the delta between the
    # reference's interior point and the robust one
    alt = None
    if world == 1 and args.alt_steps > 0:
        other = "robust" if args.qp_profile == "hpipm" else "hpipm"
        pr_main = wl.pr
        wl.pr = native_problem(lay, args, other)
        try:
            wl.step()
            torch.cuda.synchronize()
            aevs = [[torch.cuda.Event(enable_timing=True) for _ in range(n_ev)] for _ in range(args.alt_steps)]
            ta = time.perf_counter()
            for i in range(args.alt_steps):
                wl.step(aevs[i])
            torch.cuda.synchronize()
            ta = time.perf_counter() - ta
            ainfo = wl.out["info"].cpu().numpy()
            aexit = wl.out["exit"].cpu().numpy()
            alt = {"qp_profile": other, "value": round(args.alt_steps * wl.B / ta, 2),
                   "ms_per_step": round(ta / args.alt_steps * 1e3, 4),
                   "solve_kernel_ms": round(float(np.mean([e[wl.phases.index("solve")].elapsed_time(
                       e[wl.phases.index("solve") + 1]) for e in aevs])), 4),
                   "success_frac": float((aexit == 1).mean()), "qp_iters_per_solve": float(ainfo[:, 1].mean())}
        finally:
            wl.pr = pr_main
            wl.step()
            torch.cuda.synchronize()
    ranks_seen = 1
    if world > 1:
        rs = torch.ones(1, dtype=torch.float64, device=dev)
        all_reduce_(rs, dist.ReduceOp.SUM)
        ranks_seen = int(rs.item())
    B = wl.B
    value = args.steps * B * world / elapsed
    exit_h, xt_h, info_h = (wl.out[k].cpu().numpy() for k in ("exit", "xtraj", "info"))

    # roofline: the solve is fp64-latency bound, so it is priced against the fp64
    # vector peak with the ALGORITHM's operations (flopmodel.py: analytic counts per SQP and IPM
    # iteration, times the iterations each solve of this batch executed); HBM stays a secondary
    # figure with SURVEY.md §8(d)'s algorithmic bytes per solve
    from oscar_mpc_planner_mr_modification_amd import flopmodel

    # the executed algorithm: the base Mehrotra count plus, on HPIPM's profile,
    # the refinement test of every IPM iteration; the rare centring / refinement solves are added by
    # executed_flops below at the rates of the oracle's run on a sample of the batch (none without it)
    flop_base = float(flopmodel.solve_ops(lay, info_h).sum())
    flop = float(flopmodel.solve_ops_executed(lay, info_h, args.qp_profile).sum())
    tflops = flop / (kern_ms * 1e-3) / 1e12
    bps = algorithmic_bytes_per_solve(lay)
    achieved = bps * B / (kern_ms * 1e-3) / 1e9
    traffic, f64, counters = load_counters(args.traffic_json, args.config, B)
    roofline = {"bound": "fp64_valu", "achieved": round(tflops, 3), "peak": FP64_VALU_PEAK_TFLOPS,
                "unit": "TFLOP/s", "frac": tflops / FP64_VALU_PEAK_TFLOPS, "traffic": traffic,
                "kernel": "sqp_kernel", "kernel_ms": round(kern_ms, 4),
                "flop_per_solve": round(flop / B),
                "flop_model": ("analytic (flopmodel.solve_ops_executed) x executed iterations: the Mehrotra iteration, "
                               "HPIPM's refinement test per IPM iteration" if args.qp_profile == "hpipm" else
                               "analytic (flopmodel.solve_ops) x executed iterations"),
                "flop_per_solve_base": round(flop_base / B),
                "frac_base": (flop_base / (kern_ms * 1e-3) / 1e12) / FP64_VALU_PEAK_TFLOPS,
                "hbm": {"achieved": round(achieved, 3), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": achieved / HBM_PEAK_GBS, "bytes_per_solve": bps, "traffic": traffic},
                "counters": counters}
    def executed_flops(rare, source):
        """add the rare interior-point passes at the oracle sample's rates per IPM iteration"""
        if args.qp_profile != "hpipm" or rare[0] <= 0:
            return
        cr, ir = rare[1] / rare[0], rare[2] / rare[0]
        fl = float(flopmodel.solve_ops_executed(lay, info_h, "hpipm", cr, ir).sum())
        tf = fl / (kern_ms * 1e-3) / 1e12
        roofline.update({"achieved": round(tf, 3), "frac": tf / FP64_VALU_PEAK_TFLOPS, "flop_per_solve": round(fl / B)})
        roofline["flop_model"] += (f", centring re-solves ({cr:.4f} per IPM iteration) and refinement solves "
                                   f"({ir:.4f}) at {source} rates")

    if f64:
        # cross-check from the PMC pass on the same sources: issued fp64 FLOP/s of the solve kernel
        # (SQ_INSTS_VALU_*_F64 x 64 lanes, masked lanes included) and that figure weighted by the
        # kernel's VALU lane utilisation (rocprofv3 VALUUtilization)
        tf = f64["flop"] / (kern_ms * 1e-3) / 1e12
        roofline["fp64_valu_issued"] = {"achieved_tflops": round(tf, 3), "peak_tflops": FP64_VALU_PEAK_TFLOPS,
                                        "frac": tf / FP64_VALU_PEAK_TFLOPS}
        if f64.get("lane_util"):
            lu = f64["lane_util"]
            roofline["fp64_valu_lane_weighted"] = {"achieved_tflops": round(tf * lu, 3), "lane_util": round(lu, 4),
                                                   "frac": tf * lu / FP64_VALU_PEAK_TFLOPS}
    if "prepare" in phase_ms and hasattr(wl, "producer_roofline"):
        roofline["producer"] = wl.producer_roofline(phase_ms["prepare"])
    # MFMA utilisation (north_star asks for it): zero by design -- no v_mfma in any kernel's ISA
    # (scripts/isa_mfma_count.sh -> profiles/r04_isa_mfma.txt); DESIGN.md §3 "Why not MFMA"
    roofline["mfma"] = {
        "util": 0.0, "mfma_instructions_in_sqp_kernel": 0, "evidence": "profiles/r04_isa_mfma.txt",
        "why": ("no condensing: the stage-banded QP is factorised by a Riccati recursion over "
                f"{lay.nu + lay.nx}x{lay.nu + lay.nx} fp64 stage blocks, so there is no dense KKT GEMM; the blocks are far "
                "below a 16x16x4 f64 MFMA tile, the recursion is a chain of dependent 2x2 pivots, and gfx950's "
                "fp64 MFMA peak equals its fp64 vector peak, so MFMA could not raise this roofline")}
    ok = exit_h == 1
    stats = {"success_frac": float(ok.mean()), "rti_iters_per_solve": float(info_h[:, 0].mean()),
             "qp_iters_per_solve": float(info_h[:, 1].mean()), "qp_warm_start": args.qp_warm_start,
             "qp_warm_first": args.qp_warm_first, "solver_type": args.solver_type, "qp_profile": args.qp_profile,
             "scene_gen_s": round(wl.gen_s, 2)}
    if isinstance(wl, ShmpcWorkload):
        stats["scene_feasible_frac"] = float((wl.best.cpu().numpy() >= 0).mean())
    if isinstance(wl, TmpcWorkload):
        stats["scene_feasible_frac"] = float(ok.reshape(-1, wl.G).any(1).mean())
    result = {
        "metric": METRIC, "value": round(value, 2), "unit": "solves/s",
        # distinct devices used (a gloo rehearsal shares them between ranks)
        "n_gpus": world if backend == "nccl" else min(world, n_dev),
        "ranks_seen": ranks_seen,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f64",
        "data": f"synthetic (seeded scenes, SURVEY.md §8d {args.config})",
        "config": dict({"workload": wl.workload}, **wl.config,
                       parallelism=f"scene-sharded x{world}" + ((" + RCCL all-gather of winners" if backend == "nccl" else
                                                                   " + gloo all-gather of winners (rehearsal: "
                                                                   f"{world} ranks on {torch.cuda.device_count()} "
                                                                   "GPU(s), not a scaling figure)")
                                                                  if world > 1 else "")),
        "roofline": roofline,
        "solver_stats": stats,
        "phases_ms": {p: round(v, 4) for p, v in phase_ms.items()},
    }
    if alt is not None:
        alt["value_ratio_to_headline"] = round(alt["value"] / value, 4)
        result["qp_profile_alt"] = alt
    if backend == "gloo" and world > 1:
        # several ranks on one device: the rate is not a scaling figure
        result["rehearsal"] = {"backend": "gloo", "ranks": world, "devices": min(world, n_dev),
                               "rate_is_scaling_figure": False}

    if not args.no_cpu:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle_py

        oracle_py.build()
        orc = oracle_py.Oracle(lay, qp_warm_start=args.qp_warm_start, qp_warm_first=args.qp_warm_first,
                                             solver_type=args.solver_type, qp_profile=args.qp_profile)
        threads = wl.threads
        if world == 1:
            # CPU baseline: chunks of the same batch until ~cpu_seconds of CPU work, checked on the way
            done, t_cpu, dx_ok, dx_fail, agree, compared = 0, 0.0, 0.0, 0.0, 0, 0
            rare = np.zeros(3)
            while done < B and t_cpu < args.cpu_seconds:
                hi = min(B, done + CHECK_CHUNK)
                sec, a, f, g, n, rr = oracle_check(wl, orc, done, hi, exit_h, xt_h, info_h, threads)
                t_cpu += sec
                dx_ok, dx_fail, agree, compared = max(dx_ok, a), max(dx_fail, f), agree + g, compared + n
                rare += rr
                done = hi
            executed_flops(rare, f"the oracle's on the first {done} solves of this batch")

            def rate(n, nthreads):
                prm, wrm, xin = wl.host_inputs(0, min(n, B))
                tc = time.perf_counter()
                orc.solve_batch(prm, wrm, xin, nthreads=nthreads)
                return len(prm) / (time.perf_counter() - tc)

            share = cpu_share()
            result["cpu_baseline"] = {"value": round(done / t_cpu, 2), "unit": "solves/s", "cores": threads,
                                      "kind": "port",
                                      "sample": f"first {done} of the {B} solves of this batch, C oracle (same "
                                                f"algorithm), OpenMP {threads} threads = the job's CPU share",
                                      "single_thread_solves_per_s": round(rate(64, 1), 2),
                                      "eight_thread_solves_per_s": round(rate(512, 8), 2) if threads >= 8 else None,
                                      "host": share,
                                      "nproc_leg": ("same as value (share == nproc)" if share["share"] == share["nproc"]
                                                    else f"value is the {share['share']}-thread share of this job; "
                                                         f"nproc = {share['nproc']} counts the whole host")}
            result["vs_cpu_baseline"] = round(value / (done / t_cpu), 2)
            ranks_checked = 1
        else:
            # every rank checks a sample of its own shard; reduced over ranks
            n = min(RANK_SAMPLE, B)
            _, dx_ok, dx_fail, agree, compared, rare = oracle_check(wl, orc, 0, n, exit_h, xt_h, info_h, threads)
            executed_flops(rare, f"the oracle's on this rank's first {n} solves")
            t = torch.tensor([dx_ok, dx_fail, agree, compared, 1.0], dtype=torch.float64, device=dev)
            tm = t.clone()
            all_reduce_(tm, dist.ReduceOp.MAX)
            all_reduce_(t, dist.ReduceOp.SUM)
            dx_ok, dx_fail, agree, compared, ranks_checked = float(tm[0]), float(tm[1]), int(t[2]), int(t[3]), int(t[4])
        result["parity"] = {"max_abs_dx": dx_ok, "max_abs_dx_failed_same_path": dx_fail,
                            "exit_agreement": agree / max(1, compared), "solves_compared": compared,
                            "ranks_checked": ranks_checked, "tolerance": 1e-4}
        if isinstance(wl, ShmpcWorkload):
            result["parity"]["producer_max_abs_diff"] = wl.producer_check()
    if rank == 0:
        print(json.dumps(result))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
