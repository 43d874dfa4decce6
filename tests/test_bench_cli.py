"""bench.py's launch contract, checked without a GPU: `bench.py --gpus N` starts its own
N ranks (a child torch.distributed.run) when no launcher is present, --gpus must match a
launcher's world size, and both are decided before any GPU call."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_gpus_flag_spawns_its_own_ranks():
    """plain `bench.py --gpus 2` (no launcher) runs two ranks that rendezvous on 127.0.0.1;
    rank 0 alone prints, and it saw both ranks (--spawn-check: the rank plumbing on gloo)"""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                             "MASTER_PORT")}
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--spawn-check"], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    line = json.loads(lines[0])
    assert line["ranks_seen"] == 2 and line["n_gpus"] == 2
    assert line["gather_ok"], line


def test_gpus_8_spawns_eight_ranks_and_gathers_the_c4_shards():
    """the width the driver's scaling run uses: `bench.py --gpus 8` (no launcher) starts eight ranks,
    and the step's winner all-gather is exact over BASELINE config 4's 16,384 scenes (2,048 per rank,
    N 30 records) and over an uneven 16,387-scene sharding"""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                             "MASTER_PORT")}
    env["OMP_NUM_THREADS"] = "1"
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "8", "--config", "C4", "--spawn-check"], cwd=ROOT,
                       env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    line = json.loads(lines[0])
    assert line["ranks_seen"] == 8 and line["n_gpus"] == 8
    assert line["scenes_per_rank"] == 2048 and line["gather_even_scenes"] == 16384
    assert line["gather_uneven_scenes"] == 16387 and line["gather_ok"], line


def test_gpus_flag_must_match_launcher_world_size():
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "LOCAL_RANK")}
    env["WORLD_SIZE"] = "1"
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2"], cwd=ROOT, env=env, capture_output=True,
                       text=True, timeout=120)
    assert r.returncode != 0
    assert "WORLD_SIZE=1" in r.stderr and "torch.distributed.run" in r.stderr


def test_cpu_share_is_bounded_by_the_host():
    sys.path.insert(0, ROOT)
    import bench
    s = bench.cpu_share()
    assert 1 <= s["share"] <= s["affinity"] <= s["nproc"]


def test_unknown_collective_backend_is_refused():
    """MPCG_BENCH_BACKEND selects RCCL (default) or the gloo rehearsal; anything else stops
    before any GPU call."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["MPCG_BENCH_BACKEND"] = "mpi"
    r = subprocess.run([sys.executable, "bench.py"], cwd=ROOT, env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode != 0
    assert "MPCG_BENCH_BACKEND=mpi" in r.stderr


def test_source_hash_tracks_kernel_sources():
    sys.path.insert(0, ROOT)
    from oscar_mpc_planner_mr_modification_amd import _build
    h = _build.source_hash()
    assert len(h) == 64 and h == _build.source_hash()


def test_flop_model_uses_executed_iterations():
    """roofline.achieved counts the algorithm's fp64 operations (flopmodel.py) times the SQP and
    IPM iterations each solve executed: linear in both counts, more rows -> more operations."""
    import numpy as np
    sys.path.insert(0, ROOT)
    from oscar_mpc_planner_mr_modification_amd import flopmodel
    from oscar_mpc_planner_mr_modification_amd.layouts import config_layout
    c1, c2, c4 = (config_layout(c) for c in ("C1", "C2", "C4"))
    lin, ipm = flopmodel.linearisation_ops(c2), flopmodel.ipm_iteration_ops(c2)
    info = np.array([[10, 40, 0, 0], [1, 7, 1, 0], [0, 0, 0, 0]])
    np.testing.assert_array_equal(flopmodel.solve_ops(c2, info), [10 * lin + 40 * ipm, lin + 7 * ipm, 0])
    assert flopmodel.ipm_iteration_ops(c1) < ipm < flopmodel.ipm_iteration_ops(c4)
    # C2 (N 20, nu 2, nx 5): 5-12 MFLOP per solve at 10 SQP and ~40 IPM iterations
    assert 5e6 < 10 * lin + 40 * ipm < 12e6
