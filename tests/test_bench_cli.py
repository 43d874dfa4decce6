"""bench.py's launch contract, checked without a GPU: --gpus must match the
launcher's world size, and the mismatch is reported before any GPU call."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_gpus_flag_must_match_world_size():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2"], cwd=ROOT, env=env, capture_output=True,
                       text=True, timeout=120)
    assert r.returncode != 0
    assert "WORLD_SIZE=1" in r.stderr and "torch.distributed.run" in r.stderr


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
