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


def test_source_hash_tracks_kernel_sources():
    sys.path.insert(0, ROOT)
    from oscar_mpc_planner_mr_modification_amd import _build
    h = _build.source_hash()
    assert len(h) == 64 and h == _build.source_hash()
