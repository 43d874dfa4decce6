"""World-size-2 gloo rehearsal of the multi-GPU path (CPU): contiguous scene
shards, per-rank solve + selection, one all-gather of winner records; the
gathered records equal the single-process result.  The per-rank solve uses
the CPU oracle here (the HIP path needs a GPU); sharding, record layout and
the collective are the product code in distributed.py."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _solve_records(first, count, G):
    import sys
    ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle_py
    from oscar_mpc_planner_mr_modification_amd.distributed import winner_records
    from oscar_mpc_planner_mr_modification_amd.layouts import config_layout
    from oscar_mpc_planner_mr_modification_amd.selection import find_best_planner_host
    from oscar_mpc_planner_mr_modification_amd.synthetic import make_batch

    lay = config_layout("C1")
    if count == 0:
        from oscar_mpc_planner_mr_modification_amd.distributed import winner_width
        return torch.empty((0, winner_width(lay.N)), dtype=torch.float64)
    b = make_batch(lay, count, G, seed=77, first_scene=first)
    r = oracle_py.Oracle(lay, sqp_iters=3).solve_batch(b.params, b.warm, b.xinit, nthreads=1)
    best, _ = find_best_planner_host(count, G, lay.N, r["xtraj"], r["pobj"], r["status"], b.prev_traj, 0.05,
                                     np.ones(count * G, bool))
    return winner_records(torch.from_numpy(r["xtraj"]), torch.from_numpy(r["utraj"]), torch.from_numpy(r["pobj"]),
                          torch.from_numpy(best), G)


def _worker(rank, world, port, total, G, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oscar_mpc_planner_mr_modification_amd.distributed import gather_winners, shard
    first, count = shard(total, world, rank)
    rec = _solve_records(first, count, G)
    allrec = gather_winners(rec, world, total=total)
    if rank == 0:
        q.put(allrec.numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,total", [(2, 4), (2, 5), (4, 7), (4, 2), (8, 11), (8, 5)])
def test_shard_and_gather_equals_single_process(world, total):
    """Equal shards (4 over 2), uneven shards (5 over 2, 7 over 4, 11 over 8) and ranks
    without scenes (2 over 4, 5 over 8): the gathered records equal one process's."""
    G = 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, total, G, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    ref = _solve_records(0, total, G).numpy()
    np.testing.assert_array_equal(got, ref)


def test_shard_covers_every_scene_once():
    from oscar_mpc_planner_mr_modification_amd.distributed import shard
    for total in (1, 7, 1024, 16384):
        for world in (1, 2, 4, 8):
            seen = []
            for r in range(world):
                f, c = shard(total, world, r)
                seen.extend(range(f, f + c))
            assert seen == list(range(total))
