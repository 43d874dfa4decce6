"""Scene sharding over GPUs and the gather of winning trajectories
(SURVEY.md §8e).

Scenes are independent and the G guesses of a scene only meet in the
per-scene argmin, so scenes are split into contiguous blocks, one per rank,
with every guess of a scene on the same GPU; the only exchange is one
all-gather of the per-scene winner records after the batched solve (RCCL over
xGMI on MI355X; gloo in the CPU tests).
"""
from __future__ import annotations


def shard(total_scenes: int, world: int, rank: int) -> tuple[int, int]:
    """Contiguous block of ceil(total/world) scenes for `rank`: (first, count)."""
    per = -(-total_scenes // world)
    first = min(total_scenes, rank * per)
    return first, max(0, min(total_scenes, first + per) - first)


def winner_width(N: int, nx: int = 5, nu: int = 2) -> int:
    """xtraj (N+1)*nx | utraj N*nu | pobj | planner index"""
    return (N + 1) * nx + N * nu + 2


def winner_records(xtraj, utraj, pobj, best, G, out=None):
    """Per-scene record of the selected planner (torch tensors, any device).
    best == -1 (every planner failed) records planner 0, whose exit code the
    reference returns in that case (guidance_constraints.cpp:429-442), with
    index -1 kept in the last column."""
    import torch

    S = best.shape[0]
    B, N1, nx = xtraj.shape
    N = N1 - 1
    nu = utraj.shape[2]
    w = winner_width(N, nx, nu)
    if out is None:
        out = torch.empty((S, w), dtype=xtraj.dtype, device=xtraj.device)
    flat = torch.arange(S, device=best.device) * G + best.long().clamp(min=0)
    out[:, :N1 * nx] = xtraj[flat].reshape(S, -1)
    out[:, N1 * nx:N1 * nx + N * nu] = utraj[flat].reshape(S, -1)
    out[:, -2] = pobj[flat]
    out[:, -1] = best.to(xtraj.dtype)
    return out


def gather_winners(records, world: int, out=None, group=None, total: int | None = None):
    """All-gather of the per-rank record blocks (one collective).

    `total` is the number of scenes over all ranks, sharded by `shard()`. The
    blocks may then differ in size (total % world != 0, or ranks without
    scenes): every rank pads its block to ceil(total / world) rows, one
    equal-size all-gather moves the padded blocks, and the real rows are
    compacted in rank order.  Without `total` the blocks must all have
    records.shape[0] rows (the bench's weak-scaling shards); `out` is then
    the (world * rows, width) result buffer."""
    import torch
    import torch.distributed as dist

    if world == 1:
        return records
    width = records.shape[1]
    if total is None:
        per, counts = records.shape[0], None
    else:
        per = -(-total // world)
        counts = [shard(total, world, r)[1] for r in range(world)]
        rank = dist.get_rank(group)
        if records.shape[0] != counts[rank]:
            raise ValueError(f"rank {rank} holds {records.shape[0]} records, its shard has {counts[rank]}")
    if counts is None:
        send = records.contiguous()
        buf = out if out is not None else torch.empty((per * world, width), dtype=records.dtype,
                                                      device=records.device)
    else:
        send = torch.zeros((per, width), dtype=records.dtype, device=records.device)
        send[:records.shape[0]] = records
        buf = torch.empty((per * world, width), dtype=records.dtype, device=records.device)
    if dist.get_backend(group) == "gloo":
        # gloo all-gathers host tensors: device blocks are staged through the host (the
        # rehearsal of the multi-rank path on one GPU, bench.py MPCG_BENCH_BACKEND=gloo)
        send_h = send.cpu()
        parts = [torch.empty_like(send_h) for _ in range(world)]
        dist.all_gather(parts, send_h, group=group)
        buf.copy_(torch.cat(parts, 0))
    else:
        dist.all_gather_into_tensor(buf, send, group=group)
    if counts is None:
        return buf
    blocks = [buf[r * per:r * per + counts[r]] for r in range(world)]
    res = torch.cat(blocks, 0)
    if out is not None:
        out.copy_(res)
        return out
    return res


def all_reduce_(t, op, group=None):
    """In-place all-reduce of `t` (any device); under gloo the tensor is staged through
    the host, as gloo reduces host tensors."""
    import torch.distributed as dist

    if dist.get_backend(group) == "gloo" and t.device.type != "cpu":
        h = t.cpu()
        dist.all_reduce(h, op=op, group=group)
        t.copy_(h)
    else:
        dist.all_reduce(t, op=op, group=group)
    return t
