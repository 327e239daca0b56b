"""Frame-sharded data parallelism across the GPUs of a node (BASELINE config 5).

Frames are independent (models.py:42-69 and bev.py:166-246 keep no cross-frame state), so rank r of
N takes frames [r*B/N, (r+1)*B/N), runs the whole path locally with replicated weights, and the only
collective is ONE all-gather of the int8 occupancy grids (2.56 MB per rank at B=512, N=8: ~17 us per
xGMI link) — RCCL (`nccl` backend) on the GPUs, gloo in the CPU tests.
"""
from __future__ import annotations

from typing import Callable

import torch
import torch.distributed as dist


def shard_bounds(total: int, world: int, rank: int) -> tuple[int, int]:
    """Contiguous, balanced shard of `total` frames for `rank` (sizes differ by at most one)."""
    if world <= 0 or not (0 <= rank < world):
        raise ValueError("bad world/rank")
    base, rem = divmod(total, world)
    start = rank * base + min(rank, rem)
    return start, start + base + (1 if rank < rem else 0)


def gather_grids(local: torch.Tensor, total: int, group=None) -> torch.Tensor:
    """All-gather per-rank (b_r, h, w) int8 grids into (total, h, w) in rank order."""
    world = dist.get_world_size(group)
    sizes = [shard_bounds(total, world, r) for r in range(world)]
    counts = [e - s for s, e in sizes]
    if local.shape[0] != counts[dist.get_rank(group)]:
        raise ValueError("local shard size does not match shard_bounds")
    m = max(counts)
    pad = local
    if local.shape[0] != m:
        pad = torch.zeros((m,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
        pad[: local.shape[0]] = local
    if dist.get_backend(group) == "nccl":
        buf = torch.empty((world * m,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
        dist.all_gather_into_tensor(buf, pad.contiguous(), group=group)
        if all(c == m for c in counts):
            return buf                        # equal shards: rank order already, no copy
        parts = list(buf.split(m))
    else:
        # gloo (CPU tests, and the single-GPU functional run of bench.py's N > 1 branch): host copies
        host = pad.cpu().contiguous()
        parts = [torch.empty_like(host) for _ in range(world)]
        dist.all_gather(parts, host, group=group)
        return torch.cat([p[:c] for p, c in zip(parts, counts)], 0).to(local.device)
    return torch.cat([p[:c] for p, c in zip(parts, counts)], 0)


def run_sharded(frames: torch.Tensor, step: Callable[[torch.Tensor], torch.Tensor], group=None) -> torch.Tensor:
    """frames: the FULL batch (every rank holds it, or a view of it); each rank runs `step` on its
    shard and the grids are all-gathered. Returns (B, h, w) on every rank."""
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    s, e = shard_bounds(frames.shape[0], world, rank)
    local = step(frames[s:e])
    return gather_grids(local, frames.shape[0], group)
