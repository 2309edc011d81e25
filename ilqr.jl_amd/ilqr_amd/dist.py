"""Multi-GPU plumbing: one process per GPU, torch.distributed (RCCL on ROCm).

Trajectories (independent MPC instances / seeds) shard trivially: rank r owns a
contiguous block of the global batch and runs the whole fit locally — there is
no exchange inside an iteration. The only collective is the result exchange
after a fit: an all-gather of per-trajectory costs and status words (a few KB
per rank, latency-bound over xGMI), done once.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def shard_range(n: int, rank: int, world: int):
    """Contiguous block [lo, hi) of n trajectories owned by `rank` (ragged-safe)."""
    base, rem = divmod(n, world)
    lo = rank * base + min(rank, rem)
    return lo, lo + base + (1 if rank < rem else 0)


def all_gather_ragged(t: torch.Tensor, group=None) -> torch.Tensor:
    """Concatenate a 1-D per-rank tensor across ranks in rank order (sizes may differ)."""
    world = dist.get_world_size(group)
    n = torch.tensor([t.numel()], dtype=torch.int64, device=t.device)
    sizes = [torch.empty_like(n) for _ in range(world)]
    dist.all_gather(sizes, n, group=group)
    sizes = [int(s.item()) for s in sizes]
    m = max(sizes)
    buf = torch.zeros(m, dtype=t.dtype, device=t.device)
    buf[: t.numel()] = t
    out = [torch.empty_like(buf) for _ in range(world)]
    dist.all_gather(out, buf, group=group)
    return torch.cat([o[:s] for o, s in zip(out, sizes)])


def gather_fit_results(cost: torch.Tensor, status: torch.Tensor, group=None):
    """All-gather a fit's per-trajectory cost (f64) and status (i32) → global arrays."""
    return all_gather_ragged(cost, group), all_gather_ragged(status, group)
