"""Multi-GPU sharding of independent envs (one process per GPU, no collective on the step path).

Envs are independent, so rank r of W simply owns global env ids
[r*E, (r+1)*E): its handle is created with env_id_offset = r*E, and every
random draw (auto-reset goals, benchmark actions) is keyed by the global env
id, so a sharded run reproduces the single-GPU run env for env.  The only
collectives are outside the step loop: the max-over-ranks timing reduction
and an optional all-gather of a 4-float episode-statistics vector per rank.
"""
from __future__ import annotations

from typing import Optional, Sequence

import torch


def shard_offset(rank: int, envs_per_rank: int) -> int:
    return rank * envs_per_rank


def max_over_ranks(value: float, dist=None, device: Optional[torch.device] = None) -> float:
    """Wall time of a barrier-bracketed region = max over ranks."""
    t = torch.tensor([value], dtype=torch.float64, device=device)
    if dist is not None and dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def gather_stats(stats: Sequence[float], dist=None, device: Optional[torch.device] = None) -> torch.Tensor:
    """All-gather [episodes, successes, return_sum, length_sum] from every rank -> [W, 4]."""
    t = torch.tensor(list(stats), dtype=torch.float64, device=device)
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return t[None, :]
    out = [torch.empty_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(out, t)
    return torch.stack(out)
