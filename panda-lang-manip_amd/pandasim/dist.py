"""Multi-GPU partition of the env batch.

Envs are independent, so the path shards with no exchange per step: rank r of
W owns the contiguous global env ids [r*B/W, (r+1)*B/W) and seeds env g with
``seed0 + g``, which makes a W-rank run identical, env for env, to a 1-rank
run of the same global batch.  The only collective is an optional gather of
per-env episode statistics (returns, successes) to rank 0, once per reporting
interval: ``dist.gather`` to rank 0 -- RCCL over xGMI on GPUs (backend
"nccl"), gloo in the CPU tests.  One process per GPU.
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch
import torch.distributed as dist


def shard_range(global_batch: int, world_size: int, rank: int) -> Tuple[int, int]:
    """(first global env id, env count) owned by `rank`; remainders go to the
    lowest ranks so every env is owned exactly once."""
    if global_batch < world_size:
        raise ValueError(f"global batch {global_batch} < world size {world_size}")
    if not 0 <= rank < world_size:
        raise ValueError(f"rank {rank} outside [0, {world_size})")
    base, rem = divmod(global_batch, world_size)
    count = base + (1 if rank < rem else 0)
    start = rank * base + min(rank, rem)
    return start, count


def shard_seeds(seed0: int, global_batch: int, world_size: int, rank: int) -> torch.Tensor:
    """uint64 reset seeds (as int64 bits) of this rank's envs: seed0 + global id."""
    start, count = shard_range(global_batch, world_size, rank)
    return torch.arange(count, dtype=torch.int64) + (seed0 + start)


class EpisodeStats:
    """Per-env running return and last finished episode's return/success,
    updated on device from a step's (reward, terminated, truncated)."""

    def __init__(self, num_envs: int, device):
        self.running = torch.zeros(num_envs, dtype=torch.float32, device=device)
        self.last_return = torch.zeros(num_envs, dtype=torch.float32, device=device)
        self.last_success = torch.zeros(num_envs, dtype=torch.float32, device=device)
        self.episodes = torch.zeros(num_envs, dtype=torch.int32, device=device)

    def update(self, reward: torch.Tensor, terminated: torch.Tensor, truncated: torch.Tensor) -> None:
        self.running.add_(reward)
        done = (terminated != 0) | (truncated != 0)
        self.last_return = torch.where(done, self.running, self.last_return)
        self.last_success = torch.where(done, (terminated != 0).to(torch.float32), self.last_success)
        self.episodes.add_(done.to(torch.int32))
        self.running.masked_fill_(done, 0.0)

    def reset(self, mask: Optional[torch.Tensor] = None) -> None:
        """env.reset() (of every env, or of `mask`): the running return
        restarts at 0, as gymnasium's RecordEpisodeStatistics does; the last
        finished episode's figures stay."""
        if mask is None:
            self.running.zero_()
        else:
            self.running.masked_fill_(mask.to(self.running.device).bool(), 0.0)

    def packed(self) -> torch.Tensor:
        """[3, B] float32: last return, last success, episode count."""
        return torch.stack([self.last_return, self.last_success, self.episodes.to(torch.float32)])


def gather_to_rank0(local: torch.Tensor, group=None) -> Optional[torch.Tensor]:
    """Concatenate every rank's [..., B_r] tensor along the last dim (rank
    order = global env order) on rank 0 only (``dist.gather``: RCCL
    point-to-point into rank 0 on GPUs, gloo on the CPU).  Shards may differ
    in size (shard_range gives the lowest ranks one more env when the global
    batch does not divide): every rank pads to the largest shard and rank 0
    trims.  Returns the full tensor on rank 0, None elsewhere; on a single
    process it returns `local`."""
    if not dist.is_available() or not dist.is_initialized():
        return local
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    local = local.contiguous()
    n = local.shape[-1]
    sizes = torch.tensor([n], dtype=torch.int64, device=local.device)
    all_sizes = [torch.zeros_like(sizes) for _ in range(world)]
    dist.all_gather(all_sizes, sizes, group=group)
    counts = [int(t.item()) for t in all_sizes]
    n_max = max(counts)
    if n < n_max:
        local = torch.cat([local, local.new_zeros(local.shape[:-1] + (n_max - n,))], dim=-1)
    dst = dist.get_global_rank(group, 0) if group is not None else 0
    parts = [torch.empty_like(local) for _ in range(world)] if rank == 0 else None
    dist.gather(local, parts, dst=dst, group=group)
    if rank != 0:
        return None
    return torch.cat([p[..., :c] for p, c in zip(parts, counts)], dim=-1)


def max_over_ranks(value: float, device, group=None) -> float:
    """Max of a host scalar over ranks (bench timing)."""
    if not dist.is_available() or not dist.is_initialized():
        return value
    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return float(t.item())
