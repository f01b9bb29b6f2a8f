"""Env-parallel sharding across GPUs (one process per GPU, torch.distributed over RCCL/xGMI).

The E envs are independent: rank r of P owns the contiguous block
[offset_r, offset_r + E_r) and steps it with no collective on the step path.  The device-reset
RNG is keyed by the GLOBAL env index (env_offset), so a sharded run draws the same episodes as a
single-GPU run of the whole batch.  The only exchange is the optional CTDE `global_state`
all-gather (all_gather_into_tensor; backend "nccl" is RCCL on ROCm).
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def shard_bounds(num_envs_global: int, world_size: int, rank: int) -> tuple[int, int]:
    """(env_offset, local_count) of `rank` for a contiguous balanced split."""
    if world_size < 1 or not (0 <= rank < world_size):
        raise ValueError(f"bad rank {rank} / world_size {world_size}")
    base, rem = divmod(int(num_envs_global), int(world_size))
    count = base + (1 if rank < rem else 0)
    offset = rank * base + min(rank, rem)
    return offset, count


def gather_global_state(local: torch.Tensor, group=None) -> torch.Tensor:
    """All-gather the per-env CTDE critic input [E_local, 6N+3] into [E_global, 6N+3].

    Requires equal local batch sizes (weak-scaling shards).  One collective per call — gather
    every K steps or at batch boundaries."""
    if not dist.is_available() or not dist.is_initialized():
        return local
    ws = dist.get_world_size(group)
    out = torch.empty((ws * local.shape[0],) + tuple(local.shape[1:]), dtype=local.dtype,
                      device=local.device)
    dist.all_gather_into_tensor(out, local.contiguous(), group=group)
    return out
