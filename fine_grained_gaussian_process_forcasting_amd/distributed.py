"""Batch sharding of independent GP windows over ranks + the one exchange step
the path has: an all-reduce (SUM) of the per-rank MLL / ELL partial sums.

One process per GPU (torchrun), ``torch.distributed`` with backend "nccl"
(= RCCL on ROCm, over xGMI). Windows are independent, so the data
path needs no collective; only the scalar objective is reduced, as one fp64
value (8 bytes) per step. Works unchanged with the gloo backend on CPU tensors
(tests/test_distributed.py).
"""
from __future__ import annotations

import os
from typing import Optional, Tuple

import torch
import torch.distributed as dist


def env_rank_world() -> Tuple[int, int, int]:
    """(rank, local_rank, world_size) from the torchrun environment (1 process = 0,0,1)."""
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    return rank, local, world


def shard_range(total: int, rank: int, world: int) -> Tuple[int, int]:
    """Contiguous slice [lo, hi) of ``total`` windows for ``rank`` (sizes differ by <= 1)."""
    if world <= 0 or not (0 <= rank < world):
        raise ValueError(f"bad rank/world {rank}/{world}")
    base, rem = divmod(total, world)
    lo = rank * base + min(rank, rem)
    hi = lo + base + (1 if rank < rem else 0)
    return lo, hi


def allreduce_sum_f64(partial: torch.Tensor, group=None, async_op: bool = False):
    """SUM-all-reduce a partial objective as one fp64 scalar; returns (tensor, work)."""
    t = partial.detach().to(torch.float64).reshape(1)
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size(group) == 1:
        return t, None
    work = dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group, async_op=async_op)
    return t, work


def global_mean_objective(per_window: torch.Tensor, total_windows: int, group=None) -> torch.Tensor:
    """Mean over ALL windows of all ranks of a per-window objective (MLL or ELBO term)."""
    t, work = allreduce_sum_f64(per_window.sum(dtype=torch.float64), group=group)
    if work is not None:
        work.wait()
    return t / float(total_windows)
