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


def allreduce_shared_grads(params, group=None, scale: float = 1.0) -> Optional[torch.Tensor]:
    """Sum the gradients of the SHARED GP parameters over ranks with ONE collective
    (SURVEY.md §8e): every rank back-propagated its own shard of windows, so the shared
    hyper-parameters / inducing points / q(u) hold partial gradients. They are packed
    into one flat fp32 buffer (variational: M*D + 2M + D + 4 floats, ~9 KB at M=64,
    D=32 -- latency-bound, one xGMI hop), SUM-all-reduced, scaled and written back.
    Parameters without a gradient contribute zeros. Returns the flat buffer."""
    params = [p for p in params if p is not None]
    if not params:
        return None
    dev = params[0].device
    flat = torch.cat([(p.grad if p.grad is not None else torch.zeros_like(p)).reshape(-1).float().to(dev)
                      for p in params])
    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=group)
    if scale != 1.0:
        flat.mul_(scale)
    o = 0
    for p in params:
        n = p.numel()
        g = flat[o:o + n].view_as(p).to(p.dtype)
        if p.grad is None:
            p.grad = g.clone()
        else:
            p.grad.copy_(g)
        o += n
    return flat


class ObjectiveAccumulator:
    """Per-step objective values kept on the device and reduced across ranks with ONE
    all-reduce for many steps (the per-step value is only logged): no collective and no
    extra launch sits on the critical path of a step, which matters at 64 windows per
    GPU. ``slot()`` hands the kernel a (B,) row to write its per-window
    objective into; ``add()`` stores an already-reduced scalar instead."""

    def __init__(self, steps: int, device, group=None, width: int = 1):
        self.rows = torch.zeros(max(1, steps), width, dtype=torch.float32, device=device)
        self.n = 0
        self.group = group

    def slot(self) -> torch.Tensor:
        r = self.rows[self.n]
        self.n += 1
        return r

    def add(self, partial: torch.Tensor) -> None:
        self.rows[self.n, :1].copy_(partial.detach().reshape(1).to(self.rows.dtype))
        self.n += 1

    def reduce(self, async_op: bool = False):
        """(per-step sums over the rows, fp64, summed over ranks; work handle or None)."""
        tot = self.rows[:self.n].sum(1, dtype=torch.float64)
        if dist.is_available() and dist.is_initialized() and dist.get_world_size(self.group) > 1:
            work = dist.all_reduce(tot, op=dist.ReduceOp.SUM, group=self.group, async_op=async_op)
            return tot, work
        return tot, None
