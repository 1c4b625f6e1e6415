"""CPU: the N>1 path (window sharding + fp64 SUM all-reduce of the objective) with
gloo, world_size 2, exactly as bench.py / the MLL helpers use it with RCCL."""
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


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from fine_grained_gaussian_process_forcasting_amd.distributed import (
        allreduce_sum_f64, env_rank_world, global_mean_objective, shard_range)
    r, lr, w = env_rank_world()
    total = 37
    lo, hi = shard_range(total, r, w)
    per_window = torch.arange(total, dtype=torch.float32)[lo:hi] * 0.5 - 3.0
    mean = global_mean_objective(per_window, total)
    t, work = allreduce_sum_f64(torch.tensor(float(hi - lo)), async_op=True)
    work.wait()
    q.put((rank, float(mean), float(t.item()), (lo, hi)))
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_world2_objective_allreduce():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = float((np.arange(37) * 0.5 - 3.0).mean())
    assert all(abs(m - want) < 1e-9 for _, m, _, _ in res)
    assert all(t == 37.0 for _, _, t, _ in res)
    assert res[0][3] == (0, 19) and res[1][3] == (19, 37)


def _grad_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from fine_grained_gaussian_process_forcasting_amd.distributed import (
        ObjectiveAccumulator, allreduce_shared_grads, shard_range)
    B, N, M, D = 10, 6, 4, 3
    g = torch.Generator().manual_seed(0)
    X = torch.randn(B, N, D, generator=g, dtype=torch.float64)
    Z = torch.randn(M, D, generator=g, dtype=torch.float64)

    def loss_of(Xs, Zp, lsp, mp):
        # a smooth stand-in with the same sharing pattern as the GP: per-window terms of
        # shared (Z, lengthscale, q(u) mean) parameters, summed over windows
        K = torch.exp(-0.5 * ((Xs.unsqueeze(-2) - Zp) / lsp).pow(2).sum(-1))   # (b, N, M)
        return (K @ mp).pow(2).sum()

    def params():
        return (Z.clone().requires_grad_(True), torch.full((D,), 0.8, dtype=torch.float64, requires_grad=True),
                torch.linspace(-1, 1, M, dtype=torch.float64).requires_grad_(True))
    lo, hi = shard_range(B, rank, world)
    Zp, lsp, mp = params()
    loss_of(X[lo:hi], Zp, lsp, mp).backward()
    unused = torch.zeros(2, dtype=torch.float64, requires_grad=True)   # no grad on any rank
    allreduce_shared_grads([Zp, lsp, mp, unused])
    Zf, lf, mf = params()
    loss_of(X, Zf, lf, mf).backward()
    ok = all(torch.allclose(a.grad, b.grad, rtol=1e-5, atol=1e-6) for a, b in ((Zp, Zf), (lsp, lf), (mp, mf)))
    ok = ok and torch.equal(unused.grad, torch.zeros(2, dtype=torch.float64))
    acc = ObjectiveAccumulator(3, "cpu")
    for k in range(3):
        acc.add(torch.tensor(float(rank + k)))
    rows = ObjectiveAccumulator(2, "cpu", width=3)
    for k in range(2):
        rows.slot().copy_(torch.tensor([1.0, 2.0, float(rank + k)]))
    rv, rw = rows.reduce()
    ok = ok and rv.tolist() == [6.0 + 1.0, 6.0 + 3.0]
    vals, work = acc.reduce(async_op=True)
    work.wait()
    q.put((rank, ok, vals.tolist()))
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_world2_shared_grad_allreduce_matches_single_rank():
    """Training over 2 ranks: each rank back-propagates its window shard, ONE flat
    all-reduce of the shared-parameter gradients reproduces the
    single-rank full-batch gradient; the per-step objectives are reduced once."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_grad_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(ok for _, ok, _ in res)
    assert all(v == [1.0, 3.0, 5.0] for _, _, v in res)
