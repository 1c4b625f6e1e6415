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
