"""CPU baseline as P single-thread worker processes (bench.py cpu_baseline leg).

The multi-thread leg of bench.py times GPyTorch's own CPU arithmetic the way the reference
would run it (one process, MKL threads over a batched cholesky_ex), which barely
parallelises. This script measures what the host's cores can do instead: P processes, one
thread each, every one timing oracle.exact_mll_torch_cpu on its own batch of windows for the
same wall-clock interval, started together behind a barrier. It runs as a CPU-only child of
bench.py (started with subprocess, never touching the GPU), so the spawned workers do not
inherit any GPU state.

    python scripts/cpu_baseline_procs.py P SECONDS N D   ->   one JSON line
"""
import json
import math
import multiprocessing as mp
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LN2 = math.log(2.0)


def _worker(rank, seconds, N, D, barrier, q):
    os.environ["OMP_NUM_THREADS"] = "1"
    sys.path.insert(0, ROOT)
    import torch
    torch.set_num_threads(1)
    from oracle import gp_oracle as O
    Bs = 8
    g = torch.Generator().manual_seed(rank)
    X = torch.randn(Bs, N, D, generator=g) / math.sqrt(D)
    y = torch.randn(Bs, N, generator=g)
    O.exact_mll_torch_cpu(X, y, LN2, LN2, 0.0, LN2 + 1e-4)   # warm-up
    barrier.wait()
    n = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        O.exact_mll_torch_cpu(X, y, LN2, LN2, 0.0, LN2 + 1e-4)
        n += Bs
    q.put((n, time.perf_counter() - t0))


def main():
    P, seconds, N, D = int(sys.argv[1]), float(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
    ctx = mp.get_context("spawn")
    barrier, q = ctx.Barrier(P), ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, seconds, N, D, barrier, q)) for r in range(P)]
    for p in procs:
        p.start()
    res = [q.get(timeout=600) for _ in range(P)]
    for p in procs:
        p.join(timeout=60)
    windows = sum(n for n, _ in res)
    wall = max(dt for _, dt in res)
    print(json.dumps({"value": windows / wall, "processes": P, "windows": windows, "seconds": wall,
                      "per_process": [n / dt for n, dt in res]}))


if __name__ == "__main__":
    main()
