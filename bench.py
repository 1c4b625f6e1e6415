"""Benchmark of the MI355X GP hot path (BASELINE.json metric: GP windows/sec).

Workload (BASELINE.json configs[3], the north-star shape, which fits one GPU):
synthetic exact-GP windows B=512 per GPU, N=256, D=32 — per step the fused kernel
builds the RBF Gram, runs the jittered Cholesky, the forward solve and the MLL for
every window, writes L (B,N,N) and the MLL, then the ranks SUM-all-reduce the MLL
partial (one fp64, RCCL over xGMI; overlapped with the next step's kernel).
Scaling is weak: every rank owns 512 windows; value = total windows / time.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

Rank 0 prints ONE JSON line (contract in the task statement / DESIGN.md §6).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from fine_grained_gaussian_process_forcasting_amd import ops  # noqa: E402
from fine_grained_gaussian_process_forcasting_amd.distributed import (  # noqa: E402
    allreduce_sum_f64, env_rank_world)

HBM_PEAK = 8.0e12          # B/s, MI355X_MICROARCH.md chip table (spec)
FP32_PEAK = 157.3e12       # FLOP/s, vector == f32 MFMA
LN2 = math.log(2.0)


def bytes_per_window(N, D):   # X read + y read + L write + MLL write
    return 4 * (N * D + N + N * N + 1)


def flops_per_window(N, D):
    return 3 * D * N * (N + 1) // 2 + N ** 3 // 3 + N * N + 3 * N


def make_inputs(B, N, D, device, seed):
    g = torch.Generator().manual_seed(seed)
    X = (torch.randn(B, N, D, generator=g) / math.sqrt(D)).to(device)
    y = torch.randn(B, N, generator=torch.Generator().manual_seed(seed + 1)).to(device)
    return X, y


def cpu_baseline(N, D, seconds=12.0):
    """GPyTorch's own CPU arithmetic for this path (oracle.exact_mll_torch_cpu: the
    _sq_dist GEMM, torch.linalg.cholesky_ex + jitter ladder, cholesky_solve, logdet;
    MKL/LAPACK) timed on the host cores, fp32 like the reference."""
    from oracle import gp_oracle as O
    threads = torch.get_num_threads()
    Bs = 64
    g = torch.Generator().manual_seed(0)
    X = torch.randn(Bs, N, D, generator=g) / math.sqrt(D)
    y = torch.randn(Bs, N, generator=g)
    O.exact_mll_torch_cpu(X, y, LN2, LN2, 0.0, LN2 + 1e-4)  # warm-up
    n = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        O.exact_mll_torch_cpu(X, y, LN2, LN2, 0.0, LN2 + 1e-4)
        n += Bs
    dt = time.perf_counter() - t0
    return {"value": n / dt, "unit": "windows/s", "cores": int(threads), "kind": "port",
            "sample": f"{n} windows (batches of {Bs}, N={N}, D={D}) through "
                      f"oracle.exact_mll_torch_cpu (GPyTorch's torch-CPU arithmetic, fp32) over "
                      f"{dt:.1f}s; torch threads={threads}, os.cpu_count()={os.cpu_count()}"}


def load_traffic(N, D, B):
    """HBM bytes per launch from the committed rocprofv3 PMC summary (profiles/), if any."""
    p = os.path.join(ROOT, "profiles", "pmc_exact_summary.json")
    try:
        with open(p) as f:
            d = json.load(f)
        key = f"B{B}_N{N}_D{D}"
        return d.get(key, {}).get("hbm_bytes_per_launch")
    except OSError:
        return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--B", type=int, default=512, help="windows per GPU")
    ap.add_argument("--N", type=int, default=256)
    ap.add_argument("--D", type=int, default=32)
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-grad", action="store_true", help="skip the backward side measurement")
    args = ap.parse_args()

    rank, local, world = env_rank_world()
    if world != args.gpus:
        if world == 1 and args.gpus > 1:
            raise SystemExit("--gpus > 1 must be launched with torch.distributed.run")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    B, N, D = args.B, args.N, args.D
    X, y = make_inputs(B, N, D, dev, seed=1000 * rank)
    hyper = ops.pack_exact_hyper(LN2, LN2 + 1e-4, 0.0, LN2, dev)   # GPyTorch init values

    def step():
        out = ops.exact_mll(X, y, None, None, None, None, hyper=hyper)
        return out

    pending = []
    for _ in range(args.warmup):
        out = step()
        _, w = allreduce_sum_f64(out.mll.sum(dtype=torch.float64), async_op=True)
        if w is not None:
            pending.append(w)
    for w in pending:
        w.wait()
    pending.clear()
    torch.cuda.synchronize()
    # numerical status of the warm-up output (one sync, outside the timed region)
    ops.check_cholesky_info(out.info, 1e-6, inputs=(X,))

    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(args.steps)]
    totals = []
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.steps):
        ev[k][0].record()
        out = step()
        ev[k][1].record()
        tot, w = allreduce_sum_f64(out.mll.sum(dtype=torch.float64), async_op=True)
        totals.append(tot)
        if w is not None:
            pending.append(w)
    for w in pending:
        w.wait()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    kern_ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
    if world > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        km = torch.tensor([kern_ms], device=dev, dtype=torch.float64)
        dist.all_reduce(km, op=dist.ReduceOp.MAX)
        kern_ms = float(km.item())
    mean_mll = float(totals[-1].item()) / (B * world)

    # Secondary (not the headline): the analytic backward of the same windows
    # (gpk_exact_mll_grad_f32), outside the timed region above.
    grad_ms = None
    if not args.no_grad:
        fw = ops.exact_mll(X, y, None, None, None, None, hyper=hyper, want_L=True, want_z=True)
        gout = torch.ones(B, device=dev)
        ops.exact_mll_grad(X, fw.L, fw.z, hyper, gout)
        torch.cuda.synchronize()
        gev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
               for _ in range(5)]
        for a, b in gev:
            a.record()
            ops.exact_mll_grad(X, fw.L, fw.z, hyper, gout)
            b.record()
        torch.cuda.synchronize()
        grad_ms = float(np.mean([a.elapsed_time(b) for a, b in gev]))

    if rank == 0:
        value = B * world * args.steps / elapsed
        bpw, fpw = bytes_per_window(N, D), flops_per_window(N, D)
        achieved = bpw * B / (kern_ms * 1e-3)
        line = {
            "metric": "GP windows/sec (BxN RBF+Cholesky+ELBO)",
            "value": value,
            "unit": "windows/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic",
            "config": {"workload": "exact-GP windows (BASELINE configs[3]): RBF Gram + jittered "
                                   "Cholesky + forward solve + MLL, L written; MLL all-reduced",
                       "windows_per_gpu": B, "N": N, "D": D, "global_batch": B * world,
                       "parallelism": f"window-sharded x{world}", "kernel": "gpk_exact_mll_f32"},
            "roofline": {"bound": "hbm", "achieved": achieved / 1e9, "peak": HBM_PEAK / 1e9,
                         "unit": "GB/s", "frac": achieved / HBM_PEAK,
                         "traffic": load_traffic(N, D, B),
                         "kernel_ms": kern_ms, "bytes_per_window": bpw,
                         "fp32_flops_per_window": fpw,
                         "fp32_frac": fpw * B / (kern_ms * 1e-3) / FP32_PEAK},
            "mean_mll": mean_mll,
        }
        if grad_ms is not None:
            line["backward"] = {"kernel": "gpk_exact_mll_grad_f32", "kernel_ms": grad_ms,
                                "windows_per_s_per_gpu": B / (grad_ms * 1e-3),
                                "note": "analytic dX/dy/dhyper of the same windows; not the headline"}
        if world == 1 and not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(N, D, args.cpu_seconds)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
