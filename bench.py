"""Benchmark of the MI355X GP hot path (BASELINE.json metric: GP windows/sec).

Headline workload (BASELINE.json configs[3], the north-star shape, which fits one GPU):
synthetic exact-GP windows, N=256, D=32 -- per step the fused kernel builds the RBF Gram,
runs the jittered Cholesky, the forward solve and the MLL for every window and writes L
(B,N,N) and the MLL. Weak scaling (default): every rank owns B=512 windows. Strong
scaling (--strong): B=512 windows in total, sharded with shard_range. The K timed steps
(one eager launch each; --graph: one HIP-graph replay of the K launches) are bracketed by
one pair of HIP events on the launch stream (roofline.kernel_ms = their elapsed time / K,
which agrees with the rocprofv3 kernel average plus the inter-kernel gap). The per-step MLL
partial sums stay on the device and are SUM-all-reduced across ranks once (RCCL over
xGMI) at the end of the timed region (distributed.ObjectiveAccumulator), so no
collective sits on a step's critical path.

Side legs in the same JSON line (not the headline):
  variational  BASELINE configs[4] per GPU: DeepGP variational path B=1024 N=256 M=64
               D=32 -- shared K_ZZ factor (gpk_kzz_chol_f64) + column-tiled predictive
               mean / variance / ELL (gpk_variational_f32), and the fused adjoint
               (gpk_variational_adjoint_f32), with its compute roofline;
  backward     the exact path's analytic adjoint on the headline windows;
  posterior    the exact path's eval-mode posterior (mean + variance at N new points per
               window) from the headline windows' factor;
  exact_large  B=512 windows of N=800 (256 < N <= 800, GPyTorch's Cholesky regime): the
               blocked forward and backward of gpk_exact_large.hip;
  e2e_step     the cfg-3 forecast -> GP blur -> denoise train step, eager and HIP-graph
               captured (scripts/gp_step.py, graphs.GraphedStep);
  cpu_baseline the reference's CPU arithmetic (GPyTorch's torch-CPU calls restated in
               oracle/) on the GPU box's host cores, all threads and 1 thread, plus the
               variational path; and the MLL relative error of the GPU kernel vs the
               fp64 oracle on a window sample (parity unpinned vs GPyTorch: DESIGN §2).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--strong]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N
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
    ObjectiveAccumulator, env_rank_world, shard_range)

HBM_PEAK = 8.0e12          # B/s, MI355X_MICROARCH.md chip table (spec)
FP32_PEAK = 157.3e12       # FLOP/s, vector == f32 MFMA
FP64_PEAK = 78.6e12        # FLOP/s, f64 vector == f64 MFMA
LN2 = math.log(2.0)


def bytes_per_window(N, D):   # X read + y read + L write + MLL write
    return 4 * (N * D + N + N * N + 1)


def flops_per_window(N, D):
    return 3 * D * N * (N + 1) // 2 + N ** 3 // 3 + N * N + 3 * N


def var_bytes_per_window(N, D):   # SURVEY.md §8d cfg 5: X + y read, mean + var write, ELL
    return 4 * (N * D + N + 2 * N + 1)


def var_flops_per_window(N, M, D):  # SURVEY.md §8d cfg 5: (fp32, fp64)
    return 3 * D * M * N + 5 * M * N + 2 * D * N + 8 * N, M * M * N


def var_adj_flops_per_window(N, M, D):
    """The REFERENCE's backward of one window (what autograd runs through GPyTorch's
    VariationalStrategy, DeepGP.py:14-73): it keeps A = L^-1 K_ZX and K_ZX from the forward,
    so nothing is recomputed. fp64: the triangular-solve adjoint dK = L^-T dA (M^2 N) and the
    window's share of dL^-1 = -tril(dK A^T) (M^2 N) = 2 M^2 N; fp32: the RBF adjoint's
    Q^T zs and Q X contractions (2 x 2MND) plus the elementwise dA / Q / dX work (~10MN + 6DN).
    DESIGN.md §4.5; what the kernels actually execute is var_adj_impl_flops_per_window."""
    return 4 * M * N * D + 10 * M * N + 6 * D * N, 2 * M * M * N


def var_adj_impl_flops_per_window(N, M, D, saved):
    """What the adjoint kernels execute per window, recomputation included: the f32 K_ZX Gram
    (3DMN + 5MN) is always recomputed; without a saved forward state (M <= 64, the register
    path) A = L^-1 K_ZX is recomputed too (+M^2 N fp64). Reported beside the reference count,
    never used for the roofline fraction."""
    f32, f64 = var_adj_flops_per_window(N, M, D)
    return f32 + 3 * D * M * N + 5 * M * N, f64 + (0 if saved else M * M * N)


def cpu_model():
    """The host CPU's model name (/proc/cpuinfo), for the cpu_baseline record."""
    try:
        with open("/proc/cpuinfo") as f:
            for ln in f:
                if ln.startswith("model name"):
                    return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    import platform
    return platform.processor() or "unknown"


def make_inputs(B, N, D, device, seed):
    g = torch.Generator().manual_seed(seed)
    X = (torch.randn(B, N, D, generator=g) / math.sqrt(D)).to(device)
    y = torch.randn(B, N, generator=torch.Generator().manual_seed(seed + 1)).to(device)
    return X, y


def time_launches(fn, n):
    """Mean time of n back-to-back calls of ``fn`` from ONE pair of HIP events on the
    current (launch) stream. An event pair around every launch would add several us of
    event overhead to each measured kernel."""
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        out = fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n, out


def time_graph(fn, n, warm=3):
    """GPU time of ONE call of ``fn``: n calls captured into one HIP graph, replayed once
    untimed (the first replay of a fresh graph exec uploads it), then one timed replay
    between HIP events, / n. No host work sits between the launches, so this is what the
    kernels take back to back -- the way a captured training step (graphs.GraphedStep) runs
    them. (The headline loop captures its K launches the same way, in main.)"""
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(warm):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(n):
            out = fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n, out


def time_side(fn, n):
    """(graph ms, eager ms, result) of a side-leg op: graph replay (time_graph) and n eager
    back-to-back calls after 3 warm-up calls (time_launches; includes host launch work)."""
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    eager, out = time_launches(fn, n)
    try:
        graph, out = time_graph(fn, n)
    except Exception:   # capture not possible here: report the eager time only
        graph = None
    return graph, eager, out


def cpu_exact_baseline(N, D, seconds, threads):
    """GPyTorch's own CPU arithmetic for this path (oracle.exact_mll_torch_cpu: the
    _sq_dist GEMM, torch.linalg.cholesky_ex + jitter ladder, cholesky_solve, logdet;
    MKL/LAPACK) timed on the host cores, fp32 like the reference."""
    from oracle import gp_oracle as O
    prev = torch.get_num_threads()
    torch.set_num_threads(threads)
    try:
        Bs = 64 if threads > 1 else 8
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
    finally:
        torch.set_num_threads(prev)
    return n / dt, f"{n} windows (batches of {Bs}, N={N}, D={D}) in {dt:.1f}s"


def cpu_var_baseline(N, M, D, seconds, threads):
    """The reference's variational forward on the CPU (oracle.variational_forward_torch_cpu:
    GPyTorch's torch calls incl. the per-window fp64 K_ZZ Cholesky of the expanded Z)."""
    from oracle import gp_oracle as O
    prev = torch.get_num_threads()
    torch.set_num_threads(threads)
    try:
        Bs = 64 if threads > 1 else 8
        g = torch.Generator().manual_seed(0)
        X = torch.randn(Bs, N, D, generator=g) / math.sqrt(D)
        Z = torch.randn(M, D, generator=g) / math.sqrt(D)
        args = (X, Z, np.full(D, LN2), LN2, torch.randn(D, generator=g), 0.1,
                1e-3 * torch.randn(M, generator=g), torch.ones(M))
        O.variational_forward_torch_cpu(*args)
        n = 0
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < seconds:
            O.variational_forward_torch_cpu(*args)
            n += Bs
        dt = time.perf_counter() - t0
    finally:
        torch.set_num_threads(prev)
    return n / dt, f"{n} windows (batches of {Bs}, N={N}, M={M}, D={D}) in {dt:.1f}s"


def cpu_exact_procs(N, D, seconds, procs):
    """The same arithmetic as P single-thread worker processes (scripts/cpu_baseline_procs.py,
    run as a CPU-only child: it never touches the GPU): what the host's cores deliver."""
    import subprocess
    env = dict(os.environ, HIP_VISIBLE_DEVICES="", CUDA_VISIBLE_DEVICES="", OMP_NUM_THREADS="1")
    try:
        r = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "cpu_baseline_procs.py"), str(procs),
                            str(seconds), str(N), str(D)], env=env, capture_output=True, text=True,
                           timeout=seconds + 300)
        lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
        if r.returncode != 0 or not lines:
            return {"error": (r.stderr or r.stdout)[-400:]}
        return json.loads(lines[-1])
    except Exception as e:  # a side leg never takes the headline line down
        return {"error": f"{type(e).__name__}: {e}"}


def mll_rel_err(X, y, mll_gpu, n=32):
    """Per-window relative error of the GPU MLL vs the fp64 oracle on a window sample."""
    from oracle import gp_oracle as O
    idx = np.linspace(0, X.shape[0] - 1, min(n, X.shape[0])).astype(int)
    ref = O.exact_mll(X[idx].cpu().double().numpy(), y[idx].cpu().double().numpy(), LN2, LN2, 0.0,
                      LN2 + 1e-4)
    got = mll_gpu[idx].cpu().double().numpy()
    return float(np.max(np.abs(got - ref.mll) / np.abs(ref.mll)))


def load_traffic(key):
    """HBM bytes per launch from the committed rocprofv3 PMC summary (profiles/), if any."""
    p = os.path.join(ROOT, "profiles", "pmc_summary.json")
    try:
        with open(p) as f:
            d = json.load(f)
        return d.get(key, {}).get("hbm_bytes_per_launch")
    except OSError:
        return None


def variational_leg(dev, B, N, M, D, steps, warmup, world, seed, label="BASELINE configs[4]"):
    """BASELINE configs[4] per GPU: forward (K_ZZ factor + predictive mean / var / ELL)
    and the fused backward, each timed over back-to-back launches (time_launches)."""
    g = torch.Generator().manual_seed(seed)
    X = (torch.randn(B, N, D, generator=g) / math.sqrt(D)).to(dev)
    y = torch.randn(B, N, generator=g).to(dev)
    Z = (torch.randn(M, D, generator=g) / math.sqrt(D)).to(dev)
    vm = (1e-3 * torch.randn(M, generator=g)).to(dev)
    vs = (0.5 + 0.5 * torch.rand(M, generator=g)).to(dev)
    w = torch.randn(D, generator=g).to(dev)
    ls = torch.full((D,), LN2, device=dev)
    kz_h = torch.cat([torch.tensor([LN2], device=dev), ls]).contiguous()
    hyper = ops.pack_variational_hyper(LN2, LN2 + 1e-4, 1e-4, 0.1, w, ls, D, dev)
    gm = torch.randn(B, N, device=dev)
    gv = torch.randn(B, N, device=dev)
    def step():
        kz = ops.kzz_cholesky(Z, None, None, jitter=1e-4, hyper=kz_h)
        out = ops.variational_forward(X, Z, kz.Linv, vm, vs, y=y, hyper=hyper, want_flags=False, save=True)
        adj = ops.variational_adjoint(X, Z, kz.Linv, vm, vs, hyper, gm, gv, saved=out.saved)
        return kz, out, adj

    for _ in range(warmup):
        kz, out, adj = step()
    torch.cuda.synchronize()
    saved = out.saved   # the training forward's state (M > 64; None: the adjoint recomputes)
    # each phase in its own back-to-back loop (same inputs as the step's): GPU time from a
    # graph replay (time_graph), the eager loop beside it. "fwd" is the inference forward,
    # "fwd_train" the training forward that also keeps A for the adjoint ("bwd").
    phases = {"kzz": lambda: ops.kzz_cholesky(Z, None, None, jitter=1e-4, hyper=kz_h),
              "fwd": lambda: ops.variational_forward(X, Z, kz.Linv, vm, vs, y=y, hyper=hyper, want_flags=False),
              "fwd_train": lambda: ops.variational_forward(X, Z, kz.Linv, vm, vs, y=y, hyper=hyper,
                                                           want_flags=False, save=True),
              "bwd": lambda: ops.variational_adjoint(X, Z, kz.Linv, vm, vs, hyper, gm, gv, saved=saved)}
    ms, eager = {}, {}
    for k, fn in phases.items():
        gms, ems, _ = time_side(fn, steps)
        ms[k] = gms if gms is not None else ems
        eager[k] = ems
    if world > 1:
        t = torch.tensor([ms["kzz"], ms["fwd"], ms["fwd_train"], ms["bwd"]], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        ms = dict(zip(["kzz", "fwd", "fwd_train", "bwd"], t.tolist()))
    f32, f64 = var_flops_per_window(N, M, D)
    roof_s = f64 / FP64_PEAK + f32 / FP32_PEAK          # per window, fp64 + fp32 roofs added
    a32, a64 = var_adj_flops_per_window(N, M, D)
    adj_roof_s = a64 / FP64_PEAK + a32 / FP32_PEAK
    t_fwd_s = ms["fwd"] * 1e-3
    achieved = (f32 + f64) * B / t_fwd_s
    return {
        "workload": f"DeepGP variational ({label}): B={B} N={N} M={M} D={D} per GPU",
        "windows_per_s_fwd": B * world / ((ms["kzz"] + ms["fwd"]) * 1e-3),
        "windows_per_s_train_step": B * world / ((ms["kzz"] + ms["fwd_train"] + ms["bwd"]) * 1e-3),
        "kernel_ms": {"gpk_kzz_chol_f64": ms["kzz"], "gpk_variational_f32": ms["fwd"],
                      "gpk_variational_train_f32": ms["fwd_train"],
                      "gpk_variational_adjoint_f32": ms["bwd"]},
        "adjoint_path": "saved-state (forward keeps A)" if saved is not None else "recompute",
        "eager_ms": {"gpk_kzz_chol_f64": eager["kzz"], "gpk_variational_f32": eager["fwd"],
                     "gpk_variational_train_f32": eager["fwd_train"],
                     "gpk_variational_adjoint_f32": eager["bwd"],
                     "note": "eager back-to-back calls incl. host launch work; kernel_ms = graph replay"},
        "roofline": {"kernel": "gpk_var_fwd_r_kernel" if (M <= 64 and D <= 32) else "gpk_var_fwd_l_kernel",
                     "bound": "mfma",
                     "achieved": achieved / 1e12, "peak": (f32 + f64) / roof_s / 1e12,
                     "unit": "TFLOP/s", "frac": roof_s * B / t_fwd_s,
                     "flops_per_window": {"fp32": f32, "fp64": f64},
                     "hbm_frac": var_bytes_per_window(N, D) * B / t_fwd_s / HBM_PEAK,
                     "traffic": load_traffic(f"var_B{B}_N{N}_M{M}_D{D}")},
        "backward_roofline": {"kernel": "gpk_variational_adjoint_f32 (all launches)", "bound": "mfma",
                              "achieved": sum(var_adj_flops_per_window(N, M, D)) * B / (ms["bwd"] * 1e-3) / 1e12,
                              "peak": sum(var_adj_flops_per_window(N, M, D)) / adj_roof_s / 1e12,
                              "unit": "TFLOP/s", "frac": adj_roof_s * B / (ms["bwd"] * 1e-3),
                              "flops_per_window": dict(zip(("fp32", "fp64"), var_adj_flops_per_window(N, M, D))),
                              "flops_basis": "the reference's backward (A and K_ZX kept by autograd; no recompute)",
                              "implementation_flops_per_window": dict(zip(("fp32", "fp64"), var_adj_impl_flops_per_window(
                                  N, M, D, saved is not None))),
                              "traffic": load_traffic(f"var_adjoint_B{B}_N{N}_M{M}_D{D}"),
                              "algorithmic_bytes": 4 * (2 * B * N * D + 2 * B * N)},
        "mean_ell": float(out.ell.double().mean()),
        "elbo_rel_err_vs_fp64_oracle": elbo_rel_err(X, y, Z, ls, w, vm, vs, out.ell, D),
        "info": int(kz.info.item()),
    }


def elbo_rel_err(X, y, Z, ls, w, vm, vs, ell_gpu, num_data, n=32):
    """BASELINE's 'ELBO rel-err' on a window sample (outside every timed region): the
    per-window ELBO of forecast_denoising.py:86-89 -- sum_i ELL_i / N - KL / num_data with
    num_data = d -- from the kernel's ELL sums, against the fp64 oracle
    (oracle.variational_forward + oracle.deep_elbo; parity unpinned vs GPyTorch itself)."""
    from oracle import gp_oracle as O
    idx = np.linspace(0, X.shape[0] - 1, min(n, X.shape[0])).astype(int)
    N = X.shape[1]
    m64, s64 = vm.cpu().double().numpy(), vs.cpu().double().numpy()
    ref = O.variational_forward(X[idx].cpu().double().numpy(), Z.cpu().double().numpy(),
                                ls.cpu().double().numpy(), LN2, w.cpu().double().numpy(), 0.1,
                                m64, s64, jitter=1e-4, dtype=np.float64)
    want = O.deep_elbo(y[idx].cpu().double().numpy(), ref.mean, ref.var, LN2 + 1e-4, m64, s64, num_data)
    got = ell_gpu[idx].cpu().double().numpy() / N - O.kl_meanfield(m64, s64) / num_data
    return float(np.max(np.abs(got - want) / np.abs(want)))


def variant_leg(name, B, N, D, steps):
    """Kernel time of a measurement-only variant build of the exact kernel (build_native.VARIANTS)
    on the headline shape, timed in a child process that loads that build (GPK_LIB)."""
    import subprocess
    lib = os.path.join(ROOT, "fine_grained_gaussian_process_forcasting_amd", "_lib_variants", name, "libgpk.so")
    if not os.path.exists(lib):
        return {"error": f"variant build {name} not present (build_native.build_variant)"}
    env = dict(os.environ, GPK_LIB=lib)
    try:
        r = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "time_exact.py"), str(B), str(N), str(D),
                            str(steps)], env=env, capture_output=True, text=True, timeout=300)
        lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
        if r.returncode != 0 or not lines:
            return {"error": (r.stderr or r.stdout)[-400:]}
        return json.loads(lines[-1])
    except Exception as e:  # a side leg never takes the headline line down
        return {"error": f"{type(e).__name__}: {e}"}


def e2e_leg(steps=10):
    """the cfg-3 forecast -> GP blur -> denoise train step (b=256, enc 192 /
    dec 96, d 32, M 256), eager (the reference's loop) and HIP-graph captured
    (graphs.GraphedStep), with and without the GP branch (scripts/gp_step.py)."""
    import importlib.util
    try:
        spec = importlib.util.spec_from_file_location("gp_step", os.path.join(ROOT, "scripts", "gp_step.py"))
        mod = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(mod)
        res = mod.run("cfg3", steps)
        res["note"] = "windows/s = b / step time; GP share = step(gp) - step(no gp); not the headline"
        return res
    except Exception as e:  # a side leg never takes the headline line down
        return {"error": f"{type(e).__name__}: {e}"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--B", type=int, default=512, help="windows per GPU (weak) or in total (--strong)")
    ap.add_argument("--N", type=int, default=256)
    ap.add_argument("--D", type=int, default=32)
    ap.add_argument("--strong", action="store_true", help="B is the global batch, sharded over ranks")
    ap.add_argument("--var-B", type=int, default=1024)
    ap.add_argument("--var-N", type=int, default=256)
    ap.add_argument("--var-M", type=int, default=64)
    ap.add_argument("--no-var", action="store_true", help="skip the variational side leg")
    ap.add_argument("--no-var3", action="store_true", help="skip the cfg-3 (M=256) variational legs")
    ap.add_argument("--cpu-seconds", type=float, default=6.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-grad", action="store_true", help="skip the backward side measurement")
    ap.add_argument("--no-e2e", action="store_true", help="skip the end-to-end train-step side leg")
    ap.add_argument("--no-cfg2", action="store_true", help="skip the B=128 N=128 side leg")
    ap.add_argument("--no-large", action="store_true", help="skip the B=512 N=800 side leg")
    ap.add_argument("--no-variants", action="store_true",
                    help="skip the measurement-only variant builds (e.g. under rocprofv3)")
    ap.add_argument("--backend", default="nccl", choices=("nccl", "gloo"),
                    help="process-group backend (nccl = RCCL; gloo only for the one-GPU world-2 test)")
    ap.add_argument("--graph", action="store_true",
                    help="time one HIP-graph replay of the K launches instead of K eager launches "
                         "(measured slower on MI355X: 72.5 vs 60.9 us per launch, DESIGN.md §6)")
    ap.add_argument("--share-device", action="store_true",
                    help="every rank uses cuda:0 (tests/test_world2_gpu.py: two ranks on one GPU)")
    args = ap.parse_args()

    rank, local, world = env_rank_world()
    if world != args.gpus and world == 1 and args.gpus > 1:
        raise SystemExit("--gpus > 1 must be launched with torch.distributed.run")
    local = 0 if args.share_device else local
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    # under torchrun the process group is created even at world size 1, so the RCCL
    # init / barrier / MAX all-reduce path of the timed region runs on a one-GPU box too
    pg = world > 1 or "RANK" in os.environ
    if pg:
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")

    N, D = args.N, args.D
    if args.strong:
        lo, hi = shard_range(args.B, rank, world)
        B, B_total = hi - lo, args.B
        X_all, y_all = make_inputs(args.B, N, D, "cpu", seed=0)
        X, y = X_all[lo:hi].to(dev), y_all[lo:hi].to(dev)
    else:
        B, B_total = args.B, args.B * world
        X, y = make_inputs(B, N, D, dev, seed=1000 * rank)
    hyper = ops.pack_exact_hyper(LN2, LN2 + 1e-4, 0.0, LN2, dev)   # GPyTorch init values

    info = torch.empty(B, device=dev, dtype=torch.int32)
    Lbuf = torch.empty(B, N, N, device=dev, dtype=torch.float32)   # L written every step

    def step(mll_out):
        # one launch per step: the per-window MLL lands in the accumulator's row
        return ops.exact_mll(X, y, None, None, None, None, hyper=hyper, mll_out=mll_out,
                             info_out=info, L_out=Lbuf)

    warm = ObjectiveAccumulator(args.warmup, dev, width=B)
    for _ in range(args.warmup):
        out = step(warm.slot())
    warm.reduce()          # loads the reduction / collective kernels outside the timed region
    torch.cuda.synchronize()
    ops.check_cholesky_info(out.info, 1e-6, inputs=(X,))   # one sync, outside the timed region

    # the timed region: the K steps (one exact-kernel launch each, each writing its own
    # accumulator row) bracketed by ONE pair of HIP events on the launch stream;
    # roofline.kernel_ms = their elapsed time / K (an event pair around every launch adds 4-12 us
    # of event overhead per 70 us kernel, and the same to the timed loop). --graph: the K
    # launches are captured into ONE HIP graph outside the timed region (one untimed replay
    # uploads it) and the timed region replays it; measured SLOWER than the eager loop on
    # MI355X (72.5 vs 60.9 us per launch): the replay's per-node overhead exceeds the host
    # launch work, which the eager loop hides behind 60 us kernels.
    acc = ObjectiveAccumulator(args.steps, dev, width=B)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    graph = None
    if args.graph:
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            step(warm.rows[0])
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            for _ in range(args.steps):
                step(acc.slot())
        graph.replay()          # upload (the same values the timed replay writes)
        torch.cuda.synchronize()
    if pg:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev0.record()
    if graph is not None:
        graph.replay()
    else:
        for _ in range(args.steps):
            step(acc.slot())
    ev1.record()
    totals, work = acc.reduce()
    torch.cuda.synchronize()
    if pg:
        dist.barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    kern_ms = ev0.elapsed_time(ev1) / args.steps
    ops.check_cholesky_info(info, 1e-6, inputs=(X,))
    rank_times = None
    if pg:
        t = torch.tensor([elapsed, kern_ms], device=dev, dtype=torch.float64)
        every = [torch.zeros_like(t) for _ in range(world)]
        dist.all_gather(every, t)
        rank_times = [[float(v) for v in r.tolist()] for r in every]
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, kern_ms = (float(v) for v in t.tolist())
    mean_mll = float(totals[-1].item()) / B_total
    eager_kern_ms = None
    if graph is not None:   # the eager loop beside the graph replay (same launches)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.steps):
            step(warm.rows[0])
        e1.record()
        torch.cuda.synchronize()
        eager_kern_ms = e0.elapsed_time(e1) / args.steps
    else:                   # the timed loop itself was the eager one
        eager_kern_ms = kern_ms

    # 256 < N <= 800 (GPyTorch's Cholesky regime, the blocked kernels of gpk_exact_large.hip):
    # B=512 windows of N=800, forward and backward, eager back-to-back calls
    large = None
    if rank == 0 and not args.no_large:
        BL, NL = 512, 800
        XL, yL = make_inputs(BL, NL, D, dev, seed=17)
        fl = ops.exact_mll(XL, yL, None, None, None, None, hyper=hyper, want_L=True, want_z=True)
        goutL = torch.ones(BL, device=dev)
        torch.cuda.synchronize()
        fwd_l, _ = time_launches(lambda: ops.exact_mll(XL, yL, None, None, None, None, hyper=hyper), 5)
        bwd_l, _ = time_launches(lambda: ops.exact_mll_grad(XL, fl.L, fl.z, hyper, goutL), 3)
        fl_f = NL ** 3 / 3 + 2 * NL * NL * D + 2 * NL * NL      # Cholesky, _sq_dist Gram, solve
        by_f = 4 * (NL * D + 2 * NL + NL * NL)                 # X, y in; L, z out
        large = {"workload": "exact-GP windows B=512 N=800 D=32 (256 < N <= 800: GPyTorch's "
                             "Cholesky regime), L written",
                 "kernel": "gpk_exact_mll_f32 / gpk_exact_mll_grad_f32 (gpk_exact_large.hip)",
                 "fwd_ms": fwd_l, "bwd_ms": bwd_l, "windows_per_s": BL / (fwd_l * 1e-3),
                 "fwd_fp32_frac": fl_f * BL / (fwd_l * 1e-3) / FP32_PEAK,
                 "fwd_hbm_frac_algorithmic": by_f * BL / (fwd_l * 1e-3) / HBM_PEAK,
                 "info_max": int(fl.info.abs().max()),
                 "note": "right-looking 32-wide panels with the window's matrix in HBM: bound by the "
                         "trailing matrix's traffic (DESIGN.md 4.10); not the headline"}
        del XL, yL, fl
    # BASELINE configs[1] (B=128, N=128, D=32): a side leg, same kernel, its own roofline
    cfg2 = None
    if rank == 0 and not args.no_cfg2:
        X2, y2 = make_inputs(128, 128, D, dev, seed=11)
        g2, e2, o2 = time_side(lambda: ops.exact_mll(X2, y2, None, None, None, None, hyper=hyper), 20)
        ms2 = g2 if g2 is not None else e2
        b2, f2 = bytes_per_window(128, D), flops_per_window(128, D)
        cfg2 = {"workload": "exact-GP windows B=128 N=128 D=32 (BASELINE configs[1]), L written",
                "kernel_ms": ms2, "eager_ms": e2, "windows_per_s": 128 / (ms2 * 1e-3),
                "hbm_frac": b2 * 128 / (ms2 * 1e-3) / HBM_PEAK,
                "fp32_frac": f2 * 128 / (ms2 * 1e-3) / FP32_PEAK,
                "note": "128 windows occupy half of the 256 CUs: latency-bound by one window's chain"}
        assert bool((o2.info == 0).all())

    # the per-rank share of a strong-scaled B=512 job at G = 2, 4, 8 GPUs, timed on this GPU
    # (window sharding has no exchange on the step's path, so the G-GPU step time is the
    # slowest rank's kernel time plus the one all-reduce at the end of the timed region)
    strong_share = None
    if rank == 0 and world == 1 and not args.strong and not args.no_cfg2:
        strong_share = {"note": "per-rank share of a strong-scaled B=512 job timed on one GPU; "
                                "implied G-GPU speed-up = t(512) / t(512/G)"}
        for G in (2, 4, 8):
            Bs = 512 // G
            Xs_, ys_ = X[:Bs].contiguous(), y[:Bs].contiguous()
            Ls_ = torch.empty(Bs, N, N, device=dev)
            f = lambda: ops.exact_mll(Xs_, ys_, None, None, None, None, hyper=hyper, L_out=Ls_)  # noqa: E731
            gG, eG, _ = time_side(f, 20)
            msG = gG if (gG is not None and graph is not None) else eG   # as the headline loop is timed
            strong_share[f"G{G}"] = {"windows_per_rank": Bs, "kernel_ms": msG, "graph_ms": gG,
                                     "implied_speedup": kern_ms / msG if B == 512 else None}

    grad_ms = post_ms = grad_eager = post_eager = None
    if not args.no_grad:
        fw = ops.exact_mll(X, y, None, None, None, None, hyper=hyper, want_L=True, want_z=True)
        gout = torch.ones(B, device=dev)
        gg, grad_eager, _ = time_side(lambda: ops.exact_mll_grad(X, fw.L, fw.z, hyper, gout), 10)
        grad_ms = gg if gg is not None else grad_eager
        # eval-mode posterior at Ns = N new points per window from the same factor
        Xs = make_inputs(B, N, D, dev, seed=77 + rank)[0]
        gp_, post_eager, _ = time_side(lambda: ops.exact_posterior(X, fw.L, fw.z, hyper, Xs), 10)
        post_ms = gp_ if gp_ is not None else post_eager

    var = None
    if not args.no_var:
        var = variational_leg(dev, args.var_B, args.var_N, args.var_M, D, max(20, args.steps // 2),
                              3, world, seed=7 + rank)

    # the cfg-3 GP shape the reference trains (DeepGP default M=256; enc N=192, dec N=96, b=256)
    var3 = None
    if rank == 0 and not args.no_var3:
        var3 = {f"N{n}": variational_leg(dev, 256, n, 256, D, 20, 3, 1, seed=13 + n,
                                         label=f"cfg-3 GP shape, {'enc' if n == 192 else 'dec'}")
                for n in (192, 96)}

    if rank == 0:
        value = B_total * args.steps / elapsed
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
            "scaling": "strong" if args.strong else "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "precision": "f32 inputs / outputs, fp32 RBF exponent, diagonal factor and TRSM; the Gram "
                         "and the trailing Cholesky updates on split-f16 MFMA (hi + lo planes, 22 "
                         "significant bits, every product exact, fp32 accumulation: DESIGN.md §4.1)",
            "data": "synthetic",
            "config": {"workload": "exact-GP windows (BASELINE configs[3]): RBF Gram + jittered "
                                   "Cholesky + forward solve + MLL, L written; MLL partials "
                                   "all-reduced once per timed region",
                       "windows_per_gpu": B, "N": N, "D": D, "global_batch": B_total,
                       "parallelism": f"window-sharded x{world}", "kernel": "gpk_exact_mll_f32",
                       "process_group": args.backend if pg else None},
            "roofline": {"bound": "hbm", "achieved": achieved / 1e9, "peak": HBM_PEAK / 1e9,
                         "unit": "GB/s", "frac": achieved / HBM_PEAK,
                         "traffic": load_traffic(f"exact_B{B}_N{N}_D{D}"),
                         "kernel": "gpk_exact_kernel", "kernel_ms": kern_ms,
                         "timed_loop": "one HIP-graph replay of the K launches" if graph is not None
                                       else "K eager launches",
                         "eager_kernel_ms": eager_kern_ms,
                         "bytes_per_window": bpw, "fp32_flops_per_window": fpw,
                         "fp32_frac": fpw * B / (kern_ms * 1e-3) / FP32_PEAK},
            "mean_mll": mean_mll,
        }
        if world == 1 and not args.no_variants:
            v = variant_leg("f32update", B, N, D, args.steps)
            if "kernel_ms" in v:
                v["hbm_frac"] = bpw * B / (v["kernel_ms"] * 1e-3) / HBM_PEAK
                v["slowdown_vs_split_f16"] = v["kernel_ms"] / kern_ms
            v["note"] = ("the same kernel with the trailing Cholesky updates on fp32 MFMA "
                         "(mfma_f32_16x16x4f32, 24-bit operands) instead of split-f16: a separate "
                         "build (build_native.VARIANTS), timed in a child process; not the headline")
            line["fp32_update"] = v
        if rank_times is not None:
            line["rank_times"] = {"ms_per_step": [r[0] / args.steps * 1e3 for r in rank_times],
                                  "kernel_ms": [r[1] for r in rank_times],
                                  "note": "per-rank values before the MAX all-reduce"}
        if grad_ms is not None:
            line["backward"] = {"kernel": "gpk_exact_mll_grad_f32", "kernel_ms": grad_ms, "eager_ms": grad_eager,
                                "windows_per_s_per_gpu": B / (grad_ms * 1e-3),
                                "note": "analytic dX/dy/dhyper of the same windows; not the headline"}
        if post_ms is not None:
            pb = 4 * (2 * N * D + N * (N + 1) // 2 + N + 2 * N)     # X, Xs, lower L, z; mean + var
            pf = 2 * N * N * D + N * N * N + 2 * N * N + 10 * N * N  # Gram, TRSM, mean/var, RBF
            line["posterior"] = {"kernel": "gpk_exact_posterior_f32", "kernel_ms": post_ms, "eager_ms": post_eager,
                                 "test_points_per_window": N,
                                 "windows_per_s_per_gpu": B / (post_ms * 1e-3),
                                 "hbm_frac": pb * B / (post_ms * 1e-3) / HBM_PEAK,
                                 "fp32_frac": pf * B / (post_ms * 1e-3) / FP32_PEAK,
                                 "note": "eval-mode exact posterior mean + variance; not the headline"}
        if cfg2 is not None:
            line["cfg2"] = cfg2
        if large is not None:
            line["exact_large"] = large
        if var is not None:
            line["variational"] = var
            line["elbo_rel_err_vs_fp64_oracle"] = var["elbo_rel_err_vs_fp64_oracle"]
        if var3 is not None:
            line["variational_cfg3"] = var3
        if rank == 0 and strong_share is not None:
            line["strong_share"] = strong_share
        if world == 1 and not args.no_e2e:
            line["e2e_step"] = e2e_leg()
        if world == 1 and not args.no_cpu_baseline:
            # the cores this process may run on (sched_getaffinity), capped at the job's CPU
            # share (OMP_NUM_THREADS: 16 per GPU on the pool); os.cpu_count() is the machine
            affinity = len(os.sched_getaffinity(0))
            share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or affinity
            cores = max(1, min(affinity, share))
            nthr = torch.get_num_threads()
            v_all, s_all = cpu_exact_baseline(N, D, args.cpu_seconds, nthr)
            v_one, s_one = cpu_exact_baseline(N, D, args.cpu_seconds / 2, 1)
            procs = cpu_exact_procs(N, D, args.cpu_seconds, cores)
            v_procs = procs.get("value")
            best, best_cores = max((v_procs or 0.0, cores), (v_all, nthr), (v_one, 1))
            line["cpu_baseline"] = {
                "value": best, "unit": "windows/s", "cores": best_cores, "kind": "port",
                "cpu_model": cpu_model(), "os_cpu_count": os.cpu_count(), "affinity_cores": affinity,
                "sample": f"the best of three ways to run oracle.exact_mll_torch_cpu (GPyTorch's "
                          f"torch-CPU arithmetic, fp32, MKL) on this host: {cores} single-thread "
                          f"processes (the job's CPU share of {affinity} affinity cores), one process "
                          f"on {nthr} threads, one thread",
                "processes": {"value": v_procs, "cores": cores, "detail": procs},
                "threads": {"value": v_all, "cores": nthr, "sample": s_all,
                            "note": "one process, MKL threads over a batched cholesky_ex: how the "
                                    "reference itself would run it"},
                "one_thread": {"value": v_one, "cores": 1, "sample": s_one},
                "gpu_over_cpu": value / best,
                "mll_rel_err_vs_fp64_oracle": mll_rel_err(X, y, out.mll),
            }
            if v_procs:
                # the whole host: the measured per-process rate times every affinity core. An
                # extrapolation, not a run -- the GPU pool caps a job's worker processes at its
                # CPU share (OMP_NUM_THREADS), so `cores` single-thread processes is the most it runs.
                whole = v_procs / cores * affinity
                line["cpu_baseline"]["all_affinity_cores"] = {
                    "value": whole, "cores": affinity, "measured": False,
                    "basis": f"{v_procs / cores:.0f} windows/s per single-thread process "
                             f"(measured, {cores} processes) x {affinity} affinity cores, assuming "
                             f"linear scaling across sockets",
                    "gpu_over_cpu": value / whole}
            if var is not None:
                vv, sv = cpu_var_baseline(args.var_N, args.var_M, D, args.cpu_seconds, nthr)
                line["cpu_baseline"]["variational"] = {
                    "value": vv, "unit": "windows/s", "cores": nthr, "kind": "port",
                    "sample": f"{sv} through oracle.variational_forward_torch_cpu (the reference's "
                              f"per-window fp64 K_ZZ Cholesky + TRSM), forward only"}
        print(json.dumps(line), flush=True)
    if pg:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
