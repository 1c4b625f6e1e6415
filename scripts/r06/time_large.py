"""Times the N > 256 exact kernels (forward MLL, backward, posterior) with HIP events over
back-to-back launches, and GPyTorch's fp32 torch-CPU arithmetic on a bounded sample beside them."""
import json
import math
import sys
import time

import torch

sys.path.insert(0, ".")
from fine_grained_gaussian_process_forcasting_amd import ops

dev = torch.device("cuda:0")
LN2 = math.log(2.0)
res = []


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


for B, N, D in [(256, 384, 32), (512, 512, 32), (512, 800, 32), (64, 800, 32)]:
    g = torch.Generator().manual_seed(N)
    X = (torch.randn(B, N, D, generator=g) / math.sqrt(D)).to(dev)
    y = torch.randn(B, N, generator=g).to(dev)
    Xs = (torch.randn(B, 256, D, generator=g) / math.sqrt(D)).to(dev)
    h = ops.pack_exact_hyper(1.3, LN2 + 1e-4, 0.0, torch.tensor([LN2]), dev)
    f = ops.exact_mll(X, y, None, None, None, None, hyper=h, want_L=True, want_z=True)
    assert int(f.info.abs().max()) == 0
    gout = torch.ones(B, device=dev)
    t_f = timed(lambda: ops.exact_mll(X, y, None, None, None, None, hyper=h, want_L=True))
    t_b = timed(lambda: ops.exact_mll_grad(X, f.L, f.z, h, gout))
    t_p = timed(lambda: ops.exact_posterior(X, f.L, f.z, h, Xs))
    # GPyTorch's fp32 torch-CPU arithmetic (cholesky_ex + triangular solve) on 8 windows, 16 threads
    torch.set_num_threads(16)
    Xc, yc = X[:8].cpu(), y[:8].cpu()
    t0 = time.perf_counter()
    xs = Xc / LN2
    d = torch.cdist(xs, xs) ** 2
    K = 1.3 * torch.exp(-0.5 * d) + (LN2 + 1e-4) * torch.eye(N)
    L, _ = torch.linalg.cholesky_ex(K)
    z = torch.linalg.solve_triangular(L, yc.unsqueeze(-1), upper=False)
    cpu_ms = (time.perf_counter() - t0) * 1e3 / 8
    r = {"B": B, "N": N, "D": D, "fwd_ms": t_f, "bwd_ms": t_b, "post_ms_256_test_points": t_p,
         "fwd_windows_per_s": B / (t_f * 1e-3), "cpu_fp32_ms_per_window_16_threads": cpu_ms,
         "fp32_flops_fwd_per_window": N ** 3 / 3 + 2 * N * N * D}
    r["fwd_tflops"] = r["fp32_flops_fwd_per_window"] * B / (t_f * 1e-3) / 1e12
    print(json.dumps(r), flush=True)
    res.append(r)
json.dump(res, open("gpurun_out/" + (sys.argv[1] if len(sys.argv) > 1 else "large") + "/time_large.json", "w"), indent=1)
