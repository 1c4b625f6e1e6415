"""Exact backward timing (gpk_exact_mll_grad_f32) of one libgpk build (GPK_LIB), HIP events
over back-to-back calls, at the bench shape and two other NB = 16 shapes."""
import math
import os
import sys

import torch

sys.path.insert(0, ".")
from fine_grained_gaussian_process_forcasting_amd import ops

dev = torch.device("cuda:0")
LN2 = math.log(2.0)
out = []
for B, N, D in [(512, 256, 32), (512, 250, 7), (512, 256, 64)]:
    g = torch.Generator().manual_seed(N + D)
    X = (torch.randn(B, N, D, generator=g) / math.sqrt(D)).to(dev)
    y = torch.randn(B, N, generator=g).to(dev)
    h = ops.pack_exact_hyper(LN2, LN2 + 1e-4, 0.0, torch.tensor([LN2]), dev)
    f = ops.exact_mll(X, y, None, None, None, None, hyper=h, want_L=True, want_z=True)
    gout = torch.ones(B, device=dev)
    run = lambda: ops.exact_mll_grad(X, f.L, f.z, h, gout)
    for _ in range(3):
        run()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        run()
    e1.record()
    torch.cuda.synchronize()
    out.append(f"B={B} N={N} D={D} {e0.elapsed_time(e1) / 20 * 1e3:.1f} us")
print((os.environ.get("GPK_LIB") or "_lib/product/libgpk.so").split("/")[-2], " | ".join(out), flush=True)
