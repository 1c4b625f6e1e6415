"""Backward timing of one libgpk build (GPK_LIB) at N = 800 for the knockout A/B of
gpk_lg_grad_kernel (a knockout build's gradients are meaningless; only the time is read)."""
import math
import os
import sys

import torch

sys.path.insert(0, ".")
from fine_grained_gaussian_process_forcasting_amd import ops

dev = torch.device("cuda:0")
LN2 = math.log(2.0)
out = []
for B, N, D in [(64, 800, 32), (512, 800, 32)]:
    g = torch.Generator().manual_seed(N)
    X = (torch.randn(B, N, D, generator=g) / math.sqrt(D)).to(dev)
    y = torch.randn(B, N, generator=g).to(dev)
    h = ops.pack_exact_hyper(1.3, LN2 + 1e-4, 0.0, torch.tensor([LN2]), dev)
    f = ops.exact_mll(X, y, None, None, None, None, hyper=h, want_L=True, want_z=True)
    gout = torch.ones(B, device=dev)
    run = lambda: ops.exact_mll_grad(X, f.L, f.z, h, gout)
    run()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(3):
        run()
    e1.record()
    torch.cuda.synchronize()
    out.append(f"B={B} {e0.elapsed_time(e1) / 3:.3f} ms")
print((os.environ.get("GPK_LIB") or "_lib/product/x").split("/")[-2], " | ".join(out), flush=True)
