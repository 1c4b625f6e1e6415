"""Forward timing of one libgpk build (GPK_LIB) at N = 800, for the knockout A/B of
gpk_exact_large.hip (results of a knockout build are meaningless; only the time is read)."""
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
    f = lambda: ops.exact_mll(X, y, None, None, None, None, hyper=h, want_L=True)
    f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        f()
    e1.record()
    torch.cuda.synchronize()
    out.append(f"B={B} {e0.elapsed_time(e1) / 5:.3f} ms")
print(os.environ.get("GPK_LIB", "product"), " | ".join(out), flush=True)
