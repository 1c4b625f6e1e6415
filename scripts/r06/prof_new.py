"""Launches of the round-6 kernels for rocprofv3 (kernel stats / PMC passes): the fused exact
backward at the bench shape, and the N > 256 forward / backward / posterior at N = 800."""
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from fine_grained_gaussian_process_forcasting_amd import ops

dev = torch.device("cuda:0")
LN2 = math.log(2.0)
for B, N, D, reps in [(512, 256, 32, 5), (512, 800, 32, 2)]:
    g = torch.Generator().manual_seed(N)
    X = (torch.randn(B, N, D, generator=g) / math.sqrt(D)).to(dev)
    y = torch.randn(B, N, generator=g).to(dev)
    Xs = (torch.randn(B, 256, D, generator=g) / math.sqrt(D)).to(dev)
    h = ops.pack_exact_hyper(1.3, LN2 + 1e-4, 0.0, torch.tensor([LN2]), dev)
    f = ops.exact_mll(X, y, None, None, None, None, hyper=h, want_L=True, want_z=True)
    gout = torch.ones(B, device=dev)
    for _ in range(reps):
        ops.exact_mll_grad(X, f.L, f.z, h, gout)
        if N > 256:
            ops.exact_mll(X, y, None, None, None, None, hyper=h, want_L=True)
            ops.exact_posterior(X, f.L, f.z, h, Xs)
    torch.cuda.synchronize()
print("PROF_NEW_DONE")
