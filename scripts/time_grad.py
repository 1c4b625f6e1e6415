"""Kernel time of the exact backward (and forward) at B=512 N=256 D=32 with HIP events;
GPK_LIB selects an A/B build.   python scripts/time_grad.py [B] [N] [D]"""
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fine_grained_gaussian_process_forcasting_amd import ops  # noqa: E402

B, N, D = (int(v) for v in (sys.argv[1:] + ["512", "256", "32"])[:3])
dev = torch.device("cuda", 0)
g = torch.Generator().manual_seed(0)
X = (torch.randn(B, N, D, generator=g) / math.sqrt(D)).to(dev)
y = torch.randn(B, N, generator=g).to(dev)
h = ops.pack_exact_hyper(math.log(2), math.log(2) + 1e-4, 0.0, math.log(2), dev)
f = ops.exact_mll(X, y, None, None, None, None, hyper=h, want_L=True, want_z=True)
gout = torch.ones(B, device=dev)
for _ in range(3):
    ops.exact_mll_grad(X, f.L, f.z, h, gout)
torch.cuda.synchronize()
ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(10)]
for a, b in ev:
    a.record()
    ops.exact_mll_grad(X, f.L, f.z, h, gout)
    b.record()
torch.cuda.synchronize()
ms = sorted(a.elapsed_time(b) for a, b in ev)
print(f"{os.environ.get('GPK_LIB', 'default')}: grad median {ms[5]:.4f} ms min {ms[0]:.4f}", flush=True)
