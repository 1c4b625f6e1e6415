"""Time the shared K_ZZ factor + inverse (gpk_kzz_chol_f64) at M = 64 and 256 (D = 32)."""
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fine_grained_gaussian_process_forcasting_amd import ops  # noqa: E402

dev = torch.device("cuda", 0)
LN2 = math.log(2.0)
for M in (64, 256):
    g = torch.Generator().manual_seed(0)
    Z = (torch.randn(M, 32, generator=g) / math.sqrt(32)).to(dev)
    h = torch.cat([torch.tensor([LN2]), torch.full((32,), LN2)]).to(dev)
    for _ in range(3):
        kz = ops.kzz_cholesky(Z, None, None, jitter=1e-4, hyper=h)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        kz = ops.kzz_cholesky(Z, None, None, jitter=1e-4, hyper=h)
    e1.record()
    torch.cuda.synchronize()
    I = torch.eye(M, dtype=torch.float64, device=dev)
    err = float((kz.Linv @ kz.L - I).abs().max())
    print(f"M={M}: {e0.elapsed_time(e1) / 20 * 1e3:.1f} us per factor+inverse, |Linv L - I|max {err:.2e}, info {int(kz.info[0])}")

# the K_ZZ adjoint (gpk_kzz_backward_f64) on the same factor
for M in (64, 256):
    g = torch.Generator().manual_seed(1)
    Z = (torch.randn(M, 32, generator=g) / math.sqrt(32)).to(dev)
    s2 = torch.tensor(LN2, device=dev)
    ls = torch.full((32,), LN2, device=dev)
    kz = ops.kzz_cholesky(Z, s2, ls, jitter=1e-4)
    G = torch.randn(M, M, generator=g, dtype=torch.float64).tril().to(dev)
    for _ in range(3):
        ops.kzz_backward(G, kz.L, kz.Linv, Z, s2, ls)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        ops.kzz_backward(G, kz.L, kz.Linv, Z, s2, ls)
    e1.record()
    torch.cuda.synchronize()
    print(f"M={M}: {e0.elapsed_time(e1) / 20 * 1e3:.1f} us per K_ZZ adjoint")
