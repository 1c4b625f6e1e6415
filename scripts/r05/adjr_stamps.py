"""Per-phase cycle totals of gpk_var_adj_r_kernel (cfg 5) from a GPK_ADJR_STAMPS=1 build:
GPK_LIB=.../_lib_ab/st/libgpk.so python scripts/r05/adjr_stamps.py"""
import ctypes
import math
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from fine_grained_gaussian_process_forcasting_amd import ops, _native  # noqa: E402

B, N, M, D = 1024, 256, 64, 32
LN2 = math.log(2.0)
dev = torch.device("cuda", 0)
g = torch.Generator().manual_seed(0)
X = (torch.randn(B, N, D, generator=g) / math.sqrt(D)).to(dev)
Z = (torch.randn(M, D, generator=g) / math.sqrt(D)).to(dev)
vm = (1e-3 * torch.randn(M, generator=g)).to(dev)
vs = (0.5 + 0.5 * torch.rand(M, generator=g)).to(dev)
w = torch.randn(D, generator=g).to(dev)
ls = torch.full((D,), LN2, device=dev)
kz_h = torch.cat([torch.tensor([LN2], device=dev), ls]).contiguous()
hyper = ops.pack_variational_hyper(LN2, LN2 + 1e-4, 1e-4, 0.1, w, ls, D, dev)
gm = torch.randn(B, N, generator=g).to(dev)
gv = torch.randn(B, N, generator=g).to(dev)
kz = ops.kzz_cholesky(Z, None, None, jitter=1e-4, hyper=kz_h)
for _ in range(3):
    ops.variational_adjoint(X, Z, kz.Linv, vm, vs, hyper, gm, gv)
torch.cuda.synchronize()
lib = _native.lib()
nw = 256 * 8
buf = (ctypes.c_uint * (nw * 16))()
assert lib.gpk_dev_adjr_stamps(buf, nw * 16) == 0
a = np.frombuffer(buf, dtype=np.uint32).reshape(nw, 16)[:, :10].astype(np.float64)
chunks = B * ((N + 31) // 32) / nw
names = ["loop", "points+K", "A=L^-1K", "var/dA/rows", "G", "dK/Q", "r/q rows", "Q^T zs", "QX", "dX"]
tot = a.sum(1).mean()
print(f"cycles per wave {tot:.0f} ({chunks:.1f} chunks/wave): per chunk {tot / chunks:.0f}")
for k, n in enumerate(names):
    print(f"  {n:12s} {a[:, k].mean() / chunks:9.0f} cyc/chunk  {100 * a[:, k].mean() / tot:5.1f} %")
