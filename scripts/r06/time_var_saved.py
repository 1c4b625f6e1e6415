"""Kernel time of the saved-state variational adjoint (the training pair's backward,
gpk_variational_adjoint_saved_f32) at one cfg-3 shape from the libgpk.so that GPK_LIB names.
    GPK_LIB=... python scripts/r06/time_var_saved.py [B] [N] [M] [D]   -> one JSON line"""
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from fine_grained_gaussian_process_forcasting_amd import ops  # noqa: E402

B, N, M, D = (int(v) for v in (sys.argv[1:] + ["256", "192", "256", "32"])[:4])
LN2 = math.log(2.0)
dev = torch.device("cuda", 0)
g = torch.Generator().manual_seed(13 + N)
X = (torch.randn(B, N, D, generator=g) / math.sqrt(D)).to(dev)
y = torch.randn(B, N, generator=g).to(dev)
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
out = ops.variational_forward(X, Z, kz.Linv, vm, vs, y=y, hyper=hyper, want_flags=False, save=True)
assert out.saved is not None


def timeit(fn, n=30):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n):
        r = fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / n, r


t, adj = timeit(lambda: ops.variational_adjoint(X, Z, kz.Linv, vm, vs, hyper, gm, gv, saved=out.saved))
print(json.dumps({"adj_ms": t, "dX_norm": float(adj.dX.double().norm()), "dLinv_norm": float(adj.dLinv.norm()),
                  "dZ_norm": float(adj.dZ.double().norm())}))
