"""Kernel times of the variational path (K_ZZ factor, forward, adjoint) with HIP events;
GPK_LIB selects an A/B build.   python scripts/time_var.py [B] [N] [M] [D]"""
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fine_grained_gaussian_process_forcasting_amd import ops  # noqa: E402

B, N, M, D = (int(v) for v in (sys.argv[1:] + ["1024", "256", "64", "32"])[:4])
LN2 = math.log(2.0)
dev = torch.device("cuda", 0)
g = torch.Generator().manual_seed(0)
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


def timeit(fn, n=30):
    # back-to-back calls between one event pair: the GPU stays busy, so host launch
    # latency is hidden whenever the kernels are longer than it
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / n


t_k = timeit(lambda: ops.kzz_cholesky(Z, None, None, jitter=1e-4, hyper=kz_h))
t_f = timeit(lambda: ops.variational_forward(X, Z, kz.Linv, vm, vs, y=y, hyper=hyper, want_flags=False))
t_a = timeit(lambda: ops.variational_adjoint(X, Z, kz.Linv, vm, vs, hyper, gm, gv))
print(f"{os.environ.get('GPK_LIB', 'default')}: B={B} N={N} M={M} D={D} kzz {t_k:.4f} fwd {t_f:.4f} adj {t_a:.4f} ms",
      flush=True)
