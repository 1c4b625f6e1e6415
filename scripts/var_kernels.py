"""Run the variational kernels (K_ZZ factor, forward, adjoint) at BASELINE cfg 5
(B=1024 N=256 M=64 D=32) and the cfg-3 GP shapes (B=256, N=192 enc / 96 dec, M=256,
D=32) a few times -- a target for rocprofv3 kernel traces and PMC passes.

    python scripts/var_kernels.py [reps] [cfg5|cfg3|all]
"""
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fine_grained_gaussian_process_forcasting_amd import ops  # noqa: E402

LN2 = math.log(2.0)


def run(B, N, M, D, reps, dev):
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
    gm = torch.randn(B, N, device=dev)
    gv = torch.randn(B, N, device=dev)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
    tk = tf = tb = 0.0
    for r in range(reps + 1):
        ev[0].record()
        kz = ops.kzz_cholesky(Z, None, None, jitter=1e-4, hyper=kz_h)
        ev[1].record()
        ops.variational_forward(X, Z, kz.Linv, vm, vs, y=y, hyper=hyper, want_flags=False)
        ev[2].record()
        ops.variational_adjoint(X, Z, kz.Linv, vm, vs, hyper, gm, gv)
        ev[3].record()
        torch.cuda.synchronize()
        if r:
            tk += ev[0].elapsed_time(ev[1])
            tf += ev[1].elapsed_time(ev[2])
            tb += ev[2].elapsed_time(ev[3])
    print(f"B={B} N={N} M={M} D={D}: kzz {tk / reps:.3f} ms  fwd {tf / reps:.3f} ms  adj {tb / reps:.3f} ms",
          flush=True)


if __name__ == "__main__":
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    which = sys.argv[2] if len(sys.argv) > 2 else "all"
    dev = torch.device("cuda:0")
    if which in ("cfg5", "all"):
        run(1024, 256, 64, 32, reps, dev)
    if which in ("cfg3", "all"):
        run(256, 192, 256, 32, reps, dev)
        run(256, 96, 256, 32, reps, dev)
