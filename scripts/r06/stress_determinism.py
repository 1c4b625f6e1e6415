"""Race hunt on the final build: every production kernel launched many times on the same
inputs, every output compared BITWISE with the first launch (the kernels promise fixed-order
reductions, so any difference is a synchronisation bug). Prints one line per kernel."""
import math
import sys

import torch

sys.path.insert(0, ".")
from fine_grained_gaussian_process_forcasting_amd import ops

dev = torch.device("cuda:0")
LN2 = math.log(2.0)
REPS = int(sys.argv[1]) if len(sys.argv) > 1 else 100
bad_total = 0


def check(name, fn, reps=REPS):
    global bad_total
    ref = [t.clone() for t in fn()]
    bad = 0
    for _ in range(reps - 1):
        out = fn()
        if not all(torch.equal(a, b) for a, b in zip(ref, out)):
            bad += 1
    torch.cuda.synchronize()
    bad_total += bad
    print(f"{name:58s} {reps} launches, {bad} differ", flush=True)


def inputs(B, N, D, seed):
    g = torch.Generator().manual_seed(seed)
    return ((torch.randn(B, N, D, generator=g) / math.sqrt(D)).to(dev),
            torch.randn(B, N, generator=g).to(dev))


for B, N, D in [(512, 256, 32), (128, 128, 32), (64, 256, 32), (320, 250, 8)]:
    X, y = inputs(B, N, D, N + B)
    h = ops.pack_exact_hyper(LN2, LN2 + 1e-4, 0.0, torch.tensor([LN2]), dev)
    f = ops.exact_mll(X, y, None, None, None, None, hyper=h, want_L=True, want_z=True)
    check(f"exact forward B={B} N={N} D={D}",
          lambda: (lambda o: (o.mll, o.L, o.z, o.info))(
              ops.exact_mll(X, y, None, None, None, None, hyper=h, want_L=True, want_z=True)))
    gout = torch.ones(B, device=dev)
    check(f"exact backward B={B} N={N} D={D}",
          lambda: (lambda r: (r.dX, r.dy, r.dhyp))(ops.exact_mll_grad(X, f.L, f.z, h, gout)))
for B, N, D, Ns in [(16, 300, 8, 40), (8, 800, 32, 64)]:
    X, y = inputs(B, N, D, N)
    Xs = inputs(B, Ns, D, N + 1)[0]
    h = ops.pack_exact_hyper(1.3, LN2 + 1e-4, 0.2, torch.tensor([LN2]), dev)
    f = ops.exact_mll(X, y, None, None, None, None, hyper=h, want_L=True, want_z=True)
    r = max(10, REPS // 5)
    check(f"N>256 forward B={B} N={N} D={D}",
          lambda: (lambda o: (o.mll, o.L, o.z, o.info))(
              ops.exact_mll(X, y, None, None, None, None, hyper=h, want_L=True, want_z=True)), r)
    gout = torch.ones(B, device=dev)
    check(f"N>256 backward B={B} N={N} D={D}",
          lambda: (lambda g: (g.dX, g.dy, g.dhyp))(ops.exact_mll_grad(X, f.L, f.z, h, gout)), r)
    check(f"N>256 posterior B={B} N={N} Ns={Ns}",
          lambda: (lambda p: (p.mean, p.var))(ops.exact_posterior(X, f.L, f.z, h, Xs)), r)
# variational path: the K_ZZ factor + inverse, the forward (cfg 5 register path and the M = 256
# saved-state training forward), both adjoints and the K_ZZ adjoint
for B, N, M, D in [(1024, 256, 64, 32), (256, 192, 256, 32)]:
    g = torch.Generator().manual_seed(M + N)
    X = (torch.randn(B, N, D, generator=g) / math.sqrt(D)).to(dev)
    Z = (torch.randn(M, D, generator=g) / math.sqrt(D)).to(dev)
    vmean = (0.3 * torch.randn(M, generator=g)).to(dev)
    vstd = (0.5 + 0.5 * torch.rand(M, generator=g)).to(dev)
    w = (0.1 * torch.randn(D, generator=g)).to(dev)
    ls = torch.full((D,), 1.2)
    fz = ops.kzz_cholesky(Z, 1.1, ls.to(dev), jitter=1e-4)
    check(f"K_ZZ factor + inverse M={M}", lambda: (lambda o: (o.L, o.Linv, o.info))(
        ops.kzz_cholesky(Z, 1.1, ls.to(dev), jitter=1e-4)))
    hyper = ops.pack_variational_hyper(1.1, 0.7, 1e-4, 0.05, w, ls.to(dev), D, dev)
    save = M > 64
    fw = ops.variational_forward(X, Z, fz.Linv, vmean, vstd, hyper=hyper, save=save)
    check(f"variational forward B={B} N={N} M={M} save={save}", lambda: (lambda o: (o.mean, o.var) + (
        (o.saved,) if o.saved is not None else ()))(
        ops.variational_forward(X, Z, fz.Linv, vmean, vstd, hyper=hyper, save=save)))
    gm = (torch.randn(B, N, generator=g) * 1e-2).to(dev)
    gv = (torch.randn(B, N, generator=g) * 1e-2).to(dev)
    adj = lambda: ops.variational_adjoint(X, Z, fz.Linv, vmean, vstd, hyper, gm, gv, saved=fw.saved)
    check(f"variational adjoint B={B} N={N} M={M} saved={save}",
          lambda: (lambda r: (r.dX, r.dLinv, r.dpar, r.dZ))(adj()))
    dL = adj().dLinv
    check(f"K_ZZ adjoint M={M}", lambda: tuple(t for t in ops.kzz_backward(
        dL, fz.L, fz.Linv, Z, torch.tensor(1.1, device=dev), ls.to(dev)) if torch.is_tensor(t)))
print(f"TOTAL differing launches: {bad_total}", flush=True)
sys.exit(1 if bad_total else 0)
