"""The exact-GP path for 256 < N <= 800 (csrc/gpk_exact_large.hip) against the fp64 oracle.

GPyTorch keeps the exact MLL on Cholesky up to settings.max_cholesky_size = 800, so the
reference's ExactGPModel (denoising_model/GPModel.py:4-13) factors windows of any N up to
there; above 256 the blocked kernels run (the window's matrix in HBM, 32-wide panels). Same
bars as the N <= 256 tests: 1e-4 relative, norm-wise per window for L / z / gradient blocks,
per window for the MLL; info codes exactly GPyTorch's (0 / -t after t jitter rungs / k > 0).
"""
import math
import warnings

import numpy as np
import pytest
import torch

from oracle import gp_oracle as O

pytestmark = pytest.mark.gpu

LN2 = float(np.log(2.0))
NOISE0 = LN2 + 1e-4
TOL = 1e-4


def _rel_rows(a, b):
    a = np.asarray(a, np.float64).reshape(a.shape[0], -1)
    b = np.asarray(b, np.float64).reshape(b.shape[0], -1)
    return np.linalg.norm(a - b, axis=1) / np.linalg.norm(b, axis=1)


def _rel(a, b):
    a = np.asarray(a, np.float64).ravel()
    b = np.asarray(b, np.float64).ravel()
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


def _inputs(B, N, D, seed):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(B, N, D, generator=g) / math.sqrt(D), torch.randn(B, N, generator=g)


def _hyper(ops, dev, s2, noise, c, ls):
    return ops.pack_exact_hyper(s2, noise, c, torch.tensor(np.atleast_1d(ls), dtype=torch.float32), dev)


@pytest.mark.parametrize("B,N,D,ard", [(3, 257, 4, False), (2, 300, 32, True), (2, 511, 16, False),
                                       (2, 512, 64, False), (2, 799, 1, False), (2, 800, 32, True)])
def test_large_forward_parity(cuda_device, B, N, D, ard):
    from fine_grained_gaussian_process_forcasting_amd import ops
    X, y = _inputs(B, N, D, seed=N + D)
    ls = np.linspace(0.6, 1.4, D) if ard else LN2
    s2, c, noise = 1.3, 0.2, NOISE0
    h = _hyper(ops, cuda_device, s2, noise, c, ls)
    out = ops.exact_mll(X.to(cuda_device), y.to(cuda_device), None, None, None, None, hyper=h,
                        want_L=True, want_z=True)
    torch.cuda.synchronize()
    ref = O.exact_mll(X.double().numpy(), y.double().numpy(), ls, s2, c, noise)
    assert (out.info.cpu().numpy() == 0).all()
    L = out.L.cpu().double().numpy()
    assert np.all(np.triu(L, 1) == 0.0), "upper triangle must be exactly zero"
    assert _rel_rows(L, ref.L).max() <= TOL
    assert _rel_rows(out.z.cpu().numpy(), ref.z).max() <= TOL
    mll = out.mll.cpu().double().numpy()
    assert np.max(np.abs(mll - ref.mll) / np.abs(ref.mll)) <= TOL
    # deterministic: a second launch is bitwise identical; without want_L the MLL is unchanged
    again = ops.exact_mll(X.to(cuda_device), y.to(cuda_device), None, None, None, None, hyper=h,
                          want_L=False, want_z=True)
    torch.cuda.synchronize()
    assert again.L is None
    assert torch.equal(again.mll.cpu(), out.mll.cpu()) and torch.equal(again.z.cpu(), out.z.cpu())


def _ladder_jitter(t):
    return 1e-6 * 10 ** (t - 1) if t > 0 else 0.0


def test_large_ladder_nan_and_failures(cuda_device):
    """Singular windows (all points equal, zero noise: the in-kernel ladder restarts them), a
    NaN window and regular windows in one launch at N = 300; then an indefinite K (NotPSD)."""
    from fine_grained_gaussian_process_forcasting_amd import NanError, NotPSDError, ops
    B, N, D = 5, 300, 6
    X, y = _inputs(B, N, D, seed=5)
    for b in (0, 3):
        X[b] = X[b, :1].expand(N, D)
    X[1, 7, 2] = float("nan")
    ls, s2, noise = 0.3, 1.0, 0.0
    h = _hyper(ops, cuda_device, s2, noise, 0.0, ls)
    out = ops.exact_mll(X.to(cuda_device), y.to(cuda_device), None, None, None, None, hyper=h,
                        want_L=True, want_z=True)
    torch.cuda.synchronize()
    info = out.info.cpu().numpy()
    assert info[0] < 0 and info[3] < 0, info
    assert info[1] > 0
    assert info[2] == 0 and info[4] == 0
    L = out.L.cpu().double().numpy()
    for b in (0, 3):
        K = np.ones((N, N)) + _ladder_jitter(-int(info[b])) * np.eye(N)
        assert np.all(np.triu(L[b], 1) == 0.0)
        assert np.linalg.norm(L[b] @ L[b].T - K) / np.linalg.norm(K) <= 1e-5
    ref = O.exact_mll(X[[2, 4]].double().numpy(), y[[2, 4]].double().numpy(), ls, s2, 0.0, noise)
    assert _rel_rows(L[[2, 4]], ref.L).max() <= TOL
    mll = out.mll.cpu().double().numpy()[[2, 4]]
    assert np.max(np.abs(mll - ref.mll) / np.abs(ref.mll)) <= TOL
    with pytest.raises(NanError):
        with warnings.catch_warnings():
            warnings.simplefilter("ignore")
            ops.check_cholesky_info(out.info, 1e-6, inputs=(X,))
    X2, y2 = _inputs(2, 280, 3, seed=9)
    h2 = _hyper(ops, cuda_device, 1.0, -5.0, 0.0, 1.0)    # K - 5I is indefinite
    bad = ops.exact_mll(X2.to(cuda_device), y2.to(cuda_device), None, None, None, None, hyper=h2)
    torch.cuda.synchronize()
    assert (bad.info.cpu().numpy() > 0).all()
    assert torch.isnan(bad.mll.cpu()).all()
    with pytest.raises(NotPSDError):
        with warnings.catch_warnings():
            warnings.simplefilter("ignore")
            ops.check_cholesky_info(bad.info, 1e-6, inputs=(X2,))


@pytest.mark.parametrize("B,N,D,ard", [(2, 300, 8, True), (2, 512, 32, False), (2, 800, 16, False),
                                       (2, 333, 64, True)])
def test_large_grad_vs_oracle(cuda_device, B, N, D, ard):
    from fine_grained_gaussian_process_forcasting_amd import ops
    X, y = _inputs(B, N, D, seed=3 * N + D)
    ls = np.linspace(0.6, 1.4, D) if ard else LN2
    s2, c, noise = 1.3, 0.2, NOISE0
    gout = torch.rand(B, generator=torch.Generator().manual_seed(N)) + 0.5
    dev = cuda_device
    h = _hyper(ops, dev, s2, noise, c, ls)
    fw = ops.exact_mll(X.to(dev), y.to(dev), None, None, None, None, hyper=h, want_L=True, want_z=True)
    assert (fw.info.cpu() == 0).all()
    gr = ops.exact_mll_grad(X.to(dev), fw.L, fw.z, h, gout.to(dev))
    torch.cuda.synchronize()
    ref = O.exact_mll_grads(X.double().numpy(), y.double().numpy(), ls, s2, c, noise,
                            gout=gout.double().numpy())
    dh = gr.dhyp.sum(0).cpu().double().numpy()
    got = {"X": gr.dX.cpu().numpy(), "y": gr.dy.cpu().numpy(), "outputscale": dh[0], "noise": dh[1],
           "mean_constant": dh[2], "lengthscale": dh[3:] if ard else dh[3]}
    for k in got:
        e = _rel(got[k], ref[k])
        print(f"N={N} D={D} {k:14s} hip {e:.2e}")
        assert e <= TOL, (k, e)
    # deterministic partial sums
    gr2 = ops.exact_mll_grad(X.to(dev), fw.L, fw.z, h, gout.to(dev))
    torch.cuda.synchronize()
    assert torch.equal(gr.dhyp.cpu(), gr2.dhyp.cpu()) and torch.equal(gr.dX.cpu(), gr2.dX.cpu())


def test_large_autograd_path(cuda_device):
    """ExactGPModel-style objective through ops_autograd at N = 400: every .grad from the
    blocked HIP backward, vs the oracle."""
    from fine_grained_gaussian_process_forcasting_amd import ops_autograd
    B, N, D = 2, 400, 5
    X, y = _inputs(B, N, D, seed=17)
    dev = cuda_device
    Xd = X.to(dev).requires_grad_(True)
    yd = y.to(dev).requires_grad_(True)
    p = {k: torch.tensor(v, device=dev, requires_grad=True)
         for k, v in dict(ls=[0.9], s2=1.1, c=0.05, nz=0.3).items()}
    mll = ops_autograd.exact_log_prob(Xd, yd, p["ls"], p["s2"], p["c"], p["nz"])
    (-mll.mean()).backward()
    ref = O.exact_mll_grads(X.double().numpy(), y.double().numpy(), 0.9, 1.1, 0.05, 0.3,
                            gout=-np.ones(B) / B)
    assert _rel(Xd.grad.cpu(), ref["X"]) <= TOL
    assert _rel(yd.grad.cpu(), ref["y"]) <= TOL
    assert _rel(p["ls"].grad.cpu(), ref["lengthscale"]) <= TOL
    assert _rel(p["s2"].grad.cpu(), ref["outputscale"]) <= TOL
    assert _rel(p["c"].grad.cpu(), ref["mean_constant"]) <= TOL
    assert _rel(p["nz"].grad.cpu(), ref["noise"]) <= TOL


@pytest.mark.parametrize("B,N,Ns,D", [(2, 300, 77, 5), (2, 800, 40, 32), (3, 257, 16, 64)])
def test_large_posterior_parity(cuda_device, B, N, Ns, D):
    from fine_grained_gaussian_process_forcasting_amd import ops
    g = torch.Generator().manual_seed(N + Ns)
    X = torch.randn(B, N, D, generator=g) / math.sqrt(D)
    Xs = torch.randn(B, Ns, D, generator=g) / math.sqrt(D)
    y = torch.randn(B, N, generator=g)
    dev = cuda_device
    h = _hyper(ops, dev, LN2, NOISE0, 0.3, LN2)
    f = ops.exact_mll(X.to(dev), y.to(dev), None, None, None, None, hyper=h, want_L=True, want_z=True)
    p = ops.exact_posterior(X.to(dev), f.L, f.z, h, Xs.to(dev))
    torch.cuda.synchronize()
    assert int(f.info.abs().max()) == 0
    rm, rv = O.exact_predict(X.double().numpy(), y.double().numpy(), Xs.double().numpy(), LN2, LN2, 0.3,
                             NOISE0)
    assert _rel_rows(p.mean.cpu().numpy(), rm).max() <= TOL
    assert _rel_rows(p.var.cpu().numpy(), rv).max() <= TOL


def test_large_exact_gp_model(cuda_device):
    """ExactGPModel (GPModel.py:4-13) with 500 training points: train-mode MLL + backward,
    then eval-mode prediction, all through the blocked kernels, vs the oracle."""
    from fine_grained_gaussian_process_forcasting_amd.denoising_model.GPModel import ExactGPModel
    from fine_grained_gaussian_process_forcasting_amd.gp import GaussianLikelihood
    from fine_grained_gaussian_process_forcasting_amd.mlls import ExactMarginalLogLikelihood
    dev = cuda_device
    g = torch.Generator().manual_seed(8)
    N, D = 500, 3
    train_x = torch.rand(N, D, generator=g).to(dev)
    train_y = torch.sin(6.0 * train_x.sum(-1)).to(dev)
    test_x = torch.rand(33, D, generator=g).to(dev)
    lik = GaussianLikelihood().to(dev)
    model = ExactGPModel(train_x, train_y, lik).to(dev)
    mll = ExactMarginalLogLikelihood(lik, model)(model(train_x), train_y)
    (-mll).backward()
    s2 = float(model.covar_module.outputscale)
    ls = float(model.covar_module.base_kernel.lengthscale)
    noise = float(lik.noise)
    c = float(model.mean_module.constant)
    ref = O.exact_mll(train_x[None].cpu().double().numpy(), train_y[None].cpu().double().numpy(),
                      ls, s2, c, noise)
    assert abs(float(mll) - float(ref.mll[0])) / abs(float(ref.mll[0])) <= TOL
    assert model.covar_module.raw_outputscale.grad is not None
    assert torch.isfinite(model.covar_module.base_kernel.raw_lengthscale.grad).all()
    model.eval()
    lik.eval()
    with torch.no_grad():
        pred = lik(model(test_x))
    rm, rv = O.exact_predict(train_x[None].cpu().double().numpy(), train_y[None].cpu().double().numpy(),
                             test_x[None].cpu().double().numpy(), ls, s2, c, noise)
    assert _rel_rows(pred.mean[None].cpu().numpy(), rm).max() <= TOL
    assert _rel_rows(pred.variance[None].cpu().numpy(), rv + noise).max() <= TOL
