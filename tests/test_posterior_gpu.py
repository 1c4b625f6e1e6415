"""Exact-GP posterior at new inputs (eval mode): gpk_exact_posterior_f32 and
ExactGPModel.eval() against the fp64 oracle (oracle.exact_predict: GPyTorch's exact
prediction strategy). Parity unpinned against GPyTorch itself (not
importable here); the oracle restates upstream exact_prediction_strategies.

Tolerance: 1e-4 relative, norm-wise per window, on the posterior mean and on the
latent variance (north_star).
"""
import math
import warnings

import numpy as np
import pytest
import torch

from oracle import gp_oracle as O

pytestmark = pytest.mark.gpu
LN2 = math.log(2.0)


def _rel(a, b):
    a = np.asarray(a, np.float64).reshape(a.shape[0], -1)
    b = np.asarray(b, np.float64).reshape(b.shape[0], -1)
    return np.linalg.norm(a - b, axis=1) / np.linalg.norm(b, axis=1)


def _run(dev, X, y, Xs, ls, s2, c, noise):
    from fine_grained_gaussian_process_forcasting_amd import ops
    hyper = ops.pack_exact_hyper(s2, noise, c, torch.as_tensor(ls, dtype=torch.float32), dev)
    Xd, yd = X.to(dev), y.to(dev)
    f = ops.exact_mll(Xd, yd, None, None, None, None, want_L=True, want_z=True, hyper=hyper)
    p = ops.exact_posterior(Xd, f.L, f.z, hyper, Xs.to(dev))
    torch.cuda.synchronize()
    assert int(f.info.abs().max()) == 0
    return p.mean.cpu().double().numpy(), p.var.cpu().double().numpy()


@pytest.mark.parametrize("B,N,Ns,D", [(3, 16, 1, 4), (4, 37, 50, 5), (2, 128, 64, 32),
                                      (3, 250, 77, 1), (2, 256, 200, 32), (2, 96, 130, 64)])
def test_posterior_parity(cuda_device, B, N, Ns, D):
    g = torch.Generator().manual_seed(N + Ns + D)
    X = torch.randn(B, N, D, generator=g) / math.sqrt(D)
    Xs = torch.randn(B, Ns, D, generator=g) / math.sqrt(D)
    y = torch.randn(B, N, generator=g)
    mean, var = _run(cuda_device, X, y, Xs, LN2, LN2, 0.3, LN2 + 1e-4)
    rm, rv = O.exact_predict(X.double().numpy(), y.double().numpy(), Xs.double().numpy(), LN2, LN2, 0.3,
                             LN2 + 1e-4)
    assert _rel(mean, rm).max() <= 1e-4
    assert _rel(var, rv).max() <= 1e-4


def test_posterior_ard_offset_small_noise(cuda_device):
    """ARD lengthscales, inputs far from the origin (the centring matters), noise 1e-2,
    and test points that include the training points themselves."""
    B, N, D = 3, 64, 6
    g = torch.Generator().manual_seed(5)
    X = torch.randn(B, N, D, generator=g) + 25.0
    Xs = torch.cat([X[:, :20], torch.randn(B, 30, D, generator=g) + 25.0], 1)
    y = torch.randn(B, N, generator=g)
    ls = np.linspace(0.8, 2.0, D)
    mean, var = _run(cuda_device, X, y, Xs, ls, 1.3, -0.2, 1e-2)
    rm, rv = O.exact_predict(X.double().numpy(), y.double().numpy(), Xs.double().numpy(), ls, 1.3, -0.2,
                             1e-2)
    assert _rel(mean, rm).max() <= 1e-4
    assert _rel(var, rv).max() <= 1e-4
    assert np.all(var[:, :20] < 2e-2)   # near-interpolation at the training inputs


def test_posterior_full_size_property(cuda_device):
    """B=512 N=256 D=32 (BASELINE cfg 4 windows) with Ns=256: oracle on sampled windows,
    and on every window the size-independent identities at the training inputs:
    var_f(x_n) <= s2 and, with y = c, mean == c exactly up to rounding."""
    B, N, D = 512, 256, 32
    g = torch.Generator().manual_seed(0)
    X = torch.randn(B, N, D, generator=g) / math.sqrt(D)
    Xs = torch.randn(B, N, D, generator=g) / math.sqrt(D)
    y = torch.randn(B, N, generator=g)
    mean, var = _run(cuda_device, X, y, Xs, LN2, LN2, 0.0, LN2 + 1e-4)
    for b in (0, 137, 511):
        rm, rv = O.exact_predict(X[b:b + 1].double().numpy(), y[b:b + 1].double().numpy(),
                                 Xs[b:b + 1].double().numpy(), LN2, LN2, 0.0, LN2 + 1e-4)
        assert _rel(mean[b:b + 1], rm).max() <= 1e-4
        assert _rel(var[b:b + 1], rv).max() <= 1e-4
    assert np.all(var <= LN2 + 1e-6) and np.all(var > 0)
    m0, _ = _run(cuda_device, X, torch.full((B, N), 0.25), Xs, LN2, LN2, 0.25, LN2 + 1e-4)
    assert np.abs(m0 - 0.25).max() <= 1e-6


def test_exact_gp_model_eval_posterior(cuda_device):
    """ExactGPModel (GPModel.py:4-13) in eval mode, GPyTorch-style unbatched (N, D)
    training data: likelihood(model(test_x)) mean / variance vs the oracle, the
    training-input warning, and the prediction cache."""
    from fine_grained_gaussian_process_forcasting_amd.denoising_model.GPModel import ExactGPModel
    from fine_grained_gaussian_process_forcasting_amd.errors import GPInputWarning
    from fine_grained_gaussian_process_forcasting_amd.gp import GaussianLikelihood
    from fine_grained_gaussian_process_forcasting_amd.mlls import ExactMarginalLogLikelihood
    dev = cuda_device
    g = torch.Generator().manual_seed(3)
    N, D = 80, 3
    train_x = torch.rand(N, D, generator=g).to(dev)
    train_y = torch.sin(6.0 * train_x.sum(-1)).to(dev)
    test_x = torch.rand(41, D, generator=g).to(dev)
    lik = GaussianLikelihood().to(dev)
    model = ExactGPModel(train_x, train_y, lik).to(dev)
    # training-mode MLL of the unbatched model is a scalar
    mll = ExactMarginalLogLikelihood(lik, model)(model(train_x), train_y)
    assert mll.shape == ()
    model.eval()
    lik.eval()
    with torch.no_grad():
        pred = lik(model(test_x))
        mean, var = pred.mean, pred.variance
        assert mean.shape == (41,) and var.shape == (41,)
        L1 = model._prediction_cache[1][1]
        model(test_x[:5])
        assert model._prediction_cache[1][1] is L1          # factor reused across calls
        with warnings.catch_warnings(record=True) as w:
            warnings.simplefilter("always")
            model(train_x)
        assert any(issubclass(x.category, GPInputWarning) for x in w)
    s2 = float(model.covar_module.outputscale)
    ls = float(model.covar_module.base_kernel.lengthscale)
    noise = float(lik.noise)
    c = float(model.mean_module.constant)
    rm, rv = O.exact_predict(train_x[None].cpu().double().numpy(), train_y[None].cpu().double().numpy(),
                             test_x[None].cpu().double().numpy(), ls, s2, c, noise)
    assert _rel(mean[None].cpu().numpy(), rm).max() <= 1e-4
    assert _rel(var[None].cpu().numpy(), rv + noise).max() <= 1e-4
    # a parameter update invalidates the cached factor; train() drops it
    with torch.no_grad():
        model.covar_module.raw_outputscale.add_(0.1)
        model(test_x)
    assert model._prediction_cache[1][1] is not L1
    model.train()
    assert model._prediction_cache is None


def _posterior_fp64(Xtr, ytr, Xs, ls, s2, c, noise):
    """fp64 torch restatement of the exact posterior (mean, latent variance) for autograd."""
    d = (((Xtr.unsqueeze(-2) - Xtr.unsqueeze(-3)) / ls) ** 2).sum(-1)
    n = Xtr.shape[-2]
    K = s2 * torch.exp(-0.5 * d) + noise * torch.eye(n, dtype=torch.float64)
    L = torch.linalg.cholesky(K)
    ds = (((Xtr.unsqueeze(-2) - Xs.unsqueeze(-3)) / ls) ** 2).sum(-1)
    V = torch.linalg.solve_triangular(L, s2 * torch.exp(-0.5 * ds), upper=False)
    z = torch.linalg.solve_triangular(L, (ytr - c).unsqueeze(-1), upper=False)
    return c + (V * z).sum(-2), s2 - (V * V).sum(-2)


def test_exact_gp_model_eval_posterior_gradients(cuda_device):
    """Gradients through the eval posterior (GPyTorch allows them): with a parameter or the test
    inputs requiring grad, ExactGPModel's posterior runs the differentiable restatement; its
    values match the kernel path (gpk_exact_posterior_f32) and its gradients w.r.t. the test
    inputs and every hyper-parameter match an fp64 torch autograd restatement at 1e-4."""
    from fine_grained_gaussian_process_forcasting_amd.denoising_model.GPModel import ExactGPModel
    from fine_grained_gaussian_process_forcasting_amd.gp import GaussianLikelihood
    dev = cuda_device
    g = torch.Generator().manual_seed(11)
    N, D, Ns = 64, 3, 20
    train_x = torch.rand(N, D, generator=g).to(dev)
    train_y = torch.sin(6.0 * train_x.sum(-1)).to(dev)
    test_x = torch.rand(Ns, D, generator=g).to(dev)
    lik = GaussianLikelihood().to(dev)
    model = ExactGPModel(train_x, train_y, lik).to(dev)
    with torch.no_grad():
        model.likelihood.noise_covar.raw_noise.fill_(-2.0)
    model.eval()
    lik.eval()
    with torch.no_grad():
        ref_dist = model(test_x)
        m0, v0 = ref_dist.mean.clone(), ref_dist.variance.clone()
    xr = test_x.clone().requires_grad_(True)
    dist = model(xr)
    assert _rel(dist.mean[None].detach().cpu().numpy(), m0[None].cpu().double().numpy()).max() <= 1e-4
    assert _rel(dist.variance[None].detach().cpu().numpy(), v0[None].cpu().double().numpy()).max() <= 1e-4
    gm = torch.randn(Ns, generator=g).to(dev)
    gv = torch.randn(Ns, generator=g).to(dev)
    params = [xr, model.covar_module.raw_outputscale, model.covar_module.base_kernel.raw_lengthscale,
              model.mean_module.constant, model.likelihood.noise_covar.raw_noise]
    got = torch.autograd.grad((gm * dist.mean).sum() + (gv * dist.variance).sum(), params)
    # fp64 restatement in the same raw parameters (softplus constraints; noise > 1e-4)
    P = lambda t: t.detach().cpu().double().clone().requires_grad_(True)  # noqa: E731
    q = [P(t) for t in params]
    F = torch.nn.functional
    s2, ls = F.softplus(q[1]), F.softplus(q[2]).reshape(-1)
    c, noise = q[3].reshape(()), F.softplus(q[4]).reshape(()) + 1e-4
    mean, var = _posterior_fp64(train_x.cpu().double(), train_y.cpu().double(), q[0], ls, s2, c, noise)
    var = var.clamp_min(1e-6)
    want = torch.autograd.grad((gm.cpu().double() * mean).sum() + (gv.cpu().double() * var).sum(), q)
    for name, a, b in zip(["x", "outputscale", "lengthscale", "constant", "noise"], got, want):
        e = float((a.detach().cpu().double() - b).norm() / b.norm().clamp_min(1e-30))
        print(f"posterior grad {name:12s} {e:.2e}")
        assert e <= 1e-4, (name, e)
