"""ELBO terms on the device (gpk_gauss_ell_f32 / gpk_meanfield_kl_f32 through gpk::gauss_ell and
gpk::meanfield_kl): values and gradients against the plain-torch statement of
GaussianLikelihood.expected_log_prob(...).sum(-1) and the mean-field KL (the ELBO of
forecast_denoising.py:86-89), fp32 tolerance 1e-5 relative; plus torch.library.opcheck."""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu


def _ell_ref(y, mean, var, noise):
    return (-0.5 * (((y - mean) ** 2 + var) / noise + noise.log() + math.log(2 * math.pi))).sum(-1)


@pytest.mark.parametrize("R,N", [(1, 1), (3, 7), (256, 96), (1024, 256), (5, 300)])
def test_gauss_ell_value_and_grad(cuda_device, R, N):
    import fine_grained_gaussian_process_forcasting_amd  # noqa: F401  (registers gpk::)
    dev = cuda_device
    g = torch.Generator().manual_seed(R * 7 + N)
    y = torch.randn(R, N, generator=g).to(dev)
    mean = torch.randn(R, N, generator=g).to(dev).requires_grad_(True)
    var = (0.1 + torch.rand(R, N, generator=g)).to(dev).requires_grad_(True)
    noise = torch.tensor([0.7], device=dev, requires_grad=True)
    gell = torch.randn(R, generator=g).to(dev)
    got = torch.ops.gpk.gauss_ell(y, mean, var, noise)
    (got * gell).sum().backward()
    gm, gv, gn = mean.grad.clone(), var.grad.clone(), noise.grad.clone()
    for t in (mean, var, noise):
        t.grad = None
    ref = _ell_ref(y, mean, var, noise)
    (ref * gell).sum().backward()
    rel = lambda a, b: float((a - b).norm() / b.norm().clamp_min(1e-30))  # noqa: E731
    assert rel(got, ref) < 1e-5
    assert rel(gm, mean.grad) < 1e-5
    assert rel(gv, var.grad) < 1e-5
    assert rel(gn, noise.grad) < 1e-4


@pytest.mark.parametrize("M", [1, 16, 256, 300])
def test_meanfield_kl_value_and_grad(cuda_device, M):
    import fine_grained_gaussian_process_forcasting_amd  # noqa: F401
    dev = cuda_device
    g = torch.Generator().manual_seed(M)
    m = (0.3 * torch.randn(M, generator=g)).to(dev).requires_grad_(True)
    s = (0.5 + torch.rand(M, generator=g)).to(dev).requires_grad_(True)
    got = torch.ops.gpk.meanfield_kl(m, s)
    (2.5 * got.sum()).backward()
    gm, gs = m.grad.clone(), s.grad.clone()
    m.grad = s.grad = None
    s2 = s.pow(2)
    ref = 0.5 * (s2.sum() + m.pow(2).sum() - M - s2.log().sum())
    (2.5 * ref).backward()
    assert abs(float(got) - float(ref)) <= 1e-5 * max(1.0, abs(float(ref)))
    assert torch.allclose(gm, m.grad, rtol=1e-5, atol=1e-6)
    assert torch.allclose(gs, s.grad, rtol=1e-5, atol=1e-6)


def test_elbo_ops_opcheck(cuda_device):
    import fine_grained_gaussian_process_forcasting_amd  # noqa: F401
    dev = cuda_device
    y = torch.randn(4, 9, device=dev)
    mean = torch.randn(4, 9, device=dev, requires_grad=True)
    var = (0.2 + torch.rand(4, 9, device=dev)).requires_grad_(True)
    noise = torch.tensor([0.5], device=dev, requires_grad=True)
    torch.library.opcheck(torch.ops.gpk.gauss_ell, (y, mean, var, noise))
    m = torch.randn(12, device=dev, requires_grad=True)
    s = (0.5 + torch.rand(12, device=dev)).requires_grad_(True)
    torch.library.opcheck(torch.ops.gpk.meanfield_kl, (m, s))
    torch.library.opcheck(torch.ops.gpk.variational_elbo, (y, mean, var, noise, m, s, 0.1, 1e-6))


def test_variational_elbo_uses_fused_terms_and_matches_torch(cuda_device):
    """VariationalELBO on a DeepGPp output: the fused ELL / KL path equals the per-point
    GPyTorch-form expression (expected_log_prob(...).sum(-1) and the torch KL)."""
    from fine_grained_gaussian_process_forcasting_amd import settings
    from fine_grained_gaussian_process_forcasting_amd.denoising_model.DeepGP import DeepGPp
    from fine_grained_gaussian_process_forcasting_amd.mlls import DeepApproximateMLL, VariationalELBO
    dev = cuda_device
    torch.manual_seed(0)
    model = DeepGPp(16, 1234).to(dev)
    x = torch.randn(8, 40, 16, device=dev) / 4
    y = torch.randn(1, 8, 40, device=dev)
    with settings.num_likelihood_samples(1):
        _, dist = model.predict(x)
        mll = DeepApproximateMLL(VariationalELBO(model.likelihood, model, 16))
        got = mll(dist, y)
        lik = model.likelihood
        ll = lik.expected_log_prob(y, dist).sum(-1).div(40)
        q = model.hidden_layer.variational_strategy.variational_distribution
        s2 = q._variational_stddev.pow(2)
        kl = 0.5 * (s2.sum() + q.variational_mean.pow(2).sum() - s2.numel() - s2.log().sum())
        ref = (ll - kl / 16).mean(0)
    assert torch.allclose(got, ref, rtol=1e-5, atol=1e-6), (got, ref)


@pytest.mark.parametrize("sliced", [False, True])
def test_fused_elbo_value_and_grads_vs_unfused(cuda_device, sliced):
    """gpk::variational_elbo (VariationalELBO's fused path) against the unfused GPyTorch-form
    expression (expected_log_prob(...).sum(-1) / N - KL / num_data), value and every
    gradient (mean / var of the GP, noise, q(u)); ``sliced``: the dec point slice of a joint
    enc + dec output (strided rows, no copy), as denoise_model_2 produces it."""
    from fine_grained_gaussian_process_forcasting_amd import settings
    from fine_grained_gaussian_process_forcasting_amd.denoising_model.DeepGP import DeepGPp
    from fine_grained_gaussian_process_forcasting_amd.gp import VariationalELBO
    from fine_grained_gaussian_process_forcasting_amd.mlls import DeepApproximateMLL
    dev = cuda_device
    torch.manual_seed(3)
    model = DeepGPp(16, 77).to(dev)
    x = torch.randn(6, 50, 16, device=dev) / 4
    y = torch.randn(1, 6, 30 if sliced else 50, device=dev)
    params = [p for p in model.parameters() if p.requires_grad]

    def run(fused):
        with settings.num_likelihood_samples(1):
            _, dist = model.predict(x)
            if sliced:
                dist = dist.slice_points(20, None)
            mll = DeepApproximateMLL(VariationalELBO(model.likelihood, model, 16))
            if fused:
                out = mll(dist, y)
            else:
                base = mll.base_mll
                ll = base.likelihood.expected_log_prob(y, dist).sum(-1).div(dist.event_shape[0])
                out = (ll - base.model.variational_strategy.kl_divergence().div(base.num_data)).mean(0)
        gr = torch.autograd.grad(out.sum(), params, allow_unused=True)
        return out.detach(), gr

    a, ga = run(True)
    b, gb = run(False)
    assert torch.allclose(a, b, rtol=1e-5, atol=1e-6), (a, b)
    for p, u, v in zip(params, ga, gb):
        if v is None:
            assert u is None or float(u.abs().max()) == 0.0
            continue
        assert u is not None
        assert torch.allclose(u, v, rtol=1e-4, atol=1e-6), (p.shape, float((u - v).abs().max()))
