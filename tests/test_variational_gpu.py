"""Parity of the variational (DeepGP) kernels against the fp64 oracle.

gpk_kzz_chol_f64 (shared K_ZZ factor) and gpk_variational_f32 (batched predictive
mean / variance / expected log likelihood). Tolerance: 1e-4 relative, norm-wise
per window (north_star); the oracle is oracle/gp_oracle.py::variational_forward.
"""
import math

import numpy as np
import pytest
import torch

from oracle import gp_oracle as O

pytestmark = pytest.mark.gpu
LN2 = math.log(2.0)


def _case(B, N, M, D, seed=0, trained=False):
    g = torch.Generator().manual_seed(seed)
    X = torch.randn(B, N, D, generator=g) / math.sqrt(D)
    Z = torch.randn(M, D, generator=g) / math.sqrt(D)
    m = 1e-3 * torch.randn(M, generator=g)
    s = torch.rand(M, generator=g) * 0.5 + 0.5 if trained else torch.ones(M)
    w = torch.randn(D, generator=g)
    b0 = float(torch.randn(1, generator=g))
    y = torch.randn(B, N, generator=g)
    return X, Z, m, s, w, b0, y


def _rel(a, b):
    a = np.asarray(a, np.float64).reshape(a.shape[0], -1)
    b = np.asarray(b, np.float64).reshape(b.shape[0], -1)
    return np.linalg.norm(a - b, axis=1) / np.linalg.norm(b, axis=1)


# (130 and 250: padded last block row / column -- the inverse kernel's clamped staging and
# the factor's worker-only barrier with padded tiles)
@pytest.mark.parametrize("M,D", [(8, 4), (64, 32), (37, 5), (256, 32), (130, 16), (250, 32)])
def test_kzz_cholesky_parity(cuda_device, M, D):
    from fine_grained_gaussian_process_forcasting_amd import ops
    g = torch.Generator().manual_seed(M + D)
    Z = torch.randn(M, D, generator=g) / math.sqrt(D)
    ls = np.full(D, LN2)
    f = ops.kzz_cholesky(Z.to(cuda_device), LN2, torch.tensor(ls, dtype=torch.float32), jitter=1e-4)
    torch.cuda.synchronize()
    Kzz = O.rbf(Z.double().numpy(), Z.double().numpy(), ls, LN2, x1_eq_x2=True, zero_diag=False)
    Kzz[np.arange(M), np.arange(M)] += 1e-4
    Lref = np.linalg.cholesky(Kzz)
    L = f.L.cpu().numpy()
    assert int(f.info.item()) == 0
    assert np.linalg.norm(L - Lref) / np.linalg.norm(Lref) <= 1e-4
    Linv = f.Linv.cpu().numpy()
    assert np.linalg.norm(Linv @ Lref - np.eye(M)) <= 1e-4 * M
    assert np.all(np.triu(L, 1) == 0) and np.all(np.triu(Linv, 1) == 0)


@pytest.mark.parametrize("B,N,M,D,trained", [(3, 20, 8, 4, False), (4, 96, 64, 32, True),
                                             (2, 37, 37, 5, True), (4, 192, 256, 32, False),
                                             (8, 256, 64, 32, True),
                                             # M > 64: L^{-1}-in-registers kernel, every
                                             # (row blocks, dims) instantiation, ragged M / N
                                             (3, 70, 100, 7, True), (2, 50, 96, 20, True),
                                             (2, 33, 180, 40, True), (2, 64, 256, 16, True),
                                             (1, 40, 250, 64, True), (5, 192, 256, 32, True),
                                             # M <= 64 with D in (32, 64]: the LDS-tiled path
                                             (3, 40, 48, 48, True), (2, 30, 64, 64, True)])
def test_variational_parity(cuda_device, B, N, M, D, trained):
    from fine_grained_gaussian_process_forcasting_amd import ops
    X, Z, m, s, w, b0, y = _case(B, N, M, D, seed=B * 7 + N, trained=trained)
    ls = torch.full((D,), LN2)
    noise = LN2 + 1e-4
    dev = cuda_device
    f = ops.kzz_cholesky(Z.to(dev), LN2, ls.to(dev), jitter=1e-4)
    out = ops.variational_forward(X.to(dev), Z.to(dev), f.Linv, m.to(dev), s.to(dev), LN2, noise,
                                  1e-4, b0, w.to(dev), ls.to(dev), y=y.to(dev))
    torch.cuda.synchronize()
    ref = O.variational_forward(X.double().numpy(), Z.double().numpy(), ls.numpy(), LN2, w.numpy(),
                                b0, m.double().numpy(), s.double().numpy(), jitter=1e-4,
                                dtype=np.float64)
    assert _rel(out.mean.cpu().numpy(), ref.mean).max() <= 1e-4
    assert _rel(out.var.cpu().numpy(), ref.var).max() <= 1e-4
    ell_ref = O.expected_log_prob(y.double().numpy(), ref.mean, ref.var, noise).sum(-1)
    ell = out.ell.cpu().double().numpy()
    assert np.max(np.abs(ell - ell_ref) / np.abs(ell_ref)) <= 1e-4


def test_variational_config5_shape(cuda_device):
    """BASELINE config 5 shape: B=1024, N=256, M=64, D=32 (trained-like q(u))."""
    from fine_grained_gaussian_process_forcasting_amd import ops
    B, N, M, D = 1024, 256, 64, 32
    X, Z, m, s, w, b0, y = _case(B, N, M, D, seed=5, trained=True)
    ls = torch.full((D,), LN2)
    dev = cuda_device
    f = ops.kzz_cholesky(Z.to(dev), LN2, ls.to(dev), jitter=1e-4)
    out = ops.variational_forward(X.to(dev), Z.to(dev), f.Linv, m.to(dev), s.to(dev), LN2,
                                  LN2 + 1e-4, 1e-4, b0, w.to(dev), ls.to(dev), y=y.to(dev))
    torch.cuda.synchronize()
    sel = np.arange(0, B, 64)   # oracle on a 16-window sample of the batch
    ref = O.variational_forward(X[sel].double().numpy(), Z.double().numpy(), ls.numpy(), LN2,
                                w.numpy(), b0, m.double().numpy(), s.double().numpy(),
                                jitter=1e-4, dtype=np.float64)
    assert _rel(out.mean.cpu().numpy()[sel], ref.mean).max() <= 1e-4
    assert _rel(out.var.cpu().numpy()[sel], ref.var).max() <= 1e-4
    assert torch.isfinite(out.ell).all()


def test_variational_config5_all_windows(cuda_device):
    """BASELINE config 5 shape (B=1024, N=256, M=64, D=32, trained-like q(u)): mean and
    variance on EVERY window vs the fp64 oracle, the ELL on a 64-window sample."""
    from fine_grained_gaussian_process_forcasting_amd import ops
    B, N, M, D = 1024, 256, 64, 32
    X, Z, m, s, w, b0, y = _case(B, N, M, D, seed=5, trained=True)
    ls = torch.full((D,), LN2)
    noise = LN2 + 1e-4
    dev = cuda_device
    f = ops.kzz_cholesky(Z.to(dev), LN2, ls.to(dev), jitter=1e-4)
    out = ops.variational_forward(X.to(dev), Z.to(dev), f.Linv, m.to(dev), s.to(dev), LN2,
                                  noise, 1e-4, b0, w.to(dev), ls.to(dev), y=y.to(dev))
    torch.cuda.synchronize()
    ref = O.variational_forward(X.double().numpy(), Z.double().numpy(), ls.numpy(), LN2,
                                w.numpy(), b0, m.double().numpy(), s.double().numpy(),
                                jitter=1e-4, dtype=np.float64)
    assert _rel(out.mean.cpu().numpy(), ref.mean).max() <= 1e-4
    assert _rel(out.var.cpu().numpy(), ref.var).max() <= 1e-4
    sel = np.arange(0, B, 16)
    ell_ref = O.expected_log_prob(y[sel].double().numpy(), ref.mean[sel], ref.var[sel], noise).sum(-1)
    ell = out.ell.cpu().double().numpy()[sel]
    assert np.max(np.abs(ell - ell_ref) / np.abs(ell_ref)) <= 1e-4
    assert int(out.flags.item()) == 0


def test_variational_deterministic(cuda_device):
    """Fixed summation orders everywhere: two launches give bit-identical outputs."""
    from fine_grained_gaussian_process_forcasting_amd import ops
    B, N, M, D = 64, 192, 256, 32
    X, Z, m, s, w, b0, y = _case(B, N, M, D, seed=11, trained=True)
    ls = torch.full((D,), LN2).to(cuda_device)
    dev = cuda_device
    f = ops.kzz_cholesky(Z.to(dev), LN2, ls, jitter=1e-4)
    a = ops.variational_forward(X.to(dev), Z.to(dev), f.Linv, m.to(dev), s.to(dev), LN2, LN2,
                                1e-4, b0, w.to(dev), ls, y=y.to(dev))
    b = ops.variational_forward(X.to(dev), Z.to(dev), f.Linv, m.to(dev), s.to(dev), LN2, LN2,
                                1e-4, b0, w.to(dev), ls, y=y.to(dev))
    assert torch.equal(a.mean, b.mean) and torch.equal(a.var, b.var) and torch.equal(a.ell, b.ell)


def test_kzz_fp64_jitter_ladder(cuda_device):
    """Near-duplicate inducing points and NO variational jitter: the fp32 K_ZZ is
    numerically singular, the fp64 psd_safe_cholesky ladder (1e-8, 1e-7, 1e-6
    cumulative) must fire, report info = -t, emit GPyTorch's warning per step, and the
    factor must satisfy L L^T = K_ZZ + (cumulative jitter) I."""
    import warnings
    from fine_grained_gaussian_process_forcasting_amd import NumericalWarning, ops
    M, D = 48, 8
    g = torch.Generator().manual_seed(123)
    z0 = torch.randn(1, D, generator=g)
    Z = z0 + 1e-4 * torch.randn(M, D, generator=g)        # all points within 1e-4
    ls = torch.full((D,), LN2)
    f = ops.kzz_cholesky(Z.to(cuda_device), LN2, ls.to(cuda_device), jitter=0.0)
    torch.cuda.synchronize()
    info = int(f.info.item())
    assert info < 0, f"ladder did not fire (info={info})"
    with warnings.catch_warnings(record=True) as w:
        warnings.simplefilter("always")
        ops.check_cholesky_info(f.info, 1e-8)
    msgs = [str(x.message) for x in w if issubclass(x.category, NumericalWarning)]
    assert len(msgs) == -info and msgs[0] == "A not p.d., added jitter of 1.0e-08 to the diagonal"
    total = sum(1e-8 * 10 ** i - (1e-8 * 10 ** (i - 1) if i else 0.0) for i in range(-info))
    K = O.rbf(Z.double().numpy(), Z.double().numpy(), ls.numpy(), LN2, x1_eq_x2=True, zero_diag=False)
    L = f.L.cpu().numpy()
    resid = np.abs(L @ L.T - (K + total * np.eye(M))).max()
    assert resid <= 1e-6, resid          # fp32 rounding of K's entries is ~1e-7
    Linv = f.Linv.cpu().numpy()
    assert np.abs(Linv @ L - np.eye(M)).max() <= 1e-6 * np.abs(Linv).max()


def test_variance_clamp_flag_and_warning(cuda_device):
    """A negative K_XX jitter (test hook) drives part of the variance under 1e-6: the
    kernel clamps exactly like MVN.variance, raises the flag, and the distribution
    object emits GPyTorch's NumericalWarning."""
    import warnings
    from fine_grained_gaussian_process_forcasting_amd import NumericalWarning, ops
    from fine_grained_gaussian_process_forcasting_amd.gp import MultivariateNormal
    B, N, M, D = 4, 64, 32, 8
    X, Z, m, s, w, b0, y = _case(B, N, M, D, seed=9, trained=True)
    s = 0.1 + 0.2 * torch.rand(M, generator=torch.Generator().manual_seed(1))
    ls = torch.full((D,), LN2)
    dev = cuda_device
    f = ops.kzz_cholesky(Z.to(dev), LN2, ls.to(dev), jitter=1e-4)
    out = ops.variational_forward(X.to(dev), Z.to(dev), f.Linv, m.to(dev), s.to(dev), LN2, LN2,
                                  -0.4, b0, w.to(dev), ls.to(dev))
    ref = O.variational_forward(X.double().numpy(), Z.double().numpy(), ls.numpy(), LN2, w.numpy(), b0,
                                m.double().numpy(), s.double().numpy(), jitter=1e-4, dtype=np.float64,
                                var_jitter=-0.4)
    frac = float((ref.var <= 1e-6).mean())
    assert 0.05 < frac < 0.95, frac
    assert int(out.flags.item()) == 1
    assert np.abs(out.var.cpu().numpy() - ref.var).max() <= 1e-5
    d = MultivariateNormal(out.mean, out.var, clamp_flag=out.flags)
    with warnings.catch_warnings(record=True) as wl:
        warnings.simplefilter("always")
        _ = d.variance
    assert any(issubclass(x.category, NumericalWarning) for x in wl)
