"""CPU oracle for the GP blur/denoise hot path — TEST INFRASTRUCTURE ONLY.

This module is a NumPy/SciPy restatement of the arithmetic that GPyTorch 1.9.x /
linear_operator 0.3.x perform for the reference's GP path
(``denoising_model/GPModel.py``, ``denoising_model/DeepGP.py``,
``denoising_model/denoise_model_2.py:32-51``, ``forecast_denoising.py:86-89``).
Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import it, and only as the checker / CPU baseline. The product path
(``fine_grained_gaussian_process_forcasting_amd``) never imports it and has no CPU
fallback.

Parity status: **parity unpinned against GPyTorch itself.** GPyTorch and
linear_operator are not installed in this image (``import gpytorch`` raises
``ModuleNotFoundError``; an ordinary import error, not a permission denial) and
the reference ships no tests, golden vectors or fixtures for this path
(SURVEY.md §4, §8c). The oracle is pinned instead by closed-form known-answer
tests (N=1, N=2, K=I, the duplicate-point jitter ladder, KL at the prior) and by
an independent cross-check against ``torch.linalg`` (tests/test_oracle.py).

Every function cites the reference call site it serves and the upstream GPyTorch
module whose published algorithm it restates (upstream files carry no line
numbers here because the package is not vendored).
"""
from __future__ import annotations

import math
import warnings
from dataclasses import dataclass

import numpy as np
from scipy.linalg import lapack

LOG_2PI = math.log(2.0 * math.pi)


class NotPSDError(RuntimeError):
    """Mirror of linear_operator.utils.errors.NotPSDError."""


class NanError(RuntimeError):
    """Mirror of linear_operator.utils.errors.NanError."""


def softplus(x):
    """gpytorch.constraints.Positive transform (torch.nn.functional.softplus)."""
    x = np.asarray(x, dtype=np.float64)
    return np.where(x > 20.0, x, np.log1p(np.exp(np.minimum(x, 20.0))))


def inv_softplus(y):
    y = np.asarray(y, dtype=np.float64)
    return np.where(y > 20.0, y, np.log(np.expm1(y)))


# ---------------------------------------------------------------------------
# a2: RBF kernel (upstream gpytorch/kernels/kernel.py::Distance._sq_dist,
#     gpytorch/kernels/rbf_kernel.py, gpytorch/kernels/scale_kernel.py)
# ---------------------------------------------------------------------------
def sq_dist(x1, x2, x1_eq_x2: bool, zero_diag: bool):
    """GPyTorch ``Distance._sq_dist``: mean-centred GEMM form, clamped at 0.

    ``adj = x1.mean(-2)``; ``x1 -= adj``; ``x2 -= adj``;
    ``res = [-2 x1, |x1|^2, 1] @ [x2, 1, |x2|^2]^T``; diagonal forced to 0 when
    x1 is x2 and no gradient is required; ``clamp_min(0)``.
    Works on (..., n, d) arrays in the arrays' own dtype.
    """
    adj = x1.mean(axis=-2, keepdims=True)
    x1c = x1 - adj
    x2c = x2 - adj
    x1n = (x1c * x1c).sum(-1, keepdims=True)
    x2n = (x2c * x2c).sum(-1, keepdims=True)
    res = (-2.0 * x1c) @ np.swapaxes(x2c, -1, -2)
    res = res + x1n + np.swapaxes(x2n, -1, -2)
    if x1_eq_x2 and zero_diag:
        n = res.shape[-1]
        idx = np.arange(n)
        res[..., idx, idx] = 0.0
    return np.maximum(res, 0.0).astype(x1.dtype, copy=False)


def rbf(x1, x2, lengthscale, outputscale, x1_eq_x2=False, zero_diag=True):
    """ScaleKernel(RBFKernel) dense covariance: ``s2 * exp(-sq_dist(x1/l, x2/l)/2)``.

    ``lengthscale`` is a scalar (GPModel.py:8, no ARD) or a length-D vector
    (DeepGP.py:46-49, ``ard_num_dims=D``). ``postprocess_rbf`` = ``div_(-2).exp_()``.
    """
    dt = x1.dtype
    ls = np.asarray(lengthscale, dtype=dt)
    x1s = x1 / ls
    x2s = x2 / ls
    d = sq_dist(x1s, x2s, x1_eq_x2, zero_diag)
    return (np.asarray(outputscale, dtype=dt) * np.exp(d / dt.type(-2.0))).astype(dt)


# ---------------------------------------------------------------------------
# a7: psd_safe_cholesky (upstream linear_operator/utils/cholesky.py)
# ---------------------------------------------------------------------------
def _potrf_lower(a):
    """One LAPACK POTRF (lower) on a single matrix; returns (L, info)."""
    fn = lapack.spotrf if a.dtype == np.float32 else lapack.dpotrf
    c, info = fn(a, lower=1, clean=1, overwrite_a=0)
    if info != 0:
        c = np.tril(c)
    return c, int(info)


def cholesky_ex(A):
    """torch.linalg.cholesky_ex semantics over a batch: (L, info[b])."""
    A = np.asarray(A)
    batch = A.shape[:-2]
    n = A.shape[-1]
    flat = A.reshape(-1, n, n)
    try:
        L = np.linalg.cholesky(flat)
        info = np.zeros(flat.shape[0], dtype=np.int64)
        if not np.all(np.isfinite(L)):
            raise np.linalg.LinAlgError
    except np.linalg.LinAlgError:
        L = np.empty_like(flat)
        info = np.zeros(flat.shape[0], dtype=np.int64)
        for b in range(flat.shape[0]):
            if np.isnan(flat[b]).any():
                L[b] = np.nan
                info[b] = 1
                continue
            L[b], info[b] = _potrf_lower(flat[b])
    return L.reshape(*batch, n, n), info.reshape(batch)


@dataclass
class CholeskyResult:
    L: np.ndarray
    info: np.ndarray          # per window: 0 clean, -t after t jitter steps, k>0 failed
    jitter_steps: int         # number of global retries (warnings GPyTorch would emit)


def psd_safe_cholesky(A, jitter=None, max_tries=3, raise_on_fail=True):
    """linear_operator ``psd_safe_cholesky``: cholesky_ex, then a per-window jitter
    ladder ``jitter * 10**i`` (i < max_tries) applied only to failing windows,
    cumulatively via ``diag += jitter_new - jitter_prev`` in A's dtype.
    Default jitter: 1e-6 (fp32) / 1e-8 (fp64) (``settings.cholesky_jitter``).
    NaN input -> NanError; still failing after ``max_tries`` -> NotPSDError.
    """
    A = np.array(A, copy=True)
    L, info = cholesky_ex(A)
    win_info = np.zeros_like(info)
    if not np.any(info):
        return CholeskyResult(L, win_info, 0)
    if np.isnan(A).any():
        raise NanError(f"cholesky: {int(np.isnan(A).sum())} of {A.size} elements are NaN.")
    if jitter is None:
        jitter = 1e-6 if A.dtype == np.float32 else 1e-8
    dt = A.dtype.type
    jitter_prev = 0.0
    n = A.shape[-1]
    idx = np.arange(n)
    failing = info > 0
    steps = 0
    for i in range(max_tries):
        jitter_new = jitter * (10 ** i)
        add = dt(jitter_new - jitter_prev)
        sub = A[failing]
        sub[..., idx, idx] = sub[..., idx, idx] + add
        A[failing] = sub
        jitter_prev = jitter_new
        steps += 1
        warnings.warn(f"A not p.d., added jitter of {jitter_new:.1e} to the diagonal",
                      RuntimeWarning)
        Lf, infof = cholesky_ex(A[failing])
        L[failing] = Lf
        fidx = np.nonzero(failing)[0]
        win_info[fidx] = -(i + 1)
        still = infof > 0
        win_info[fidx[still]] = infof[still]
        failing_new = np.zeros_like(failing)
        failing_new[fidx[still]] = True
        failing = failing_new
        if not np.any(failing):
            return CholeskyResult(L, win_info, steps)
    if raise_on_fail:
        raise NotPSDError(
            f"Matrix not positive definite after repeatedly adding jitter up to {jitter_new:.1e}.")
    return CholeskyResult(L, win_info, steps)


# ---------------------------------------------------------------------------
# a1 + a3 + a4 + a6: exact GP marginal log likelihood
#   GPModel.py:5-13 (ConstantMean + ScaleKernel(RBFKernel())),
#   upstream mlls/exact_marginal_log_likelihood.py, distributions/multivariate_normal.py
#   (log_prob via inv_quad_logdet on K + sigma^2 I, Cholesky regime N <= 800)
# ---------------------------------------------------------------------------
@dataclass
class ExactMLLResult:
    L: np.ndarray        # (B, N, N) lower Cholesky factor of K + sigma^2 I (+ jitter)
    z: np.ndarray        # (B, N)   L^{-1} (y - c)
    mll: np.ndarray      # (B,)     log p(y) / N
    info: np.ndarray     # (B,)     0 / -t / k (see psd_safe_cholesky)
    K: np.ndarray        # (B, N, N) K + sigma^2 I (before jitter)


def exact_kernel_matrix(X, lengthscale, outputscale, noise, dtype=np.float64):
    """K_hat = s2 * RBF(X/l) + sigma^2 I, as ``likelihood(model(X))`` densifies it
    (GPModel.py:10-13; GaussianLikelihood marginal adds the noise diagonal)."""
    X = np.asarray(X, dtype=dtype)
    K = rbf(X, X, lengthscale, outputscale, x1_eq_x2=True, zero_diag=True)
    n = X.shape[-2]
    idx = np.arange(n)
    K[..., idx, idx] = K[..., idx, idx] + dtype(noise)
    return K


def exact_mll(X, y, lengthscale, outputscale, mean_constant, noise,
              dtype=np.float64, jitter=None, max_tries=3, raise_on_fail=True):
    """``ExactMarginalLogLikelihood(likelihood, ExactGPModel)(model(X), y)`` per window:
    ``-0.5 * (r^T K_hat^{-1} r + log|K_hat| + N log 2pi) / N`` with r = y - c,
    via L = psd_safe_cholesky(K_hat) (fp32 ladder for fp32 inputs)."""
    X = np.asarray(X, dtype=dtype)
    y = np.asarray(y, dtype=dtype)
    K = exact_kernel_matrix(X, lengthscale, outputscale, noise, dtype)
    res = psd_safe_cholesky(K, jitter=jitter, max_tries=max_tries, raise_on_fail=raise_on_fail)
    L = res.L
    r = y - dtype(mean_constant)
    z = _forward_solve(L, r)
    n = X.shape[-2]
    inv_quad = (z * z).sum(-1)
    logdet = 2.0 * np.log(np.diagonal(L, axis1=-2, axis2=-1)).sum(-1)
    mll = -0.5 * (inv_quad + logdet + n * LOG_2PI) / n
    return ExactMLLResult(L, z, mll.astype(dtype), res.info, K)


def _forward_solve(L, r):
    from scipy.linalg import solve_triangular
    L2 = L.reshape(-1, L.shape[-2], L.shape[-1])
    r2 = r.reshape(-1, r.shape[-1])
    out = np.empty_like(r2)
    for b in range(L2.shape[0]):
        out[b] = solve_triangular(L2[b], r2[b], lower=True, check_finite=False)
    return out.reshape(r.shape)


def exact_predict(X, y, Xs, lengthscale, outputscale, mean_constant, noise, dtype=np.float64):
    """ExactGP posterior (eval mode, GPModel.py:10-13 via upstream exact_prediction_strategies):
    mean = c + K_*^T K_hat^{-1} (y - c); var_f = s2 - || L^{-1} K_* ||^2 (latent f)."""
    X = np.asarray(X, dtype=dtype)
    Xs = np.asarray(Xs, dtype=dtype)
    y = np.asarray(y, dtype=dtype)
    res = exact_mll(X, y, lengthscale, outputscale, mean_constant, noise, dtype)
    Ks = rbf(X, Xs, lengthscale, outputscale)
    from scipy.linalg import solve_triangular
    B = X.shape[0]
    mean = np.empty(Xs.shape[:-1], dtype)
    var = np.empty(Xs.shape[:-1], dtype)
    for b in range(B):
        V = solve_triangular(res.L[b], Ks[b], lower=True)
        mean[b] = mean_constant + V.T @ res.z[b]
        var[b] = outputscale - (V * V).sum(0)
    return mean, var


# ---------------------------------------------------------------------------
# a8-a11, a14: variational (DeepGP) path
#   DeepGP.py:15-99; upstream variational/variational_strategy.py,
#   _variational_strategy.py, mean_field_variational_distribution.py,
#   models/deep_gps/deep_gp.py, likelihoods/gaussian_likelihood.py,
#   mlls/_approximate_mll.py, variational_elbo.py, deep_approximate_mll.py
# ---------------------------------------------------------------------------
@dataclass
class VariationalResult:
    mean: np.ndarray      # (B, N) predictive mean of q(f)
    var: np.ndarray       # (B, N) predictive variance of q(f), clamped >= min_var
    L_zz: np.ndarray      # (M, M) fp64 Cholesky of K_ZZ + jitter
    A: np.ndarray         # (B, M, N) L^{-1} K_ZX (fp64 solve, cast to input dtype)
    info: int


def variational_forward(X, Z, lengthscale, outputscale, weights, bias, m, s,
                        jitter=1e-4, dtype=np.float32, min_var=None, chol_jitter=None,
                        var_jitter=None):
    """``VariationalStrategy.forward`` (whitened) + ``LinearMean`` + MeanField q(u):

    K_ZZ + jitter (input dtype) -> fp64 -> L = psd_safe_cholesky (fp64 ladder);
    A = L^{-1} K_ZX (fp64) cast back; mean = A^T m + x w + b0;
    var = s2 + jitter + sum_m A_mi^2 (s_m^2 - 1), then MVN ``.variance`` clamp.
    Z is shared (M, D) — the reference expands it to (b, M, D), which changes
    nothing numerically (DeepGP.py:22, upstream ``_expand_inputs``).
    ``var_jitter`` (test hook) overrides the jitter added to K_XX's diagonal only, to
    drive the variance clamp in tests; None = ``jitter`` as GPyTorch.
    """
    X = np.asarray(X, dtype=dtype)
    Z = np.asarray(Z, dtype=dtype)
    ls = np.asarray(lengthscale, dtype=dtype).reshape(-1)
    Kzz = rbf(Z, Z, ls, outputscale, x1_eq_x2=True, zero_diag=False)
    Mi = np.arange(Z.shape[0])
    Kzz[Mi, Mi] = Kzz[Mi, Mi] + dtype(jitter)
    res = psd_safe_cholesky(Kzz.astype(np.float64), jitter=chol_jitter)
    L = res.L
    Kzx = rbf(np.broadcast_to(Z, X.shape[:-2] + Z.shape), X, ls, outputscale)
    from scipy.linalg import solve_triangular
    B = X.shape[0]
    A64 = np.empty(Kzx.shape, np.float64)
    for b in range(B):
        A64[b] = solve_triangular(L, Kzx[b].astype(np.float64), lower=True, check_finite=False)
    A = A64.astype(dtype)
    mvec = np.asarray(m, dtype=dtype)
    svec = np.asarray(s, dtype=dtype)
    w = np.asarray(weights, dtype=dtype).reshape(-1)
    mean = np.einsum('bmn,m->bn', A, mvec) + (X @ w) + dtype(bias)
    s2m1 = svec * svec - dtype(1.0)
    vj = jitter if var_jitter is None else var_jitter
    var = dtype(outputscale) + dtype(vj) + np.einsum('bmn,m->bn', A * A, s2m1)
    if min_var is None:
        min_var = 1e-6 if dtype == np.float32 else 1e-10
    var = np.maximum(var, dtype(min_var)).astype(dtype)
    return VariationalResult(mean.astype(dtype), var, L, A, int(res.jitter_steps))


def variational_covariance(X, Z, lengthscale, outputscale, s, jitter=1e-4, dtype=np.float64):
    """The full predictive covariance of q(f) that ``VariationalStrategy.forward`` (whitened)
    builds lazily (upstream variational_strategy.py: ``SumLinearOperator(data_data_covar
    .add_jitter(jitter), MatmulLinearOperator(interp_term^T, (S - I) interp_term))``):
    K_XX + jitter I + A^T diag(s^2 - 1) A per window, A = L^{-1} K_ZX from the fp64 factor.
    What ``MultivariateNormal.rsample`` / ``covariance_matrix`` of a DeepGP layer output
    (DeepGP.py:62-64 ``x.rsample()``) factor."""
    X = np.asarray(X, dtype=dtype)
    res = variational_forward(X, Z, lengthscale, outputscale, np.zeros(X.shape[-1]), 0.0,
                              np.zeros(np.asarray(Z).shape[0]), s, jitter=jitter, dtype=dtype)
    ls = np.asarray(lengthscale, dtype=dtype).reshape(-1)
    Kxx = np.stack([rbf(x, x, ls, outputscale, x1_eq_x2=True) for x in X])
    s2m1 = np.asarray(s, dtype=dtype) ** 2 - 1.0
    A = res.A
    N = X.shape[-2]
    return Kxx + dtype(jitter) * np.eye(N, dtype=dtype) + np.einsum('bmi,m,bmj->bij', A, s2m1, A)


def expected_log_prob(y, mean, var, noise):
    """GaussianLikelihood.expected_log_prob: -0.5 [((y-mu)^2 + v)/s2n + log s2n + log 2pi]."""
    return -0.5 * (((y - mean) ** 2 + var) / noise + np.log(noise) + LOG_2PI)


def kl_meanfield(m, s):
    """KL(N(m, diag s^2) || N(0, I)) (upstream distributions kl_mvn_mvn, whitened prior)."""
    m = np.asarray(m, np.float64)
    s2 = np.asarray(s, np.float64) ** 2
    return 0.5 * (s2.sum() + (m * m).sum() - m.size - np.log(s2).sum())


def deep_elbo(y, mean, var, noise, m, s, num_data, beta=1.0):
    """DeepApproximateMLL(VariationalELBO(lik, model, num_data))(dist, y) for S=1:
    per window ELBO_b = sum_i ELL_bi / N - KL / (num_data / beta)
    (forecast_denoising.py:86-89; num_data = d_model there)."""
    n = mean.shape[-1]
    ell = expected_log_prob(np.asarray(y, np.float64), np.asarray(mean, np.float64),
                            np.asarray(var, np.float64), float(noise)).sum(-1) / n
    return ell - kl_meanfield(m, s) / (num_data / beta)


# ---------------------------------------------------------------------------
# Torch-CPU restatement of the same exact-MLL path. GPyTorch itself dispatches
# to exactly these torch CPU kernels (MKL/LAPACK): the _sq_dist GEMM form,
# torch.linalg.cholesky_ex (+ the jitter ladder), torch.cholesky_solve for the
# inverse quadratic (linear_operator CholLinearOperator.inv_quad_logdet) and
# _chol_diag.pow(2).log().sum() for the log-determinant. Used as the timed CPU
# baseline ("port") in bench.py and cross-checked against the NumPy oracle in
# tests/test_oracle.py. CPU only.
# ---------------------------------------------------------------------------
def exact_mll_torch_cpu(X, y, lengthscale, outputscale, mean_constant, noise,
                        jitter=1e-6, max_tries=3):
    import torch
    X = torch.as_tensor(X)
    y = torch.as_tensor(y)
    assert X.device.type == "cpu"
    ls = torch.as_tensor(lengthscale, dtype=X.dtype)
    x = X / ls
    adj = x.mean(-2, keepdim=True)
    x1 = x - adj
    n1 = x1.pow(2).sum(-1, keepdim=True)
    ones = torch.ones_like(n1)
    res = torch.cat([-2.0 * x1, n1, ones], -1) @ torch.cat([x1, ones, n1], -1).transpose(-1, -2)
    res.diagonal(dim1=-2, dim2=-1).fill_(0)
    res.clamp_min_(0)
    K = res.div_(-2).exp_().mul_(outputscale)
    K.diagonal(dim1=-2, dim2=-1).add_(noise)
    L, info = torch.linalg.cholesky_ex(K)
    if bool(torch.any(info)):
        Kp = K.clone()
        prev = 0.0
        for i in range(max_tries):
            new = jitter * (10 ** i)
            Kp.diagonal(dim1=-2, dim2=-1).add_(((info > 0).to(K.dtype) * (new - prev)).unsqueeze(-1))
            prev = new
            L, info = torch.linalg.cholesky_ex(Kp)
            if not bool(torch.any(info)):
                break
        else:
            raise NotPSDError("Matrix not positive definite after repeatedly adding jitter")
    r = (y - mean_constant).unsqueeze(-1)
    sol = torch.cholesky_solve(r, L)
    inv_quad = (r * sol).sum((-1, -2))
    logdet = L.diagonal(dim1=-2, dim2=-1).pow(2).log().sum(-1)
    n = X.shape[-2]
    return L, -0.5 * (inv_quad + logdet + n * LOG_2PI) / n


# ---------------------------------------------------------------------------
# Gradients of the hot path (what torch autograd produces when train.py:166
# back-propagates through GPyTorch). Restated in torch fp64 autograd on the CPU
# with direct-difference distances (mathematically identical to the centred GEMM
# form away from the clamp); pinned against central finite differences of the
# NumPy forward above (tests/test_oracle.py). TEST INFRASTRUCTURE ONLY.
# ---------------------------------------------------------------------------
def _t64(a, grad=True):
    import torch
    return torch.tensor(np.array(a, dtype=np.float64), requires_grad=grad)


def _rbf_t(a, b, ls, s2):
    import torch
    d = (((a.unsqueeze(-2) - b.unsqueeze(-3)) / ls) ** 2).sum(-1)
    return s2 * torch.exp(-0.5 * d)


def variational_grads(X, Z, lengthscale, outputscale, weights, bias, m, s, gmean, gvar,
                      jitter=1e-4, min_var=1e-6, var_jitter=None):
    """d/dtheta of sum(gmean * mean) + sum(gvar * var) for ``variational_forward``
    (DeepGP.py:51-99 via VariationalStrategy: K_ZZ + jitter -> fp64 Cholesky,
    A = L^{-1} K_ZX, mean = A^T m + x w + b0, var = s2 + jitter + sum A^2 (s^2-1)
    clamped at min_var). Returns a dict of float64 arrays: X, Z, m, s, outputscale,
    lengthscale (D,), weights (D,), bias."""
    import torch
    X = np.asarray(X, np.float64)
    B, N, D = X.shape
    M = np.asarray(Z).shape[0]
    Xt, Zt, mt, st = _t64(X), _t64(Z), _t64(m), _t64(s)
    wt = _t64(np.reshape(weights, -1))
    s2t, b0t = _t64(float(outputscale)), _t64(float(bias))
    lst = _t64(np.broadcast_to(np.asarray(lengthscale, np.float64).reshape(-1), (D,)))
    Kzz = _rbf_t(Zt, Zt, lst, s2t) + jitter * torch.eye(M, dtype=torch.float64)
    L = torch.linalg.cholesky(Kzz)
    Kzx = _rbf_t(Zt.expand(B, M, D), Xt, lst, s2t)
    A = torch.linalg.solve_triangular(L, Kzx, upper=False)
    mean = (A * mt[:, None]).sum(-2) + Xt @ wt + b0t
    vj = jitter if var_jitter is None else var_jitter
    var = (s2t + vj + (A * A * (st * st - 1.0)[:, None]).sum(-2)).clamp_min(min_var)
    obj = (torch.as_tensor(np.asarray(gmean, np.float64)) * mean).sum() + \
          (torch.as_tensor(np.asarray(gvar, np.float64)) * var).sum()
    names = ["X", "Z", "m", "s", "outputscale", "lengthscale", "weights", "bias"]
    gs = torch.autograd.grad(obj, [Xt, Zt, mt, st, s2t, lst, wt, b0t])
    return {k: v.detach().numpy() for k, v in zip(names, gs)}


def exact_mll_grads(X, y, lengthscale, outputscale, mean_constant, noise, gout=None):
    """d/dtheta of sum_b gout_b * mll_b for ``exact_mll`` (GPModel.py:5-13 +
    ExactMarginalLogLikelihood): grads w.r.t. X, y, lengthscale (scalar or (D,)),
    outputscale, mean_constant, noise. float64 arrays."""
    import torch
    X = np.asarray(X, np.float64)
    B, N, D = X.shape
    ls_in = np.asarray(lengthscale, np.float64).reshape(-1)
    Xt, yt, lst = _t64(X), _t64(y), _t64(ls_in)
    s2t, ct, nzt = _t64(float(outputscale)), _t64(float(mean_constant)), _t64(float(noise))
    K = _rbf_t(Xt, Xt, lst, s2t) + nzt * torch.eye(N, dtype=torch.float64)
    L = torch.linalg.cholesky(K)
    r = (yt - ct).unsqueeze(-1)
    z = torch.linalg.solve_triangular(L, r, upper=False).squeeze(-1)
    logdet = 2.0 * torch.log(torch.diagonal(L, dim1=-2, dim2=-1)).sum(-1)
    mll = -0.5 * ((z * z).sum(-1) + logdet + N * LOG_2PI) / N
    g = torch.ones(B, dtype=torch.float64) if gout is None else torch.as_tensor(np.asarray(gout, np.float64))
    gs = torch.autograd.grad((g * mll).sum(), [Xt, yt, lst, s2t, ct, nzt])
    names = ["X", "y", "lengthscale", "outputscale", "mean_constant", "noise"]
    return {k: v.detach().numpy() for k, v in zip(names, gs)}


def variational_forward_torch_cpu(X, Z, lengthscale, outputscale, weights, bias, m, s, jitter=1e-4):
    """Torch-CPU restatement of what GPyTorch dispatches for VariationalStrategy.forward
    (DeepGP.py:51-73): Z expanded to the batch, K over cat[Z, x] in the
    centred _sq_dist GEMM form, K_ZZ + jitter -> .double() -> torch.linalg.cholesky_ex
    ONCE PER WINDOW (the reference's b-fold redundant factorisation), fp64
    solve_triangular for A = L^-1 K_ZX, cast to fp32, mean = A^T m + x w + b0,
    var = s2 + jitter + sum A^2 (s^2 - 1) clamped. Used as the timed CPU baseline of the
    variational path in bench.py (CPU only)."""
    import torch
    X = torch.as_tensor(X)
    Z = torch.as_tensor(Z)
    B, N, D = X.shape
    M = Z.shape[0]
    ls = torch.as_tensor(lengthscale, dtype=X.dtype).reshape(-1)
    full = torch.cat([Z.expand(B, M, D), X], -2) / ls
    adj = full[..., :M, :].mean(-2, keepdim=True)

    def sqd(a, b):
        a = a - adj
        b = b - adj
        an = a.pow(2).sum(-1, keepdim=True)
        bn = b.pow(2).sum(-1, keepdim=True)
        return (torch.cat([-2.0 * a, an, torch.ones_like(an)], -1)
                @ torch.cat([b, torch.ones_like(bn), bn], -1).transpose(-1, -2)).clamp_min_(0)
    zz = full[..., :M, :]
    Kzz = sqd(zz, zz).div_(-2).exp_().mul_(outputscale)
    Kzz.diagonal(dim1=-2, dim2=-1).add_(jitter)
    Kzx = sqd(zz, full[..., M:, :]).div_(-2).exp_().mul_(outputscale)
    L, info = torch.linalg.cholesky_ex(Kzz.double())
    A = torch.linalg.solve_triangular(L, Kzx.double(), upper=False).to(X.dtype)
    mvec = torch.as_tensor(m, dtype=X.dtype)
    svec = torch.as_tensor(s, dtype=X.dtype)
    mean = (A.transpose(-1, -2) @ mvec.unsqueeze(-1)).squeeze(-1) + X @ torch.as_tensor(weights, dtype=X.dtype).reshape(-1) + bias
    var = (outputscale + jitter + ((A * A) * (svec * svec - 1.0).unsqueeze(-1)).sum(-2)).clamp_min(1e-6)
    return mean, var
