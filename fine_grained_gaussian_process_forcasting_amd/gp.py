"""gpytorch-free building blocks of the reference GP path, backed by the gfx950 kernels.

Mirrors the GPyTorch 1.9.x objects the reference touches with
the same module / parameter names, so the reference's call sites
(denoising_model/DeepGP.py, GPModel.py, denoise_model_2.py, forecast_denoising.py:86-89,
train.py:20) read the same and its state_dicts keep their keys:

  settings.num_likelihood_samples        gpytorch.settings.num_likelihood_samples
  Positive / GreaterThan                 gpytorch.constraints (softplus transform)
  RBFKernel / ScaleKernel                gpytorch.kernels (raw_lengthscale, raw_outputscale)
  ConstantMean / LinearMean              gpytorch.means
  GaussianLikelihood                     gpytorch.likelihoods (noise_covar.raw_noise)
  MultivariateNormal                     gpytorch.distributions (mean, variance clamp)
  MeanFieldVariationalDistribution       gpytorch.variational
  VariationalStrategy                    gpytorch.variational (whitened)
  VariationalELBO / DeepApproximateMLL   gpytorch.mlls
  ExactMarginalLogLikelihood             gpytorch.mlls

All arithmetic of the hot path runs in libgpk.so (ops.py); torch is used for
parameters, the tiny constrained-value transforms and elementwise glue on the
device. Gradients: see ops_autograd.py.
"""
from __future__ import annotations

import contextlib
import math
import threading
import warnings
from typing import Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import ops
from .errors import NumericalWarning

LOG_2PI = math.log(2.0 * math.pi)


# ---------------------------------------------------------------------------
# settings (upstream gpytorch/settings.py)
# ---------------------------------------------------------------------------
class _Setting:
    """One process-wide value, like GPyTorch's ``_value_context``: entering the context
    stores the value once for the whole process (``_global_value`` is a class
    attribute there), so a value set on the main thread (train.py:20) is what the
    Optuna worker threads (train.py:86, n_jobs=4) read. Exit restores the value that
    was current on entry."""

    _lock = threading.Lock()
    _UNSET = object()

    def __init__(self, default):
        self._default = default
        self._value = self._UNSET

    def value(self, dtype=None):
        v = self._value
        if v is not self._UNSET:
            return v
        if isinstance(self._default, dict):
            return self._default.get(dtype, self._default.get(None))
        return self._default

    @contextlib.contextmanager
    def __call__(self, value):
        with self._lock:
            prev = self._value
            self._value = value
        try:
            yield
        finally:
            with self._lock:
                self._value = prev


class settings:
    """The gpytorch.settings used on this path (process-global like GPyTorch's)."""
    num_likelihood_samples = _Setting(10)          # train.py:20 sets 1
    cholesky_jitter = _Setting({torch.float32: 1e-6, torch.float64: 1e-8, None: 1e-6})
    cholesky_max_tries = _Setting(3)
    variational_cholesky_jitter = _Setting({torch.float32: 1e-4, torch.float64: 1e-6, None: 1e-4})
    min_variance = _Setting({torch.float32: 1e-6, torch.float64: 1e-10, None: 1e-6})
    max_cholesky_size = _Setting(800)


# ---------------------------------------------------------------------------
# constraints (upstream constraints/constraints.py)
# ---------------------------------------------------------------------------
class Interval(nn.Module):
    def __init__(self, lower_bound, upper_bound):
        super().__init__()
        self.register_buffer("lower_bound", torch.as_tensor(float(lower_bound)))
        self.register_buffer("upper_bound", torch.as_tensor(float(upper_bound)))

    def transform(self, raw):
        return F.softplus(raw) + self.lower_bound.to(raw.dtype)

    def inverse_transform(self, value):
        v = torch.as_tensor(value) - self.lower_bound
        return torch.where(v > 20, v, torch.log(torch.expm1(v)))


class Positive(Interval):
    def __init__(self):
        super().__init__(0.0, math.inf)


class GreaterThan(Interval):
    def __init__(self, lower_bound):
        super().__init__(lower_bound, math.inf)


# ---------------------------------------------------------------------------
# kernels / means (upstream kernels/rbf_kernel.py, scale_kernel.py, means/*)
# ---------------------------------------------------------------------------
class RBFKernel(nn.Module):
    """Lengthscale holder of gpytorch.kernels.RBFKernel; shape (*batch, 1, ard or 1)."""

    def __init__(self, ard_num_dims: Optional[int] = None, batch_shape=torch.Size([])):
        super().__init__()
        self.ard_num_dims = ard_num_dims
        n = 1 if ard_num_dims is None else ard_num_dims
        self.register_parameter("raw_lengthscale", nn.Parameter(torch.zeros(*batch_shape, 1, n)))
        self.register_module("raw_lengthscale_constraint", Positive())

    @property
    def lengthscale(self):
        return self.raw_lengthscale_constraint.transform(self.raw_lengthscale)


class ScaleKernel(nn.Module):
    def __init__(self, base_kernel: RBFKernel, batch_shape=torch.Size([]), ard_num_dims=None):
        super().__init__()
        self.base_kernel = base_kernel
        self.register_parameter("raw_outputscale", nn.Parameter(torch.zeros(torch.Size(batch_shape))))
        self.register_module("raw_outputscale_constraint", Positive())

    @property
    def outputscale(self):
        return self.raw_outputscale_constraint.transform(self.raw_outputscale)


class ConstantMean(nn.Module):
    def __init__(self, batch_shape=torch.Size([])):
        super().__init__()
        self.register_parameter("constant", nn.Parameter(torch.zeros(*batch_shape, 1)))

    def forward(self, x):
        return self.constant.expand(*x.shape[:-1])


class LinearMean(nn.Module):
    def __init__(self, input_size: int, batch_shape=torch.Size([]), bias: bool = True):
        super().__init__()
        self.register_parameter("weights", nn.Parameter(torch.randn(*batch_shape, input_size, 1)))
        if bias:
            self.register_parameter("bias", nn.Parameter(torch.randn(*batch_shape, 1)))
        else:
            self.bias = None

    def forward(self, x):
        res = x.matmul(self.weights).squeeze(-1)
        return res + self.bias if self.bias is not None else res


# ---------------------------------------------------------------------------
# distributions (upstream distributions/multivariate_normal.py)
# ---------------------------------------------------------------------------
def warn_if_clamped(flag: torch.Tensor, min_var: float) -> None:
    """GPyTorch's NumericalWarning when the variational kernel clamped a variance."""
    if int(flag.item()) & 1:
        warnings.warn(f"Negative variance values detected. This is likely due to numerical "
                      f"instabilities. Rounding negative variances up to {min_var}.",
                      NumericalWarning)


class MultivariateNormal:
    """Diagonal-query MVN of the hot path.

    Holds what the reference reads from the GP output: ``mean`` and the marginal
    ``variance`` (clamped at settings.min_variance with GPyTorch's
    NumericalWarning), batch_shape / event_shape semantics and ``expand``. Exact-GP
    priors also carry the window inputs so ``log_prob`` can run the fused kernel.
    """

    def __init__(self, mean: torch.Tensor, variance: Optional[torch.Tensor] = None,
                 exact=None, added_noise=None, clamp_flag: Optional[torch.Tensor] = None,
                 preclamped: bool = False, covar_fn=None):
        self._mean = mean
        self._variance = variance
        self._exact = exact                # (X, kernel hyper) for exact-GP priors
        self._added_noise = added_noise    # likelihood noise folded in by GaussianLikelihood
        self._clamp_flag = clamp_flag      # (1,) int32 from gpk_variational_f32: clamp fired
        self._preclamped = preclamped      # variance already clamped by the kernel, no flag
        # () -> dense (..., N, N) covariance of a variational output (its lazy covariance, as
        # GPyTorch's VariationalStrategy builds it); materialised only by covariance_matrix /
        # rsample, never on the hot path
        self._covar_fn = covar_fn

    @property
    def mean(self):
        return self._mean

    @property
    def loc(self):
        return self._mean

    @property
    def batch_shape(self):
        return self._mean.shape[:-1]

    @property
    def event_shape(self):
        return self._mean.shape[-1:]

    @property
    def variance(self):
        if self._variance is None:
            if self._exact is None:
                raise NotImplementedError("this distribution carries no variance")
            # exact-GP prior: diag K(x, x) = outputscale (the RBF is 1 on the diagonal), as
            # GPyTorch's lazy kernel diagonal returns it
            var = self._exact[2].reshape(()).expand(self._mean.shape)
        else:
            var = self._variance
        if self._added_noise is not None:
            var = var + self._added_noise
        min_var = settings.min_variance.value(var.dtype)
        if self._preclamped and self._added_noise is None:
            # a point slice of a kernel output: a clamped entry is exactly min_var
            from .ops import record_or_run
            flag = (var <= min_var).any().to(torch.int32).reshape(1)
            record_or_run("clamp", (flag, min_var), lambda: warn_if_clamped(flag, min_var))
            return var
        if self._clamp_flag is not None and self._added_noise is None:
            # the kernel already clamped (fp32 min_variance); it tells us whether it did:
            # one host read of the flag, as GPyTorch's own .lt(min_var).any() sync
            # (recorded instead while a HIP graph is captured, ops.DeferredChecks)
            from .ops import record_or_run
            flag = self._clamp_flag
            record_or_run("clamp", (flag, min_var), lambda: warn_if_clamped(flag, min_var))
            return var
        if bool((var < min_var).any()):
            warnings.warn(f"Negative variance values detected. This is likely due to numerical "
                          f"instabilities. Rounding negative variances up to {min_var}.",
                          NumericalWarning)
            var = var.clamp_min(min_var)
        return var

    @property
    def stddev(self):
        return self.variance.sqrt()

    @property
    def covariance_matrix(self):
        """Dense prior covariance of an exact-GP / layer prior, materialised on request
        (GPyTorch keeps covar_module(x) lazy and evaluates it here): outputscale * RBF with
        upstream ``_sq_dist`` semantics (inputs centred by their mean, clamp at 0, exact 0 on
        the diagonal) + the added likelihood noise on the diagonal. Not on the hot path: no
        reference caller reads it. Variational outputs are diagonal-query (their marginals
        are what the reference reads) and do not carry a covariance."""
        if self._exact is None and self._covar_fn is None:
            raise NotImplementedError("covariance_matrix is provided for exact-GP / layer priors and "
                                      "variational outputs")
        if self._exact is not None:
            X, lengthscale, outputscale, _ = self._exact
            K = rbf_covariance(X, lengthscale, outputscale)
        else:
            K = self._covar_fn()
        if self._added_noise is not None:
            K = K + torch.diag_embed(torch.as_tensor(self._added_noise, dtype=K.dtype, device=K.device)
                                     .expand(K.shape[:-1]))
        n = self._mean.shape[-1]
        if K.numel() != self._mean.numel() * n:   # an expanded distribution: its batch is a view
            K = K.expand(*self._mean.shape, n)
        return K.reshape(*self._mean.shape, n)

    @property
    def lazy_covariance_matrix(self):
        return self.covariance_matrix

    def rsample(self, sample_shape=torch.Size(), base_samples: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Reparameterised sample mean + chol(Sigma) eps (upstream MultivariateNormal.rsample: the
        covariance root by psd_safe_cholesky with the jitter ladder). Off the hot path: the dense
        covariance is materialised (covariance_matrix)."""
        cov = self.covariance_matrix
        root = psd_safe_cholesky(cov)
        shape = torch.Size(sample_shape) + self._mean.shape
        if base_samples is None:
            base_samples = torch.randn(shape, dtype=self._mean.dtype, device=self._mean.device)
        elif base_samples.shape != shape:
            raise RuntimeError(f"base_samples shape {tuple(base_samples.shape)} != {tuple(shape)}")
        return self._mean + (root @ base_samples.unsqueeze(-1)).squeeze(-1)

    def sample(self, sample_shape=torch.Size(), base_samples: Optional[torch.Tensor] = None) -> torch.Tensor:
        with torch.no_grad():
            return self.rsample(sample_shape, base_samples)

    def expand(self, batch_size):
        batch_size = torch.Size(batch_size)
        mean = self._mean.expand(*batch_size, *self.event_shape)
        var = self._variance.expand(*batch_size, *self.event_shape) if self._variance is not None else None
        exact = self._exact
        if exact is not None:
            # the prior's inputs follow the mean's batch, so covariance_matrix / log_prob of the
            # expanded distribution see one input set per batch entry (GPyTorch expands the lazy
            # kernel tensor the same way)
            X = exact[0]
            n, d = X.shape[-2:]
            if X.numel() != self.batch_shape.numel() * n * d:
                raise NotImplementedError("expand of an exact prior whose inputs do not follow its batch")
            Xe = X.reshape(*self.batch_shape, n, d).expand(*batch_size, n, d).reshape(-1, n, d)
            exact = (Xe,) + tuple(exact[1:])
        return MultivariateNormal(mean, var, exact, self._added_noise, self._clamp_flag,
                                  self._preclamped, self._covar_fn)

    def add_noise(self, noise):
        total = noise if self._added_noise is None else self._added_noise + noise
        return MultivariateNormal(self._mean, self._variance, self._exact, total, self._clamp_flag,
                                  self._preclamped, self._covar_fn)

    def slice_points(self, start, stop):
        """The marginals of points [start, stop) (diagonal-query outputs of the variational
        path only): the clamp warning then reflects exactly the sliced points."""
        if self._exact is not None or self._variance is None:
            raise NotImplementedError("point slices are defined for variational outputs")
        sl = (Ellipsis, slice(start, stop))
        cf = self._covar_fn
        sub = (lambda: cf()[..., start:stop, start:stop]) if cf is not None else None
        return MultivariateNormal(self._mean[sl], self._variance[sl], None, self._added_noise, None,
                                  preclamped=self._clamp_flag is not None or self._preclamped, covar_fn=sub)

    def log_prob(self, value: torch.Tensor) -> torch.Tensor:
        """Exact-GP marginal log density (fused RBF + Cholesky + solve + logdet kernel)."""
        if self._exact is None:
            raise NotImplementedError("log_prob is provided for exact-GP outputs (GPModel.py)")
        X, lengthscale, outputscale, constant = self._exact
        noise = self._added_noise if self._added_noise is not None else torch.zeros((), device=X.device)
        from .ops_autograd import exact_log_prob
        n = X.shape[-2]
        target = value.reshape(X.shape[:-1])
        if constant is None:
            # a general (e.g. LinearMean) prior mean: the fused kernel's constant mean is 0 and
            # the residual value - mean(x) is its target (the same MVN density)
            target = target - self._mean.reshape(X.shape[:-1])
            constant = torch.zeros((), device=X.device)
        res = exact_log_prob(X, target, lengthscale, outputscale, constant, noise) * n
        return res.reshape(value.shape[:-1])      # (N,) targets of an unbatched model -> scalar


def rbf_covariance(X: torch.Tensor, lengthscale, outputscale) -> torch.Tensor:
    """outputscale * exp(-||x_i - x_j||^2 / (2 l^2)) for X (B, N, D), as GPyTorch's
    ScaleKernel(RBFKernel) evaluates a lazy kernel tensor (upstream kernels/rbf_kernel.py,
    kernel.py ``_sq_dist``: inputs divided by the lengthscale and centred by their mean,
    ||a||^2 + ||b||^2 - 2 a.b clamped at 0, the x1 == x2 diagonal set to exactly 0)."""
    ls = torch.as_tensor(lengthscale, device=X.device, dtype=X.dtype).reshape(-1)
    xs = X / ls
    xs = xs - xs.mean(-2, keepdim=True)
    nrm = xs.pow(2).sum(-1)
    d = (nrm.unsqueeze(-1) + nrm.unsqueeze(-2) - 2.0 * xs @ xs.transpose(-1, -2)).clamp_min(0.0)
    d = d * (1.0 - torch.eye(X.shape[-2], device=X.device, dtype=X.dtype))
    s2 = torch.as_tensor(outputscale, device=X.device, dtype=X.dtype).reshape(())
    return s2 * torch.exp(-0.5 * d)


def psd_safe_cholesky(A: torch.Tensor, max_tries: Optional[int] = None) -> torch.Tensor:
    """Upstream linear_operator utils/cholesky.py psd_safe_cholesky for a dense matrix (the
    covariance roots of rsample; the hot path's factorisations run in the gfx950 kernels):
    torch.linalg.cholesky_ex, then up to max_tries retries with jitter 1e-6, 1e-5, ... (fp32;
    1e-8.. for fp64) added to the diagonal, each retry warning NumericalWarning."""
    L, info = torch.linalg.cholesky_ex(A)
    if not bool((info > 0).any()):
        return L
    if torch.isnan(A).any():
        from .errors import NanError
        raise NanError(f"cholesky_cpu: {torch.isnan(A).sum().item()} of {A.numel()} elements of the "
                       f"{tuple(A.shape)} tensor are NaN.")
    jitter = settings.cholesky_jitter.value(A.dtype)
    tries = settings.cholesky_max_tries.value() if max_tries is None else max_tries
    Aprime = A.clone()
    jitter_prev = 0.0
    for i in range(tries):
        jitter_new = jitter * (10 ** i)
        Aprime.diagonal(dim1=-2, dim2=-1).add_(jitter_new - jitter_prev)
        jitter_prev = jitter_new
        warnings.warn(f"A not p.d., added jitter of {jitter_new:.1e} to the diagonal", NumericalWarning)
        L, info = torch.linalg.cholesky_ex(Aprime)
        if not bool((info > 0).any()):
            return L
    from .errors import NotPSDError
    raise NotPSDError(f"Matrix not positive definite after repeatedly adding jitter up to {jitter_new:.1e}.")


class MultitaskMultivariateNormal:
    """Upstream distributions/multitask_multivariate_normal.py as a multi-output DeepGP layer
    returns it (DeepGPLayer.__call__: ``MultitaskMultivariateNormal(output.loc.transpose(-1, -2),
    BlockDiagLinearOperator(output.lazy_covariance_matrix, block_dim=-3), interleaved=False)``):
    a batch of O independent per-output MultivariateNormals (batch (..., O), event N) viewed with
    event shape (N, O). mean / variance are the per-output marginals transposed; the dense
    covariance is block diagonal in task-major (non-interleaved) order; rsample draws every
    output from its own full covariance."""

    def __init__(self, base: MultivariateNormal):
        self._base = base      # batch (..., O), event N

    @classmethod
    def from_batch_mvn(cls, batch_mvn: MultivariateNormal, task_dim: int = -1):
        if task_dim not in (-1, batch_mvn._mean.dim() - 2):
            raise NotImplementedError("the task dimension is the last batch dimension")
        return cls(batch_mvn)

    @property
    def num_tasks(self):
        return self._base.mean.shape[-2]

    @property
    def mean(self):
        return self._base.mean.transpose(-1, -2)

    @property
    def loc(self):
        return self.mean

    @property
    def variance(self):
        return self._base.variance.transpose(-1, -2)

    @property
    def stddev(self):
        return self.variance.sqrt()

    @property
    def batch_shape(self):
        return self._base.mean.shape[:-2]

    @property
    def event_shape(self):
        return self.mean.shape[-2:]

    @property
    def covariance_matrix(self):
        blocks = self._base.covariance_matrix          # (..., O, N, N)
        return torch.block_diag(*blocks.unbind(-3)) if blocks.dim() == 3 else \
            torch.stack([torch.block_diag(*b.unbind(-3)) for b in blocks.reshape(-1, *blocks.shape[-3:])]) \
            .reshape(*blocks.shape[:-3], blocks.shape[-3] * blocks.shape[-1], blocks.shape[-3] * blocks.shape[-1])

    @property
    def lazy_covariance_matrix(self):
        return self.covariance_matrix

    def expand(self, batch_size):
        return MultitaskMultivariateNormal(self._base.expand(torch.Size(batch_size) + self._base.mean.shape[-2:-1]))

    def add_noise(self, noise):
        return MultitaskMultivariateNormal(self._base.add_noise(noise))

    def rsample(self, sample_shape=torch.Size(), base_samples: Optional[torch.Tensor] = None) -> torch.Tensor:
        if base_samples is not None:
            base_samples = base_samples.transpose(-1, -2)
        return self._base.rsample(sample_shape, base_samples).transpose(-1, -2)

    def sample(self, sample_shape=torch.Size(), base_samples: Optional[torch.Tensor] = None) -> torch.Tensor:
        with torch.no_grad():
            return self.rsample(sample_shape, base_samples)


# ---------------------------------------------------------------------------
# likelihood (upstream likelihoods/gaussian_likelihood.py, noise_models.py)
# ---------------------------------------------------------------------------
class HomoskedasticNoise(nn.Module):
    def __init__(self, batch_shape=torch.Size([])):
        super().__init__()
        self.register_parameter("raw_noise", nn.Parameter(torch.zeros(*batch_shape, 1)))
        self.register_module("raw_noise_constraint", GreaterThan(1e-4))

    @property
    def noise(self):
        return self.raw_noise_constraint.transform(self.raw_noise)


class GaussianLikelihood(nn.Module):
    def __init__(self, batch_shape=torch.Size([])):
        super().__init__()
        self.noise_covar = HomoskedasticNoise(batch_shape)

    @property
    def noise(self):
        return self.noise_covar.noise

    def forward(self, function_dist: MultivariateNormal) -> MultivariateNormal:
        """Marginal p(y) = q(f) + noise (only the diagonal is ever read on this path)."""
        return function_dist.add_noise(self.noise.reshape(()))

    def expected_log_prob(self, target: torch.Tensor, input: MultivariateNormal) -> torch.Tensor:
        mean, variance = input.mean, input.variance
        noise = self.noise.reshape(())
        res = ((target - mean) ** 2 + variance) / noise + noise.log() + LOG_2PI
        return res.mul(-0.5)

    def expected_log_prob_sum(self, target: torch.Tensor, input: MultivariateNormal) -> torch.Tensor:
        """expected_log_prob(target, input).sum(-1) -- what VariationalELBO reads -- as ONE
        gfx950 launch forward and one backward (gpk::gauss_ell) instead of ~10 elementwise
        kernels each way; the per-point form above stays GPyTorch's API."""
        mean, variance = input.mean, input.variance
        if not (mean.is_cuda and mean.dtype == torch.float32 and variance.shape == mean.shape
                and self.noise.numel() == 1):
            # (a batched noise model has one noise per batch entry: the unfused expression)
            return self.expected_log_prob(target, input).sum(-1)
        shape = mean.shape
        N = shape[-1]
        y = torch.broadcast_to(target, shape).to(torch.float32)
        ell = torch.ops.gpk.gauss_ell(y.reshape(-1, N), mean.reshape(-1, N), variance.reshape(-1, N),
                                      self.noise.reshape(1))
        return ell.reshape(shape[:-1])


# ---------------------------------------------------------------------------
# variational distribution / strategy (upstream variational/*.py, whitened)
# ---------------------------------------------------------------------------
class MeanFieldVariationalDistribution(nn.Module):
    def __init__(self, num_inducing_points: int, batch_shape=torch.Size([]), mean_init_std=1e-3):
        super().__init__()
        self.num_inducing_points = num_inducing_points
        self.mean_init_std = mean_init_std
        self.register_parameter("variational_mean", nn.Parameter(torch.zeros(*batch_shape, num_inducing_points)))
        self.register_parameter("_variational_stddev", nn.Parameter(torch.ones(*batch_shape, num_inducing_points)))

    def initialize_variational_distribution(self):
        # prior N(0, I) (whitened): m = 0 + mean_init_std * randn, stddev = 1
        with torch.no_grad():
            self.variational_mean.data.zero_()
            self.variational_mean.data.add_(torch.randn_like(self.variational_mean), alpha=self.mean_init_std)
            self._variational_stddev.data.fill_(1.0)

    def kl_divergence(self) -> torch.Tensor:
        """KL(N(m, diag s^2) || N(0, I)) = 1/2 (sum s^2 + sum m^2 - M - sum log s^2)
        (one gfx950 launch each way, gpk::meanfield_kl, for the unbatched fp32 layer)."""
        m = self.variational_mean
        s = self._variational_stddev
        if m.is_cuda and m.dim() == 1 and m.dtype == torch.float32:
            return torch.ops.gpk.meanfield_kl(m, s).reshape(())
        s2 = s.pow(2)
        return 0.5 * (s2.sum(-1) + m.pow(2).sum(-1) - m.shape[-1] - s2.log().sum(-1))


class _MeanOutput:
    """Output o's view of a layer mean (DeepGP.py:42-45): ConstantMean(batch_shape=[O]) has one
    constant per output, the reference's LinearMean(input_dims) one weight vector for all."""

    def __init__(self, mean_module, o):
        if hasattr(mean_module, "weights"):
            w = mean_module.weights
            self.weights = w[o] if w.dim() == 3 else w
            b = mean_module.bias
            self.bias = (b[o] if b.dim() == 2 else b) if b is not None else None
        elif hasattr(mean_module, "constant"):
            c = mean_module.constant
            self.constant = c[o] if c.dim() == 2 else c
        else:
            raise NotImplementedError(f"mean module {type(mean_module).__name__}")


def variational_dense_covariance(x, Z, Linv, vstd, outputscale, lengthscale, jitter):
    """The full predictive covariance of q(f) at x (B', N, D), as upstream
    VariationalStrategy.forward (whitened) builds it lazily: K_XX + jitter I + A^T (S - I) A with
    A = L^{-1} K_ZX solved in fp64 and cast back (``L.solve(induc_data_covar.double())``),
    S = diag(stddev^2). Dense torch arithmetic on request (covariance_matrix / rsample) -- the
    hot path reads the marginals from the kernels and never calls this."""
    ls = lengthscale.reshape(-1)
    s2 = outputscale.reshape(())
    Kxx = rbf_covariance(x, ls, s2)
    zs = (Z / ls).double()
    xs = (x / ls).double()
    d = (zs.pow(2).sum(-1)[:, None] + xs.pow(2).sum(-1).unsqueeze(-2)
         - 2.0 * zs @ xs.transpose(-1, -2)).clamp_min(0.0)             # (B', M, N)
    Kzx = s2.double() * torch.exp(-0.5 * d)
    A = (Linv.double() @ Kzx).to(x.dtype)
    mid = (vstd.reshape(-1).pow(2) - 1.0).to(x.dtype)
    eye = torch.eye(x.shape[-2], dtype=x.dtype, device=x.device)
    return Kxx + jitter * eye + A.transpose(-1, -2) @ (mid[:, None] * A)


class VariationalStrategy(nn.Module):
    """Whitened VariationalStrategy for one DeepGP layer (output_dims=None).

    __call__(x) with x (..., N, D) returns q(f) as a MultivariateNormal (mean, var)
    computed by gpk_kzz_chol_f64 (ONE fp64 factorisation of the shared K_ZZ, cached across
    the calls of a step / eval batches, ops_autograd.KzzCache) + gpk_variational_f32
    (column-tiled fp64-MFMA L^{-1} K_ZX, mean, variance).
    """

    def __init__(self, model, inducing_points: torch.Tensor, variational_distribution,
                 learn_inducing_locations: bool = True, jitter_val: Optional[float] = None):
        super().__init__()
        object.__setattr__(self, "model", model)
        ip = inducing_points.clone()
        if learn_inducing_locations:
            self.register_parameter("inducing_points", nn.Parameter(ip))
        else:
            self.register_buffer("inducing_points", ip)
        self._variational_distribution = variational_distribution
        self.register_buffer("variational_params_initialized", torch.tensor(0))
        self.register_buffer("updated_strategy", torch.tensor(True))
        self.jitter_val = jitter_val
        self._initialized = False     # host mirror of the buffer: no device sync per call
        from .ops_autograd import KzzCache
        self._kzz_cache = KzzCache()
        self._kzz_caches = []            # multi-output layers: one cache per output

    def _load_from_state_dict(self, *args, **kwargs):
        super()._load_from_state_dict(*args, **kwargs)
        self._initialized = bool(int(self.variational_params_initialized))
        self._kzz_cache.clear()
        for c in self._kzz_caches:
            c.clear()

    def train(self, mode: bool = True):
        self._kzz_cache.clear()      # GPyTorch clears its cholesky cache on mode switches
        for c in self._kzz_caches:
            c.clear()
        return super().train(mode)

    @property
    def variational_distribution(self):
        return self._variational_distribution

    def _jitter(self, dtype):
        return self.jitter_val if self.jitter_val is not None else settings.variational_cholesky_jitter.value(dtype)

    def kl_divergence(self) -> torch.Tensor:
        return self._variational_distribution.kl_divergence()

    def __call__(self, x: torch.Tensor) -> MultivariateNormal:
        if not self._initialized:
            self._variational_distribution.initialize_variational_distribution()
            self.variational_params_initialized.fill_(1)
            self._initialized = True
        if self.inducing_points.dim() == 3:
            return self._call_batched(x)
        model = self.model
        batch = x.shape[:-2]
        N, D = x.shape[-2:]
        xf = x.reshape(-1, N, D)
        kern = model.covar_module
        key = (self.inducing_points, kern.raw_outputscale, kern.base_kernel.raw_lengthscale)
        q = self._variational_distribution
        mean, var, flag, cov = self._predict_one(
            xf, self.inducing_points, q.variational_mean, q._variational_stddev, kern.outputscale,
            kern.base_kernel.lengthscale, model.mean_module, self._jitter(x.dtype), self._kzz_cache, key)
        return MultivariateNormal(mean.reshape(*batch, N), var.reshape(*batch, N), clamp_flag=flag,
                                  covar_fn=lambda: cov().reshape(*batch, N, N))

    @staticmethod
    def _predict_one(xf, Z, vmean, vstd, outputscale, lengthscale, mean_module, jitter, cache, key):
        """q(f) of one output on the kernels + a lazy dense covariance for covariance_matrix /
        rsample (upstream VariationalStrategy.forward's predictive_covar)."""
        from .ops_autograd import variational_predict
        mean, var, flag, Linv = variational_predict(
            xf, Z, vmean, vstd, outputscale, lengthscale, mean_module, jitter, cache=cache,
            key_tensors=key, return_linv=True)

        def cov():
            return variational_dense_covariance(xf, Z, Linv, vstd, outputscale, lengthscale, jitter)
        return mean, var, flag, cov

    def _call_batched(self, x: torch.Tensor) -> MultivariateNormal:
        """Multi-output layer (output_dims = O, DeepGP.py:24-26): inducing points (O, M, D), q(u)
        batch (O,), kernel hyper-parameters per output; x (..., O, N, D) as DeepGPLayer.__call__
        expands it. The O outputs are independent GPs: one K_ZZ factor (cached per output) and
        one variational launch each. Returns the batch (..., O) of per-output q(f)."""
        Z = self.inducing_points
        O, M, D = Z.shape
        if x.dim() < 3 or x.shape[-3] != O:
            raise RuntimeError(f"a layer with {O} outputs takes inputs (..., {O}, N, D); got {tuple(x.shape)}")
        batch = x.shape[:-3]
        N = x.shape[-2]
        model = self.model
        kern = model.covar_module
        q = self._variational_distribution
        if len(self._kzz_caches) != O:
            from .ops_autograd import KzzCache
            self._kzz_caches = [KzzCache() for _ in range(O)]
        key = (Z, kern.raw_outputscale, kern.base_kernel.raw_lengthscale)
        s2 = kern.outputscale.reshape(O)
        ls = kern.base_kernel.lengthscale.reshape(O, -1)
        vm = q.variational_mean.reshape(O, M)
        vs = q._variational_stddev.reshape(O, M)
        means, variances, flags, covs = [], [], [], []
        for o in range(O):
            xo = x[..., o, :, :].reshape(-1, N, D)
            m, v, f, c = self._predict_one(xo, Z[o], vm[o], vs[o], s2[o], ls[o], _MeanOutput(model.mean_module, o),
                                           self._jitter(x.dtype), self._kzz_caches[o], key)
            means.append(m.reshape(*batch, N))
            variances.append(v.reshape(*batch, N))
            flags.append(f)
            covs.append(c)
        flag = flags[0]
        for f in flags[1:]:
            flag = torch.bitwise_or(flag, f)

        def cov():
            return torch.stack([c().reshape(*batch, N, N) for c in covs], dim=-3)
        return MultivariateNormal(torch.stack(means, dim=-2), torch.stack(variances, dim=-2), clamp_flag=flag,
                                  covar_fn=cov)


# ---------------------------------------------------------------------------
# marginal log likelihoods (upstream mlls/*.py)
# ---------------------------------------------------------------------------
class _ApproximateMarginalLogLikelihood(nn.Module):
    def __init__(self, likelihood, model, num_data: int, beta: float = 1.0, combine_terms: bool = True):
        super().__init__()
        self.likelihood = likelihood
        self.model = model
        self.num_data = num_data
        self.beta = beta
        self.combine_terms = combine_terms

    def _log_likelihood_term(self, approximate_dist_f, target, **kwargs):
        raise NotImplementedError

    def forward(self, approximate_dist_f: MultivariateNormal, target: torch.Tensor, **kwargs):
        num_batch = approximate_dist_f.event_shape[0]
        log_likelihood = self._log_likelihood_term(approximate_dist_f, target, **kwargs).div(num_batch)
        kl_divergence = self.model.variational_strategy.kl_divergence().div(self.num_data / self.beta)
        if self.combine_terms:
            return log_likelihood - kl_divergence
        return log_likelihood, kl_divergence, torch.zeros_like(log_likelihood)


class VariationalELBO(_ApproximateMarginalLogLikelihood):
    def forward(self, approximate_dist_f: MultivariateNormal, target: torch.Tensor, **kwargs):
        fused = self._fused(approximate_dist_f, target)
        return fused if fused is not None else super().forward(approximate_dist_f, target, **kwargs)

    def _fused(self, dist, target):
        """ELL / N - KL / (num_data / beta) for every row in ONE launch each way
        (gpk::variational_elbo) when the terms are the hot path's: a Gaussian likelihood, a
        variational output of the kernels, one unbatched mean-field strategy. Same warnings as
        the unfused expression (the variance clamp flag)."""
        if (not self.combine_terms or not isinstance(self.likelihood, GaussianLikelihood)
                or not isinstance(dist, MultivariateNormal)):
            return None
        # the fused op takes one scalar noise and returns no target gradient: a batched noise
        # model or a target that requires grad takes the unfused path
        if self.likelihood.noise.numel() != 1 or (torch.is_tensor(target) and target.requires_grad):
            return None
        mean, var = dist._mean, dist._variance
        if (var is None or dist._exact is not None or dist._added_noise is not None or not mean.is_cuda
                or mean.dtype != torch.float32 or var.shape != mean.shape
                or (dist._clamp_flag is None and not dist._preclamped)):
            return None
        strategies = [m for m in self.model.modules() if isinstance(m, VariationalStrategy)]
        if len(strategies) != 1:
            return None
        q = strategies[0].variational_distribution
        if not isinstance(q, MeanFieldVariationalDistribution) or q.variational_mean.dim() != 1:
            return None
        shape = mean.shape
        N = shape[-1]
        y = torch.broadcast_to(target, shape).to(torch.float32)
        min_var = settings.min_variance.value(var.dtype)
        elbo, flag = torch.ops.gpk.variational_elbo(
            y.reshape(-1, N), mean.reshape(-1, N), var.reshape(-1, N), self.likelihood.noise.reshape(1),
            q.variational_mean, q._variational_stddev, float(self.beta) / float(self.num_data), float(min_var))
        # MultivariateNormal.variance's clamp warning: the variational kernel's own flag when the
        # distribution carries it, else the rows' flag computed with the ELBO
        from .ops import record_or_run
        f = dist._clamp_flag if dist._clamp_flag is not None else (flag if dist._preclamped else None)
        if f is not None:
            record_or_run("clamp", (f, min_var), lambda: warn_if_clamped(f, min_var))
        return elbo.reshape(shape[:-1])

    def _log_likelihood_term(self, variational_dist_f, target, **kwargs):
        if hasattr(self.likelihood, "expected_log_prob_sum"):
            return self.likelihood.expected_log_prob_sum(target, variational_dist_f)
        return self.likelihood.expected_log_prob(target, variational_dist_f).sum(-1)


class DeepApproximateMLL(nn.Module):
    def __init__(self, base_mll):
        super().__init__()
        self.base_mll = base_mll

    def forward(self, approximate_dist_f, target, **kwargs):
        return self.base_mll(approximate_dist_f, target, **kwargs).mean(0)


class ExactMarginalLogLikelihood(nn.Module):
    def __init__(self, likelihood, model):
        super().__init__()
        self.likelihood = likelihood
        self.model = model

    def forward(self, function_dist: MultivariateNormal, target: torch.Tensor, *params):
        output = self.likelihood(function_dist)
        res = output.log_prob(target)
        num_data = function_dist.event_shape.numel()
        return res.div(num_data)


class _DeepGPVariationalStrategy:
    """DeepGP.variational_strategy: KL summed over the sub-strategies of the model."""

    def __init__(self, model):
        self._model = model

    def kl_divergence(self):
        strategies = [m for m in self._model.modules() if isinstance(m, VariationalStrategy)]
        return sum(s.kl_divergence().sum() for s in strategies)
