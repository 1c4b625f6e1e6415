"""ExactGPModel on the gfx950 kernels (reference denoising_model/GPModel.py:4-13).

Training mode: ``model(x)`` returns the prior MultivariateNormal(mean_x, covar_x)
lazily; ``ExactMarginalLogLikelihood(likelihood, model)(model(train_x), train_y)``
evaluates the per-window marginal log likelihood / N with ONE fused kernel (RBF Gram +
jittered Cholesky + forward solve + logdet): include/gpk.h::gpk_exact_mll_f32.

Eval mode: ``model(x)`` is the posterior of f at x (upstream
models/exact_gp.py __call__ -> exact_prediction_strategies.py): the training factor L
and z = L^{-1}(y - c) come from gpk_exact_mll_f32 once and are cached until a
parameter or the training data changes or ``train()`` is called (GPyTorch's
``prediction_strategy`` cache); mean and variance at x come from
gpk_exact_posterior_f32. ``likelihood(model(x))`` adds the noise. As in GPyTorch,
calling the model in eval mode on the training inputs warns (GPInputWarning) and
returns the posterior there.

Inputs may be batched (B, N, D) windows, a single (N, D) window or 1-D (N,) points,
as GPyTorch accepts; targets follow (B, N) / (N,).
"""
from __future__ import annotations

import warnings
import weakref

import torch
import torch.nn as nn

from .. import ops
from ..errors import GPInputWarning
from ..gp import ConstantMean, MultivariateNormal, RBFKernel, ScaleKernel, psd_safe_cholesky


def _as_batch(x: torch.Tensor) -> torch.Tensor:
    """(N,) -> (1, N, 1); (N, D) -> (1, N, D); (B, N, D) unchanged."""
    if x.dim() == 1:
        return x.reshape(1, -1, 1)
    if x.dim() == 2:
        return x.unsqueeze(0)
    if x.dim() == 3:
        return x
    raise ValueError(f"inputs must be (N,), (N, D) or (B, N, D), got {tuple(x.shape)}")


class _PredictionCacheHandle:
    """Lets ops_autograd.invalidate_caches() drop a model's prediction cache (HIP graph
    replays change parameters without bumping the version counters it is keyed on)."""

    def __init__(self, model):
        self._model = weakref.ref(model)

    def clear(self):
        m = self._model()
        if m is not None:
            m._prediction_cache = None


def _version_key(*ts):
    return tuple((t.data_ptr(), t._version, tuple(t.shape)) for t in ts)


class ExactGPModel(nn.Module):
    def __init__(self, train_x, train_y, likelihood):
        super().__init__()
        self.train_inputs = (train_x,)
        self.train_targets = train_y
        self.likelihood = likelihood
        self.mean_module = ConstantMean()
        self.covar_module = ScaleKernel(RBFKernel())
        self._prediction_cache = None
        self._cache_handle = _PredictionCacheHandle(self)
        from ..ops_autograd import register_cache
        register_cache(self._cache_handle)

    def set_train_data(self, inputs=None, targets=None, strict=True):
        if inputs is not None:
            x = inputs[0] if isinstance(inputs, (tuple, list)) else inputs
            if strict and x.shape != self.train_inputs[0].shape:
                raise RuntimeError("Cannot modify the shape of train inputs with strict=True")
            self.train_inputs = (x,)
        if targets is not None:
            if strict and targets.shape != self.train_targets.shape:
                raise RuntimeError("Cannot modify the shape of train targets with strict=True")
            self.train_targets = targets
        self._prediction_cache = None

    def train(self, mode: bool = True):
        self._prediction_cache = None       # GPyTorch drops its prediction strategy here
        return super().train(mode)

    def forward(self, x):
        xb = _as_batch(x)
        mean_x = self.mean_module(x if x.dim() > 1 else x.unsqueeze(-1))
        return MultivariateNormal(mean_x, None,
                                  exact=(xb, self.covar_module.base_kernel.lengthscale,
                                         self.covar_module.outputscale, self.mean_module.constant))

    def __call__(self, x=None):
        if x is None:
            x = self.train_inputs[0]
        if self.training:
            return self.forward(x)
        train_x = self.train_inputs[0]
        if x.shape == train_x.shape and torch.equal(x, train_x):
            warnings.warn("The input matches the stored training data. Did you forget to call "
                          "model.train()?", GPInputWarning)
        return self._posterior(x)

    # ---- eval mode -------------------------------------------------------------
    def _hyper(self, device):
        kern = self.covar_module
        return ops.pack_exact_hyper(kern.outputscale, self.likelihood.noise, self.mean_module.constant,
                                    kern.base_kernel.lengthscale, device)

    def _train_factor(self):
        train_x, train_y = self.train_inputs[0], self.train_targets
        kern = self.covar_module
        key = _version_key(train_x, train_y, kern.raw_outputscale, kern.base_kernel.raw_lengthscale,
                           self.mean_module.constant, self.likelihood.noise_covar.raw_noise)
        cache = self._prediction_cache
        if cache is not None and cache[0] == key:
            return cache[1]
        Xb = _as_batch(train_x).detach().float()
        yb = train_y.detach().reshape(Xb.shape[0], Xb.shape[1]).float()
        hyper = self._hyper(Xb.device).detach()
        out = ops.exact_mll(Xb, yb, None, None, None, None, want_L=True, want_z=True, hyper=hyper)
        ops.check_cholesky_info(out.info, 1e-6, inputs=(Xb, yb))
        entry = (Xb, out.L, out.z, hyper)
        self._prediction_cache = (key, entry)
        return entry

    def _posterior(self, x):
        params = [p for p in self.parameters()] + [x, self.train_inputs[0], self.train_targets]
        if torch.is_grad_enabled() and any(t.requires_grad for t in params):
            return self._posterior_autograd(x)
        Xb, L, z, hyper = self._train_factor()
        xs = _as_batch(x).float()
        if xs.shape[0] != Xb.shape[0]:
            xs = xs.expand(Xb.shape[0], *xs.shape[1:])
        from .. import library  # noqa: F401  (registers torch.ops.gpk)
        mean, var = torch.ops.gpk.exact_posterior(Xb, L, z, hyper, xs.contiguous())
        if x.dim() == 3 or Xb.shape[0] > 1:
            shape = mean.shape                    # (B, Ns): one posterior per training window
        else:
            shape = x.shape[:-1] if x.dim() > 1 else x.shape
        return MultivariateNormal(mean.reshape(shape), var.reshape(shape))

    def _posterior_autograd(self, x):
        """The eval posterior WITH gradients (GPyTorch allows them; upstream
        exact_prediction_strategies.py): the same quantities as gpk_exact_posterior_f32,
        restated in differentiable torch ops on the caller's device -- K_hat = s2 RBF(X, X) +
        noise I, L = psd_safe_cholesky(K_hat) (the fp32 jitter ladder), K* = s2 RBF(X, x) over the
        joint inputs in upstream ``_sq_dist``'s centred GEMM form, V = L^{-1} K*,
        z = L^{-1} (y - c), mean = c + V^T z, var = s2 - colsum(V o V). Taken only when a
        gradient will flow (a parameter, the inputs or the training data require grad): the
        prediction cache is not used, as GPyTorch does not cache through autograd either.
        Off the hot path: no HIP kernel serves this."""
        train_x, train_y = self.train_inputs[0], self.train_targets
        if not (x.is_cuda and train_x.is_cuda):
            raise ValueError("ExactGPModel runs on the GPU: move the model and inputs to a cuda device")
        Xb = _as_batch(train_x)
        yb = train_y.reshape(Xb.shape[0], Xb.shape[1])
        xs = _as_batch(x)
        if xs.shape[0] != Xb.shape[0]:
            xs = xs.expand(Xb.shape[0], *xs.shape[1:])
        kern = self.covar_module
        ls = kern.base_kernel.lengthscale.reshape(-1)
        s2 = kern.outputscale.reshape(())
        c = self.mean_module.constant.reshape(())
        noise = self.likelihood.noise.reshape(())
        n = Xb.shape[-2]
        full = torch.cat([Xb, xs], -2) / ls
        a = full - full.mean(-2, keepdim=True)
        nrm = a.pow(2).sum(-1, keepdim=True)
        d = (nrm + nrm.transpose(-1, -2) - 2.0 * a @ a.transpose(-1, -2)).clamp_min(0.0)
        K = s2 * torch.exp(-0.5 * d)
        eye = torch.eye(n, dtype=K.dtype, device=K.device)
        Kxx = K[..., :n, :n] * (1.0 - eye) + s2 * eye        # exact diagonal, as _sq_dist zeroes it
        L = psd_safe_cholesky(Kxx + noise * eye)
        V = torch.linalg.solve_triangular(L, K[..., :n, n:], upper=False)
        zz = torch.linalg.solve_triangular(L, (yb - c).unsqueeze(-1), upper=False)
        mean = c + (V * zz).sum(-2)
        var = s2 - (V * V).sum(-2)
        if x.dim() == 3 or Xb.shape[0] > 1:
            shape = mean.shape
        else:
            shape = x.shape[:-1] if x.dim() > 1 else x.shape
        return MultivariateNormal(mean.reshape(shape), var.reshape(shape))
