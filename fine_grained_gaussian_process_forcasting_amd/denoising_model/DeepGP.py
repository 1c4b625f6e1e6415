"""DeepGPp / ToyDeepGPHiddenLayer on the gfx950 kernels.

Same constructor signatures, RNG consumption order, module / parameter names and
outputs as the reference denoising_model/DeepGP.py:14-99 (which subclasses
gpytorch.models.deep_gps.DeepGPLayer / DeepGP), so callers and state_dicts carry over:

  hidden_layer.variational_strategy.inducing_points                         (M, D)
  hidden_layer.variational_strategy._variational_distribution.variational_mean
  hidden_layer.variational_strategy._variational_distribution._variational_stddev
  hidden_layer.mean_module.weights / .bias                                   (LinearMean)
  hidden_layer.covar_module.raw_outputscale, .base_kernel.raw_lengthscale   (ARD)
  likelihood.noise_covar.raw_noise
"""
from __future__ import annotations

import random

import numpy as np
import torch
import torch.nn as nn

from ..gp import (ConstantMean, GaussianLikelihood, LinearMean, MeanFieldVariationalDistribution,
                  MultitaskMultivariateNormal, MultivariateNormal, RBFKernel, ScaleKernel,
                  VariationalStrategy, _DeepGPVariationalStrategy, settings)


class ToyDeepGPHiddenLayer(nn.Module):
    """Reference DeepGP.py:14-73. output_dims=None (what DeepGPp builds) gives one GP; an
    integer O gives O independent output GPs (inducing points (O, M, D), q(u) and kernel
    hyper-parameters batched over O) whose output is a MultitaskMultivariateNormal with event
    shape (N, O), as GPyTorch's DeepGPLayer returns it."""

    def __init__(self, input_dims, output_dims, seed, num_inducing=256, mean_type='constant'):
        super().__init__()
        np.random.seed(seed)
        random.seed(seed)
        torch.manual_seed(seed)
        if output_dims is None:
            inducing_points = torch.randn(num_inducing, input_dims)          # DeepGP.py:22
            batch_shape = torch.Size([])
        else:
            inducing_points = torch.randn(output_dims, num_inducing, input_dims)   # DeepGP.py:25
            batch_shape = torch.Size([output_dims])
        variational_distribution = MeanFieldVariationalDistribution(num_inducing, batch_shape)
        self.variational_strategy = VariationalStrategy(self, inducing_points, variational_distribution,
                                                        learn_inducing_locations=True)
        self.input_dims = input_dims
        self.output_dims = output_dims
        if mean_type == 'constant':
            self.mean_module = ConstantMean(batch_shape=batch_shape)
        else:
            self.mean_module = LinearMean(input_dims)                     # DeepGP.py:45
        self.covar_module = ScaleKernel(RBFKernel(batch_shape=batch_shape, ard_num_dims=input_dims),
                                        batch_shape=batch_shape, ard_num_dims=None)

    def forward(self, x):
        """The layer's PRIOR at x, as reference DeepGP.py:51-54 returns it:
        MultivariateNormal(mean_module(x), covar_module(x)) with the covariance lazy, as in
        GPyTorch: ``.variance`` is the kernel diagonal (outputscale), ``.covariance_matrix``
        materialises outputscale * ARD-RBF(x, x), and ``.log_prob`` runs the fused
        RBF + jittered Cholesky kernel on the residual value - mean(x). (q(f) -- what the
        reference trains on -- comes from __call__.)"""
        mean_x = self.mean_module(x)
        xb = x.reshape(-1, x.shape[-2], x.shape[-1])
        kern = self.covar_module
        return MultivariateNormal(mean_x, None,
                                  exact=(xb, kern.base_kernel.lengthscale, kern.outputscale, None))

    def __call__(self, x, *other_inputs, **kwargs):
        """DeepGP.py:56-73 + DeepGPLayer.__call__ (upstream models/deep_gps/deep_gp.py).

        Skip connections (``other_inputs``): each extra input is expanded to
        (S, *shape) and concatenated to ``x`` on the feature axis; ``x`` is then taken
        as samples (``are_samples=True``: shape (S, ..., N, D_x)) and the output is NOT
        expanded again. Otherwise the deterministic inputs give q(f) with batch (..., )
        expanded to (S, ...), S = settings.num_likelihood_samples (1 under train.py:20).
        Both mean types run on the fused kernel: ConstantMean is LinearMean with w = 0
        and b0 = the constant (ops_autograd.variational_predict).

        A MultitaskMultivariateNormal ``x`` (a multi-output layer's output): with skip inputs it
        is ``rsample()``d from its full covariance first (DeepGP.py:62-64); alone it is sampled
        from its marginals, as DeepGPLayer.__call__ does (``Normal(mean, variance.sqrt())``), and
        the output is then not expanded. A layer with output_dims = O runs its O output GPs on
        the inputs expanded to (..., O, N, D) and returns q(f) as a MultitaskMultivariateNormal."""
        are_samples = bool(len(other_inputs))
        S = settings.num_likelihood_samples.value()
        if are_samples:
            if isinstance(x, MultitaskMultivariateNormal):
                x = x.rsample()
            processed = [inp.unsqueeze(0).expand(S, *inp.shape) for inp in other_inputs]
            x = torch.cat([x] + processed, dim=-1)
        deterministic = not are_samples
        if isinstance(x, MultitaskMultivariateNormal):
            x = torch.distributions.Normal(loc=x.mean, scale=x.variance.sqrt()).rsample()
            deterministic = False
        if x.size(-1) != self.input_dims:
            raise RuntimeError(f"Input shape did not match self.input_dims. Got total feature dims "
                               f"[{x.size(-1)}], expected [{self.input_dims}]")
        if self.output_dims is not None:
            x = x.unsqueeze(-3).expand(*x.shape[:-2], self.output_dims, *x.shape[-2:])
        output = self.variational_strategy(x)
        if self.output_dims is not None:
            output = MultitaskMultivariateNormal.from_batch_mvn(output, task_dim=-1)
        if not deterministic:
            return output
        return output.expand(torch.Size([S]) + output.batch_shape)


class DeepGPp(nn.Module):
    """Reference DeepGP.py:76-99."""

    def __init__(self, num_hidden_dims, seed):
        hidden_layer = ToyDeepGPHiddenLayer(input_dims=num_hidden_dims, output_dims=None,
                                            mean_type='linear', seed=seed)
        super().__init__()
        self.hidden_layer = hidden_layer
        self.likelihood = GaussianLikelihood()
        self.variational_strategy = _DeepGPVariationalStrategy(self)

    def forward(self, inputs):
        return self.hidden_layer(inputs)

    def __call__(self, inputs):
        return self.forward(inputs)

    def predict(self, x):
        dist = self(x)
        preds = self.likelihood(dist)
        return preds.mean, dist
