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
                  MultivariateNormal, RBFKernel, ScaleKernel, VariationalStrategy,
                  _DeepGPVariationalStrategy, settings)


class ToyDeepGPHiddenLayer(nn.Module):
    """Reference DeepGP.py:14-73 (output_dims=None is the only configuration used)."""

    def __init__(self, input_dims, output_dims, seed, num_inducing=256, mean_type='constant'):
        super().__init__()
        np.random.seed(seed)
        random.seed(seed)
        torch.manual_seed(seed)
        if output_dims is not None:
            raise NotImplementedError("multi-output DeepGP layers are not on the reference path "
                                      "(DeepGPp uses output_dims=None, DeepGP.py:77-82)")
        inducing_points = torch.randn(num_inducing, input_dims)          # DeepGP.py:22
        batch_shape = torch.Size([])
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
        return self.variational_strategy(x)

    def __call__(self, x, *other_inputs, **kwargs):
        if len(other_inputs):
            raise NotImplementedError("skip-connection inputs are unused by the reference path")
        if not isinstance(self.mean_module, LinearMean):
            raise NotImplementedError("the fused kernel implements DeepGPp's LinearMean (DeepGP.py:81)")
        output = self.variational_strategy(x)
        # DeepGPLayer.__call__: deterministic inputs -> expand to (S, *batch) with
        # S = settings.num_likelihood_samples (1 under train.py:20)
        S = settings.num_likelihood_samples.value()
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
