"""ExactGPModel on the gfx950 kernels (reference denoising_model/GPModel.py:4-13).

``model(x)`` returns the prior MultivariateNormal(mean_x, covar_x) lazily;
``ExactMarginalLogLikelihood(likelihood, model)(model(train_x), train_y)`` evaluates
the per-window marginal log likelihood / N with ONE fused kernel (RBF Gram +
jittered Cholesky + forward solve + logdet): include/gpk.h::gpk_exact_mll_f32.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from ..gp import ConstantMean, MultivariateNormal, RBFKernel, ScaleKernel


class ExactGPModel(nn.Module):
    def __init__(self, train_x, train_y, likelihood):
        super().__init__()
        self.train_inputs = (train_x,)
        self.train_targets = train_y
        self.likelihood = likelihood
        self.mean_module = ConstantMean()
        self.covar_module = ScaleKernel(RBFKernel())

    def forward(self, x):
        mean_x = self.mean_module(x)
        return MultivariateNormal(mean_x, None,
                                  exact=(x, self.covar_module.base_kernel.lengthscale,
                                         self.covar_module.outputscale, self.mean_module.constant))

    def __call__(self, x=None):
        if x is None:
            x = self.train_inputs[0]
        if not self.training and not torch.equal(x, self.train_inputs[0]):
            raise NotImplementedError("exact-GP posterior prediction at new inputs is §8f 'next' work")
        return self.forward(x)
