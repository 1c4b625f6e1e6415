"""denoise_model_2 on the gfx950 GP kernels (reference denoising_model/denoise_model_2.py:10-66).

Divergence (documented): the reference calls ``self.proj_up``
in add_gp_noise (:37) but its definition is commented out (:21), so ``--gp True``
raises AttributeError there. The evident intent, ``nn.Linear(1, d)``, is restored.
The reference's global ``torch.autograd.set_detect_anomaly(True)`` (:7) is not
replicated at import (it is a debugging mode).

forward() runs the two GP blurs of the reference (:46-47, enc then dec through the same
DeepGPp) as ONE evaluation on the points of both concatenated per window: q(f)'s marginals
are per point and the layer draws no random numbers (num_likelihood_samples = 1), so the
enc / dec means and the dec distribution are exactly the two calls' outputs, with one
variational forward + one adjoint launch chain per step instead of two (and one K_ZZ use).
``add_gp_noise`` stays the reference's single-input method.
"""
from __future__ import annotations

import random

import numpy as np
import torch
import torch.nn as nn

from .DeepGP import DeepGPp


class denoise_model_2(nn.Module):
    def __init__(self, model, model_name, gp, d, device, seed, n_noise=False, residual=False):
        super(denoise_model_2, self).__init__()
        np.random.seed(seed)
        random.seed(seed)
        torch.manual_seed(seed)
        self.denoising_model = model
        self.deep_gp = DeepGPp(d, seed)
        self.proj_up = nn.Linear(1, d)   # restored (reference :21 is commented out)
        self.gp = gp
        self.residual = residual
        self.norm = nn.LayerNorm(d)
        self.d = d
        self.device = device
        self.n_noise = n_noise
        self.residual = residual

    def add_gp_noise(self, x):
        b, s, _ = x.shape
        eps_gp, dist = self.deep_gp.predict(x)
        # proj_up(e) for in_features == 1 is e * W[:, 0] + bias: computed as a broadcast
        # multiply-add (a GEMM with K = 1 whose weight gradient is a K = b*s reduction
        # ran 0.17 ms per call in hipBLASLt at b = 256, s = 192; this is one fused
        # elementwise kernel and a plain reduction in the backward)
        e = eps_gp.permute(1, 2, 0)
        eps_gp = torch.addcmul(self.proj_up.bias, e, self.proj_up.weight.reshape(-1))
        x_noisy = x + eps_gp
        return x_noisy, dist

    def add_gp_noise_pair(self, enc, dec):
        """add_gp_noise(enc) and add_gp_noise(dec) (reference :46-47) as one GP evaluation
        over the concatenated points; returns (enc_noisy, dec_noisy, dist of dec)."""
        s_enc = enc.shape[1]
        eps_gp, dist = self.deep_gp.predict(torch.cat([enc, dec], dim=1))
        e = eps_gp.permute(1, 2, 0)
        eps = torch.addcmul(self.proj_up.bias, e, self.proj_up.weight.reshape(-1))
        return enc + eps[:, :s_enc], dec + eps[:, s_enc:], dist.slice_points(s_enc, None)

    def forward(self, enc_inputs, dec_inputs):
        eps_enc = torch.randn_like(enc_inputs)
        eps_dec = torch.randn_like(dec_inputs)
        dist = None
        if self.gp:
            enc_noisy, dec_noisy, dist = self.add_gp_noise_pair(enc_inputs, dec_inputs)
        elif self.n_noise:
            enc_noisy = enc_inputs
            dec_noisy = dec_inputs
        else:
            enc_noisy = enc_inputs.add_(eps_enc * 0.05)
            dec_noisy = dec_inputs.add_(eps_dec * 0.05)
        enc_rec, dec_rec = self.denoising_model(enc_noisy, dec_noisy)
        dec_output = dec_inputs + dec_rec
        return dec_output, dist
