"""Autograd wrappers of the gfx950 hot-path kernels.

FORWARD values always come from libgpk.so (ops.py). BACKWARD: the exact path uses
the analytic HIP adjoint gpk_exact_mll_grad_f32 (Cholesky / TRSM / RBF adjoints in
one kernel). The variational path (interim) differentiates a
torch restatement of the same forward on the SAME device (``_recompute_variational``,
fp32 RBF + fp64 solve exactly as the reference) inside ``backward`` only; its forward
values are discarded. Nothing here runs on the CPU.
"""
from __future__ import annotations

import math
from typing import Optional

import torch

from . import ops

LOG_2PI = math.log(2.0 * math.pi)


def _sq_dist(x1, x2):
    """GPyTorch Distance._sq_dist (mean-centred GEMM form, clamp at 0)."""
    adj = x1.mean(-2, keepdim=True)
    x1 = x1 - adj
    x2 = x2 - adj
    x1n = x1.pow(2).sum(-1, keepdim=True)
    x2n = x2.pow(2).sum(-1, keepdim=True)
    res = (-2.0 * x1) @ x2.transpose(-1, -2) + x1n + x2n.transpose(-1, -2)
    return res.clamp_min(0)


class _ExactMLL(torch.autograd.Function):
    """Forward: gpk_exact_mll_f32 (L and z kept when a gradient is needed).
    Backward: gpk_exact_mll_grad_f32, the analytic HIP adjoint."""

    @staticmethod
    def forward(ctx, X, y, lengthscale, outputscale, constant, noise):
        hyper = ops.pack_exact_hyper(outputscale.detach(), noise.detach(), constant.detach(),
                                     lengthscale.detach(), X.device)
        jitter = 1e-6
        need = any(ctx.needs_input_grad)
        out = ops.exact_mll(X.detach(), y.detach(), None, None, None, None, hyper=hyper,
                            jitter=jitter, want_L=need, want_z=need)
        ops.check_cholesky_info(out.info, jitter, inputs=(X, y))
        if need:
            ctx.save_for_backward(X, out.L, out.z, hyper)
        ctx.ls_shape = lengthscale.shape
        return out.mll

    @staticmethod
    def backward(ctx, grad):
        X, L, z, hyper = ctx.saved_tensors
        nx, ny = ctx.needs_input_grad[0], ctx.needs_input_grad[1]
        g = ops.exact_mll_grad(X.detach(), L, z, hyper, grad.detach(), want_dX=nx, want_dy=ny)
        dh = g.dhyp.sum(0)
        return (g.dX if nx else None, g.dy if ny else None, dh[3:].reshape(ctx.ls_shape),
                dh[0].reshape(()), dh[2].reshape(()), dh[1].reshape(()))


def exact_log_prob(X, y, lengthscale, outputscale, constant, noise) -> torch.Tensor:
    """Per-window exact-GP log marginal likelihood / N (fused HIP kernel forward)."""
    B, N, D = X.shape
    ls = lengthscale.reshape(-1)
    s2 = outputscale.reshape(())
    c = constant.reshape(())
    nz = noise.reshape(())
    return _ExactMLL.apply(X, y, ls, s2, c, nz)


def _recompute_variational(x, Z, vmean, vstd, s2, ls, w, b0, jitter):
    M = Z.shape[0]
    zs = Z / ls
    xs = x / ls
    Kzz = s2 * torch.exp(-0.5 * _sq_dist(zs, zs))
    Kzz = Kzz + jitter * torch.eye(M, device=x.device, dtype=x.dtype)
    L = torch.linalg.cholesky(Kzz.double())
    Kzx = s2 * torch.exp(-0.5 * _sq_dist(zs.expand(x.shape[0], M, -1), xs))
    A = torch.linalg.solve_triangular(L, Kzx.double(), upper=False).to(x.dtype)
    mean = (A * vmean.unsqueeze(-1)).sum(-2) + (x @ w.reshape(-1, 1)).squeeze(-1) + b0
    var = s2 + jitter + (A * ((vstd.pow(2) - 1).unsqueeze(-1) * A)).sum(-2)
    return mean, var


class _VariationalPredict(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, Z, vmean, vstd, s2, ls, w, b0, jitter):
        dev = x.device
        D = x.shape[-1]
        lsv = ls.detach().reshape(-1).expand(D).contiguous().float()
        kz = ops.kzz_cholesky(Z.detach(), None, None, jitter=jitter,
                              hyper=torch.cat([s2.detach().reshape(1).float(), lsv]))
        ops.check_cholesky_info(kz.info, 1e-8, inputs=(Z,), what="K_ZZ cholesky")
        hyper = ops.pack_variational_hyper(s2.detach(), 1.0, jitter, b0.detach(), w.detach(), lsv, D, dev)
        out = ops.variational_forward(x.detach(), Z.detach(), kz.Linv, vmean.detach(), vstd.detach(),
                                      hyper=hyper)
        ctx.jitter = jitter
        ctx.save_for_backward(x, Z, vmean, vstd, s2, ls, w, b0)
        return out.mean, out.var

    @staticmethod
    def backward(ctx, gmean, gvar):
        saved = ctx.saved_tensors
        inputs = [t.detach().requires_grad_(True) for t in saved]
        with torch.enable_grad():
            mean, var = _recompute_variational(*inputs, ctx.jitter)
            outs, gouts = [], []
            for o, g in ((mean, gmean), (var, gvar)):
                if g is not None:
                    outs.append(o)
                    gouts.append(g)
            grads = torch.autograd.grad(outs, inputs, gouts, allow_unused=True)
        return (*grads, None)


def variational_predict(x, Z, vmean, vstd, outputscale, lengthscale, mean_module, jitter):
    """q(f) mean / variance for (B, N, D) windows (HIP forward; see module docstring)."""
    w = mean_module.weights.reshape(-1)
    b0 = mean_module.bias.reshape(()) if mean_module.bias is not None else torch.zeros((), device=x.device)
    return _VariationalPredict.apply(x, Z, vmean, vstd, outputscale.reshape(()),
                                     lengthscale.reshape(-1), w, b0, float(jitter))
