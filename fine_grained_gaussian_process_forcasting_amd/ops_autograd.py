"""Autograd wrappers of the gfx950 hot-path kernels.

FORWARD values always come from libgpk.so (ops.py). BACKWARD:
the exact path uses the analytic HIP adjoint gpk_exact_mll_grad_f32 (Cholesky / TRSM /
RBF adjoints in one kernel). The variational path uses the per-window HIP adjoint
gpk_variational_adjoint_f32 (recomputed K_ZX and A = L^-1 K_ZX, dA, L^-T dA, RBF
adjoint weights); its contractions over points and windows are plain GEMMs (torch ->
rocBLAS), and the shared M x M K_ZZ factor is differentiated once per call with fp64
torch ops on the device. Nothing here runs on the CPU.
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


def _kzz_linv_t(Z, ls, s2, jitter):
    """Linv(Z, l, s2) in fp64 torch ops (M x M, differentiable): the shared K_ZZ factor
    of the forward, for its adjoint only (once per call, not per window)."""
    M = Z.shape[0]
    zs = Z / ls
    Kzz = s2 * torch.exp(-0.5 * _sq_dist(zs, zs))
    Kzz = Kzz + jitter * torch.eye(M, device=Z.device, dtype=Z.dtype)
    L = torch.linalg.cholesky(Kzz)
    return torch.linalg.solve_triangular(L, torch.eye(M, device=Z.device, dtype=Z.dtype), upper=False)


class _VariationalPredict(torch.autograd.Function):
    """Forward: gpk_kzz_chol_f64 + gpk_variational_f32. Backward: the per-window adjoint
    gpk_variational_adjoint_f32 (A, dA, L^-T dA, RBF adjoint weights, in HIP), the
    contractions over points / windows as plain GEMMs, and the M x M K_ZZ adjoint once."""

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
        ctx.save_for_backward(x, Z, vmean, vstd, s2, ls, w, b0, kz.Linv, kz.info, hyper)
        return out.mean, out.var

    @staticmethod
    def backward(ctx, gmean, gvar):
        x, Z, vmean, vstd, s2, ls, w, b0, Linv, kinfo, hyper = ctx.saved_tensors
        B, N, D = x.shape
        M = Z.shape[0]
        if gmean is None:
            gmean = torch.zeros(B, N, device=x.device)
        if gvar is None:
            gvar = torch.zeros(B, N, device=x.device)
        adj = ops.variational_adjoint(x.detach(), Z.detach(), Linv, vmean.detach(), vstd.detach(),
                                      hyper, gmean, gvar)
        lsv = ls.detach().reshape(-1).expand(D).float()
        xs = x.detach().float() / lsv
        zs = Z.detach().float() / lsv
        Q = adj.Q
        r = Q.sum(1)                                      # (B, N)
        q = Q.sum((0, 2))                                 # (M,)
        QZ = torch.einsum("bmn,md->bnd", Q, zs)
        gm = gmean.reshape(B, N).float()
        dX = (QZ - xs * r.unsqueeze(-1)) / lsv + gm.unsqueeze(-1) * w.detach().reshape(1, 1, D).float()
        P = torch.einsum("bmn,bnd->md", Q, xs)
        dZ = (P - zs * q.unsqueeze(-1)) / lsv
        dls = ((q.unsqueeze(-1) * zs * zs).sum(0) - 2.0 * (zs * P).sum(0)
               + torch.einsum("bn,bnd->d", r, xs * xs)) / lsv
        ds2 = Q.sum() / s2.detach().float() + adj.part[:, 2 * M].sum()
        dvm = adj.part[:, :M].sum(0)
        dvs = 2.0 * vstd.detach().reshape(M).float() * adj.part[:, M:2 * M].sum(0)
        dw = torch.einsum("bn,bnd->d", gm, x.detach().float())
        db0 = gm.sum()
        # shared K_ZZ factor: dLinv = sum_b dA K^T (lower part: Linv_mp is used for m >= p)
        # (batched per window, then summed: a single M x M GEMM with a B*N-long
        # contraction leaves the GPU idle -- one output tile)
        dLinv = torch.bmm(adj.dA, adj.K.double().transpose(1, 2)).sum(0).tril()
        t = int(-kinfo.item()) if int(kinfo.item()) < 0 else 0
        jit = ctx.jitter + (1e-8 * 10 ** (t - 1) if t > 0 else 0.0)
        with torch.enable_grad():
            Z2 = Z.detach().double().requires_grad_(True)
            l2 = lsv.double().requires_grad_(True)
            s22 = s2.detach().double().reshape(()).requires_grad_(True)
            gZ, gl, gs = torch.autograd.grad(_kzz_linv_t(Z2, l2, s22, jit), [Z2, l2, s22], dLinv)
        dZ = dZ + gZ.float()
        dls = dls + gl.float()
        ds2 = ds2 + gs.float()
        dls_out = dls.sum().reshape(ls.shape) if ls.numel() == 1 else dls.reshape(ls.shape)
        return (dX.to(x.dtype), dZ.to(Z.dtype), dvm.reshape(vmean.shape).to(vmean.dtype),
                dvs.reshape(vstd.shape).to(vstd.dtype), ds2.reshape(s2.shape).to(s2.dtype),
                dls_out.to(ls.dtype), dw.reshape(w.shape).to(w.dtype), db0.reshape(b0.shape).to(b0.dtype),
                None)


def variational_predict(x, Z, vmean, vstd, outputscale, lengthscale, mean_module, jitter):
    """q(f) mean / variance for (B, N, D) windows (HIP forward; see module docstring)."""
    w = mean_module.weights.reshape(-1)
    b0 = mean_module.bias.reshape(()) if mean_module.bias is not None else torch.zeros((), device=x.device)
    return _VariationalPredict.apply(x, Z, vmean, vstd, outputscale.reshape(()),
                                     lengthscale.reshape(-1), w, b0, float(jitter))
