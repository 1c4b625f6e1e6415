"""Autograd wrappers of the gfx950 hot-path kernels.

FORWARD values always come from libgpk.so (ops.py). BACKWARD:
the exact path uses the analytic HIP adjoint gpk_exact_mll_grad_f32 (Cholesky / TRSM /
RBF adjoints in one kernel). The variational path uses the fused HIP adjoint
gpk_variational_adjoint_f32 (recomputed K_ZX and A = L^-1 K_ZX, dA, L^-T dA, the RBF
adjoint contractions and dL^-1 = sum dA K_ZX^T as a split-K fp64-MFMA GEMM); the shared
K_ZZ factor is ONE autograd node per step (_KzzFactor) whose M x M adjoint runs once for
all the GP calls that used it. Nothing here runs on the CPU.
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


class _KzzState:
    """Shared between a _KzzFactor node and the cache entry that may hand it to a second
    GP call of the same step: once its backward has run, the node is spent."""
    __slots__ = ("consumed",)

    def __init__(self):
        self.consumed = False


class _KzzFactor(torch.autograd.Function):
    """Linv = chol(K_ZZ + jitter)^{-1} of the shared inducing points (gpk_kzz_chol_f64).
    One autograd node per optimizer step: every GP call of the step that uses the same
    (Z, outputscale, lengthscale) consumes this Linv, autograd sums their dLinv, and the
    K_ZZ adjoint (ops.kzz_backward) runs once."""

    @staticmethod
    def forward(ctx, Z, s2, ls, jitter, state, pre):
        if pre is None:
            D = Z.shape[-1]
            lsv = ls.detach().reshape(-1).expand(D).contiguous().float()
            kz = ops.kzz_cholesky(Z.detach(), None, None, jitter=jitter,
                                  hyper=torch.cat([s2.detach().reshape(1).float(), lsv]))
            ops.check_cholesky_info(kz.info, 1e-8, inputs=(Z,), what="K_ZZ cholesky")
            L, Linv = kz.L, kz.Linv
        else:
            L, Linv = pre
        ctx.state = state
        ctx.save_for_backward(Z, s2, ls, L, Linv)
        ctx.mark_non_differentiable(L)
        return Linv, L

    @staticmethod
    def backward(ctx, dLinv, _dL):
        Z, s2, ls, L, Linv = ctx.saved_tensors
        ctx.state.consumed = True
        if dLinv is None:
            return None, None, None, None, None, None
        dZ, ds2, dls = ops.kzz_backward(dLinv, L, Linv, Z, s2, ls)
        dls_out = dls.sum().reshape(ls.shape) if ls.numel() == 1 else dls.reshape(ls.shape)
        return (dZ.to(Z.dtype), ds2.reshape(s2.shape).to(s2.dtype), dls_out.to(ls.dtype),
                None, None, None)


class KzzCache:
    """Per-VariationalStrategy cache of the shared K_ZZ factor.

    Keyed on the identity and version counters of the inducing points and the raw
    kernel hyper-parameters plus the jitter. Training: the enc and dec GP calls of a
    step (denoise_model_2.py:50-51) share one factorisation and one adjoint; after the
    step's backward the node is spent and the next call refactors. Eval (no grad): the
    factor is reused across batches until a parameter changes, as GPyTorch's eval-mode
    ``cholesky_factor`` cache (train.py:197-213, evaluate.py:127-137). Entries are per
    model instance, so concurrent Optuna threads (train.py:86) never share one.
    """

    def __init__(self):
        self._entry = None

    def clear(self):
        self._entry = None

    @staticmethod
    def _key(tensors, jitter):
        return tuple((t.data_ptr(), t._version, tuple(t.shape), str(t.device)) for t in tensors) + (float(jitter),)

    def factor(self, Z, s2, ls, jitter, key_tensors):
        key = self._key(key_tensors, jitter)
        grad = torch.is_grad_enabled() and (Z.requires_grad or s2.requires_grad or ls.requires_grad)
        e = self._entry
        if e is not None and e["key"] == key:
            if not grad:
                return e["Linv"].detach()
            node = e.get("node")
            if node is not None and not e["state"].consumed:
                return node
            pre = (e["L"], e["Linv"])       # same factor, fresh autograd node
        else:
            pre = None
        state = _KzzState()
        if grad:
            Linv, L = _KzzFactor.apply(Z, s2, ls, float(jitter), state, pre)
            self._entry = {"key": key, "L": L.detach(), "Linv": Linv.detach(), "node": Linv,
                           "state": state}
            return Linv
        with torch.no_grad():
            Linv, L = _KzzFactor.apply(Z, s2, ls, float(jitter), state, pre)
        self._entry = {"key": key, "L": L, "Linv": Linv, "node": None, "state": state}
        return Linv


class _VariationalPredict(torch.autograd.Function):
    """Forward: gpk_variational_f32 (one column-tiled launch over all points). Backward:
    gpk_variational_adjoint_f32 (dX, dZ / dl / ds2 of the K_ZX part, dvmean, dvstd and
    dLinv, fused); dLinv flows into the shared _KzzFactor node."""

    @staticmethod
    def forward(ctx, x, Linv, Z, vmean, vstd, s2, ls, w, b0, jitter):
        dev = x.device
        D = x.shape[-1]
        lsv = ls.detach().reshape(-1).expand(D).contiguous().float()
        hyper = ops.pack_variational_hyper(s2.detach(), 1.0, jitter, b0.detach(), w.detach(), lsv, D, dev)
        out = ops.variational_forward(x.detach(), Z.detach(), Linv.detach(), vmean.detach(),
                                      vstd.detach(), hyper=hyper)
        ctx.save_for_backward(x, Linv, Z, vmean, vstd, s2, ls, w, b0, hyper)
        ctx.mark_non_differentiable(out.flags)
        return out.mean, out.var, out.flags

    @staticmethod
    def backward(ctx, gmean, gvar, _gflags):
        x, Linv, Z, vmean, vstd, s2, ls, w, b0, hyper = ctx.saved_tensors
        B, N, D = x.shape
        if gmean is None:
            gmean = torch.zeros(B, N, device=x.device)
        if gvar is None:
            gvar = torch.zeros(B, N, device=x.device)
        adj = ops.variational_adjoint(x, Z, Linv, vmean, vstd, hyper, gmean, gvar)
        gm = gmean.reshape(B * N).float()
        dw = x.detach().reshape(B * N, D).float().transpose(0, 1) @ gm     # LinearMean weights
        db0 = gm.sum()
        dls = adj.dls.sum().reshape(ls.shape) if ls.numel() == 1 else adj.dls.reshape(ls.shape)
        return (adj.dX.to(x.dtype), adj.dLinv, adj.dZ.to(Z.dtype),
                adj.dvmean.reshape(vmean.shape).to(vmean.dtype),
                adj.dvstd.reshape(vstd.shape).to(vstd.dtype), adj.ds2.reshape(s2.shape).to(s2.dtype),
                dls.to(ls.dtype), dw.reshape(w.shape).to(w.dtype), db0.reshape(b0.shape).to(b0.dtype),
                None)


def variational_predict(x, Z, vmean, vstd, outputscale, lengthscale, mean_module, jitter,
                        cache: Optional[KzzCache] = None, key_tensors=None):
    """q(f) mean / variance / clamp flag for (B, N, D) windows (HIP forward and backward;
    see module docstring). ``cache`` shares the K_ZZ factor between calls."""
    w = mean_module.weights.reshape(-1)
    b0 = mean_module.bias.reshape(()) if mean_module.bias is not None else torch.zeros((), device=x.device)
    s2 = outputscale.reshape(())
    ls = lengthscale.reshape(-1)
    if cache is None:
        cache = KzzCache()
    Linv = cache.factor(Z, s2, ls, jitter, key_tensors if key_tensors is not None else (Z, s2, ls))
    return _VariationalPredict.apply(x, Linv, Z, vmean, vstd, s2, ls, w, b0, float(jitter))
