"""torch.library registration of the gfx950 GP kernels (namespace ``gpk``).

SURVEY.md §8b ("Who calls it"): the model classes reach the kernels through
``torch.library`` custom ops with registered autograd formulas, so the ops are visible
to the dispatcher (FakeTensor shape propagation, ``torch.library.opcheck``, tracing)
instead of being opaque Python. Each op is one C-ABI call of include/gpk.h on
``torch.cuda.current_stream()`` (ops.py); nothing here computes on the CPU.

  gpk::exact_mll(X, y, hyper, jitter, max_tries) -> (mll, L, z, info)         [autograd]
  gpk::exact_mll_grad(X, L, z, hyper, gout) -> (dX, dy, dhyp)
  gpk::exact_posterior(X, L, z, hyper, Xs) -> (mean, var)                     [eval only]
  gpk::kzz_factor(Z, s2, ls, jitter, chol_jitter, max_tries) -> (Linv, L, info) [autograd]
  gpk::variational_fwd(x, Linv, Z, vmean, vstd, s2, ls, w, b0, jitter) -> (mean, var, flags, hyper)
                                                                               [autograd]
  gpk::variational_adj(x, Linv, Z, vmean, vstd, hyper, gmean, gvar) -> (dX, dLinv, dZ, dpar)
  gpk::gauss_ell(y, mean, var, noise) -> ell (R,)                             [autograd]
  gpk::meanfield_kl(m, s) -> kl (1,)                                          [autograd]
  gpk::variational_elbo(y, mean, var, noise, m, s, kl_scale, min_var) -> (elbo (R,), flag)
                                                                               [autograd]

Reference call sites they serve: GPModel.py:10-13 + ExactMarginalLogLikelihood
(exact_mll), ExactGPModel in eval mode (exact_posterior), DeepGP.py:33-73 VariationalStrategy (kzz_factor, variational_fwd),
the ELBO at forecast_denoising.py:86-89 (gauss_ell, meanfield_kl), and the backward of
train.py:166 (the *_grad / *_adj ops).
"""
from __future__ import annotations

from typing import Tuple

import torch
from torch import Tensor

from . import _native, ops

# ---------------------------------------------------------------------------
# exact GP marginal log likelihood (gpk_exact_mll_f32 / gpk_exact_mll_grad_f32)
# ---------------------------------------------------------------------------


@torch.library.custom_op("gpk::exact_mll", mutates_args=(), device_types="cuda")
def exact_mll(X: Tensor, y: Tensor, hyper: Tensor, jitter: float, max_tries: int,
              want_factor: bool) -> Tuple[Tensor, Tensor, Tensor, Tensor]:
    """want_factor=False (no gradient needed) skips writing L and z (empty outputs)."""
    out = ops.exact_mll(X, y, None, None, None, None, jitter=jitter, max_tries=max_tries,
                        want_L=want_factor, want_z=want_factor, hyper=hyper)
    if not want_factor:
        return out.mll, X.new_empty(0), X.new_empty(0), out.info
    return out.mll, out.L, out.z, out.info


@exact_mll.register_fake
def _(X, y, hyper, jitter, max_tries, want_factor):
    B, N, _ = X.shape
    if not want_factor:
        return X.new_empty(B), X.new_empty(0), X.new_empty(0), X.new_empty(B, dtype=torch.int32)
    return (X.new_empty(B), X.new_empty(B, N, N), X.new_empty(B, N),
            X.new_empty(B, dtype=torch.int32))


@torch.library.custom_op("gpk::exact_mll_grad", mutates_args=(), device_types="cuda")
def exact_mll_grad(X: Tensor, L: Tensor, z: Tensor, hyper: Tensor,
                   gout: Tensor) -> Tuple[Tensor, Tensor, Tensor]:
    g = ops.exact_mll_grad(X, L, z, hyper, gout)
    return g.dX, g.dy, g.dhyp


@exact_mll_grad.register_fake
def _(X, L, z, hyper, gout):
    B, N, D = X.shape
    return X.new_empty(B, N, D), X.new_empty(B, N), X.new_empty(B, hyper.numel())


@torch.library.custom_op("gpk::exact_posterior", mutates_args=(), device_types="cuda")
def exact_posterior(X: Tensor, L: Tensor, z: Tensor, hyper: Tensor, Xs: Tensor) -> Tuple[Tensor, Tensor]:
    p = ops.exact_posterior(X, L, z, hyper, Xs)
    return p.mean, p.var


@exact_posterior.register_fake
def _(X, L, z, hyper, Xs):
    B, Ns, _ = Xs.shape
    return Xs.new_empty(B, Ns), Xs.new_empty(B, Ns)


def _exact_setup(ctx, inputs, output):
    X, y, hyper, jitter, max_tries, want_factor = inputs
    mll, L, z, info = output
    ctx.save_for_backward(X, L, z, hyper)
    ctx.mark_non_differentiable(L, z, info)


def _exact_backward(ctx, gmll, _gL, _gz, _ginfo):
    X, L, z, hyper = ctx.saved_tensors
    if L.numel() == 0:
        raise RuntimeError("gpk::exact_mll was called with want_factor=False; no backward")
    dX, dy, dhyp = torch.ops.gpk.exact_mll_grad(X, L, z, hyper, gmll.contiguous())
    return dX, dy, dhyp.sum(0), None, None, None


exact_mll.register_autograd(_exact_backward, setup_context=_exact_setup)

# ---------------------------------------------------------------------------
# shared K_ZZ factor (gpk_kzz_chol_f64) + its M x M adjoint (ops.kzz_backward)
# ---------------------------------------------------------------------------


@torch.library.custom_op("gpk::kzz_factor", mutates_args=(), device_types="cuda")
def kzz_factor(Z: Tensor, s2: Tensor, ls: Tensor, jitter: float, chol_jitter: float,
               max_tries: int) -> Tuple[Tensor, Tensor, Tensor]:
    D = Z.shape[-1]
    lsv = ls.detach().reshape(-1).expand(D).contiguous().float()
    kz = ops.kzz_cholesky(Z.detach(), None, None, jitter=jitter, chol_jitter=chol_jitter,
                          max_tries=max_tries, hyper=torch.cat([s2.detach().reshape(1).float(), lsv]))
    return kz.Linv, kz.L, kz.info


@kzz_factor.register_fake
def _(Z, s2, ls, jitter, chol_jitter, max_tries):
    M = Z.shape[0]
    return (Z.new_empty(M, M, dtype=torch.float64), Z.new_empty(M, M, dtype=torch.float64),
            Z.new_empty(1, dtype=torch.int32))


def _kzz_setup(ctx, inputs, output):
    Z, s2, ls = inputs[:3]
    Linv, L, info = output
    ctx.save_for_backward(Z, s2, ls, L, Linv)
    ctx.mark_non_differentiable(L, info)


def _kzz_backward(ctx, dLinv, _dL, _dinfo):
    Z, s2, ls, L, Linv = ctx.saved_tensors
    if dLinv is None:
        return None, None, None, None, None, None
    dZ, ds2, dls = ops.kzz_backward(dLinv, L, Linv, Z, s2, ls)
    dls_out = dls.sum().reshape(ls.shape) if ls.numel() == 1 else dls.reshape(ls.shape)
    return (dZ.to(Z.dtype), ds2.reshape(s2.shape).to(s2.dtype), dls_out.to(ls.dtype),
            None, None, None)


kzz_factor.register_autograd(_kzz_backward, setup_context=_kzz_setup)

# ---------------------------------------------------------------------------
# variational predictive distribution (gpk_variational_f32 / gpk_variational_adjoint_f32)
# ---------------------------------------------------------------------------


def _var_hyper(x, s2, ls, w, b0, jitter):
    D = x.shape[-1]
    lsv = ls.detach().reshape(-1).expand(D).contiguous().float()
    return ops.pack_variational_hyper(s2.detach(), 1.0, jitter, b0.detach(), w.detach(), lsv, D, x.device)


def _saved_numel(x, Z, save):
    if not save:
        return 0
    B, N, D = x.shape
    return _native.lib().gpk_variational_saved_bytes(B, N, Z.shape[0], D) // 4


@torch.library.custom_op("gpk::variational_fwd", mutates_args=(), device_types="cuda")
def variational_fwd(x: Tensor, Linv: Tensor, Z: Tensor, vmean: Tensor, vstd: Tensor, s2: Tensor,
                    ls: Tensor, w: Tensor, b0: Tensor, jitter: float,
                    save: bool = False) -> Tuple[Tensor, Tensor, Tensor, Tensor, Tensor]:
    """-> (mean, var, clamp flags, packed hyper vector, saved state). The hyper vector is
    returned so the backward reuses it (one pack per GP call, not one per direction).
    ``save`` (a gradient will be needed): the forward keeps A = Linv K_ZX and the clamp mask
    for the saved-state adjoint where it serves the shape (M > 64; gpk_variational_train_f32),
    else the state is empty and the adjoint recomputes."""
    hyper = _var_hyper(x, s2, ls, w, b0, jitter)
    out = ops.variational_forward(x, Z, Linv, vmean, vstd, hyper=hyper, save=save)
    saved = out.saved if out.saved is not None else x.new_empty(0)
    return out.mean, out.var, out.flags, hyper, saved


@variational_fwd.register_fake
def _(x, Linv, Z, vmean, vstd, s2, ls, w, b0, jitter, save=False):
    B, N, D = x.shape
    return (x.new_empty(B, N), x.new_empty(B, N), x.new_empty(1, dtype=torch.int32),
            x.new_empty(4 + 2 * D), x.new_empty(_saved_numel(x, Z, save)))


@torch.library.custom_op("gpk::variational_adj", mutates_args=(), device_types="cuda")
def variational_adj(x: Tensor, Linv: Tensor, Z: Tensor, vmean: Tensor, vstd: Tensor, hyper: Tensor,
                    gmean: Tensor, gvar: Tensor, saved: Tensor) -> Tuple[Tensor, Tensor, Tensor, Tensor]:
    """-> (dX, dLinv, dZ (K_ZX part), dpar = [dvmean (M), dvstd (M), ds2, dls (D), dw (D), db0]).
    ``saved``: the forward's state (empty: recompute the forward inside the adjoint)."""
    adj = ops.variational_adjoint(x, Z, Linv, vmean, vstd, hyper, gmean, gvar,
                                  saved=saved if saved.numel() > 0 else None)
    return adj.dX, adj.dLinv, adj.dZ, adj.dpar


@variational_adj.register_fake
def _(x, Linv, Z, vmean, vstd, hyper, gmean, gvar, saved):
    M, D = Z.shape
    return (torch.empty_like(x), torch.empty_like(Linv), torch.empty_like(Z),
            x.new_empty(2 * M + 2 * D + 2))


def _var_setup(ctx, inputs, output):
    x, Linv, Z, vmean, vstd, s2, ls, w, b0, jitter = inputs[:10]
    ctx.save_for_backward(x, Linv, Z, vmean, vstd, s2, ls, w, b0, output[3], output[4])
    ctx.mark_non_differentiable(output[2], output[3], output[4])


def _var_backward(ctx, gmean, gvar, _gflags, _ghyper, _gsaved):
    x, Linv, Z, vmean, vstd, s2, ls, w, b0, hyper, saved = ctx.saved_tensors
    B, N, D = x.shape
    M = Z.shape[0]
    if gmean is None:
        gmean = x.new_zeros(B, N)
    if gvar is None:
        gvar = x.new_zeros(B, N)
    dX, dLinv, dZ, dpar = torch.ops.gpk.variational_adj(x, Linv, Z, vmean, vstd, hyper,
                                                        gmean.contiguous(), gvar.contiguous(), saved)
    dls = dpar[2 * M + 1:2 * M + 1 + D]
    dls = dls.sum().reshape(ls.shape) if ls.numel() == 1 else dls.reshape(ls.shape)
    return (dX, dLinv, dZ, dpar[:M].reshape(vmean.shape), dpar[M:2 * M].reshape(vstd.shape),
            dpar[2 * M].reshape(s2.shape), dls, dpar[2 * M + 1 + D:2 * M + 1 + 2 * D].reshape(w.shape),
            dpar[2 * M + 1 + 2 * D].reshape(b0.shape), None, None)


variational_fwd.register_autograd(_var_backward, setup_context=_var_setup)

# ---------------------------------------------------------------------------
# ELBO terms (gpk_gauss_ell_f32 / gpk_meanfield_kl_f32)
# ---------------------------------------------------------------------------


@torch.library.custom_op("gpk::gauss_ell", mutates_args=(), device_types="cuda")
def gauss_ell(y: Tensor, mean: Tensor, var: Tensor, noise: Tensor) -> Tensor:
    """(R,) sums over N of GaussianLikelihood.expected_log_prob for (R, N) rows."""
    return ops.gauss_ell(y.contiguous().float(), mean.contiguous().float(), var.contiguous().float(),
                         noise.reshape(1).contiguous().float())


@gauss_ell.register_fake
def _(y, mean, var, noise):
    return mean.new_empty(mean.shape[0])


@torch.library.custom_op("gpk::gauss_ell_grad", mutates_args=(), device_types="cuda")
def gauss_ell_grad(y: Tensor, mean: Tensor, var: Tensor, noise: Tensor,
                   gell: Tensor) -> Tuple[Tensor, Tensor, Tensor, Tensor]:
    return ops.gauss_ell_grad(y.contiguous().float(), mean.contiguous().float(), var.contiguous().float(),
                              noise.reshape(1).contiguous().float(), gell.contiguous().float())


@gauss_ell_grad.register_fake
def _(y, mean, var, noise, gell):
    return (torch.empty_like(mean), torch.empty_like(mean), torch.empty_like(mean), mean.new_empty(1))


def _ell_setup(ctx, inputs, output):
    ctx.save_for_backward(*inputs)


def _ell_backward(ctx, gell):
    y, mean, var, noise = ctx.saved_tensors
    dy, dmean, dvar, dnoise = torch.ops.gpk.gauss_ell_grad(y, mean, var, noise, gell.contiguous())
    return dy, dmean, dvar, dnoise.reshape(noise.shape)


gauss_ell.register_autograd(_ell_backward, setup_context=_ell_setup)


@torch.library.custom_op("gpk::meanfield_kl", mutates_args=(), device_types="cuda")
def meanfield_kl(m: Tensor, s: Tensor) -> Tensor:
    """(1,) KL(N(m, diag s^2) || N(0, I)) of the whitened mean-field q(u)."""
    return ops.meanfield_kl(m.contiguous().float(), s.contiguous().float())


@meanfield_kl.register_fake
def _(m, s):
    return m.new_empty(1)


@torch.library.custom_op("gpk::meanfield_kl_grad", mutates_args=(), device_types="cuda")
def meanfield_kl_grad(m: Tensor, s: Tensor, gkl: Tensor) -> Tuple[Tensor, Tensor]:
    return ops.meanfield_kl_grad(m.contiguous().float(), s.contiguous().float(), gkl.reshape(1).contiguous().float())


@meanfield_kl_grad.register_fake
def _(m, s, gkl):
    return torch.empty_like(m), torch.empty_like(s)


def _kl_setup(ctx, inputs, output):
    ctx.save_for_backward(*inputs)


def _kl_backward(ctx, gkl):
    m, s = ctx.saved_tensors
    dm, ds = torch.ops.gpk.meanfield_kl_grad(m, s, gkl)
    return dm, ds


meanfield_kl.register_autograd(_kl_backward, setup_context=_kl_setup)


@torch.library.custom_op("gpk::variational_elbo", mutates_args=(), device_types="cuda")
def variational_elbo(y: Tensor, mean: Tensor, var: Tensor, noise: Tensor, vmean: Tensor, vstd: Tensor,
                     kl_scale: float, min_var: float) -> Tuple[Tensor, Tensor]:
    """(R,) per-row ELBO ell_r / N - kl_scale KL(q(u)) and the variance-clamp flag (1,)."""
    return ops.variational_elbo(y, mean, var, noise.reshape(1).contiguous().float(), vmean, vstd, kl_scale,
                                min_var)


@variational_elbo.register_fake
def _(y, mean, var, noise, vmean, vstd, kl_scale, min_var):
    return mean.new_empty(mean.shape[0]), mean.new_empty(1, dtype=torch.int32)


@torch.library.custom_op("gpk::variational_elbo_grad", mutates_args=(), device_types="cuda")
def variational_elbo_grad(y: Tensor, mean: Tensor, var: Tensor, noise: Tensor, vmean: Tensor, vstd: Tensor,
                          kl_scale: float, gelbo: Tensor) -> Tuple[Tensor, Tensor, Tensor, Tensor, Tensor]:
    return ops.variational_elbo_grad(y, mean, var, noise.reshape(1).contiguous().float(), vmean, vstd,
                                     kl_scale, gelbo)


@variational_elbo_grad.register_fake
def _(y, mean, var, noise, vmean, vstd, kl_scale, gelbo):
    R, N = mean.shape
    return (mean.new_empty(R, N), mean.new_empty(R, N), mean.new_empty(1), torch.empty_like(vmean),
            torch.empty_like(vstd))


def _elbo_setup(ctx, inputs, output):
    y, mean, var, noise, vmean, vstd, kl_scale, min_var = inputs
    ctx.kl_scale = kl_scale
    ctx.save_for_backward(y, mean, var, noise, vmean, vstd)
    ctx.mark_non_differentiable(output[1])


def _elbo_backward(ctx, gelbo, _gflag):
    y, mean, var, noise, vmean, vstd = ctx.saved_tensors
    dmean, dvar, dnoise, dm, ds = torch.ops.gpk.variational_elbo_grad(y, mean, var, noise, vmean, vstd,
                                                                      ctx.kl_scale, gelbo.contiguous())
    return (None, dmean, dvar, dnoise.reshape(noise.shape), dm.reshape(vmean.shape), ds.reshape(vstd.shape),
            None, None)


variational_elbo.register_autograd(_elbo_backward, setup_context=_elbo_setup)
