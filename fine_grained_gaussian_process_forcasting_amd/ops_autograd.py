"""Differentiable entry points of the gfx950 hot-path kernels.

Every forward and backward goes through the ``gpk::*`` torch.library custom ops
(library.py), i.e. through libgpk.so: the exact path's backward is the analytic HIP
adjoint gpk_exact_mll_grad_f32 (Cholesky / TRSM / RBF adjoints in one kernel); the
variational path's backward is the fused HIP adjoint gpk_variational_adjoint_f32
(recomputed K_ZX and A = L^-1 K_ZX, dA, L^-T dA, the RBF adjoint contractions and
dL^-1 = sum dA K_ZX^T as a split-K fp64-MFMA GEMM), and the shared K_ZZ factor is ONE
autograd node per step (gpk::kzz_factor) whose M x M adjoint runs once for all the GP
calls that used it. Nothing here runs on the CPU.
"""
from __future__ import annotations

import math
import weakref
from typing import Optional

import torch

from . import library  # noqa: F401  (registers the gpk:: ops)
from . import ops

LOG_2PI = math.log(2.0 * math.pi)

# Every factor / prediction cache of the package (objects with .clear()). Their keys
# are tensor version counters, which a HIP graph replay does not bump, so
# graphs.GraphedStep clears them all after each replay.
_CACHES: "weakref.WeakSet" = weakref.WeakSet()


def register_cache(obj) -> None:
    _CACHES.add(obj)


def invalidate_caches() -> None:
    for c in list(_CACHES):
        c.clear()


def exact_log_prob(X, y, lengthscale, outputscale, constant, noise) -> torch.Tensor:
    """Per-window exact-GP log marginal likelihood / N (fused HIP kernel forward, analytic
    HIP backward). The hyper vector is packed differentiably, so gpk::exact_mll's
    gradient reaches s2, noise, c and the lengthscale(s)."""
    hyper = torch.cat([outputscale.reshape(1), noise.reshape(1), constant.reshape(1),
                       lengthscale.reshape(-1)]).float()
    need = torch.is_grad_enabled() and any(t.requires_grad for t in (X, y, hyper))
    mll, _, _, info = torch.ops.gpk.exact_mll(X.float(), y.float(), hyper, 1e-6, 3, bool(need))
    ops.check_cholesky_info(info, 1e-6, inputs=(X, y))
    return mll


class KzzCache:
    """Per-VariationalStrategy cache of the shared K_ZZ factor.

    Keyed on the identity and version counters of the inducing points and the raw
    kernel hyper-parameters plus the jitter. Training: the enc and dec GP calls of a
    step (denoise_model_2.py:50-51) share one factorisation and one K_ZZ adjoint; a
    gradient hook marks the entry spent once the step's backward reaches it, and the
    next call refactors. Eval (no grad): the factor is reused across batches until a
    parameter changes, as GPyTorch's eval-mode ``cholesky_factor`` cache
    (train.py:197-213, evaluate.py:127-137). Entries are per model instance, so
    concurrent Optuna threads (train.py:86) never share one.
    """

    def __init__(self):
        self._entry = None
        register_cache(self)

    def clear(self):
        self._entry = None

    @staticmethod
    def _key(tensors, jitter):
        return tuple((t.data_ptr(), t._version, tuple(t.shape), str(t.device)) for t in tensors) + (float(jitter),)

    def factor(self, Z, s2, ls, jitter, key_tensors):
        key = self._key(key_tensors, jitter)
        grad = torch.is_grad_enabled() and (Z.requires_grad or s2.requires_grad or ls.requires_grad)
        e = self._entry
        if e is not None and e["key"] == key and e["grad"] == grad and not e["spent"]:
            return e["Linv"]
        Linv, _, info = torch.ops.gpk.kzz_factor(Z, s2, ls, float(jitter), 1e-8, 3)
        entry = {"key": key, "grad": grad, "Linv": Linv, "spent": False, "info": info, "Z": Z}
        if grad:
            def _spent(g, entry=entry):
                entry["spent"] = True        # this step's backward consumed the node
                return g
            Linv.register_hook(_spent)
        self._entry = entry
        return Linv

    def note_consumers(self, *outputs):
        """Mark the current grad-mode entry spent as soon as ANY backward pass reaches an
        output computed from it -- also an ``autograd.grad`` over a subset of inputs that
        stops short of the factor (the factor's own hook never fires then), so the next
        forward refactors instead of reusing a factor whose consumers' graph was freed."""
        e = self._entry
        if e is None or not e["grad"]:
            return

        def _spent(g, entry=e):
            entry["spent"] = True
            return g
        for t in outputs:
            if isinstance(t, torch.Tensor) and t.requires_grad:
                t.register_hook(_spent)

    def check_pending(self):
        """psd_safe_cholesky's verdict on a freshly computed factor (one host sync). Called
        after the first kernel that consumes the factor has been queued, so the GPU is
        not idle while the host waits; raises / warns exactly as GPyTorch during the call."""
        e = self._entry
        if e is not None and e.get("info") is not None:
            info, Z = e["info"], e["Z"]
            e["info"] = None
            e["Z"] = None
            ops.check_cholesky_info(info, 1e-8, inputs=(Z,), what="K_ZZ cholesky")


def _mean_params(mean_module, D, device):
    """(w, b0) of the kernel's mean x.w + b0 (DeepGP.py:42-45): LinearMean as is;
    ConstantMean c as w = 0 (no gradient), b0 = c, so d/dc = sum of the mean gradient."""
    if hasattr(mean_module, "weights"):
        w = mean_module.weights.reshape(-1)
        b0 = mean_module.bias.reshape(()) if mean_module.bias is not None else torch.zeros((), device=device)
        return w, b0
    if hasattr(mean_module, "constant"):
        return torch.zeros(D, device=device), mean_module.constant.reshape(())
    raise NotImplementedError(f"mean module {type(mean_module).__name__} is not on the reference path "
                              "(DeepGP.py:42-45: ConstantMean or LinearMean)")


def variational_predict(x, Z, vmean, vstd, outputscale, lengthscale, mean_module, jitter,
                        cache: Optional[KzzCache] = None, key_tensors=None, return_linv: bool = False):
    """q(f) mean / variance / clamp flag for (B, N, D) windows (HIP forward and backward;
    see module docstring). ``cache`` shares the K_ZZ factor between calls; ``return_linv``
    appends the factor's L^{-1} (for a lazily materialised covariance)."""
    w, b0 = _mean_params(mean_module, x.shape[-1], x.device)
    s2 = outputscale.reshape(())
    ls = lengthscale.reshape(-1)
    if cache is None or key_tensors is None:
        # no caller-held parameters to key on: a fresh, private factor (keys on derived
        # temporaries could alias reused allocator memory and return a stale factor)
        cache = KzzCache()
        key_tensors = (Z, s2, ls)
    Linv = cache.factor(Z, s2, ls, jitter, key_tensors)
    # training (a gradient will flow): the forward keeps A for the saved-state adjoint
    save = torch.is_grad_enabled() and any(t.requires_grad for t in (x, Linv, Z, vmean, vstd, s2, ls, w, b0))
    mean, var, flags, _, _ = torch.ops.gpk.variational_fwd(x, Linv, Z, vmean, vstd, s2, ls, w, b0,
                                                           float(jitter), save)
    cache.note_consumers(mean, var)
    cache.check_pending()
    if return_linv:
        return mean, var, flags, Linv
    return mean, var, flags
