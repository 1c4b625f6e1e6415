"""Torch-facing launchers for the gfx950 GP kernels (no compute happens here).

Each function validates shapes/dtypes/devices on the host, allocates outputs with
torch (device memory, caller stream), and enqueues ONE C-ABI call on
``torch.cuda.current_stream()``. Tensors must live on a ROCm device; there is
no CPU path.
"""
from __future__ import annotations

import math
import warnings
from dataclasses import dataclass
from typing import Optional

import torch

from . import _native
from .errors import GpkInternalError, NanError, NotPSDError, NumericalWarning


def _require_device(*ts: torch.Tensor) -> None:
    for t in ts:
        if not t.is_cuda:
            raise ValueError("gpk ops run only on a ROCm device (tensor.is_cuda must be True); "
                             "there is no CPU fallback")


def _stream_ptr(device: torch.device) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def _scalar_tensor(v, device) -> torch.Tensor:
    if isinstance(v, torch.Tensor):
        return v.detach().reshape(-1).to(device=device, dtype=torch.float32)
    # a fill kernel, not a host->device copy: graph-capture safe
    return torch.full((1,), float(v), device=device, dtype=torch.float32)


def pack_exact_hyper(outputscale, noise, mean_constant, lengthscale, device) -> torch.Tensor:
    """Device vector {s2, noise, c, lengthscale...} consumed by gpk_exact_mll_f32."""
    parts = [_scalar_tensor(outputscale, device)[:1], _scalar_tensor(noise, device)[:1],
             _scalar_tensor(mean_constant, device)[:1], _scalar_tensor(lengthscale, device)]
    return torch.cat(parts).contiguous()


@dataclass
class ExactMLLOut:
    mll: torch.Tensor            # (B,)
    L: Optional[torch.Tensor]    # (B, N, N) lower Cholesky factor of K + noise I (+ jitter)
    z: Optional[torch.Tensor]    # (B, N)   L^{-1}(y - c)
    info: torch.Tensor           # (B,) int32 (0 / -t / k, see include/gpk.h)


EXACT_REG_MAX_N = 256   # largest N of the register / LDS-resident exact kernels (gpk_internal.h)


def exact_mll(X: torch.Tensor, y: torch.Tensor, lengthscale, outputscale, mean_constant, noise,
              jitter: float = 1e-6, max_tries: int = 3, want_L: bool = True,
              want_z: bool = False, hyper: Optional[torch.Tensor] = None,
              mll_out: Optional[torch.Tensor] = None, info_out: Optional[torch.Tensor] = None,
              L_out: Optional[torch.Tensor] = None) -> ExactMLLOut:
    """Fused exact-GP log marginal likelihood per window (one gfx950 kernel launch).

    X: (B, N, D) float32, y: (B, N) float32 on the same ROCm device. ``lengthscale``
    is a scalar or a length-D vector (ARD). Hyperparameters may be python floats or
    device tensors (no host sync either way). See include/gpk.h::gpk_exact_mll_f32.
    """
    if X.dim() != 3:
        raise ValueError(f"X must be (B, N, D), got {tuple(X.shape)}")
    B, N, D = X.shape
    if y.shape != (B, N):
        raise ValueError(f"y must be (B, N) = {(B, N)}, got {tuple(y.shape)}")
    _require_device(X, y)
    X = X.contiguous().float()
    y = y.contiguous().float()
    dev = X.device
    if hyper is None:
        hyper = pack_exact_hyper(outputscale, noise, mean_constant, lengthscale, dev)
    n_ls = hyper.numel() - 3
    if n_ls not in (1, D):
        raise ValueError(f"lengthscale must have 1 or D={D} entries, got {n_ls}")
    if mll_out is not None and (mll_out.shape != (B,) or mll_out.dtype != torch.float32
                                or not mll_out.is_contiguous() or mll_out.device != dev):
        raise ValueError("mll_out must be a contiguous (B,) float32 tensor on X's device")
    if info_out is not None and (info_out.shape != (B,) or info_out.dtype != torch.int32
                                 or not info_out.is_contiguous() or info_out.device != dev):
        raise ValueError("info_out must be a contiguous (B,) int32 tensor on X's device")
    mll = mll_out if mll_out is not None else torch.empty(B, device=dev, dtype=torch.float32)
    info = info_out if info_out is not None else torch.empty(B, device=dev, dtype=torch.int32)
    if L_out is not None and (L_out.shape != (B, N, N) or L_out.dtype != torch.float32
                              or not L_out.is_contiguous() or L_out.device != dev):
        raise ValueError("L_out must be a contiguous (B, N, N) float32 tensor on X's device")
    # Above EXACT_REG_MAX_N the blocked kernels (gpk_exact_large.hip) factor in place in L, so
    # it is allocated even when the caller does not keep it.
    need_L = want_L or N > EXACT_REG_MAX_N
    L = (L_out if L_out is not None else torch.empty(B, N, N, device=dev, dtype=torch.float32)) if need_L else None
    z = torch.empty(B, N, device=dev, dtype=torch.float32) if want_z else None
    rc = _native.lib().gpk_exact_mll_f32(
        X.data_ptr(), y.data_ptr(), hyper.data_ptr(), n_ls, B, N, D, float(jitter), int(max_tries),
        L.data_ptr() if L is not None else None, z.data_ptr() if z is not None else None,
        mll.data_ptr(), info.data_ptr(), _stream_ptr(dev))
    _native.check(rc, "gpk_exact_mll_f32")
    return ExactMLLOut(mll, L if want_L else None, z, info)


@dataclass
class ExactMLLGrad:
    dX: Optional[torch.Tensor]   # (B, N, D)
    dy: Optional[torch.Tensor]   # (B, N)
    dhyp: torch.Tensor           # (B, 3 + n_ls): per-window d/d{s2, noise, c, lengthscale...}


def exact_mll_grad(X: torch.Tensor, L: torch.Tensor, z: torch.Tensor, hyper: torch.Tensor,
                   gout: torch.Tensor, want_dX: bool = True, want_dy: bool = True) -> ExactMLLGrad:
    """Analytic backward of ``exact_mll`` (one gfx950 kernel launch, see
    include/gpk.h::gpk_exact_mll_grad_f32). ``L`` and ``z`` are the forward's outputs,
    ``gout`` (B,) the incoming gradient of each window's MLL."""
    B, N, D = X.shape
    _require_device(X, L, z, hyper, gout)
    X = X.contiguous().float()
    L = L.contiguous().float()
    z = z.contiguous().float()
    gout = gout.reshape(B).contiguous().float()
    dev = X.device
    n_ls = hyper.numel() - 3
    lib = _native.lib()
    ws = torch.empty(max(1, lib.gpk_exact_grad_workspace_bytes(B, N) // 4), device=dev,
                     dtype=torch.float32)
    dX = torch.empty(B, N, D, device=dev, dtype=torch.float32) if want_dX else None
    dy = torch.empty(B, N, device=dev, dtype=torch.float32) if want_dy else None
    dhyp = torch.empty(B, 3 + n_ls, device=dev, dtype=torch.float32)
    rc = lib.gpk_exact_mll_grad_f32(
        X.data_ptr(), L.data_ptr(), z.data_ptr(), hyper.data_ptr(), n_ls, B, N, D, gout.data_ptr(),
        ws.data_ptr(), dX.data_ptr() if dX is not None else None,
        dy.data_ptr() if dy is not None else None, dhyp.data_ptr(), _stream_ptr(dev))
    _native.check(rc, "gpk_exact_mll_grad_f32")
    return ExactMLLGrad(dX, dy, dhyp)


@dataclass
class ExactPosterior:
    mean: torch.Tensor   # (B, Ns) posterior mean of f
    var: torch.Tensor    # (B, Ns) posterior variance of f (unclamped)


def exact_posterior(X: torch.Tensor, L: torch.Tensor, z: torch.Tensor, hyper: torch.Tensor,
                    Xs: torch.Tensor) -> ExactPosterior:
    """Exact-GP posterior at the test inputs ``Xs`` (B, Ns, D) from the training factor
    ``L`` and ``z = L^{-1}(y - c)`` of ``exact_mll`` (one gfx950 kernel launch, see
    include/gpk.h::gpk_exact_posterior_f32). ``hyper`` is the exact path's device vector."""
    if X.dim() != 3 or Xs.dim() != 3:
        raise ValueError("X and Xs must be (B, N, D) and (B, Ns, D)")
    B, N, D = X.shape
    if Xs.shape[0] != B or Xs.shape[2] != D:
        raise ValueError(f"Xs must be (B, Ns, D) = ({B}, Ns, {D}), got {tuple(Xs.shape)}")
    if L.shape != (B, N, N) or z.shape != (B, N):
        raise ValueError("L / z do not match X")
    _require_device(X, L, z, hyper, Xs)
    X = X.detach().contiguous().float()
    Xs = Xs.detach().contiguous().float()
    L = L.detach().contiguous().float()
    z = z.detach().contiguous().float()
    Ns = Xs.shape[1]
    dev = X.device
    mean = torch.empty(B, Ns, device=dev, dtype=torch.float32)
    var = torch.empty(B, Ns, device=dev, dtype=torch.float32)
    rc = _native.lib().gpk_exact_posterior_f32(
        X.data_ptr(), L.data_ptr(), z.data_ptr(), hyper.data_ptr(), hyper.numel() - 3, Xs.data_ptr(),
        B, N, Ns, D, mean.data_ptr(), var.data_ptr(), _stream_ptr(dev))
    _native.check(rc, "gpk_exact_posterior_f32")
    return ExactPosterior(mean, var)


INFO_TIMEOUT = 1 << 20   # gpk_exact.hip kInfoTimeout: a bounded LDS spin-wait expired


class DeferredChecks:
    """Host-side verdicts recorded while a HIP graph is being captured.

    A captured step cannot read device memory on the host (the capture would break),
    so psd_safe_cholesky's info check and the variance-clamp flag are RECORDED instead.
    Each recorded check is condensed IN THE GRAPH into a 3-int verdict (max info,
    ladder steps, NaN in the inputs / clamp bit) by one gpk_record_check launch, written
    into slot ``replay % slots`` of a device ring; ``finalize()`` (captured at the end of
    the step) advances the replay counter. ``check(n)`` after n replays reads the ring with ONE device->host copy and
    warns / raises for each of the n replays in order, exactly as the eager calls would
    have -- so a block of ``slots`` replays costs one host sync, not one per check.
    """

    MAX_ITEMS = 16   # recorded checks per step (the cfg-3 step records 2-3)

    def __init__(self, device=None, slots: int = 1):
        self.items = []
        self.slots = max(1, int(slots))
        self.ring = None
        # (1,) int32 device flag: any hard failure since reset_sticky(); (1,) int64 replay
        # counter. Allocated before the capture (a tensor created inside it would be
        # re-zeroed by every replay)
        self.sticky = torch.zeros(1, dtype=torch.int32, device=device) if device is not None else None
        self.counter = torch.zeros(1, dtype=torch.int64, device=device) if device is not None else None
        self._ring = (torch.zeros(self.slots, self.MAX_ITEMS, 3, dtype=torch.int32, device=device)
                      if device is not None else None)
        self._keep = []   # tensors the recorded verdict launches read (kept alive with the graph)

    def add(self, kind: str, args: tuple) -> None:
        """Record a check; in a capture also its in-graph verdict (include/gpk.h::
        gpk_record_check: one small kernel per check, the ring slot of this replay)."""
        self.items.append((kind, args))
        if self.sticky is None:
            if kind == "cholesky":
                raise RuntimeError("DeferredChecks used in a capture without a device flag "
                                   "(construct it with device=...)")
            return
        if not self.sticky.is_cuda:   # host tensors (tests of the bookkeeping): torch ops
            if kind == "cholesky":
                self.sticky.copy_(torch.maximum(self.sticky, (args[0] > 0).any().to(torch.int32).reshape(1)))
            return
        item = len(self.items) - 1
        if item >= self.MAX_ITEMS:
            raise RuntimeError(f"more than {self.MAX_ITEMS} numerical checks recorded in one step")
        t = args[0]
        if kind == "cholesky":
            info = t.reshape(-1)
            ins = [x.detach().reshape(-1).float() for x in args[4] if x is not None][:2]
            ins = [x if x.is_contiguous() else x.contiguous() for x in ins]
            p = [(x.data_ptr(), x.numel()) for x in ins] + [(None, 0)] * (2 - len(ins))
            rc = _native.lib().gpk_record_check(info.data_ptr(), info.numel(), p[0][0], p[0][1], p[1][0],
                                                p[1][1], 0, self._ring.data_ptr(), self.counter.data_ptr(),
                                                self.slots, item, self.MAX_ITEMS, self.sticky.data_ptr(),
                                                _stream_ptr(info.device))
            self._keep.append(ins)
        else:
            flag = t.reshape(-1).to(torch.int32)
            rc = _native.lib().gpk_record_check(flag.data_ptr(), 1, None, 0, None, 0, 1, self._ring.data_ptr(),
                                                self.counter.data_ptr(), self.slots, item, self.MAX_ITEMS,
                                                None, _stream_ptr(flag.device))
            self._keep.append([flag])
        _native.check(rc, "gpk_record_check")

    def finalize(self) -> None:
        """Captured at the end of the step: advance the replay counter (the ring slot)."""
        if not self.items or self.counter is None or not self.counter.is_cuda:
            return
        rc = _native.lib().gpk_record_check(None, 0, None, 0, None, 0, 2, None, self.counter.data_ptr(),
                                            self.slots, 0, self.MAX_ITEMS, None,
                                            _stream_ptr(self.counter.device))
        _native.check(rc, "gpk_record_check")
        self.ring = self._ring[:, :len(self.items)]

    def reset_sticky(self) -> None:
        if self.sticky is not None:
            self.sticky.zero_()

    def _replay_verdicts(self, n: int):
        """Host copy of the last n replays' verdicts, oldest first (one sync)."""
        both = torch.cat([self.ring.reshape(-1).to(torch.int64), self.counter.reshape(-1)]).cpu()
        cnt = int(both[-1])
        ring = both[:-1].reshape(self.ring.shape)
        n = min(n, self.slots, cnt)
        return [ring[(cnt - n + r) % self.slots] for r in range(n)]

    def check(self, n: int = 1) -> None:
        if self.ring is None:        # nothing condensed (e.g. recorded outside GraphedStep)
            for kind, args in self.items:
                if kind == "cholesky":
                    info, jitter, what, max_tries, inputs = args
                    check_cholesky_info(info, jitter, inputs, what, max_tries)
                else:
                    from .gp import warn_if_clamped
                    warn_if_clamped(*args)
        else:
            for verdicts in self._replay_verdicts(n):
                for (kind, args), v in zip(self.items, verdicts.tolist()):
                    if kind == "cholesky":
                        _raise_or_warn_verdict(v, args[1], args[2], args[3])
                    elif v[0] & 1:
                        from .gp import warn_if_clamped
                        warn_if_clamped(torch.ones(1, dtype=torch.int32), args[1])
        if self.sticky is not None and int(self.sticky.item()) != 0:
            raise NotPSDError("a replay of this check block failed psd_safe_cholesky (not PD after "
                              "the jitter ladder, or NaN inputs); state rolled back to the block start")


def _raise_or_warn_verdict(v, jitter: float, what: str, max_tries: int) -> None:
    """check_cholesky_info from a condensed verdict [max info, ladder steps, NaN inputs]."""
    max_info, steps, nan = v
    if max_info >= INFO_TIMEOUT:
        raise GpkInternalError(f"{what}: kernel spin-wait timed out (info = 1<<20)")
    failed = max_info > 0
    if failed and nan:
        raise NanError(f"{what}: NaN elements in the inputs.")
    if failed:
        steps = max_tries
    for i in range(steps):
        warnings.warn(f"A not p.d., added jitter of {jitter * (10 ** i):.1e} to the diagonal",
                      NumericalWarning)
    if failed:
        raise NotPSDError(f"Matrix not positive definite after repeatedly adding jitter up to "
                          f"{jitter * 10 ** (max_tries - 1):.1e}.")


_RECORDERS: list = []


def record_or_run(kind: str, args: tuple, run) -> None:
    """Run a host-side check now, or record it when the current stream is capturing."""
    if torch.cuda.is_available() and torch.cuda.is_current_stream_capturing():
        if not _RECORDERS:
            raise RuntimeError("gpk: a HIP graph capture reached a host-side numerical check; "
                               "capture through graphs.GraphedStep, which defers the checks")
        _RECORDERS[-1].add(kind, args)
        return
    run()


def check_cholesky_info(info: torch.Tensor, jitter: float, inputs=(), what: str = "cholesky",
                        max_tries: int = 3) -> None:
    """GPyTorch's psd_safe_cholesky bookkeeping, from the per-window info codes.

    One device->host sync (GPyTorch pays the same: ``torch.any(info)``). Emits the
    same NumericalWarning text per ladder step and raises NanError / NotPSDError.
    When any window is still not PD, psd_safe_cholesky has walked the whole ladder
    (``max_tries`` warnings) before raising, whatever the other windows needed.
    Under HIP graph capture the check is recorded (DeferredChecks) instead.
    """
    if torch.cuda.is_available() and torch.cuda.is_current_stream_capturing():
        record_or_run("cholesky", (info, jitter, what, max_tries, tuple(inputs)), None)
        return
    info_h = info.detach().to("cpu")
    if not bool((info_h != 0).any()):
        return
    if bool((info_h >= INFO_TIMEOUT).any()):
        raise GpkInternalError(f"{what}: kernel spin-wait timed out (info = 1<<20) in windows "
                               f"{torch.nonzero(info_h >= INFO_TIMEOUT).flatten().tolist()[:16]}")
    failed = bool((info_h > 0).any())
    if failed:
        for t in inputs:
            if t is not None and bool(torch.isnan(t).any()):
                raise NanError(f"{what}: {int(torch.isnan(t).sum())} of {t.numel()} elements of the "
                               f"{tuple(t.shape)} tensor are NaN.")
    steps = int((-info_h[info_h < 0]).max()) if bool((info_h < 0).any()) else 0
    if failed:
        steps = max_tries
    for i in range(steps):
        warnings.warn(f"A not p.d., added jitter of {jitter * (10 ** i):.1e} to the diagonal",
                      NumericalWarning)
    if failed:
        raise NotPSDError(
            f"Matrix not positive definite after repeatedly adding jitter up to "
            f"{jitter * 10 ** (max_tries - 1):.1e}. Failing windows: "
            f"{torch.nonzero(info_h > 0).flatten().tolist()[:16]}")


LOG_2PI = math.log(2 * math.pi)


# ---------------------------------------------------------------------------
# Variational (DeepGP) path
# ---------------------------------------------------------------------------
@dataclass
class KzzFactor:
    L: torch.Tensor      # (M, M) float64 lower Cholesky factor of K_ZZ + jitter
    Linv: torch.Tensor   # (M, M) float64 L^{-1}
    info: torch.Tensor   # (1,) int32


def kzz_cholesky(Z: torch.Tensor, outputscale, lengthscale, jitter: float = 1e-4,
                 chol_jitter: float = 1e-8, max_tries: int = 3,
                 hyper: Optional[torch.Tensor] = None) -> KzzFactor:
    """Shared inducing-point factorisation (include/gpk.h::gpk_kzz_chol_f64)."""
    if Z.dim() != 2:
        raise ValueError(f"Z must be (M, D), got {tuple(Z.shape)}")
    _require_device(Z)
    Z = Z.detach().contiguous().float()
    M, D = Z.shape
    dev = Z.device
    if hyper is None:
        hyper = torch.cat([_scalar_tensor(outputscale, dev)[:1],
                           _scalar_tensor(lengthscale, dev).expand(D) if _scalar_tensor(lengthscale, dev).numel() == 1
                           else _scalar_tensor(lengthscale, dev)]).contiguous()
    if hyper.numel() != 1 + D:
        raise ValueError(f"kzz hyper must hold 1 + D = {1 + D} values, got {hyper.numel()}")
    L = torch.empty(M, M, device=dev, dtype=torch.float64)
    Linv = torch.empty(M, M, device=dev, dtype=torch.float64)
    info = torch.empty(1, device=dev, dtype=torch.int32)
    rc = _native.lib().gpk_kzz_chol_f64(Z.data_ptr(), hyper.data_ptr(), M, D, float(jitter),
                                        float(chol_jitter), int(max_tries), L.data_ptr(),
                                        Linv.data_ptr(), info.data_ptr(), _stream_ptr(dev))
    _native.check(rc, "gpk_kzz_chol_f64")
    return KzzFactor(L, Linv, info)


@dataclass
class VariationalOut:
    mean: torch.Tensor           # (B, N)
    var: torch.Tensor            # (B, N) clamped at 1e-6
    ell: Optional[torch.Tensor]  # (B,) sum over N of the expected log likelihood
    flags: Optional[torch.Tensor]  # (1,) int32: bit 0 = the variance clamp fired
    saved: Optional[torch.Tensor] = None  # training state for variational_adjoint (M > 64), or None


_CONST_PAIRS: dict = {}


def _const_pair(a: float, b: float, device) -> torch.Tensor:
    """Device tensor [a, b] for python-float hyper entries, cached per (device, a, b) so a
    step packs its hyper vector with ONE cat kernel. Never cached while a HIP graph is being
    captured (the tensor would live in the graph's private pool): GraphedStep's eager
    warm-up steps populate the cache first."""
    key = (str(torch.device(device)), float(a), float(b))
    t = _CONST_PAIRS.get(key)
    if t is not None:
        return t
    t = torch.stack([torch.full((), float(a), device=device), torch.full((), float(b), device=device)])
    if not (torch.cuda.is_available() and torch.cuda.is_current_stream_capturing()):
        _CONST_PAIRS[key] = t
    return t


def pack_variational_hyper(outputscale, noise, jitter, bias, weights, lengthscale, D, device):
    ls = _scalar_tensor(lengthscale, device)
    if ls.numel() == 1:
        ls = ls.expand(D)
    w = _scalar_tensor(weights, device).reshape(-1)
    if w.numel() != D:
        raise ValueError(f"LinearMean weights must have D={D} entries, got {w.numel()}")
    if not isinstance(noise, torch.Tensor) and not isinstance(jitter, torch.Tensor):
        mid = _const_pair(noise, jitter, device)
    else:
        mid = torch.cat([_scalar_tensor(noise, device)[:1], _scalar_tensor(jitter, device)[:1]])
    return torch.cat([_scalar_tensor(outputscale, device)[:1], mid, _scalar_tensor(bias, device)[:1],
                      w, ls]).contiguous()


def variational_forward(X: torch.Tensor, Z: torch.Tensor, Linv: torch.Tensor, vmean: torch.Tensor,
                        vstd: torch.Tensor, outputscale=None, noise=None, jitter=None, bias=None,
                        weights=None, lengthscale=None, y: Optional[torch.Tensor] = None,
                        hyper: Optional[torch.Tensor] = None, want_flags: bool = True,
                        save: bool = False) -> VariationalOut:
    """Batched q(f) mean / variance (+ expected log likelihood sum when y is given)
    for the whitened mean-field VariationalStrategy (include/gpk.h::gpk_variational_f32).
    ``save=True`` (training): where the saved-state adjoint serves the shape (M > 64), the
    forward also keeps A = Linv K_ZX and the clamp mask (gpk_variational_train_f32) in
    ``out.saved`` for ``variational_adjoint(..., saved=out.saved)``; None elsewhere."""
    if X.dim() != 3:
        raise ValueError(f"X must be (B, N, D), got {tuple(X.shape)}")
    B, N, D = X.shape
    M = Z.shape[0]
    if Z.shape != (M, D):
        raise ValueError(f"Z must be (M, {D}), got {tuple(Z.shape)}")
    if Linv.shape != (M, M) or Linv.dtype != torch.float64:
        raise ValueError("Linv must be (M, M) float64 from kzz_cholesky")
    _require_device(X, Z, Linv, vmean, vstd)
    dev = X.device
    X = X.detach().contiguous().float()
    Z = Z.detach().contiguous().float()
    Linv = Linv.detach().contiguous()
    vmean = vmean.detach().contiguous().float().reshape(-1)
    vstd = vstd.detach().contiguous().float().reshape(-1)
    if hyper is None:
        hyper = pack_variational_hyper(outputscale, noise, jitter, bias, weights, lengthscale, D, dev)
    if y is not None:
        if y.shape != (B, N):
            raise ValueError(f"y must be (B, N) = {(B, N)}, got {tuple(y.shape)}")
        _require_device(y)
        y = y.detach().contiguous().float()
    mean = torch.empty(B, N, device=dev, dtype=torch.float32)
    var = torch.empty(B, N, device=dev, dtype=torch.float32)
    ell = torch.empty(B, device=dev, dtype=torch.float32) if y is not None else None
    flags = torch.empty(1, device=dev, dtype=torch.int32) if want_flags else None
    lib = _native.lib()
    nsaved = lib.gpk_variational_saved_bytes(B, N, M, D) if (save and B > 0) else 0
    if nsaved > 0:
        saved = torch.empty(nsaved // 4, device=dev, dtype=torch.float32)
        rc = lib.gpk_variational_train_f32(
            X.data_ptr(), Z.data_ptr(), Linv.data_ptr(), vmean.data_ptr(), vstd.data_ptr(),
            hyper.data_ptr(), y.data_ptr() if y is not None else None, B, N, M, D,
            mean.data_ptr(), var.data_ptr(), ell.data_ptr() if ell is not None else None,
            flags.data_ptr() if flags is not None else None, saved.data_ptr(), _stream_ptr(dev))
        _native.check(rc, "gpk_variational_train_f32")
        return VariationalOut(mean, var, ell, flags, saved)
    rc = lib.gpk_variational_f32(
        X.data_ptr(), Z.data_ptr(), Linv.data_ptr(), vmean.data_ptr(), vstd.data_ptr(),
        hyper.data_ptr(), y.data_ptr() if y is not None else None, B, N, M, D,
        mean.data_ptr(), var.data_ptr(), ell.data_ptr() if ell is not None else None,
        flags.data_ptr() if flags is not None else None, _stream_ptr(dev))
    _native.check(rc, "gpk_variational_f32")
    return VariationalOut(mean, var, ell, flags)


@dataclass
class VariationalAdjoint:
    dX: torch.Tensor      # (B, N, D)
    dLinv: torch.Tensor   # (M, M) float64, lower: sum over points of dA K_ZX^T
    dpar: torch.Tensor    # (2M + 2D + 2,) the packed parameter gradients below
    dZ: torch.Tensor      # (M, D) the K_ZX part of dZ
    dvmean: torch.Tensor  # (M,)
    dvstd: torch.Tensor   # (M,)
    ds2: torch.Tensor     # () K_ZX + variance parts
    dls: torch.Tensor     # (D,) the K_ZX part
    dw: torch.Tensor      # (D,) LinearMean weights
    db0: torch.Tensor     # () LinearMean bias


def variational_adjoint(X: torch.Tensor, Z: torch.Tensor, Linv: torch.Tensor, vmean: torch.Tensor,
                        vstd: torch.Tensor, hyper: torch.Tensor, gmean: torch.Tensor,
                        gvar: torch.Tensor, saved: Optional[torch.Tensor] = None) -> VariationalAdjoint:
    """Adjoint of ``variational_forward`` except the shared K_ZZ factor (fused gfx950
    kernels behind include/gpk.h::gpk_variational_adjoint_f32; from the training forward's
    ``saved`` state: gpk_variational_adjoint_saved_f32)."""
    B, N, D = X.shape
    M = Z.shape[0]
    _require_device(X, Z, Linv, vmean, vstd, hyper, gmean, gvar)
    dev = X.device
    X = X.detach().contiguous().float()
    Z = Z.detach().contiguous().float()
    Linv = Linv.detach().contiguous().double()
    vmean = vmean.detach().reshape(M).contiguous().float()
    vstd = vstd.detach().reshape(M).contiguous().float()
    gmean = gmean.detach().reshape(B, N).contiguous().float()
    gvar = gvar.detach().reshape(B, N).contiguous().float()
    lib = _native.lib()
    if saved is not None:
        # the C entry point receives a bare pointer: the dtype and device are checked here
        if saved.dtype != torch.float32 or saved.device != dev:
            raise ValueError(f"saved state must be float32 on {dev} (got {saved.dtype} on {saved.device}): "
                             f"pass variational_forward(save=True).saved unchanged")
        if saved.numel() * 4 != lib.gpk_variational_saved_bytes(B, N, M, D):
            raise ValueError("saved state does not match this shape (variational_forward(save=True))")
        nbytes = lib.gpk_variational_adjoint_saved_workspace_bytes(B, N, M, D)
    else:
        nbytes = lib.gpk_variational_adjoint_workspace_bytes(B, N, M, D)
    if nbytes == 0:
        raise ValueError(f"unsupported variational shape B={B} N={N} M={M} D={D}")
    ws = torch.empty(nbytes, device=dev, dtype=torch.uint8)
    dX = torch.empty(B, N, D, device=dev, dtype=torch.float32)
    dLinv = torch.empty(M, M, device=dev, dtype=torch.float64)
    dZ = torch.empty(M, D, device=dev, dtype=torch.float32)
    dpar = torch.empty(2 * M + 2 * D + 2, device=dev, dtype=torch.float32)
    if saved is not None:
        _require_device(saved)
        rc = lib.gpk_variational_adjoint_saved_f32(
            X.data_ptr(), Z.data_ptr(), Linv.data_ptr(), vmean.data_ptr(), vstd.data_ptr(),
            hyper.data_ptr(), gmean.data_ptr(), gvar.data_ptr(), saved.detach().contiguous().data_ptr(),
            B, N, M, D, ws.data_ptr(), dX.data_ptr(), dLinv.data_ptr(), dZ.data_ptr(), dpar.data_ptr(),
            _stream_ptr(dev))
        _native.check(rc, "gpk_variational_adjoint_saved_f32")
    else:
        rc = lib.gpk_variational_adjoint_f32(
            X.data_ptr(), Z.data_ptr(), Linv.data_ptr(), vmean.data_ptr(), vstd.data_ptr(),
            hyper.data_ptr(), gmean.data_ptr(), gvar.data_ptr(), B, N, M, D, ws.data_ptr(),
            dX.data_ptr(), dLinv.data_ptr(), dZ.data_ptr(), dpar.data_ptr(), _stream_ptr(dev))
        _native.check(rc, "gpk_variational_adjoint_f32")
    return VariationalAdjoint(dX, dLinv, dpar, dZ, dpar[:M], dpar[M:2 * M], dpar[2 * M],
                              dpar[2 * M + 1:2 * M + 1 + D], dpar[2 * M + 1 + D:2 * M + 1 + 2 * D],
                              dpar[2 * M + 1 + 2 * D])


def kzz_backward(dLinv: torch.Tensor, L: torch.Tensor, Linv: torch.Tensor, Z: torch.Tensor,
                 outputscale: torch.Tensor, lengthscale: torch.Tensor):
    """Back-propagate dObjective/dLinv (lower, fp64) through Linv = chol(K_ZZ + jitter)^{-1}
    to (dZ, d outputscale, d lengthscale): once per optimizer step for all GP calls that
    shared the factor (include/gpk.h::gpk_kzz_backward_f64: five fp64-MFMA tile GEMMs
    Lbar = -tril(Linv^T G Linv^T), S = Linv^T Phi(L^T Lbar) Linv, then the RBF adjoint over
    K_ZZ with Kbar = (S + S^T)/2). Returns (dZ (M, D) float, ds2 (), dls (D,)) -- dls per
    dimension even for a shared lengthscale (the caller sums)."""
    M, D = Z.shape
    _require_device(dLinv, L, Linv, Z)
    dev = Z.device
    ls = lengthscale.detach().reshape(-1).float()
    hyper = torch.cat([outputscale.detach().reshape(1).float(), ls.expand(D) if ls.numel() == 1 else ls])
    lib = _native.lib()
    ws = torch.empty(lib.gpk_kzz_backward_workspace_bytes(M, D), device=dev, dtype=torch.uint8)
    dZ = torch.empty(M, D, device=dev, dtype=torch.float32)
    dhyp = torch.empty(1 + D, device=dev, dtype=torch.float32)
    rc = lib.gpk_kzz_backward_f64(dLinv.detach().contiguous().double().data_ptr(),
                                  L.detach().contiguous().data_ptr(), Linv.detach().contiguous().data_ptr(),
                                  Z.detach().contiguous().float().data_ptr(), hyper.data_ptr(), M, D,
                                  ws.data_ptr(), dZ.data_ptr(), dhyp.data_ptr(), _stream_ptr(dev))
    _native.check(rc, "gpk_kzz_backward_f64")
    return dZ, dhyp[0], dhyp[1:]


# ---------------------------------------------------------------------------
# ELBO terms (gpk_gauss_ell_f32 / gpk_meanfield_kl_f32)
# ---------------------------------------------------------------------------
def gauss_ell(y: torch.Tensor, mean: torch.Tensor, var: torch.Tensor, noise: torch.Tensor) -> torch.Tensor:
    """Per-row sum of GaussianLikelihood.expected_log_prob for (R, N) rows (one launch)."""
    R, N = mean.shape
    _require_device(y, mean, var, noise)
    dev = mean.device
    ell = torch.empty(R, device=dev, dtype=torch.float32)
    rc = _native.lib().gpk_gauss_ell_f32(y.data_ptr(), mean.data_ptr(), var.data_ptr(), noise.data_ptr(),
                                         R, N, ell.data_ptr(), _stream_ptr(dev))
    _native.check(rc, "gpk_gauss_ell_f32")
    return ell


def gauss_ell_grad(y, mean, var, noise, gell):
    """(dy, dmean, dvar, dnoise (1,)) of sum_r gell_r ell_r (one launch + one sum)."""
    R, N = mean.shape
    _require_device(y, mean, var, noise, gell)
    dev = mean.device
    dy = torch.empty(R, N, device=dev, dtype=torch.float32)
    dmean = torch.empty(R, N, device=dev, dtype=torch.float32)
    dvar = torch.empty(R, N, device=dev, dtype=torch.float32)
    part = torch.empty(R, device=dev, dtype=torch.float32)
    rc = _native.lib().gpk_gauss_ell_grad_f32(y.data_ptr(), mean.data_ptr(), var.data_ptr(), noise.data_ptr(),
                                              gell.data_ptr(), R, N, dy.data_ptr(), dmean.data_ptr(),
                                              dvar.data_ptr(), part.data_ptr(), _stream_ptr(dev))
    _native.check(rc, "gpk_gauss_ell_grad_f32")
    return dy, dmean, dvar, part.sum().reshape(1)


def meanfield_kl(m: torch.Tensor, s: torch.Tensor) -> torch.Tensor:
    """KL(N(m, diag s^2) || N(0, I)) as a (1,) tensor (one launch)."""
    _require_device(m, s)
    kl = torch.empty(1, device=m.device, dtype=torch.float32)
    rc = _native.lib().gpk_meanfield_kl_f32(m.data_ptr(), s.data_ptr(), m.numel(), kl.data_ptr(), None,
                                            None, None, _stream_ptr(m.device))
    _native.check(rc, "gpk_meanfield_kl_f32")
    return kl


def meanfield_kl_grad(m, s, gkl):
    _require_device(m, s, gkl)
    dm = torch.empty_like(m)
    ds = torch.empty_like(s)
    rc = _native.lib().gpk_meanfield_kl_f32(m.data_ptr(), s.data_ptr(), m.numel(), None, gkl.data_ptr(),
                                            dm.data_ptr(), ds.data_ptr(), _stream_ptr(m.device))
    _native.check(rc, "gpk_meanfield_kl_f32")
    return dm, ds


def _rows(t: torch.Tensor):
    """(tensor, leading dimension) of a (R, N) float32 view with unit column stride."""
    if t.dim() != 2 or t.stride(1) != 1 or t.dtype != torch.float32:
        t = t.contiguous().float()
    return t, (t.stride(0) if t.shape[0] > 1 else t.shape[1])


def variational_elbo(y, mean, var, noise, vmean, vstd, kl_scale: float, min_var: float):
    """(elbo (R,), clamp flag (1,) int32) of include/gpk.h::gpk_variational_elbo_f32."""
    _require_device(y, mean, var, noise, vmean, vstd)
    R, N = mean.shape
    y, ldy = _rows(y)
    mean, ldm = _rows(mean)
    var, ldv = _rows(var)
    dev = mean.device
    elbo = torch.empty(R, device=dev, dtype=torch.float32)
    flag = torch.empty(1, device=dev, dtype=torch.int32)
    m = vmean.detach().reshape(-1).contiguous().float()
    s = vstd.detach().reshape(-1).contiguous().float()
    rc = _native.lib().gpk_variational_elbo_f32(y.data_ptr(), ldy, mean.data_ptr(), ldm, var.data_ptr(), ldv,
                                                noise.data_ptr(), m.data_ptr(), s.data_ptr(), m.numel(), R, N,
                                                float(kl_scale), float(min_var), elbo.data_ptr(), flag.data_ptr(),
                                                _stream_ptr(dev))
    _native.check(rc, "gpk_variational_elbo_f32")
    return elbo, flag


def variational_elbo_grad(y, mean, var, noise, vmean, vstd, kl_scale: float, gelbo):
    """(dmean, dvar, dnoise (1,), dvmean, dvstd) for the objective sum_r gelbo_r elbo_r."""
    R, N = mean.shape
    y, ldy = _rows(y)
    mean, ldm = _rows(mean)
    var, ldv = _rows(var)
    dev = mean.device
    m = vmean.detach().reshape(-1).contiguous().float()
    s = vstd.detach().reshape(-1).contiguous().float()
    dmean = torch.empty(R, N, device=dev, dtype=torch.float32)
    dvar = torch.empty(R, N, device=dev, dtype=torch.float32)
    part = torch.empty(R, device=dev, dtype=torch.float32)
    dm = torch.empty_like(m)
    ds = torch.empty_like(s)
    g = gelbo.reshape(-1).contiguous().float()
    rc = _native.lib().gpk_variational_elbo_grad_f32(y.data_ptr(), ldy, mean.data_ptr(), ldm, var.data_ptr(),
                                                     ldv, noise.data_ptr(), m.data_ptr(), s.data_ptr(), m.numel(),
                                                     R, N, float(kl_scale), g.data_ptr(), dmean.data_ptr(),
                                                     dvar.data_ptr(), part.data_ptr(), dm.data_ptr(),
                                                     ds.data_ptr(), _stream_ptr(dev))
    _native.check(rc, "gpk_variational_elbo_grad_f32")
    return dmean, dvar, part.sum().reshape(1), dm, ds
