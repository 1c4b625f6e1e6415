"""ctypes binding of libgpk.so — the C ABI declared in include/gpk.h.

The shared library is built in-tree by ``build_native.py`` (``__graft_entry__.build``)
and is the ONLY compute path of this package: if it is missing or fails to load,
every op raises ``NativeLibraryError``; there is no CPU or eager fallback.
"""
from __future__ import annotations

import ctypes
import os
import threading

# GPK_LIB overrides the in-tree build (A/B experiments with build_native.py --out-dir).
_LIB_PATH = os.environ.get("GPK_LIB") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "_lib",
                                                       "libgpk.so")
_lock = threading.Lock()
_lib = None

c_float_p = ctypes.c_void_p  # device pointers are passed as raw addresses
c_int = ctypes.c_int
c_double = ctypes.c_double
c_void_p = ctypes.c_void_p
c_size_t = ctypes.c_size_t

# name -> (restype, argtypes); must mirror include/gpk.h exactly.
SIGNATURES = {
    "gpk_version": (c_int, []),
    "gpk_strerror": (ctypes.c_char_p, [c_int]),
    "gpk_exact_max_n": (c_int, []),
    "gpk_exact_mll_f32": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int,
                                  c_double, c_int, c_void_p, c_void_p, c_void_p, c_void_p,
                                  c_void_p]),
    "gpk_exact_grad_workspace_bytes": (c_size_t, [c_int, c_int]),
    "gpk_exact_mll_grad_f32": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int,
                                       c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                       c_void_p]),
    "gpk_exact_posterior_f32": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_int,
                                        c_int, c_int, c_int, c_void_p, c_void_p, c_void_p]),
    "gpk_kzz_chol_f64": (c_int, [c_void_p, c_void_p, c_int, c_int, ctypes.c_float, c_double, c_int,
                                 c_void_p, c_void_p, c_void_p, c_void_p]),
    "gpk_kzz_backward_workspace_bytes": (c_size_t, [c_int, c_int]),
    "gpk_kzz_backward_f64": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int,
                                     c_void_p, c_void_p, c_void_p, c_void_p]),
    "gpk_gauss_ell_f32": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_void_p,
                                  c_void_p]),
    "gpk_gauss_ell_grad_f32": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int,
                                       c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "gpk_meanfield_kl_f32": (c_int, [c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_void_p,
                                     c_void_p]),
    "gpk_variational_elbo_f32": (c_int, [c_void_p, ctypes.c_longlong, c_void_p, ctypes.c_longlong, c_void_p, ctypes.c_longlong, c_void_p, c_void_p,
                                         c_void_p, c_int, c_int, c_int, ctypes.c_float, ctypes.c_float,
                                         c_void_p, c_void_p, c_void_p]),
    "gpk_variational_elbo_grad_f32": (c_int, [c_void_p, ctypes.c_longlong, c_void_p, ctypes.c_longlong, c_void_p, ctypes.c_longlong, c_void_p,
                                              c_void_p, c_void_p, c_int, c_int, c_int, ctypes.c_float,
                                              c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                              c_void_p]),
    "gpk_record_check": (c_int, [c_void_p, c_int, c_void_p, ctypes.c_longlong, c_void_p, ctypes.c_longlong,
                                 c_int, c_void_p, c_void_p, c_int, c_int, c_int, c_void_p, c_void_p]),
    "gpk_variational_f32": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                    c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_void_p,
                                    c_void_p, c_void_p, c_void_p]),
    "gpk_variational_adjoint_workspace_bytes": (c_size_t, [c_int, c_int, c_int, c_int]),
    "gpk_variational_adjoint_f32": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                            c_void_p, c_void_p, c_void_p, c_int, c_int, c_int,
                                            c_int, c_void_p, c_void_p, c_void_p, c_void_p,
                                            c_void_p, c_void_p]),
    "gpk_variational_saved_bytes": (c_size_t, [c_int, c_int, c_int, c_int]),
    "gpk_variational_train_f32": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                          c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_void_p,
                                          c_void_p, c_void_p, c_void_p, c_void_p]),
    "gpk_variational_adjoint_saved_workspace_bytes": (c_size_t, [c_int, c_int, c_int, c_int]),
    "gpk_variational_adjoint_saved_f32": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                                  c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int,
                                                  c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p,
                                                  c_void_p, c_void_p]),
    "gpk_window_gather_f32": (c_int, [c_void_p, ctypes.c_longlong, c_int, c_void_p, c_int, c_int, c_int,
                                      c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p]),
}
DEBUG_SIGNATURES = {
    "gpk_debug_exact_stamps": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int,
                                       c_double, c_int, c_void_p, c_void_p, c_void_p, c_void_p,
                                       c_void_p, c_void_p]),
}


class NativeLibraryError(RuntimeError):
    pass


class GpkError(RuntimeError):
    """Non-zero return code from a gpk_* entry point."""


def library_path() -> str:
    return _LIB_PATH


def lib():
    """Load libgpk.so once (thread-safe) and bind every symbol of include/gpk.h."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(_LIB_PATH):
            raise NativeLibraryError(
                f"libgpk.so not found at {_LIB_PATH}; run `python build_native.py` "
                "(or __graft_entry__.build()). There is no fallback path.")
        try:
            handle = ctypes.CDLL(_LIB_PATH)
        except OSError as e:  # pragma: no cover - depends on the box
            raise NativeLibraryError(f"failed to load {_LIB_PATH}: {e}") from e
        for name, (res, args) in {**SIGNATURES, **DEBUG_SIGNATURES}.items():
            fn = getattr(handle, name)
            fn.restype = res
            fn.argtypes = args
        _lib = handle
        return _lib


def check(rc: int, what: str) -> None:
    if rc != 0:
        msg = lib().gpk_strerror(rc).decode()
        raise GpkError(f"{what} failed with code {rc}: {msg}")
