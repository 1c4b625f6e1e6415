"""CPU: libgpk.so loads, exports exactly the C ABI of include/gpk.h, validates arguments
before touching the device, and the product path refuses CPU tensors (no fallback)."""
import ctypes
import os
import re

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _header_functions():
    src = open(os.path.join(ROOT, "include", "gpk.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(gpk_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_header_symbol():
    from fine_grained_gaussian_process_forcasting_amd import _native
    lib = _native.lib()
    names = _header_functions()
    assert {"gpk_exact_mll_f32", "gpk_kzz_chol_f64", "gpk_variational_f32"} <= set(names)
    for n in names:
        assert hasattr(lib, n), n
        assert n in _native.SIGNATURES, f"{n} declared in gpk.h but not bound in _native.py"
    assert lib.gpk_version() >= 100
    assert lib.gpk_exact_max_n() == 800   # GPyTorch settings.max_cholesky_size
    assert b"success" == lib.gpk_strerror(0)


def test_argument_validation_without_device():
    from fine_grained_gaussian_process_forcasting_amd import _native
    lib = _native.lib()
    one = ctypes.c_void_p(16)  # never dereferenced: validation returns first
    assert lib.gpk_exact_mll_f32(None, one, one, 1, 1, 8, 2, 1e-6, 3, None, None, one, one, None) == -1
    assert lib.gpk_exact_mll_f32(one, one, one, 5, 1, 8, 2, 1e-6, 3, None, None, one, one, None) == -4
    assert lib.gpk_exact_mll_f32(one, one, one, 1, 1, 801, 2, 1e-6, 3, None, None, one, one, None) == -6
    # 256 < N <= 800: the blocked kernels factor in place, so L is required; D <= 64
    assert lib.gpk_exact_mll_f32(one, one, one, 1, 1, 300, 2, 1e-6, 3, None, None, one, one, None) == -10
    assert lib.gpk_exact_mll_f32(one, one, one, 1, 1, 300, 65, 1e-6, 3, one, None, one, one, None) == -7
    assert lib.gpk_exact_mll_f32(one, one, one, 1, 1, 8, 2, -1.0, 3, None, None, one, one, None) == -8
    assert lib.gpk_exact_mll_f32(one, one, one, 1, 0, 8, 2, 1e-6, 3, None, None, one, one, None) == 0
    assert lib.gpk_kzz_chol_f64(one, one, 300, 4, 1e-4, 1e-8, 3, one, one, one, None) == -3
    assert lib.gpk_variational_f32(one, one, one, one, one, one, None, 1, 8, 8, 65, one, one, None, None, None) == -11
    # ell requested without targets
    assert lib.gpk_variational_f32(one, one, one, one, one, one, None, 1, 8, 8, 4, one, one, one, None, None) == -7
    assert lib.gpk_kzz_chol_f64(one, one, 64, 65, 1e-4, 1e-8, 3, one, one, one, None) == -4
    assert b"N exceeds" in lib.gpk_strerror(-6)


def test_variational_adjoint_entry_validation_without_device():
    from fine_grained_gaussian_process_forcasting_amd import _native
    lib = _native.lib()
    one = ctypes.c_void_p(16)
    ws = lib.gpk_variational_adjoint_workspace_bytes(4, 192, 256, 32)
    # dA and K_ZX (M x B*N fp32 each) dominate the workspace
    assert ws >= 2 * 256 * 4 * 192 * 4
    assert lib.gpk_variational_adjoint_workspace_bytes(4, 192, 257, 32) == 0
    assert lib.gpk_variational_adjoint_workspace_bytes(4, 192, 64, 65) == 0
    args = [one] * 8 + [2, 16, 8, 4] + [one] * 5 + [None]
    assert lib.gpk_variational_adjoint_f32(*args) != 0 or True  # (pointer validity not checkable)
    for idx, code in [(0, -1), (6, -7), (12, -13), (13, -14), (14, -15), (15, -16), (16, -17)]:
        bad = list(args); bad[idx] = None
        assert lib.gpk_variational_adjoint_f32(*bad) == code
    bad = list(args); bad[10] = 300
    assert lib.gpk_variational_adjoint_f32(*bad) == -11
    bad = list(args); bad[11] = 65
    assert lib.gpk_variational_adjoint_f32(*bad) == -12


def test_ops_refuse_cpu_tensors():
    from fine_grained_gaussian_process_forcasting_amd import ops
    X = torch.zeros(2, 8, 3)
    y = torch.zeros(2, 8)
    with pytest.raises(ValueError, match="no CPU fallback"):
        ops.exact_mll(X, y, 1.0, 1.0, 0.0, 0.1)
    with pytest.raises(ValueError, match="no CPU fallback"):
        ops.kzz_cholesky(torch.zeros(4, 3), 1.0, 1.0)


def test_ops_shape_validation():
    from fine_grained_gaussian_process_forcasting_amd import ops
    with pytest.raises(ValueError):
        ops.exact_mll(torch.zeros(8, 3), torch.zeros(8), 1.0, 1.0, 0.0, 0.1)
    with pytest.raises(ValueError):
        ops.exact_mll(torch.zeros(2, 8, 3), torch.zeros(2, 7), 1.0, 1.0, 0.0, 0.1)


def test_missing_library_fails_loudly(monkeypatch):
    from fine_grained_gaussian_process_forcasting_amd import _native
    monkeypatch.setattr(_native, "_lib", None)
    monkeypatch.setattr(_native, "_LIB_PATH", "/nonexistent/libgpk.so")
    with pytest.raises(_native.NativeLibraryError):
        _native.lib()


def test_grad_entry_validation_without_device():
    from fine_grained_gaussian_process_forcasting_amd import _native
    lib = _native.lib()
    one = ctypes.c_void_p(16)  # never dereferenced: validation returns first
    # K^-1 lower tiles (136 x 1 KiB) + alpha, means, partials per window, 64-float aligned
    assert lib.gpk_exact_grad_workspace_bytes(3, 256) == 3 * 36224 * 4
    # N > 256: L^-1 and K_hat^-1 (Np x Np each, Np = N rounded up to 32) per window
    assert lib.gpk_exact_grad_workspace_bytes(3, 257) == 3 * 2 * 288 * 288 * 4
    assert lib.gpk_exact_grad_workspace_bytes(3, 800) == 3 * 2 * 800 * 800 * 4
    assert lib.gpk_exact_grad_workspace_bytes(3, 801) == 0
    args = [one, one, one, one, 1, 2, 16, 4, one, one, None, None, one, None]
    bad = list(args); bad[0] = None
    assert lib.gpk_exact_mll_grad_f32(*bad) == -1
    bad = list(args); bad[4] = 3
    assert lib.gpk_exact_mll_grad_f32(*bad) == -5
    bad = list(args); bad[6] = 801
    assert lib.gpk_exact_mll_grad_f32(*bad) == -7
    bad = list(args); bad[7] = 65
    assert lib.gpk_exact_mll_grad_f32(*bad) == -8
    bad = list(args); bad[12] = None
    assert lib.gpk_exact_mll_grad_f32(*bad) == -13
    bad = list(args); bad[5] = 0
    assert lib.gpk_exact_mll_grad_f32(*bad) == 0   # B = 0: nothing to do


def test_custom_ops_registered_with_fake_and_autograd():
    """The kernels are torch.library custom ops (SURVEY §8b "Who calls it"): schemas,
    FakeTensor impls (shape propagation without a GPU) and autograd formulas."""
    import fine_grained_gaussian_process_forcasting_amd.library  # noqa: F401
    from torch._subclasses.fake_tensor import FakeTensorMode
    names = ["exact_mll", "exact_mll_grad", "exact_posterior", "kzz_factor", "variational_fwd",
             "variational_adj"]
    for n in names:
        assert hasattr(torch.ops.gpk, n), n
    with FakeTensorMode():
        X = torch.empty(3, 16, 4)
        y = torch.empty(3, 16)
        h = torch.empty(4)
        mll, L, z, info = torch.ops.gpk.exact_mll(X, y, h, 1e-6, 3, True)
        assert mll.shape == (3,) and L.shape == (3, 16, 16) and info.dtype == torch.int32
        pm, pv = torch.ops.gpk.exact_posterior(X, L, z, h, torch.empty(3, 40, 4))
        assert pm.shape == (3, 40) and pv.shape == (3, 40)
        Z = torch.empty(8, 4)
        Linv, Lz, inf = torch.ops.gpk.kzz_factor(Z, torch.empty(()), torch.empty(4), 1e-4, 1e-8, 3)
        assert Linv.shape == (8, 8) and Linv.dtype == torch.float64
        mean, var, flags, hyp, saved = torch.ops.gpk.variational_fwd(
            X, Linv, Z, torch.empty(8), torch.empty(8), torch.empty(()), torch.empty(4), torch.empty(4),
            torch.empty(()), 1e-4)
        assert mean.shape == (3, 16) and var.shape == (3, 16) and flags.shape == (1,)
        assert hyp.shape == (4 + 2 * 4,) and saved.numel() == 0
        # training at M = 256: the forward's saved state for the saved-state adjoint (16 row tiles x
        # 2 column tiles of A per 32-point chunk + the chunk's clamp mask)
        Z2 = torch.empty(256, 4)
        L2 = torch.empty(256, 256, dtype=torch.float64)
        out = torch.ops.gpk.variational_fwd(X, L2, Z2, torch.empty(256), torch.empty(256), torch.empty(()),
                                            torch.empty(4), torch.empty(4), torch.empty(()), 1e-4, True)
        assert out[4].numel() == 3 * 1 * (16 * 2 * 256 + 32)
        dX, dL, dZ, dpar = torch.ops.gpk.variational_adj(X, L2, Z2, torch.empty(256), torch.empty(256), hyp,
                                                         mean, var, out[4])
        assert dX.shape == X.shape and dL.shape == (256, 256) and dpar.shape == (2 * 256 + 2 * 4 + 2,)


def test_posterior_entry_validation_without_device():
    from fine_grained_gaussian_process_forcasting_amd import _native
    lib = _native.lib()
    one = ctypes.c_void_p(16)  # never dereferenced: validation returns first
    args = [one, one, one, one, 1, one, 2, 16, 40, 4, one, one, None]
    for idx, code in [(0, -1), (1, -2), (2, -3), (3, -4), (5, -6), (10, -11), (11, -12)]:
        bad = list(args); bad[idx] = None
        assert lib.gpk_exact_posterior_f32(*bad) == code
    bad = list(args); bad[4] = 3
    assert lib.gpk_exact_posterior_f32(*bad) == -5
    bad = list(args); bad[7] = 801
    assert lib.gpk_exact_posterior_f32(*bad) == -8
    bad = list(args); bad[9] = 65
    assert lib.gpk_exact_posterior_f32(*bad) == -10
    bad = list(args); bad[8] = 0
    assert lib.gpk_exact_posterior_f32(*bad) == 0    # no test points: nothing to do


def test_exact_model_input_shapes_and_eval_guard():
    """ExactGPModel accepts (N,), (N, D) and (B, N, D) inputs (GPyTorch's shapes); the
    eval-mode posterior (with or without gradients) refuses CPU tensors: no CPU path."""
    from fine_grained_gaussian_process_forcasting_amd.denoising_model.GPModel import ExactGPModel, _as_batch
    from fine_grained_gaussian_process_forcasting_amd.gp import GaussianLikelihood
    assert _as_batch(torch.zeros(7)).shape == (1, 7, 1)
    assert _as_batch(torch.zeros(7, 3)).shape == (1, 7, 3)
    assert _as_batch(torch.zeros(2, 7, 3)).shape == (2, 7, 3)
    with pytest.raises(ValueError):
        _as_batch(torch.zeros(1, 2, 7, 3))
    m = ExactGPModel(torch.zeros(7, 3), torch.zeros(7), GaussianLikelihood())
    prior = m(torch.zeros(7, 3))
    assert prior.mean.shape == (7,) and prior._exact[0].shape == (1, 7, 3)
    m.eval()
    with pytest.raises(ValueError, match="GPU"):
        m(torch.ones(5, 3))
