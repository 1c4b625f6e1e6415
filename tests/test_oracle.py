"""CPU: pin the oracle (closed forms, independent torch.linalg restatement, fixtures)."""
import math
import os
import warnings

import numpy as np
import pytest
import torch

from oracle import gp_oracle as O

LN2 = math.log(2.0)
GOLD = os.path.join(os.path.dirname(__file__), "golden")


def test_softplus_init_values():
    assert abs(O.softplus(0.0) - LN2) < 1e-15
    assert abs(O.softplus(0.0) + 1e-4 - 0.693247) < 1e-6       # GaussianLikelihood init noise
    assert abs(O.inv_softplus(O.softplus(0.37)) - 0.37) < 1e-12


def test_known_answer_n1():
    X = np.zeros((1, 1, 3))
    y = np.array([[0.7]])
    r = O.exact_mll(X, y, 0.5, 0.8, 0.1, 0.3)
    v = 1.1
    assert abs(r.L[0, 0, 0] - math.sqrt(v)) < 1e-14
    want = -0.5 * (0.36 / v + math.log(v) + math.log(2 * math.pi))
    assert abs(r.mll[0] - want) < 1e-14


def test_known_answer_n2_closed_form():
    x = np.array([[[0.0], [1.0]]])
    y = np.array([[0.3, -0.4]])
    ls, s2, noise = 0.8, 1.5, 0.2
    k = s2 * math.exp(-0.5 * (1.0 / ls) ** 2)
    a = s2 + noise
    L11, L21 = math.sqrt(a), k / math.sqrt(a)
    L22 = math.sqrt(a - L21 ** 2)
    r = O.exact_mll(x, y, ls, s2, 0.0, noise)
    assert np.allclose(r.L[0], [[L11, 0], [L21, L22]], atol=1e-14)
    K = np.array([[a, k], [k, a]])
    inv_quad = y[0] @ np.linalg.solve(K, y[0])
    want = -0.5 * (inv_quad + math.log(np.linalg.det(K)) + 2 * math.log(2 * math.pi)) / 2
    assert abs(r.mll[0] - want) < 1e-13


def test_known_answer_identity_kernel():
    X = np.arange(40 * 3, dtype=np.float64).reshape(1, 40, 3) * 10
    r = O.exact_mll(X, np.ones((1, 40)), 0.01, 0.8, 0.0, 0.2)
    assert np.allclose(r.L[0], np.eye(40), atol=1e-12)


def test_jitter_ladder_duplicates_fp32():
    X = np.zeros((2, 5, 3), np.float32)
    with warnings.catch_warnings(record=True) as w:
        warnings.simplefilter("always")
        r = O.exact_mll(X, np.ones((2, 5), np.float32), 1.0, 1.0, 0.0, 0.0, dtype=np.float32)
    assert (r.info == -1).all()
    assert any("added jitter of 1.0e-06" in str(x.message) for x in w)


def test_not_psd_raises():
    X = np.random.default_rng(0).standard_normal((1, 8, 2))
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        with pytest.raises(O.NotPSDError):
            O.exact_mll(X, np.ones((1, 8)), 1.0, 1.0, 0.0, -5.0)


def test_nan_raises():
    X = np.random.default_rng(0).standard_normal((1, 8, 2))
    X[0, 2, 1] = np.nan
    with pytest.raises(O.NanError):
        O.exact_mll(X, np.ones((1, 8)), 1.0, 1.0, 0.0, 0.1)


def test_kl_at_prior_is_zero():
    assert abs(O.kl_meanfield(np.zeros(16), np.ones(16))) < 1e-15
    m, s = np.array([0.3, -0.1]), np.array([0.7, 1.2])
    want = 0.5 * ((s ** 2).sum() + (m ** 2).sum() - 2 - np.log(s ** 2).sum())
    assert abs(O.kl_meanfield(m, s) - want) < 1e-15


def test_sq_dist_matches_direct():
    rng = np.random.default_rng(1)
    a, b = rng.standard_normal((7, 4)), rng.standard_normal((9, 4))
    direct = ((a[:, None, :] - b[None, :, :]) ** 2).sum(-1)
    assert np.allclose(O.sq_dist(a, b, False, False), direct, atol=1e-12)


def test_oracle_vs_torch_linalg_restatement():
    """Independent restatement (torch CPU, the kernels GPyTorch dispatches to)."""
    rng = np.random.default_rng(2)
    X = rng.standard_normal((5, 48, 6)) / math.sqrt(6)
    y = rng.standard_normal((5, 48))
    r = O.exact_mll(X, y, LN2, LN2, 0.1, LN2 + 1e-4)
    L, mll = O.exact_mll_torch_cpu(torch.from_numpy(X), torch.from_numpy(y), LN2, LN2, 0.1, LN2 + 1e-4)
    assert np.allclose(L.numpy(), r.L, atol=1e-12)
    assert np.allclose(mll.numpy(), r.mll, atol=1e-12)


def test_variational_oracle_self_consistency():
    """A = L^-1 K_ZX must satisfy L A = K_ZX; var formula vs explicit matrices."""
    rng = np.random.default_rng(4)
    X = rng.standard_normal((2, 10, 3))
    Z = rng.standard_normal((6, 3))
    m, s = rng.standard_normal(6) * 1e-3, rng.uniform(0.5, 1.0, 6)
    ls, w = np.full(3, 0.9), rng.standard_normal(3)
    r = O.variational_forward(X, Z, ls, 1.2, w, 0.3, m, s, jitter=1e-4, dtype=np.float64)
    Kzx = O.rbf(np.broadcast_to(Z, (2, 6, 3)), X, ls, 1.2)
    assert np.allclose(np.einsum('ij,bjn->bin', r.L_zz, r.A), Kzx, atol=1e-12)
    S = np.diag(s ** 2)
    for b in range(2):
        cov = 1.2 + 1e-4 + np.diag(r.A[b].T @ (S - np.eye(6)) @ r.A[b])
        assert np.allclose(r.var[b], cov, atol=1e-12)


@pytest.mark.parametrize("name", ["exact_B4_N16_D4", "exact_B2_N128_D32", "exact_B3_N37_D5_ard_like"])
def test_golden_exact(name):
    d = np.load(os.path.join(GOLD, name + ".npz"))
    ls, s2, c, noise = d["hyper"]
    r = O.exact_mll(d["X"].astype(np.float64), d["y"].astype(np.float64), ls, s2, c, noise)
    assert np.allclose(r.L, d["L"], atol=1e-12)
    assert np.allclose(r.mll, d["mll"], atol=1e-12)
    assert np.allclose(r.z, d["z"], atol=1e-10)


@pytest.mark.parametrize("name", ["var_B3_N20_M8_D4", "var_B2_N64_M16_D8"])
def test_golden_variational(name):
    d = np.load(os.path.join(GOLD, name + ".npz"))
    r = O.variational_forward(d["X"].astype(np.float64), d["Z"].astype(np.float64), d["ls"], float(d["s2"]),
                              d["w"].astype(np.float64), float(d["b0"]), d["m"].astype(np.float64),
                              d["s"].astype(np.float64), jitter=float(d["jitter"]), dtype=np.float64)
    assert np.allclose(r.mean, d["mean"], atol=1e-12)
    assert np.allclose(r.var, d["var"], atol=1e-12)
    elbo = O.deep_elbo(d["y"].astype(np.float64), r.mean, r.var, float(d["noise"]), d["m"], d["s"],
                       num_data=d["X"].shape[-1])
    assert np.allclose(elbo, d["elbo"], atol=1e-12)


def _fd(f, x, h=1e-6):
    return (f(x + h) - f(x - h)) / (2 * h)


def test_variational_grads_vs_finite_differences():
    """Pin the gradient oracle: central differences of the NumPy fp64 forward."""
    rng = np.random.default_rng(3)
    B, N, M, D = 2, 7, 5, 3
    X = rng.standard_normal((B, N, D)) / math.sqrt(D)
    Z = rng.standard_normal((M, D)) / math.sqrt(D)
    ls = np.array([0.7, 0.9, 1.1]); s2 = 0.8
    w = rng.standard_normal(D); b0 = 0.3
    m = rng.standard_normal(M) * 0.5; s = rng.uniform(0.5, 1.0, M)
    gm = rng.standard_normal((B, N)); gv = rng.standard_normal((B, N))
    G = O.variational_grads(X, Z, ls, s2, w, b0, m, s, gm, gv)

    def obj(X=X, Z=Z, ls=ls, s2=s2, w=w, b0=b0, m=m, s=s):
        r = O.variational_forward(X, Z, ls, s2, w, b0, m, s, jitter=1e-4, dtype=np.float64)
        return float((gm * r.mean).sum() + (gv * r.var).sum())

    def bump(a, idx, h):
        a = np.array(a, dtype=np.float64, copy=True); a[idx] += h; return a
    checks = [
        (G["outputscale"], _fd(lambda h: obj(s2=s2 + h), 0.0)),
        (G["bias"], _fd(lambda h: obj(b0=b0 + h), 0.0)),
        (G["lengthscale"][1], _fd(lambda h: obj(ls=bump(ls, 1, h)), 0.0)),
        (G["Z"][2, 1], _fd(lambda h: obj(Z=bump(Z, (2, 1), h)), 0.0)),
        (G["X"][1, 4, 2], _fd(lambda h: obj(X=bump(X, (1, 4, 2), h)), 0.0)),
        (G["m"][3], _fd(lambda h: obj(m=bump(m, 3, h)), 0.0)),
        (G["s"][0], _fd(lambda h: obj(s=bump(s, 0, h)), 0.0)),
        (G["weights"][2], _fd(lambda h: obj(w=bump(w, 2, h)), 0.0)),
    ]
    for got, want in checks:
        assert abs(got - want) <= 1e-6 * max(1.0, abs(want)), (got, want)


def test_exact_grads_vs_finite_differences():
    rng = np.random.default_rng(4)
    B, N, D = 2, 9, 3
    X = rng.standard_normal((B, N, D)) / math.sqrt(D)
    y = rng.standard_normal((B, N))
    ls, s2, c, nz = 0.8, 1.2, 0.1, 0.3
    gout = np.array([0.7, -1.3])
    G = O.exact_mll_grads(X, y, ls, s2, c, nz, gout)

    def obj(X=X, y=y, ls=ls, s2=s2, c=c, nz=nz):
        return float((gout * O.exact_mll(X, y, ls, s2, c, nz).mll).sum())

    def bump(a, idx, h):
        a = np.array(a, dtype=np.float64, copy=True); a[idx] += h; return a
    checks = [
        (G["outputscale"], _fd(lambda h: obj(s2=s2 + h), 0.0)),
        (G["noise"], _fd(lambda h: obj(nz=nz + h), 0.0)),
        (G["mean_constant"], _fd(lambda h: obj(c=c + h), 0.0)),
        (G["lengthscale"][0], _fd(lambda h: obj(ls=ls + h), 0.0)),
        (G["X"][1, 3, 2], _fd(lambda h: obj(X=bump(X, (1, 3, 2), h)), 0.0)),
        (G["y"][0, 5], _fd(lambda h: obj(y=bump(y, (0, 5), h)), 0.0)),
    ]
    for got, want in checks:
        assert abs(got - want) <= 1e-6 * max(1.0, abs(want)), (got, want)
