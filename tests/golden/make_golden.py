"""Regenerate the golden fixtures of tests/golden/ from the fp64 oracle.

No reference-generated vectors exist for this path (GPyTorch is not installed and
the reference ships no tests), so these fixtures pin the ORACLE
(CPU restatement of GPyTorch 1.9.x, oracle/gp_oracle.py) against future edits;
the oracle itself is pinned by the closed-form cases in tests/test_oracle.py.
Run:  python tests/golden/make_golden.py
"""
import math
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from oracle import gp_oracle as O  # noqa: E402

LN2 = math.log(2.0)


def exact_case(name, B, N, D, seed, ls=LN2, s2=LN2, c=0.0, noise=LN2 + 1e-4):
    rng = np.random.default_rng(seed)
    X = (rng.standard_normal((B, N, D)) / math.sqrt(D)).astype(np.float32)
    y = rng.standard_normal((B, N)).astype(np.float32)
    r = O.exact_mll(X.astype(np.float64), y.astype(np.float64), ls, s2, c, noise)
    np.savez_compressed(os.path.join(HERE, f"{name}.npz"), X=X, y=y,
                        hyper=np.array([ls, s2, c, noise]), L=r.L, z=r.z, mll=r.mll, info=r.info)


def variational_case(name, B, N, M, D, seed, trained):
    rng = np.random.default_rng(seed)
    X = (rng.standard_normal((B, N, D)) / math.sqrt(D)).astype(np.float32)
    Z = (rng.standard_normal((M, D)) / math.sqrt(D)).astype(np.float32)
    m = (1e-3 * rng.standard_normal(M)).astype(np.float32)
    s = (rng.uniform(0.5, 1.0, M) if trained else np.ones(M)).astype(np.float32)
    w = rng.standard_normal(D).astype(np.float32)
    b0 = np.float32(rng.standard_normal())
    y = rng.standard_normal((B, N)).astype(np.float32)
    ls = np.full(D, LN2)
    r = O.variational_forward(X.astype(np.float64), Z.astype(np.float64), ls, LN2, w.astype(np.float64),
                              float(b0), m.astype(np.float64), s.astype(np.float64), jitter=1e-4,
                              dtype=np.float64)
    noise = LN2 + 1e-4
    elbo = O.deep_elbo(y.astype(np.float64), r.mean, r.var, noise, m, s, num_data=D)
    np.savez_compressed(os.path.join(HERE, f"{name}.npz"), X=X, Z=Z, m=m, s=s, w=w, b0=b0, y=y,
                        ls=ls, s2=LN2, noise=noise, jitter=1e-4, mean=r.mean, var=r.var,
                        L_zz=r.L_zz, elbo=elbo)


if __name__ == "__main__":
    exact_case("exact_B4_N16_D4", 4, 16, 4, seed=11)
    exact_case("exact_B2_N128_D32", 2, 128, 32, seed=12)
    exact_case("exact_B3_N37_D5_ard_like", 3, 37, 5, seed=13, ls=1.3, s2=0.9, c=0.25, noise=0.05)
    variational_case("var_B3_N20_M8_D4", 3, 20, 8, 4, seed=21, trained=False)
    variational_case("var_B2_N64_M16_D8", 2, 64, 16, 8, seed=22, trained=True)
    print("fixtures written to", HERE)
