"""Negative control of the GPK_EPOCH_CHECK build (gpk_exact_dev.h): the GPK_EPOCH_CHECK=2
build marks one panel tile of step 3 with a wrong epoch, so every consumer of it must report
the mismatch -- each window of the column-plan launch (N = 256, B = 512) ends with
info = 1<<20 (ops raises GpkInternalError). Run with GPK_LIB=.../_lib_ab/epoch2/libgpk.so."""
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from fine_grained_gaussian_process_forcasting_amd import ops  # noqa: E402

dev = torch.device("cuda", 0)
g = torch.Generator().manual_seed(0)
B, N, D = 512, 256, 32
X = (torch.randn(B, N, D, generator=g) / math.sqrt(D)).to(dev)
y = torch.randn(B, N, generator=g).to(dev)
h = ops.pack_exact_hyper(math.log(2), math.log(2) + 1e-4, 0.0, math.log(2), dev)
out = ops.exact_mll(X, y, None, None, None, None, hyper=h)
info = out.info.cpu()
n_bad = int((info == ops.INFO_TIMEOUT).sum())
print(f"lib={os.environ.get('GPK_LIB')} windows={B} flagged={n_bad}")
assert n_bad == B, "the epoch check did not fire on the sabotaged tile"
print("EPOCH_NEGATIVE_OK")
