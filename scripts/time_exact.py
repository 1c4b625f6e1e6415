"""Kernel time of gpk_exact_mll_f32 at one shape from the libgpk.so that GPK_LIB names (or the
in-tree build): bench.py runs it as a child process for the measurement-only variant builds
(build_native.VARIANTS). Prints one JSON line {"kernel_ms": ..., "mll_mean": ...}.

    GPK_LIB=.../_lib_variants/f32update/libgpk.so python scripts/time_exact.py B N D steps
"""
import json
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from fine_grained_gaussian_process_forcasting_amd import ops  # noqa: E402

B, N, D, steps = (int(v) for v in sys.argv[1:5])
dev = torch.device("cuda:0")
g = torch.Generator().manual_seed(1000)
X = (torch.randn(B, N, D, generator=g) / math.sqrt(D)).to(dev)
y = torch.randn(B, N, generator=torch.Generator().manual_seed(1001)).to(dev)
LN2 = math.log(2.0)
hyper = ops.pack_exact_hyper(LN2, LN2 + 1e-4, 0.0, LN2, dev)
L = torch.empty(B, N, N, device=dev)
f = lambda: ops.exact_mll(X, y, None, None, None, None, hyper=hyper, L_out=L)  # noqa: E731
for _ in range(5):
    out = f()
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(steps):
    out = f()
e1.record()
torch.cuda.synchronize()
assert bool((out.info == 0).all())
print(json.dumps({"kernel_ms": e0.elapsed_time(e1) / steps, "mll_mean": float(out.mll.mean())}))
