"""Phase clocks of a GPK_KZZ_STAMPS=1 build (GPK_LIB): Linv[0][1..9] =
prologue, tile build, phase 1, phase 2, zero fill, then phase-1 step parts
(publish+barrier, chol+l rows, barrier, update) summed over steps.
   python scripts/kzz_stamps.py [M] [D]"""
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fine_grained_gaussian_process_forcasting_amd import ops  # noqa: E402

M, D = (int(v) for v in (sys.argv[1:] + ["256", "32"])[:2])
LN2 = math.log(2.0)
dev = torch.device("cuda", 0)
g = torch.Generator().manual_seed(0)
Z = (torch.randn(M, D, generator=g) / math.sqrt(D)).to(dev)
kz_h = torch.cat([torch.tensor([LN2]), torch.full((D,), LN2)]).to(dev)
for _ in range(3):
    kz = ops.kzz_cholesky(Z, None, None, jitter=1e-4, hyper=kz_h)
torch.cuda.synchronize()
v = kz.Linv[0, 1:10].cpu().tolist()
names = ["prologue", "build", "phase1", "phase2", "zero", "p1.publish", "p1.chol_rows", "p1.barrier2", "p1.update"]
print(f"M={M} D={D} info={int(kz.info[0])} " + " ".join(f"{n}={x:.0f}" for n, x in zip(names, v)), flush=True)
