"""Per-tile error map of the exact kernel's L vs the fp64 oracle (B=512 N=256: column plan)."""
import math, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np, torch
from fine_grained_gaussian_process_forcasting_amd import ops
from oracle import gp_oracle as O
B, N, D = 512, 256, 32
g = torch.Generator().manual_seed(0)
X = torch.randn(B, N, D, generator=g) / math.sqrt(D)
y = torch.randn(B, N, generator=torch.Generator().manual_seed(1))
LN2 = math.log(2)
out = ops.exact_mll(X.cuda(), y.cuda(), LN2, LN2, 0.0, LN2 + 1e-4, want_z=True)
torch.cuda.synchronize()
ref = O.exact_mll(X.double().numpy(), y.double().numpy(), LN2, LN2, 0.0, LN2 + 1e-4)
Lall = out.L.cpu().double().numpy()
werr = np.abs(Lall - ref.L).reshape(B, -1).max(1)
bad = np.nonzero(werr > 1e-5)[0]
print("bad windows:", len(bad), bad[:40].tolist(), "block%2:", np.bincount(bad % 2, minlength=2).tolist())
idx = bad[:3].tolist() or [0]
L = Lall[idx]
ref.L = ref.L[idx]
for n, b in enumerate(idx):
    e = np.abs(L[n] - ref.L[n]).reshape(16, 16, 16, 16).max(axis=(1, 3))
    print(f"window {b}: max err {e.max():.2e}")
    for i in range(16):
        print(" ".join("  .  " if e[i, j] < 1e-5 else f"{e[i, j]:.0e}" for j in range(16)))
