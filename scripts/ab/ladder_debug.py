"""Debug: the jitter ladder in both layouts: per-window info codes (debug builds decode timeouts)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np, torch
from fine_grained_gaussian_process_forcasting_amd import ops
dev = torch.device("cuda:0")
def dec(v):
    if v < (1 << 30):
        return v
    return dict(wk_att=(v >> 26) & 15, diag_att=(v >> 22) & 15, sync=(v >> 16) & 63, tgt=(v >> 8) & 255, idx=v & 255)
for B in (8, 300):
    N, D = 256, 8
    g = torch.Generator().manual_seed(21)
    X = torch.randn(B, N, D, generator=g) / np.sqrt(D)
    y = torch.randn(B, N, generator=g)
    dup = [3] + ([100, 257] if B > 257 else [])
    for b in dup:
        X[b] = X[b, :1].expand(N, D)
    for rep in range(3):
        out = ops.exact_mll(X.to(dev), y.to(dev), 0.3, 1.0, 0.0, 0.0, want_z=True)
        torch.cuda.synchronize()
        info = out.info.cpu().numpy()
        bad = [(b, dec(int(info[b]))) for b in range(B) if info[b] != 0]
        print("B", B, "rep", rep, "nonzero info:", bad[:20], flush=True)
