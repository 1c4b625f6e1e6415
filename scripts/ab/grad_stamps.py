"""Per-step timeline of the exact backward's solve kernel from a GPK_GRAD_STAMPS=1 build
(GPK_LIB): python scripts/ab/grad_stamps.py  (B=512 N=256 D=32). Timing tool only."""
import math, os, sys
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from fine_grained_gaussian_process_forcasting_amd import ops

B, N, D, NB, W = 512, 256, 32, 16, 16
dev = torch.device("cuda", 0)
g = torch.Generator().manual_seed(0)
X = (torch.randn(B, N, D, generator=g) / math.sqrt(D)).to(dev)
y = torch.randn(B, N, generator=g).to(dev)
h = ops.pack_exact_hyper(math.log(2), math.log(2) + 1e-4, 0.0, math.log(2), dev)
f = ops.exact_mll(X, y, None, None, None, None, hyper=h, want_L=True, want_z=True)
gout = torch.ones(B, device=dev)
for _ in range(3):
    gr = ops.exact_mll_grad(X, f.L, f.z, h, gout)
torch.cuda.synchronize()
st = gr.dX.contiguous().view(torch.int64).view(B, -1)[:, :2 * NB * W * 4].cpu().numpy()
st = st.reshape(B, 2 * NB, W, 4).astype(np.float64)
st -= st.reshape(B, -1).min(1)[:, None, None, None]
tot = st.reshape(B, -1).max(1)
print(f"window span (s_memtime ticks, 100 MHz): mean {tot.mean():.0f}")
m = st.mean(0)   # (steps, waves, 4)
print(" s | start(w0) math(w0) math(max) math(w15) bar-pass put(w0) | step len")
for s in range(2 * NB):
    w0 = m[s, 0]
    nxt = m[s + 1, 0, 0] if s + 1 < 2 * NB else m[s, :, 3].max()
    print(f"{s:2d} | {w0[0]:8.0f} {w0[1]-w0[0]:7.0f} {np.max(m[s, :, 1] - m[s, :, 0]):8.0f} {m[s,15,1]-m[s,15,0]:8.0f}"
          f" {m[s, :, 2].mean() - m[s, :, 1].max():8.0f} {w0[3]-w0[2]:7.0f} | {nxt - w0[0]:7.0f}")
