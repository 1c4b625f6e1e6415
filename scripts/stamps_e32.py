"""Diagnostic: per-step timeline of the 32-column exact kernel (STAMPS build), N=256 D=32."""
import math, sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from fine_grained_gaussian_process_forcasting_amd import _native, ops

B, N, D = int(sys.argv[1]) if len(sys.argv) > 1 else 512, 256, 32
dev = torch.device("cuda:0")
X = (torch.randn(B, N, D) / math.sqrt(D)).to(dev)
y = torch.randn(B, N).to(dev)
LN2 = math.log(2)
hyp = ops.pack_exact_hyper(LN2, LN2 + 1e-4, 0.0, LN2, dev)
L = torch.empty(B, N, N, device=dev); mll = torch.empty(B, device=dev)
info = torch.empty(B, dtype=torch.int32, device=dev)
STRIDE = 32 + 16 * 8 * 8
st = torch.zeros(B, STRIDE, dtype=torch.int64, device=dev)
lib = _native.lib()
for it in range(5):
    rc = lib.gpk_debug_exact_stamps(X.data_ptr(), y.data_ptr(), hyp.data_ptr(), 1, B, N, D, 1e-6, 3,
                                    L.data_ptr(), None, mll.data_ptr(), info.data_ptr(), st.data_ptr(),
                                    torch.cuda.current_stream().cuda_stream)
    assert rc == 0
torch.cuda.synchronize()
assert int(info.abs().max()) == 0
s = st.cpu().numpy().astype(np.int64)
t0 = s[:, 0]
tl = s[:, 32:].reshape(B, 16, 8, 8)
rel = np.where(tl > 0, tl - t0[:, None, None, None], -1).astype(np.float64)
rel[tl <= 0] = np.nan
m = np.nanmean(rel, axis=0)
print(f"B={B}: prologue end {np.mean(s[:, 1] - t0):.0f} cycles after kernel start")
print(" S | diag: F32 start  F_a  W32  Hin  LAdone | workers (mean): start  Wwait  Await  trsm  Psync  hand  bulk+rhs  end | max end")
for S in range(8):
    d = m[S, 7]
    w = np.nanmean(m[S, :7], axis=0)
    we = np.nanmax(m[S, :7, 7]) if not np.all(np.isnan(m[S, :7, 7])) else float("nan")
    print(f"{S:2d} | " + " ".join(f"{v:7.0f}" for v in d[:5]) + " | " + " ".join(f"{v:7.0f}" for v in w[:8]) + f" | {we:7.0f}")
ends = rel[:, :, :7, 3]
tot = np.nanmax(rel.reshape(B, -1), axis=1)
print(f"last stamp: mean {np.mean(tot):.0f}")
