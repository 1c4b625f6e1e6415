"""Diagnostic: per-phase clocks of the exact kernel (STAMPS build), N=256 D=32."""
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
s_all = st.cpu().numpy()
s = s_all[:, :32].astype(np.float64)
names = ["prologue", "RBF rows 0-1"]
tot = s[:, 8]
print(f"B={B} total cycles: mean {tot.mean():.0f} min {tot.min():.0f} max {tot.max():.0f}")
print(f"clock GHz (memtime/realtime): {np.mean(s[:, 8] / (s[:, 9] / 100e6)) / 1e9:.3f}")
for i, n in enumerate(names):
    print(f"  {n:22s} {s[:, i].mean():10.0f}  ({100 * s[:, i].mean() / tot.mean():5.1f}%)")
for i, n in [(24, "pro: X loads+staging+max"), (25, "pro: column partials"), (26, "pro: mean"),
             (27, "pro: centre+split"), (18, "w0: trailing upd"), (19, "w0: RHS+zeroL+RBF"), (20, "w0: TRSM"), (21, "w0: step counter"),
             (22, "w0: hand-over"), (23, "w0: wait R_kk^-T"), (2, "diag: tile load"), (3, "diag: sweep"), (4, "diag: publish"), (13, "diag: factor"), (14, "diag: wait look-ahead tiles"), (15, "diag: look-ahead compute")]:
    print(f"  {n:28s} {s[:, i].mean():10.0f}  ({100 * s[:, i].mean() / tot.mean():5.1f}%)")

hw = s[:, 10].astype(np.int64)
hw0 = s[:, 11].astype(np.int64)
simd = (hw >> 4) & 3
cu = (hw >> 8) & 15
sh = (hw >> 12) & 1
se = (hw >> 13) & 7
xcc = s[:, 12].astype(np.int64) & 15
key = ((xcc * 8 + se) * 2 + sh) * 16 + cu
from collections import defaultdict
groups = defaultdict(list)
for bb in range(B):
    groups[int(key[bb])].append(int(simd[bb]))
same = sum(1 for v in groups.values() if len(v) == 2 and v[0] == v[1])
print(f"CUs hosting 2 WGs: {sum(1 for v in groups.values() if len(v) == 2)}; diag waves on the same SIMD: {same}; groups={len(groups)}")
print("sample hw_id:", [hex(int(x)) for x in hw[:8]])

# per-step timeline (absolute s_memtime, made relative to each window's earliest event)
tl = s_all[:, 32:].reshape(B, 16, 8, 8).astype(np.int64)
valid = tl > 0
base = np.where(valid, tl, np.iinfo(np.int64).max).reshape(B, -1).min(1)
rel = np.where(valid, tl - base[:, None, None, None], -1).astype(np.float64)
rel[~valid] = np.nan
m = np.nanmean(rel, axis=0)  # (16 steps, 8 waves, 8 events)
print("per-step timeline (cycles from the window's first timeline event, mean over windows)")
print(" k | diag: fac0  fac1  LAin  LAdone | workers (mean over waves): start  waitW  trsm  count  hand  trail  rest | max-wave rest")
for k in range(16):
    d = m[k, 7]
    w = np.nanmean(m[k, :7], axis=0)
    wb = np.nanmax(m[k, :7, 6])
    print(f"{k:2d} | {d[0]:6.0f} {d[1]:6.0f} {d[2]:6.0f} {d[3]:6.0f} | " + " ".join(f"{v:6.0f}" for v in w[:7]) + f" | {wb:6.0f}")
print("per-wave busy cycles (trsm + hand + trail + rest) and waits (W + counter) at k=1,2,3,8:")
for k in (1, 2, 3, 8):
    busy = (m[k, :7, 2] - m[k, :7, 1]) + (m[k, :7, 6] - m[k, :7, 3])
    wait = (m[k, :7, 1] - m[k, :7, 0]) + (m[k, :7, 3] - m[k, :7, 2])
    print(k, " ".join(f"{v:5.0f}" for v in busy), " wait:", " ".join(f"{v:5.0f}" for v in wait))
