"""Per-step timeline of the exact kernel's column-ownership plan (STAMPS build, N=256 D=32).

Worker events per (step k, wave w): 0 start, 2 row k + RHS k, 4 R_kk^-T arrived,
5 TRSM + the next step's hand-over (HO_{k+1}) done, 1 trailing update done, 6 RHS rows + bulk
count, 3 RBF + zero-L (step end),
7 cumulative cycles spent in flag waits (panel / z / counters; not the R_kk^-T wait).
Diagonal wave (w = 7): 0 factor start, 1 factor done (R_kk^-T published), 2 look-ahead
tiles arrived, 3 look-ahead done.

    python scripts/r05/stamps_col.py [B]
"""
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from fine_grained_gaussian_process_forcasting_amd import _native, ops  # noqa: E402

B, N, D = int(sys.argv[1]) if len(sys.argv) > 1 else 512, 256, 32
dev = torch.device("cuda:0")
X = (torch.randn(B, N, D) / math.sqrt(D)).to(dev)
y = torch.randn(B, N).to(dev)
LN2 = math.log(2)
hyp = ops.pack_exact_hyper(LN2, LN2 + 1e-4, 0.0, LN2, dev)
L = torch.empty(B, N, N, device=dev)
mll = torch.empty(B, device=dev)
info = torch.empty(B, dtype=torch.int32, device=dev)
STRIDE = 32 + 16 * 8 * 8
st = torch.zeros(B, STRIDE, dtype=torch.int64, device=dev)
lib = _native.lib()
for it in range(5):
    st.zero_()
    rc = lib.gpk_debug_exact_stamps(X.data_ptr(), y.data_ptr(), hyp.data_ptr(), 1, B, N, D, 1e-6, 3,
                                    L.data_ptr(), None, mll.data_ptr(), info.data_ptr(), st.data_ptr(),
                                    torch.cuda.current_stream().cuda_stream)
    assert rc == 0
torch.cuda.synchronize()
assert bool((info == 0).all()), info
s_all = st.cpu().numpy()
tot = s_all[:, 8].astype(np.float64)
print(f"B={B} window cycles: mean {tot.mean():.0f} min {tot.min():.0f} max {tot.max():.0f}")
tl = s_all[:, 32:].reshape(B, 16, 8, 8).astype(np.int64)
ev = tl.copy()
ev[:, :, :7, 7] = 0
valid = ev > 0
base = np.where(valid, ev, np.iinfo(np.int64).max).reshape(B, -1).min(1)
rel = np.where(valid, ev - base[:, None, None, None], 0).astype(np.float64)
rel[~valid] = np.nan
m = np.nanmean(rel, axis=0)                      # (16, 8, 8)
wcum = tl[:, :, :7, 7].astype(np.float64)        # cumulative waits (B, 16, 7)
wstep = np.diff(np.concatenate([np.zeros((B, 1, 7)), wcum], axis=1), axis=1)
wstep[:, 15] = np.nan
ws = np.nanmean(wstep, axis=0)                   # (16, 7)
print(" k | diag fac0   fac1   LAin LAdone (LA wait) | wrk start  end  (dur) | mean per wave:  rowK  "
      "Wwait TRSM+HO trail  rhs+cnt  rbf+zl | flag-wait | slowest wave end")
for k in range(16):
    d = m[k, 7]
    w = m[k, :7]                                   # (7, 8)
    st0 = np.nanmean(w[:, 0])
    en = np.nanmean(w[:, 3])
    ph = [np.nanmean(w[:, 2] - w[:, 0]), np.nanmean(w[:, 4] - w[:, 2]), np.nanmean(w[:, 5] - w[:, 4]),
          np.nanmean(w[:, 1] - w[:, 5]), np.nanmean(w[:, 6] - w[:, 1]), np.nanmean(w[:, 3] - w[:, 6])]
    law = d[2] - d[1] if k < 15 else float("nan")
    print(f"{k:2d} | {d[0]:7.0f} {d[1]:6.0f} {d[2]:6.0f} {d[3]:6.0f} ({law:5.0f}) | {st0:7.0f} {en:6.0f} "
          f"({en - st0:5.0f}) | " + " ".join(f"{v:6.0f}" for v in ph) +
          f" | {np.nanmean(ws[k]):6.0f} | {np.nanmax(w[:, 3]):6.0f}")
print("per-wave flag-wait cycles per step (rows k, columns wave 0..6):")
for k in range(15):
    print(f"{k:2d} " + " ".join(f"{v:6.0f}" for v in ws[k]))
print("per-wave step duration (start k+1 - start k):")
for k in range(15):
    print(f"{k:2d} " + " ".join(f"{v:6.0f}" for v in (m[k + 1, :7, 0] - m[k, :7, 0])))
