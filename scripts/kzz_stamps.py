"""Per-step phase clocks of a GPK_KZZ_STAMPS=1 build of gpk_kzz16_kernel (load it with
GPK_LIB=<path>): info[1 + 3k .. 3 + 3k] = s_memtime at step k's start, after its diagonal
barrier and after its TRSM barrier (workgroup thread 0, first attempt); info[1 + 3T + 3k ..]
= the diagonal wave's factor of tile (k, k): hand-over seen, tile in registers, factor done.
   GPK_LIB=... python scripts/kzz_stamps.py [M] [D]"""
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fine_grained_gaussian_process_forcasting_amd import _native  # noqa: E402

M, D = (int(v) for v in (sys.argv[1:] + ["256", "32"])[:2])
LN2 = math.log(2.0)
dev = torch.device("cuda", 0)
g = torch.Generator().manual_seed(0)
Z = (torch.randn(M, D, generator=g) / math.sqrt(D)).to(dev)
h = torch.cat([torch.tensor([LN2]), torch.full((D,), LN2)]).to(dev)
T = (M + 15) // 16
L = torch.empty(M, M, dtype=torch.float64, device=dev)
Li = torch.empty(M, M, dtype=torch.float64, device=dev)
info = torch.zeros(8 + 16 * T, dtype=torch.int32, device=dev)
lib = _native.lib()
for _ in range(3):
    rc = lib.gpk_kzz_chol_f64(Z.data_ptr(), h.data_ptr(), M, D, 1e-4, 1e-8, 3, L.data_ptr(), Li.data_ptr(),
                              info.data_ptr(), torch.cuda.current_stream().cuda_stream)
    assert rc == 0, f"rc={rc}"
torch.cuda.synchronize()
v = info.cpu().tolist()
st = [v[1 + 3 * k: 4 + 3 * k] for k in range(T)]
rows = []
for k in range(T):
    nxt = st[k + 1][0] if k + 1 < T else None
    diag = (st[k][1] - st[k][0]) & 0xffffffff
    trsm = (st[k][2] - st[k][1]) & 0xffffffff
    upd = ((nxt - st[k][2]) & 0xffffffff) if nxt is not None else 0
    rows.append((diag, trsm, upd))
print(f"M={M} D={D} info={v[0]}  per step (s_memtime ticks): diag+barrier / trsm+barrier / update")
for k, (a, b, c) in enumerate(rows):
    print(f"k={k:2d} {a:7d} {b:7d} {c:7d}")
tot = [sum(r[i] for r in rows) for i in range(3)]
print("sum", tot, "total", sum(tot))
ds = [v[1 + 3 * T + 3 * k: 4 + 3 * T + 3 * k] for k in range(T)]
print("diagonal wave, factor of (k,k) (ticks): look-ahead start -> sweep start / sweep + LDS writes; "
      "look-ahead start relative to the previous step's TRSM barrier")
for k in range(1, T):
    ld = (ds[k][1] - ds[k][0]) & 0xffffffff
    sw = (ds[k][2] - ds[k][1]) & 0xffffffff
    ho = (ds[k][0] - st[k - 1][2]) & 0xffffffff
    print(f"k={k:2d} look-ahead {ld:6d} sweep {sw:6d}  start-after-trsm {ho:6d}")
iv = v[1 + 6 * T: 1 + 6 * T + T + 1]
print("inverse kernel, block column 0 (ticks): prologue", (iv[1] - iv[0]) & 0xffffffff, " steps",
      [(iv[2 + k] - iv[1 + k]) & 0xffffffff for k in range(T - 1)], " total", (iv[T] - iv[0]) & 0xffffffff)
print("look-ahead detail (ticks): operands in -> R done / -> T'' + row-major write done / -> diag blocks stored / -> sweep start")
for k in range(1, T):
    a = v[1 + 8 * T + 4 * k: 5 + 8 * T + 4 * k]
    sw = ds[k][1]
    print(f"k={k:2d} load {(a[0] - ds[k][0]) & 0xffffffff:6d} R {(a[1] - a[0]) & 0xffffffff:6d} T'' {(a[2] - a[1]) & 0xffffffff:6d} "
          f"stores {(a[3] - a[2]) & 0xffffffff:6d} to-sweep {(sw - a[3]) & 0xffffffff:6d}")
print("inverse, owner wave of each step (block column 0; ticks from the previous barrier): S done / X done / staging stored / barrier")
for k in range(1, T - 1):
    o = v[1 + 12 * T + 4 * k: 5 + 12 * T + 4 * k]
    prev = iv[1 + k]
    print(f"k={k:2d} S {(o[0] - prev) & 0xffffffff:6d} X {(o[1] - o[0]) & 0xffffffff:6d} store {(o[2] - o[1]) & 0xffffffff:6d} "
          f"barrier {(o[3] - o[2]) & 0xffffffff:6d}")
