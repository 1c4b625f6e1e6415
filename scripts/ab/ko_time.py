"""Time the exact kernel of ONE libgpk.so build (GPK_LIB) on the bench shapes.
Prints one JSON line: B=512 N=256 (L written / not), B=64 and B=128 N=256 (small-batch
layout), B=128 N=128 (cfg 2). Development A/B tool (knockout builds give wrong results)."""
import json, math, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
from fine_grained_gaussian_process_forcasting_amd import ops

dev = torch.device("cuda:0")
LN2 = math.log(2.0)
hyp = ops.pack_exact_hyper(LN2, LN2 + 1e-4, 0.0, LN2, dev)


def t(B, N, D=32, want_L=True, n=40):
    g = torch.Generator().manual_seed(0)
    X = (torch.randn(B, N, D, generator=g) / math.sqrt(D)).to(dev)
    y = torch.randn(B, N, generator=g).to(dev)
    L = torch.empty(B, N, N, device=dev) if want_L else None
    f = lambda: ops.exact_mll(X, y, None, None, None, None, hyper=hyp, want_L=want_L, L_out=L)  # noqa
    for _ in range(5):
        o = f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        o = f()
    e1.record()
    torch.cuda.synchronize()
    return round(e0.elapsed_time(e1) / n * 1e3, 2), float(o.mll.float().mean())


res = {"lib": os.environ.get("GPK_LIB", "default").split("/")[-2]}
for key, args in [("b512", (512, 256)), ("b512_noL", (512, 256, 32, False)), ("b64", (64, 256)),
                  ("b128", (128, 256)), ("cfg2", (128, 128))]:
    res[key] = t(*args)
print(json.dumps(res), flush=True)
