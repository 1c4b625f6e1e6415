"""Time the variational (DeepGP) forward and backward at BASELINE cfg 5 (B=1024 N=256 M=64 D=32)."""
import math, os, sys, types
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from fine_grained_gaussian_process_forcasting_amd import ops_autograd

B, N, M, D = (int(a) for a in (sys.argv[1:5] if len(sys.argv) > 4 else (1024, 256, 64, 32)))
dev = torch.device("cuda:0")
g = torch.Generator().manual_seed(0)
P = lambda t: t.to(dev).requires_grad_(True)  # noqa: E731
X = P(torch.randn(B, N, D, generator=g) / math.sqrt(D))
Z = P(torch.randn(M, D, generator=g) / math.sqrt(D))
m, s = P(1e-3 * torch.randn(M, generator=g)), P(torch.ones(M))
w, b0 = P(torch.randn(D, generator=g)), P(torch.zeros(()))
ls, s2 = P(torch.full((D,), math.log(2))), P(torch.tensor(math.log(2)))
mm = types.SimpleNamespace(weights=w, bias=b0)
gm, gv = torch.randn(B, N, device=dev), torch.randn(B, N, device=dev)


def fwd():
    return ops_autograd.variational_predict(X, Z, m, s, s2, ls, mm, 1e-4)


for _ in range(3):
    mean, var = fwd()
    ((gm * mean).sum() + (gv * var).sum()).backward()
torch.cuda.synchronize()
e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
reps = 10
tf = tb = 0.0
for _ in range(reps):
    e[0].record()
    mean, var = fwd()
    e[1].record()
    ((gm * mean).sum() + (gv * var).sum()).backward()
    e[2].record()
    torch.cuda.synchronize()
    tf += e[0].elapsed_time(e[1])
    tb += e[1].elapsed_time(e[2])
tf, tb = tf / reps, tb / reps
print(f"variational B={B} N={N} M={M} D={D}: forward {tf*1e3:.1f} us, backward {tb*1e3:.1f} us "
      f"({B / ((tf + tb) * 1e-3):.3e} windows/s fwd+bwd)")
