"""Time the exact-GP forward (L + z kept) and the analytic backward at B=512 N=256 D=32."""
import math, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from fine_grained_gaussian_process_forcasting_amd import ops

B, N, D = (int(a) for a in (sys.argv[1:4] if len(sys.argv) > 3 else (512, 256, 32)))
dev = torch.device("cuda:0")
g = torch.Generator().manual_seed(0)
X = (torch.randn(B, N, D, generator=g) / math.sqrt(D)).to(dev)
y = torch.randn(B, N, generator=g).to(dev)
LN2 = math.log(2)
hyp = ops.pack_exact_hyper(LN2, LN2 + 1e-4, 0.0, LN2, dev)
gout = torch.ones(B, device=dev)
fw = ops.exact_mll(X, y, None, None, None, None, hyper=hyp, want_L=True, want_z=True)
for _ in range(3):
    ops.exact_mll_grad(X, fw.L, fw.z, hyp, gout)
torch.cuda.synchronize()
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
reps = 10
s.record()
for _ in range(reps):
    fw = ops.exact_mll(X, y, None, None, None, None, hyper=hyp, want_L=True, want_z=True)
e.record(); torch.cuda.synchronize()
tf = s.elapsed_time(e) / reps
s.record()
for _ in range(reps):
    ops.exact_mll_grad(X, fw.L, fw.z, hyp, gout)
e.record(); torch.cuda.synchronize()
tb = s.elapsed_time(e) / reps
print(f"B={B} N={N} D={D}: forward(L,z) {tf*1e3:.1f} us, backward {tb*1e3:.1f} us "
      f"({B / ((tf + tb) * 1e-3):.3e} windows/s fwd+bwd)")
