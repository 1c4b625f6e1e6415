"""cfg-3 GP shape variational legs only (b=256, N=192/96, M=256, D=32): kernel ms + rooflines."""
import json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import bench

dev = torch.device("cuda:0")
out = {}
for n in ((int(sys.argv[1]),) if len(sys.argv) > 1 else (192, 96)):
    r = bench.variational_leg(dev, 256, n, 256, 32, 10, 3, 1, seed=13 + n, label="cfg-3")
    out[f"N{n}"] = {"kernel_ms": r["kernel_ms"], "fwd_frac": r["roofline"]["frac"],
                    "bwd_frac": r["backward_roofline"]["frac"], "elbo_err": r["elbo_rel_err_vs_fp64_oracle"]}
print(json.dumps(out, indent=1))
