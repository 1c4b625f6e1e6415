"""Time the forecast -> GP blur -> denoise training step at the BASELINE end-to-end shapes
and the GP share of it (reference forecast_denoising.py:69-105,
denoise_model_2.py:42-59, train.py:152-167).

The step mirrors Forecast_denoising.forward + loss.backward() + an Adam step:
  enc/dec nn.Linear embeddings -> backbone -> denoise_model_2 (GP blur of enc AND dec with
  the package's DeepGPp: M = 256 inducing points, d = 32) -> backbone again -> final
  projection; loss = MSE + clip(lam, 0, 0.005) * (-ELBO) with the ELBO of
  forecast_denoising.py:86-89 (num_data = d).
Backbone: the reference's ATA / Autoformer Transformer cannot travel to the GPU box (no
reference source ships), so a torch.nn.Transformer encoder/decoder of the same width
(d_model 32, 8 heads, d_ff 128, 1 layer) stands in -- the GP part is the package's real
path. Batches come from the GPU-resident window sampler (data.batch_sampled_data on a
synthetic traffic-like frame): no per-step host->device copy.

GP share = t(step with gp=True) - t(step with the GP blur off, same backbone work).
Both eager (the reference's loop) and HIP-graph-captured (graphs.GraphedStep: one graph
launch per step, the numerical verdicts of 10 replays read with one host sync) timings
are reported.

    python scripts/gp_step.py [cfg3|cfg1] [steps] [graph-gp]
"""
import json
import math
import os
import sys
import time

import numpy as np
import pandas as pd
import torch
import torch.nn as nn

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from fine_grained_gaussian_process_forcasting_amd import settings  # noqa: E402
from fine_grained_gaussian_process_forcasting_amd.data import batch_sampled_data  # noqa: E402
from fine_grained_gaussian_process_forcasting_amd.denoising_model.denoise_model_2 import denoise_model_2  # noqa: E402
from fine_grained_gaussian_process_forcasting_amd.mlls import DeepApproximateMLL, VariationalELBO  # noqa: E402
from fine_grained_gaussian_process_forcasting_amd.graphs import GraphedStep  # noqa: E402


class Backbone(nn.Module):
    def __init__(self, d, heads=8):
        super().__init__()
        self.enc = nn.TransformerEncoder(nn.TransformerEncoderLayer(d, heads, 4 * d, 0.0, batch_first=True), 1)
        self.dec = nn.TransformerDecoder(nn.TransformerDecoderLayer(d, heads, 4 * d, 0.0, batch_first=True), 1)

    def forward(self, enc, dec):
        e = self.enc(enc)
        return e, self.dec(dec, e)


class Model(nn.Module):
    """Forecast_denoising (forecast_denoising.py:14-105) with a stand-in backbone."""

    def __init__(self, nin, d, pred_len, gp, seed=1234):
        super().__init__()
        torch.manual_seed(seed)
        self.lam = nn.Parameter(torch.randn(1))
        self.backbone = Backbone(d)
        self.de_model = denoise_model_2(self.backbone, "stand-in", gp, d, None, seed, n_noise=not gp)
        self.final_projection = nn.Linear(d, 1)
        self.enc_embedding = nn.Linear(nin, d)
        self.dec_embedding = nn.Linear(nin, d)
        self.d, self.pred_len, self.gp = d, pred_len, gp

    def forward(self, enc, dec, y):
        enc = self.enc_embedding(enc)
        dec = self.dec_embedding(dec)
        eo, do = self.backbone(enc, dec)
        out, dist = self.de_model(eo.clone(), do.clone())
        final = self.final_projection(out[:, -self.pred_len:, :])
        mll_error = 0.0
        if self.gp:
            mll = DeepApproximateMLL(VariationalELBO(self.de_model.deep_gp.likelihood, self.de_model.deep_gp, self.d))
            mll_error = -mll(dist, y.permute(2, 0, 1)).mean()
        return nn.MSELoss()(y, final) + torch.clip(self.lam, min=0, max=0.005) * mll_error


def traffic_like_frame(n_ids, n_per, nin, seed=0):
    rng = np.random.default_rng(seed)
    cols = {"id": np.repeat(np.arange(n_ids, dtype=np.float64), n_per),
            "t": np.tile(np.arange(n_per, dtype=np.float64), n_ids)}
    cols["values"] = rng.standard_normal(n_ids * n_per)
    for k in range(nin - 1):
        cols[f"x{k}"] = rng.standard_normal(n_ids * n_per)
    return pd.DataFrame(cols)


class _Null:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


class _T:
    def __init__(self, name):
        self.name = name


def run(cfg, steps, modes=("eager", "graph", "eager_anomaly"), gps=(True, False)):
    dev = torch.device("cuda:0")
    b, nin = (256, 4) if cfg == "cfg3" else (32, 5)
    n_enc, pred_len, d = 192, 96, 32
    T = n_enc + 2 * pred_len
    frame = traffic_like_frame(8, 2000, nin)
    coldef = [("id", None, _T("ID")), ("t", None, _T("TIME")), ("values", None, _T("TARGET"))] + \
             [(f"x{k}", None, _T("KNOWN_INPUT")) for k in range(nin - 1)]
    train, _, _ = batch_sampled_data(frame, 0.8, (b * (steps + 4), b), T, n_enc, pred_len, coldef, b, device=dev)
    batches = list(train)
    res = {}
    for mode in modes:
        r = {}
        for gp in gps:
            model = Model(nin, d, pred_len, gp).to(dev)
            # capturable=True in both modes, so the two time the same Adam arithmetic
            opt = torch.optim.Adam(model.parameters(), lr=1e-4, betas=(0.9, 0.98), eps=1e-9,
                                   capturable=True)
            # eager_anomaly: the reference's global torch.autograd.set_detect_anomaly(True)
            # (train.py:18, forecast_denoising.py:11; SURVEY B7 / §8d cfg 3 "off and on")
            anomaly = torch.autograd.detect_anomaly() if mode == "eager_anomaly" else _Null()
            with settings.num_likelihood_samples(1), anomaly:
                if mode in ("eager", "eager_anomaly"):
                    def step(k):
                        enc, dec, y = batches[k % len(batches)]
                        loss = model(enc, dec, y)
                        opt.zero_grad()
                        loss.backward()
                        opt.step()
                        return loss
                    for k in range(3):
                        step(k)
                else:
                    # the verdicts of 10 replays are read with one host sync (per-replay
                    # warnings preserved, graphs.GraphedStep): replays stay back to back
                    gstep = GraphedStep(lambda enc, dec, y: model(enc, dec, y), opt, batches[0],
                                        check_every=10)

                    def step(k):
                        return gstep(*batches[k % len(batches)])
                    for k in range(10):       # untimed replays: the first launches of a fresh
                        step(k)               # graph exec carry one-time upload costs
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for k in range(steps):
                    loss = step(k + 3)
                torch.cuda.synchronize()
                dt = (time.perf_counter() - t0) / steps
            r["gp" if gp else "no_gp"] = {"ms_per_step": dt * 1e3, "windows_per_s": b / dt,
                                          "loss": float(loss)}
        if len(r) == 2:
            r["gp_share_ms"] = r["gp"]["ms_per_step"] - r["no_gp"]["ms_per_step"]
            r["gp_share_frac"] = r["gp_share_ms"] / r["gp"]["ms_per_step"]
        res[mode] = r
    res["config"] = {"cfg": cfg, "b": b, "enc": n_enc, "dec": pred_len, "d_model": d, "M": 256,
                     "backbone": "torch.nn.Transformer stand-in (d 32, 8 heads, d_ff 128, 1 layer)",
                     "anomaly_mode": {m: m == "eager_anomaly" for m in modes},
                     "input": "GPU-resident window sampler"}
    return res


if __name__ == "__main__":
    cfg = sys.argv[1] if len(sys.argv) > 1 else "cfg3"
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    if len(sys.argv) > 3 and sys.argv[3] in ("graph-gp", "graph-nogp", "eager-gp", "eager-nogp"):
        mode, gp = sys.argv[3].split("-")                 # profiling / A/B: one step kind
        print(json.dumps(run(cfg, steps, modes=(mode,), gps=(gp == "gp",))), flush=True)
    else:
        print(json.dumps(run(cfg, steps)), flush=True)
