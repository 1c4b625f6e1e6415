"""Generate the backbone-activation fixtures used by tests/test_e2e_gpu.py.

Runs in the build container ONLY (it imports the reference backbone read-only from
/root/reference; nothing from the reference is copied -- only the output tensors are
committed). The GP path's inputs in the reference training step are the backbone
outputs ``enc_outputs`` / ``dec_outputs`` that Forecast_denoising.forward hands to
denoise_model_2 (forecast_denoising.py:75-83); this script produces them with the
reference's own Transformer (modules/transformer.py:9-43) for

  cfg1  solar, Autoformer (attn_type='autoformer'), src/tgt input size 5, d_model 32,
        8 heads, stack 1, enc 192 / dec 96 steps   (BASELINE configs[0]; batch 32)
  cfg3  traffic, ATA (attn_type='ATA'), src/tgt input size 4, d_model 32, 8 heads,
        stack 1, enc 192 / dec 96 steps            (BASELINE configs[2]; batch 256)

from synthetic z-scored inputs ~N(0, 1) (the datasets need the network), the
enc/dec embeddings nn.Linear(input, d_model) as at forecast_denoising.py:65-66, seed
1234 (train.py:254). ``WINDOWS[cfg]`` distinct windows (cfg1: all 32 of its batch; cfg3:
128, half of its batch of 256) are stored as float16 (the values are inputs; both the HIP
path and the oracle read the same float32 up-cast) with targets y ~ N(0, 1) of shape
(windows, 96, 1). Tests tile them to the batch size.

    PYTHONDONTWRITEBYTECODE=1 python -B tests/golden/make_backbone_fixtures.py
"""
import os
import random
import sys

import numpy as np
import torch
import torch.nn as nn

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))
WINDOWS = {"cfg1_solar_autoformer": 32, "cfg3_traffic_ata": 128}
ENC, DEC, D, HEADS, SEED = 192, 96, 32, 8, 1234


def main():
    sys.dont_write_bytecode = True
    sys.path.insert(0, REF)
    from modules.transformer import Transformer  # reference backbone (read-only import)

    for name, attn, nin in [("cfg1_solar_autoformer", "autoformer", 5), ("cfg3_traffic_ata", "ATA", 4)]:
        np.random.seed(SEED)
        random.seed(SEED)
        torch.manual_seed(SEED)
        model = Transformer(src_input_size=nin, tgt_input_size=nin, pred_len=DEC, d_model=D,
                            d_ff=4 * D, d_k=D // HEADS, d_v=D // HEADS, n_heads=HEADS, n_layers=1,
                            src_pad_index=0, tgt_pad_index=0, device=torch.device("cpu"),
                            attn_type=attn, seed=SEED)
        enc_emb, dec_emb = nn.Linear(nin, D), nn.Linear(nin, D)
        g = torch.Generator().manual_seed(SEED + 1)
        nw = WINDOWS[name]
        enc_in = torch.randn(nw, ENC, nin, generator=g)
        dec_in = torch.randn(nw, DEC, nin, generator=g)
        y = torch.randn(nw, DEC, 1, generator=g)
        with torch.no_grad():
            enc_out, dec_out = model(enc_emb(enc_in), dec_emb(dec_in))
        path = os.path.join(OUT, f"backbone_{name}.npz")
        np.savez_compressed(path, enc=enc_out.numpy().astype(np.float16),
                            dec=dec_out.numpy().astype(np.float16),
                            y=y.numpy().astype(np.float16),
                            meta=np.array([f"attn={attn} input={nin} d_model={D} heads={HEADS} "
                                           f"stack=1 enc={ENC} dec={DEC} seed={SEED}"]))
        print(path, os.path.getsize(path), tuple(enc_out.shape), tuple(dec_out.shape),
              float(enc_out.std()), float(dec_out.std()))


if __name__ == "__main__":
    main()
