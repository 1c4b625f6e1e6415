"""Golden vectors for the GPU-resident window sampler.

Runs in the build container ONLY: imports the reference's own sampler
(Utils/base_train.py:100-153 batch_sampled_data -> :29-97 sample_train_val_test)
read-only from /root/reference and runs it on a small synthetic traffic-like dataframe
(columns of data/traffic.py:26-33: id, hours_from_start, values, time_on_day,
day_of_week, categorical_id). Only data is committed: the dataframe itself and every
batch the reference's train / valid / test DataLoaders yield (float32), so tests can
rebuild the table and check the HIP gather bit for bit without the reference.

Two cases: one where max_samples < the number of valid windows (np.random.choice
without replacement) and one where it exceeds them (the reference's "maximum samples
exceeds" branch: a permutation, with the trailing windows left as zeros).

    PYTHONDONTWRITEBYTECODE=1 python -B tests/golden/make_sampler_fixtures.py
"""
import os
import sys

import numpy as np
import pandas as pd

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))


def synthetic_frame(n_ids=5, seed=11):
    rng = np.random.default_rng(seed)
    rows = []
    for k in range(n_ids):
        n = int(rng.integers(70, 130))
        t = np.arange(n, dtype=np.float64)
        rows.append(pd.DataFrame({
            "id": np.full(n, float(k)),
            "hours_from_start": t + rng.integers(0, 5),
            "values": np.sin(t / 7.0 + k) + 0.1 * rng.standard_normal(n),
            "time_on_day": (t % 24) / 23.0,
            "day_of_week": ((t // 24) % 7) / 6.0,
            "categorical_id": np.full(n, float(k)),
        }))
    df = pd.concat(rows, ignore_index=True)
    return df.sample(frac=1.0, random_state=seed).reset_index(drop=True)   # unsorted on purpose


def main():
    sys.dont_write_bytecode = True
    sys.path.insert(0, REF)
    from Utils import base
    from Utils.base_train import batch_sampled_data
    DT, IT = base.DataTypes, base.InputTypes
    coldef = [("id", DT.REAL_VALUED, IT.ID), ("hours_from_start", DT.REAL_VALUED, IT.TIME),
              ("values", DT.REAL_VALUED, IT.TARGET), ("time_on_day", DT.REAL_VALUED, IT.KNOWN_INPUT),
              ("day_of_week", DT.REAL_VALUED, IT.KNOWN_INPUT),
              ("categorical_id", DT.CATEGORICAL, IT.STATIC_INPUT)]
    for name, max_samples in [("choice", (40, 12)), ("exceeds", (4000, 1000))]:
        df = synthetic_frame()
        frame = df.copy()
        n_enc, pred_len = 24, 12
        T = n_enc + 2 * pred_len
        train, valid, test = batch_sampled_data(frame, 0.6, max_samples, T, n_enc, pred_len, coldef, 8)
        out = {"frame": df[[c for c, _, _ in coldef]].to_numpy(np.float64),
               "columns": np.array([c for c, _, _ in coldef]),
               "params": np.array([0.6, max_samples[0], max_samples[1], T, n_enc, pred_len, 8])}
        for split, dl in [("train", train), ("valid", valid), ("test", test)]:
            enc, dec, y = zip(*[(e.numpy(), d.numpy(), t.numpy()) for e, d, t in dl])
            out[f"{split}_enc"] = np.stack(enc)
            out[f"{split}_dec"] = np.stack(dec)
            out[f"{split}_y"] = np.stack(y)
        path = os.path.join(OUT, f"sampler_{name}.npz")
        np.savez_compressed(path, **out)
        print(path, os.path.getsize(path), {k: v.shape for k, v in out.items()})


if __name__ == "__main__":
    main()
