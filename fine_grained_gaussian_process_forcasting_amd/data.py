"""GPU-resident training-window sampler.

Drop-in for the reference's ``batch_sampled_data`` (Utils/base_train.py:100-153) and
its per-window slicing ``sample_train_val_test`` (:29-97): the same splits, the same
window choice (the reference's ``np.random`` call sequence after
``np.random.seed(2436)``, reproduced exactly on the host: it is an index computation),
and the same (enc, dec, y) tensors, bit for bit -- but the feature table lives in HBM
as float32 and the windows are gathered there by the HIP kernel behind
include/gpk.h::gpk_window_gather_f32. The per-step host->device copy of train.py:160-161
disappears: batches are views of device tensors.

The returned loaders iterate like ``DataLoader(TensorDataset(enc, dec, y),
batch_size, drop_last=True)`` (sequential, no shuffle), as the reference builds them.
"""
from __future__ import annotations

import random
from dataclasses import dataclass
from typing import List, Sequence, Tuple

import numpy as np
import torch

from . import _native


def _col_by_type(input_type, column_definition):
    cols = [c for c, _, t in column_definition if t == input_type]
    if len(cols) != 1:
        raise ValueError(f"Invalid number of columns for {input_type}")
    return cols[0]


def _type_name(t):
    return getattr(t, "name", str(t))


def _input_cols(column_definition):
    """enc_input_cols of the reference: every column that is not the ID or TIME input."""
    return [c for c, _, t in column_definition if _type_name(t) not in ("ID", "TIME")]


def window_rows(ids: np.ndarray, lo: int, hi: int, max_samples: int, time_steps: int) -> np.ndarray:
    """First row (global index into the sorted table) of every window
    ``sample_train_val_test`` would slice from the split rows [lo, hi), in the
    reference's order, consuming the global numpy RNG exactly as it does
    (Utils/base_train.py:41-62); -1 for the zero windows it leaves when max_samples
    exceeds the valid sampling locations (:59-65)."""
    seg = ids[lo:hi]
    locs: List[Tuple[int, int]] = []           # (first row of the identifier's group, start_idx)
    if seg.size:
        uniq, first = np.unique(seg, return_index=True)     # groupby(id): sorted keys
        counts = np.diff(np.append(first, seg.size))
        for g0, n in zip(first, counts):
            if n >= time_steps:
                locs += [(lo + int(g0), time_steps + i) for i in range(n - time_steps + 1)]
    if 0 < max_samples < len(locs):
        pick = np.random.choice(len(locs), max_samples, replace=False)
    else:
        pick = np.random.choice(len(locs), len(locs), replace=False)
    out = np.full(max_samples, -1, dtype=np.int64)
    for i, k in enumerate(pick[:max_samples]):
        g0, start = locs[k]
        out[i] = g0 + start - time_steps
    return out


@dataclass
class WindowBatches:
    """Device-resident windows of one split; iterates like the reference's DataLoader."""
    enc: torch.Tensor      # (S, n_enc, F)
    dec: torch.Tensor      # (S, T - n_enc - pred_len, F)
    y: torch.Tensor        # (S, pred_len, 1)
    batch_size: int

    def __len__(self):
        return self.enc.shape[0] // self.batch_size

    def __iter__(self):
        bs = self.batch_size
        for k in range(len(self)):
            yield self.enc[k * bs:(k + 1) * bs], self.dec[k * bs:(k + 1) * bs], self.y[k * bs:(k + 1) * bs]


class GPUWindowTable:
    """The (id, time)-sorted feature table in HBM plus the per-row identifiers."""

    def __init__(self, data, column_definition: Sequence, device):
        id_col = _col_by_type(_enum_of(column_definition, "ID"), column_definition)
        time_col = _col_by_type(_enum_of(column_definition, "TIME"), column_definition)
        target_col = _col_by_type(_enum_of(column_definition, "TARGET"), column_definition)
        cols = _input_cols(column_definition)
        # the reference sorts in place with DataFrame.sort_values(by=[id, time])
        data = data.sort_values(by=[id_col, time_col])
        self.ids = data[id_col].to_numpy()
        self.n_rows = len(data)
        self.F = len(cols)
        self.target_index = cols.index(target_col)
        # float64 frame -> float32, the rounding torch.FloatTensor applies to the numpy windows
        host = np.ascontiguousarray(data[cols].to_numpy(np.float64).astype(np.float32))
        self.table = torch.from_numpy(host).to(device)
        self.device = self.table.device

    def gather(self, rows: np.ndarray, time_steps: int, n_enc: int, pred_len: int):
        rows = np.asarray(rows, dtype=np.int64)
        ok = (rows == -1) | ((rows >= 0) & (rows + time_steps <= self.n_rows))
        if not ok.all():
            raise ValueError("window rows out of range of the table")
        B = rows.size
        n_dec = time_steps - n_enc - pred_len
        dev = self.device
        enc = torch.empty(B, n_enc, self.F, device=dev, dtype=torch.float32)
        dec = torch.empty(B, n_dec, self.F, device=dev, dtype=torch.float32)
        y = torch.empty(B, pred_len, 1, device=dev, dtype=torch.float32)
        r = torch.from_numpy(rows).to(dev)
        rc = _native.lib().gpk_window_gather_f32(
            self.table.data_ptr(), self.n_rows, self.F, r.data_ptr(), B, time_steps, n_enc, pred_len,
            self.target_index, enc.data_ptr(), dec.data_ptr(), y.data_ptr(),
            torch.cuda.current_stream(dev).cuda_stream)
        _native.check(rc, "gpk_window_gather_f32")
        return enc, dec, y


def _enum_of(column_definition, name):
    for _, _, t in column_definition:
        if _type_name(t) == name:
            return t
    raise ValueError(f"no {name} column in the column definition")


def batch_sampled_data(data, train_percent, max_samples, time_steps, num_encoder_steps, pred_len,
                       column_definition, batch_size, device="cuda", tgt_all=False):
    """Utils/base_train.py:100-153 on the GPU: (train, valid, test) loaders of device
    windows. Same splits (train = first train_percent of the sorted rows, valid = the
    next half of the rest -- empty when that half rounds to 0, as ``data[a:-0]`` --,
    test = all rows), same seeds (2436), same window choice and order."""
    np.random.seed(2436)
    random.seed(2436)
    table = GPUWindowTable(data, column_definition, device)
    n = table.n_rows
    train_len = int(n * train_percent)
    valid_len = int((n - train_len) / 2)
    valid_hi = n - valid_len if valid_len > 0 else train_len      # data[train_len:-0] is empty
    train_max, valid_max = max_samples
    out = []
    for lo, hi, ms in [(0, train_len, train_max), (train_len, valid_hi, valid_max), (0, n, valid_max)]:
        rows = window_rows(table.ids, lo, hi, ms, time_steps)
        enc, dec, y = table.gather(rows, time_steps, num_encoder_steps, pred_len)
        out.append(WindowBatches(enc, dec, y, batch_size))
    return tuple(out)
