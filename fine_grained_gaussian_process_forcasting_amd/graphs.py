"""HIP-graph capture of a whole training step (forward + backward + optimizer step).

The reference trains eagerly (train.py:152-167): every step re-issues a few hundred
small kernels from Python, so at the BASELINE shapes the step is bound by host launch
overhead, not by the GP kernels. ``GraphedStep`` captures ONE step of
the caller's own loss function once and replays it: one graph launch per step. The
GP ops are capture-safe by construction -- they launch on the current stream, allocate
through PyTorch's caching allocator, never copy host data to the device, and their
host-side numerical verdicts (psd_safe_cholesky info codes, the variance-clamp flag)
are recorded during capture (ops.DeferredChecks) and evaluated after each replay, so a
replay warns / raises exactly as the eager step would for the same data.

    step = GraphedStep(model, optimizer, (enc0, dec0, y0), loss_index=1)
    for enc, dec, y in batches:
        out, loss, mse = step(enc, dec, y)   # copies into the static inputs, replays

``loss_fn`` returns the loss tensor, or a tuple whose ``loss_index``-th entry is the loss
(``Forecast_denoising.forward`` returns ``(final_outputs, loss, mse_loss)``,
forecast_denoising.py:105); the call returns the same structure, as graph-owned tensors
rewritten by every replay.

Requirements (checked): CUDA/ROCm tensors, an optimizer built with
``capturable=True`` (Adam/AdamW keep their step counters on the device), input shapes
fixed across steps. The ``warmup`` eager steps that precede the capture are real
training steps on the sample inputs (PyTorch's documented whole-network capture
recipe). The package's factor caches are keyed on tensor version counters, which a
replay does not bump, so they are invalidated after every replay.
"""
from __future__ import annotations

from typing import Callable, Sequence

import torch

from . import ops
from .ops_autograd import invalidate_caches


class GraphedStep:
    def __init__(self, loss_fn: Callable[..., object], optimizer: torch.optim.Optimizer,
                 sample_inputs: Sequence[torch.Tensor], warmup: int = 3, check_every: int = 1,
                 loss_index: int = 0):
        if not torch.cuda.is_available():
            raise RuntimeError("GraphedStep needs a ROCm device (HIP graphs); there is no CPU path")
        for t in sample_inputs:
            if not (isinstance(t, torch.Tensor) and t.is_cuda):
                raise ValueError("GraphedStep inputs must be device tensors")
        for gdict in optimizer.param_groups:
            if "capturable" in gdict and not gdict["capturable"]:
                raise ValueError(f"{type(optimizer).__name__} must be built with capturable=True "
                                 "to be captured in a HIP graph")
        if check_every < 1:
            raise ValueError("check_every must be >= 1")
        self.loss_fn = loss_fn
        self.optimizer = optimizer
        self.check_every = check_every
        self.loss_index = loss_index
        self.static_inputs = [t.detach().clone() for t in sample_inputs]
        self._n = 0

        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(warmup):
                self._eager_step()
        torch.cuda.current_stream().wait_stream(side)

        self.graph = torch.cuda.CUDAGraph()
        self.checks = ops.DeferredChecks()
        optimizer.zero_grad(set_to_none=True)
        ops._RECORDERS.append(self.checks)
        try:
            # captured on the warm-up stream: the parameters' gradient-accumulation
            # nodes keep the stream they were created on
            with torch.cuda.graph(self.graph, stream=side):
                self.static_outputs = self.loss_fn(*self.static_inputs)
                self._loss(self.static_outputs).backward()
                self.optimizer.step()
        finally:
            ops._RECORDERS.remove(self.checks)
        invalidate_caches()

    def _loss(self, outputs) -> torch.Tensor:
        return outputs[self.loss_index] if isinstance(outputs, (tuple, list)) else outputs

    def _eager_step(self) -> None:
        self.optimizer.zero_grad(set_to_none=True)
        self._loss(self.loss_fn(*self.static_inputs)).backward()
        self.optimizer.step()

    def __call__(self, *inputs: torch.Tensor):
        if len(inputs) != len(self.static_inputs):
            raise ValueError(f"expected {len(self.static_inputs)} inputs, got {len(inputs)}")
        for dst, src in zip(self.static_inputs, inputs):
            if src.shape != dst.shape:
                raise ValueError(f"input shape {tuple(src.shape)} != captured {tuple(dst.shape)}")
            if src.data_ptr() != dst.data_ptr():
                dst.copy_(src, non_blocking=True)
        self.graph.replay()
        invalidate_caches()
        self._n += 1
        if self._n % self.check_every == 0:
            self.checks.check()
        return self.static_outputs
