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
fixed across steps, and a learning rate that the graph can see: a float ``lr`` is baked
into the captured optimizer step, so a schedule that rewrites ``param_group['lr']`` on
the host (the reference's NoamOpt, train.py:147) must hold the lr in a device tensor
(``Adam(..., lr=torch.tensor(0.0, device=...), capturable=True)``) and update it in
place; changing a float lr after capture raises instead of silently training at the
capture-time rate.

Failure semantics match the eager step: eager ``psd_safe_cholesky`` raises
NotPSDError / NanError in the forward, before the backward and the optimizer step
touch anything. A replay has already run the optimizer step when its verdict is
read, so every replay that a check covers is bracketed: the parameters and the
optimizer state are snapshotted (device copies) when a check block starts, a sticky
device flag collects every hard failure (info > 0) of every replay in the block, and
on a failure the snapshot is restored before the error is raised -- the parameters
and Adam moments come back exactly as they were before the failing block. Every
replay condenses its verdicts into a device ring slot, so a block of ``check_every``
replays is checked with ONE host sync and still warns once per replay, in order
(``check_every`` > 1 keeps the replays back to back on the GPU).

Cost and granularity of the rollback: the snapshot is one ``_foreach_copy_`` of every
parameter and every optimizer-state tensor (≈ 3x the parameter bytes under Adam), issued
once per check block, outside the graph. With ``check_every = k`` a failure restores the
state from before the block's FIRST replay, so the successful replays that preceded the
failing one inside the block are undone too (the eager loop would have kept them); pick
``check_every = 1`` for eager-exact failure granularity, or a larger block for fewer host
syncs and snapshots (``scripts/gp_step.py`` times the graphed step with ``check_every = 10``:
its numbers include one snapshot per 10 replays). ``rollback=False`` skips the snapshot
entirely: a failing block still raises, but leaves the parameters as the replays left them.

The ``warmup`` eager steps that precede the capture are real
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
                 loss_index: int = 0, rollback: bool = True):
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
        self._lr_captured = [g.get("lr") for g in optimizer.param_groups]
        self.loss_fn = loss_fn
        self.optimizer = optimizer
        self.check_every = check_every
        self.loss_index = loss_index
        self.rollback_enabled = rollback
        self.static_inputs = [t.detach().clone() for t in sample_inputs]
        self._n = 0

        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(warmup):
                self._eager_step()
        torch.cuda.current_stream().wait_stream(side)

        self.graph = torch.cuda.CUDAGraph()
        self.checks = ops.DeferredChecks(device=self.static_inputs[0].device, slots=check_every)
        optimizer.zero_grad(set_to_none=True)
        ops._RECORDERS.append(self.checks)
        try:
            # captured on the warm-up stream: the parameters' gradient-accumulation
            # nodes keep the stream they were created on
            with torch.cuda.graph(self.graph, stream=side):
                self.static_outputs = self.loss_fn(*self.static_inputs)
                self._loss(self.static_outputs).backward()
                self.optimizer.step()
                self.checks.finalize()     # this replay's verdicts -> the device ring
        finally:
            ops._RECORDERS.remove(self.checks)
        invalidate_caches()
        # rollback state: every parameter of the optimizer and every tensor of its state
        self._state = [p for g in optimizer.param_groups for p in g["params"]]
        for p in list(self._state):
            for v in optimizer.state.get(p, {}).values():
                if isinstance(v, torch.Tensor) and v.is_cuda:
                    self._state.append(v)
        self._backup = [t.detach().clone() for t in self._state] if rollback else None
        self._block_open = False

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
        for g, lr0 in zip(self.optimizer.param_groups, self._lr_captured):
            lr = g.get("lr")
            if isinstance(lr0, torch.Tensor):
                if lr is not lr0:
                    raise ValueError("param_group['lr'] was replaced after capture; update the "
                                     "captured lr tensor in place (lr.fill_(...)) instead")
            elif lr != lr0:
                raise ValueError(f"param_group['lr'] changed from {lr0} to {lr} after capture, but a "
                                 "float lr is fixed inside the HIP graph; build the optimizer with a "
                                 "device-tensor lr and update it in place")
        if not self._block_open:
            # start of a check block: snapshot parameters + optimizer state (device copies,
            # stream-ordered before the replay) and clear the sticky failure flag
            if self._backup is not None:
                torch._foreach_copy_(self._backup, [t.detach() for t in self._state])
            self.checks.reset_sticky()
            self._block_open = True
        self.graph.replay()
        invalidate_caches()
        self._n += 1
        if self._n % self.check_every == 0:
            self._block_open = False
            try:
                self.checks.check(self.check_every)
            except Exception:
                self.rollback()
                raise
        return self.static_outputs

    def rollback(self) -> None:
        """Restore the parameters and optimizer state saved at the start of the current
        check block (called automatically when a replay's verdict raises)."""
        if self._backup is not None:
            with torch.no_grad():
                torch._foreach_copy_([t.detach() for t in self._state], self._backup)
        self._block_open = False
