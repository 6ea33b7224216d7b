"""One data-parallel training step on MI355X: the hot path of BaseTrainer._train_step
(spine_vision/training/trainers/base.py:571-599, localization.py:186-209,
classification.py:269-290), re-designed around flat buffers:

    zero grads (one memset) -> forward (HIP backbone + torch head) -> loss -> backward
    (HIP backbone backward; per-block bucket all-reduce over RCCL on a side stream) ->
    global-norm clip coefficient (device scalar) -> fused AdamW (+bf16 shadow refresh)

The loss stays on the device (the reference's per-step ``loss.item()`` host sync is deferred to the
caller), so the host can run ahead and enqueue the next step while the GPU works.
"""

from __future__ import annotations

import os
from collections import deque
from typing import Any, Callable

import torch
import torch.distributed as dist

from .. import kernels as K
from .comm import BufferSync, GradBucketer, broadcast_parameters
from .flat import FlatArena
from .optim import FlatAdamW


class InflightLimiter:
    """Bounds how many enqueued training steps the host may run ahead of the GPU.

    Tensors handed to the weight-gradient side stream (``record_stream``) and the all-reduce stream
    can only be reused by the caching allocator once the GPU has passed them.  A host that runs
    unboundedly ahead therefore keeps every in-flight step's activations allocated.  Measured on
    ConvNeXt-base bs32: 124 GB reserved; ConvNeXt-large bs64 filled the 288 GB and fell into
    allocator free-and-retry at 165 img/s.  After each step an event is recorded, and the host waits
    for the step ``max_inflight`` steps back.  The GPU still always has a full step queued.
    """

    def __init__(self, max_inflight: int | None = None) -> None:
        if max_inflight is None:  # SV_MAX_INFLIGHT: 0 = unbounded
            max_inflight = int(os.environ.get("SV_MAX_INFLIGHT", "2"))
        self.max_inflight = int(max_inflight)
        self._events: deque = deque()

    def step_done(self) -> None:
        if self.max_inflight <= 0 or not torch.cuda.is_initialized():
            return
        ev = torch.cuda.Event()
        ev.record()
        self._events.append(ev)
        while len(self._events) > self.max_inflight:
            self._events.popleft().synchronize()


class StepEngine:
    def __init__(self, model: torch.nn.Module, device: torch.device | str, *, lr: float = 1e-4,
                 weight_decay: float = 1e-5, betas=(0.9, 0.999), eps: float = 1e-8,
                 grad_clip: float | None = 1.0, distributed: bool | None = None, bucket_mb: float = 64.0) -> None:
        self.model = model
        self.device = torch.device(device)
        self.grad_clip = grad_clip
        self.arena = FlatArena(model, self.device, with_shadow=self.device.type == "cuda")
        self.optimizer = FlatAdamW(self.arena, lr=lr, betas=betas, eps=eps, weight_decay=weight_decay)
        if distributed is None:
            distributed = dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1
        self.distributed = distributed
        self.bucketer = None
        self.buffer_sync = None
        if distributed:
            broadcast_parameters(self.arena, model)
            self.bucketer = GradBucketer(self.arena, bucket_mb=bucket_mb)
            self.bucketer.attach(model)
            self.buffer_sync = BufferSync(model)
        self.last_grad_norm: torch.Tensor | None = None
        self.limiter = InflightLimiter() if self.device.type == "cuda" else None

    def step(self, loss_fn: Callable[[torch.nn.Module], torch.Tensor]) -> torch.Tensor:
        """Run one optimisation step; returns the (device) loss tensor."""
        self.optimizer.zero_grad()
        if self.buffer_sync is not None:
            self.buffer_sync.sync()
        loss = loss_fn(self.model)
        loss.backward()
        if self.bucketer is not None:
            self.bucketer.finish()
        scale = None
        if self.grad_clip:
            nc = K.grad_clip_coef(self.arena.grad_flat, self.grad_clip)
            self.last_grad_norm = nc[0:1]
            scale = nc[1:2]
        self.optimizer.step(grad_scale=scale)
        if self.limiter is not None:
            self.limiter.step_done()
        return loss.detach()

    # convenience wrappers for the two reference trainers' batch layouts
    def step_localization(self, image: torch.Tensor, coords: torch.Tensor, mask: torch.Tensor) -> torch.Tensor:
        return self.step(lambda m: m.get_loss(m(image), coords, mask=mask))

    def step_classification(self, image: torch.Tensor, targets: dict[str, Any]) -> torch.Tensor:
        return self.step(lambda m: m.get_loss(m(image), targets))
