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


class ParamGate:
    """Where a forward may start while the previous step's AdamW still runs (StepEngine(overlap_optimizer=True)).

    The optimizer updates the flat arena in chunks on its own stream -- one chunk per group of the backbone's
    ``param_gate_groups()`` (stem, stages, in forward order and arena order), the rest (the model's heads) last -- and
    records an event after each.  The backbone calls ``wait(module)`` before it reads a group's parameters (or their
    bf16 shadow) and ``wait_all()`` before returning, so the heads' reads follow every chunk.  With no optimizer in
    flight both are no-ops."""

    def __init__(self, arena: FlatArena, groups: list) -> None:
        end = {id(p): o + p.numel() for p, o in zip(arena.params, arena.offsets)}
        self.bounds: list[int] = []
        self._chunk: dict[int, int] = {}
        for g in groups:
            ends = [end[id(p)] for p in g.parameters() if id(p) in end]
            if not ends:
                continue
            b = max(ends)
            if self.bounds and b <= self.bounds[-1]:
                raise ValueError("ParamGate: groups out of arena order")
            self.bounds.append(b)
        if not self.bounds or self.bounds[-1] < arena.numel:
            self.bounds.append(arena.numel)
        for g in groups:
            ends = [end[id(p)] for p in g.parameters() if id(p) in end]
            if ends:
                self._chunk[id(g)] = next(i for i, b in enumerate(self.bounds) if b >= max(ends))
        self.events: list | None = None

    def wait(self, module: torch.nn.Module, stream: torch.cuda.Stream | None = None) -> None:
        if self.events is None:
            return
        k = self._chunk.get(id(module), len(self.events) - 1)
        (stream or torch.cuda.current_stream()).wait_event(self.events[k])

    def wait_all(self, stream: torch.cuda.Stream | None = None) -> None:
        if self.events is not None:
            (stream or torch.cuda.current_stream()).wait_event(self.events[-1])


class _Graphed:
    """One captured training step: static inputs, the HIP graph, its loss output and the device AdamW
    scalars [runs][4] refilled before each replay from a small ring of pinned host buffers."""

    def __init__(self, static_inputs, graph, loss, hyper, ranges) -> None:
        self.static_inputs = static_inputs
        self.graph = graph
        self.loss = loss
        self.hyper = hyper
        self.ranges = ranges
        self.ring = [torch.empty(hyper.shape, dtype=torch.float32, pin_memory=True) for _ in range(4)]
        self.ring_events: list = [None] * len(self.ring)
        self.replays = 0


def _copy_into(dst, src) -> None:
    if isinstance(dst, torch.Tensor):
        if dst.data_ptr() != src.data_ptr():
            dst.copy_(src, non_blocking=True)
    elif isinstance(dst, dict):
        for k in dst:
            _copy_into(dst[k], src[k])
    else:
        for d, s_ in zip(dst, src):
            _copy_into(d, s_)


def _clone(x):
    if isinstance(x, torch.Tensor):
        return x.clone()
    if isinstance(x, dict):
        return {k: _clone(v) for k, v in x.items()}
    return type(x)(_clone(v) for v in x)


def _sig(x):
    if isinstance(x, torch.Tensor):
        return (tuple(x.shape), x.dtype, x.device)
    if isinstance(x, dict):
        return tuple((k, _sig(v)) for k, v in sorted(x.items()))
    return tuple(_sig(v) for v in x)


class StepEngine:
    def __init__(self, model: torch.nn.Module, device: torch.device | str, *, lr: float = 1e-4,
                 weight_decay: float = 1e-5, betas=(0.9, 0.999), eps: float = 1e-8,
                 grad_clip: float | None = 1.0, distributed: bool | None = None, bucket_mb: float = 64.0,
                 cuda_graph: bool = False, comm_reserve_cus: int | None = None,
                 overlap_optimizer: bool | None = None) -> None:
        # a backbone whose backward queries events (ConvNeXt's lean side-stream release) declares
        # graph_safe = False and cannot be captured: asking for it is an error, not a silent fallback.
        if cuda_graph:
            unsafe = [type(m).__name__ for m in model.modules() if getattr(m, "graph_safe", True) is False]
            if unsafe:
                raise ValueError(f"cuda_graph=True: {unsafe[0]} is not capture-safe (graph_safe = False)")
        self.model = model
        self.device = torch.device(device)
        if self.device.type == "cuda":  # the kernel library's per-device context (sv_ctx), queried up front
            from .. import native as nv

            self.ctx = nv.device_context(self.device.index if self.device.index is not None else
                                         torch.cuda.current_device())
        self.grad_clip = grad_clip
        self.arena = FlatArena(model, self.device, with_shadow=self.device.type == "cuda")
        self.optimizer = FlatAdamW(self.arena, lr=lr, betas=betas, eps=eps, weight_decay=weight_decay)
        if distributed is None:
            distributed = dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1
        self.distributed = distributed
        self.bucketer = None
        self.buffer_sync = None
        # CUs kept free for RCCL's all-reduce kernels while the backward runs (SV_COMM_RESERVE_CUS; default 0): the
        # backward's persistent GEMM grids are capped at CUs - reserve, and with SV_COMM_CU_MASK=1 the step and the
        # side streams also run on CU-masked streams (training/cumask.py).  Measured on MI355X (DESIGN.md
        # "Multi-GPU", tests/test_comm_reserve_gpu.py, tools/cu_mask_probe.py): neither bounds a comm kernel's
        # start latency -- the data- and weight-gradient GEMMs of the two streams together still cover every CU --
        # and they cost 2.2 % (caps) and 12-24 % (masks) of the step, so the default reserves nothing
        if comm_reserve_cus is None:
            comm_reserve_cus = int(os.environ.get("SV_COMM_RESERVE_CUS", "0")) if distributed else 0
        self.comm_reserve_cus = comm_reserve_cus if self.device.type == "cuda" else 0
        self._stream = None
        if self.comm_reserve_cus > 0:
            mask = os.environ.get("SV_COMM_CU_MASK", "0") != "0"
            if mask:
                from .cumask import reserved_stream

                self._stream = reserved_stream(self.device, self.comm_reserve_cus, "main")
            for m in model.modules():
                if hasattr(m, "comm_reserve_cus"):
                    m.comm_reserve_cus = self.comm_reserve_cus
                    m.comm_cu_mask = mask
        # SV_MAIN_STREAM_PRIO=1 (A/B): the step on a high-priority stream, so that when CUs free up the critical path's
        # next kernel is dispatched before the weight-gradient side stream's queued workgroups
        if self._stream is None and self.device.type == "cuda" and os.environ.get("SV_MAIN_STREAM_PRIO", "0") != "0":
            self._stream = torch.cuda.Stream(self.device, priority=-1)
        if distributed:
            broadcast_parameters(self.arena, model)
            self.bucketer = GradBucketer(self.arena, bucket_mb=bucket_mb)
            self.bucketer.attach(model)
            self.buffer_sync = BufferSync(model)
        self.last_grad_norm: torch.Tensor | None = None
        self.after_backward: Callable[[], None] | None = None  # called once the backward is enqueued (bench)
        self.limiter = InflightLimiter() if self.device.type == "cuda" else None
        # cuda_graph: the whole step (zero grads, forward, backward, clip, AdamW) captured once per input
        # signature as a HIP graph and replayed -- for the launch-bound ResNet step the host enqueue of
        # ~700 kernels (9.6 ms) exceeded the GPU time.  Single-process only (no RCCL inside the graph).
        self.cuda_graph = bool(cuda_graph) and not distributed and self.device.type == "cuda"
        self._graphs: dict = {}
        self._warm: set = set()
        # overlap_optimizer: AdamW runs on its own stream in backbone-stage chunks, and the next step's forward starts
        # each stage once that stage's chunk is done (ParamGate) instead of after the whole update; the next step's
        # gradient zeroing follows the update on that stream and the backward waits for it.  Same arithmetic, same
        # bits.  Parameters read between steps outside the backbone's forward need sync_params() first.  Only for a
        # model whose one gate-aware backbone (param_gate_groups) leads the arena; SV_OPT_OVERLAP=1 turns it on.
        if overlap_optimizer is None:
            overlap_optimizer = os.environ.get("SV_OPT_OVERLAP", "0") != "0"
        self.gate: ParamGate | None = None
        self._opt_stream = None
        self._opt_pending = False
        self._opt_keep = None
        if overlap_optimizer and self.device.type == "cuda" and not self.cuda_graph:
            gated = [m for m in model.modules() if hasattr(m, "param_gate_groups")]
            if len(gated) == 1:
                bb = gated[0]
                first = next((p for p in bb.parameters()), None)
                if first is not None and self.arena.offsets[self.arena.index_of(first)] == 0:
                    self.gate = ParamGate(self.arena, bb.param_gate_groups())
                    bb.param_gate = self.gate
                    self._opt_stream = torch.cuda.Stream(self.device)

    def step(self, loss_fn: Callable[[torch.nn.Module], torch.Tensor]) -> torch.Tensor:
        """Run one optimisation step; returns the (device) loss tensor."""
        if self._stream is None:
            return self._step(loss_fn)
        # the CU-reserved stream: ordered after the caller's stream (the inputs), and the caller's stream after it
        cur = torch.cuda.current_stream(self.device)
        self._stream.wait_stream(cur)
        with torch.cuda.stream(self._stream):
            loss = self._step(loss_fn)
        cur.wait_stream(self._stream)
        return loss

    def sync_params(self, stream: torch.cuda.Stream | None = None) -> None:
        """Order ``stream`` (default: the current one) after an optimizer update still running on the overlap
        stream -- before reading parameters, their gradients or the AdamW state outside the backbone's forward."""
        if self._opt_pending:
            (stream or torch.cuda.current_stream(self.device)).wait_stream(self._opt_stream)

    def _step(self, loss_fn: Callable[[torch.nn.Module], torch.Tensor]) -> torch.Tensor:
        zero_ev = None
        if self._opt_pending:
            # the previous update still reads the gradients: zero them after it, on its stream
            with torch.cuda.stream(self._opt_stream):
                self.optimizer.zero_grad()
            zero_ev = self._opt_stream.record_event()
        else:
            self.optimizer.zero_grad()
        if self.buffer_sync is not None:
            self.buffer_sync.sync()
        loss = loss_fn(self.model)  # the backbone waits for each stage's chunk of the previous update (ParamGate)
        if zero_ev is not None:
            torch.cuda.current_stream(self.device).wait_event(zero_ev)
            self._opt_pending = False
            self.gate.events = None
        loss.backward()
        if self.bucketer is not None:
            self.bucketer.finish()
        if self.after_backward is not None:
            self.after_backward()
        scale = None
        nc = None
        if self.grad_clip:
            nc = K.grad_clip_coef(self.arena.grad_flat, self.grad_clip)
            self.last_grad_norm = nc[0:1]
            scale = nc[1:2]
        if self.gate is not None:
            self._opt_stream.wait_stream(torch.cuda.current_stream(self.device))
            self.gate.events = self.optimizer.step_chunked(self.gate.bounds, self._opt_stream, grad_scale=scale)
            self._opt_keep = nc  # read on the overlap stream: alive until the next step has waited for it
            self._opt_pending = True
        else:
            self.optimizer.step(grad_scale=scale)
        if self.limiter is not None:
            self.limiter.step_done()
        return loss.detach()

    def step_graphed(self, fn: Callable[..., torch.Tensor], inputs: tuple) -> torch.Tensor:
        """step(lambda m: fn(m, *inputs)) through a captured graph: the first call per input signature runs
        eagerly (lazy kernel attributes, caches, side streams), the second captures and replays, later
        calls copy the inputs into the static buffers and replay.  Returns a fresh copy of the loss."""
        if not self.cuda_graph:
            return self.step(lambda m: fn(m, *inputs))
        sig = _sig(inputs)
        if sig not in self._warm:
            self._warm.add(sig)
            return self.step(lambda m: fn(m, *inputs))
        ranges, vals = self.optimizer.begin_graph_step()
        key = (sig, ranges)
        ent = self._graphs.get(key)
        if ent is None:
            hyper = torch.zeros(len(ranges), 4, device=self.device, dtype=torch.float32)
            static = _clone(inputs)
            torch.cuda.synchronize(self.device)
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph):
                self.optimizer.zero_grad()
                loss = fn(self.model, *static)
                loss.backward()
                scale = None
                if self.grad_clip:
                    nc = K.grad_clip_coef(self.arena.grad_flat, self.grad_clip)
                    self.last_grad_norm = nc[0:1]
                    scale = nc[1:2]
                self.optimizer.step_graph(ranges, hyper, grad_scale=scale)
                loss = loss.detach()
            ent = self._graphs[key] = _Graphed(static, graph, loss, hyper, ranges)
        slot = ent.replays % len(ent.ring)
        if ent.ring_events[slot] is not None:
            ent.ring_events[slot].synchronize()  # the H2D copy that last read this pinned buffer is done
        buf = ent.ring[slot]
        buf.copy_(torch.tensor(vals, dtype=torch.float32))
        ent.hyper.copy_(buf, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        ent.ring_events[slot] = ev
        ent.replays += 1
        _copy_into(ent.static_inputs, inputs)
        ent.graph.replay()
        out = ent.loss.clone()
        if self.limiter is not None:
            self.limiter.step_done()
        return out

    # convenience wrappers for the two reference trainers' batch layouts
    def step_localization(self, image: torch.Tensor, coords: torch.Tensor, mask: torch.Tensor) -> torch.Tensor:
        return self.step_graphed(lambda m, x, c, k: m.get_loss(m(x), c, mask=k), (image, coords, mask))

    def step_classification(self, image: torch.Tensor, targets: dict[str, Any]) -> torch.Tensor:
        return self.step_graphed(lambda m, x, t: m.get_loss(m(x), t), (image, targets))
