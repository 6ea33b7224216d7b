"""Data-parallel gradient exchange over RCCL (torch.distributed "nccl" backend on ROCm).

Replaces what accelerate.prepare() sets up for the reference (DDP with default 25 MB buckets,
spine_vision/training/trainers/base.py:253-266; container accelerate/accelerator.py:1892-1894) with
an MI355X-first scheme:

* gradients already live in ONE flat f32 buffer (FlatArena), so a bucket is a contiguous slice that
  is all-reduced in place -- no flatten/unflatten copies;
* buckets are formed from the END of the buffer (backward produces gradients in reverse parameter
  order) with a large default size (64 MB) suited to xGMI's per-link ring bandwidth on MI355X;
* the moment the backbone reports a block's gradients final (``grad_ready_hook``) or autograd
  finishes a head parameter (post-accumulate hook), the bucket's readiness is checked; a ready
  bucket records an event on the compute stream, the dedicated high-priority comm stream waits on
  it, and the AVG all-reduce is issued from that stream -- it overlaps the rest of the backward;
* ``finish()`` makes the compute stream wait for every outstanding all-reduce before clip/AdamW.

``broadcast_parameters`` mirrors DDP's initial rank-0 parameter/buffer broadcast.  The bucket
logic is backend-agnostic (gloo on CPU tensors in the unit tests).
"""

from __future__ import annotations

from collections import deque

import torch
import torch.distributed as dist

from .flat import FlatArena


def plan_buckets(arena: FlatArena, bucket_mb: float) -> list[tuple[int, int, list[int]]]:
    """Contiguous buckets (start, end, param indices) of the flat gradient buffer, built from its END
    (backward produces gradients in reverse parameter order), each at least ``bucket_mb``."""
    cap = max(1, int(bucket_mb * 1024 * 1024 // 4))
    buckets: list[tuple[int, int, list[int]]] = []
    cur: list[int] = []
    cur_end = None
    n = len(arena.params)
    for i in reversed(range(n)):
        s = arena.offsets[i]
        e = arena.offsets[i + 1] if i + 1 < n else arena.numel
        if cur_end is None:
            cur_end = e
        cur.append(i)
        if cur_end - s >= cap:
            buckets.append((s, cur_end, cur))
            cur, cur_end = [], None
    if cur:
        buckets.append((arena.offsets[cur[-1]], cur_end, cur))
    return buckets


def _attach_ready(model: torch.nn.Module, arena: FlatArena, mark_ready) -> list:
    """Route gradient readiness to ``mark_ready``: backbones report per block (grad_ready_hook), the
    autograd-managed parameters (the torch head) through post-accumulate hooks.  Returns the hook handles."""
    backbone_params = set()
    for m in model.modules():
        if hasattr(m, "grad_ready_hook"):
            m.grad_ready_hook = mark_ready
            backbone_params |= {id(p) for p in m.parameters()}
    hooks = []
    for p in arena.params:
        if id(p) not in backbone_params and p.requires_grad:
            hooks.append(p.register_post_accumulate_grad_hook(lambda t: mark_ready([t])))
    return hooks


class GradBucketer:
    def __init__(self, arena: FlatArena, bucket_mb: float = 64.0, group=None) -> None:
        self.arena = arena
        self.group = group
        self.world = dist.get_world_size(group)
        # buckets over parameter indices, built from the end of the buffer
        self.buckets: list[tuple[int, int, list[int]]] = plan_buckets(arena, bucket_mb)  # (start, end, params)
        self.param_bucket = {}
        for b, (_, _, idx) in enumerate(self.buckets):
            for i in idx:
                self.param_bucket[id(arena.params[i])] = b
        self.use_streams = arena.grad_flat.is_cuda
        self.comm_stream = torch.cuda.Stream(priority=-1) if self.use_streams else None
        self._hooks = []
        # timing (bench.py): HIP events around every bucket's all-reduce on the comm stream, and around
        # the compute stream's join (the exposed, un-overlapped part of the exchange)
        self.timing = False
        self._bucket_ev = deque(maxlen=64 * len(self.buckets))  # the last 64 steps' bucket events
        self._join_ev = None
        self.reset()

    def reset(self) -> None:
        self.pending = [len(idx) for (_, _, idx) in self.buckets]
        self.seen: set[int] = set()
        self.works = []
        self.launched = [False] * len(self.buckets)
        # per bucket: the last readiness event of EVERY stream that reported some of its gradients (stream handle ->
        # event).  Backbones report from the stream that wrote the gradients (ConvNeXt: block weight gradients on its
        # side stream, downsample / stem ones on the main stream), so the all-reduce must wait for each of them, not
        # only for the stream of the last report
        self.ready_ev: list[dict] = [dict() for _ in self.buckets]

    def attach(self, model: torch.nn.Module) -> None:
        """Route readiness from backbones (grad_ready_hook) and autograd-managed params."""
        self._hooks += _attach_ready(model, self.arena, self.mark_ready)

    def mark_ready(self, params) -> None:
        touched: list[int] = []
        for p in params:
            if id(p) in self.seen or id(p) not in self.param_bucket:
                continue
            self.seen.add(id(p))
            b = self.param_bucket[id(p)]
            self.pending[b] -= 1
            if b not in touched:
                touched.append(b)
        if not touched:
            return
        if self.use_streams:
            # one event on the reporting stream, kept per (bucket, stream): a later report from the same stream
            # supersedes it (stream order)
            cur = torch.cuda.current_stream()
            ev = torch.cuda.Event()
            ev.record(cur)
            for b in touched:
                self.ready_ev[b][cur.cuda_stream] = ev
        for b in touched:
            if self.pending[b] == 0:
                self._launch(b)

    def _wait_ready(self, b: int) -> None:
        """The comm stream waits for every stream that wrote bucket b's gradients (and for the launching stream)."""
        cur = torch.cuda.current_stream()
        evs = self.ready_ev[b]
        if cur.cuda_stream not in evs:
            ev = torch.cuda.Event()
            ev.record(cur)
            evs[cur.cuda_stream] = ev
        for ev in evs.values():
            self.comm_stream.wait_event(ev)

    def _launch(self, b: int) -> None:
        s, e, _ = self.buckets[b]
        view = self.arena.grad_flat[s:e]
        op = dist.ReduceOp.AVG if dist.get_backend(self.group) == "nccl" else dist.ReduceOp.SUM
        if self.use_streams:
            self._wait_ready(b)
            with torch.cuda.stream(self.comm_stream):
                e0 = None
                if self.timing:
                    e0 = torch.cuda.Event(enable_timing=True)
                    e0.record()
                w = dist.all_reduce(view, op=op, group=self.group, async_op=True)
                if op == dist.ReduceOp.AVG:
                    # RCCL: the comm stream waits on RCCL's internal stream (no host block), so later
                    # buckets, the timing event and the compute stream's join are ordered after it
                    w.wait()
                    w = None
                if e0 is not None and w is None:
                    e1 = torch.cuda.Event(enable_timing=True)
                    e1.record()
                    self._bucket_ev.append((e0, e1, view.numel() * view.element_size()))
            # gloo on device tensors: wait() blocks the host until the reduce is done, so it is deferred
            # to finish() (the backward keeps being enqueued meanwhile); its timing event is recorded there,
            # after the wait, so the bucket's time covers the exchange and not only its enqueue
            self.works.append((w, view, op, e0))
        else:
            w = dist.all_reduce(view, op=op, group=self.group, async_op=True)
            self.works.append((w, view, op, None))
        self.launched[b] = True

    def finish(self) -> None:
        """Launch buckets that never became ready (frozen / unused params), then wait for all."""
        for b in range(len(self.buckets)):
            if not self.launched[b]:
                self._launch(b)
        for w, view, op, e0 in self.works:
            if w is None:
                continue
            if self.use_streams:
                with torch.cuda.stream(self.comm_stream):
                    w.wait()
                    if e0 is not None:
                        e1 = torch.cuda.Event(enable_timing=True)
                        e1.record()
                        self._bucket_ev.append((e0, e1, view.numel() * view.element_size()))
                    if op == dist.ReduceOp.SUM and self.world > 1:
                        view.div_(self.world)
                continue
            w.wait()
            if op == dist.ReduceOp.SUM and self.world > 1:
                view.div_(self.world)
        if self.use_streams:
            cur = torch.cuda.current_stream()
            pre = None
            if self.timing:
                pre = torch.cuda.Event(enable_timing=True)
                pre.record(cur)
            cur.wait_stream(self.comm_stream)
            if pre is not None:
                post = torch.cuda.Event(enable_timing=True)
                post.record(cur)
                self._join_ev = (pre, post)
        self.reset()

    def timing_stats(self) -> dict:
        """All-reduce bus bandwidth and overlap of the timed steps (call after a synchronize).

        busbw = 2 (n-1)/n x bytes / time per bucket (the ring all-reduce convention);
        comm_overlap_frac = 1 - exposed / total, where exposed is the time the compute stream waited
        for the exchange after its own backward work was done (last step)."""
        if not self._bucket_ev:
            return {}
        torch.cuda.synchronize()
        n = self.world
        tot_ms = sum(a.elapsed_time(b) for a, b, _ in self._bucket_ev)
        tot_bytes = sum(nb for _, _, nb in self._bucket_ev)
        busbw = [2.0 * (n - 1) / n * nb / (a.elapsed_time(b) * 1e-3) / 1e9 for a, b, nb in self._bucket_ev]
        exposed = self._join_ev[0].elapsed_time(self._join_ev[1]) if self._join_ev else None
        nsteps = max(1, len(self._bucket_ev) // max(1, len(self.buckets)))
        return {
            "buckets": len(self.buckets),
            "bucket_mb": round(tot_bytes / len(self._bucket_ev) / 2**20, 1),
            "allreduce_ms_per_step": round(tot_ms / nsteps, 3),
            "allreduce_busbw_gbs": round(2.0 * (n - 1) / n * tot_bytes / (tot_ms * 1e-3) / 1e9, 1),
            "allreduce_busbw_gbs_max_bucket": round(max(busbw), 1),
            "exposed_ms_last_step": round(exposed, 3) if exposed is not None else None,
            "comm_overlap_frac": (round(max(0.0, 1.0 - exposed / (tot_ms / nsteps)), 4)
                                  if exposed is not None and tot_ms > 0 else None),
        }

    def clear_timing(self) -> None:
        self._bucket_ev.clear()
        self._join_ev = None


class BucketTimeline:
    """Single-GPU rehearsal of the data-parallel exchange (bench.py, world 1): the bucket plan GradBucketer
    would use, an event recorded on the stream where each bucket's last gradient becomes final (the moment
    its all-reduce would launch), and the backward's start / end events.  ``predict`` replays those ready
    times through a model of the comm stream (buckets in ready order, each taking its ring all-reduce time at
    a given bus bandwidth) to estimate the exposed exchange and the N-GPU scaling."""

    def __init__(self, arena: FlatArena, model: torch.nn.Module, bucket_mb: float = 64.0) -> None:
        self.arena = arena
        self.buckets = plan_buckets(arena, bucket_mb)
        self.param_bucket = {id(arena.params[i]): b for b, (_, _, idx) in enumerate(self.buckets) for i in idx}
        self.active = False
        self._hooks = _attach_ready(model, arena, self.mark_ready)
        self.reset()

    def reset(self) -> None:
        self.pending = [len(idx) for (_, _, idx) in self.buckets]
        self.seen: set[int] = set()
        self.ready_ev: list = [None] * len(self.buckets)

    def mark_ready(self, params) -> None:
        if not self.active:
            return
        for p in params:
            if id(p) in self.seen or id(p) not in self.param_bucket:
                continue
            self.seen.add(id(p))
            b = self.param_bucket[id(p)]
            self.pending[b] -= 1
            if self.pending[b] == 0:
                ev = torch.cuda.Event(enable_timing=True)
                ev.record()  # on the stream that made the gradient final (the side stream for most blocks)
                self.ready_ev[b] = ev

    def ready_ms(self, start_ev) -> list:
        """Per bucket: (MB, ms after ``start_ev`` at which it became ready, or None)."""
        torch.cuda.synchronize()
        out = []
        for (s, e, _), ev in zip(self.buckets, self.ready_ev):
            out.append((round((e - s) * 4 / 2**20, 2), round(start_ev.elapsed_time(ev), 3) if ev is not None else None))
        return out

    @staticmethod
    def expected_max(samples, n: int) -> float:
        """E[max of ``n`` independent draws] from the empirical distribution ``samples`` (order statistics:
        sum_i x_(i) [(i/N)^n - ((i-1)/N)^n]).  A collective starts when its slowest rank's comm kernel has started, so
        at ``n`` ranks each bucket waits for the max of ``n`` start latencies, not one rank's."""
        xs = sorted(float(x) for x in samples)
        N = len(xs)
        if N == 0:
            return 0.0
        return sum(x * ((i / N) ** n - ((i - 1) / N) ** n) for i, x in enumerate(xs, start=1))

    # HBM bytes a ring all-reduce moves per rank per byte reduced: reduce-scatter (n-1)/n x {local chunk read, the
    # peer's chunk landing in the staging buffer (written) and read back, the sum written} + all-gather (n-1)/n x
    # {the peer's chunk written, read to forward} = 6 (n-1)/n
    RCCL_HBM_PER_BYTE = 6.0

    @staticmethod
    def predict(ready: list, bwd_end_ms: float, step_ms: float, world: int, busbw_gbs: float,
                reserve_cost: float = 0.0, launch_delay_ms=0.0, latency_samples_ms=None, hbm_gbs: float = 0.0) -> dict:
        """Exposed exchange and scaling at ``world`` ranks if every bucket's ring all-reduce takes
        2 (n-1)/n x bytes / busbw on one comm stream, launched at its ready time (a bucket never ready in the
        backward launches at its end); the step grows by what finishes after the backward's end.
        ``reserve_cost``: the measured fractional slowdown of the step under the data-parallel CU reserve,
        which stretches the whole timeline (ready times, backward end, step) before the exchange is added;
        ``launch_delay_ms``: (mid, end) -- how long a comm kernel may wait behind the backward's kernels after its
        ready event while the backward runs (mid), and its start latency once the compute queues are idle (end).  A
        bucket that becomes ready shortly before the backward's end waits at most for the rest of the backward:
        delay = min(mid, time left in the backward + end).  A scalar applies to both.
        ``latency_samples_ms``: measured per-launch start latencies during the backward (tests/test_comm_reserve_gpu.py);
        when given, the mid delay of every bucket is the expected MAX over ``world`` ranks' draws from them (the
        collective waits for its slowest rank) -- never below it: max(that, the scalar mid) is NOT taken, the scalar is
        then ignored, so the caller picks the model.
        ``hbm_gbs`` > 0: RCCL's own HBM traffic (RCCL_HBM_PER_BYTE (n-1)/n x the bytes reduced) competes with the
        backward; charged as a stretch of the backward by traffic / hbm_gbs (an upper bound: it assumes the backward is
        HBM-bound for the whole overlap)."""
        f = 1.0 + reserve_cost
        bwd_end_ms, step_dp = bwd_end_ms * f, step_ms * f
        d_mid, d_end = launch_delay_ms if isinstance(launch_delay_ms, (tuple, list)) else (launch_delay_ms,) * 2
        if latency_samples_ms:
            d_mid = BucketTimeline.expected_max(latency_samples_ms, world)
        total_mb = sum(mb for mb, _ in ready)
        hbm_ms = 0.0
        if hbm_gbs > 0 and world > 1:
            hbm_ms = BucketTimeline.RCCL_HBM_PER_BYTE * (world - 1) / world * total_mb * 2**20 / (hbm_gbs * 1e9) * 1e3
        # the stretch is spread over the backward: a bucket ready at r has paid (r / bwd_end) of it
        g = 1.0 + hbm_ms / bwd_end_ms if bwd_end_ms > 0 else 1.0
        t = 0.0
        for mb, r in sorted(ready, key=lambda x: (x[1] is None, x[1] if x[1] is not None else 0.0)):
            rr = r * f * g if r is not None else bwd_end_ms * g
            start = max(t, rr + min(d_mid, max(0.0, bwd_end_ms * g - rr) + d_end))
            t = start + 2.0 * (world - 1) / world * mb * 2**20 / (busbw_gbs * 1e9) * 1e3
        bwd_end_g = bwd_end_ms * g
        exposed = max(0.0, t - bwd_end_g)
        step_pred = step_dp + hbm_ms + exposed
        return {"world": world, "busbw_gbs": busbw_gbs, "reserve_cost_frac": reserve_cost,
                "launch_delay_ms": [round(d_mid, 6), d_end],
                "launch_delay_model": (f"expected max over {world} ranks of {len(latency_samples_ms)} measured latencies"
                                       if latency_samples_ms else "fixed"),
                "rccl_hbm_stretch_ms": round(hbm_ms, 3),
                "comm_end_ms": round(t, 3), "exposed_ms": round(exposed, 3),
                "predicted_step_ms": round(step_pred, 3),
                "predicted_scaling": round(world * step_ms / step_pred, 3)}


class BufferSync:
    """DDP's per-forward ``broadcast_buffers=True`` (the reference's accelerate default): rank 0's
    floating buffers -- the ResNet BatchNorm running statistics -- overwrite every rank's before
    each step.  The buffers are rebound as views of ONE flat f32 tensor so the sync is a single
    broadcast (ResNet-50: 53k floats) instead of ~160 small ones.  Integer buffers
    (num_batches_tracked) advance identically on every rank and are not sent."""

    def __init__(self, model: torch.nn.Module, src: int = 0, group=None) -> None:
        self.src, self.group = src, group
        slots = []
        for mod in model.modules():
            for name, b in mod._buffers.items():
                if b is not None and b.is_floating_point():
                    slots.append((mod, name, b))
        self.flat = None
        if not slots:
            return
        total = sum(b.numel() for _, _, b in slots)
        self.flat = torch.empty(total, device=slots[0][2].device, dtype=torch.float32)
        off = 0
        with torch.no_grad():
            for mod, name, b in slots:
                v = self.flat[off : off + b.numel()].view_as(b)
                v.copy_(b)
                mod._buffers[name] = v
                off += b.numel()

    def sync(self) -> None:
        if self.flat is not None:
            dist.broadcast(self.flat, self.src, group=self.group)


def broadcast_parameters(arena: FlatArena, model: torch.nn.Module, src: int = 0, group=None) -> None:
    """DDP's constructor-time broadcast: rank 0's parameters and buffers to every rank."""
    dist.broadcast(arena.param_flat, src, group=group)
    for b in model.buffers():
        dist.broadcast(b, src, group=group)
    if arena.shadow_flat is not None:
        arena.refresh_shadow()
