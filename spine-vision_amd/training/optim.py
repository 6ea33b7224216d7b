"""AdamW over the flat arena -- the optimizer behind ``BaseTrainer._create_optimizer``
(spine_vision/training/trainers/base.py:384-390: ``torch.optim.AdamW(params, lr, weight_decay)``,
betas (0.9, 0.999), eps 1e-8, one param group, weight decay on every parameter).

It is a ``torch.optim.Optimizer`` so LR schedulers (CosineAnnealingLR etc.) drive
``param_groups[0]["lr"]`` as in the reference, and its ``state_dict`` has torch's AdamW layout
(per-parameter ``step``/``exp_avg``/``exp_avg_sq``) so checkpoints interchange with the reference's.
``step()`` is one HIP kernel per contiguous run of trainable parameters; the clip coefficient is a
device scalar (no host sync); the bf16 GEMM shadow is refreshed in the same pass.
"""

from __future__ import annotations

import torch

from .. import kernels as K
from .flat import FlatArena, _align


class FlatAdamW(torch.optim.Optimizer):
    def __init__(self, arena: FlatArena, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8,
                 weight_decay: float = 1e-2) -> None:
        defaults = dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay, amsgrad=False, maximize=False,
                        foreach=None, capturable=False, differentiable=False, fused=None,
                        decoupled_weight_decay=True)  # torch.optim.AdamW's param-group keys
        super().__init__(arena.params, defaults)
        self.arena = arena
        self.exp_avg = torch.zeros_like(arena.param_flat)
        self.exp_avg_sq = torch.zeros_like(arena.param_flat)
        # torch.optim.AdamW keeps one step count PER PARAMETER, starting when the parameter first
        # takes a step.  A backbone frozen for ``freeze_backbone_epochs`` (the reference's
        # localization.py:383-389 hook) therefore starts its bias correction at step 1 after the
        # unfreeze, not at the head's count.  Runs of the flat buffer are cut where the counts differ.
        self._steps = [0] * len(arena.params)

    @torch.no_grad()
    def step(self, closure=None, grad_scale: torch.Tensor | None = None):
        """One AdamW update of every trainable parameter; ``grad_scale`` is an optional device
        scalar multiplying the gradients first (the clip coefficient)."""
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        group = self.param_groups[0]
        a = self.arena
        shadow = a.shadow_flat
        for s, e, st in self._runs():
            K.adamw_flat(a.param_flat[s:e], a.grad_flat[s:e], self.exp_avg[s:e], self.exp_avg_sq[s:e],
                         shadow[s:e] if shadow is not None else None, lr=group["lr"], beta1=group["betas"][0],
                         beta2=group["betas"][1], eps=group["eps"], weight_decay=group["weight_decay"],
                         step=st, grad_scale=grad_scale)
        return loss

    @torch.no_grad()
    def step_chunked(self, bounds: list[int], stream: torch.cuda.Stream,
                     grad_scale: torch.Tensor | None = None) -> list[torch.cuda.Event]:
        """step() on ``stream`` in arena chunks [0, bounds[0]), [bounds[0], bounds[1]), ... (bounds ascending, the
        last = arena.numel): the same per-element update (bitwise step()'s), one event recorded after each chunk, so
        that a forward can start on a stage as soon as that stage's chunk is done (StepEngine(overlap_optimizer))."""
        group = self.param_groups[0]
        a = self.arena
        shadow = a.shadow_flat
        runs = self._runs()
        events = []
        lo = 0
        with torch.cuda.stream(stream):
            for hi in bounds:
                for s, e, st in runs:
                    s_, e_ = max(s, lo), min(e, hi)
                    if s_ >= e_:
                        continue
                    K.adamw_flat(a.param_flat[s_:e_], a.grad_flat[s_:e_], self.exp_avg[s_:e_], self.exp_avg_sq[s_:e_],
                                 shadow[s_:e_] if shadow is not None else None, lr=group["lr"],
                                 beta1=group["betas"][0], beta2=group["betas"][1], eps=group["eps"],
                                 weight_decay=group["weight_decay"], step=st, grad_scale=grad_scale)
                events.append(stream.record_event())
                lo = hi
        return events

    def _runs(self) -> list[tuple[int, int, int]]:
        """Advance the step count of every trainable parameter and return the maximal contiguous
        [start, end) ranges of trainable parameters that share a (new) step count."""
        a = self.arena
        runs: list[list[int]] = []
        for i, (p, o) in enumerate(zip(a.params, a.offsets)):
            if not p.requires_grad:
                continue
            self._steps[i] += 1
            e = o + _align(p.numel())
            if runs and runs[-1][1] == o and runs[-1][2] == self._steps[i]:
                runs[-1][1] = e
            else:
                runs.append([o, e, self._steps[i]])
        return [tuple(r) for r in runs]

    # -- graph replay (StepEngine(cuda_graph=True)) ----------------------------------------------
    def begin_graph_step(self) -> tuple[tuple, list[list[float]]]:
        """Advance the step counts as step() would and return (the runs' [start, end) ranges, per run the
        f32 [lr, 1 - b1^step, sqrt(1 - b2^step)] the captured update reads from device memory)."""
        group = self.param_groups[0]
        b1, b2 = group["betas"]
        runs = self._runs()
        return (tuple((s, e) for s, e, _ in runs),
                [K.adamw_hyper(group["lr"], b1, b2, st) + [0.0] for _, _, st in runs])

    @torch.no_grad()
    def step_graph(self, ranges: tuple, hyper: torch.Tensor, grad_scale: torch.Tensor | None = None) -> None:
        """The update of step() for the given runs with lr / bias corrections from ``hyper`` [runs][4]
        (device): what a captured graph replays; the host counts advance in begin_graph_step."""
        group = self.param_groups[0]
        a = self.arena
        shadow = a.shadow_flat
        for i, (s, e) in enumerate(ranges):
            K.adamw_flat(a.param_flat[s:e], a.grad_flat[s:e], self.exp_avg[s:e], self.exp_avg_sq[s:e],
                         shadow[s:e] if shadow is not None else None, lr=0.0, beta1=group["betas"][0],
                         beta2=group["betas"][1], eps=group["eps"], weight_decay=group["weight_decay"], step=1,
                         grad_scale=grad_scale, hyper=hyper[i])

    @property
    def _step(self) -> int:
        """Largest per-parameter step count (the count of an optimizer that never froze anything)."""
        return max(self._steps) if self._steps else 0

    def zero_grad(self, set_to_none: bool = True) -> None:  # grads live in the arena: always zero
        self.arena.zero_grad()

    # -- torch AdamW-compatible state dict ---------------------------------------------------------
    def state_dict(self):
        sd = super().state_dict()
        a = self.arena
        state = {}
        for i, (p, o) in enumerate(zip(a.params, a.offsets)):
            if self._steps[i] == 0:  # torch writes no state for a parameter that never stepped
                continue
            n = p.numel()
            state[i] = {
                "step": torch.tensor(float(self._steps[i])),
                "exp_avg": self.exp_avg[o : o + n].view_as(p).clone(),
                "exp_avg_sq": self.exp_avg_sq[o : o + n].view_as(p).clone(),
            }
        sd["state"] = state
        return sd

    def load_state_dict(self, state_dict):
        groups = state_dict["param_groups"]
        for g, sg in zip(self.param_groups, groups):
            for k, v in sg.items():
                if k != "params":
                    g[k] = v
        a = self.arena
        st = state_dict.get("state", {})
        with torch.no_grad():
            for i, (p, o) in enumerate(zip(a.params, a.offsets)):
                s = st.get(i)
                n = p.numel()
                if not s:
                    self._steps[i] = 0
                    self.exp_avg[o : o + n].zero_()
                    self.exp_avg_sq[o : o + n].zero_()
                    continue
                self.exp_avg[o : o + n].copy_(s["exp_avg"].reshape(-1).to(self.exp_avg.device))
                self.exp_avg_sq[o : o + n].copy_(s["exp_avg_sq"].reshape(-1).to(self.exp_avg.device))
                self._steps[i] = int(float(s["step"]))
