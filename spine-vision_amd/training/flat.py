"""Flat parameter / gradient / shadow arena.

Every parameter of a model is re-homed into ONE contiguous f32 buffer (``p.data`` becomes a view),
every ``p.grad`` into a second one with identical offsets, and the bf16 weight shadow read by the
MFMA GEMMs into a third.  That turns the reference's per-tensor optimizer and clip
(``torch.optim.AdamW`` foreach + ``clip_grad_norm_``, spine_vision/training/trainers/base.py:384-390,
592-597) into single streaming kernels, and lets the DDP bucketer all-reduce contiguous slices of
the gradient buffer in place (no gather/scatter copies).  Offsets are 64-byte aligned so every
kernel can use 16-byte vector accesses on any slice.
"""

from __future__ import annotations

import torch
import torch.nn as nn

from .. import kernels as K

ALIGN = 16  # elements (64 B)


def _align(n: int) -> int:
    return (n + ALIGN - 1) // ALIGN * ALIGN


class FlatArena:
    def __init__(self, model: nn.Module, device: torch.device | str, with_shadow: bool = True) -> None:
        self.model = model
        self.device = torch.device(device)
        seen: set[int] = set()
        self.params: list[nn.Parameter] = []
        self.names: list[str] = []
        for name, p in model.named_parameters():
            if id(p) in seen:
                continue
            seen.add(id(p))
            self.params.append(p)
            self.names.append(name)
        self.offsets: list[int] = []
        off = 0
        for p in self.params:
            self.offsets.append(off)
            off += _align(p.numel())
        self.numel = off
        self.param_flat = torch.zeros(off, device=self.device, dtype=torch.float32)
        self.grad_flat = torch.zeros(off, device=self.device, dtype=torch.float32)
        with torch.no_grad():
            for p, o in zip(self.params, self.offsets):
                v = self.param_flat[o : o + p.numel()].view_as(p)
                v.copy_(p.detach().to(self.device, torch.float32))
                p.data = v
                p.grad = self.grad_flat[o : o + p.numel()].view_as(p)
        self.shadow_flat = None
        self.shadow: dict[int, torch.Tensor] = {}
        if with_shadow:
            self.shadow_flat = torch.empty(off, device=self.device, dtype=torch.bfloat16)
            for p, o in zip(self.params, self.offsets):
                self.shadow[id(p)] = self.shadow_flat[o : o + p.numel()].view_as(p)
            self.refresh_shadow()
            # a load_state_dict through the model (or through the backbone alone, e.g. loading
            # best_model.pt before evaluate/predict) rewrites the f32 masters in place: re-derive the
            # bf16 shadow the GEMMs read, or they would mix stale bf16 weights with fresh f32 ones
            hooked = [model] + [m for m in model.modules() if hasattr(m, "set_weight_shadow") and m is not model]
            for m in hooked:
                m.register_load_state_dict_post_hook(lambda _m, _keys: self.refresh_shadow())
            for m in model.modules():
                if hasattr(m, "set_weight_shadow"):
                    m.set_weight_shadow(self.shadow)

    # ------------------------------------------------------------------------------------------
    def index_of(self, p: torch.Tensor) -> int:
        for i, q in enumerate(self.params):
            if q is p:
                return i
        raise KeyError("parameter not in arena")

    def span(self, p: torch.Tensor) -> tuple[int, int]:
        i = self.index_of(p)
        return self.offsets[i], self.offsets[i] + _align(self.params[i].numel())

    def refresh_shadow(self) -> None:
        """Re-derive the bf16 shadow from the f32 master weights (after init / load_state_dict)."""
        if self.shadow_flat is not None:
            K.cast_bf16(self.param_flat, self.shadow_flat)

    def zero_grad(self) -> None:
        self.grad_flat.zero_()
        # re-attach in case user code set p.grad = None
        for p, o in zip(self.params, self.offsets):
            if p.grad is None or p.grad.data_ptr() != self.grad_flat[o:].data_ptr():
                p.grad = self.grad_flat[o : o + p.numel()].view_as(p)

    def check_bound(self) -> None:
        """Raise if a parameter was re-bound outside the arena (e.g. model.to() after creation)."""
        for p, o in zip(self.params, self.offsets):
            if p.data_ptr() != self.param_flat[o:].data_ptr():
                raise RuntimeError("parameter storage moved out of the flat arena; rebuild the arena")

    def trainable_runs(self) -> list[tuple[int, int]]:
        """Maximal contiguous [start, end) element ranges of parameters with requires_grad."""
        runs: list[tuple[int, int]] = []
        for p, o in zip(self.params, self.offsets):
            if not p.requires_grad:
                continue
            e = o + _align(p.numel())
            if runs and runs[-1][1] == o:
                runs[-1] = (runs[-1][0], e)
            else:
                runs.append((o, e))
        return runs
