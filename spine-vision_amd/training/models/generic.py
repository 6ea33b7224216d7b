"""Models around the backbone -- drop-ins for ``CoordinateRegressor`` and ``Classifier``
(spine_vision/training/models/generic.py:48-492): same constructor signatures, module names
(``backbone``, ``head.{0,2,5}`` / ``dropout``, ``heads.<task>``), forward outputs and loss semantics.

The backbone runs on the HIP kernel library; the tiny heads (0.27 M params) stay PyTorch modules.
``CoordinateRegressor.get_loss`` computes the masked mean without boolean indexing (which forces a
device->host sync every step in the reference, generic.py:411-413): sum(mask*loss)/sum(mask), 0 when
no element is valid -- numerically the same mean over the valid elements.
"""

from __future__ import annotations

import os
from typing import Any, Literal

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from ...core.tasks import (
    TaskConfig,
    compute_predictions_for_tasks,
    compute_probabilities_for_tasks,
    create_loss_functions,
    get_strategy,
    get_tasks,
)
from ...native import SV_HEAD_BCE, SV_HEAD_CE
from .backbone import BackboneFactory


class BaseModel(nn.Module):
    """Interface of spine_vision/training/models/base.py:17-178."""

    @property
    def name(self) -> str:  # pragma: no cover - overridden
        raise NotImplementedError

    def predict(self, x: torch.Tensor, **kwargs: Any):
        self.eval()
        with torch.no_grad():
            return self.forward(x, **kwargs)

    def count_parameters(self) -> int:
        return sum(p.numel() for p in self.parameters() if p.requires_grad)

    def freeze_backbone(self) -> None:
        for p in self.backbone.parameters():
            p.requires_grad = False

    def unfreeze_backbone(self) -> None:
        for p in self.backbone.parameters():
            p.requires_grad = True

    def get_features(self, x: torch.Tensor) -> torch.Tensor:
        return self.backbone(x)


# SV_FUSED_HEADS=0: one GEMM per classification head (A/B runs)
_FUSED_HEADS = os.environ.get("SV_FUSED_HEADS", "1") != "0"
# the multi-task loss over the fused head's logits in one HIP launch (kernels.head_loss; SV_FUSED_LOSS=0: torch's
# per-task modules, ~60 launches at bs32)
_FUSED_LOSS = os.environ.get("SV_FUSED_LOSS", "1") != "0"


class _HeadOutputs(dict):
    """The per-task logits (views of one [B, sum(classes)] tensor, ``.logits``) from the fused head."""

    logits: torch.Tensor


class _FusedHeadLoss(torch.autograd.Function):
    """sum_k w_k loss_k(logits[:, cols_k], target_k) and its logits gradient from one launch (sv_head_loss); the
    backward scales the saved gradient by the incoming one."""

    @staticmethod
    def forward(ctx, logits, specs, *targets):
        from ...kernels import head_loss

        loss, dl = head_loss(logits.detach(), [sp + (t,) for sp, t in zip(specs, targets)])
        ctx.save_for_backward(dl)
        return loss

    @staticmethod
    def backward(ctx, g):
        (dl,) = ctx.saved_tensors
        return (dl * g, None) + (None,) * (len(ctx.needs_input_grad) - 2)


class Classifier(BaseModel):
    def __init__(self, backbone: str = "resnet50", tasks: list[TaskConfig] | None = None, pretrained: bool = True,
                 dropout: float = 0.3, freeze_backbone: bool = False, precision: str | None = None) -> None:
        super().__init__()
        self._backbone_name = backbone
        self._tasks = tasks if tasks is not None else get_tasks()
        self._task_names = [t.name for t in self._tasks]
        self.backbone, self._feature_dim = BackboneFactory.create(backbone, pretrained, precision=precision)
        self.dropout = nn.Dropout(dropout)
        self.heads = nn.ModuleDict({t.name: nn.Linear(self._feature_dim, t.num_classes) for t in self._tasks})
        self._loss_functions, self._loss_weights = create_loss_functions(self._tasks)
        if freeze_backbone:
            self.freeze_backbone()

    @property
    def name(self) -> str:
        return f"Classifier-{self._backbone_name}"

    @property
    def task_names(self) -> list[str]:
        return self._task_names

    @property
    def tasks(self) -> list[TaskConfig]:
        return self._tasks

    @property
    def feature_dim(self) -> int:
        return self._feature_dim

    def forward(self, x: torch.Tensor, **kwargs: Any) -> dict[str, torch.Tensor]:
        f = self.dropout(self.backbone(x))
        if f.is_cuda and len(self.heads) > 1 and _FUSED_HEADS:
            # the task heads as ONE [B, F] x [F, sum(classes)] product (one GEMM forward, one per gradient):
            # each head alone is a skinny GEMM that the vendor library runs on a single workgroup
            # (11-56 us each at F = 2048, B = 32); the parameters stay per head (state-dict keys unchanged)
            hs = list(self.heads.values())
            w = torch.cat([h.weight for h in hs])
            b = torch.cat([h.bias for h in hs])
            out = torch.addmm(b, f, w.t())
            res = _HeadOutputs(zip(self.heads.keys(), out.split([h.out_features for h in hs], dim=1)))
            res.logits = out
            return res
        return {n: h(f) for n, h in self.heads.items()}

    def _fused_loss_specs(self, predictions, targets):
        """(specs, targets) for _FusedHeadLoss when every task's loss is a default CrossEntropyLoss / BCEWithLogitsLoss
        over the fused head's logits, else None."""
        logits = getattr(predictions, "logits", None)
        if not (_FUSED_LOSS and logits is not None and logits.is_cuda and logits.dtype == torch.float32
                and logits.dim() == 2 and logits.is_contiguous()):
            return None
        specs, tgts, off = [], [], 0
        for t in self._tasks:
            if t.name not in predictions or t.name not in targets:
                return None
            fn = self._loss_functions[t.name]
            tgt = get_strategy(t).format_target(targets[t.name])
            if type(fn) is nn.CrossEntropyLoss and fn.weight is None and fn.ignore_index == -100 \
                    and fn.reduction == "mean" and tgt.dtype == torch.int64 and tgt.dim() == 1:
                kind, sm = SV_HEAD_CE, fn.label_smoothing
            elif type(fn) is nn.BCEWithLogitsLoss and fn.weight is None and fn.pos_weight is None \
                    and fn.reduction == "mean" and tgt.dtype == torch.float32:
                kind, sm = SV_HEAD_BCE, 0.0
            else:
                return None
            n = predictions[t.name].shape[1]
            if tgt.numel() != logits.shape[0] * (1 if kind == SV_HEAD_CE else n) or not tgt.is_cuda:
                return None
            specs.append((kind, off, n, float(self._loss_weights[t.name]), float(sm)))
            tgts.append(tgt.contiguous())
            off += n
        return tuple(specs), tgts

    def get_loss(self, predictions: dict[str, torch.Tensor], targets: dict[str, torch.Tensor], **kwargs: Any):
        fused = self._fused_loss_specs(predictions, targets)
        if fused is not None:
            specs, tgts = fused
            return _FusedHeadLoss.apply(predictions.logits, specs, *tgts)
        total = torch.zeros((), device=next(self.parameters()).device)
        for t in self._tasks:
            if t.name not in predictions or t.name not in targets:
                continue
            tgt = get_strategy(t).format_target(targets[t.name])
            total = total + self._loss_weights[t.name] * self._loss_functions[t.name](predictions[t.name], tgt)
        return total

    def get_loss_breakdown(self, predictions, targets) -> dict[str, torch.Tensor]:
        return {
            t.name: self._loss_functions[t.name](predictions[t.name], get_strategy(t).format_target(targets[t.name]))
            for t in self._tasks if t.name in predictions and t.name in targets
        }

    def predict(self, x: torch.Tensor, **kwargs: Any) -> dict[str, np.ndarray]:
        self.eval()
        with torch.no_grad():
            out = self.forward(x, **kwargs)
        return compute_predictions_for_tasks(out, self._tasks)

    def predict_proba(self, x: torch.Tensor, **kwargs: Any) -> dict[str, np.ndarray]:
        self.eval()
        with torch.no_grad():
            out = self.forward(x, **kwargs)
        return compute_probabilities_for_tasks(out, self._tasks)


class CoordinateRegressor(BaseModel):
    def __init__(self, backbone: str = "convnext_base", num_outputs: int = 2, pretrained: bool = True,
                 dropout: float = 0.2, freeze_backbone: bool = False, head_config: Any = None,
                 num_levels: int = 5, loss_type: Literal["mse", "smooth_l1", "huber"] = "smooth_l1",
                 precision: str | None = None) -> None:
        super().__init__()
        if head_config is not None:
            raise NotImplementedError("custom head_config is outside the MI355X training path (default head only)")
        self._backbone_name = backbone
        self._num_outputs, self._num_levels = num_outputs, num_levels
        self._loss_type = loss_type
        self.backbone, self._feature_dim = BackboneFactory.create(backbone, pretrained, precision=precision)
        self.head = nn.Sequential(
            nn.LayerNorm(self._feature_dim),
            nn.Dropout(dropout),
            nn.Linear(self._feature_dim, 256),
            nn.GELU(),
            nn.Dropout(dropout / 2),
            nn.Linear(256, num_levels * num_outputs),
            nn.Sigmoid(),
        )
        if loss_type not in ("mse", "smooth_l1", "huber"):
            raise ValueError(f"Unknown loss type: {loss_type}")
        if freeze_backbone:
            self.freeze_backbone()

    @property
    def name(self) -> str:
        return f"Regressor-{self._backbone_name}"

    @property
    def feature_dim(self) -> int:
        return self._feature_dim

    @property
    def num_levels(self) -> int:
        return self._num_levels

    def forward(self, x: torch.Tensor, **kwargs: Any) -> torch.Tensor:
        return self.head(self.backbone(x)).view(-1, self._num_levels, self._num_outputs)

    def _elementwise(self, pred: torch.Tensor, target: torch.Tensor) -> torch.Tensor:
        if self._loss_type == "mse":
            return F.mse_loss(pred, target, reduction="none")
        if self._loss_type == "smooth_l1":
            return F.smooth_l1_loss(pred, target, reduction="none", beta=1.0)
        return F.huber_loss(pred, target, reduction="none", delta=0.1)

    def get_loss(self, predictions: torch.Tensor, targets: torch.Tensor, mask: torch.Tensor | None = None,
                 **kwargs: Any) -> torch.Tensor:
        elem = self._elementwise(predictions, targets)
        if mask is None:
            return elem.mean()
        m = (mask != 0).to(elem.dtype).unsqueeze(-1).expand_as(elem)
        return (elem * m).sum() / m.sum().clamp(min=1.0)
