"""FocalLoss for binary tasks (reference: spine_vision/training/losses.py:90-139).

Same constructor (gamma, alpha, pos_weight, reduction), same validation and the same arithmetic order
as the reference: p_t from sigmoid(logits), focal weight (1 - p_t)^gamma times the element-wise BCE
on logits (pos_weight applied inside the BCE), then alpha_t, then the reduction.  Pinned against the
reference module's own outputs in tests/golden/focal_loss.json.
"""

from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F


class FocalLoss(nn.Module):
    """FL(p_t) = -alpha_t (1 - p_t)^gamma log(p_t) on logits."""

    def __init__(self, gamma: float = 2.0, alpha: float | None = None, pos_weight: float | None = None,
                 reduction: str = "mean") -> None:
        super().__init__()
        if reduction not in ("none", "mean", "sum"):
            raise ValueError(f"Invalid reduction: {reduction}. Must be 'none', 'mean', or 'sum'.")
        self.gamma, self.alpha, self.pos_weight, self.reduction = gamma, alpha, pos_weight, reduction

    def forward(self, logits: torch.Tensor, targets: torch.Tensor) -> torch.Tensor:
        p = torch.sigmoid(logits)
        p_t = p * targets + (1 - p) * (1 - targets)
        weight = (1 - p_t) ** self.gamma
        pw = torch.tensor(self.pos_weight).to(logits.device) if self.pos_weight is not None else None
        loss = weight * F.binary_cross_entropy_with_logits(logits, targets, reduction="none", pos_weight=pw)
        if self.alpha is not None:
            loss = (self.alpha * targets + (1 - self.alpha) * (1 - targets)) * loss
        if self.reduction == "mean":
            return loss.mean()
        if self.reduction == "sum":
            return loss.sum()
        return loss

    def extra_repr(self) -> str:
        parts = [f"gamma={self.gamma}"]
        if self.alpha is not None:
            parts.append(f"alpha={self.alpha}")
        if self.pos_weight is not None:
            parts.append(f"pos_weight={self.pos_weight}")
        parts.append(f"reduction={self.reduction!r}")
        return ", ".join(parts)
