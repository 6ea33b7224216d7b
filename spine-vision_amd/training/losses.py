"""FocalLoss for binary tasks (reference: spine_vision/training/losses.py:90-139)."""

from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F


class FocalLoss(nn.Module):
    """FL(p_t) = -alpha_t (1 - p_t)^gamma log(p_t) on logits, mean over elements."""

    def __init__(self, gamma: float = 2.0, alpha: float | None = None, reduction: str = "mean") -> None:
        super().__init__()
        self.gamma, self.alpha, self.reduction = gamma, alpha, reduction

    def forward(self, logits: torch.Tensor, targets: torch.Tensor) -> torch.Tensor:
        targets = targets.float()
        bce = F.binary_cross_entropy_with_logits(logits, targets, reduction="none")
        p = torch.sigmoid(logits)
        p_t = p * targets + (1 - p) * (1 - targets)
        loss = (1 - p_t) ** self.gamma * bce
        if self.alpha is not None:
            loss = (self.alpha * targets + (1 - self.alpha) * (1 - targets)) * loss
        if self.reduction == "mean":
            return loss.mean()
        if self.reduction == "sum":
            return loss.sum()
        return loss
