"""One fp32 CPU training step of the reference trainer (TEST INFRASTRUCTURE ONLY).

Restates LocalizationTrainer._train_step (spine_vision/training/trainers/localization.py:186-209) /
ClassificationTrainer._train_step (trainers/classification.py:269-290) on the CPU path, where
accelerate drops fp16 autocast (SURVEY.md §0 finding 2), i.e. plain fp32:
    optimizer.zero_grad(); pred = model(x); loss = get_loss(...); loss.backward()
    clip_grad_norm_(params, grad_clip)            (accelerator.clip_grad_norm_, base.py:592-595)
    optimizer.step()                              (torch.optim.AdamW(lr, weight_decay), base.py:384-390)
"""

from __future__ import annotations

import torch


def make_optimizer(model: torch.nn.Module, lr: float = 1e-4, weight_decay: float = 1e-5) -> torch.optim.AdamW:
    return torch.optim.AdamW(model.parameters(), lr=lr, weight_decay=weight_decay)


def adamw_reference(p, g, m, v, *, lr, beta1, beta2, eps, weight_decay, step):
    """Elementwise AdamW exactly as torch.optim.AdamW(foreach=False) computes it (float64 bias
    corrections), used to pin the flat HIP optimizer kernel."""
    p = p * (1 - lr * weight_decay)
    m = m + (g - m) * (1 - beta1)
    v = v * beta2 + g * g * (1 - beta2)
    bc1 = 1 - beta1**step
    bc2 = 1 - beta2**step
    denom = v.sqrt() / (bc2**0.5) + eps
    return p - (lr / bc1) * m / denom, m, v


def train_step_localization(model, opt, img, coords, mask, grad_clip: float | None = 1.0):
    opt.zero_grad()
    pred = model(img)
    loss = model.get_loss(pred, coords, mask)
    loss.backward()
    norm = None
    if grad_clip:
        norm = torch.nn.utils.clip_grad_norm_(model.parameters(), grad_clip)
    opt.step()
    return float(loss.item()), pred.detach(), norm


def train_step_classification(model, opt, img, targets, grad_clip: float | None = 1.0):
    opt.zero_grad()
    preds = model(img)
    loss = model.get_loss(preds, targets)
    loss.backward()
    norm = None
    if grad_clip:
        norm = torch.nn.utils.clip_grad_norm_(model.parameters(), grad_clip)
    opt.step()
    return float(loss.item()), {k: v.detach() for k, v in preds.items()}, norm
