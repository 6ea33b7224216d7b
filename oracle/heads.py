"""fp32 CPU restatement of the reference models around the backbone (TEST INFRASTRUCTURE ONLY).

CoordinateRegressor: spine_vision/training/models/generic.py:286-417
  head (generic.py:343-351): LayerNorm(F) -> Dropout(p) -> Linear(F,256) -> GELU -> Dropout(p/2)
                             -> Linear(256, L*2) -> Sigmoid ; forward views [B, L, 2] (generic.py:391)
  loss (generic.py:354-361, 410-417): masked-select valid levels, SmoothL1Loss(beta=1) mean
                             (or MSELoss / HuberLoss(delta=0.1)); 0.0 if no valid element.
Classifier: generic.py:48-177
  forward: Dropout(p) on features, then one Linear(F, n_task) per task (generic.py:143-145)
  loss: sum_t w_t * loss_t, targets formatted per strategy (core/tasks.py:177-183, 217-221);
        CrossEntropyLoss(label_smoothing) for multiclass, BCEWithLogitsLoss for binary
        (trainers/classification.py:45-88 sets label_smoothing=0.1 on multiclass tasks).
"""

from __future__ import annotations

import torch
import torch.nn as nn

# (name, num_classes, task_type) for the tasks used by the BASELINE classification config
TASKS = {"pfirrmann": (5, "multiclass"), "modic": (4, "multiclass"), "herniation": (1, "binary")}


class CoordinateRegressor(nn.Module):
    def __init__(self, backbone: nn.Module, feature_dim: int, dropout: float = 0.2, num_levels: int = 5,
                 num_outputs: int = 2, loss_type: str = "smooth_l1") -> None:
        super().__init__()
        self.backbone = backbone
        self.num_levels, self.num_outputs = num_levels, num_outputs
        self.head = nn.Sequential(
            nn.LayerNorm(feature_dim),
            nn.Dropout(dropout),
            nn.Linear(feature_dim, 256),
            nn.GELU(),
            nn.Dropout(dropout / 2),
            nn.Linear(256, num_levels * num_outputs),
            nn.Sigmoid(),
        )
        self.loss_fn = {"mse": nn.MSELoss(), "smooth_l1": nn.SmoothL1Loss(), "huber": nn.HuberLoss(delta=0.1)}[loss_type]

    def forward(self, x):
        return self.head(self.backbone(x)).view(-1, self.num_levels, self.num_outputs)

    def get_loss(self, pred, target, mask=None):
        if mask is not None:
            m = mask.unsqueeze(-1).expand_as(pred).bool()
            vp, vt = pred[m], target[m]
            if vp.numel() == 0:
                return torch.tensor(0.0)
            return self.loss_fn(vp, vt)
        return self.loss_fn(pred, target)


class Classifier(nn.Module):
    def __init__(self, backbone: nn.Module, feature_dim: int, tasks=("pfirrmann", "modic", "herniation"),
                 dropout: float = 0.3, label_smoothing: float = 0.1) -> None:
        super().__init__()
        self.backbone = backbone
        self.dropout = nn.Dropout(dropout)
        self.task_names = list(tasks)
        self.heads = nn.ModuleDict({t: nn.Linear(feature_dim, TASKS[t][0]) for t in tasks})
        self.losses = {
            t: (nn.CrossEntropyLoss(label_smoothing=label_smoothing) if TASKS[t][1] == "multiclass"
                else nn.BCEWithLogitsLoss())
            for t in tasks
        }

    def forward(self, x):
        f = self.dropout(self.backbone(x))
        return {t: h(f) for t, h in self.heads.items()}

    def get_loss(self, preds, targets):
        total = torch.tensor(0.0)
        for t in self.task_names:
            tgt = targets[t]
            if TASKS[t][1] == "multiclass":
                tgt = tgt.long()
            else:
                tgt = tgt.float()
                if tgt.dim() == 1:
                    tgt = tgt.unsqueeze(-1)
            total = total + 1.0 * self.losses[t](preds[t], tgt)
        return total
