"""Validation metrics (reference: spine_vision/training/metrics.py:121-185; epoch-end, host numpy).

LocalizationMetrics: MED (mean Euclidean distance in normalised coordinates), its std/median,
per-axis MAE, PCK@thresholds (percent), per-level MED.  ClassifierMetrics: per-task accuracy and
macro-F1 (multiclass) / F1 (binary) computed with numpy -- the reference's torchmetrics collections
are validation-only and outside the hot path.
"""

from __future__ import annotations

from typing import Any

import numpy as np
import torch


class LocalizationMetrics:
    def __init__(self, pck_thresholds=(0.02, 0.05, 0.10), level_names=None) -> None:
        self.pck_thresholds = list(pck_thresholds)
        self.level_names = list(level_names or [])

    def compute(self, predictions, targets, levels=None, **kwargs: Any) -> dict[str, float]:
        p = predictions.cpu().numpy() if isinstance(predictions, torch.Tensor) else np.asarray(predictions)
        t = targets.cpu().numpy() if isinstance(targets, torch.Tensor) else np.asarray(targets)
        if p.size == 0:
            return {}
        d = np.sqrt(((p - t) ** 2).sum(axis=1))
        m = {"med": float(d.mean()), "med_std": float(d.std()), "med_median": float(np.median(d))}
        ae = np.abs(p - t)
        m.update(mae_x=float(ae[:, 0].mean()), mae_y=float(ae[:, 1].mean()), mae=float(ae.mean()))
        for th in self.pck_thresholds:
            m[f"pck@{th:.2f}"] = float((d < th).mean() * 100)
        if levels is not None:
            lv = np.asarray(levels)
            for i, name in enumerate(self.level_names):
                sel = lv == i
                if sel.any():
                    m[f"med_{name}"] = float(d[sel].mean())
        return m


class ClassifierMetrics:
    def __init__(self, target_labels: list[str]) -> None:
        from ..core.tasks import get_task

        self.tasks = [get_task(t) for t in target_labels]
        self.reset()

    def reset(self) -> None:
        self._p: dict[str, list] = {t.name: [] for t in self.tasks}
        self._t: dict[str, list] = {t.name: [] for t in self.tasks}

    def update(self, predictions: dict[str, torch.Tensor], targets) -> None:
        from ..core.tasks import get_strategy

        td = targets.to_dict() if hasattr(targets, "to_dict") else targets
        for t in self.tasks:
            if t.name in predictions and t.name in td:
                self._p[t.name].append(get_strategy(t).compute_predictions(predictions[t.name]).cpu().numpy().ravel())
                self._t[t.name].append(td[t.name].cpu().numpy().ravel().astype(np.int64))

    def compute(self) -> dict[str, float]:
        out: dict[str, float] = {}
        f1s = []
        for t in self.tasks:
            if not self._p[t.name]:
                continue
            p, y = np.concatenate(self._p[t.name]), np.concatenate(self._t[t.name])
            out[f"{t.name}_accuracy"] = float((p == y).mean())
            ncls = max(t.num_classes, 2)
            per = []
            for c in range(ncls) if t.is_multiclass else [1]:
                tp = float(((p == c) & (y == c)).sum())
                fp = float(((p == c) & (y != c)).sum())
                fn = float(((p != c) & (y == c)).sum())
                per.append(0.0 if tp == 0 else 2 * tp / (2 * tp + fp + fn))
            f1 = float(np.mean(per))
            out[f"{t.name}_{'macro_f1' if t.is_multiclass else 'f1'}"] = f1
            f1s.append(f1)
        if f1s:
            out["macro_f1"] = float(np.mean(f1s))
        return out
