"""Validation metrics (reference: spine_vision/training/metrics.py:121-185; epoch-end, host numpy).

LocalizationMetrics: MED (mean Euclidean distance in normalised coordinates), its std/median,
per-axis MAE, PCK@thresholds (percent), per-level MED.  ClassifierMetrics: the reference's
ClassifierMetrics (metrics.py:321-518) key for key, in numpy.
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
    """Per-task validation metrics with the reference's keys and units
    (spine_vision/training/metrics.py:321-518; ClassificationMetrics 220-316):

    * multiclass (argmax): ``{task}_accuracy`` (percent), ``{task}_balanced_acc`` (mean per-class
      recall, percent), macro F1 over all ``num_classes`` classes (per-class F1 = 2PR/(P+R), 0 when
      P+R = 0);
    * binary (sigmoid > 0.5): ``{task}_accuracy`` (percent), ``{task}_precision``, ``{task}_recall``,
      ``{task}_f1``;
    * ``overall_accuracy`` = mean of the ``*_accuracy`` values; ``f1`` (single task) or ``macro_f1``
      (mean of the task F1s, several tasks) -- the checkpoint-selection metric.
    Multiclass tasks are reported before binary ones, each in ``target_labels`` order, as in the
    reference's dict insertion order."""

    def __init__(self, target_labels: list[str] | None = None, tasks=None) -> None:
        from ..core.tasks import get_task

        if target_labels is None:
            target_labels = [t.name for t in tasks] if tasks is not None else []
        by_name = {t.name: t for t in tasks} if tasks is not None else {}
        self.tasks = [by_name.get(n) or get_task(n) for n in target_labels]
        self._mc = [t for t in self.tasks if t.task_type == "multiclass"]
        self._bin = [t for t in self.tasks if t.task_type == "binary"]
        self.reset()

    def reset(self) -> None:
        self._p: dict[str, list] = {t.name: [] for t in self.tasks}
        self._t: dict[str, list] = {t.name: [] for t in self.tasks}

    @property
    def is_single_task(self) -> bool:
        return len(self._mc) + len(self._bin) == 1

    def update(self, predictions, targets) -> None:
        td = targets.to_dict() if hasattr(targets, "to_dict") else targets

        def get(obj, k):
            return obj.get(k) if isinstance(obj, dict) else getattr(obj, k, None)

        for t in self._mc:
            p, y = get(predictions, t.name), get(td, t.name)
            if p is not None and y is not None:
                self._p[t.name].append(p.detach().argmax(dim=1).cpu().numpy())
                self._t[t.name].append(y.detach().cpu().numpy())
        for t in self._bin:
            p, y = get(predictions, t.name), get(td, t.name)
            if p is not None and y is not None:
                self._p[t.name].append(torch.sigmoid(p.detach().float()).cpu().numpy())
                self._t[t.name].append(y.detach().cpu().numpy())

    def compute(self) -> dict[str, float]:
        out: dict[str, float] = {}
        f1s: list[float] = []
        for t in self._mc:
            if not self._p[t.name]:
                continue
            p, y = np.concatenate(self._p[t.name]), np.concatenate(self._t[t.name])
            out[f"{t.name}_accuracy"] = float(np.mean(p == y) * 100)
            rec, f1 = [], []
            for c in range(t.num_classes):
                tp = int(np.sum((p == c) & (y == c)))
                fp = int(np.sum((p == c) & (y != c)))
                fn = int(np.sum((p != c) & (y == c)))
                pr = tp / (tp + fp) if tp + fp > 0 else 0.0
                rc = tp / (tp + fn) if tp + fn > 0 else 0.0
                rec.append(rc)
                f1.append(2 * pr * rc / (pr + rc) if pr + rc > 0 else 0.0)
            out[f"{t.name}_balanced_acc"] = float(np.mean(rec) * 100)
            f1s.append(float(np.mean(f1)))
        for t in self._bin:
            if not self._p[t.name]:
                continue
            p = (np.concatenate(self._p[t.name]).ravel() > 0.5).astype(int)
            y = np.concatenate(self._t[t.name]).ravel().astype(int)
            out[f"{t.name}_accuracy"] = float(np.mean(p == y) * 100)
            tp = int(np.sum((p == 1) & (y == 1)))
            fp = int(np.sum((p == 1) & (y == 0)))
            fn = int(np.sum((p == 0) & (y == 1)))
            pr = tp / (tp + fp) if tp + fp > 0 else 0.0
            rc = tp / (tp + fn) if tp + fn > 0 else 0.0
            f1 = 2 * pr * rc / (pr + rc) if pr + rc > 0 else 0.0
            out[f"{t.name}_precision"] = float(pr)
            out[f"{t.name}_recall"] = float(rc)
            out[f"{t.name}_f1"] = float(f1)
            f1s.append(f1)
        accs = [v for k, v in out.items() if k.endswith("_accuracy")]
        out["overall_accuracy"] = float(np.mean(accs)) if accs else 0.0
        if f1s:
            out["f1" if self.is_single_task else "macro_f1"] = float(f1s[0] if self.is_single_task else np.mean(f1s))
        return out
