"""ClassificationTrainer -- drop-in for spine_vision/training/trainers/classification.py:45-559.

Same ClassificationConfig fields/defaults (resnet18, 256x256, dropout 0.3, label_smoothing 0.1,
weighted sampling), same task construction (_create_tasks_for_training: label smoothing on
multiclass, BCE/Focal on binary), same multi-task step (classification.py:269-290), F1 as the
checkpoint metric.  Rank-local validation metrics (the reference does not gather them either).
"""

from __future__ import annotations

from pathlib import Path

from typing import Any

import torch

from ...core.tasks import AVAILABLE_TASK_NAMES, TaskConfig, get_task
from ..datasets.classification import ClassificationCollator, ClassificationDataset, create_weighted_sampler
from ..metrics import ClassifierMetrics
from ..models.generic import Classifier
from .base import BaseTrainer, TrainingConfig, logger


def _create_tasks_for_training(target_labels: list[str] | None = None, label_smoothing: float = 0.1,
                               use_focal_loss: bool = False, focal_gamma: float = 2.0,
                               focal_alpha: float | None = None) -> list[TaskConfig]:
    labels = list(AVAILABLE_TASK_NAMES) if target_labels is None else target_labels
    bad = set(labels) - set(AVAILABLE_TASK_NAMES)
    if bad:
        raise ValueError(f"Invalid target labels: {bad}. Available: {AVAILABLE_TASK_NAMES}")
    out = []
    for lab in labels:
        t = get_task(lab)
        if t.is_multiclass:
            t = t.with_overrides(label_smoothing=label_smoothing)
        elif t.is_binary:
            t = t.with_overrides(use_focal_loss=use_focal_loss, focal_gamma=focal_gamma, focal_alpha=focal_alpha)
        out.append(t)
    return out


class ClassificationConfig(TrainingConfig):
    task: str = "classification"
    data_path: Path = Path("data/processed/classification")
    backbone: str = "resnet18"
    pretrained: bool = True
    dropout: float = 0.3
    freeze_backbone_epochs: int = 0
    label_smoothing: float = 0.1
    use_weighted_sampling: bool = True
    sampler_label: str | None = None
    levels: list[str] | None = None
    series_types: list[str] | None = None
    target_labels: list[str] | None = None
    output_size: tuple[int, int] = (256, 256)
    augment: bool = True
    use_focal_loss: bool = False
    focal_gamma: float = 2.0
    focal_alpha: float | None = None
    visualize_predictions: bool = True
    num_visualization_samples: int = 16
    max_samples_per_cell: int = 4


class ClassificationTrainer(BaseTrainer):
    def __init__(self, config: ClassificationConfig, model: Classifier | None = None, train_dataset=None,
                 val_dataset=None) -> None:
        common = dict(val_ratio=config.val_split, levels=config.levels, series_types=config.series_types,
                      target_labels=config.target_labels, output_size=config.output_size,
                      device_transform=config.device_transform)
        if train_dataset is None:
            train_dataset = ClassificationDataset(Path(config.data_path), split="train", augment=config.augment,
                                                  **common)
        if val_dataset is None:
            val_dataset = ClassificationDataset(Path(config.data_path), split="val", augment=False, **common)
        if config.device_transform:
            # row f1: datasets that support it yield the uint8 [H,W,3] crop (normalised on the device)
            for ds in (train_dataset, val_dataset):
                if hasattr(ds, "device_transform"):
                    ds.device_transform = True
        target_labels = config.target_labels or list(AVAILABLE_TASK_NAMES)
        self._sampler_obj = None
        if config.use_weighted_sampling and hasattr(train_dataset, "records"):
            label = config.sampler_label or target_labels[0]
            self._sampler_obj = create_weighted_sampler(train_dataset, label)
            logger.info("Using weighted sampling based on '%s' label", label)
        tasks = _create_tasks_for_training(config.target_labels, config.label_smoothing, config.use_focal_loss,
                                           config.focal_gamma, config.focal_alpha)
        if model is None:
            model = Classifier(backbone=config.backbone, tasks=tasks, pretrained=config.pretrained,
                               dropout=config.dropout, freeze_backbone=config.freeze_backbone_epochs > 0,
                               precision=config.effective_precision)
        super().__init__(config, model, train_dataset, val_dataset)
        self._target_labels = target_labels
        self._tasks = tasks
        self.metrics = ClassifierMetrics(target_labels=target_labels)
        self._backbone_unfrozen = config.freeze_backbone_epochs == 0

    def _collate_fn(self):
        return ClassificationCollator()

    def _sampler(self, dataset, shuffle: bool):
        if shuffle and getattr(self, "_sampler_obj", None) is not None:
            g = torch.Generator()
            g.manual_seed(self.config.seed)
            self._sampler_obj.generator = g  # one synchronised stream, sharded by batch across ranks
            return self._sampler_obj
        return super()._sampler(dataset, shuffle)

    def _unpack_batch(self, batch: dict[str, Any]):
        return batch["image"], batch["targets"]

    def _train_step(self, batch: dict[str, Any]) -> torch.Tensor:
        from ... import kernels as K

        # device_transform: Resize (ragged batch) and affine / jitter of the uint8 crops on the GPU
        image = K.device_images(batch, self.device)
        targets = batch["targets"].to(self.device).to_dict()
        return self._optimize(lambda: self.model.get_loss(self.model(image), targets))

    def _validate_epoch(self) -> tuple[float, dict[str, float]]:
        from ... import kernels as K

        self.model.eval()
        self.metrics.reset()
        total, n = 0.0, 0
        with torch.no_grad():
            for batch in self.val_loader:
                image = K.device_images(batch, self.device) if "resize" in batch else batch["image"].to(self.device)
                targets = batch["targets"].to(self.device)
                pred = self.model(image)
                total += float(self.model.get_loss(pred, targets.to_dict()))
                n += 1
                self.metrics.update(pred, targets)
        return total / max(n, 1), self.metrics.compute()

    def on_epoch_begin(self, epoch: int) -> None:
        if not self._backbone_unfrozen and epoch >= self.config.freeze_backbone_epochs:
            self.model.unfreeze_backbone()
            self._backbone_unfrozen = True

    def get_metric_for_checkpoint(self, val_loss, metrics) -> float:
        if "f1" in metrics:
            return -metrics["f1"]
        if "macro_f1" in metrics:
            return -metrics["macro_f1"]
        return super().get_metric_for_checkpoint(val_loss, metrics)
