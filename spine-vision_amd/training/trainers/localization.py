"""LocalizationTrainer -- drop-in for spine_vision/training/trainers/localization.py:33-533.

Same LocalizationConfig fields/defaults (backbone convnext_base, 512x512, smooth_l1, dropout 0.2,
PCK thresholds ...), same constructor (model / datasets built from the config when not given), same
masked-loss training step (localization.py:186-209) run through the MI355X step (base.py), MED/PCK
validation with an all-gather across ranks, MED as the checkpoint metric, backbone unfreeze hook.
"""

from __future__ import annotations

from pathlib import Path
from typing import Any, Literal

import numpy as np
import torch

from ..datasets.localization import (
    IDX_TO_LEVEL,
    NUM_LEVELS,
    LocalizationCollator,
    LocalizationDataset,
)
from ..metrics import LocalizationMetrics
from ..models.generic import CoordinateRegressor
from .base import BaseTrainer, TrainingConfig, TrainingResult, logger


class LocalizationConfig(TrainingConfig):
    task: str = "localization"
    backbone: str = "convnext_base"
    pretrained: bool = True
    freeze_backbone_epochs: int = 0
    dropout: float = 0.2
    loss_type: Literal["mse", "smooth_l1", "huber"] = "smooth_l1"
    num_levels: int = NUM_LEVELS
    series_types: list[str] | None = None
    sources: list[str] | None = None
    image_size: tuple[int, int] = (512, 512)
    augment: bool = True
    augment_coords: bool = False
    """MI355X build addition: move the keypoints with the train-time flip / affine.  The reference
    augments the image only (its coords come from the CSV), so False keeps its behaviour."""
    pck_thresholds: list[float] = [0.02, 0.05, 0.10]
    visualize_predictions: bool = True
    num_visualization_samples: int = 16


class LocalizationTrainer(BaseTrainer):
    def __init__(self, config: LocalizationConfig, model: CoordinateRegressor | None = None,
                 train_dataset=None, val_dataset=None) -> None:
        if model is None:
            model = CoordinateRegressor(backbone=config.backbone, num_outputs=2, pretrained=config.pretrained,
                                        dropout=config.dropout, freeze_backbone=config.freeze_backbone_epochs > 0,
                                        num_levels=config.num_levels, loss_type=config.loss_type,
                                        precision=config.effective_precision)
        if train_dataset is None:
            train_dataset = LocalizationDataset(Path(config.data_path), split="train", val_ratio=config.val_split,
                                                series_types=config.series_types, sources=config.sources,
                                                image_size=config.image_size, augment=config.augment,
                                                device_transform=config.device_transform,
                                                augment_coords=config.augment_coords)
        if val_dataset is None:
            val_dataset = LocalizationDataset(Path(config.data_path), split="val", val_ratio=config.val_split,
                                              series_types=config.series_types, sources=config.sources,
                                              image_size=config.image_size, augment=False,
                                              device_transform=config.device_transform)
        super().__init__(config, model, train_dataset, val_dataset)
        self.metrics = LocalizationMetrics(pck_thresholds=config.pck_thresholds,
                                           level_names=list(IDX_TO_LEVEL.values()))
        self._backbone_unfrozen = config.freeze_backbone_epochs == 0

    def _collate_fn(self):
        return LocalizationCollator()

    def _unpack_batch(self, batch: dict[str, Any]):
        return batch["image"], batch["coords"]

    def _train_step(self, batch: dict[str, Any]) -> torch.Tensor:
        from ... import kernels as K

        dev = self.device
        # device_transform: Resize (ragged batch) and flip / affine / jitter of the uint8 batch on the GPU
        image = K.device_images(batch, dev)
        coords = batch["coords"].to(dev, non_blocking=True)
        mask = batch["mask"].to(dev, non_blocking=True)
        return self._optimize(lambda: self.model.get_loss(self.model(image), coords, mask=mask))

    def _validate_epoch(self) -> tuple[float, dict[str, float]]:
        from ... import kernels as K

        self.model.eval()
        total, n = 0.0, 0
        P, T, Mk = [], [], []
        dev = self.device
        with torch.no_grad():
            for batch in self.val_loader:
                coords, mask = (batch[k].to(dev) for k in ("coords", "mask"))
                image = K.device_images(batch, dev) if "resize" in batch else batch["image"].to(dev)
                pred = self.model(image)
                total += float(self.model.get_loss(pred, coords, mask=mask))
                n += 1
                P.append(self._gather(pred).cpu())
                T.append(self._gather(coords).cpu())
                Mk.append(self._gather(mask).cpu())
        if not P:
            return 0.0, {}
        fp, ft, fl = self._flatten_with_mask(torch.cat(P), torch.cat(T), torch.cat(Mk))
        return total / n, self.metrics.compute(fp, ft, fl)

    @staticmethod
    def _flatten_with_mask(predictions, targets, masks):
        sel = masks.numpy() > 0
        lv = np.broadcast_to(np.arange(predictions.shape[1]), sel.shape)
        return predictions.numpy()[sel], targets.numpy()[sel], lv[sel]

    def _compute_metrics(self, predictions, targets) -> dict[str, float]:
        return self.metrics.compute(predictions.numpy(), targets.numpy())

    def on_train_begin(self) -> None:
        if self.config.freeze_backbone_epochs > 0:
            logger.info("Backbone frozen for first %d epochs", self.config.freeze_backbone_epochs)
        if hasattr(self.train_dataset, "get_stats"):
            logger.info("Train dataset stats: %s", self.train_dataset.get_stats())

    def on_epoch_begin(self, epoch: int) -> None:
        if not self._backbone_unfrozen and epoch >= self.config.freeze_backbone_epochs:
            logger.info("Unfreezing backbone at epoch %d", epoch + 1)
            self.model.unfreeze_backbone()
            self._backbone_unfrozen = True

    def on_train_end(self, result: TrainingResult) -> None:
        pass  # plots are out of scope

    def get_metric_for_checkpoint(self, val_loss, metrics) -> float:
        if "med" in metrics:
            return metrics["med"]
        return super().get_metric_for_checkpoint(val_loss, metrics)

    def evaluate(self, test_dataset=None) -> dict[str, float]:
        if test_dataset is None:
            c = self.config
            test_dataset = LocalizationDataset(Path(c.data_path), split="test", val_ratio=c.val_split,
                                               series_types=c.series_types, sources=c.sources,
                                               image_size=c.image_size, augment=False,
                                               device_transform=c.device_transform)
        saved = self.val_loader
        self.val_loader = self._create_dataloader(test_dataset, shuffle=False)
        try:
            _, metrics = self._validate_epoch()
        finally:
            self.val_loader = saved
        for k, v in metrics.items():
            logger.info("  %s: %.4f", k, v)
        return metrics
