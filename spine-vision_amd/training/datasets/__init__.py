"""Batch contract of the hot path: the collated dicts the trainers consume.

LocalizationCollator / ClassificationCollator / DynamicTargets keep the reference's batch layout
(spine_vision/training/datasets/localization.py:315-337, classification.py:416-493).  The
synthetic datasets produce the BASELINE input spec (uint8 grayscale -> RGB -> /255 -> ImageNet
normalise); LocalizationDataset reads the reference's annotations.csv + PNG layout (augmentation
is the next row, f1).
"""

from .classification import (
    ClassificationCollator,
    DynamicTargets,
    SyntheticClassificationDataset,
    create_weighted_sampler,
)
from .localization import (
    IDX_TO_LEVEL,
    NUM_LEVELS,
    LocalizationCollator,
    LocalizationDataset,
    SyntheticLocalizationDataset,
)

__all__ = [
    "ClassificationCollator", "DynamicTargets", "IDX_TO_LEVEL", "LocalizationCollator", "LocalizationDataset",
    "NUM_LEVELS", "SyntheticClassificationDataset", "SyntheticLocalizationDataset", "create_weighted_sampler",
]
