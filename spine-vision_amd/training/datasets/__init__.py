"""Batch contract of the hot path: the collated dicts the trainers consume.

LocalizationCollator / ClassificationCollator / DynamicTargets keep the reference's batch layout
(spine_vision/training/datasets/localization.py:315-337, classification.py:416-493).  The
synthetic datasets produce the BASELINE input spec (uint8 grayscale -> RGB -> /255 -> ImageNet
normalise); LocalizationDataset reads the reference's annotations.csv + PNG layout; with
``device_transform`` the ToTensor/Normalize tail runs on the GPU (row f1).  ``split_patients`` is the
reference's patient-stratified train/val/test split (row f4).
"""

from .augment import apply_pil, sample_params
from .classification import (
    ClassificationCollator,
    ClassificationDataset,
    DynamicTargets,
    SyntheticClassificationDataset,
    create_weighted_sampler,
)
from .stratification import (
    get_patient_multilabel_matrix,
    get_patient_single_label,
    split_patients,
)
from .localization import (
    IDX_TO_LEVEL,
    NUM_LEVELS,
    LocalizationCollator,
    LocalizationDataset,
    SyntheticLocalizationDataset,
)

__all__ = [
    "ClassificationCollator", "ClassificationDataset", "DynamicTargets", "apply_pil", "sample_params", "IDX_TO_LEVEL", "LocalizationCollator", "LocalizationDataset",
    "NUM_LEVELS", "SyntheticClassificationDataset", "SyntheticLocalizationDataset", "create_weighted_sampler",
    "get_patient_multilabel_matrix", "get_patient_single_label", "split_patients",
]
