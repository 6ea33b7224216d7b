from .base import BaseConfig, BaseTrainer, EpochResult, ShardedBatchSampler, TrainingConfig, TrainingResult
from .classification import ClassificationConfig, ClassificationTrainer
from .localization import LocalizationConfig, LocalizationTrainer

__all__ = [
    "BaseConfig", "BaseTrainer", "ClassificationConfig", "ClassificationTrainer", "EpochResult",
    "LocalizationConfig", "LocalizationTrainer", "ShardedBatchSampler", "TrainingConfig", "TrainingResult",
]
