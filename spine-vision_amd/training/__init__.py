"""Training path: models, flat-buffer optimizer, RCCL gradient exchange, step engine, trainers."""

from .comm import GradBucketer, broadcast_parameters
from .engine import StepEngine
from .flat import FlatArena
from .models.backbone import BACKBONES, BackboneFactory
from .models.generic import BaseModel, Classifier, CoordinateRegressor
from .optim import FlatAdamW
from .trainers import (
    BaseTrainer,
    ClassificationConfig,
    ClassificationTrainer,
    LocalizationConfig,
    LocalizationTrainer,
    TrainingConfig,
    TrainingResult,
)

__all__ = [
    "BACKBONES", "BackboneFactory", "BaseModel", "Classifier", "CoordinateRegressor", "FlatAdamW", "FlatArena",
    "GradBucketer", "StepEngine", "broadcast_parameters", "BaseTrainer", "ClassificationConfig",
    "ClassificationTrainer", "LocalizationConfig", "LocalizationTrainer", "TrainingConfig", "TrainingResult",
]
