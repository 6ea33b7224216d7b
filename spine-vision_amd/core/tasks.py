"""Classification task registry and per-task-type strategies.

Behavioural mirror of spine_vision/core/tasks.py (TaskConfig 34-107, strategies 142-335, registry
368-427, create_loss_functions 483-502): the same task names / class counts / types, the same loss
per task type (CrossEntropyLoss(label_smoothing) for multiclass & ordinal, BCEWithLogitsLoss or
FocalLoss for binary & multilabel, MSELoss for regression), the same target formatting (long for
CE, float [B,1] for BCE) and prediction / probability rules.  torchmetrics collections (validation
only, out of the hot path) are not part of this package.
"""

from __future__ import annotations

from dataclasses import asdict, dataclass, field
from typing import Any, Callable, Literal

import numpy as np
import torch
import torch.nn as nn
from torch import Tensor

TaskType = Literal["binary", "multiclass", "multilabel", "ordinal", "regression"]


@dataclass(frozen=True)
class TaskConfig:
    name: str
    num_classes: int
    task_type: TaskType
    display_name: str = ""
    class_names: tuple[str, ...] = ()
    color: str = "#1f77b4"
    label_smoothing: float = 0.0
    use_focal_loss: bool = False
    focal_gamma: float = 2.0
    focal_alpha: float | None = None
    loss_weight: float = 1.0
    custom_loss_fn: Callable[[], nn.Module] | None = field(default=None, repr=False)
    custom_metrics_fn: Callable[[], Any] | None = field(default=None, repr=False)

    def __post_init__(self) -> None:
        if not self.display_name:
            object.__setattr__(self, "display_name", self.name.replace("_", " ").title())
        if not self.class_names and self.task_type == "multiclass":
            object.__setattr__(self, "class_names", tuple(f"Class {i}" for i in range(self.num_classes)))

    def with_overrides(self, **kwargs: Any) -> "TaskConfig":
        d = asdict(self)
        d.update(kwargs)
        return TaskConfig(**d)

    @property
    def is_binary(self) -> bool:
        return self.task_type == "binary"

    @property
    def is_multiclass(self) -> bool:
        return self.task_type == "multiclass"


class TaskStrategy:
    def get_loss_fn(self, task: TaskConfig) -> nn.Module:
        raise NotImplementedError

    def compute_predictions(self, logits: Tensor) -> Tensor:
        raise NotImplementedError

    def compute_probabilities(self, logits: Tensor) -> Tensor:
        raise NotImplementedError

    def format_target(self, target: Tensor) -> Tensor:
        raise NotImplementedError


class _SigmoidFamily(TaskStrategy):
    def get_loss_fn(self, task: TaskConfig) -> nn.Module:
        if task.custom_loss_fn is not None:
            return task.custom_loss_fn()
        if task.use_focal_loss:
            from ..training.losses import FocalLoss

            return FocalLoss(gamma=task.focal_gamma, alpha=task.focal_alpha)
        return nn.BCEWithLogitsLoss()

    def compute_probabilities(self, logits: Tensor) -> Tensor:
        return torch.sigmoid(logits)


class BinaryStrategy(_SigmoidFamily):
    def compute_predictions(self, logits: Tensor) -> Tensor:
        p = (torch.sigmoid(logits) > 0.5).int()
        return p.squeeze(-1) if p.shape[-1] == 1 else p

    def format_target(self, target: Tensor) -> Tensor:
        target = target.float() if target.dtype != torch.float32 else target
        return target.unsqueeze(-1) if target.dim() == 1 else target


class MultilabelStrategy(_SigmoidFamily):
    def compute_predictions(self, logits: Tensor) -> Tensor:
        return (torch.sigmoid(logits) > 0.5).int()

    def format_target(self, target: Tensor) -> Tensor:
        return target.float() if target.dtype != torch.float32 else target


class MulticlassStrategy(TaskStrategy):
    def get_loss_fn(self, task: TaskConfig) -> nn.Module:
        if task.custom_loss_fn is not None:
            return task.custom_loss_fn()
        return nn.CrossEntropyLoss(label_smoothing=task.label_smoothing)

    def compute_predictions(self, logits: Tensor) -> Tensor:
        return torch.argmax(logits, dim=1)

    def compute_probabilities(self, logits: Tensor) -> Tensor:
        return torch.softmax(logits, dim=1)

    def format_target(self, target: Tensor) -> Tensor:
        return target.long() if target.dtype != torch.int64 else target


class OrdinalStrategy(MulticlassStrategy):
    """Ordinal tasks are trained as multiclass (as in the reference)."""


class RegressionStrategy(TaskStrategy):
    def get_loss_fn(self, task: TaskConfig) -> nn.Module:
        return task.custom_loss_fn() if task.custom_loss_fn is not None else nn.MSELoss()

    def compute_predictions(self, logits: Tensor) -> Tensor:
        return logits

    def compute_probabilities(self, logits: Tensor) -> Tensor:
        return logits

    def format_target(self, target: Tensor) -> Tensor:
        return target.float() if target.dtype != torch.float32 else target


_STRATEGIES: dict[str, TaskStrategy] = {
    "binary": BinaryStrategy(),
    "multiclass": MulticlassStrategy(),
    "multilabel": MultilabelStrategy(),
    "ordinal": OrdinalStrategy(),
    "regression": RegressionStrategy(),
}


def get_strategy(task: TaskConfig | str) -> TaskStrategy:
    t = task.task_type if isinstance(task, TaskConfig) else task
    if t not in _STRATEGIES:
        raise ValueError(f"Unknown task type: {t}")
    return _STRATEGIES[t]


def _binary(name: str, display: str, color: str) -> TaskConfig:
    return TaskConfig(name=name, num_classes=1, task_type="binary", display_name=display, color=color)


TASK_REGISTRY: dict[str, TaskConfig] = {
    "pfirrmann": TaskConfig("pfirrmann", 5, "multiclass", "Pfirrmann Grade",
                            ("Grade I", "Grade II", "Grade III", "Grade IV", "Grade V"), "#1f77b4"),
    "modic": TaskConfig("modic", 4, "multiclass", "Modic Type", ("Normal", "Type I", "Type II", "Type III"),
                        "#ff7f0e"),
    "herniation": _binary("herniation", "Disc Herniation", "#2ca02c"),
    "bulging": _binary("bulging", "Disc Bulging", "#d62728"),
    "upper_endplate": _binary("upper_endplate", "Upper Endplate Defect", "#9467bd"),
    "lower_endplate": _binary("lower_endplate", "Lower Endplate Defect", "#8c564b"),
    "spondy": _binary("spondy", "Spondylolisthesis", "#e377c2"),
    "narrowing": _binary("narrowing", "Disc Narrowing", "#7f7f7f"),
}
AVAILABLE_TASK_NAMES: tuple[str, ...] = tuple(TASK_REGISTRY)


def get_task(name: str) -> TaskConfig:
    if name not in TASK_REGISTRY:
        raise KeyError(f"Unknown task: {name}. Available: {list(TASK_REGISTRY)}")
    return TASK_REGISTRY[name]


def get_tasks(names: list[str] | None = None) -> list[TaskConfig]:
    return list(TASK_REGISTRY.values()) if names is None else [get_task(n) for n in names]


def register_task(task: TaskConfig) -> None:
    if task.name in TASK_REGISTRY:
        raise ValueError(f"Task '{task.name}' already registered")
    TASK_REGISTRY[task.name] = task


def create_loss_functions(tasks: list[TaskConfig]) -> tuple[nn.ModuleDict, dict[str, float]]:
    fns = nn.ModuleDict({t.name: get_strategy(t).get_loss_fn(t) for t in tasks})
    return fns, {t.name: t.loss_weight for t in tasks}


def compute_predictions_for_tasks(outputs: dict[str, Tensor], tasks: list[TaskConfig]) -> dict[str, np.ndarray]:
    return {t.name: get_strategy(t).compute_predictions(outputs[t.name]).cpu().numpy()
            for t in tasks if t.name in outputs}


def compute_probabilities_for_tasks(outputs: dict[str, Tensor], tasks: list[TaskConfig]) -> dict[str, np.ndarray]:
    return {t.name: get_strategy(t).compute_probabilities(outputs[t.name]).cpu().numpy()
            for t in tasks if t.name in outputs}
