"""Classification batches (reference: spine_vision/training/datasets/classification.py:416-493,
sampling.py:16-84)."""

from __future__ import annotations

from collections import Counter
from typing import Any

import torch
from torch.utils.data import Dataset, WeightedRandomSampler

from ...core.tasks import get_task
from .localization import normalize_u8


def construct_3channel(t2: torch.Tensor | None, t1: torch.Tensor | None) -> torch.Tensor:
    """uint8 [H,W] planes -> [H,W,3]: [T2,T1,T2] with both, else the one plane replicated
    (reference training/datasets/classification.py:40-68)."""
    if t2 is not None and t1 is not None:
        return torch.stack([t2, t1, t2], dim=-1)
    if t2 is not None:
        return torch.stack([t2, t2, t2], dim=-1)
    if t1 is not None:
        return torch.stack([t1, t1, t1], dim=-1)
    raise ValueError("At least one of t2_crop or t1_crop must be provided")


class DynamicTargets:
    """Per-task target tensors with .to(device) / .to_dict() / attribute access."""

    def __init__(self, data: dict[str, torch.Tensor]) -> None:
        self._data = data

    def to(self, device) -> "DynamicTargets":
        return DynamicTargets({k: v.to(device, non_blocking=True) for k, v in self._data.items()})

    def to_dict(self) -> dict[str, torch.Tensor]:
        return self._data

    def __getattr__(self, name: str):
        if name.startswith("_"):
            return object.__getattribute__(self, name)
        if name in self._data:
            return self._data[name]
        raise AttributeError(f"No target named '{name}'")

    def __contains__(self, name: str) -> bool:
        return name in self._data

    @property
    def labels(self) -> list[str]:
        return list(self._data)


class ClassificationCollator:
    def __call__(self, samples: list[dict[str, Any]]) -> dict[str, Any]:
        labels = list(samples[0]["targets"])
        tg = {}
        for lab in labels:
            dtype = torch.long if get_task(lab).is_multiclass else torch.float32
            tg[lab] = torch.tensor([s["targets"][lab] for s in samples], dtype=dtype)
        return {"image": torch.stack([s["image"] for s in samples]), "targets": DynamicTargets(tg),
                "level_idx": torch.tensor([s.get("level_idx", 0) for s in samples], dtype=torch.long),
                "metadata": [s.get("metadata", {}) for s in samples]}


class SyntheticClassificationDataset(Dataset):
    """Seeded synthetic IVD crops: channels [T2, T1, T2] from two uint8 planes -> /255 -> ImageNet
    normalise; labels pfirrmann U{0..4}, modic U{0..3}, herniation Bernoulli(0.3).  ``records``
    mirrors the reference's record dicts so create_weighted_sampler works unchanged.
    ``device_transform``: yield the uint8 [H,W,3] crop of construct_3channel instead (the ResNet
    backbone normalises it on the GPU, row f1)."""

    def __init__(self, n: int, output_size: tuple[int, int] = (256, 256), seed: int = 42,
                 target_labels: list[str] | None = None, device_transform: bool = False) -> None:
        self.n, self.output_size, self.seed = n, tuple(output_size), seed
        self.device_transform = device_transform
        self.target_labels = target_labels or ["pfirrmann", "modic", "herniation"]
        g = torch.Generator().manual_seed(seed)
        self.records = [
            {"pfirrmann": int(torch.randint(1, 6, (), generator=g)), "modic": int(torch.randint(0, 4, (), generator=g)),
             "herniation": int(torch.rand((), generator=g) < 0.3), "patient_id": i // 2}
            for i in range(n)
        ]

    def __len__(self) -> int:
        return self.n

    def __getitem__(self, i: int) -> dict[str, Any]:
        g = torch.Generator().manual_seed(self.seed * 1_000_003 + i)
        t2 = torch.randint(0, 256, self.output_size, generator=g, dtype=torch.uint8)
        t1 = torch.randint(0, 256, self.output_size, generator=g, dtype=torch.uint8)
        img = construct_3channel(t2, t1) if self.device_transform else normalize_u8(torch.stack([t2, t1, t2]))
        r = self.records[i]
        values = {"pfirrmann": r["pfirrmann"] - 1, "modic": r["modic"], "herniation": float(r["herniation"])}
        return {"image": img, "targets": {k: values[k] for k in self.target_labels}, "level_idx": i % 5,
                "metadata": {"patient_id": r["patient_id"]}}

    def get_stats(self) -> dict[str, Any]:
        return {"num_samples": self.n, "source": "synthetic"}

    def get_label_distribution(self) -> dict[str, dict[int, int]]:
        return {k: dict(Counter(r[k] for r in self.records)) for k in ("pfirrmann", "modic", "herniation")}


_RECORD_KEY = {"pfirrmann": "pfirrmann", "modic": "modic", "herniation": "herniation", "bulging": "bulging",
               "upper_endplate": "upper_endplate", "lower_endplate": "lower_endplate", "spondy": "spondylolisthesis",
               "narrowing": "narrowing"}


def create_weighted_sampler(dataset, target_label: str) -> WeightedRandomSampler:
    """Inverse-class-frequency sampling (1/N_c per sample), replacement=True (sampling.py:16-84)."""
    if target_label not in _RECORD_KEY:
        raise ValueError(f"Invalid target_label: {target_label}. Valid labels: {list(_RECORD_KEY)}")
    key = _RECORD_KEY[target_label]
    vals = [r[key] - 1 if target_label == "pfirrmann" else r[key] for r in dataset.records]
    counts = Counter(vals)
    return WeightedRandomSampler(weights=[1.0 / counts[v] for v in vals], num_samples=len(vals), replacement=True)
