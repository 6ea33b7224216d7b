"""Classification data (reference: spine_vision/training/datasets/classification.py:40-493,
sampling.py:16-84): the crop dataset over the dataset CLI's annotations.csv, its transforms, the
batch contract and the weighted sampler."""

from __future__ import annotations

import csv
from collections import Counter
from pathlib import Path
from typing import Any, Literal

import numpy as np
import torch
from torch.utils.data import Dataset, WeightedRandomSampler

from ...core.tasks import AVAILABLE_TASK_NAMES, get_task
from .localization import IDX_TO_LEVEL, normalize_u8
from .resize import collate_images
from .stratification import split_patients


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
        out = {**collate_images(samples), "targets": DynamicTargets(tg),
               "level_idx": torch.tensor([s.get("level_idx", 0) for s in samples], dtype=torch.long),
               "metadata": [s.get("metadata", {}) for s in samples]}
        if "augment" in samples[0]:  # device_transform: per-sample augmentation parameters [B,10]
            out["augment"] = torch.stack([s["augment"] for s in samples])
        return out


class ClassificationDataset(Dataset):
    """Pre-extracted IVD crops (``spine-vision dataset classification`` output: images/ + annotations.csv
    with image_path, patient_id, ivd_level, series_type, source and the label columns), T1/T2 crops of
    one (source, patient, level) paired into one record, filtered by series types and levels, split by
    patient (``split_patients``, patient-stratified as the reference), transformed Resize ->
    [RandomAffine -> ColorJitter when augmenting] -> ToTensor -> Normalize on the [T2,T1,T2] image
    (reference training/datasets/classification.py:71-413).

    ``device_transform``: yield the resized uint8 [H,W,3] crop (and the augmentation parameters under
    "augment"); the ResNet stem gather normalises it on the GPU and ``kernels.augment_u8`` augments it."""

    _LABEL_COLS = {"pfirrmann": "pfirrmann_grade", "modic": "modic", "herniation": "disc_herniation",
                   "bulging": "disc_bulging", "upper_endplate": "up_endplate", "lower_endplate": "low_endplate",
                   "spondylolisthesis": "spondylolisthesis", "narrowing": "disc_narrowing"}

    def __init__(self, data_path: Path, split: Literal["train", "val", "test", "all"] = "all", val_ratio: float = 0.10,
                 test_ratio: float = 0.10, levels: list[str] | None = None, series_types: list[str] | None = None,
                 target_labels: list[str] | None = None, output_size: tuple[int, int] = (256, 256),
                 augment: bool = True, normalize: bool = True, seed: int = 42, device_transform: bool = False) -> None:
        self.data_path = Path(data_path)
        self.split = split
        self.output_size = tuple(output_size)
        self.augment = augment and split == "train"
        self.normalize = normalize
        self.device_transform = device_transform
        valid_series = {"sag_t1", "sag_t2"}
        if series_types is not None:
            bad = set(series_types) - valid_series
            if bad:
                raise ValueError(f"Invalid series types: {bad}. Valid types: {valid_series}")
            self.series_types = set(series_types)
        else:
            self.series_types = valid_series
        if target_labels is not None:
            bad = set(target_labels) - set(AVAILABLE_TASK_NAMES)
            if bad:
                raise ValueError(f"Invalid target labels: {bad}. Available labels: {AVAILABLE_TASK_NAMES}")
            self.target_labels = list(target_labels)
        else:
            self.target_labels = list(AVAILABLE_TASK_NAMES)
        self.records = self._load_and_pair_annotations()
        if levels:
            keep = set(levels)
            self.records = [r for r in self.records if IDX_TO_LEVEL.get(r["level_idx"]) in keep]
        train_p, val_p, test_p = split_patients(self._get_unique_patients(), self.records, self.target_labels,
                                                val_ratio, test_ratio, seed)
        chosen = {"train": train_p, "val": val_p, "test": test_p}.get(split)
        if chosen is not None:
            self.records = [r for r in self.records if r["patient_key"] in chosen]

    def _load_and_pair_annotations(self) -> list[dict[str, Any]]:
        csv_path = self.data_path / "annotations.csv"
        if not csv_path.exists():
            raise FileNotFoundError(f"Annotations not found: {csv_path}")
        groups: dict[tuple[str, str, int], dict[str, Any]] = {}
        with open(csv_path, newline="") as f:
            for row in csv.DictReader(f):
                key = (row["source"], row["patient_id"], int(row["ivd_level"]))
                g = groups.get(key)
                if g is None:
                    g = groups[key] = {
                        "source": row["source"], "patient_id": row["patient_id"],
                        "patient_key": f"{row['source']}_{row['patient_id']}", "ivd_level": key[2],
                        "level_idx": key[2] - 1, "t1_path": None, "t2_path": None,
                        **{k: int(row[c]) for k, c in self._LABEL_COLS.items()},
                    }
                if row["series_type"] == "sag_t1":
                    g["t1_path"] = self.data_path / row["image_path"]
                elif row["series_type"] == "sag_t2":
                    g["t2_path"] = self.data_path / row["image_path"]
        need_t1, need_t2 = "sag_t1" in self.series_types, "sag_t2" in self.series_types
        out = []
        for g in groups.values():
            has1, has2 = g["t1_path"] is not None, g["t2_path"] is not None
            if (need_t1 and need_t2 and has1 and has2) or (need_t1 and not need_t2 and has1) or \
                    (need_t2 and not need_t1 and has2):
                out.append(g)
        return out

    def _get_unique_patients(self) -> list[str]:
        return list(set(r["patient_key"] for r in self.records))

    def __len__(self) -> int:
        return len(self.records)

    def __getitem__(self, idx: int) -> dict[str, Any]:
        from PIL import Image

        from .augment import apply_pil, sample_params

        r = self.records[idx]
        t1 = np.array(Image.open(r["t1_path"]).convert("L")) if r["t1_path"] is not None else None
        t2 = np.array(Image.open(r["t2_path"]).convert("L")) if r["t2_path"] is not None else None
        rgb = construct_3channel(None if t2 is None else torch.from_numpy(t2),
                                 None if t1 is None else torch.from_numpy(t1)).numpy()
        params = sample_params(self.output_size[0], self.output_size[1], flip=False) if self.augment else None
        out: dict[str, Any] = {}
        if self.device_transform:  # [h,w,3] at native size: Resize on the GPU (kernels.resize_u8)
            image = torch.from_numpy(np.ascontiguousarray(rgb))
            out["resize_to"] = tuple(self.output_size)
            if params is not None:
                out["augment"] = params
        else:
            im = Image.fromarray(rgb).resize((self.output_size[1], self.output_size[0]), Image.BILINEAR)
            if params is not None:
                im = apply_pil(im, params)
            x = torch.from_numpy(np.asarray(im, dtype=np.uint8).copy()).permute(2, 0, 1)
            image = normalize_u8(x) if self.normalize else x.float().div(255)
        values = {"pfirrmann": r["pfirrmann"] - 1, "modic": r["modic"], "herniation": [float(r["herniation"])],
                  "bulging": [float(r["bulging"])], "upper_endplate": [float(r["upper_endplate"])],
                  "lower_endplate": [float(r["lower_endplate"])], "spondy": [float(r["spondylolisthesis"])],
                  "narrowing": [float(r["narrowing"])]}
        out.update({"image": image, "targets": {k: v for k, v in values.items() if k in self.target_labels},
                    "level_idx": r["level_idx"],
                    "metadata": {"source": r["source"], "patient_id": r["patient_id"],
                                 "level": IDX_TO_LEVEL.get(r["level_idx"], ""), "ivd": r["ivd_level"]}})
        return out

    def get_stats(self) -> dict[str, Any]:
        return {"num_samples": len(self.records), "num_patients": len(self._get_unique_patients()),
                "levels": dict(Counter(IDX_TO_LEVEL.get(r["level_idx"], "") for r in self.records)),
                "pfirrmann": dict(Counter(r["pfirrmann"] for r in self.records)),
                "modic": dict(Counter(r["modic"] for r in self.records)),
                "sources": dict(Counter(r["source"] for r in self.records)),
                "series_types": list(self.series_types), "target_labels": self.target_labels, "split": self.split}

    def get_label_distribution(self) -> dict[str, dict]:
        key = {"spondy": "spondylolisthesis"}
        return {lab: dict(Counter(r[key.get(lab, lab)] for r in self.records)) for lab in self.target_labels}

    def compute_class_weights(self) -> dict[str, torch.Tensor]:
        n = len(self.records)
        w: dict[str, torch.Tensor] = {}
        if "pfirrmann" in self.target_labels:
            cnt = Counter(r["pfirrmann"] - 1 for r in self.records)
            w["pfirrmann"] = torch.tensor([n / (5 * cnt.get(i, 1)) for i in range(5)], dtype=torch.float32)
        if "modic" in self.target_labels:
            cnt = Counter(r["modic"] for r in self.records)
            w["modic"] = torch.tensor([n / (4 * cnt.get(i, 1)) for i in range(4)], dtype=torch.float32)
        for lab, key in {"herniation": "herniation", "bulging": "bulging", "upper_endplate": "upper_endplate",
                         "lower_endplate": "lower_endplate", "spondy": "spondylolisthesis",
                         "narrowing": "narrowing"}.items():
            if lab in self.target_labels:
                pos = sum(r[key] for r in self.records)
                w[lab] = torch.tensor([(n - pos) / max(pos, 1)])
        return w


class SyntheticClassificationDataset(Dataset):
    """Seeded synthetic IVD crops: channels [T2, T1, T2] from two uint8 planes -> /255 -> ImageNet
    normalise; labels pfirrmann U{0..4}, modic U{0..3}, herniation Bernoulli(0.3).  ``records``
    mirrors the reference's record dicts so create_weighted_sampler works unchanged.
    ``device_transform``: yield the uint8 [H,W,3] crop of construct_3channel instead (the ResNet
    backbone normalises it on the GPU, row f1)."""

    def __init__(self, n: int, output_size: tuple[int, int] = (256, 256), seed: int = 42,
                 target_labels: list[str] | None = None, device_transform: bool = False, augment: bool = False) -> None:
        self.n, self.output_size, self.seed = n, tuple(output_size), seed
        self.device_transform = device_transform
        self.augment = augment
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
        img = construct_3channel(t2, t1)
        extra: dict[str, Any] = {}
        if self.augment:  # the reference's RandomAffine -> ColorJitter (host PIL, or parameters for the GPU)
            from .augment import apply_pil, sample_params

            params = sample_params(self.output_size[0], self.output_size[1], flip=False)
            if self.device_transform:
                extra["augment"] = params
            else:
                from PIL import Image

                img = torch.from_numpy(np.asarray(apply_pil(Image.fromarray(img.numpy()), params)).copy())
        if not self.device_transform:
            img = normalize_u8(img.permute(2, 0, 1))
        r = self.records[i]
        values = {"pfirrmann": r["pfirrmann"] - 1, "modic": r["modic"], "herniation": float(r["herniation"])}
        return {**extra, "image": img, "targets": {k: values[k] for k in self.target_labels}, "level_idx": i % 5,
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
