"""Localization batches (reference: spine_vision/training/datasets/localization.py:41-337)."""

from __future__ import annotations

import csv
from collections import Counter, defaultdict
from pathlib import Path
from typing import Any, Literal

import numpy as np
import torch
from torch.utils.data import Dataset

from .resize import collate_images

LEVELS = ("L1/L2", "L2/L3", "L3/L4", "L4/L5", "L5/S1")
NUM_LEVELS = len(LEVELS)
IDX_TO_LEVEL = dict(enumerate(LEVELS))
LEVEL_TO_IDX = {v: k for k, v in IDX_TO_LEVEL.items()}
SERIES_TYPE_TO_IDX = {"sag_t1": 0, "sag_t2": 1, "ct": 2}
_MEAN = torch.tensor([0.485, 0.456, 0.406]).view(3, 1, 1)
_STD = torch.tensor([0.229, 0.224, 0.225]).view(3, 1, 1)


def normalize_u8(img_u8: torch.Tensor) -> torch.Tensor:
    """uint8 [H,W] or [3,H,W] -> ToTensor (/255) -> ImageNet Normalize, f32 [3,H,W]."""
    x = img_u8.float() / 255.0
    if x.dim() == 2:
        x = x.unsqueeze(0).expand(3, -1, -1)
    return (x - _MEAN) / _STD


class LocalizationDataset(Dataset):
    """annotations.csv (image_path, level, relative_x, relative_y, series_type, source) + images.
    Per sample: image [3,H,W] (convert("RGB") -> Resize -> [HFlip, RandomAffine, ColorJitter when
    augmenting] -> ToTensor -> Normalize), coords [5,2], mask [5], series_type_idx, metadata -- the
    reference's record layout, transform chain (localization.py:196-233, 254) and image split.

    ``device_transform``: yield the decoded uint8 plane [h,w] at its native size (and, when augmenting, the
    sample's augmentation parameters under "augment", drawn like torchvision); the trainer runs the Resize
    (``kernels.resize_u8``), the flip / affine / jitter (``kernels.augment_u8``) and ToTensor -> Normalize
    on the GPU.  MRI PNGs are
    grayscale; an image whose RGB channels differ raises in this mode (use the host transform).
    ``augment_coords``: move the keypoints with the flip / affine (the reference does not)."""

    def __init__(self, data_path: Path, split: Literal["train", "val", "test", "all"] = "all", val_ratio: float = 0.15,
                 test_ratio: float = 0.05, series_types: list[str] | None = None, sources: list[str] | None = None,
                 image_size: tuple[int, int] = (256, 256), augment: bool = True, normalize: bool = True,
                 seed: int = 42, device_transform: bool = False, augment_coords: bool = False) -> None:
        self.data_path = Path(data_path)
        self.device_transform = device_transform
        self.augment_coords = augment_coords
        self.split = split
        self.image_size = tuple(image_size)
        self.augment = augment and split == "train"
        self.normalize = normalize
        ann = self.data_path / "annotations.csv"
        if not ann.exists():
            raise FileNotFoundError(f"Annotations not found: {ann}")
        with open(ann, newline="") as f:
            recs = list(csv.DictReader(f))
        if series_types:
            recs = [r for r in recs if r["series_type"] in series_types]
        if sources:
            recs = [r for r in recs if r["source"] in sources]
        self.image_records: dict[str, dict[str, Any]] = {}
        for r in recs:
            d = self.image_records.setdefault(r["image_path"], {"coords": {}, "series_type": r["series_type"],
                                                                "source": r["source"]})
            lvl = LEVEL_TO_IDX.get(r["level"], None)
            if lvl is None:
                lvl = int(r["level"])
            d["coords"][lvl] = (float(r["relative_x"]), float(r["relative_y"]))
        images = list(self.image_records)
        perm = np.random.RandomState(seed).permutation(len(images))
        n_test, n_val = int(len(images) * test_ratio), int(len(images) * val_ratio)
        idx = {"test": perm[:n_test], "val": perm[n_test:n_test + n_val], "train": perm[n_test + n_val:]}
        keep = set(images[i] for i in idx[split]) if split != "all" else set(images)
        self.image_list = [im for im in images if im in keep]

    def __len__(self) -> int:
        return len(self.image_list)

    def _load(self, rel: str, resize: bool = True):
        """convert("RGB") -> Resize (torchvision Resize on PIL = Image.resize((w, h), BILINEAR)); the
        device_transform path leaves the resize to the GPU (kernels.resize_u8, bit-identical)."""
        from PIL import Image

        im = Image.open(self.data_path / rel).convert("RGB")
        if not resize:
            return im
        return im.resize((self.image_size[1], self.image_size[0]), Image.BILINEAR)

    def __getitem__(self, i: int) -> dict[str, Any]:
        from .augment import apply_pil, sample_params, transform_coords

        rel = self.image_list[i]
        rec = self.image_records[rel]
        im = self._load(rel, resize=not self.device_transform)
        params = sample_params(self.image_size[0], self.image_size[1], flip=True) if self.augment else None
        out: dict[str, Any] = {}
        if self.device_transform:  # decoded uint8 [h,w] at native size; resized, augmented, normalised on the GPU
            rgb = np.asarray(im, dtype=np.uint8)
            if not (np.array_equal(rgb[..., 0], rgb[..., 1]) and np.array_equal(rgb[..., 0], rgb[..., 2])):
                raise ValueError(f"{rel}: device_transform expects grayscale images (RGB channels differ)")
            image = torch.from_numpy(rgb[..., 0].copy())
            out["resize_to"] = self.image_size
            if params is not None:
                out["augment"] = params
        else:
            if params is not None:
                im = apply_pil(im, params)
            x = torch.from_numpy(np.asarray(im, dtype=np.uint8).copy()).permute(2, 0, 1)
            image = normalize_u8(x) if self.normalize else x.float().div(255)
        coords = torch.zeros(NUM_LEVELS, 2)
        mask = torch.zeros(NUM_LEVELS)
        for lvl, (x_, y_) in rec["coords"].items():
            coords[lvl, 0], coords[lvl, 1], mask[lvl] = x_, y_, 1.0
        if params is not None and self.augment_coords:
            coords = transform_coords(coords, params, self.image_size[0], self.image_size[1]) * mask[:, None]
        out.update({"image": image, "coords": coords, "mask": mask,
                    "series_type_idx": SERIES_TYPE_TO_IDX.get(rec["series_type"], 0),
                    "metadata": {"image_path": rel, "source": rec["source"], "series_type": rec["series_type"]}})
        return out

    def get_stats(self) -> dict[str, Any]:
        lc: dict[int, int] = defaultdict(int)
        for rel in self.image_list:
            for lvl in self.image_records[rel]["coords"]:
                lc[lvl] += 1
        return {"num_images": len(self.image_list), "num_annotations": sum(lc.values()),
                "levels": {IDX_TO_LEVEL[k]: v for k, v in sorted(lc.items())},
                "series_types": dict(Counter(self.image_records[r]["series_type"] for r in self.image_list)),
                "sources": dict(Counter(self.image_records[r]["source"] for r in self.image_list)),
                "split": self.split}


class SyntheticLocalizationDataset(Dataset):
    """Seeded synthetic samples with the BASELINE input spec: uint8 grayscale U{0..255} -> RGB ->
    /255 -> ImageNet normalise; coords U(0.05, 0.95); ~10% of levels masked.  ``augment``: the
    reference's train augmentation, host (PIL) or device (``device_transform``) path as in
    LocalizationDataset."""

    def __init__(self, n: int, image_size: tuple[int, int] = (512, 512), seed: int = 42,
                 device_transform: bool = False, augment: bool = False) -> None:
        self.n, self.image_size, self.seed = n, tuple(image_size), seed
        self.device_transform = device_transform
        self.augment = augment

    def __len__(self) -> int:
        return self.n

    def __getitem__(self, i: int) -> dict[str, Any]:
        g = torch.Generator().manual_seed(self.seed * 1_000_003 + i)
        u8 = torch.randint(0, 256, self.image_size, generator=g, dtype=torch.uint8)
        coords = torch.rand(NUM_LEVELS, 2, generator=g) * 0.9 + 0.05
        mask = (torch.rand(NUM_LEVELS, generator=g) >= 0.1).float()
        out: dict[str, Any] = {}
        if self.augment:
            from .augment import apply_pil, sample_params

            params = sample_params(self.image_size[0], self.image_size[1], flip=True)
            if self.device_transform:
                out["augment"] = params
            else:
                from PIL import Image

                u8 = torch.from_numpy(np.asarray(apply_pil(Image.fromarray(u8.numpy(), "L"), params)).copy())
        out.update({"image": u8 if self.device_transform else normalize_u8(u8), "coords": coords, "mask": mask,
                    "series_type_idx": 1,
                    "metadata": {"image_path": f"synthetic_{i}.png", "source": "synthetic", "series_type": "sag_t2"}})
        return out

    def get_stats(self) -> dict[str, Any]:
        return {"num_images": self.n, "source": "synthetic"}


class LocalizationCollator:
    """training/datasets/localization.py:315-337 of the reference (+ "augment" [B,10] when present)."""

    def __call__(self, samples: list[dict[str, Any]]) -> dict[str, Any]:
        out = {
            **collate_images(samples),  # stacked, or a ragged batch for the device resize
            "coords": torch.stack([s["coords"] for s in samples]),
            "mask": torch.stack([s["mask"] for s in samples]),
            "series_type_idx": torch.tensor([s["series_type_idx"] for s in samples], dtype=torch.long),
            "metadata": [s["metadata"] for s in samples],
        }
        if "augment" in samples[0]:  # device_transform: per-sample augmentation parameters [B,10]
            out["augment"] = torch.stack([s["augment"] for s in samples])
        return out
