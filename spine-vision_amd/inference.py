"""Localization inference consumer (row f2): the reference's
``spine_vision/datasets/classification/cropping.py:407-483`` (``load_localization_model``,
``predict_ivd_locations``) over the HIP ConvNeXt, plus a batched form for many slices.

The reference loads the checkpoint with ``torch.load(..., weights_only=False)``; here the safe loader
(``weights_only=True``) is used, which reads every checkpoint the trainers write (tensors, plain
dicts / lists / numbers / strings) and executes nothing from the file.  Preprocessing matches the
reference: min-max to uint8 (``spine_vision/io/__init__.py:15-30``), ``convert("RGB")``,
``transforms.Resize(image_size)`` on the PIL image (= ``Image.resize((w, h), BILINEAR)``), ToTensor,
ImageNet Normalize.  The batched form does the Normalize on the GPU (the stem's uint8 gather in bf16,
``sv_normalize_u8_gray`` in fp32), bitwise equal to the host transform for grayscale slices.
"""

from __future__ import annotations

from pathlib import Path

import numpy as np
import torch

from .training.datasets.localization import normalize_u8
from .training.models.generic import CoordinateRegressor

IMAGENET_MEAN = [0.485, 0.456, 0.406]  # cropping.py:23
IMAGENET_STD = [0.229, 0.224, 0.225]  # cropping.py:24


def normalize_to_uint8(arr: np.ndarray) -> np.ndarray:
    """Min-max normalisation to [0, 255] uint8 (reference ``spine_vision/io/__init__.py:15-30``):
    float32 arithmetic, truncating cast, a constant array left as is (then cast)."""
    a = arr.astype(np.float32)
    lo, hi = a.min(), a.max()
    if hi - lo > 0:
        a = (a - lo) / (hi - lo) * 255
    return a.astype(np.uint8)


def _backbone_name(variant: str) -> str:
    # cropping.py:424-428
    return f"convnext_{variant}" if not variant.startswith("v2_") else f"convnextv2_{variant[3:]}"


def load_localization_model(model_path: Path, variant: str, device: str, precision: str | None = None) -> torch.nn.Module:
    """CoordinateRegressor(convnext_<variant>, 5 levels) with the checkpoint's ``model_state_dict``, on
    ``device``, in eval mode (cropping.py:407-440).  ``precision``: the HIP backbone's compute mode
    (None = the default bf16; "fp32" = the parity mode)."""
    model = CoordinateRegressor(backbone=_backbone_name(variant), pretrained=False, num_levels=5, precision=precision)
    ck = torch.load(Path(model_path), map_location="cpu", weights_only=True)
    model.load_state_dict(ck["model_state_dict"])
    model.to(device)
    model.eval()
    return model


def _resized_rgb_u8(image: np.ndarray, image_size: tuple[int, int]) -> np.ndarray:
    from PIL import Image

    pil = Image.fromarray(normalize_to_uint8(image)).convert("RGB")
    pil = pil.resize((int(image_size[1]), int(image_size[0])), Image.BILINEAR)
    return np.array(pil, dtype=np.uint8)  # writable copy (torch.from_numpy)


def predict_ivd_locations(model: torch.nn.Module, image: np.ndarray, device: str,
                          image_size: tuple[int, int]) -> dict[int, tuple[float, float]]:
    """Relative (x, y) of the 5 IVD levels of one 2-D slice (cropping.py:443-483)."""
    rgb = _resized_rgb_u8(image, image_size)
    tensor = normalize_u8(torch.from_numpy(rgb).permute(2, 0, 1)).unsqueeze(0).to(device)
    with torch.no_grad():
        out = model(tensor).float().cpu().numpy()[0]  # [num_levels, 2]
    return {i: (float(out[i, 0]), float(out[i, 1])) for i in range(out.shape[0])}


def predict_ivd_locations_batch(model: torch.nn.Module, images: list[np.ndarray], device: str,
                                image_size: tuple[int, int], batch_size: int = 32) -> list[dict[int, tuple[float, float]]]:
    """``predict_ivd_locations`` for many slices, ``batch_size`` at a time: the host only resizes to
    uint8 and the ToTensor / Normalize runs on the GPU (the model's uint8 input path), so a batch crosses
    PCIe at 1 B per pixel.  Same predictions as the per-slice call (grayscale slices)."""
    preds: list[dict[int, tuple[float, float]]] = []
    for s in range(0, len(images), batch_size):
        planes = [_resized_rgb_u8(im, image_size)[..., 0] for im in images[s:s + batch_size]]
        u8 = torch.from_numpy(np.stack(planes)).to(device)
        with torch.no_grad():
            out = model(u8).float().cpu().numpy()
        preds += [{i: (float(o[i, 0]), float(o[i, 1])) for i in range(o.shape[0])} for o in out]
    return preds
