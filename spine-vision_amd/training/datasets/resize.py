"""Resize on the device (row f1): the host half of ``kernels.resize_u8``.

The reference resizes every decoded image with torchvision ``Resize(size)`` on a PIL image
(spine_vision/training/datasets/localization.py:199, classification.py:250), i.e. PIL
``Image.resize((W, H), Image.BILINEAR)`` -- Pillow's libImaging/Resample.c.  Its per-axis filter tables
are computed in double precision and rounded to int32 fixed point; this module restates that
computation (``pil_bilinear_coeffs``) operation for operation, so the device kernel, which applies the
tables with Pillow's integer arithmetic, is bit-identical to PIL.  Tables are cached per (in, out) size.

``ragged_batch`` packs decoded images of any sizes into one flat uint8 buffer plus the descriptor /
table buffers sv_resize_u8 reads; the collators call it in the loader workers, the trainer hands the
three tensors to the device.
"""

from __future__ import annotations

import math
from functools import lru_cache

import numpy as np
import torch

PRECISION_BITS = 22  # Resample.c: 32 - 8 - 2


@lru_cache(maxsize=256)
def pil_bilinear_coeffs(in_size: int, out_size: int) -> tuple[np.ndarray, np.ndarray]:
    """(bounds int32 [out, 2] = {first tap, count}, coef int32 [out, taps]) of Pillow's precompute_coeffs
    (BILINEAR: triangle filter, support 1) followed by normalize_coeffs_8bpc, for the box [0, in_size)."""
    if in_size <= 0 or out_size <= 0:
        raise ValueError("resize: sizes must be positive")
    scale = float(in_size) / out_size  # (in1 - in0) / outSize
    filterscale = scale if scale >= 1.0 else 1.0
    support = 1.0 * filterscale
    ksize = int(math.ceil(support)) * 2 + 1
    ss = 1.0 / filterscale
    xx = np.arange(out_size, dtype=np.float64)
    center = 0.0 + (xx + 0.5) * scale
    xmin = np.trunc(center - support + 0.5).astype(np.int64)  # C (int) truncates toward zero
    xmin = np.maximum(xmin, 0)
    xmax = np.trunc(center + support + 0.5).astype(np.int64)
    xmax = np.minimum(xmax, in_size)
    count = xmax - xmin
    taps = np.arange(ksize, dtype=np.int64)
    arg = ((taps[None, :] + xmin[:, None]).astype(np.float64) - center[:, None] + 0.5) * ss
    a = np.abs(arg)
    w = np.where(a < 1.0, 1.0 - a, 0.0)
    valid = taps[None, :] < count[:, None]
    w = np.where(valid, w, 0.0)
    ww = np.zeros(out_size, dtype=np.float64)
    for t in range(ksize):  # sequential sum, as the C loop (adding 0.0 for absent taps is exact)
        ww = ww + w[:, t]
    safe = np.where(ww != 0.0, ww, 1.0)
    k = np.where((ww != 0.0)[:, None] & valid, w / safe[:, None], np.where(valid, w, 0.0))
    fx = k * float(1 << PRECISION_BITS)
    coef = np.where(k < 0, np.trunc(-0.5 + fx), np.trunc(0.5 + fx)).astype(np.int32)
    bounds = np.stack([xmin, count], axis=1).astype(np.int32)
    return bounds, coef


def output_size(size, h: int, w: int) -> tuple[int, int]:
    """(H, W) torchvision Resize(size) gives for an h x w image: a pair is (H, W); an int resizes the
    shorter side to it and keeps the aspect ratio (int(size * long / short), no max_size)."""
    if isinstance(size, (tuple, list)) and len(size) == 2:
        return int(size[0]), int(size[1])
    s = int(size[0] if isinstance(size, (tuple, list)) else size)
    short, long_ = (w, h) if w <= h else (h, w)
    new_short, new_long = s, int(s * long_ / short)
    return (new_long, new_short) if w <= h else (new_short, new_long)


def ragged_batch(images: list, out_hw: tuple[int, int]) -> dict[str, torch.Tensor]:
    """Pack decoded uint8 images ([h, w] or [h, w, 3], any sizes, one channel count) for sv_resize_u8:
    {"src": flat uint8, "desc": int64 [B, 8], "coef": int32 tables, "out_hw": int64 [2]}."""
    H, W = out_hw
    arrs = [np.ascontiguousarray(np.asarray(im, dtype=np.uint8)) for im in images]
    C = 1 if arrs[0].ndim == 2 else arrs[0].shape[2]
    if any((a.ndim == 2) != (C == 1) or (a.ndim == 3 and a.shape[2] != C) for a in arrs):
        raise ValueError("ragged_batch: every image needs the same channel count (1 or 3)")
    tables: dict[tuple[int, int], int] = {}
    chunks: list[np.ndarray] = []
    used = 0

    def table(n_in: int, n_out: int) -> tuple[int, int]:
        nonlocal used
        key = (n_in, n_out)
        bounds, coef = pil_bilinear_coeffs(n_in, n_out)
        if key not in tables:
            tables[key] = used
            flat = np.concatenate([bounds.reshape(-1), coef.reshape(-1)])
            chunks.append(flat)
            used += flat.size
        return tables[key], coef.shape[1]

    desc = np.zeros((len(arrs), 8), dtype=np.int64)
    off = 0
    for b, a in enumerate(arrs):
        h, w = a.shape[:2]
        xo, kx = table(w, W)
        yo, ky = table(h, H)
        desc[b] = (off, h, w, xo, kx, yo, ky, 0)
        off += a.size
    src = np.concatenate([a.reshape(-1) for a in arrs]) if arrs else np.zeros(0, np.uint8)
    return {"src": torch.from_numpy(src), "desc": torch.from_numpy(desc),
            "coef": torch.from_numpy(np.concatenate(chunks).astype(np.int32)),
            "out_hw": torch.tensor([H, W, C], dtype=torch.int64)}


def collate_images(samples: list[dict]) -> dict:
    """The image part of a batch: stacked when every image already has its target size (or none is
    set), else a ragged batch for the device resize ({"image": None, "resize": ragged_batch(...)}).
    A device_transform dataset yields its decoded uint8 image at native size with "resize_to" = (H, W)."""
    imgs = [s["image"] for s in samples]
    target = samples[0].get("resize_to")
    if target is None or all(tuple(im.shape[:2]) == tuple(target) for im in imgs):
        return {"image": torch.stack([torch.as_tensor(im) for im in imgs])}
    return {"image": None, "resize": ragged_batch([np.asarray(im) for im in imgs], tuple(target))}
