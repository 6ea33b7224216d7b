"""CPU: the host half of the device resize (row f1) against PIL itself.

The reference's first transform is torchvision Resize on a PIL image = ``Image.resize((W, H), BILINEAR)``
(spine_vision/training/datasets/localization.py:199, classification.py:250).  ``pil_bilinear_coeffs``
restates Pillow's filter tables (libImaging/Resample.c precompute_coeffs + normalize_coeffs_8bpc); applied
here with the integer arithmetic sv_resize_u8 uses (one output pixel at a time, the horizontal result of
each vertical tap rounded to uint8 first), the result must equal PIL's bit for bit -- shrinking (antialias
support), enlarging, odd ratios, 1-pixel edges, grayscale and RGB, noise and smooth content."""

import numpy as np
import pytest
import torch
from PIL import Image

from spine_vision_amd.training.datasets.resize import output_size, pil_bilinear_coeffs, ragged_batch


def fused_resize(img: np.ndarray, H: int, W: int) -> np.ndarray:
    """The kernel's arithmetic in numpy (test restatement of csrc/resize.hip)."""
    h, w = img.shape[:2]
    x3 = img.reshape(h, w, -1).astype(np.int64)
    bx, kx = pil_bilinear_coeffs(w, W)
    by, ky = pil_bilinear_coeffs(h, H)
    out = np.empty((H, W, x3.shape[2]), np.uint8)
    for y in range(H):
        sv = np.full((W, x3.shape[2]), 1 << 21, np.int64)
        for j in range(by[y, 1]):
            row = x3[by[y, 0] + j]
            sh = np.full((W, x3.shape[2]), 1 << 21, np.int64)
            for i in range(kx.shape[1]):
                cols = np.minimum(bx[:, 0] + i, w - 1)
                live = (i < bx[:, 1])[:, None]
                sh += np.where(live, row[cols] * kx[:, i][:, None], 0)
            sv += np.clip(sh >> 22, 0, 255) * ky[y, j]
        out[y] = np.clip(sv >> 22, 0, 255)
    return out.reshape((H, W) + img.shape[2:])


CASES = [(512, 512, 512, 512), (600, 700, 512, 512), (1024, 1024, 512, 512), (300, 257, 512, 512),
         (97, 1001, 256, 256), (512, 512, 256, 256), (1, 5, 3, 7), (7, 3, 1, 1), (640, 480, 512, 384),
         (2000, 1500, 256, 256), (333, 333, 128, 96)]


@pytest.mark.parametrize("h,w,H,W", CASES)
@pytest.mark.parametrize("mode", ["L", "RGB"])
@pytest.mark.parametrize("content", ["noise", "smooth"])
def test_resize_tables_match_pil(h, w, H, W, mode, content):
    rng = np.random.default_rng(h * 7 + w)
    shape = (h, w) if mode == "L" else (h, w, 3)
    if content == "noise":
        img = rng.integers(0, 256, shape, dtype=np.uint8)
    else:  # gradients hit the rounding boundaries of the fixed-point sums
        yy, xx = np.meshgrid(np.linspace(0, 1, h), np.linspace(0, 1, w), indexing="ij")
        base = (255 * (0.5 + 0.5 * np.sin(6 * xx + 3 * yy))).astype(np.uint8)
        img = base if mode == "L" else np.stack([base, 255 - base, base // 2], axis=-1)
    ref = np.asarray(Image.fromarray(img, mode).resize((W, H), Image.BILINEAR))
    assert np.array_equal(fused_resize(img, H, W), ref)


def test_output_size_like_torchvision():
    assert output_size((512, 384), 100, 200) == (512, 384)
    assert output_size(256, 600, 400) == (384, 256)  # shorter side (w) -> 256, aspect kept
    assert output_size(256, 400, 600) == (256, 384)
    assert output_size([300], 300, 300) == (300, 300)


def test_ragged_batch_layout():
    imgs = [np.zeros((5, 7), np.uint8), np.ones((9, 4), np.uint8), np.full((5, 7), 3, np.uint8)]
    rb = ragged_batch(imgs, (6, 6))
    d = rb["desc"].numpy()
    assert d[:, 0].tolist() == [0, 35, 71] and d[:, 1].tolist() == [5, 9, 5] and d[:, 2].tolist() == [7, 4, 7]
    assert rb["src"].numel() == 35 + 36 + 35 and rb["out_hw"].tolist() == [6, 6, 1]
    assert d[0, 3] == d[2, 3] and d[0, 5] == d[2, 5]  # one table per (in, out) size
    coef = rb["coef"].numpy()
    b, k = pil_bilinear_coeffs(7, 6)
    o = d[0, 3]
    assert np.array_equal(coef[o:o + 12].reshape(6, 2), b) and np.array_equal(coef[o + 12:o + 12 + k.size].reshape(k.shape), k)
    assert rb["src"].dtype == torch.uint8 and rb["coef"].dtype == torch.int32
