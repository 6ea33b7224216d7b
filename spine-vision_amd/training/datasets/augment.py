"""Train-time augmentation of the reference transform chains (row f1).

Reference (applied after ``Resize`` by torchvision to PIL images in the DataLoader workers):
  * localization (training/datasets/localization.py:202-216): RandomHorizontalFlip(0.5) ->
    RandomAffine(degrees=10, translate=(0.05, 0.05), scale=(0.95, 1.05)) -> ColorJitter(brightness=0.2,
    contrast=0.2);
  * classification (training/datasets/classification.py:276-289): RandomAffine(...) -> ColorJitter(...).

torchvision is not a dependency here.  ``sample_params`` draws the random parameters with the same
torch RNG calls, in the same order, as those torchvision classes (so a seeded worker draws the same
values); ``apply_pil`` applies them with the same PIL calls torchvision's functional API makes (the
host path, and the checker of the device path); ``kernels.augment_u8`` applies them on the GPU
with Pillow's arithmetic restated bit for bit (csrc/augment.hip).

Coordinates: the reference moves NO keypoint with the flip or the affine (localization.py:283-299
builds coords from the CSV after the image transform) -- kept as-is for drop-in parity.
``transform_coords`` is the geometrically consistent map for callers that opt in
(``LocalizationConfig.augment_coords``).
"""

from __future__ import annotations

import math

import numpy as np
import torch

# params vector layout (float64 [10]), shared with csrc/augment.hip
P_FLIP, P_A0, P_BRIGHT, P_CONTRAST, P_ORDER = 0, 1, 7, 8, 9


def inverse_affine_matrix(center, angle, translate, scale, shear=(0.0, 0.0)) -> list[float]:
    """torchvision.transforms.functional._get_inverse_affine_matrix (inverted=True): output -> input
    pixel map [a0, a1, a2, a3, a4, a5] as PIL's Image.transform(AFFINE) consumes it."""
    rot = math.radians(angle)
    sx, sy = math.radians(shear[0]), math.radians(shear[1])
    cx, cy = center
    tx, ty = translate
    a = math.cos(rot - sy) / math.cos(sy)
    b = -math.cos(rot - sy) * math.tan(sx) / math.cos(sy) - math.sin(rot)
    c = math.sin(rot - sy) / math.cos(sy)
    d = -math.sin(rot - sy) * math.tan(sx) / math.cos(sy) + math.cos(rot)
    m = [d, -b, 0.0, -c, a, 0.0]
    m = [x / scale for x in m]
    m[2] += m[0] * (-cx - tx) + m[1] * (-cy - ty)
    m[5] += m[3] * (-cx - tx) + m[4] * (-cy - ty)
    m[2] += cx
    m[5] += cy
    return m


def sample_params(height: int, width: int, *, flip: bool, degrees: float = 10.0, translate=(0.05, 0.05),
                  scale=(0.95, 1.05), brightness: float = 0.2, contrast: float = 0.2) -> torch.Tensor:
    """Draw one sample's augmentation like torchvision's RandomHorizontalFlip(0.5) [if ``flip``] ->
    RandomAffine.get_params -> ColorJitter.get_params (global torch RNG, same calls, same order).
    Returns float64 [10] = {flip, a0..a5, brightness, contrast, order (0: brightness first)}."""
    p = torch.zeros(10, dtype=torch.float64)
    if flip:
        p[P_FLIP] = float(torch.rand(1) < 0.5)
    angle = float(torch.empty(1).uniform_(-degrees, degrees).item())
    max_dx, max_dy = float(translate[0] * width), float(translate[1] * height)  # img_size = [width, height]
    tx = int(round(torch.empty(1).uniform_(-max_dx, max_dx).item()))
    ty = int(round(torch.empty(1).uniform_(-max_dy, max_dy).item()))
    sc = float(torch.empty(1).uniform_(scale[0], scale[1]).item())
    m = inverse_affine_matrix([width * 0.5, height * 0.5], angle, (tx, ty), sc)
    p[P_A0:P_A0 + 6] = torch.tensor(m, dtype=torch.float64)
    fn_idx = torch.randperm(4)
    b = float(torch.empty(1).uniform_(max(0.0, 1 - brightness), 1 + brightness))
    c = float(torch.empty(1).uniform_(max(0.0, 1 - contrast), 1 + contrast))
    order = fn_idx.tolist()
    p[P_BRIGHT], p[P_CONTRAST] = b, c
    p[P_ORDER] = 0.0 if order.index(0) < order.index(1) else 1.0
    return p


def apply_pil(img, params: torch.Tensor):
    """The host path: the PIL calls torchvision's functional API makes for these parameters
    (F.hflip -> Image.transpose; F.affine -> Image.transform(AFFINE, NEAREST, fillcolor 0);
    F.adjust_brightness / adjust_contrast -> ImageEnhance)."""
    from PIL import Image, ImageEnhance

    p = params.tolist()
    if p[P_FLIP]:
        img = img.transpose(Image.FLIP_LEFT_RIGHT)
    fill = 0 if img.mode == "L" else tuple([0] * len(img.getbands()))
    img = img.transform(img.size, Image.AFFINE, p[P_A0:P_A0 + 6], Image.NEAREST, fillcolor=fill)
    ops = [lambda im: ImageEnhance.Brightness(im).enhance(p[P_BRIGHT]),
           lambda im: ImageEnhance.Contrast(im).enhance(p[P_CONTRAST])]
    for op in (ops if p[P_ORDER] == 0.0 else ops[::-1]):
        img = op(img)
    return img


def transform_coords(coords: torch.Tensor, params: torch.Tensor, height: int, width: int) -> torch.Tensor:
    """Opt-in consistent keypoints: relative (x, y) in [0, 1] through the same flip and affine as the
    image (pixel centres; the forward map is the inverse of the output->input matrix)."""
    p = params.tolist()
    a0, a1, a2, a3, a4, a5 = p[P_A0:P_A0 + 6]
    det = a0 * a4 - a1 * a3
    inv = np.array([[a4, -a1], [-a3, a0]]) / det
    x = coords[..., 0].double() * width
    y = coords[..., 1].double() * height
    if p[P_FLIP]:
        x = width - x
    u = torch.from_numpy(inv[0, 0] * (x.numpy() - a2) + inv[0, 1] * (y.numpy() - a5))
    v = torch.from_numpy(inv[1, 0] * (x.numpy() - a2) + inv[1, 1] * (y.numpy() - a5))
    return torch.stack([u / width, v / height], dim=-1).to(coords.dtype)
