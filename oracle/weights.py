"""Deterministic, platform-independent parameter and input generator (TEST INFRASTRUCTURE ONLY).

splitmix64 over a counter, keyed by an FNV-1a hash of the state_dict key, gives the same float32
values on any machine (pure numpy integer arithmetic), so the GPU box regenerates exactly the
weights the goldens were made with.
"""

from __future__ import annotations

import re

import numpy as np
import torch

_MASK = np.uint64(0xFFFFFFFFFFFFFFFF)


def fnv1a64(s: str) -> int:
    h = 0xCBF29CE484222325
    for b in s.encode():
        h ^= b
        h = (h * 0x100000001B3) & 0xFFFFFFFFFFFFFFFF
    return h


def splitmix64(seed: int, n: int) -> np.ndarray:
    """n uint64 outputs of splitmix64 with state seed + (i+1)*golden."""
    with np.errstate(over="ignore"):
        i = np.arange(1, n + 1, dtype=np.uint64)
        z = (np.uint64(seed) + i * np.uint64(0x9E3779B97F4A7C15)) & _MASK
        z = ((z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)) & _MASK
        z = ((z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)) & _MASK
        z = z ^ (z >> np.uint64(31))
    return z


def uniform(key: str, n: int, lo: float, hi: float, seed: int = 42) -> np.ndarray:
    z = splitmix64(fnv1a64(key) ^ seed, n)
    u = (z >> np.uint64(40)).astype(np.float64) / float(1 << 24)  # 24-bit mantissa in [0,1)
    return (lo + (hi - lo) * u).astype(np.float32)


def _range_for(key: str, shape: tuple[int, ...]) -> tuple[float, float]:
    """Value ranges that keep every layer non-degenerate (the survey's 'parity is vacuous at
    gamma=1e-6' warning): layer-scale gamma in [0.05, 0.3], LN affine near 1/0, fan-in scaled
    weights, non-trivial BN running statistics."""
    name = key.rsplit(".", 1)[-1]
    if name == "gamma":
        return 0.05, 0.3
    if name == "running_var":
        return 0.5, 1.5
    if name == "running_mean":
        return -0.2, 0.2
    if name == "num_batches_tracked":
        return 0.0, 0.0
    if len(shape) == 1:
        if name == "weight":  # LayerNorm / BatchNorm affine scale
            return 0.8, 1.2
        return -0.1, 0.1  # biases
    fan_in = int(np.prod(shape[1:]))
    a = 1.0 / np.sqrt(fan_in)
    return -a, a


_BLOCK_BN = re.compile(r"(.*layer\d+\.\d+)\.bn(\d)\.weight$")


def _last_bns(keys) -> dict[str, int]:
    """Per residual block (``...layerN.i``): the index of its last BatchNorm (bn2 Basic, bn3 Bottleneck)."""
    last: dict[str, int] = {}
    for k in keys:
        m = _BLOCK_BN.match(k)
        if m:
            last[m.group(1)] = max(last.get(m.group(1), 0), int(m.group(2)))
    return last


def _range_conditioned(key: str, shape: tuple[int, ...], last: dict[str, int]) -> tuple[float, float]:
    """Well-conditioned ResNet fixture: He-uniform conv weights (variance 2/fan_in, the
    scale a ReLU network keeps its activations at) and each residual block's LAST BatchNorm scale in
    [0.05, 0.3] -- a trained network's small residual-branch scale, the counterpart of ConvNeXt's layer-scale
    gamma range above and of timm's zero_init_last.  Everything else as _range_for.  Measured on CPU at
    ResNet-50 256x256 B=2 against float64: fp32 logits 5e-7-1e-6 (train) / 1.5e-7-9e-7 (eval) instead of
    1.7e-5-2.6e-5, and the per-step amplification of a perturbation that made the default fixture's
    bf16 logits 7-21% off drops to 0.8-1.5%."""
    m = _BLOCK_BN.match(key)
    if m and int(m.group(2)) == last[m.group(1)]:
        return 0.05, 0.3
    if len(shape) == 4:
        a = float(np.sqrt(6.0 / np.prod(shape[1:])))
        return -a, a
    return _range_for(key, shape)


def fill_module(module: torch.nn.Module, seed: int = 42, prefix: str = "", conditioned: bool = False) -> torch.nn.Module:
    """Overwrite every parameter and floating buffer of ``module`` with generated values
    (``conditioned``: the ResNet fixture of _range_conditioned)."""
    sd = module.state_dict()
    last = _last_bns(sd.keys()) if conditioned else {}
    with torch.no_grad():
        for key, t in sd.items():
            if not t.is_floating_point():
                continue
            if conditioned:
                lo, hi = _range_conditioned(key, tuple(t.shape), last)
            else:
                lo, hi = _range_for(key, tuple(t.shape))
            v = uniform(prefix + key, t.numel(), lo, hi, seed).reshape(tuple(t.shape))
            t.copy_(torch.from_numpy(v))
    return module


def state_dict_for(module: torch.nn.Module, seed: int = 42, prefix: str = "") -> dict[str, torch.Tensor]:
    out = {}
    for key, t in module.state_dict().items():
        if not t.is_floating_point():
            out[key] = t.clone()
            continue
        lo, hi = _range_for(key, tuple(t.shape))
        out[key] = torch.from_numpy(uniform(prefix + key, t.numel(), lo, hi, seed).reshape(tuple(t.shape)))
    return out


# ---- synthetic batches (BASELINE.md / SURVEY.md §8(d) input spec) ---------------------------------
IMAGENET_MEAN = (0.485, 0.456, 0.406)
IMAGENET_STD = (0.229, 0.224, 0.225)


def uint8_images(key: str, B: int, H: int, W: int, seed: int = 42) -> np.ndarray:
    z = splitmix64(fnv1a64(key) ^ seed, B * H * W)
    return (z >> np.uint64(56)).astype(np.uint8).reshape(B, H, W)


def normalize_gray(u8: np.ndarray) -> torch.Tensor:
    """uint8 [B,H,W] grayscale -> replicate to RGB (training/datasets/localization.py:254) -> /255
    (ToTensor) -> ImageNet Normalize -> f32 NCHW."""
    x = torch.from_numpy(u8.astype(np.float32) / 255.0)[:, None].expand(-1, 3, -1, -1)
    mean = torch.tensor(IMAGENET_MEAN).view(1, 3, 1, 1)
    std = torch.tensor(IMAGENET_STD).view(1, 3, 1, 1)
    return ((x - mean) / std).contiguous()


def localization_batch(B: int, H: int, W: int, seed: int = 42, levels: int = 5):
    img = normalize_gray(uint8_images("loc.image", B, H, W, seed))
    coords = torch.from_numpy(uniform("loc.coords", B * levels * 2, 0.05, 0.95, seed).reshape(B, levels, 2))
    m = uniform("loc.mask", B * levels, 0.0, 1.0, seed).reshape(B, levels)
    mask = torch.from_numpy((m >= 0.1).astype(np.float32))
    return img, coords, mask


def classification_batch(B: int, H: int, W: int, seed: int = 42):
    t2 = uint8_images("cls.t2", B, H, W, seed).astype(np.float32) / 255.0
    t1 = uint8_images("cls.t1", B, H, W, seed).astype(np.float32) / 255.0
    x = torch.from_numpy(np.stack([t2, t1, t2], axis=1))  # [T2, T1, T2] channels
    mean = torch.tensor(IMAGENET_MEAN).view(1, 3, 1, 1)
    std = torch.tensor(IMAGENET_STD).view(1, 3, 1, 1)
    img = ((x - mean) / std).contiguous()
    u = uniform("cls.labels", B * 3, 0.0, 1.0, seed).reshape(3, B)
    targets = {
        "pfirrmann": torch.from_numpy(np.minimum((u[0] * 5).astype(np.int64), 4)),
        "modic": torch.from_numpy(np.minimum((u[1] * 4).astype(np.int64), 3)),
        "herniation": torch.from_numpy((u[2] < 0.3).astype(np.float32)),
    }
    return img, targets
