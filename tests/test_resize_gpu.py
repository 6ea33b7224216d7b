"""GPU: the device resize (row f1) bit for bit against PIL, the reference's own first transform
(torchvision Resize on a PIL image = Image.resize((W, H), BILINEAR); spine_vision/training/datasets/
localization.py:199, classification.py:250) -- ragged batches of native-size images, grayscale and RGB,
shrinking and enlarging -- and the device_transform loader path (native-size PNGs -> GPU resize -> the
stem's ToTensor / Normalize) against the host transform chain on the same files."""

import csv

import numpy as np
import pytest
import torch
from PIL import Image

from spine_vision_amd import kernels as K
from spine_vision_amd.training.datasets.resize import ragged_batch

pytestmark = pytest.mark.gpu

SIZES = [(600, 700), (1024, 1024), (300, 257), (97, 1001), (512, 512), (1, 5), (640, 480), (2000, 1500), (511, 513)]


@pytest.mark.parametrize("out_hw", [(512, 512), (256, 256), (384, 512), (1, 1)])
@pytest.mark.parametrize("mode", ["L", "RGB"])
def test_resize_u8_matches_pil(dev, out_hw, mode):
    rng = np.random.default_rng(out_hw[0] + len(mode))
    imgs = []
    for k, (h, w) in enumerate(SIZES):
        shape = (h, w) if mode == "L" else (h, w, 3)
        if k % 2:
            imgs.append(rng.integers(0, 256, shape, dtype=np.uint8))
        else:  # smooth content: sums near the fixed-point rounding boundaries
            yy, xx = np.meshgrid(np.linspace(0, 1, h), np.linspace(0, 1, w), indexing="ij")
            base = (255 * (0.5 + 0.5 * np.sin(7 * xx + 2 * yy + k))).astype(np.uint8)
            imgs.append(base if mode == "L" else np.stack([base, 255 - base, base // 3], axis=-1))
    rb = ragged_batch(imgs, out_hw)
    H, W, C = rb["out_hw"].tolist()
    out = K.resize_u8(rb["src"].to(dev), rb["desc"].to(dev), rb["coef"].to(dev), len(imgs), H, W, C).cpu().numpy()
    for b, im in enumerate(imgs):
        ref = np.asarray(Image.fromarray(im, mode).resize((W, H), Image.BILINEAR))
        assert np.array_equal(out[b], ref), (b, im.shape)


def test_device_resize_loader_matches_host_transform(dev, tmp_path):
    """LocalizationDataset over native-size PNGs: device_transform batches (ragged, resized on the GPU, then
    normalised by the same kernels as the model's stem) equal the host chain (PIL Resize -> ToTensor ->
    Normalize) bit for bit."""
    from spine_vision_amd.training.datasets import LocalizationCollator, LocalizationDataset

    (tmp_path / "img").mkdir()
    rng = np.random.default_rng(3)
    rows = []
    for i, (h, w) in enumerate([(600, 500), (512, 512), (730, 610), (480, 640)]):
        name = f"img/s{i}.png"
        Image.fromarray(rng.integers(0, 256, (h, w), dtype=np.uint8), "L").save(tmp_path / name)
        for lname in ("L1/L2", "L3/L4"):
            rows.append({"image_path": name, "level": lname, "relative_x": 0.4, "relative_y": 0.5,
                         "series_type": "sag_t2", "source": "rsna"})
    with open(tmp_path / "annotations.csv", "w", newline="") as f:
        wr = csv.DictWriter(f, fieldnames=list(rows[0]))
        wr.writeheader()
        wr.writerows(rows)
    kw = dict(image_size=(512, 512), val_ratio=0.0, test_ratio=0.0, augment=False)
    host = LocalizationDataset(tmp_path, split="train", **kw)
    devds = LocalizationDataset(tmp_path, split="train", device_transform=True, **kw)
    col = LocalizationCollator()
    hb = col([host[i] for i in range(len(host))])
    db = col([devds[i] for i in range(len(devds))])
    assert db["image"] is None and "resize" in db
    u8 = K.device_images(db, dev)
    assert tuple(u8.shape) == (len(host), 512, 512)
    x = K.normalize_u8_gray(u8)
    assert torch.equal(x.cpu(), hb["image"])
