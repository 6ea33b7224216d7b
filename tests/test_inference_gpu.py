"""Row f2 on the GPU: ``load_localization_model`` + ``predict_ivd_locations`` (reference
spine_vision/datasets/classification/cropping.py:407-483) through the HIP ConvNeXt, against the
predictions the reference's own functions produced (tests/golden/make_golden_predict.py; torchvision's
Resize / ToTensor / Normalize restated by that script's shim), and the batched form against the
per-slice one."""

import json
import os
import sys

import pytest
import torch

from oracle import weights as ow
from spine_vision_amd.inference import load_localization_model, predict_ivd_locations, predict_ivd_locations_batch
from spine_vision_amd.training import CoordinateRegressor

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))
GOLD = json.load(open(os.path.join(HERE, "golden", "predict_ivd.json")))


def _ckpt(tmp_path):
    m = CoordinateRegressor("convnext_base", pretrained=False, dropout=0.0, precision="fp32")
    ow.fill_module(m)
    path = tmp_path / "best_model.pt"
    torch.save({"model_state_dict": m.state_dict(), "epoch": 0}, path)
    return path


@pytest.mark.parametrize("precision,tol", [("fp32", 1e-3), ("bf16", 2e-2)])
def test_predict_ivd_locations_matches_reference(dev, tmp_path, precision, tol):
    from make_golden_predict import test_images

    model = load_localization_model(_ckpt(tmp_path), "base", "cuda", precision=precision)
    assert not model.training
    size = tuple(GOLD["image_size"])
    for im, g in zip(test_images(), GOLD["images"]):
        pred = predict_ivd_locations(model, im, "cuda", size)
        assert sorted(pred) == list(range(5))
        for k, (x, y) in pred.items():
            rx, ry = g["pred"][str(k)]
            assert abs(x - rx) <= tol * abs(rx) and abs(y - ry) <= tol * abs(ry), (precision, k, (x, y), (rx, ry))


def test_predict_batch_matches_per_slice(dev, tmp_path):
    from make_golden_predict import test_images

    model = load_localization_model(_ckpt(tmp_path), "base", "cuda", precision="fp32")
    ims = test_images()
    size = tuple(GOLD["image_size"])
    single = [predict_ivd_locations(model, im, "cuda", size) for im in ims]
    batch = predict_ivd_locations_batch(model, ims, "cuda", size, batch_size=2)
    for a, b in zip(single, batch):
        for k in a:
            assert abs(a[k][0] - b[k][0]) < 1e-5 and abs(a[k][1] - b[k][1]) < 1e-5
