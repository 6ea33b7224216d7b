"""Golden for the localization inference consumer (row f2), produced by the REFERENCE's own code:
``load_localization_model`` + ``predict_ivd_locations`` (spine_vision/datasets/classification/
cropping.py:407-483) and ``normalize_to_uint8`` (spine_vision/io/__init__.py:15-30), imported from
/root/reference with the shims of make_golden.py (build container only):

    python tests/golden/make_golden_predict.py      -> tests/golden/predict_ivd.json

torchvision is not installed here: the three transforms the reference composes are supplied by a
shim restating them (Resize on a PIL image = ``Image.resize((w, h), BILINEAR)``, ToTensor = HWC uint8
-> CHW float / 255, Normalize = (x - mean) / std); everything else -- the min-max to uint8, the RGB
conversion, the model construction and checkpoint load, the forward, the output dict -- is the
reference's code.  The model is CoordinateRegressor(convnext_base) with the oracle/weights.py fill
(regenerated bit-identically by the GPU test); only outputs are stored.
"""

from __future__ import annotations

import json
import os
import sys
import tempfile
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_golden import ROOT, import_reference  # noqa: E402

sys.path.insert(0, ROOT)
from oracle import weights as ow  # noqa: E402

IMG_SIZE = (64, 64)


def test_images():
    """Two synthetic slices in a uint16-like range (H x W not the model size, so Resize does work)."""
    a = ow.uniform("predict.img0", 96 * 80, 0.0, 4000.0).reshape(96, 80).astype(np.float32)
    b = ow.uniform("predict.img1", 72 * 90, -200.0, 1500.0).reshape(72, 90).astype(np.float32)
    return [a, b]


def _torchvision_shim():
    from PIL import Image

    tv = types.ModuleType("torchvision")
    t = types.ModuleType("torchvision.transforms")

    class Compose:
        def __init__(self, ts):
            self.ts = ts

        def __call__(self, x):
            for f in self.ts:
                x = f(x)
            return x

    class Resize:
        def __init__(self, size):
            self.size = size

        def __call__(self, img):
            return img.resize((self.size[1], self.size[0]), Image.BILINEAR)

    class ToTensor:
        def __call__(self, img):
            return torch.from_numpy(np.array(img, dtype=np.uint8)).permute(2, 0, 1).contiguous().float().div(255)

    class Normalize:
        def __init__(self, mean, std):
            self.mean = torch.tensor(mean).view(-1, 1, 1)
            self.std = torch.tensor(std).view(-1, 1, 1)

        def __call__(self, x):
            return (x - self.mean) / self.std

    t.Compose, t.Resize, t.ToTensor, t.Normalize = Compose, Resize, ToTensor, Normalize
    tv.transforms = t
    sys.modules["torchvision"] = tv
    sys.modules["torchvision.transforms"] = t


def main():
    _, generic = import_reference()
    _torchvision_shim()  # after the reference's shims: transformers probes for a real torchvision
    from spine_vision.datasets.classification import cropping
    from spine_vision.io import normalize_to_uint8

    ref = generic.CoordinateRegressor(backbone="convnext_base", pretrained=False, num_levels=5)
    ow.fill_module(ref)
    tmp = tempfile.mkdtemp()
    path = os.path.join(tmp, "best_model.pt")
    torch.save({"model_state_dict": ref.state_dict()}, path)
    model = cropping.load_localization_model(path, "base", "cpu")
    out = {"image_size": list(IMG_SIZE), "images": []}
    for im in test_images():
        u8 = normalize_to_uint8(im)
        pred = cropping.predict_ivd_locations(model, im, "cpu", IMG_SIZE)
        out["images"].append({"u8_sum": int(u8.astype(np.int64).sum()), "u8_sq": int((u8.astype(np.int64) ** 2).sum()),
                              "pred": {str(k): list(v) for k, v in pred.items()}})
    with open(os.path.join(HERE, "predict_ivd.json"), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
