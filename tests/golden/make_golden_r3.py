"""Round-3 golden fixtures, produced by the REFERENCE's own code (imported from /root/reference with the
shims of make_golden.py; run in the build container only -- the GPU box never needs the reference):

    python tests/golden/make_golden_r3.py

  loss_variants.json   CoordinateRegressor.get_loss (reference training/models/generic.py:393-417) for
                       every loss_type the reference accepts (generic.py:354-361: nn.MSELoss,
                       nn.SmoothL1Loss, nn.HuberLoss(delta=0.1)) on fixed predictions / targets, with
                       mask=None, a partial mask, a one-level mask and an all-invalid mask: the loss,
                       dL/dpredictions, and whether the returned loss carries a graph (the all-invalid
                       case returns a constant torch.tensor(0.0), generic.py:414-415).
Inputs are regenerated bit-identically by oracle/weights.py; only outputs are stored.
"""

from __future__ import annotations

import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_golden import ROOT, import_reference  # noqa: E402

sys.path.insert(0, ROOT)
from oracle import weights as ow  # noqa: E402


def loss_inputs():
    """(pred [B,5,2] in (0,1), target [B,5,2], masks); stored in the fixture beside the outputs."""
    B = 4
    pred = ow.uniform("lv.pred", B * 10, 0.02, 0.98).reshape(B, 5, 2)
    # targets near and far from the predictions: |d| spans both sides of huber's delta = 0.1
    tgt = np.clip(pred + ow.uniform("lv.off", B * 10, -0.35, 0.35).reshape(B, 5, 2), 0.0, 1.0).astype(np.float32)
    partial = (ow.uniform("lv.mask", B * 5, 0.0, 1.0).reshape(B, 5) > 0.3).astype(np.float32)
    one = np.zeros((B, 5), np.float32)
    one[2, 3] = 1.0
    masks = {"none": None, "partial": partial, "one": one, "all_invalid": np.zeros((B, 5), np.float32)}
    return pred, tgt, masks


def main():
    _, generic = import_reference()
    pred, tgt, masks = loss_inputs()
    out = {"generator": "tests/golden/make_golden_r3.py", "shape": list(pred.shape), "cases": [],
           "pred": pred.reshape(-1).tolist(), "target": tgt.reshape(-1).tolist(),
           "masks": {k: (None if v is None else v.reshape(-1).tolist()) for k, v in masks.items()}}
    for lt in ("mse", "smooth_l1", "huber"):
        model = generic.CoordinateRegressor(backbone="resnet18", pretrained=False, dropout=0.0, loss_type=lt)
        for mname, m in masks.items():
            p = torch.from_numpy(pred.copy()).requires_grad_(True)
            t = torch.from_numpy(tgt)
            loss = model.get_loss(p, t, mask=None if m is None else torch.from_numpy(m))
            case = {"loss_type": lt, "mask": mname, "loss": float(loss), "requires_grad": bool(loss.requires_grad)}
            if loss.requires_grad:
                loss.backward()
                case["grad"] = p.grad.reshape(-1).tolist()
            out["cases"].append(case)
    with open(os.path.join(HERE, "loss_variants.json"), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    print("ok")


if __name__ == "__main__":
    main()
