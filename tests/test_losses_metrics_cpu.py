"""CPU: FocalLoss, ClassifierMetrics and LocalizationMetrics against outputs of the REFERENCE's own
modules (tests/golden/focal_loss.json, metrics.json -- written by tests/golden/make_golden_r2.py from
spine_vision/training/losses.py:90-139 and metrics.py:121-185, 321-518)."""

import json
import os

import numpy as np
import pytest
import torch

from spine_vision_amd.training.losses import FocalLoss
from spine_vision_amd.training.metrics import ClassifierMetrics, LocalizationMetrics

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _load(name):
    with open(os.path.join(GOLD, name)) as f:
        return json.load(f)


def test_focal_loss_matches_reference():
    g = _load("focal_loss.json")
    logits = torch.tensor(g["logits"]).reshape(g["shape"])
    targets = torch.tensor(g["targets"]).reshape(g["shape"])
    for c in g["cases"]:
        out = FocalLoss(gamma=c["gamma"], alpha=c["alpha"], pos_weight=c["pos_weight"], reduction=c["reduction"])(
            logits, targets)
        np.testing.assert_allclose(out.reshape(-1).numpy(), np.array(c["out"], dtype=np.float32), rtol=1e-6,
                                   atol=1e-7, err_msg=str(c))
    with pytest.raises(ValueError):
        FocalLoss(reduction="avg")


def test_classifier_metrics_match_reference():
    g = _load("metrics.json")
    n = g["n"]
    shapes = {"pfirrmann": (n, 5), "modic": (n, 4), "herniation": (n, 1)}
    preds = {k: torch.tensor(v).reshape(shapes[k]) for k, v in g["preds"].items()}
    tg = {"pfirrmann": torch.tensor(g["targets"]["pfirrmann"], dtype=torch.int64),
          "modic": torch.tensor(g["targets"]["modic"], dtype=torch.int64),
          "herniation": torch.tensor(g["targets"]["herniation"]).reshape(n, 1)}
    for key, ref in g["classifier"].items():
        labels = key.split(",")
        cm = ClassifierMetrics(target_labels=labels)
        cm.update({k: preds[k][:20] for k in labels}, {k: tg[k][:20] for k in labels})
        cm.update({k: preds[k][20:] for k in labels}, {k: tg[k][20:] for k in labels})
        got = cm.compute()
        assert set(got) == set(ref), (key, sorted(got), sorted(ref))
        for k in ref:
            assert got[k] == pytest.approx(ref[k], rel=1e-12, abs=1e-12), (key, k)


def test_localization_metrics_match_reference():
    g = _load("metrics.json")["localization"]
    p = np.array(g["pred"], dtype=np.float32).reshape(-1, 2)
    t = np.array(g["target"], dtype=np.float32).reshape(-1, 2)
    lm = LocalizationMetrics(pck_thresholds=[0.02, 0.05, 0.10], level_names=g["level_names"])
    got = lm.compute(p, t, np.array(g["levels"]))
    assert set(got) == set(g["metrics"]), (sorted(got), sorted(g["metrics"]))
    for k, v in g["metrics"].items():
        assert got[k] == pytest.approx(v, rel=1e-6, abs=1e-7), k


@pytest.mark.parametrize("loss_type", ["mse", "smooth_l1", "huber"])
def test_regressor_loss_variants_match_reference(loss_type):
    """CoordinateRegressor.get_loss for every loss_type against the reference module's own outputs
    (tests/golden/loss_variants.json, make_golden_r3.py; reference generic.py:354-361, 393-417): loss and
    dL/dpred with mask=None, a partial mask and a single valid level.

    All-invalid mask (documented divergence, DESIGN.md "Losses"): the reference returns a constant
    torch.tensor(0.0) without a graph, so its accelerator.backward() raises; the build returns a
    differentiable 0 (no host sync to detect the case), whose gradient is exactly zero -- the step then
    runs AdamW on zero gradients (weight decay and moment decay only)."""
    from spine_vision_amd.training import CoordinateRegressor

    g = _load("loss_variants.json")
    shape = g["shape"]
    pred0 = torch.tensor(g["pred"]).reshape(shape)
    tgt = torch.tensor(g["target"]).reshape(shape)
    model = CoordinateRegressor("resnet18", pretrained=False, dropout=0.0, loss_type=loss_type)
    cases = [c for c in g["cases"] if c["loss_type"] == loss_type]
    assert len(cases) == 4
    for c in cases:
        m = g["masks"][c["mask"]]
        mask = None if m is None else torch.tensor(m).reshape(shape[:2])
        p = pred0.clone().requires_grad_(True)
        loss = model.get_loss(p, tgt, mask=mask)
        if c["requires_grad"]:
            loss.backward()
            np.testing.assert_allclose(float(loss), c["loss"], rtol=1e-6, atol=0)
            np.testing.assert_allclose(p.grad.reshape(-1).numpy(), np.array(c["grad"], np.float32), rtol=1e-5,
                                       atol=1e-9)
        else:
            assert c["mask"] == "all_invalid" and c["loss"] == 0.0
            assert float(loss) == 0.0
            loss.backward()
            assert float(p.grad.abs().max()) == 0.0
