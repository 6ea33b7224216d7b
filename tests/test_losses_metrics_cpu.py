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
