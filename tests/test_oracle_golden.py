"""CPU: the oracle (fp32 restatement) reproduces the goldens produced by the REFERENCE's own code
(tests/golden/make_golden.py: spine_vision imported with shims, LocalizationTrainer._train_step on the
CPU path) and the inputs regenerate bit-identically from oracle/weights.py."""

import json
import os

import numpy as np
import pytest
import torch

from oracle import convnext as oc
from oracle import heads as oh
from oracle import resnet as orn
from oracle import step as ostep
from oracle import weights as ow

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
META = json.load(open(os.path.join(GOLD, "golden_meta.json")))


def checksum(t):
    t = t.detach().double()
    return [float(t.sum()), float((t * t).sum()), float(t.abs().max())]


def test_inputs_regenerate():
    img, coords, mask = ow.localization_batch(2, 64, 64)
    m = META["loc_inputs"]
    assert np.allclose(checksum(img), m["img"], rtol=1e-12)
    assert np.allclose(checksum(coords), m["coords"], rtol=1e-12)
    assert np.allclose(checksum(mask), m["mask"], rtol=1e-12)


def test_reference_pins_recorded():
    # recorded when the goldens were made: reference code path vs oracle, and HF vs oracle
    for k in ("loc_forward_ref_vs_oracle_maxabs", "loc_loss_ref_vs_oracle_abs", "loc_step_loss_ref_vs_oracle_abs",
              "loc_step_param_ref_vs_oracle_maxabs", "cls_resnet50_forward_ref_vs_oracle_maxabs",
              "cls_resnet18_forward_ref_vs_oracle_maxabs"):
        assert META[k] <= 1e-6, k
    assert META["hf_convnext_base_pooled_maxabs"] <= 1e-4 * META["hf_convnext_base_pooled_scale"]
    assert META["hf_resnet50_pooled_maxabs"] <= 1e-4 * META["hf_resnet50_pooled_scale"]


def test_oracle_localization_forward_and_step():
    g = np.load(os.path.join(GOLD, "localization_convnext_base_64.npz"))
    img, coords, mask = ow.localization_batch(2, 64, 64)
    model = oh.CoordinateRegressor(oc.create("convnext_base"), 1024, dropout=0.0)
    ow.fill_module(model)
    model.eval()
    with torch.no_grad():
        pred = model(img)
        loss = model.get_loss(pred, coords, mask)
    assert np.allclose(pred.numpy(), g["pred"], rtol=0, atol=1e-6)
    assert abs(float(loss) - float(g["loss"])) < 1e-7
    model.train()
    opt = ostep.make_optimizer(model)
    step_loss, _, _ = ostep.train_step_localization(model, opt, img, coords, mask)
    assert abs(step_loss - float(g["step_loss"])) < 1e-7
    params = dict(model.named_parameters())
    for k, ref in META["loc_after_step_checksums"].items():
        assert np.allclose(checksum(params[k]), ref, rtol=1e-6, atol=1e-9), k
        if "after_step/" + k in g:
            assert np.allclose(params[k].detach().numpy(), g["after_step/" + k], atol=1e-7), k


@pytest.mark.parametrize("backbone,nf", [("resnet18", 512), ("resnet50", 2048)])
def test_oracle_classification_forward(backbone, nf):
    g = np.load(os.path.join(GOLD, f"classification_{backbone}_64.npz"))
    img, targets = ow.classification_batch(4, 64, 64)
    model = oh.Classifier(orn.create(backbone), nf, dropout=0.0)
    ow.fill_module(model)
    model.train()
    with torch.no_grad():
        out = model(img)
        loss = model.get_loss(out, targets)
    for k, v in out.items():
        assert np.allclose(v.numpy(), g[f"logits/{k}"], atol=1e-5), k
    assert abs(float(loss) - float(g["loss"])) < 1e-5


def test_adamw_restatement_matches_torch():
    torch.manual_seed(0)
    p = torch.randn(1000, dtype=torch.float64)
    grads = [torch.randn(1000, dtype=torch.float64) for _ in range(3)]
    q = p.clone().requires_grad_(True)
    opt = torch.optim.AdamW([q], lr=1e-3, weight_decay=1e-2)
    m = torch.zeros_like(p)
    v = torch.zeros_like(p)
    for s, gr in enumerate(grads, 1):
        q.grad = gr.clone()
        opt.step()
        p, m, v = ostep.adamw_reference(p, gr, m, v, lr=1e-3, beta1=0.9, beta2=0.999, eps=1e-8,
                                        weight_decay=1e-2, step=s)
    assert torch.allclose(p, q.detach(), rtol=1e-12, atol=1e-14)
