"""StepEngine(overlap_optimizer=True): AdamW on its own stream in backbone-stage chunks, the next forward gated per stage
(training.engine.ParamGate).  The same arithmetic as the serial update, so the same bits: parameters, AdamW state and
losses after a few steps equal the serial engine's exactly (ConvNeXt-base, bf16 and fp32, 64 x 64 and a frozen
backbone), and an eval forward between steps sees the updated weights."""
import pytest
import torch

import bench
from oracle import weights as ow
from spine_vision_amd.training import CoordinateRegressor, StepEngine

pytestmark = pytest.mark.gpu


def _run(dev, overlap, precision, steps=3, freeze=False, eval_between=False):
    m = CoordinateRegressor("convnext_base", pretrained=False, dropout=0.0, precision=precision)
    ow.fill_module(m)
    m = m.to(dev).train()
    if freeze:
        m.freeze_backbone()
    eng = StepEngine(m, dev, lr=1e-3, weight_decay=1e-5, grad_clip=1.0, overlap_optimizer=overlap)
    assert (eng.gate is not None) == overlap
    img, co, mk = bench.synthetic_batch(2, 64, 64, dev, 77)
    losses, evals = [], []
    for _ in range(steps):
        losses.append(eng.step_localization(img, co, mk))
        if eval_between:
            m.eval()
            with torch.no_grad():
                evals.append(m(img).detach().clone())
            m.train()
    eng.sync_params()
    torch.cuda.synchronize()
    state = {k: v.detach().cpu().clone() for k, v in m.state_dict().items()}
    return ([float(x) for x in losses], state, eng.optimizer.exp_avg.cpu(), eng.optimizer.exp_avg_sq.cpu(),
            [e.cpu() for e in evals])


@pytest.mark.parametrize("precision", ["bf16", "fp32"])
def test_overlapped_update_is_the_serial_update(dev, precision):
    l0, s0, m0, v0, _ = _run(dev, False, precision)
    l1, s1, m1, v1, _ = _run(dev, True, precision)
    assert l0 == l1
    for k in s0:
        assert torch.equal(s0[k], s1[k]), k
    assert torch.equal(m0, m1) and torch.equal(v0, v1)


def test_overlapped_update_frozen_backbone_and_eval_between_steps(dev):
    l0, s0, _, _, e0 = _run(dev, False, "bf16", freeze=True, eval_between=True)
    l1, s1, _, _, e1 = _run(dev, True, "bf16", freeze=True, eval_between=True)
    assert l0 == l1 and all(torch.equal(a, b) for a, b in zip(e0, e1))
    for k in s0:
        assert torch.equal(s0[k], s1[k]), k
    l2, _, _, _, e2 = _run(dev, True, "bf16", eval_between=True)
    l3, _, _, _, e3 = _run(dev, False, "bf16", eval_between=True)
    assert l2 == l3 and all(torch.equal(a, b) for a, b in zip(e2, e3))
