"""Whole-backbone parity: HIP ConvNeXt vs the fp32 CPU oracle on identical generated weights.

fp32 (parity) mode: features and every parameter gradient within 1e-3 relative (north_star bar).
bf16 mode: features within bf16 tolerance (documented in DESIGN.md; SURVEY.md §0 finding 5).
"""

import pytest
import torch

from oracle import convnext as oc
from oracle import weights as ow
from spine_vision_amd.backbone import create_convnext

pytestmark = pytest.mark.gpu


def rel(a, b):
    a = a.detach().float().cpu()
    b = b.detach().float().cpu()
    return ((a - b).norm() / (b.norm() + 1e-30)).item()


def _pair(name, precision, dev):
    ref = ow.fill_module(oc.create(name))
    hip = create_convnext(name, precision=precision)
    missing, unexpected = hip.load_state_dict(ref.state_dict(), strict=True)
    assert not missing and not unexpected
    return ref, hip.to(dev)


@pytest.mark.parametrize("name,res", [("convnext_base", 64), ("convnext_large", 64)])
def test_convnext_fp32_forward_backward(dev, name, res):
    ref, hip = _pair(name, "fp32", dev)
    img, _, _ = ow.localization_batch(2, res, res)
    f_ref = ref(img)
    f_hip = hip(img.to(dev))
    assert rel(f_hip, f_ref) < 1e-4
    dfeat = torch.from_numpy(ow.uniform("dfeat", f_ref.numel(), -1, 1).reshape(f_ref.shape))
    f_ref.backward(dfeat)
    f_hip.backward(dfeat.to(dev))
    worst = 0.0
    for (n1, p1), (n2, p2) in zip(ref.named_parameters(), hip.named_parameters()):
        assert n1 == n2
        r = rel(p2.grad, p1.grad)
        worst = max(worst, r)
        assert r < 1e-3, f"{n1}: rel {r}"
    print(f"{name}@{res}: worst grad rel {worst:.2e}")


def test_convnext_bf16_forward(dev):
    ref, hip = _pair("convnext_base", "bf16", dev)
    img, _, _ = ow.localization_batch(2, 64, 64)
    with torch.no_grad():
        f_ref = ref(img)
        f_hip = hip(img.to(dev))
    r = rel(f_hip, f_ref)
    print(f"[parity] convnext_base@64 B2 bf16 features rel {r:.3e}")
    assert r < 2e-2


def test_convnext_bf16_backward(dev):
    """bf16 mode backward (bf16 GEMM operands incl. the bf16 gradient-stream copy and the gamma-folded
    fc2 weight) against the fp32 oracle: per-tensor relative L2 of every gradient within bf16 bounds."""
    ref, hip = _pair("convnext_base", "bf16", dev)
    img, _, _ = ow.localization_batch(2, 64, 64)
    f_ref = ref(img)
    f_hip = hip(img.to(dev))
    dfeat = torch.from_numpy(ow.uniform("dfeat", f_ref.numel(), -1, 1).reshape(f_ref.shape))
    f_ref.backward(dfeat)
    f_hip.backward(dfeat.to(dev))
    worst = 0.0
    for (n1, p1), (n2, p2) in zip(ref.named_parameters(), hip.named_parameters()):
        r = rel(p2.grad, p1.grad)
        worst = max(worst, r)
        assert r < 5e-2, f"{n1}: rel {r}"
    print(f"[parity] convnext_base@64 B2 bf16 backbone grads: worst rel {worst:.3e}")
