"""Parity at the BASELINE geometry (VERDICT r1 "what's weak" 1): the HIP path against the fp32 CPU
oracle at the sizes the bench runs, so the production GEMM schedules (the 256x256 v8 dispatch at
>= 256 tiles, gemm.hip) and the bf16 lean side-stream backward are covered end to end, and
ConvNeXt-large runs in bf16.

* fp32 (parity mode) @512: predicted coordinates and EVERY gradient within 1e-3 relative
  (north_star bar: "outputs within 1e-3 of CPU reference").
* bf16: bf16 misses 1e-3 by construction (finding 5: 3.4e-3 feature error measured
  in the survey).  Each bound below is about 2x the error measured on MI355X for exactly this case
  (the measured values are in the comment beside it and in DESIGN.md); a bf16 accuracy regression of
  2x fails.  Relative error = ||hip - ref||_2 / ||ref||_2 per tensor.
"""

import numpy as np
import pytest
import torch

from oracle import convnext as oc
from oracle import heads as oh
from oracle import resnet as orn
from oracle import weights as ow

pytestmark = pytest.mark.gpu

# (pred bound, worst-gradient bound, median-gradient bound), ~2x the values measured on MI355X
# (gpurun_out r2b, round 2): base@512 B2 3.1e-4 / 6.1e-3 / 3.8e-3; large@64 B2 3.9e-4 / 9.1e-3 / 6.0e-3;
# large@512 B1 3.7e-4 / 6.1e-3 / 3.8e-3
BF16_BOUNDS = {
    ("convnext_base", 512, 2): (7e-4, 1.3e-2, 8e-3),
    ("convnext_large", 64, 2): (8e-4, 2e-2, 1.2e-2),
    ("convnext_large", 512, 1): (8e-4, 1.3e-2, 8e-3),
}


def rel(a, b):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    return float((a - b).norm() / (b.norm() + 1e-30))


def _loc_pair(name, precision, dev):
    from spine_vision_amd.training import CoordinateRegressor

    nf = {"convnext_base": 1024, "convnext_large": 1536}[name]
    ref = oh.CoordinateRegressor(oc.create(name), nf, dropout=0.0)
    ow.fill_module(ref)
    hip = CoordinateRegressor(name, pretrained=False, dropout=0.0, precision=precision)
    missing, unexpected = hip.load_state_dict(ref.state_dict(), strict=False)
    assert not unexpected and not [k for k in missing if "num_batches" not in k]
    return ref.train(), hip.to(dev).train()


def _loc_case(name, res, B, precision, dev):
    ref, hip = _loc_pair(name, precision, dev)
    img, coords, mask = ow.localization_batch(B, res, res)
    p_ref = ref(img)
    ref.get_loss(p_ref, coords, mask).backward()
    p_hip = hip(img.to(dev))
    hip.get_loss(p_hip, coords.to(dev), mask.to(dev)).backward()
    torch.cuda.synchronize()
    errs = {}
    for (n1, a), (n2, b) in zip(ref.named_parameters(), hip.named_parameters()):
        assert n1 == n2
        errs[n1] = rel(b.grad, a.grad)
    return rel(p_hip, p_ref), errs


def _report(tag, pred_err, errs):
    worst = max(errs, key=errs.get)
    med = float(np.median(list(errs.values())))
    print(f"[parity] {tag}: pred rel {pred_err:.3e}  grad worst {errs[worst]:.3e} ({worst})  grad median {med:.3e}")
    return errs[worst], med


def test_convnext_base_512_fp32(dev):
    pred, errs = _loc_case("convnext_base", 512, 2, "fp32", dev)
    worst, _ = _report("convnext_base@512 B2 fp32", pred, errs)
    assert pred < 1e-3
    bad = {k: v for k, v in errs.items() if v >= 1e-3}
    assert not bad, bad


@pytest.mark.parametrize("name,res,B", [("convnext_base", 512, 2), ("convnext_large", 64, 2),
                                        ("convnext_large", 512, 1)])
def test_convnext_bf16_geometry(dev, name, res, B):
    pred, errs = _loc_case(name, res, B, "bf16", dev)
    worst, med = _report(f"{name}@{res} B{B} bf16", pred, errs)
    bp, bw, bm = BF16_BOUNDS[(name, res, B)]
    assert pred < bp and worst < bw and med < bm, (pred, worst, med)


@pytest.mark.parametrize("knob", ["lean_sync", "overlap_wgrad"])
def test_convnext_bf16_schedule_knobs_match_default(dev, knob):
    """SV_LEAN_SYNC=0 / SV_SIDE_STREAM=0 change only WHERE the same kernels run (one main->side hand-off
    per block vs three; weight gradients on the side stream vs the main stream): every gradient must equal
    the default schedule's bit for bit."""
    from spine_vision_amd.backbone import create_convnext

    ref = ow.fill_module(oc.create("convnext_base"))
    img, _, _ = ow.localization_batch(2, 128, 128)
    grads = []
    for off in (False, True):
        hip = create_convnext("convnext_base", precision="bf16")
        hip.load_state_dict(ref.state_dict(), strict=True)
        hip = hip.to(dev)
        if off:
            setattr(hip, knob, False)
        f = hip(img.to(dev))
        dfeat = torch.from_numpy(ow.uniform("dfeat", f.numel(), -1, 1).reshape(f.shape)).to(dev)
        f.backward(dfeat)
        torch.cuda.synchronize()
        grads.append([p.grad.detach().cpu().clone() for p in hip.parameters()])
    for a, b in zip(*grads):
        assert torch.equal(a, b)


def test_resnet_bf16_side_stream_matches_single_stream(dev):
    """ResNet bf16 backward: the per-block weight gradients on the side stream (default) against every
    kernel on the current stream (SV_SIDE_STREAM=0): same kernels, so every gradient and the BatchNorm
    running statistics must be equal bit for bit."""
    from spine_vision_amd.backbone import create_resnet

    ref = ow.fill_module(orn.create("resnet50"))
    img, _ = ow.classification_batch(2, 128, 128)
    out = []
    for overlap in (True, False):
        hip = create_resnet("resnet50", precision="bf16")
        hip.load_state_dict(ref.state_dict(), strict=True)
        hip = hip.to(dev).train()
        hip.overlap_wgrad = overlap
        f = hip(img.to(dev))
        dfeat = torch.from_numpy(ow.uniform("dfeat", f.numel(), -1, 1).reshape(f.shape)).to(dev)
        f.backward(dfeat)
        torch.cuda.synchronize()
        out.append([p.grad.detach().cpu().clone() for p in hip.parameters()] +
                   [b.detach().cpu().clone() for b in hip.buffers()])
    for a, b in zip(*out):
        assert torch.equal(a, b)
