"""Parity at the batch the bench runs (r4, next 1-2): BASELINE configs[1] (ConvNeXt-base 512x512,
bs32, bf16), configs[4] (ConvNeXt-large 512x512, bs64 per GPU, bf16) and configs[3] (ResNet-50 256x256, bs32, 3 heads,
bf16), whole model, through StepEngine -- the flat parameter / gradient buffers and the bf16 weight shadow the bench
step uses -- so the production kernel schedule is value-checked end to end: the fused narrow-stage MLP, persistent v9
with several 256x256 tiles per workgroup and its fused epilogues, the lean side-stream backward, the split-K weight
gradients at their production splits (ConvNeXt-large bs64: the whole-chip target of the > 150 GFLOP weight gradients)
with their bf16 slabs and folds, the gathered ResNet convolutions.

* ConvNeXt: predicted coordinates and every parameter gradient against oracle/bf16emu.py's emulation of the bf16
  path at the same batch (float64 and float32, on the GPU's float units), relative to the bf16 noise floor, and
  against the reference's own autocast recipe at bf16 width (no farther from the fp32 reference than it):
  tests/test_parity_geometry_gpu.py bf16_parity.  The fp32 reference is the CPU oracle at B=32; at B=64 (69 TFLOP
  of ConvNeXt-large) it is the same arithmetic in float64 on the GPU (the emulation with its roundings removed,
  equal to autograd of the oracle to ~1e-15).
* ResNet-50: against the bf16 emulation (oracle/bf16emu.py) relative to the bf16 noise floor, as
  tests/test_resnet_parity_256_gpu.py does at B=2.

Reference: the default batch_size=32 (spine_vision/training/trainers/base.py:72), LocalizationTrainer._train_step
(trainers/localization.py:186-209), ClassificationTrainer._train_step (trainers/classification.py:269-290); configs[4]:
convnext_large (models/backbone.py:51), bs64 per GPU.  The StepEngine steps run with lr = 0 and no weight decay, so the
gradients compared are those of the weights the forward used."""

import numpy as np
import pytest
import torch

from oracle import convnext as oc
from oracle import heads as oh
from oracle import weights as ow

pytestmark = pytest.mark.gpu


def rel(a, b):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    return float((a - b).norm() / (b.norm() + 1e-30))


def _hip_step(name, B, dev):
    """One StepEngine step of the bf16 HIP regressor at batch B (lr 0) -> (ref oracle module, batch, (pred, grads))."""
    from spine_vision_amd.training import CoordinateRegressor, StepEngine

    nf = {"convnext_base": 1024, "convnext_large": 1536}[name]
    ref = oh.CoordinateRegressor(oc.create(name), nf, dropout=0.0)
    ow.fill_module(ref)
    img, coords, mask = ow.localization_batch(B, 512, 512)
    hip = CoordinateRegressor(name, pretrained=False, dropout=0.0, precision="bf16")
    missing, unexpected = hip.load_state_dict(ref.state_dict(), strict=False)
    assert not unexpected and not [k for k in missing if "num_batches" not in k]
    hip = hip.to(dev).train()
    eng = StepEngine(hip, dev, lr=0.0, weight_decay=0.0, grad_clip=1.0)
    out = {}

    def loss_fn(m):
        out["pred"] = m(img.to(dev))
        return m.get_loss(out["pred"], coords.to(dev), mask.to(dev))

    eng.step(loss_fn)
    torch.cuda.synchronize()
    hip_grads = {n: p.grad.detach().cpu().clone() for n, p in hip.named_parameters()}
    pred_hip = out["pred"].detach().cpu()
    del eng, hip, out
    torch.cuda.empty_cache()
    return ref.train(), (img, coords, mask), (pred_hip, hip_grads)


@pytest.mark.timeout(900)
def test_convnext_base_512_bs32_bf16_step(dev):
    from test_parity_geometry_gpu import autocast_grads, bf16_parity, emu_grads

    torch.set_num_threads(max(1, min(16, torch.get_num_threads())))
    ref, (img, coords, mask), hip = _hip_step("convnext_base", 32, dev)
    e64 = emu_grads(ref, img, coords, mask, dev, torch.float64)
    e32 = emu_grads(ref, img, coords, mask, dev, torch.float32)
    auto = autocast_grads(ref, img, coords, mask, dev)
    # the fp32 oracle at the same batch (CPU, ~30 s on the box's 16 threads)
    p_ref = ref(img)
    ref.get_loss(p_ref, coords, mask).backward()
    fp32 = (p_ref.detach(), {n: p.grad.detach() for n, p in ref.named_parameters()})
    bf16_parity("convnext_base@512 B32 bf16 (StepEngine)", hip, fp32, e64, e32, auto)


@pytest.mark.timeout(900)
def test_convnext_large_512_bs64_bf16_step(dev):
    """configs[4] (missing 3 / next 1): ConvNeXt-large 512x512 at 64 images per GPU through StepEngine --
    the split the bs64 weight gradients take (> 150 GFLOP each: the whole-chip target) is the one the emulation
    rounds its bf16 slabs at."""
    from test_parity_geometry_gpu import autocast_grads, bf16_parity, emu_grads

    ref, (img, coords, mask), hip = _hip_step("convnext_large", 64, dev)
    e64 = emu_grads(ref, img, coords, mask, dev, torch.float64)
    e32 = emu_grads(ref, img, coords, mask, dev, torch.float32)
    fp64 = emu_grads(ref, img, coords, mask, dev, torch.float64, rounding=False)
    auto = autocast_grads(ref, img, coords, mask, dev)
    bf16_parity("convnext_large@512 B64 bf16 (StepEngine)", hip, fp64, e64, e32, auto)


@pytest.mark.timeout(900)
def test_resnet50_256_bs32_bf16_step(dev):
    """configs[3] at its per-GPU batch: the kernels against the bf16 emulation (floor check), and the design against
    the reference's autocast recipe at B=32, where train-mode BatchNorm is well-conditioned (this
    replaces the self-calibrated BF16_VS_FP32 bound as the ResNet bf16 design pin)."""
    from test_resnet_parity_256_gpu import bf16_vs_emulation, design_vs_autocast, report_floor

    torch.set_num_threads(max(1, min(16, torch.get_num_threads())))
    lerr, table, kept = bf16_vs_emulation(dev, "train", 32, engine=True, keep=True)
    report_floor("resnet50@256 B32 bf16 train (StepEngine)", lerr, table)
    design_vs_autocast("resnet50@256 B32 bf16 train (StepEngine)", *kept, dev)
