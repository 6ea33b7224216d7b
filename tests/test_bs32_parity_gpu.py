"""Parity at the batch the bench runs: BASELINE configs[1] (ConvNeXt-base 512x512, bs32,
bf16) and configs[3] (ResNet-50 256x256, bs32, 3 heads, bf16), whole model, through StepEngine -- the flat
parameter / gradient buffers and the bf16 weight shadow the bench step uses -- so the production kernel schedule
is value-checked end to end: persistent v9 with several 256x256 tiles per workgroup and its fused epilogues, the
lean side-stream backward, the split-K weight gradients and their folds, the gathered ResNet convolutions.

* ConvNeXt: predicted coordinates and every parameter gradient against the fp32 CPU oracle at B=32, under the
  bf16 bounds of tests/test_parity_geometry_gpu.py (BF16_BOUNDS, measured at B=2).
* ResNet-50: against the bf16 emulation (oracle/bf16emu.py) relative to the bf16 noise floor, as
  tests/test_resnet_parity_256_gpu.py does at B=2.

Reference: the default batch_size=32 (spine_vision/training/trainers/base.py:72), LocalizationTrainer._train_step
(trainers/localization.py:186-209), ClassificationTrainer._train_step (trainers/classification.py:269-290).
The StepEngine steps run with lr = 0 and no weight decay, so the gradients compared are those of the weights
the forward used."""

import numpy as np
import pytest
import torch

from oracle import convnext as oc
from oracle import heads as oh
from oracle import weights as ow

pytestmark = pytest.mark.gpu

# (pred, worst gradient, median gradient) -- the B=2 bounds of test_parity_geometry_gpu.BF16_BOUNDS
CONVNEXT_BF16 = (7e-4, 1.3e-2, 8e-3)


def rel(a, b):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    return float((a - b).norm() / (b.norm() + 1e-30))


@pytest.mark.timeout(900)
def test_convnext_base_512_bs32_bf16_step(dev):
    from spine_vision_amd.training import CoordinateRegressor, StepEngine

    torch.set_num_threads(max(1, min(16, torch.get_num_threads())))
    B = 32
    ref = oh.CoordinateRegressor(oc.create("convnext_base"), 1024, dropout=0.0)
    ow.fill_module(ref)
    img, coords, mask = ow.localization_batch(B, 512, 512)
    hip = CoordinateRegressor("convnext_base", pretrained=False, dropout=0.0, precision="bf16")
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
    # the fp32 oracle at the same batch (CPU, ~30 s on the box's 16 threads)
    ref.train()
    p_ref = ref(img)
    ref.get_loss(p_ref, coords, mask).backward()
    pred = rel(pred_hip, p_ref)
    errs = {n: rel(hip_grads[n], p.grad) for n, p in ref.named_parameters()}
    worst = max(errs, key=errs.get)
    med = float(np.median(list(errs.values())))
    print(f"[parity] convnext_base@512 B32 bf16 (StepEngine): pred rel {pred:.3e}  grad worst {errs[worst]:.3e} "
          f"({worst})  grad median {med:.3e}")
    bp, bw, bm = CONVNEXT_BF16
    assert pred < bp and errs[worst] < bw and med < bm, (pred, errs[worst], med)


@pytest.mark.timeout(900)
def test_resnet50_256_bs32_bf16_step(dev):
    from test_resnet_parity_256_gpu import bf16_vs_emulation, report_floor

    torch.set_num_threads(max(1, min(16, torch.get_num_threads())))
    lerr, table = bf16_vs_emulation(dev, "train", 32, engine=True)
    report_floor("resnet50@256 B32 bf16 train (StepEngine)", lerr, table)
