"""ResNet-50 classification parity at the BASELINE geometry (configs[3]: 256x256, 3 heads), whole model,
on a WELL-CONDITIONED fixture: ``oracle.weights.fill_module(conditioned=True)``
-- He-uniform conv weights, each residual block's last BatchNorm scale in [0.05, 0.3], non-trivial BN
running statistics.  On the default fixture a perturbation grows ~1.2x per block, so even torch's own CPU
bf16 autocast was 7-21% off the fp32 logits and the old test could only bound bf16 against it.

north_star: "per-head classification logits match the reference PyTorch-CPU path within 1e-3 relative".
Reference: spine_vision/training/models/generic.py:134-177 (Classifier.forward / get_loss), timm ResNet-50
via models/backbone.py:29.

* fp32 (parity mode), eval and train mode BN: every head's logits within 1e-3 (relative L2 and
  max |delta| / max |ref|) of the fp32 CPU oracle.
* fp32 gradients: eval mode -- every parameter gradient within 1e-3 of the fp32 oracle.  Train mode --
  BatchNorm over B=2 batch statistics makes the backward itself ill-conditioned (the fp32 oracle is up to
  5.5e-3 off float64 on this fixture, measured on CPU; a ReLU-mask flip at fp32 rounding moves whole
  gradient rows), so each HIP gradient is held against float64 within max(1e-3, 3x the fp32 oracle's own
  error), as in test_resnet_fp32_forward_backward.
* bf16: bounds ~2x the error measured on MI355X for exactly these cases (values beside BF16_BOUNDS and in
  DESIGN.md "Oracle and parity").
"""

import copy

import numpy as np
import pytest
import torch

from oracle import heads as oh
from oracle import resnet as orn
from oracle import weights as ow

pytestmark = pytest.mark.gpu

LABELS = ["pfirrmann", "modic", "herniation"]
# (logits rel-L2 bound, worst-gradient bound, median-gradient bound) for bf16, ~2x measured on MI355X
# (gpurun_out/r4a, round 3): eval 1.57e-2 / 8.7e-2 (conv1.weight) / 2.14e-2; train 1.06e-2 / 0.517 / 0.369.
# The train-mode gradients are ill-conditioned in ANY reduced precision: torch's CPU bf16 autocast of the
# same model is 0.35-0.37 (median) / 0.48-0.52 (worst) off fp32 at B=2 and at B=8 (measured in the build
# container), and even the fp32 oracle is 1.6e-3 (median) off float64: a train-mode BatchNorm projects its
# input gradient to zero mean per channel, so the BN scale / shift gradients upstream are small
# differences of large sums.
BF16_BOUNDS = {
    "eval": (3.2e-2, 0.18, 4.5e-2),
    "train": (2.2e-2, 1.05, 0.75),
}


def rel(a, b):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    return float((a - b).norm() / (b.norm() + 1e-30))


def maxrel(a, b):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    return float((a - b).abs().max() / (b.abs().max() + 1e-30))


def _case(dev, precision, mode):
    from spine_vision_amd.training import Classifier
    from spine_vision_amd.training.trainers.classification import _create_tasks_for_training

    tasks = _create_tasks_for_training(target_labels=LABELS, label_smoothing=0.1)
    ref = oh.Classifier(orn.create("resnet50"), 2048, dropout=0.0)
    ow.fill_module(ref, conditioned=True)
    r64 = copy.deepcopy(ref).double()
    hip = Classifier(backbone="resnet50", tasks=tasks, pretrained=False, dropout=0.0, precision=precision)
    hip.load_state_dict(ref.state_dict(), strict=True)
    train = mode == "train"
    ref.train(train)
    r64.train(train)
    hip = hip.to(dev).train(train)
    img, targets = ow.classification_batch(2, 256, 256)
    o_ref = ref(img)
    ref.get_loss(o_ref, targets).backward()
    o64 = r64(img.double())
    r64.get_loss(o64, targets).backward()
    o_hip = hip(img.to(dev))
    hip.get_loss(o_hip, {k: v.to(dev) for k, v in targets.items()}).backward()
    torch.cuda.synchronize()
    logit = {k: (rel(o_hip[k], o_ref[k]), maxrel(o_hip[k], o_ref[k])) for k in LABELS}
    p64 = dict(r64.named_parameters())
    hp = dict(hip.named_parameters())
    grads = {}
    for n, p in ref.named_parameters():
        grads[n] = (rel(hp[n].grad, p.grad), rel(hp[n].grad, p64[n].grad), rel(p.grad, p64[n].grad))
    buf = {}
    if train:  # running statistics after one train-mode forward
        hb = dict(hip.named_buffers())
        for n, b in ref.named_buffers():
            if b.is_floating_point():
                buf[n] = rel(hb[n], b)
    return logit, grads, buf


def _report(tag, logit, grads):
    lw = max(v[0] for v in logit.values())
    gv = {n: v[0] for n, v in grads.items()}
    worst = max(gv, key=gv.get)
    med = float(np.median(list(gv.values())))
    print(f"[parity] {tag}: logits rel {lw:.3e} (max-abs rel {max(v[1] for v in logit.values()):.3e})  "
          f"grad vs fp32 oracle worst {gv[worst]:.3e} ({worst}) median {med:.3e}")
    return lw, gv[worst], med


@pytest.mark.parametrize("mode", ["eval", "train"])
def test_resnet50_256_fp32(dev, mode):
    logit, grads, buf = _case(dev, "fp32", mode)
    _report(f"resnet50@256 B2 fp32 {mode}", logit, grads)
    for k, (r, mr) in logit.items():
        assert r < 1e-3 and mr < 1e-3, (k, r, mr)
    if mode == "eval":
        bad = {n: v[0] for n, v in grads.items() if v[0] >= 1e-3}
    else:
        bad = {n: v for n, v in grads.items() if v[1] >= max(1e-3, 3.0 * v[2])}
        w = max(grads, key=lambda n: grads[n][1])
        print(f"[parity] fp32 train: worst vs float64 {grads[w][1]:.3e} ({w}; fp32 oracle {grads[w][2]:.3e})")
    assert not bad, bad
    assert all(v < 1e-5 for v in buf.values()), buf


@pytest.mark.parametrize("mode", ["eval", "train"])
def test_resnet50_256_bf16(dev, mode):
    logit, grads, buf = _case(dev, "bf16", mode)
    lw, worst, med = _report(f"resnet50@256 B2 bf16 {mode}", logit, grads)
    bl, bw, bm = BF16_BOUNDS[mode]
    assert lw < bl and worst < bw and med < bm, (lw, worst, med)
    assert all(v < 1e-2 for v in buf.values()), buf
