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
* bf16: against ``oracle.bf16emu`` -- the same model in float64 with a bf16
  rounding at exactly the HIP path's store points, forward and backward -- relative to the bf16 NOISE FLOOR,
  the distance between that emulation in float64 and in float32 (two valid roundings-at-the-same-points
  computations; see oracle/bf16emu.py floor_check).  Measured on CPU: the floor is 0.24-0.26 (train) and
  0.03 (eval) median per gradient tensor at B=2..32, so no fixed bound below it can hold for ANY bf16
  implementation; the HIP distance is held to a small multiple of it per tensor, with a cosine / norm guard
  that a dropped or zeroed gradient cannot pass.  The fp32-oracle distances are printed as
  measurements only.
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
# floor_check parameters: median / worst ratio of the HIP distance to the bf16 noise floor, the floor's lower
# clamp, and the cosine guard.  Measured on MI355X (profiles/round4/r7c_tests.log): ratio median 0.97-1.02,
# worst 1.24-1.53, min cosine 0.934-0.999 (B=2 eval / train, B=32 train) -- the HIP path is as far from the
# float64 emulation as the float32 emulation is
FLOOR = {"ratio_median": 1.5, "ratio_max": 2.5, "min_floor": 1e-2, "min_cos": 0.9}
# the reference-anchored bound beside the floor check (an emulation that rounds where the HIP path rounds
# cannot see a rounding scheme drifting away from the reference's autocast): the bf16 path against the fp32 oracle
# (logits rel, worst gradient, median gradient), ~2x the round-3 measurements (DESIGN.md "Classification at the
# BASELINE geometry": eval 1.6e-2 / 8.7e-2 / 2.1e-2, train 1.1e-2 / 0.52 / 0.37)
BF16_VS_FP32 = {"eval": (3.2e-2, 0.18, 4.5e-2), "train": (2.2e-2, 1.05, 0.75)}


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


def bf16_vs_emulation(dev, mode, B, engine=False, keep=False):
    """HIP bf16 (whole model, optionally through StepEngine's flat buffers / bf16 shadow as the bench runs it)
    against oracle.bf16emu in float64 and float32; -> (logit errors, floor_check table), plus with ``keep``
    (HIP logits, HIP gradients, the oracle module, image, targets) for the design check."""
    from oracle import bf16emu as be
    from spine_vision_amd.training import Classifier, StepEngine
    from spine_vision_amd.training.trainers.classification import _create_tasks_for_training

    tasks = _create_tasks_for_training(target_labels=LABELS, label_smoothing=0.1)
    ref = oh.Classifier(orn.create("resnet50"), 2048, dropout=0.0)
    ow.fill_module(ref, conditioned=True)
    train = mode == "train"
    img, targets = ow.classification_batch(B, 256, 256)
    o64, g64, b64 = be.classifier_grads(ref, img, targets, torch.float64, train)
    o32, g32, _ = be.classifier_grads(ref, img, targets, torch.float32, train)
    hip = Classifier(backbone="resnet50", tasks=tasks, pretrained=False, dropout=0.0, precision="bf16")
    hip.load_state_dict(ref.state_dict(), strict=True)
    hip = hip.to(dev).train(train)
    tg = {k: v.to(dev) for k, v in targets.items()}
    if engine:  # lr 0: the step's AdamW leaves the weights (and the compared gradients) as the forward saw them
        eng = StepEngine(hip, dev, lr=0.0, weight_decay=0.0, grad_clip=1.0)
        logits = {}
        eng.step(lambda m: _keep(logits, m(img.to(dev))) and m.get_loss(logits, tg))
    else:
        logits = hip(img.to(dev))
        hip.get_loss(logits, tg).backward()
    torch.cuda.synchronize()
    lerr = {k: (rel(logits[k], o64[k]), rel(o32[k], o64[k])) for k in LABELS}
    table = be.floor_check({n: p.grad for n, p in hip.named_parameters()}, g64, g32, **FLOOR)
    if train:
        hb = dict(hip.named_buffers())
        berr = {n: rel(hb[n], b) for n, b in b64.items()}
        assert all(v < 1e-2 for v in berr.values()), berr
    if keep:
        hg = {n: p.grad.detach().float().cpu() for n, p in hip.named_parameters()}
        return lerr, table, ({k: v.detach().float().cpu() for k, v in logits.items()}, hg, ref, img, targets)
    return lerr, table


# Design check margin on the GRADIENTS (not the logits): train-mode BatchNorm keeps ResNet-50's gradients badly
# conditioned even at B=32 on this fixture -- measured on MI355X (r13a): HIP 0.346 median / 0.529 worst and the
# reference's autocast recipe 0.350 / 0.522 from fp32, the same size as the bf16 noise floor itself (float64 vs float32
# emulation at the same rounding points: 0.24-0.26 median).  Any two bf16 computations land that far from fp32 and
# their worst tensors trade places from one fixture to the next; a design that rounds in the wrong place shows up as a
# SYSTEMATIC excess, which the 10 % margin still catches (the logits keep the strict bound: 1.37e-2 vs 1.52e-2).
DESIGN_GRAD_MARGIN = 1.10


def design_vs_autocast(tag, hip_logits, hip_grads, ref, img, targets, dev):
    """The design pin (as the ConvNeXt bf16_parity's): the HIP bf16 path no farther from the fp32
    reference than the reference's own recipe -- the oracle model under torch.autocast at the same bf16 width
    (trainers/base.py:230-237, trainers/classification.py:269-290: conv / linear in bf16, BatchNorm in the input's
    width with f32 statistics) -- on the worst head's logits (strictly), the median and the worst gradient (within
    DESIGN_GRAD_MARGIN, see above).  The fp32 reference is the CPU oracle (train-mode BN over the same batch)."""
    m32 = copy.deepcopy(ref).train()
    m32.zero_grad(set_to_none=True)
    o32 = m32(img)
    m32.get_loss(o32, targets).backward()
    g32 = {n: q.grad.detach().float() for n, q in m32.named_parameters()}
    ma = copy.deepcopy(ref).to(dev).train()
    ma.zero_grad(set_to_none=True)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        oa = ma(img.to(dev))
    oa = {k: v.float() for k, v in oa.items()}
    ma.get_loss(oa, {k: v.to(dev) for k, v in targets.items()}).backward()
    torch.cuda.synchronize()
    ga = {n: q.grad.detach().float().cpu() for n, q in ma.named_parameters()}
    del ma
    torch.cuda.empty_cache()
    lh = max(rel(hip_logits[k], o32[k]) for k in LABELS)
    la = max(rel(oa[k], o32[k]) for k in LABELS)
    eh = {n: rel(hip_grads[n], g) for n, g in g32.items()}
    ea = {n: rel(ga[n], g) for n, g in g32.items()}
    wh, wa = max(eh, key=eh.get), max(ea, key=ea.get)
    mh, ma_ = float(np.median(list(eh.values()))), float(np.median(list(ea.values())))
    print(f"[design] {tag}: vs fp32 -- HIP logits {lh:.3e} grad median {mh:.3e} worst {eh[wh]:.3e} ({wh}); "
          f"autocast-bf16 logits {la:.3e} grad median {ma_:.3e} worst {ea[wa]:.3e} ({wa})")
    assert lh <= la, (lh, la)
    assert mh <= DESIGN_GRAD_MARGIN * ma_ and eh[wh] <= DESIGN_GRAD_MARGIN * ea[wa], (mh, ma_, eh[wh], ea[wa])
    return lh, la, mh, ma_


def _keep(d, out):
    d.update(out)
    return True


def report_floor(tag, lerr, table):
    ratios = {n: v[2] for n, v in table.items()}
    worst = max(ratios, key=ratios.get)
    errs = [v[0] for v in table.values()]
    floors = [v[1] for v in table.values()]
    print(f"[parity] {tag}: logits rel vs emu64 {max(v[0] for v in lerr.values()):.3e} (floor "
          f"{max(v[1] for v in lerr.values()):.3e}); grad vs emu64 median {np.median(errs):.3e} (floor median "
          f"{np.median(floors):.3e}); ratio median {np.median(list(ratios.values())):.2f}, worst {ratios[worst]:.2f} "
          f"({worst}); min cosine {min(v[3] for v in table.values()):.3f}")
    for k, (e, f) in lerr.items():
        assert e <= 4.0 * max(f, 1e-3), (k, e, f)
        assert e < 2e-2, (k, e)  # absolute too: the logits north_star bounds (measured 2.6e-3 .. 7.4e-3)
    return float(np.median(errs))


@pytest.mark.parametrize("mode", ["eval", "train"])
def test_resnet50_256_bf16_vs_emulation(dev, mode):
    lerr, table = bf16_vs_emulation(dev, mode, 2)
    med = report_floor(f"resnet50@256 B2 bf16 {mode}", lerr, table)
    if mode == "eval":  # an absolute bound where the noise floor allows one (floor median 1.4e-2; train: 0.25)
        assert med < 5e-2, med


@pytest.mark.parametrize("mode", ["eval", "train"])
def test_resnet50_256_bf16_vs_fp32(dev, mode):
    """The bf16 path against the fp32 oracle -- the reference's own arithmetic -- under absolute bounds (BF16_VS_FP32,
    ~2x measured).  Most of that distance is the bf16 noise itself (test_resnet50_256_bf16_vs_emulation pins the
    kernels against it); this bound is what catches a rounding design that drifts from the reference."""
    logit, grads, buf = _case(dev, "bf16", mode)
    lw, worst, med = _report(f"resnet50@256 B2 bf16 {mode} (vs fp32 oracle)", logit, grads)
    bl, bw, bm = BF16_VS_FP32[mode]
    assert lw < bl and worst < bw and med < bm, (lw, worst, med)
    assert all(v < 1e-2 for v in buf.values()), buf
