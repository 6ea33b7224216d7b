"""Parity at the BASELINE geometry (VERDICT r1 "what's weak" 1): the HIP path against the fp32 CPU
oracle at the sizes the bench runs, so the production GEMM schedules (the 256x256 v8 dispatch at
>= 256 tiles, gemm.hip) and the bf16 lean side-stream backward are covered end to end, and
ConvNeXt-large runs in bf16.

* fp32 (parity mode) @512: predicted coordinates and EVERY gradient within 1e-3 relative
  (north_star bar: "outputs within 1e-3 of CPU reference").
* bf16: bf16 misses 1e-3 by construction (finding 5), so the bf16 path
  is pinned two ways, neither calibrated on its own measurement:
  - the KERNELS against ``oracle.bf16emu.ConvNeXtBf16Emu``: the oracle's arithmetic in float64 with a bf16 rounding at
    exactly the HIP path's store points (z, y, GELU(h), GELU'(h), dh, dy, dz, the bf16 gradient copies, every split-K
    slab at the split the build picks), relative to the bf16 noise floor -- the same emulation in float32, whose
    distance to the float64 one is what any implementation that rounds at those points but accumulates in another
    order must show (floor_check: per-tensor ratio, median ratio, cosine, norm);
  - the DESIGN against the reference's own recipe: the reference trains under autocast (trainers/base.py:230-237,
    localization.py:195-200); the oracle model run under torch.autocast at the same bf16 width is that recipe's
    rounding, and the HIP path must be no farther from the fp32 oracle than it (pred, worst and median gradient).
  Measured on CPU at 512x512 B=2 (this module's emulation): floor median 1.1e-3 (worst 2.9e-3); emulation vs fp32
  3.8e-3 median / 5.9e-3 worst, pred 3.1e-4; autocast-bf16 vs fp32 1.1e-2 median / 0.26 worst, pred 2.0e-3.
Relative error = ||hip - ref||_2 / ||ref||_2 per tensor.
"""

import copy

import numpy as np
import pytest
import torch

from oracle import bf16emu as be
from oracle import convnext as oc
from oracle import heads as oh
from oracle import resnet as orn
from oracle import weights as ow

pytestmark = pytest.mark.gpu

# floor_check parameters for ConvNeXt (see oracle/bf16emu.py floor_check): the HIP distance to the float64 emulation
# against the float32 emulation's, per tensor (floors below FLOOR_MIN clamped up to it)
FLOOR = {"ratio_median": 1.5, "ratio_max": 3.0, "min_floor": 2e-4, "min_cos": 0.999}


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


def _loc_case(name, res, B, precision, dev, keep=False):
    ref, hip = _loc_pair(name, precision, dev)
    img, coords, mask = ow.localization_batch(B, res, res)
    p_ref = ref(img)
    ref.get_loss(p_ref, coords, mask).backward()
    p_hip = hip(img.to(dev))
    hip.get_loss(p_hip, coords.to(dev), mask.to(dev)).backward()
    torch.cuda.synchronize()
    if keep:  # for the bf16 checks: everything on the host, the HIP model released
        hg = {n: p.grad.detach().cpu() for n, p in hip.named_parameters()}
        rg = {n: p.grad.detach() for n, p in ref.named_parameters()}
        return (p_hip.detach().cpu(), hg), (p_ref.detach(), rg), (ref, img, coords, mask)
    errs = {}
    for (n1, a), (n2, b) in zip(ref.named_parameters(), hip.named_parameters()):
        assert n1 == n2
        errs[n1] = rel(b.grad, a.grad)
    return rel(p_hip, p_ref), errs


def emu_split():
    """The split-K geometry the build picks for a weight gradient (pure host arithmetic of kernels.py)."""
    from spine_vision_amd import kernels as K

    def split(N, Kd, M, target):
        s_ = K._wgrad_split_for(N, Kd, M, target)
        return s_, K._bf16_slabs(N, Kd, M, s_, True)

    return split


def emu_grads(ref, img, coords, mask, dev, dtype, rounding=True):
    """oracle.bf16emu's regressor step on the GPU's float units (torch's native kernels: MIOpen off), -> (pred,
    {name: grad}) on the host.  rounding=False: the reference arithmetic itself (the emulation with every bf16
    rounding removed, equal to autograd of the oracle to ~1e-15 in float64)."""
    import time

    saved = (be.bf16_round, be.STORE_BF16)
    t0 = time.time()
    try:
        if not rounding:
            be.bf16_round, be.STORE_BF16 = (lambda t: t), False
        with torch.backends.cudnn.flags(enabled=False):
            pred, g = be.regressor_grads(ref, img, coords, mask, dtype, emu_split(), 256, device=dev)
        out = pred.cpu(), {n: v.detach().cpu() for n, v in g.items()}
        del g
        print(f"[emu] {dtype} rounding={rounding} B{img.shape[0]}: {time.time() - t0:.1f} s", flush=True)
        return out
    finally:
        be.bf16_round, be.STORE_BF16 = saved
        torch.cuda.empty_cache()


def autocast_grads(ref, img, coords, mask, dev):
    """The reference's own mixed-precision recipe at bf16 width: the oracle model (fp32 master weights) under
    torch.autocast -- conv / linear in bf16, LayerNorm in f32 (trainers/base.py:230-237, localization.py:195-200)."""
    m = copy.deepcopy(ref).to(dev)
    m.zero_grad(set_to_none=True)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        p = m(img.to(dev))
    m.get_loss(p.float(), coords.to(dev), mask.to(dev)).backward()
    torch.cuda.synchronize()
    out = p.detach().float().cpu(), {n: q.grad.detach().float().cpu() for n, q in m.named_parameters()}
    del m
    torch.cuda.empty_cache()
    return out


def bf16_parity(tag, hip, fp32, e64, e32, auto):
    """hip / fp32 / e64 / e32 / auto: (pred, {name: grad}).  Kernels against the bf16 emulation (floor_check);
    design against the reference's autocast recipe (no farther from fp32 than it)."""
    fl = be.floor_check(hip[1], e64[1], e32[1], **FLOOR)
    ratios = {n: v[2] for n, v in fl.items()}
    wr = max(ratios, key=ratios.get)
    pe, pf = rel(hip[0], e64[0]), rel(e32[0], e64[0])
    eh = {n: rel(hip[1][n], g) for n, g in fp32[1].items()}
    ea = {n: rel(auto[1][n], g) for n, g in fp32[1].items()}
    ee = {n: rel(e64[1][n], g) for n, g in fp32[1].items()}
    ph, pa, pee = rel(hip[0], fp32[0]), rel(auto[0], fp32[0]), rel(e64[0], fp32[0])
    wh, wa = max(eh, key=eh.get), max(ea, key=ea.get)
    print(f"[parity] {tag}: vs emu64 pred {pe:.3e} (floor {pf:.3e}), grad ratio median "
          f"{np.median(list(ratios.values())):.2f} worst {ratios[wr]:.2f} ({wr}), floor median "
          f"{np.median([v[1] for v in fl.values()]):.3e}, min cosine {min(v[3] for v in fl.values()):.5f}")
    print(f"[parity] {tag}: vs fp32 -- HIP pred {ph:.3e} grad median {np.median(list(eh.values())):.3e} worst "
          f"{eh[wh]:.3e} ({wh}); emu64 pred {pee:.3e} median {np.median(list(ee.values())):.3e}; autocast-bf16 pred "
          f"{pa:.3e} median {np.median(list(ea.values())):.3e} worst {ea[wa]:.3e} ({wa})")
    assert pe <= 3.0 * max(pf, 1e-5), (pe, pf)
    assert ph <= pa and np.median(list(eh.values())) <= np.median(list(ea.values())) and eh[wh] <= ea[wa], \
        (ph, pa, eh[wh], ea[wa])
    return fl


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


@pytest.mark.timeout(600)
@pytest.mark.parametrize("name,res,B", [("convnext_base", 512, 2), ("convnext_large", 64, 2),
                                        ("convnext_large", 512, 1)])
def test_convnext_bf16_geometry(dev, name, res, B):
    hip, fp32, (ref, img, coords, mask) = _loc_case(name, res, B, "bf16", dev, keep=True)
    torch.cuda.empty_cache()
    e64 = emu_grads(ref, img, coords, mask, dev, torch.float64)
    e32 = emu_grads(ref, img, coords, mask, dev, torch.float32)
    auto = autocast_grads(ref, img, coords, mask, dev)
    bf16_parity(f"{name}@{res} B{B} bf16", hip, fp32, e64, e32, auto)


@pytest.mark.parametrize("knob", ["lean_sync", "overlap_wgrad", "tail_main", "tail_main_before_stem"])
def test_convnext_bf16_schedule_knobs_match_default(dev, knob, monkeypatch):
    """SV_LEAN_SYNC=0 / SV_SIDE_STREAM=0 / SV_TAIL_MAIN=0 change only WHERE the same kernels run (one main->side
    hand-off per block vs three; weight gradients on the side stream vs the main stream; the last block's fc1 and
    depthwise weight gradients after the stem on the main stream vs on the side stream): every gradient must equal
    the default schedule's bit for bit."""
    from spine_vision_amd.backbone import convnext as cx
    from spine_vision_amd.backbone import create_convnext

    ref = ow.fill_module(oc.create("convnext_base"))
    img, _, _ = ow.localization_batch(2, 128, 128)
    grads = []
    for off in (False, True):
        hip = create_convnext("convnext_base", precision="bf16")
        hip.load_state_dict(ref.state_dict(), strict=True)
        hip = hip.to(dev)
        hip.fused_mlp_bwd = False  # the fused backward runs only in the lean schedule: compare the same kernels
        if knob.startswith("tail_main"):
            monkeypatch.setattr(cx, "_TAIL_MAIN", 0 if not off else (2 if knob.endswith("stem") else 1))
        elif off:
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
