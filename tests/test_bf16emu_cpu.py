"""CPU: the ConvNeXt bf16 emulation (oracle/bf16emu.py ConvNeXtBf16Emu, test infrastructure) that the GPU parity tests
hold the HIP bf16 path against.

* With every bf16 rounding removed it IS the oracle: its explicit backward (LayerNorm, GELU, depthwise, layer-scale,
  downsample, stem, pooled head) equals torch autograd of oracle/convnext.py + oracle/heads.py in float64 to ~1e-15.
* With the roundings, its distance to the fp32 oracle is bf16-sized and smaller than the reference's own autocast
  recipe at bf16 width (the anchor the GPU tests use), and the float32 emulation -- the noise floor -- is closer to the
  float64 one than either.
* The slab rule: a split-K weight gradient's per-slice bf16 rounding is applied over contiguous row slices, and a
  split of 1 (or f32 slabs) is the plain product."""

import copy

import numpy as np
import pytest
import torch

from oracle import bf16emu as be
from oracle import convnext as oc
from oracle import heads as oh
from oracle import weights as ow


def _rel(a, b):
    return float((a.double() - b.double()).norm() / (b.double().norm() + 1e-300))


def _case(B=2, res=64):
    ref = oh.CoordinateRegressor(oc.create("convnext_base"), 1024, dropout=0.0)
    ow.fill_module(ref)
    return ref.train(), ow.localization_batch(B, res, res)


def _split(N, K, M, target):  # a production-like rule: bf16 slabs over 2 slices where the rows allow it
    return (2, True) if M % 128 == 0 and min(N, K) >= 128 else (1, False)


def test_emulation_without_rounding_is_the_oracle(monkeypatch):
    torch.set_num_threads(min(8, torch.get_num_threads()))
    ref, (img, coords, mask) = _case()
    r64 = copy.deepcopy(ref).double()
    p = r64(img.double())
    r64.get_loss(p, coords.double(), mask).backward()
    monkeypatch.setattr(be, "bf16_round", lambda t: t)
    monkeypatch.setattr(be, "STORE_BF16", False)
    pe, ge = be.regressor_grads(ref, img, coords, mask, torch.float64, _split)
    assert _rel(pe, p.detach()) < 1e-13
    worst = max(_rel(ge[n], q.grad) for n, q in r64.named_parameters())
    assert worst < 1e-12, worst


def test_emulation_distances_order():
    torch.set_num_threads(min(8, torch.get_num_threads()))
    ref, (img, coords, mask) = _case()
    p32 = ref(img)
    ref.get_loss(p32, coords, mask).backward()
    g32 = {n: q.grad.clone() for n, q in ref.named_parameters()}
    p64e, g64e = be.regressor_grads(ref, img, coords, mask, torch.float64, _split)
    p32e, g32e = be.regressor_grads(ref, img, coords, mask, torch.float32, _split)
    with torch.autocast("cpu", dtype=torch.bfloat16):
        ref.zero_grad()
        pa = ref(img)
    ref.get_loss(pa.float(), coords, mask).backward()
    ga = {n: q.grad.clone() for n, q in ref.named_parameters()}
    emu = np.median([_rel(g64e[n], g32[n]) for n in g32])
    auto = np.median([_rel(ga[n], g32[n]) for n in g32])
    floor = np.median([_rel(g32e[n], g64e[n]) for n in g32])
    assert 1e-4 < emu < auto, (emu, auto)  # bf16-sized, and below the reference recipe's own bf16 distance
    assert floor < emu, (floor, emu)
    assert _rel(p64e, p32.detach()) < _rel(pa.float(), p32.detach())


def test_slab_wgrad_rounds_each_contiguous_slice():
    g = torch.Generator().manual_seed(3)
    A = torch.randn(512, 8, generator=g, dtype=torch.float64)
    B = torch.randn(512, 4, generator=g, dtype=torch.float64)
    full = A.t() @ B
    assert torch.equal(be._slab_wgrad(A, B, 1, True), full)
    assert torch.equal(be._slab_wgrad(A, B, 4, False), full)
    want = sum(be.bf16_round(A[s * 128:(s + 1) * 128].t() @ B[s * 128:(s + 1) * 128]) for s in range(4))
    assert torch.equal(be._slab_wgrad(A, B, 4, True), want)
    assert not torch.equal(want, full)


def test_emulation_follows_the_depthwise_operand_precision():
    """The emulation rounds the depthwise conv's operands to bf16 exactly when the product runs the matrix-core kernels
    (SV_DW_MFMA, same default in both)."""
    from oracle import bf16emu
    from spine_vision_amd import kernels as K

    assert bf16emu.DW_BF16_OPERANDS == K.DW_MFMA and bf16emu.DW_BF16_WGRAD == K.DW_MFMA_WGRAD
