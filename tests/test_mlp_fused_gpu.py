"""GPU: the fused ConvNeXt MLP forward (csrc/mlp.hip, sv_mlp_fwd) against the two-GEMM path it
replaces -- linear_fwd with the GELU-dual (training) / GELU (eval) epilogue, then the gamma-residual epilogue -- and
against a torch fp32 product of the same bf16 operands.

The fused kernel feeds every accumulator the same MFMA with the same operands in the same k order as the unfused
kernels (fc1's W1 rows permuted at DMA time exactly as v9 permutes a bf16-output B operand, so the GELU'd hidden
fragment IS fc2's operand), and runs the same epilogue arithmetic, so x_out, GELU'(h) and GELU(h) must be equal
BIT for bit.  Shapes: ragged row counts (a partial last tile), and the production shapes of ConvNeXt-base bs32 512x512
(S1: M 524288, C 128; S2: 131072, 256) and ConvNeXt-large bs64 (S1: 1048576, 192).  The whole-model check: a
ConvNeXt bf16 forward + backward with the fused MLP on and off gives the same features and gradients bit for bit.
Reference: timm ConvNeXtBlock.mlp + gamma + shortcut (spine_vision/training/models/backbone.py:50,164-170)."""

import pytest
import torch

from spine_vision_amd import kernels as K
from spine_vision_amd import native as nv

pytestmark = pytest.mark.gpu


def _ops(dev, M, C, seed):
    g = torch.Generator().manual_seed(seed)
    bf = torch.bfloat16
    return {
        "y": torch.randn(M, C, generator=g).to(bf).to(dev),
        "w1": (torch.randn(4 * C, C, generator=g) * 0.08).to(bf).to(dev),
        "b1": (torch.randn(4 * C, generator=g) * 0.1).to(dev),
        "w2": (torch.randn(C, 4 * C, generator=g) * 0.05).to(bf).to(dev),
        "b2": (torch.randn(C, generator=g) * 0.1).to(dev),
        "gam": (torch.rand(C, generator=g) * 0.25 + 0.05).to(dev),
        "x": torch.randn(M, C, generator=g).to(dev),
    }


def _unfused(o, train):
    M, C = o["y"].shape
    dev = o["y"].device
    a = torch.empty(M, 4 * C, device=dev, dtype=torch.bfloat16)
    gh = torch.empty_like(a) if train else None
    if train:
        K.linear_fwd(o["y"], o["w1"], out=gh, out2=a, bias=o["b1"], epilogue=nv.SV_EPI_BIAS_GELU_DUAL)
    else:
        K.linear_fwd(o["y"], o["w1"], out=a, bias=o["b1"], epilogue=nv.SV_EPI_BIAS_GELU)
    xo = torch.empty(M, C, device=dev)
    K.linear_fwd(a, o["w2"], out=xo, bias=o["b2"], gamma=o["gam"], residual=o["x"], epilogue=nv.SV_EPI_BIAS_GAMMA_RES)
    return xo, gh, a


def _fused(o, train):
    M, C = o["y"].shape
    dev = o["y"].device
    gh = torch.full((M, 4 * C), float("nan"), device=dev, dtype=torch.bfloat16) if train else None
    a = torch.full((M, 4 * C), float("nan"), device=dev, dtype=torch.bfloat16) if train else None
    xo = torch.full((M, C), float("nan"), device=dev)
    K.mlp_fwd(o["y"], o["w1"], o["b1"], o["w2"], o["b2"], o["gam"], o["x"], out=xo, gelu_grad=gh, gelu_out=a)
    return xo, gh, a


def _torch_ref(o):
    h = o["y"].float() @ o["w1"].float().t() + o["b1"]
    a = torch.nn.functional.gelu(h).to(torch.bfloat16).float()
    return o["gam"] * (a @ o["w2"].float().t() + o["b2"]) + o["x"]


def _check(o, train):
    xo, gh, a = _fused(o, train)
    xr, ghr, ar = _unfused(o, train)
    torch.cuda.synchronize()
    assert torch.equal(xo, xr), float((xo - xr).abs().max())
    if train:
        assert torch.equal(gh, ghr) and torch.equal(a, ar)
    ref = _torch_ref(o)
    err = float((xo - ref).norm() / ref.norm())
    assert err < 2e-3, err


@pytest.mark.parametrize("C", [128, 192, 256])
@pytest.mark.parametrize("train", [True, False], ids=["train", "eval"])
@pytest.mark.parametrize("M", [4096, 1000, 8 * 256 * 3 + 17])
def test_mlp_fused_matches_two_gemm_path(dev, C, train, M):
    _check(_ops(dev, M, C, seed=M + C), train)


@pytest.mark.timeout(300)
@pytest.mark.parametrize("M,C", [(524288, 128), (131072, 256), (1048576, 192)], ids=["base-S1", "base-S2", "large-S1"])
def test_mlp_fused_production_shapes(dev, M, C):
    o = _ops(dev, M, C, seed=7)
    _check(o, True)
    xo, _, _ = _fused(o, False)
    xr, _, _ = _unfused(o, False)
    assert torch.equal(xo, xr)


def test_mlp_fused_rejects_bad_arguments(dev):
    o = _ops(dev, 256, 128, seed=1)
    with pytest.raises(ValueError):
        K.mlp_fwd(o["y"], o["w1"], o["b1"], o["w2"], o["b2"], o["gam"], o["x"], out=o["x"])  # aliasing
    y = torch.zeros(256, 512, device=dev, dtype=torch.bfloat16)
    w1 = torch.zeros(2048, 512, device=dev, dtype=torch.bfloat16)
    w2 = torch.zeros(512, 2048, device=dev, dtype=torch.bfloat16)
    with pytest.raises(ValueError):  # C = 512: not a fused-MLP shape
        K.mlp_fwd(y, w1, torch.zeros(2048, device=dev), w2, torch.zeros(512, device=dev), torch.zeros(512, device=dev),
                  torch.zeros(256, 512, device=dev), out=torch.empty(256, 512, device=dev))


@pytest.mark.parametrize("name", ["convnext_base", "convnext_large"])
def test_convnext_fused_mlp_model_bitwise(dev, name):
    """Whole backbone, bf16: the fused MLP on (default) and off give the same features and every gradient bit for
    bit (S1 / S2 of base, S1 of large run fused)."""
    from oracle import convnext as oc
    from oracle import weights as ow
    from spine_vision_amd.backbone import create_convnext

    ref = ow.fill_module(oc.create(name))
    img, _, _ = ow.localization_batch(2, 128, 128)
    res = []
    for fused in (True, False):
        hip = create_convnext(name, precision="bf16")
        hip.load_state_dict(ref.state_dict(), strict=True)
        hip = hip.to(dev)
        hip.fused_mlp = fused
        f = hip(img.to(dev))
        dfeat = torch.from_numpy(ow.uniform("dfeat", f.numel(), -1, 1).reshape(f.shape)).to(dev)
        f.backward(dfeat)
        hip.eval()
        with torch.no_grad():
            fe = hip(img.to(dev))
        torch.cuda.synchronize()
        res.append([f.detach().cpu(), fe.cpu()] + [p.grad.detach().cpu().clone() for p in hip.parameters()])
    for i, (u, v) in enumerate(zip(*res)):
        assert torch.equal(u, v), i
