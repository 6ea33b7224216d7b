"""The depthwise 7x7 conv on the matrix cores (csrc/dwmfma.hip: sv_dwconv7_fwd_mfma / sv_dwconv7_bwd_data_mfma; VERDICT
r5 next 4) against a float64 conv over the same bf16-rounded operands -- timm ConvNeXtBlock.conv_dw
(spine_vision/training/models/backbone.py:50) under torch.autocast(bfloat16), which rounds conv_dw's input and weight
to bf16.  The MFMA sums in f32, so z differs from bf16(reference) only where that sum's rounding flips the bf16
rounding (bounded per element by one bf16 step), and dx by f32 summation error."""
import pytest
import torch
import torch.nn.functional as F

from spine_vision_amd import kernels as K

pytestmark = pytest.mark.gpu

SHAPES = [(2, 32, 32, 512), (2, 128, 128, 128), (4, 16, 16, 1024), (2, 64, 64, 256), (1, 23, 37, 96), (3, 9, 5, 64)]
IDS = ["S3", "S1", "S4", "S2", "ragged", "tiny"]


def _q(t):
    return t.to(torch.bfloat16).to(torch.float64)


def _operands(dev, shape, seed, xdtype=torch.float32):
    B, H, W, C = shape
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(B, H, W, C, generator=g).to(xdtype).to(dev)
    w = (torch.randn(C, 1, 7, 7, generator=g) * 0.15).to(dev)
    b = (torch.randn(C, generator=g) * 0.1).to(dev)
    return x, w, b


@pytest.mark.parametrize("shape", SHAPES, ids=IDS)
@pytest.mark.parametrize("xdtype", [torch.float32, torch.bfloat16], ids=["xf32", "xbf16"])
def test_dw_mfma_forward(dev, shape, xdtype):
    B, H, W, C = shape
    x, w, b = _operands(dev, shape, seed=sum(shape), xdtype=xdtype)
    z = K.dwconv7_fwd_mfma(x, w, b)
    z2 = K.dwconv7_fwd_mfma(x, w, b)
    ref = F.conv2d(_q(x).permute(0, 3, 1, 2), _q(w), b.double(), padding=3, groups=C).permute(0, 2, 3, 1)
    torch.cuda.synchronize()
    assert torch.equal(z, z2), "run to run"
    zf = z.double()
    err = (zf - ref).abs()
    # one bf16 rounding step of the result (2^-8 relative) plus the f32 sum's own error
    bound = ref.abs() * 2.0**-8 + 1e-6 * float(ref.abs().max())
    assert not (err > bound).any(), (int((err > bound).sum()), float(err.max()))
    exact = float((z == ref.to(torch.bfloat16)).float().mean())
    print(f"[dw mfma fwd] {shape} x {xdtype}: {exact:.5f} of z equal bf16(ref), max err {float(err.max()):.2e}")
    assert exact > 0.99


@pytest.mark.parametrize("shape", SHAPES, ids=IDS)
@pytest.mark.parametrize("accumulate", [True, False], ids=["acc", "store"])
def test_dw_mfma_backward_data(dev, shape, accumulate):
    B, H, W, C = shape
    _, w, _ = _operands(dev, shape, seed=7 + sum(shape))
    g = torch.Generator().manual_seed(3)
    dz = (torch.randn(B, H, W, C, generator=g) * 0.5).to(torch.bfloat16).to(dev)
    dx0 = torch.randn(B, H, W, C, generator=g).to(dev)
    dx = dx0.clone()
    dxb = torch.empty(B, H, W, C, device=dev, dtype=torch.bfloat16)
    K.call("sv_dwconv7_bwd_data_mfma", K.ptr(dz), K.ptr(w), K.ptr(dx), K.ptr(dxb), int(accumulate), B, H, W, C)
    ref = torch.nn.grad.conv2d_input((B, C, H, W), _q(w), dz.double().permute(0, 3, 1, 2), padding=3,
                                     groups=C).permute(0, 2, 3, 1)
    if accumulate:
        ref = ref + dx0.double()
    torch.cuda.synchronize()
    err = (dx.double() - ref).abs()
    scale = float(ref.abs().max())
    assert float(err.max()) <= 2e-6 * scale, (float(err.max()), scale)
    assert torch.equal(dxb, dx.to(torch.bfloat16)), "the bf16 copy is bf16(dx)"
    print(f"[dw mfma bwd] {shape} acc={accumulate}: max err {float(err.max()):.2e} of {scale:.2e}")


def test_dw_mfma_rejects_bad_channels(dev):
    x, w, b = _operands(dev, (1, 8, 8, 48), seed=1)
    with pytest.raises(Exception):
        K.dwconv7_fwd_mfma(x, w, b)


@pytest.mark.parametrize("shape", SHAPES, ids=IDS)
@pytest.mark.parametrize("xdtype", [torch.float32, torch.bfloat16], ids=["xf32", "xbf16"])
def test_dw_mfma_weight_gradient(dev, shape, xdtype, monkeypatch):
    """sv_dwconv7_bwd_weight_mfma (through K.dwconv7_bwd_weight, partials folded): the 49 taps and the bias of every
    channel against a float64 conv2d_weight over bf16(x) and the bf16 dz; bitwise run to run."""
    monkeypatch.setattr(K, "DW_MFMA_WGRAD", True)  # opt-in in the product (slower than the VALU kernel, DESIGN)
    B, H, W, C = shape
    x, _, _ = _operands(dev, shape, seed=11 + sum(shape), xdtype=xdtype)
    g = torch.Generator().manual_seed(5)
    dz = (torch.randn(B, H, W, C, generator=g) * 0.5).to(torch.bfloat16).to(dev)
    outs = []
    for _ in range(2):
        dw = torch.zeros(C, 49, device=dev)
        db = torch.zeros(C, device=dev)
        K.dwconv7_bwd_weight(dz, x, dw=dw, db=db)
        outs.append((dw, db))
    ref = torch.nn.grad.conv2d_weight(_q(x).permute(0, 3, 1, 2), (C, 1, 7, 7), dz.double().permute(0, 3, 1, 2),
                                      padding=3, groups=C).view(C, 49)
    refb = dz.double().sum((0, 1, 2))
    torch.cuda.synchronize()
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1]), "run to run"
    dw, db = outs[0]
    # f32 sums of B H W products (exact bf16 x bf16 products): relative to the sum of |terms| of each tap
    absref = torch.nn.grad.conv2d_weight(_q(x).abs().permute(0, 3, 1, 2), (C, 1, 7, 7),
                                         dz.double().abs().permute(0, 3, 1, 2), padding=3, groups=C).view(C, 49)
    err = (dw.double() - ref).abs()
    assert not (err > 1e-5 * absref + 1e-12).any(), (float((err / (absref + 1e-30)).max()))
    errb = (db.double() - refb).abs()
    assert not (errb > 1e-5 * dz.double().abs().sum((0, 1, 2)) + 1e-12).any()
    print(f"[dw mfma wgrad] {shape} x {xdtype}: max err / sum|terms| {float((err / (absref + 1e-30)).max()):.2e}")
