"""Per-kernel parity on the MI355X: every HIP entry point against a plain PyTorch fp32 CPU
reference of the same op (fp32/f32-MFMA mode to ~1e-5, bf16 mode to bf16 tolerances)."""

import pytest
import torch
import torch.nn.functional as F

from spine_vision_amd import kernels as K
from spine_vision_amd import native as nv

pytestmark = pytest.mark.gpu


def rel(a, b):
    a = a.detach().float().cpu()
    b = b.detach().float().cpu()
    return ((a - b).norm() / (b.norm() + 1e-30)).item()


def maxrel(a, b, floor=1e-3):
    a = a.detach().float().cpu()
    b = b.detach().float().cpu()
    return ((a - b).abs() / (b.abs() + floor * b.abs().max())).max().item()


def bf(t):
    return t.to(torch.bfloat16).float()


# ---------------------------------------------------------------------------------------- GEMM
@pytest.mark.parametrize("compute_bf16", [False, True])
@pytest.mark.parametrize("a_kmajor", [True, False])
@pytest.mark.parametrize("b_kmajor", [True, False])
@pytest.mark.parametrize("shape", [(256, 128, 64), (200, 136, 96), (8, 512, 40), (1000, 24, 1024),
                                   (1024, 512, 512), (264, 392, 128), (4096, 256, 2048)])
def test_gemm_layouts(dev, compute_bf16, a_kmajor, b_kmajor, shape):
    M, N, Kd = shape
    g = torch.Generator().manual_seed(M * 7 + N * 3 + Kd)
    Am = torch.randn(M, Kd, generator=g)
    Bm = torch.randn(Kd, N, generator=g)
    ref = (bf(Am) @ bf(Bm)) if compute_bf16 else Am.double() @ Bm.double()
    dtA = torch.bfloat16 if compute_bf16 else torch.float32
    Ast = (Am if a_kmajor else Am.t()).contiguous().to(dtA)
    Bst = (Bm.t() if b_kmajor else Bm).contiguous().to(dtA)
    C = torch.empty(M, N, device=dev)
    K.gemm(Ast.to(dev), Bst.to(dev), M=M, N=N, K=Kd, a_kmajor=a_kmajor, b_kmajor=b_kmajor,
           lda=Kd if a_kmajor else M, ldb=Kd if b_kmajor else N, C=C, compute_bf16=compute_bf16)
    tol = 2e-3 if compute_bf16 else 1e-5
    assert rel(C, ref) < tol


def test_gemm_f32_operand_bf16_compute_with_scale(dev):
    M, N, Kd = 300, 256, 128
    g = torch.Generator().manual_seed(1)
    A = torch.randn(M, Kd, generator=g)
    W = torch.randn(Kd, N, generator=g)  # stored [K][N] -> b_kmajor False (dgrad layout)
    s = torch.rand(Kd, generator=g) + 0.5
    C = torch.empty(M, N, device=dev)
    K.gemm(A.to(dev), W.to(torch.bfloat16).to(dev), M=M, N=N, K=Kd, a_kmajor=True, b_kmajor=False, lda=Kd, ldb=N,
           C=C, a_scale_k=s.to(dev), compute_bf16=True)
    ref = bf(A * s) @ bf(W)
    assert rel(C, ref) < 2e-3


@pytest.mark.parametrize("compute_bf16", [False, True])
def test_gemm_epilogues(dev, compute_bf16):
    M, Cc = 384, 128
    g = torch.Generator().manual_seed(2)
    y = torch.randn(M, Cc, generator=g)
    w1 = torch.randn(4 * Cc, Cc, generator=g) * 0.1
    b1 = torch.randn(4 * Cc, generator=g) * 0.1
    w2 = torch.randn(Cc, 4 * Cc, generator=g) * 0.05
    b2 = torch.randn(Cc, generator=g) * 0.1
    gam = torch.rand(Cc, generator=g) * 0.25 + 0.05
    x = torch.randn(M, Cc, generator=g)
    act = torch.bfloat16 if compute_bf16 else torch.float32
    q = bf if compute_bf16 else (lambda t: t)
    # fc1 + GELU2
    h = torch.empty(M, 4 * Cc, device=dev, dtype=act)
    a = torch.empty_like(h)
    K.linear_fwd(y.to(act).to(dev), w1.to(act).to(dev), out=h, out2=a, bias=b1.to(dev),
                 epilogue=nv.SV_EPI_BIAS_GELU2, compute_bf16=compute_bf16)
    h_ref = q(y) @ q(w1).t() + b1
    tol = 1e-2 if compute_bf16 else 1e-5
    assert rel(h, h_ref) < tol
    assert rel(a, F.gelu(h_ref)) < tol
    # fc1 + GELU dual: C = GELU'(h), C2 = GELU(h)
    gh = torch.empty_like(h)
    a2 = torch.empty_like(h)
    K.linear_fwd(y.to(act).to(dev), w1.to(act).to(dev), out=gh, out2=a2, bias=b1.to(dev),
                 epilogue=nv.SV_EPI_BIAS_GELU_DUAL, compute_bf16=compute_bf16)
    hr = h_ref.clone().requires_grad_(True)
    F.gelu(hr).sum().backward()
    assert rel(a2, F.gelu(h_ref)) < tol
    assert rel(gh, hr.grad) < tol
    # fc1 + GELU, one output (eval forward): the same GELU(h) as the dual epilogue's C2, bit for bit
    a3 = torch.empty_like(h)
    K.linear_fwd(y.to(act).to(dev), w1.to(act).to(dev), out=a3, bias=b1.to(dev), epilogue=nv.SV_EPI_BIAS_GELU,
                 compute_bf16=compute_bf16)
    assert rel(a3, F.gelu(h_ref)) < tol
    assert torch.equal(a3, a2)
    # fc2 + gamma + residual
    out = torch.empty(M, Cc, device=dev)
    K.linear_fwd(a, w2.to(act).to(dev), out=out, bias=b2.to(dev), gamma=gam.to(dev), residual=x.to(dev),
                 epilogue=nv.SV_EPI_BIAS_GAMMA_RES, compute_bf16=compute_bf16)
    a_used = a.float().cpu()
    out_ref = x + gam * (a_used @ q(w2).t() + b2)
    assert rel(out, out_ref) < tol
    # dgrad through fc2 + GELU'
    d = torch.randn(M, Cc, generator=g)
    dh = torch.empty(M, 4 * Cc, device=dev, dtype=act)
    K.linear_dgrad(d.to(dev), w2.to(act).to(dev), out=dh, epilogue=nv.SV_EPI_GELU_GRAD, a_scale_k=gam.to(dev),
                   aux=h, compute_bf16=compute_bf16)
    hh = h.float().cpu().requires_grad_(True)
    F.gelu(hh).backward(q(d * gam) @ q(w2))
    assert rel(dh, hh.grad) < tol
    # the same through the stored GELU' (SV_EPI_MUL_AUX)
    dh2 = torch.empty_like(dh)
    K.linear_dgrad(d.to(dev), w2.to(act).to(dev), out=dh2, epilogue=nv.SV_EPI_MUL_AUX, a_scale_k=gam.to(dev),
                   aux=gh, compute_bf16=compute_bf16)
    assert rel(dh2, (q(d * gam) @ q(w2)) * gh.float().cpu()) < tol
    # wgrad slabs (+ fused bias-gradient column sums)
    cs = torch.zeros(Cc, device=dev)
    G = K.linear_wgrad(d.to(dev), a, bias_out=cs, compute_bf16=compute_bf16)
    G_ref = q(d).t() @ a_used
    assert rel(G, G_ref) < tol
    assert rel(cs, q(d).sum(0)) < tol


@pytest.mark.parametrize("M", [37, 4096, 70000, 65536])
@pytest.mark.parametrize("compute_bf16", [False, True])
@pytest.mark.parametrize("slabs", ["f32", "bf16"])
def test_wgrad_split_and_bias(dev, M, compute_bf16, slabs, monkeypatch):
    """split-K weight gradient + fused bias column sum; ``slabs``: the f32 or the bf16 split-K slabs (the latter
    taken only by the v9 shapes, here M = 65536 / 4096 with the default split)."""
    monkeypatch.setattr(K, "_WGRAD_BF16_SLABS", slabs == "bf16")
    g = torch.Generator().manual_seed(M)
    N, Kd = 256, 512
    dy = torch.randn(M, N, generator=g)
    x = torch.randn(M, Kd, generator=g)
    out = torch.ones(N, Kd, device=dev)
    bias = torch.ones(N, device=dev)
    dt = torch.bfloat16 if compute_bf16 else torch.float32
    q = bf if compute_bf16 else (lambda t: t.double())
    K.linear_wgrad(dy.to(dt).to(dev), x.to(dt).to(dev), out=out, accumulate=True, bias_out=bias,
                   compute_bf16=compute_bf16)
    tol = (4e-3 if slabs == "bf16" else 2e-3) if compute_bf16 else 1e-5
    assert rel(out, q(dy).t() @ q(x) + 1) < tol
    assert rel(bias, q(dy).sum(0) + 1) < (2e-3 if compute_bf16 else 1e-5)


def test_reduce_partials_deep(dev):
    g = torch.Generator().manual_seed(3)
    P, n = 300, 12345 * 4
    part = torch.randn(P, n, generator=g)
    out = torch.zeros(n, device=dev)
    K.reduce_into(part.to(dev).reshape(-1), P, out, accumulate=False)
    assert rel(out, part.double().sum(0)) < 1e-6


# ---------------------------------------------------------------------------------- LayerNorm
@pytest.mark.parametrize("C,rows", [(128, 333), (128, 9001), (192, 333), (192, 9001), (256, 333), (384, 1001),
                                    (512, 333), (512, 9001), (768, 1001), (1024, 333), (1536, 555), (2048, 77)])
def test_layernorm_fwd_bwd(dev, C, rows):
    g = torch.Generator().manual_seed(C + rows)
    x = torch.randn(rows, C, generator=g) * 2 + 0.5
    w = torch.rand(C, generator=g) + 0.5
    b = torch.randn(C, generator=g)
    dy = torch.randn(rows, C, generator=g)
    y, mean, rstd = K.layernorm_fwd(x.to(dev), w.to(dev), b.to(dev), out_dtype=torch.float32)
    xr = x.clone().requires_grad_(True)
    wr = w.clone().requires_grad_(True)
    br = b.clone().requires_grad_(True)
    yr = F.layer_norm(xr, (C,), wr, br, 1e-6)
    yr.backward(dy)
    assert rel(y, yr) < 1e-5
    dw = torch.zeros(C, device=dev)
    db = torch.zeros(C, device=dev)
    dx = K.layernorm_bwd(dy.to(dev), x.to(dev), mean, rstd, w.to(dev), dw=dw, db=db)
    assert rel(dx, xr.grad) < 1e-5
    assert rel(dw, wr.grad) < 1e-5
    assert rel(db, br.grad) < 1e-5


# ------------------------------------------------------------------------------ depthwise conv
@pytest.mark.parametrize("shape", [(2, 16, 16, 128), (1, 13, 11, 64), (3, 4, 4, 256), (2, 2, 2, 192), (2, 32, 32, 512),
                                   (1, 37, 45, 128)])
def test_dwconv7_fwd_bwd(dev, shape):
    B, H, W, C = shape
    g = torch.Generator().manual_seed(B * H * W + C)
    x = torch.randn(B, H, W, C, generator=g)
    w = torch.randn(C, 1, 7, 7, generator=g) * 0.1
    bias = torch.randn(C, generator=g) * 0.1
    lnw = torch.rand(C, generator=g) + 0.5
    lnb = torch.randn(C, generator=g) * 0.1
    dy = torch.randn(B, H, W, C, generator=g)
    z, y, mean, rstd = K.dwconv7_ln_fwd(x.to(dev), w.to(dev), bias.to(dev), lnw.to(dev), lnb.to(dev),
                                        act_dtype=torch.float32)
    xr = x.permute(0, 3, 1, 2).contiguous().requires_grad_(True)
    wr = w.clone().requires_grad_(True)
    br = bias.clone().requires_grad_(True)
    zr = F.conv2d(xr, wr, br, padding=3, groups=C)
    zr_nhwc = zr.permute(0, 2, 3, 1)
    yr = F.layer_norm(zr_nhwc, (C,), lnw, lnb, 1e-6)
    assert rel(z, zr_nhwc) < 1e-5
    assert rel(y.view(B, H, W, C), yr) < 1e-5
    # backward of the conv alone: dz given
    zr_nhwc.backward(dy)
    dx = torch.zeros(B, H, W, C, device=dev)
    dxb = torch.empty(B, H, W, C, device=dev, dtype=torch.bfloat16)
    K.dwconv7_bwd_data(dy.to(dev), w.to(dev), dx, accumulate=True, dx_bf16=dxb)
    assert torch.equal(dxb.cpu(), dx.cpu().to(torch.bfloat16))
    assert rel(dx, xr.grad.permute(0, 2, 3, 1)) < 1e-5
    dw = torch.zeros(C, 49, device=dev)
    db = torch.zeros(C, device=dev)
    K.dwconv7_bwd_weight(dy.to(dev), x.to(dev), dw=dw, db=db)
    assert rel(dw, wr.grad.view(C, 49)) < 1e-5
    assert rel(db, br.grad) < 1e-5


# ------------------------------------------------------------------------ stem / downsample / pool
@pytest.mark.parametrize("C", [128, 192])
def test_stem(dev, C):
    g = torch.Generator().manual_seed(C)
    B, H, W = 2, 32, 24
    img = torch.randn(B, 3, H, W, generator=g)
    w = torch.randn(C, 3, 4, 4, generator=g) * 0.2
    b = torch.randn(C, generator=g) * 0.1
    lnw = torch.rand(C, generator=g) + 0.5
    lnb = torch.randn(C, generator=g) * 0.1
    y, mean, rstd = K.stem_fwd(img.to(dev), w.to(dev), b.to(dev), lnw.to(dev), lnb.to(dev))
    wr, br, lwr, lbr = (t.clone().requires_grad_(True) for t in (w, b, lnw, lnb))
    zr = F.conv2d(img, wr, br, stride=4).permute(0, 2, 3, 1)
    yr = F.layer_norm(zr, (C,), lwr, lbr, 1e-6)
    assert rel(y, yr) < 1e-5
    dy = torch.randn(yr.shape, generator=g)
    yr.backward(dy)
    grads = [torch.zeros_like(t, device=dev) for t in (w, b, lnw, lnb)]
    K.stem_bwd(img.to(dev), w.to(dev), b.to(dev), lnw.to(dev), mean, rstd, dy.to(dev),
               dw=grads[0], db=grads[1], dlnw=grads[2], dlnb=grads[3])
    for got, ref in zip(grads, (wr.grad, br.grad, lwr.grad, lbr.grad)):
        assert rel(got, ref) < 1e-5


def _ref_patches(img):
    """[B,3,H,W] -> [B*(H/4)*(W/4), 64] rows, k = ci*16 + kh*4 + kw (48..63 zero), as f32."""
    B, _, H, W = img.shape
    p = img.view(B, 3, H // 4, 4, W // 4, 4).permute(0, 2, 4, 1, 3, 5).reshape(-1, 48)
    return torch.cat([p, torch.zeros(p.shape[0], 16)], 1)


def test_stem_patchify_and_weight_pack(dev):
    g = torch.Generator().manual_seed(11)
    B, H, W, C = 3, 32, 40, 128
    img = torch.randn(B, 3, H, W, generator=g)
    got = K.stem_patchify(img.to(dev)).cpu()
    assert torch.equal(got, _ref_patches(img).to(torch.bfloat16))  # bitwise: same RNE rounding
    w = torch.randn(C, 3, 4, 4, generator=g)
    wp = K.stem_weight_pack(w.to(dev)).cpu()
    assert torch.equal(wp[:, :48], w.view(C, 48).to(torch.bfloat16)) and not wp[:, 48:].any()


def test_normalize_u8_gray_bitwise(dev):
    """Device transform == the reference's CPU transform (Image.convert("RGB") -> ToTensor -> Normalize,
    localization.py:196-233, 254) bit for bit, and the u8 stem gather == the gather of that tensor."""
    from spine_vision_amd.training.datasets.localization import normalize_u8

    g = torch.Generator().manual_seed(5)
    B, H, W = 2, 64, 48
    u8 = torch.randint(0, 256, (B, H, W), generator=g, dtype=torch.uint8)
    u8[0, 0, :4] = torch.tensor([0, 1, 254, 255], dtype=torch.uint8)
    ref = torch.stack([normalize_u8(u8[i]) for i in range(B)])
    got = K.normalize_u8_gray(u8.to(dev)).cpu()
    assert torch.equal(got, ref)
    assert torch.equal(K.stem_patchify(u8.to(dev)).cpu(), K.stem_patchify(ref.to(dev)).cpu())


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_image_u8_hwc_to_nhwc_bitwise(dev, dtype):
    """Classification device transform: uint8 [B,H,W,3] crops ([T2,T1,T2]) -> ToTensor -> Normalize ->
    NHWC stem operand, bit for bit the host transform (f32) or its RNE bf16 rounding, pad channels 0."""
    from spine_vision_amd.training.datasets.classification import construct_3channel
    from spine_vision_amd.training.datasets.localization import normalize_u8

    g = torch.Generator().manual_seed(6)
    B, H, W = 3, 32, 20
    t2 = torch.randint(0, 256, (B, H, W), generator=g, dtype=torch.uint8)
    t1 = torch.randint(0, 256, (B, H, W), generator=g, dtype=torch.uint8)
    t2[0, 0, :4] = torch.tensor([0, 1, 254, 255], dtype=torch.uint8)
    u8 = torch.stack([construct_3channel(t2[i], t1[i]) for i in range(B)])
    ref = torch.stack([normalize_u8(torch.stack([t2[i], t1[i], t2[i]])) for i in range(B)]).permute(0, 2, 3, 1)
    Cs = 8 if dtype == torch.bfloat16 else 4
    got = K.image_u8_hwc_to_nhwc(u8.to(dev), Cs, dtype).cpu()
    assert got.shape == (B, H, W, Cs)
    assert torch.equal(got[..., :3], ref.to(dtype)) and not got[..., 3:].any()
    # the f32 NCHW route of the same batch gives the same stem operand
    nchw = ref.permute(0, 3, 1, 2).contiguous()
    assert torch.equal(got, K.image_to_nhwc(nchw.to(dev), Cs, dtype).cpu())


def test_stem_mfma_path(dev):
    """bf16 stem = patch gather + v3 GEMM (K 64) + LayerNorm; weight grad = split-K wgrad over 48 of
    the 64 patch columns.  Against torch fp32 conv + LN on the same bf16-rounded operands."""
    g = torch.Generator().manual_seed(3)
    B, H, W, C = 2, 64, 64, 128
    img = torch.randn(B, 3, H, W, generator=g)
    w = torch.randn(C, 3, 4, 4, generator=g) * 0.2
    b = torch.randn(C, generator=g) * 0.1
    patches = K.stem_patchify(img.to(dev))
    z = torch.empty(patches.shape[0], C, device=dev, dtype=torch.bfloat16)
    K.linear_fwd(patches, K.stem_weight_pack(w.to(dev)), out=z, bias=b.to(dev), compute_bf16=True)
    zr = F.conv2d(bf(img), bf(w), b, stride=4).permute(0, 2, 3, 1).reshape(-1, C)
    assert rel(z, zr) < 4e-3
    dz = torch.randn(patches.shape[0], C, generator=g).to(torch.bfloat16)
    dw = torch.zeros(C, 48, device=dev)
    db = torch.zeros(C, device=dev)
    K.linear_wgrad(dz.to(dev), patches, out=dw, accumulate=True, bias_out=db, compute_bf16=True, cols=48)
    ref_w = dz.float().t() @ _ref_patches(bf(img))[:, :48]
    assert rel(dw, ref_w) < 2e-3
    assert rel(db, dz.float().sum(0)) < 1e-4


@pytest.mark.parametrize("C,B,H,W", [(128, 2, 8, 6), (256, 2, 8, 6), (128, 2, 128, 128), (256, 6, 64, 64)])
def test_downsample(dev, C, B, H, W):
    """Small shapes, and shapes with more patches than the launch has waves (B*H*W/4 > 4096), where each wave
    walks several patches with the next one's loads in flight (C <= 256)."""
    g = torch.Generator().manual_seed(C + 1)
    x = torch.randn(B, H, W, C, generator=g)
    lnw = torch.rand(C, generator=g) + 0.5
    lnb = torch.randn(C, generator=g) * 0.1
    wc = torch.randn(2 * C, C, 2, 2, generator=g) * 0.05
    bc = torch.randn(2 * C, generator=g) * 0.1
    patches, mean, rstd = K.downsample_fwd(x.to(dev), lnw.to(dev), lnb.to(dev), act_dtype=torch.float32)
    out = torch.empty(B * (H // 2) * (W // 2), 2 * C, device=dev)
    K.linear_fwd(patches, wc.reshape(2 * C, 4 * C).to(dev), out=out, bias=bc.to(dev), compute_bf16=False)
    xr = x.clone().requires_grad_(True)
    lwr, lbr = lnw.clone().requires_grad_(True), lnb.clone().requires_grad_(True)
    n = F.layer_norm(xr, (C,), lwr, lbr, 1e-6).permute(0, 3, 1, 2)
    o = F.conv2d(n, wc, bc, stride=2).permute(0, 2, 3, 1)
    assert rel(out.view(o.shape), o) < 1e-5
    dpatch = torch.randn(patches.shape, generator=g)
    # autograd of the LN+gather alone: reconstruct patches from n and backprop dpatch
    Ho, Wo = H // 2, W // 2
    pr = n.reshape(B, C, Ho, 2, Wo, 2).permute(0, 2, 4, 1, 3, 5).reshape(B * Ho * Wo, 4 * C)
    assert rel(patches, pr) < 1e-5
    pr.backward(dpatch)
    dlnw = torch.zeros(C, device=dev)
    dlnb = torch.zeros(C, device=dev)
    dx, dxb = K.downsample_bwd(dpatch.to(dev), x.to(dev), mean, rstd, lnw.to(dev), dlnw=dlnw, dlnb=dlnb,
                               with_bf16=True)
    assert torch.equal(dxb.cpu(), dx.cpu().to(torch.bfloat16))
    assert rel(dx, xr.grad) < 1e-5
    assert rel(dlnw, lwr.grad) < 1e-5
    assert rel(dlnb, lbr.grad) < 1e-5


def test_scale_rows_bf16(dev):
    g = torch.Generator().manual_seed(11)
    W = torch.randn(96, 200, generator=g)
    sc = torch.rand(96, generator=g)
    out = K.scale_rows_bf16(W.to(dev), sc.to(dev))
    assert torch.equal(out.cpu(), (W * sc[:, None]).to(torch.bfloat16))


@pytest.mark.parametrize("shape", [(3, 4, 5, 1024), (2, 16, 16, 512)])
def test_pool_ln(dev, shape):
    g = torch.Generator().manual_seed(5)
    B, H, W, C = shape
    x = torch.randn(B, H, W, C, generator=g)
    lnw = torch.rand(C, generator=g) + 0.5
    lnb = torch.randn(C, generator=g) * 0.1
    feat, pooled, mean, rstd = K.pool_ln_fwd(x.to(dev), lnw.to(dev), lnb.to(dev))
    xr = x.clone().requires_grad_(True)
    lwr, lbr = lnw.clone().requires_grad_(True), lnb.clone().requires_grad_(True)
    fr = F.layer_norm(xr.mean((1, 2)), (C,), lwr, lbr, 1e-6)
    assert rel(feat, fr) < 1e-5
    df = torch.randn(B, C, generator=g)
    fr.backward(df)
    dlnw = torch.zeros(C, device=dev)
    dlnb = torch.zeros(C, device=dev)
    dx, dxb = K.pool_ln_bwd(df.to(dev), pooled, mean, rstd, lnw.to(dev), (B, H, W, C), dlnw=dlnw, dlnb=dlnb,
                            with_bf16=True)
    assert torch.equal(dxb.cpu(), dx.cpu().to(torch.bfloat16))
    assert rel(dx, xr.grad) < 1e-5
    assert rel(dlnw, lwr.grad) < 1e-5
    assert rel(dlnb, lbr.grad) < 1e-5


# ----------------------------------------------------------------------------------- optimizer
def test_adamw_and_clip(dev):
    from oracle.step import adamw_reference

    g = torch.Generator().manual_seed(9)
    n = 100_003
    p = torch.randn(n, generator=g)
    gr = torch.randn(n, generator=g) * 3
    m = torch.randn(n, generator=g) * 0.1
    v = torch.rand(n, generator=g) * 0.1
    out = K.grad_clip_coef(gr.to(dev), 1.0)
    norm = gr.double().norm().item()
    assert abs(out[0].item() - norm) / norm < 1e-5
    coef = min(1.0, 1.0 / (norm + 1e-6))
    assert abs(out[1].item() - coef) / coef < 1e-5
    pd, md, vd = p.to(dev), m.to(dev), v.to(dev)
    pb = torch.empty(n, device=dev, dtype=torch.bfloat16)
    K.adamw_flat(pd, gr.to(dev), md, vd, pb, lr=1e-3, beta1=0.9, beta2=0.999, eps=1e-8, weight_decay=1e-2, step=3,
                 grad_scale=out[1:2])
    pr, mr, vr = adamw_reference(p.double(), gr.double() * coef, m.double(), v.double(), lr=1e-3, beta1=0.9,
                                 beta2=0.999, eps=1e-8, weight_decay=1e-2, step=3)
    assert maxrel(pd, pr) < 1e-5
    assert maxrel(md, mr) < 1e-5
    assert maxrel(vd, vr) < 1e-5
    assert torch.equal(pb.cpu(), pd.cpu().to(torch.bfloat16))


# ------------------------------------------------- bf16 gradient paths (bf16 mode: dy, dz in bf16)
@pytest.mark.parametrize("C", [128, 512, 768])
@pytest.mark.parametrize("dy_f32", [False, True])
def test_layernorm_bwd_bf16_io(dev, C, dy_f32):
    g = torch.Generator().manual_seed(C + 1)
    x = (torch.randn(333, C, generator=g) * 2 + 0.5).to(torch.bfloat16)
    w = torch.rand(C, generator=g) + 0.5
    dy = torch.randn(333, C, generator=g)
    if not dy_f32:  # (f32, bf16, bf16) is the stem's combination: f32 gradient stream, bf16 saved input
        dy = dy.to(torch.bfloat16)
    xr = x.double().requires_grad_(True)
    wr = w.double().requires_grad_(True)
    yr = F.layer_norm(xr, (C,), wr, None, 1e-6)
    yr.backward(dy.double())
    xd = x.to(dev)
    _, mean, rstd = K.layernorm_fwd(xd, w.to(dev), torch.zeros(C, device=dev), out_dtype=torch.float32)
    dw = torch.zeros(C, device=dev)
    db = torch.zeros(C, device=dev)
    dx = K.layernorm_bwd(dy.to(dev), xd, mean, rstd, w.to(dev), dw=dw, db=db, out_dtype=torch.bfloat16)
    assert dx.dtype == torch.bfloat16
    assert rel(dx, xr.grad) < 8e-3  # output rounded to bf16
    assert rel(dw, wr.grad) < 1e-5
    assert rel(db, dy.double().sum(0)) < 1e-5


@pytest.mark.parametrize("shape", [(2, 16, 16, 128), (1, 13, 11, 64), (1, 37, 45, 256), (2, 9, 7, 192)])
def test_dwconv7_fwd_bf16_io(dev, shape):
    """bf16 input / bf16 output forward (the bf16 step's x is f32, the lean paths feed bf16); C % 128 == 0
    runs the two-channels-per-lane kernel, 64 / 192 the one-channel kernel."""
    B, H, W, C = shape
    g = torch.Generator().manual_seed(B * H * W + C + 11)
    x = torch.randn(B, H, W, C, generator=g).to(torch.bfloat16)
    w = torch.randn(C, 1, 7, 7, generator=g) * 0.1
    bias = torch.randn(C, generator=g) * 0.1
    ones, zeros = torch.ones(C), torch.zeros(C)
    z, _, _, _ = K.dwconv7_ln_fwd(x.to(dev), w.to(dev), bias.to(dev), ones.to(dev), zeros.to(dev),
                                  act_dtype=torch.bfloat16)
    zr = F.conv2d(x.permute(0, 3, 1, 2).double(), w.double(), bias.double(), padding=3, groups=C)
    assert z.dtype == torch.bfloat16
    assert rel(z.view(B, H, W, C), zr.permute(0, 2, 3, 1)) < 8e-3  # output rounded to bf16


@pytest.mark.parametrize("shape", [(2, 16, 16, 128), (1, 13, 11, 64), (1, 37, 45, 256)])
def test_dwconv7_bwd_bf16_dz(dev, shape, monkeypatch):
    """The VALU kernels (f32 taps); the matrix-core backward-data (bf16 taps) is pinned by test_dw_mfma_gpu.py."""
    monkeypatch.setattr(K, "DW_MFMA", False)
    B, H, W, C = shape
    g = torch.Generator().manual_seed(B * H * W + C + 7)
    x = torch.randn(B, H, W, C, generator=g)
    w = torch.randn(C, 1, 7, 7, generator=g) * 0.1
    dz = torch.randn(B, H, W, C, generator=g).to(torch.bfloat16)
    xr = x.permute(0, 3, 1, 2).double().requires_grad_(True)
    wr = w.double().requires_grad_(True)
    zr = F.conv2d(xr, wr, None, padding=3, groups=C)
    zr.permute(0, 2, 3, 1).backward(dz.double())
    base = torch.randn(B, H, W, C, generator=g)
    dx = base.clone().to(dev)
    K.dwconv7_bwd_data(dz.to(dev), w.to(dev), dx, accumulate=True)
    assert rel(dx - base.to(dev), xr.grad.permute(0, 2, 3, 1)) < 1e-5
    dw = torch.zeros(C, 49, device=dev)
    db = torch.zeros(C, device=dev)
    K.dwconv7_bwd_weight(dz.to(dev), x.to(dev), dw=dw, db=db)
    assert rel(dw, wr.grad.view(C, 49)) < 1e-5
    assert rel(db, dz.double().sum((0, 1, 2))) < 1e-5


# ------------------------------------------------- fc2 wgrad + layer-scale finish (fused reduce)
@pytest.mark.parametrize("M,C,compute_bf16", [(4096, 128, True), (2048, 192, False), (1024, 512, True)])
@pytest.mark.parametrize("slabs", ["f32", "bf16"])
def test_layerscale_wgrad_fused(dev, M, C, compute_bf16, slabs, monkeypatch):
    """fc2 weight gradient + layer-scale finish against float64 on the same operands: f32 split-K slabs within f32
    accumulation (1e-4); bf16 slabs (each slice's partial rounded to bf16 once) within bf16 rounding (4e-3)."""
    monkeypatch.setattr(K, "_WGRAD_BF16_SLABS", slabs == "bf16")
    g = torch.Generator().manual_seed(M + C)
    d = torch.randn(M, C, generator=g)
    a = torch.randn(M, 4 * C, generator=g)
    w2 = torch.randn(C, 4 * C, generator=g) * 0.05
    gam = torch.rand(C, generator=g) + 0.1
    b2 = torch.randn(C, generator=g) * 0.1
    base = [torch.randn(C, 4 * C, generator=g), torch.randn(C, generator=g), torch.randn(C, generator=g)]
    dt_ = torch.bfloat16 if compute_bf16 else torch.float32
    dq, aq = d.to(dt_), a.to(dt_)
    G = dq.double().t() @ aq.double()
    cs = dq.double().sum(0)
    ref_w = base[0].double() + gam.double()[:, None] * G
    ref_g = base[1].double() + (w2.double() * G).sum(1) + b2.double() * cs
    ref_b = base[2].double() + gam.double() * cs
    dw2, dgam, db2 = (t.clone().to(dev) for t in base)
    K.layerscale_wgrad(dq.to(dev), aq.to(dev), w2.to(dev), gam.to(dev), b2.to(dev), dw2=dw2, dgamma=dgam, db2=db2,
                       compute_bf16=compute_bf16)
    tol = (4e-3 if slabs == "bf16" else 1e-4) if compute_bf16 else 1e-5
    assert rel(dw2, ref_w) < tol
    assert rel(dgam, ref_g) < tol
    assert rel(db2, ref_b) < (1e-4 if compute_bf16 else 1e-5)  # the bias gradient: f32 column sums either way


@pytest.mark.parametrize("case", ["dual", "gelu", "residual"])
def test_gemm_v8_dispatch_shapes(dev, case):
    """Shapes large enough (>= 256 tiles of 256x256) that sv_gemm dispatches the v8 kernel by default:
    the fc1 GELU-dual epilogue and the long-K (>= 2048) residual epilogue.  Checked on 512 sampled rows
    against a torch fp32 reference on the same bf16 operands."""
    g = torch.Generator().manual_seed(8 if case == "dual" else 9)
    if case in ("dual", "gelu"):
        M, N, Kd = 16384, 4096, 256
    else:
        M, N, Kd = 65536, 256, 2048
    A = (torch.randn(M, Kd, generator=g) * 0.5).to(torch.bfloat16)
    W = (torch.randn(N, Kd, generator=g) * 0.05).to(torch.bfloat16)
    b = torch.randn(N, generator=g) * 0.1
    rows = torch.randperm(M, generator=g)[:512]
    ref = A[rows].float() @ W.float().t() + b
    Ad, Wd = A.to(dev), W.to(dev)
    if case == "dual":
        gh = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        a = torch.empty_like(gh)
        K.linear_fwd(Ad, Wd, out=gh, out2=a, bias=b.to(dev), epilogue=nv.SV_EPI_BIAS_GELU_DUAL)
        hr = ref.clone().requires_grad_(True)
        F.gelu(hr).sum().backward()
        assert rel(a[rows.to(dev)], F.gelu(ref)) < 1e-2
        assert rel(gh[rows.to(dev)], hr.grad) < 1e-2
    elif case == "gelu":
        a = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        K.linear_fwd(Ad, Wd, out=a, bias=b.to(dev), epilogue=nv.SV_EPI_BIAS_GELU)
        assert rel(a[rows.to(dev)], F.gelu(ref)) < 1e-2
    else:
        gam = torch.rand(N, generator=g) * 0.25 + 0.05
        x = torch.randn(M, N, generator=g)
        out = torch.empty(M, N, device=dev)
        K.linear_fwd(Ad, Wd, out=out, bias=b.to(dev), gamma=gam.to(dev), residual=x.to(dev),
                     epilogue=nv.SV_EPI_BIAS_GAMMA_RES)
        assert rel(out[rows.to(dev)], x[rows] + gam * ref) < 1e-5 + 2e-3


def test_reduce_multi_matches_pair_and_torch(dev):
    """sv_reduce_partials_multi (one launch for a block's weight-gradient folds): a wide split-K slab is
    summed in reduce_partials' order (bitwise equal to reduce_into), deep narrow partials (LayerNorm /
    depthwise shapes, ragged n) within f32 rounding of a float64 sum; accumulate honoured per segment."""
    g = torch.Generator().manual_seed(11)
    shapes = [(16, 2048 * 512, True), (16, 512, True), (300, 1024, True), (64, 512 * 49, True), (64, 510, False),
              (7, 70000, False)]
    parts = [torch.randn(P, n, generator=g).to(dev) for P, n, _ in shapes]
    outs = [torch.randn(n, generator=g).to(dev) for _, n, _ in shapes]
    ref_outs = [o.clone() for o in outs]
    K.reduce_multi([(p, o, P, acc) for p, o, (P, _, acc) in zip(parts, outs, shapes)])
    torch.cuda.synchronize()
    # the wide slab: bitwise what the pair path computes
    pair = ref_outs[0].clone()
    K.reduce_into(parts[0], 16, pair, accumulate=True)
    torch.cuda.synchronize()
    assert torch.equal(outs[0], pair)
    for p, o, r, (P, n, acc) in zip(parts, outs, ref_outs, shapes):
        ref = p.double().sum(0) + (r.double() if acc else 0)
        err = float((o.double() - ref).abs().max() / (ref.abs().max() + 1e-30))
        assert err < 1e-5, (P, n, acc, err)


def test_device_context(dev):
    """sv_ctx: one reference-counted context per device holding what the launches are sized
    by -- the CU count the persistent grids use, the LDS limit, the kernels whose LDS limit was raised there."""
    from spine_vision_amd import native as nv

    a, b = nv.DeviceContext(dev.index or 0), nv.DeviceContext(dev.index or 0)
    try:
        assert a.handle == b.handle != 0
        i = a.info()
        props = torch.cuda.get_device_properties(dev)
        assert i.device == (dev.index or 0) and i.compute_units == props.multi_processor_count
        assert i.lds_bytes_per_wg >= 65536 and i.arch.decode().startswith("gfx950") and i.refs >= 2
        x = torch.randn(4096, 512, device=dev).to(torch.bfloat16)
        w = torch.randn(2048, 512, device=dev).to(torch.bfloat16)
        K.linear_fwd(x, w, out=torch.empty(4096, 2048, device=dev, dtype=torch.bfloat16))  # a 160 KiB-LDS v9 launch
        torch.cuda.synchronize()
        assert a.info().lds_raised_kernels >= 1
    finally:
        a.close()
        b.close()
    assert nv.device_context(dev.index or 0).info().refs >= 1  # the process's own context stays
