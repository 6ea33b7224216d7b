"""One launch per BatchNorm where the rows are few (sv_bn_bwd_small / sv_bn_act_small; kernels.bn_small_ok: ResNet
layers 3-4 at 256 px, rows <= 8192) against the multi-launch path it replaces (statistics partials, their fold, the
apply / activation), BIT FOR BIT: every sum is taken in that path's order, so the data gradients, the gamma / beta
gradients, the masked gradient written in place, mean / rstd, the running statistics and the activations must be
equal, not close.  Then a whole ResNet-50 train step with the one-launch forms on and off.

Reference: timm ResNet's BatchNorm2d forward / autograd backward (spine_vision/training/models/backbone.py:166);
the multi-launch path is itself pinned against torch in tests/test_resnet_gpu.py."""

import contextlib

import pytest
import torch

from spine_vision_amd import kernels as K
from spine_vision_amd.backbone import create_resnet

pytestmark = pytest.mark.gpu
BF = torch.bfloat16

# ResNet-50 @256 bs32: layer3 (8192 rows: C 256 inner, 1024 out), layer4 (2048 rows: 512 / 2048); ragged row counts;
# layer1 at a small batch (the 4-channel-per-lane geometry limit C = 64)
SHAPES = [(8192, 256), (8192, 1024), (2048, 512), (2048, 2048), (6000, 256), (520, 64), (4096, 64)]


@contextlib.contextmanager
def multi_launch():
    old = K._BN_SMALL
    K._BN_SMALL = False
    try:
        yield
    finally:
        K._BN_SMALL = old


def _bn_inputs(rows, C, seed, dev):
    g = torch.Generator().manual_seed(seed)
    y = (torch.randn(rows, C, generator=g) * 1.3 + 0.2).to(dev, BF)
    gam = (torch.rand(C, generator=g) + 0.5).to(dev)
    bet = (torch.randn(C, generator=g) * 0.3).to(dev)
    mean, rstd = K.bn_stats(y)
    return g, y, gam, bet, mean, rstd


def _grads(C, dev, seed, n=2):
    g = torch.Generator().manual_seed(seed)
    return [torch.randn(C, generator=g).to(dev) for _ in range(n)]  # accumulated onto non-zero gradients


def _eq(*pairs):
    for i, (a, b) in enumerate(pairs):
        assert torch.equal(a, b), (i, float((a.float() - b.float()).abs().max()))


@pytest.fixture(autouse=True)
def one_launch_on():
    """The one-launch forms are opt-in (measured slower in the step, kernels.py); these tests turn them on."""
    old = K._BN_SMALL
    K._BN_SMALL = True
    yield
    K._BN_SMALL = old


def test_small_geometry_covers_resnet50_layers_3_4():
    """The bench configuration's layer3 / layer4 BatchNorms fit the one-launch geometry, layer1 / 2 do not."""
    for rows, C in [(8192, 256), (8192, 1024), (2048, 512), (2048, 2048)]:
        assert K.bn_small_ok(rows, C)
    for rows, C in [(131072, 64), (131072, 256), (32768, 128), (32768, 512), (9000, 256)]:
        assert not K.bn_small_ok(rows, C)


@pytest.mark.parametrize("rows,C", SHAPES)
@pytest.mark.parametrize("batch_stats", [True, False])
def test_bwd_small_mask_inplace_bitwise(dev, rows, C, batch_stats):
    """A block-output BatchNorm (f32 gradient, ReLU mask from the saved activation, masked gradient written over
    dout): sv_bn_bwd_small mode MASK == sv_bn_bwd_stats_mask + sv_bn_bwd_finish + sv_bn_bwd_apply."""
    assert K.bn_small_ok(rows, C)
    g, y, gam, bet, mean, rstd = _bn_inputs(rows, C, rows + C, dev)
    act = K.bn_act(y, mean, rstd, gam, bet, relu=True, out_dtype=BF)
    dout = torch.randn(rows, C, generator=g).to(dev)
    dg1, db1 = _grads(C, dev, 1)
    dg2, db2 = dg1.clone(), db1.clone()
    d1 = dout.clone()
    dx1 = K.bn_bwd(d1, y, mean, rstd, gam, act=act, dgamma=dg1, dbeta=db1, dx_dtype=BF, mask_inplace=True,
                   batch_stats=batch_stats)
    with multi_launch():
        d2 = dout.clone()
        dx2 = K.bn_bwd(d2, y, mean, rstd, gam, act=act, dgamma=dg2, dbeta=db2, dx_dtype=BF, mask_inplace=True,
                       batch_stats=batch_stats)
    torch.cuda.synchronize()
    _eq((dx1, dx2), (d1, d2), (dg1, dg2), (db1, db2))
    assert torch.equal(d1, dout * (act > 0).float())


@pytest.mark.parametrize("rows,C", SHAPES)
@pytest.mark.parametrize("given", [False, True])
def test_bwd_small_relu_bitwise(dev, rows, C, given):
    """An inner BatchNorm + its own ReLU (bf16 gradient, mask recomputed from y): sv_bn_bwd_small mode RELU ==
    sv_bn_relu_bwd_stats + finish + sv_bn_relu_bwd_apply; ``given``: the statistics partials handed over by the
    data gradient's producer (sv_conv_bwd_data_bn: [ceil(rows/64)][2][C]), only folded."""
    g, y, gam, bet, mean, rstd = _bn_inputs(rows, C, 3 * rows + C, dev)
    da = torch.randn(rows, C, generator=g).to(dev, BF)
    part = torch.randn((rows + 63) // 64, 2, C, generator=g).to(dev) if given else None
    dg1, db1 = _grads(C, dev, 2)
    dg2, db2 = dg1.clone(), db1.clone()
    dx1 = K.bn_bwd(da, y, mean, rstd, gam, relu_beta=bet, dgamma=dg1, dbeta=db1, dx_dtype=BF, part=part)
    with multi_launch():
        dx2 = K.bn_bwd(da, y, mean, rstd, gam, relu_beta=bet, dgamma=dg2, dbeta=db2, dx_dtype=BF, part=part)
    torch.cuda.synchronize()
    _eq((dx1, dx2), (dg1, dg2), (db1, db2))


@pytest.mark.parametrize("rows,C", [(8192, 1024), (2048, 2048), (6000, 256), (520, 64)])
@pytest.mark.parametrize("dx_dtype", [BF, torch.float32])
def test_bwd_small_dual_bitwise(dev, rows, C, dx_dtype):
    """A projection-shortcut block's two output BatchNorms from one masked gradient: sv_bn_bwd_small mode DUAL ==
    sv_bn_bwd_stats_mask_dual + two finishes + sv_bn_bwd_apply_dual."""
    g, y, gam, bet, m1, r1 = _bn_inputs(rows, C, 5 * rows + C, dev)
    yd = (torch.randn(rows, C, generator=g) * 1.5 - 0.2).to(dev, BF)
    gd, bd = (torch.rand(C, generator=g) + 0.5).to(dev), (torch.randn(C, generator=g) * 0.3).to(dev)
    m2, r2 = K.bn_stats(yd)
    out = K.bn_act(y, m1, r1, gam, bet, res=yd, res_bn=(m2, r2, gd, bd), relu=True, out_dtype=BF)
    d0 = torch.randn(rows, C, generator=g).to(dev)
    ga = _grads(C, dev, 3, 4)
    gb = [t.clone() for t in ga]
    d1 = d0.clone()
    x1, x2 = K.bn_bwd_dual(d1, y, m1, r1, gam, out, yd, m2, r2, gd, dgamma=ga[0], dbeta=ga[1], dgamma2=ga[2],
                           dbeta2=ga[3], dx_dtype=dx_dtype)
    with multi_launch():
        d2 = d0.clone()
        e1, e2 = K.bn_bwd_dual(d2, y, m1, r1, gam, out, yd, m2, r2, gd, dgamma=gb[0], dbeta=gb[1], dgamma2=gb[2],
                               dbeta2=gb[3], dx_dtype=dx_dtype)
    torch.cuda.synchronize()
    _eq((d1, d2), (x1, e1), (x2, e2), *zip(ga, gb))


def _partials(y: torch.Tensor) -> torch.Tensor:
    """Unshifted per-64-row column sums / sums of squares of y, [ceil(rows/64)][2][C] (the conv epilogue's
    SV_EPI_STORE_STATS layout)."""
    rows, C = y.shape
    P = (rows + 63) // 64
    yf = torch.zeros(P * 64, C, device=y.device)
    yf[:rows] = y.float()
    yf = yf.view(P, 64, C)
    return torch.stack([yf.sum(1), (yf * yf).sum(1)], 1).contiguous()


def _bn_state(C, dev, seed):
    g = torch.Generator().manual_seed(seed)
    gam = (torch.rand(C, generator=g) + 0.5).to(dev)
    bet = (torch.randn(C, generator=g) * 0.3).to(dev)
    rm = (torch.randn(C, generator=g) * 0.1).to(dev)
    rv = (torch.rand(C, generator=g) + 0.5).to(dev)
    nbt = torch.tensor(7, device=dev, dtype=torch.int64)
    return gam, bet, rm, rv, nbt


@pytest.mark.parametrize("rows,C", SHAPES)
@pytest.mark.parametrize("res", ["none", "identity", "bn"])
def test_act_small_bitwise(dev, rows, C, res):
    """sv_bn_act_small == sv_bn_stats_finish (y = NULL, the conv epilogue's partials) + sv_bn_act_fwd: mean, rstd,
    running mean / var, num_batches_tracked and the activation, with no residual, the identity shortcut and the
    projection shortcut's BatchNorm (its statistics folded in the same launch)."""
    g = torch.Generator().manual_seed(7 * rows + C)
    y = (torch.randn(rows, C, generator=g) * 1.1 + 0.3).to(dev, BF)
    part = _partials(y)
    st1 = _bn_state(C, dev, 1)
    st2 = tuple(t.clone() for t in st1)
    x = yd = pd = None
    if res == "identity":
        x = torch.randn(rows, C, generator=g).to(dev, BF)
    elif res == "bn":
        yd = (torch.randn(rows, C, generator=g) * 0.7 - 0.1).to(dev, BF)
        pd = _partials(yd)
        sd1 = _bn_state(C, dev, 2)
        sd2 = tuple(t.clone() for t in sd1)
    gam, bet, rm, rv, nbt = st1
    prm = (gam, bet, 1e-5, 0.1, rm, rv, nbt)
    if res == "bn":
        out1, m1, r1, md1, rd1 = K.bn_act_small(y, part, prm, res=yd, res_part=pd,
                                                res_params=(sd1[0], sd1[1], 1e-5, 0.1, sd1[2], sd1[3], sd1[4]),
                                                relu=True, out_dtype=BF)
    else:
        out1, m1, r1 = K.bn_act_small(y, part, prm, res=x, relu=True, out_dtype=BF)
    gam2, bet2, rm2, rv2, nbt2 = st2
    m2, r2 = K.bn_stats_from_partials(part, rows, eps=1e-5, momentum=0.1, running_mean=rm2, running_var=rv2,
                                      num_batches_tracked=nbt2)
    if res == "bn":
        md2, rd2 = K.bn_stats_from_partials(pd, rows, eps=1e-5, momentum=0.1, running_mean=sd2[2], running_var=sd2[3],
                                            num_batches_tracked=sd2[4])
        out2 = K.bn_act(y, m2, r2, gam2, bet2, res=yd, res_bn=(md2, rd2, sd2[0], sd2[1]), relu=True, out_dtype=BF)
    else:
        out2 = K.bn_act(y, m2, r2, gam2, bet2, res=x, relu=True, out_dtype=BF)
    torch.cuda.synchronize()
    _eq((out1, out2), (m1, m2), (r1, r2), (rm, rm2), (rv, rv2), (nbt, nbt2))
    if res == "bn":
        _eq((md1, md2), (rd1, rd2), *zip(sd1[2:], sd2[2:]))


@pytest.mark.timeout(600)
def test_resnet50_step_small_bn_bitwise(dev):
    """A whole ResNet-50 bf16 train forward + backward at B=4, 128 px (layers 1-4 all within the one-launch
    geometry there) with the one-launch BatchNorms on and off: features, every parameter gradient and every
    BatchNorm buffer bit for bit."""
    torch.manual_seed(0)
    a = create_resnet("resnet50", precision="bf16").to(dev)
    b = create_resnet("resnet50", precision="bf16").to(dev)
    b.load_state_dict(a.state_dict())
    x = torch.rand(4, 3, 128, 128, generator=torch.Generator().manual_seed(1)).to(dev)
    out = {}
    old = K._BN_SMALL
    try:
        for name, m, flag in (("small", a, True), ("multi", b, False)):
            K._BN_SMALL = flag
            m.train()
            for _ in range(2):  # the second pass replays the captured forward
                m.zero_grad(set_to_none=True)
                f = m(x)
                f.backward(torch.linspace(-1, 1, f.numel(), device=dev).view_as(f))
            torch.cuda.synchronize()
            out[name] = f.detach().clone()
    finally:
        K._BN_SMALL = old
    assert torch.equal(out["small"], out["multi"])
    for (n, p), (_, q) in zip(a.named_parameters(), b.named_parameters()):
        assert torch.equal(p.grad, q.grad), n
    for (n, p), (_, q) in zip(a.named_buffers(), b.named_buffers()):
        assert torch.equal(p, q), n
