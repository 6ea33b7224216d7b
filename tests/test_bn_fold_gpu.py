"""The BatchNorm statistics fold inside the consuming pass (sv_bn_act_fold / sv_bn_bwd_apply_fold) against the
separate fold launch (sv_bn_stats_finish / sv_bn_bwd_finish + the apply pass, SV_BN_FOLD=0): bit for bit, at the
ResNet-50 bs32 256^2 shapes (the stem's 8192 partials take 8 chunks, layer 1's 2048 two), across repeated launches
(the counters re-arm) and under graph capture and replay."""
import pytest
import torch

from spine_vision_amd import kernels as K

pytestmark = pytest.mark.gpu

# rows, C: the stem (B32 x 128^2), layer 1 (B32 x 64^2) at 64 / 256 channels, layers 2-4, and a small C = 32
ACT_SHAPES = [(524288, 64), (131072, 64), (131072, 256), (32768, 512), (8192, 1024), (2048, 2048), (4160, 32)]


def _partials(y):
    """unshifted per-64-row partials [ceil(rows/64)][2][C] of y (what the conv epilogue writes)"""
    rows, C = y.shape
    P = (rows + 63) // 64
    yf = torch.zeros(P * 64, C, device=y.device)
    yf[:rows] = y.float()
    yf = yf.view(P, 64, C)
    return torch.stack([yf.sum(1), (yf * yf).sum(1)], 1).contiguous()


def _params(C, g, dev):
    return ((torch.rand(C, generator=g) + 0.5).to(dev), (torch.randn(C, generator=g) * 0.3).to(dev), 1e-5, 0.1,
            torch.randn(C, generator=g).to(dev), (torch.rand(C, generator=g) + 0.5).to(dev),
            torch.zeros((), dtype=torch.int64, device=dev))


def _clone_params(p):
    return p[:4] + tuple(t.clone() for t in p[4:])


@pytest.mark.parametrize("form", ["plain", "identity", "projection"])
@pytest.mark.parametrize("rows,C", ACT_SHAPES, ids=lambda v: str(v))
def test_act_fold_matches_separate(dev, rows, C, form):
    g = torch.Generator().manual_seed(rows + C)
    y = (torch.randn(rows, C, generator=g) * 2 + 0.5).to(dev, torch.bfloat16)
    part = _partials(y)
    assert bool(K.value("sv_bn_fold_ok", rows, C, part.shape[0]))
    pa = _params(C, g, dev)
    res = res_part = pr = None
    if form != "plain":
        res = (torch.randn(rows, C, generator=g) - 0.3).to(dev, torch.bfloat16)
    if form == "projection":
        res_part = _partials(res)
        pr = _params(C, g, dev)
    outs = []
    for fold in (True, False, True):  # the second fold launch reuses the re-armed counters
        p1 = _clone_params(pa)
        p2 = _clone_params(pr) if pr is not None else None
        if fold:
            r = K.bn_act_fold(y, part, p1, res=res, res_part=res_part, res_params=p2, relu=True,
                              out_dtype=torch.bfloat16)
        else:
            with pytest.MonkeyPatch.context() as mp:
                mp.setattr(K, "_BN_FOLD", False)
                mp.setattr(K, "_BN_SMALL", False)
                r = K.bn_act_partials(y, part, p1, res=res, res_part=res_part, res_params=p2, relu=True,
                                      out_dtype=torch.bfloat16)
        outs.append(list(r) + list(p1[4:]) + (list(p2[4:]) if p2 is not None else []))
    torch.cuda.synchronize()
    for a, b in zip(outs[0], outs[1]):
        assert torch.equal(a, b)
    for a, b in zip(outs[0], outs[2]):
        assert torch.equal(a, b)
    ctl, _ = K._fold_ws(y.device)
    assert int(ctl[:4].abs().sum()) == 0 and int(ctl[16:].abs().sum()) == 0, ctl[:8]
    # and the statistics against float64
    m64 = y.double().mean(0)
    assert float((outs[0][1].double() - m64).abs().max()) < 1e-4 * (1 + float(m64.abs().max()))


BWD_SHAPES = [(131072, 64), (131072, 256), (32768, 128), (8192, 512), (2048, 2048)]


def _bwd_case(rows, C, g, dev):
    y = torch.randn(rows, C, generator=g).to(dev, torch.bfloat16)
    gam = (torch.rand(C, generator=g) + 0.5).to(dev)
    bet = (torch.randn(C, generator=g) * 0.3).to(dev)
    mean, rstd = K.bn_stats(y)
    a = K.bn_act(y, mean, rstd, gam, bet, relu=True, out_dtype=torch.bfloat16)
    d = torch.randn(rows, C, generator=g).to(dev, torch.bfloat16)
    return y, gam, bet, mean, rstd, a, d


def _both(fn):
    """fn() with the fold kernels, without, and with again -> three result lists"""
    out = []
    for fold in (True, False, True):
        with pytest.MonkeyPatch.context() as mp:
            mp.setattr(K, "_BN_FOLD", fold)
            mp.setattr(K, "_BN_SMALL", False)
            out.append(fn())
    torch.cuda.synchronize()
    return out


def _assert_same(out):
    for k in (1, 2):
        for a, b in zip(out[0], out[k]):
            assert torch.equal(a, b)


@pytest.mark.parametrize("mode", ["mask", "relu", "relu_given", "eval"])
@pytest.mark.parametrize("rows,C", BWD_SHAPES, ids=lambda v: str(v))
def test_bwd_apply_fold_matches_separate(dev, rows, C, mode):
    g = torch.Generator().manual_seed(rows * 3 + C)
    y, gam, bet, mean, rstd, a, d = _bwd_case(rows, C, g, dev)
    given = None
    if mode == "relu_given":  # partials as a producer hands them over (any fixed values fold the same way)
        given = torch.randn((rows + 63) // 64, 2, C, generator=g).to(dev)

    def run():
        dg, db = torch.zeros(C, device=dev), torch.zeros(C, device=dev)
        dout = d.clone()
        if mode in ("mask", "eval"):
            dx = K.bn_bwd(dout, y, mean, rstd, gam, act=a, dgamma=dg, dbeta=db, dx_dtype=torch.bfloat16,
                          mask_inplace=True, batch_stats=mode != "eval")
        else:
            dx = K.bn_bwd(dout, y, mean, rstd, gam, relu_beta=bet, dgamma=dg, dbeta=db, dx_dtype=torch.bfloat16,
                          part=given)
        return [dx, dg, db, dout]

    _assert_same(_both(run))


@pytest.mark.parametrize("rows,C", [(131072, 256), (32768, 512), (8192, 1024), (2048, 2048)], ids=lambda v: str(v))
def test_bwd_apply_dual_fold_matches_separate(dev, rows, C):
    g = torch.Generator().manual_seed(rows + 7 * C)
    y, gam, bet, mean, rstd, _, d = _bwd_case(rows, C, g, dev)
    yd = (torch.randn(rows, C, generator=g) * 1.5 - 0.2).to(dev, torch.bfloat16)
    gd, bd = (torch.rand(C, generator=g) + 0.5).to(dev), (torch.randn(C, generator=g) * 0.3).to(dev)
    m2, r2 = K.bn_stats(yd)
    out = K.bn_act(y, mean, rstd, gam, bet, res=yd, res_bn=(m2, r2, gd, bd), relu=True, out_dtype=torch.bfloat16)

    def run():
        gr = [torch.zeros(C, device=dev) for _ in range(4)]
        gm = d.clone()
        dx, dx2 = K.bn_bwd_dual(gm, y, mean, rstd, gam, out, yd, m2, r2, gd, dgamma=gr[0], dbeta=gr[1],
                                dgamma2=gr[2], dbeta2=gr[3], dx_dtype=torch.bfloat16)
        return [dx, dx2, gm] + gr

    _assert_same(_both(run))


@pytest.mark.parametrize("B,H,W,C", [(32, 128, 128, 64), (2, 33, 30, 64)])
def test_bwd_apply_pool_fold_matches_separate(dev, B, H, W, C):
    g = torch.Generator().manual_seed(B * H + W)
    y, gam, bet, mean, rstd, a, _ = _bwd_case(B * H * W, C, g, dev)
    _, idx = K.maxpool_fwd(a.view(B, H, W, C))
    dpool = torch.randn(B, idx.shape[1], idx.shape[2], C, generator=g).to(dev, torch.bfloat16)

    def run():
        dg, db = torch.zeros(C, device=dev), torch.zeros(C, device=dev)
        dx = K.bn_relu_bwd_pooled(dpool, idx, H, W, y, mean, rstd, gam, bet, dgamma=dg, dbeta=db,
                                  dx_dtype=torch.bfloat16)
        return [dx, dg, db]

    _assert_same(_both(run))


def test_act_fold_graph_replay(dev):
    """Captured once, replayed three times: each replay equals the eager launch (the counters the graph's kernel
    uses are re-armed by every launch), and no poll timed out."""
    rows, C = 131072, 64
    g = torch.Generator().manual_seed(5)
    y = torch.randn(rows, C, generator=g).to(dev, torch.bfloat16)
    part = _partials(y)
    pa = _params(C, g, dev)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        ref = K.bn_act_fold(y, part, _clone_params(pa), relu=True, out_dtype=torch.bfloat16)
        graph = torch.cuda.CUDAGraph()
        p_g = _clone_params(pa)
        with torch.cuda.graph(graph, stream=s):
            got = K.bn_act_fold(y, part, p_g, relu=True, out_dtype=torch.bfloat16)
    torch.cuda.current_stream().wait_stream(s)
    for _ in range(3):
        graph.replay()
        torch.cuda.synchronize()
        for a, b in zip(ref, got):
            assert torch.equal(a, b)
    assert int(p_g[6]) == 3
    assert K.bn_fold_timeouts(y.device) == 0


@pytest.mark.parametrize("rows,C", [(524288, 64), (131072, 256), (1000, 2048), (70000, 96)], ids=lambda v: str(v))
def test_split_finish_matches_sequential(dev, rows, C):
    """The separate folds with a workspace (one workgroup per 1024-partial chunk, the last adding the chunk sums)
    against the same launch without one (one workgroup folds the chunks in turn): bit for bit, forward statistics
    with running statistics and backward sums with dgamma / dbeta, twice (the arrival counters re-arm)."""
    from spine_vision_amd import native as nv

    g = torch.Generator().manual_seed(rows + C)
    P = (rows + 63) // 64
    part = torch.randn(P, 2, C, generator=g).to(dev).abs()
    outs = []
    for ws in (True, False, True):
        cw = K._fin_ws(dev) if ws else (None, None)
        mean, rstd = torch.empty(C, device=dev), torch.empty(C, device=dev)
        rm, rv = torch.zeros(C, device=dev), torch.ones(C, device=dev)
        nbt = torch.zeros((), dtype=torch.int64, device=dev)
        K.call("sv_bn_stats_finish", None, nv.SV_F32, K.ptr(part), P, rows, C, 1e-5, 0.1, K.ptr(mean), K.ptr(rstd),
               K.ptr(rm), K.ptr(rv), K.ptr(nbt), *cw)
        sums = torch.empty(2, C, device=dev)
        dg, db = torch.ones(C, device=dev), torch.zeros(C, device=dev)
        K.call("sv_bn_bwd_finish", K.ptr(part), P, C, K.ptr(sums), K.ptr(dg), K.ptr(db), *cw)
        outs.append([mean, rstd, rm, rv, nbt, sums, dg, db])
    torch.cuda.synchronize()
    for k in (1, 2):
        for a, b in zip(outs[0], outs[k]):
            assert torch.equal(a, b)
    assert int(outs[0][4]) == 1
    ctl, _ = K._fold_ws(dev)
    assert int(ctl.abs().sum()) == 0
    # against float64
    s64 = part.double().sum(0)
    assert float(((outs[0][5].double() - s64).abs() / s64.abs().clamp(min=1e-6)).max()) < 1e-5
