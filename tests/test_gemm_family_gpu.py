"""GPU: every bf16 GEMM family forced through the per-call policy (sv_gemm_policy.impl: 2 = gemm2.hip BK64x3,
3 = gemm3.hip BK32x3, 8 = gemm8.hip 256x256, 9 = gemm9.hip persistent 256x256 BK64) against the measured
per-shape dispatch (impl 0), on every operand layout and epilogue the ConvNeXt step uses, ragged M/N included
-- the knob is tested, not dormant.  Every family accumulates each 16x16 output fragment over k in the same
order with the same MFMA, so the outputs must be BIT-identical; a torch fp32 product on the same bf16 operands
checks the values.

The bs32 cases run the production schedule the bench times: at ConvNeXt-base 512x512
bs32 the persistent v9 kernel processes SEVERAL 256x256 tiles per workgroup (S1 fc1: 4096 tiles on 256 CUs),
with the fused GELU-dual, gamma-residual and x GELU' epilogues keeping stores and operand loads in flight
across tiles; they are checked bit for bit against v3 (one workgroup per tile) and against torch fp32, under
the forward's default policy and the backward's (one persistent workgroup per CU, raised priority, the
data-parallel grid cap)."""

import pytest
import torch

from spine_vision_amd import kernels as K
from spine_vision_amd import native as nv

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _f32_slabs(monkeypatch):
    """These tests pin the kernel families against each other on f32 split-K slabs; the bf16 slabs of the production
    schedule have their own test (test_wgrad_bf16_slabs)."""
    monkeypatch.setattr(K, "_WGRAD_BF16_SLABS", False)


def _ops(dev, M, C, seed):
    g = torch.Generator().manual_seed(seed)
    bf = torch.bfloat16
    t = {
        "y": torch.randn(M, C, generator=g).to(bf).to(dev),
        "w1": (torch.randn(4 * C, C, generator=g) * 0.05).to(bf).to(dev),
        "w2": (torch.randn(C, 4 * C, generator=g) * 0.05).to(bf).to(dev),
        "b1": (torch.randn(4 * C, generator=g) * 0.1).to(dev),
        "b2": (torch.randn(C, generator=g) * 0.1).to(dev),
        "gam": (torch.rand(C, generator=g) * 0.25 + 0.05).to(dev),
        "x": torch.randn(M, C, generator=g).to(dev),
        "a": torch.randn(M, 4 * C, generator=g).to(bf).to(dev),
        "gh": torch.randn(M, 4 * C, generator=g).to(bf).to(dev),
        "dy": torch.randn(M, C, generator=g).to(bf).to(dev),
        "dh": torch.randn(M, 4 * C, generator=g).to(bf).to(dev),
    }
    return t


def _funcs(t, dev, M, C):
    bf = torch.bfloat16

    def fc1_fwd(pol):
        o, o2 = torch.empty(M, 4 * C, device=dev, dtype=bf), torch.empty(M, 4 * C, device=dev, dtype=bf)
        K.linear_fwd(t["y"], t["w1"], out=o, out2=o2, bias=t["b1"], epilogue=nv.SV_EPI_BIAS_GELU_DUAL, policy=pol)
        return torch.cat([o, o2])

    def fc2_fwd(pol):
        o = torch.empty(M, C, device=dev)
        K.linear_fwd(t["a"], t["w2"], out=o, bias=t["b2"], gamma=t["gam"], residual=t["x"],
                     epilogue=nv.SV_EPI_BIAS_GAMMA_RES, policy=pol)
        return o

    def fc2_dgrad(pol):
        o = torch.empty(M, 4 * C, device=dev, dtype=bf)
        K.linear_dgrad(t["dy"], t["w2"], out=o, epilogue=nv.SV_EPI_MUL_AUX, aux=t["gh"], policy=pol)
        return o

    def fc1_dgrad(pol):
        o = torch.empty(M, C, device=dev, dtype=bf)
        K.linear_dgrad(t["dh"], t["w1"], out=o, policy=pol)
        return o

    def wgrad(pol):  # the fc2 weight gradient d^T a with its fused bias column sum (split-K slabs + fold)
        bo = torch.zeros(C, device=dev)
        o = K.linear_wgrad(t["dy"], t["a"], bias_out=bo, bias_accumulate=False, policy=pol)
        return torch.cat([o.reshape(-1), bo])

    def wgrad1(pol):  # the fc1 weight gradient dh^T y
        return K.linear_wgrad(t["dh"], t["y"], policy=pol).reshape(-1)

    return [("fc1_fwd", fc1_fwd), ("fc2_fwd", fc2_fwd), ("fc2_dgrad", fc2_dgrad), ("fc1_dgrad", fc1_dgrad),
            ("wgrad", wgrad), ("wgrad1", wgrad1)]


def _same(name, ref, got, C, tag):
    if name == "wgrad":
        # the families fold the fused bias column sum in different f32 orders (v2 per BK-64 chunk, v3 per
        # BK-32 step, v9 per lane group of its A fragments): the weight gradient is bit-identical, db within ~1 ulp
        nw = ref.numel() - C
        assert torch.equal(ref[:nw], got[:nw]), (tag, name, float((ref[:nw] - got[:nw]).abs().max()))
        r = float((ref[nw:] - got[nw:]).norm() / ref[nw:].norm())
        assert r < 1e-6, (tag, name, r)
        return
    assert torch.equal(ref, got), (tag, name, float((ref.float() - got.float()).abs().max()))


@pytest.mark.parametrize("impl", [2, 3, 8, 9])
@pytest.mark.parametrize("M,C", [(3000, 128), (8192, 256), (2048 + 96, 512)])
def test_gemm_family_bitwise_vs_dispatch(dev, impl, M, C):
    t = _ops(dev, M, C, M + C)
    for name, fn in _funcs(t, dev, M, C):
        ref = fn(None)
        got = fn(nv.policy(impl=impl))
        torch.cuda.synchronize()
        _same(name, ref, got, C, f"impl{impl}")
    # values: fc1 dgrad against torch fp32 on the same bf16 operands
    o = dict(_funcs(t, dev, M, C))["fc1_dgrad"](None)
    r = t["dh"].float() @ t["w1"].float()
    assert float((o.float() - r).norm() / r.norm()) < 5e-3


def _rel(a, b):
    a, b = a.double(), b.double()
    return float((a - b).norm() / (b.norm() + 1e-30))


def _torch_refs(t, M, C):
    """fp32 products of the same bf16 operands (torch on the GPU; GELU in erf form, its derivative Phi + x phi)."""
    y, w1, w2 = t["y"].float(), t["w1"].float(), t["w2"].float()
    h = y @ w1.t() + t["b1"]
    phi = torch.exp(-0.5 * h * h) * 0.3989422804014327
    Phi = 0.5 * (1.0 + torch.erf(h * 0.7071067811865476))
    ref = {"fc1_fwd": (Phi + h * phi, h * Phi)}
    del phi, Phi, h
    ref["fc2_fwd"] = t["gam"] * (t["a"].float() @ w2.t() + t["b2"])  # the delta over the residual
    ref["fc2_dgrad"] = (t["dy"].float() @ w2) * t["gh"].float()
    ref["fc1_dgrad"] = t["dh"].float() @ w1
    ref["wgrad"] = (t["dy"].float().t() @ t["a"].float(), t["dy"].float().sum(0))
    ref["wgrad1"] = t["dh"].float().t() @ y
    return ref


# ConvNeXt-base 512x512 bs32: S1 (M = 32*128^2, C = 128), S3 (32*32^2, 512), S4 (32*16^2, 1024); ConvNeXt-large
# 512x512 bs64 (BASELINE configs[4]): S1 (64*128^2, 192, partial 256-column tiles) and S3 (64*32^2, 768, the stage
# of 27 of its 36 blocks; its weight gradients at split 4 = 144 workgroups)
_BS32 = [(524288, 128), (32768, 512), (8192, 1024), (1048576, 192), (65536, 768)]


@pytest.mark.timeout(600)
@pytest.mark.parametrize("M,C", _BS32, ids=["S1", "S3", "S4", "large-S1", "large-S3"])
def test_gemm_bs32_production_schedule(dev, M, C):
    """The bs32 shapes the bench runs: the dispatch's schedule (v9 with several tiles per persistent workgroup
    where it picks v9) under the forward's default policy AND the lean backward's (one persistent workgroup per
    CU, raised priority, grid capped at 224 as under data parallelism) equals v3 (one workgroup per tile) bit for
    bit on every epilogue, and v3's values match torch fp32 on the same bf16 operands."""
    t = _ops(dev, M, C, 7 + C)
    funcs = _funcs(t, dev, M, C)
    bwd = nv.policy(wg_per_cu=1, priority=1, grid_cap=224)
    outs = {}
    for name, fn in funcs:
        ref = fn(nv.policy(impl=3))
        for tag, pol in (("default", None), ("backward", bwd)):
            got = fn(pol)
            torch.cuda.synchronize()
            _same(name, ref, got, C, tag)
            del got
        outs[name] = ref
    ref = _torch_refs(t, M, C)
    n = M * 4 * C
    r = {
        "fc1_fwd GELU'": _rel(outs["fc1_fwd"][:M].float(), ref["fc1_fwd"][0]),
        "fc1_fwd GELU": _rel(outs["fc1_fwd"][M:].float(), ref["fc1_fwd"][1]),
        "fc2_fwd": _rel(outs["fc2_fwd"] - t["x"], ref["fc2_fwd"]),
        "fc2_dgrad": _rel(outs["fc2_dgrad"].float(), ref["fc2_dgrad"]),
        "fc1_dgrad": _rel(outs["fc1_dgrad"].float(), ref["fc1_dgrad"]),
        "wgrad": _rel(outs["wgrad"][:C * 4 * C], ref["wgrad"][0].reshape(-1)),
        "wgrad bias": _rel(outs["wgrad"][C * 4 * C:], ref["wgrad"][1]),
        "wgrad1": _rel(outs["wgrad1"], ref["wgrad1"].reshape(-1)),
    }
    print(f"[bs32] M={M} C={C} rel vs torch fp32: " + ", ".join(f"{k} {v:.2e}" for k, v in r.items()))
    assert n > 0
    # bf16 outputs: the store's rounding (2^-9 relative at most, ~1e-3 RMS); f32 outputs: accumulation order
    for k in ("fc1_fwd GELU'", "fc1_fwd GELU", "fc2_dgrad", "fc1_dgrad"):
        assert r[k] < 4e-3, (k, r[k])
    for k in ("fc2_fwd", "wgrad", "wgrad bias", "wgrad1"):
        assert r[k] < 1e-4, (k, r[k])


def test_gemm_priority_is_bitwise_neutral(dev):
    """policy.priority only raises the waves' issue priority (the lean backward's side-stream wgrads): the
    split-K weight gradient is bit-identical either way."""
    g = torch.Generator().manual_seed(3)
    bf = torch.bfloat16
    dy = torch.randn(8192, 256, generator=g).to(bf).to(dev)
    a = torch.randn(8192, 1024, generator=g).to(bf).to(dev)
    ref = K.linear_wgrad(dy, a, policy=nv.policy(wg_per_cu=1))  # the backward's residency policy
    got = K.linear_wgrad(dy, a, policy=nv.policy(wg_per_cu=1, priority=1))
    torch.cuda.synchronize()
    assert torch.equal(ref, got)


@pytest.mark.parametrize("impl", [0, 3, 9])
def test_gemm_grid_cap_bitwise(dev, impl):
    """policy.grid_cap (the ResNet side stream's weight gradients, the data-parallel comm reserve): the kernels
    are persistent over their tiles, so a capped grid computes every tile exactly as the full grid does --
    forward, data-gradient and split-K weight-gradient GEMMs equal bit for bit at caps of 37 and 96."""
    g = torch.Generator().manual_seed(5)
    bf = torch.bfloat16
    M, C = 8192, 256
    y = torch.randn(M, C, generator=g).to(bf).to(dev)
    w1 = (torch.randn(4 * C, C, generator=g) * 0.05).to(bf).to(dev)
    dh = torch.randn(M, 4 * C, generator=g).to(bf).to(dev)

    def run(cap):
        pol = nv.policy(impl=impl, grid_cap=cap)
        o = torch.empty(M, 4 * C, device=dev, dtype=bf)
        K.linear_fwd(y, w1, out=o, policy=pol)
        d = torch.empty(M, C, device=dev, dtype=bf)
        K.linear_dgrad(dh, w1, out=d, compute_bf16=True, policy=pol)
        wg = K.linear_wgrad(dh, y, compute_bf16=True, policy=pol)
        torch.cuda.synchronize()
        return o.float(), d.float(), wg

    ref = run(0)
    for cap in (37, 96):
        for a, b in zip(ref, run(cap)):
            assert torch.equal(a, b)


def test_gemm_policy_is_per_call(dev):
    """A policy travels with its call only: a capped launch on a side stream leaves an uncapped launch issued
    meanwhile on the default stream untouched (both bitwise the reference), and an invalid policy is refused
    with an error rather than applied."""
    g = torch.Generator().manual_seed(6)
    bf = torch.bfloat16
    M, C = 8192, 512
    dh = torch.randn(M, 4 * C, generator=g).to(bf).to(dev)
    y = torch.randn(M, C, generator=g).to(bf).to(dev)
    ref = K.linear_wgrad(dh, y)
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        capped = K.linear_wgrad(dh, y, policy=nv.policy(grid_cap=17, priority=1, wg_per_cu=1))
    plain = K.linear_wgrad(dh, y)
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    assert torch.equal(ref, capped) and torch.equal(ref, plain)
    with pytest.raises(RuntimeError, match="policy"):
        K.linear_wgrad(dh, y, policy=nv.policy(impl=5))


@pytest.mark.parametrize("M,C", [(4096, 128), (131072, 256), (32768, 512), (8192, 1024), (2048 + 512, 512),
                                 (6272, 512)],
                         ids=["half-tiles", "S2", "S3", "S4", "ragged-split", "split7"])
def test_wgrad_inkernel_fold_bitwise(dev, M, C):
    """The split-K fold inside the persistent v9 weight-gradient GEMM (sv_gemm_desc.fold_out) equals the slabs +
    separate fold bit for bit -- written or accumulated, under the default grid (every slice its own workgroup: the
    spread form, each slice's workgroup summing 1/split of its tile's rows), a grid cap that makes every workgroup
    fold several tiles (37: the last-arriver form), the backward's policy, and the v3 family (slabs + fold pass) --
    and so does the layer-scale fc2 finish over the folded G."""
    g = torch.Generator().manual_seed(M + C)
    bf = torch.bfloat16
    dh = torch.randn(M, 4 * C, generator=g).to(bf).to(dev)
    y = torch.randn(M, C, generator=g).to(bf).to(dev)
    d = torch.randn(M, C, generator=g).to(bf).to(dev)
    a = torch.randn(M, 4 * C, generator=g).to(bf).to(dev)
    w2 = (torch.randn(C, 4 * C, generator=g) * 0.05).to(dev)
    gam = (torch.rand(C, generator=g) * 0.25 + 0.05).to(dev)
    b2 = (torch.randn(C, generator=g) * 0.1).to(dev)
    base = torch.randn(4 * C, C, generator=g).to(dev)
    base_b = torch.randn(4 * C, generator=g).to(dev)

    saved = (K._INKERNEL_FOLD, K._FOLD_MAX_SPLIT)

    def run(fold, pol):
        K._INKERNEL_FOLD = fold
        K._FOLD_MAX_SPLIT = 64  # also the deeper splits (C = 128: 64 slices of half-empty 256x256 tiles)
        try:
            o1, b1 = base.clone(), base_b.clone()
            K.linear_wgrad(dh, y, out=o1, accumulate=True, bias_out=b1, policy=pol)
            o2 = torch.empty(4 * C, C, device=dev)
            K.linear_wgrad(dh, y, out=o2, accumulate=False, policy=pol)
            dw2, dga, db = base.t().contiguous().clone(), gam.clone() * 0.5, b2.clone() * 0.5
            K.layerscale_wgrad(d, a, w2, gam, b2, dw2=dw2, dgamma=dga, db2=db, policy=pol)
            torch.cuda.synchronize()
            return o1, b1, o2, dw2, dga, db
        finally:
            K._INKERNEL_FOLD, K._FOLD_MAX_SPLIT = saved

    split = K._wgrad_split_for(4 * C, C, M)
    if M == 6272:
        # a split that does not divide the 256-row tile (per-slice rows 37: the last slice's range runs past its
        # tile) over 8 M tiles, so an unclamped spread fold would add the next tile's rows twice
        assert split == 7 and 256 % split != 0
    ref = run(False, None)
    for pol in (None, nv.policy(grid_cap=37), nv.policy(wg_per_cu=1, priority=1, grid_cap=224), nv.policy(impl=3)):
        # (v3 sums the fused bias column in its own order: its reference is its own slabs + fold)
        r_ = run(False, pol) if pol is not None and pol.impl == 3 else ref
        got = run(True, pol)
        for i, (r, o) in enumerate(zip(r_, got)):
            assert torch.equal(r, o), (pol, i, split, float((r - o).abs().max()))


@pytest.mark.timeout(300)
def test_wgrad_spread_fold_under_uneven_load(dev):
    """The spread fold's hand-off (write-through slabs, one agent-scope add per workgroup, an sc1 poll, sc1 loads)
    under uneven load: each fold GEMM is launched while a persistent GEMM on a second stream holds part of the chip,
    so a tile's slices land at different times and their workgroups wait on one another.  Every word of every
    repetition must equal the separate fold's result (MI355X_MICROARCH.md: test hand-offs under uneven load)."""
    g = torch.Generator().manual_seed(11)
    bf = torch.bfloat16
    M, C = 32768, 512
    dh = torch.randn(M, 4 * C, generator=g).to(bf).to(dev)
    y = torch.randn(M, C, generator=g).to(bf).to(dev)
    xa = torch.randn(65536, 1024, generator=g).to(bf).to(dev)
    wb = torch.randn(2048, 1024, generator=g).to(bf).to(dev)
    busy = torch.empty(65536, 2048, device=dev, dtype=bf)
    saved = K._INKERNEL_FOLD
    try:
        K._INKERNEL_FOLD = False
        ref = K.linear_wgrad(dh, y, out=torch.empty(4 * C, C, device=dev))
        K._INKERNEL_FOLD = True
        side = torch.cuda.Stream(device=dev)
        outs = []
        for rep in range(6):
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):  # a 2-tile-per-CU persistent GEMM beside the fold (cap varies the skew)
                K.linear_fwd(xa, wb, out=busy, policy=nv.policy(grid_cap=64 + 32 * rep))
            outs.append(K.linear_wgrad(dh, y, out=torch.empty(4 * C, C, device=dev)))
            torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
    finally:
        K._INKERNEL_FOLD = saved
    for i, o in enumerate(outs):
        assert torch.equal(o, ref), (i, float((o - ref).abs().max()))


@pytest.mark.parametrize("M,C", [(32768, 512), (131072, 256), (8192, 1024)])
def test_wgrad_bf16_slabs(dev, M, C, monkeypatch):
    """Opt-in bf16 split-K slabs for the v9 weight gradients (SV_WGRAD_BF16_SLABS): the fold equals, bit for bit, the
    f32 slabs of the same GEMM rounded to bf16 (RNE) and summed in f32 in slice order; the fc2 layer-scale finish
    over bf16 slabs stays within bf16 rounding of the f32-slab result (a weight gradient the reference's autocast
    rounds to bf16 once)."""
    g = torch.Generator().manual_seed(M // 1024 + C)
    bf = torch.bfloat16
    dh = torch.randn(M, 4 * C, generator=g).to(bf).to(dev)
    y = torch.randn(M, C, generator=g).to(bf).to(dev)
    nw, kw = 4 * C, C
    split = K._wgrad_split_for(nw, kw, M)
    assert split > 1
    slab = torch.empty(split * nw * kw, device=dev)
    K.gemm(dh, y, M=nw, N=kw, K=M, a_kmajor=False, b_kmajor=False, lda=nw, ldb=kw, epilogue=nv.SV_EPI_SLAB, C=slab,
           split_k=split)
    ref = torch.zeros(nw * kw, device=dev)
    base = torch.randn(nw * kw, generator=g).to(dev)
    for p in range(split):
        ref = ref + slab[p * nw * kw:(p + 1) * nw * kw].to(bf).float()
    ref = ref + base
    monkeypatch.setattr(K, "_WGRAD_BF16_SLABS", True)
    out = base.clone().view(nw, kw)
    K.linear_wgrad(dh, y, out=out, accumulate=True)
    torch.cuda.synchronize()
    assert torch.equal(out.view(-1), ref), float((out.view(-1) - ref).abs().max())
    # fc2: the layer-scale finish over bf16 slabs against the f32 slabs
    d = torch.randn(M, C, generator=g).to(bf).to(dev)
    a = torch.randn(M, 4 * C, generator=g).to(bf).to(dev)
    w2 = (torch.randn(C, 4 * C, generator=g) * 0.05).to(dev)
    gam, b2 = (torch.rand(C, generator=g) + 0.1).to(dev), torch.randn(C, generator=g).to(dev)
    res = {}
    for flag in (False, True):
        monkeypatch.setattr(K, "_WGRAD_BF16_SLABS", flag)
        dw2, dgm, db2 = torch.zeros(C, 4 * C, device=dev), torch.zeros(C, device=dev), torch.zeros(C, device=dev)
        K.layerscale_wgrad(d, a, w2, gam, b2, dw2=dw2, dgamma=dgm, db2=db2)
        res[flag] = (dw2, dgm, db2)
    torch.cuda.synchronize()
    for i, name in enumerate(("dW2", "dgamma", "db2")):
        r = _rel(res[True][i], res[False][i])
        assert r < 4e-3, (name, r)
    assert torch.equal(res[True][2], res[False][2])  # the bias gradient comes from the f32 column sums
