"""GPU: every bf16 GEMM family forced through sv_gemm_set_impl (2 = gemm2.hip BK64x3, 3 = gemm3.hip
BK32x3, 8 = gemm8.hip 256x256, 9 = gemm9.hip persistent 256x256 BK64) against the measured per-shape dispatch (impl 0), on every operand
layout and epilogue the ConvNeXt step uses, ragged M/N included -- the knob is tested, not dormant.
Every family accumulates each 16x16 output fragment over k in the same order with the same MFMA, so the
outputs must be BIT-identical; a torch fp32 product on the same bf16 operands checks the values."""

import pytest
import torch

from spine_vision_amd import kernels as K
from spine_vision_amd import native as nv

pytestmark = pytest.mark.gpu


def _impl(i):
    return nv.value("sv_gemm_set_impl", i)


def _run_both(fn, impl):
    prev = _impl(0)
    try:
        a = fn()
        torch.cuda.synchronize()
        _impl(impl)
        b = fn()
        torch.cuda.synchronize()
    finally:
        _impl(prev)
    return a, b


@pytest.mark.parametrize("impl", [2, 3, 8, 9])
@pytest.mark.parametrize("M,C", [(3000, 128), (8192, 256), (2048 + 96, 512)])
def test_gemm_family_bitwise_vs_dispatch(dev, impl, M, C):
    g = torch.Generator().manual_seed(M + C)
    bf = torch.bfloat16
    y = (torch.randn(M, C, generator=g)).to(bf).to(dev)
    w1 = (torch.randn(4 * C, C, generator=g) * 0.05).to(bf).to(dev)
    w2 = (torch.randn(C, 4 * C, generator=g) * 0.05).to(bf).to(dev)
    b1 = (torch.randn(4 * C, generator=g) * 0.1).to(dev)
    b2 = (torch.randn(C, generator=g) * 0.1).to(dev)
    gam = (torch.rand(C, generator=g) * 0.25 + 0.05).to(dev)
    x = torch.randn(M, C, generator=g).to(dev)
    a = torch.randn(M, 4 * C, generator=g).to(bf).to(dev)
    gh = torch.randn(M, 4 * C, generator=g).to(bf).to(dev)
    dy = torch.randn(M, C, generator=g).to(bf).to(dev)
    dh = torch.randn(M, 4 * C, generator=g).to(bf).to(dev)

    def fc1_fwd():
        o, o2 = torch.empty(M, 4 * C, device=dev, dtype=bf), torch.empty(M, 4 * C, device=dev, dtype=bf)
        K.linear_fwd(y, w1, out=o, out2=o2, bias=b1, epilogue=nv.SV_EPI_BIAS_GELU_DUAL)
        return torch.cat([o, o2])

    def fc2_fwd():
        o = torch.empty(M, C, device=dev)
        K.linear_fwd(a, w2, out=o, bias=b2, gamma=gam, residual=x, epilogue=nv.SV_EPI_BIAS_GAMMA_RES)
        return o

    def fc2_dgrad():
        o = torch.empty(M, 4 * C, device=dev, dtype=bf)
        K.linear_dgrad(dy, w2, out=o, epilogue=nv.SV_EPI_MUL_AUX, aux=gh)
        return o

    def fc1_dgrad():
        o = torch.empty(M, C, device=dev, dtype=bf)
        K.linear_dgrad(dh, w1, out=o)
        return o

    def wgrad():
        bo = torch.zeros(C, device=dev)
        o = K.linear_wgrad(dy, a, bias_out=bo, bias_accumulate=False)
        return torch.cat([o.reshape(-1), bo])

    for name, fn in [("fc1_fwd", fc1_fwd), ("fc2_fwd", fc2_fwd), ("fc2_dgrad", fc2_dgrad), ("fc1_dgrad", fc1_dgrad),
                     ("wgrad", wgrad)]:
        ref, got = _run_both(fn, impl)
        if name == "wgrad":
            # the families fold the fused bias column sum in different f32 orders (v2 per BK-64 chunk,
            # v3 per BK-32 step, v9 per lane group of its A fragments): the weight gradient is
            # bit-identical, db within ~1 ulp
            nw = ref.numel() - C
            assert torch.equal(ref[:nw], got[:nw]), (impl, name, float((ref[:nw] - got[:nw]).abs().max()))
            r = float((ref[nw:] - got[nw:]).norm() / ref[nw:].norm())
            assert r < 1e-6, (impl, name, r)
            continue
        assert torch.equal(ref, got), (impl, name, float((ref.float() - got.float()).abs().max()))
    # values: fc1 dgrad against torch fp32 on the same bf16 operands
    o = fc1_dgrad()
    r = dh.float() @ w1.float()
    assert float((o.float() - r).norm() / r.norm()) < 5e-3


def test_gemm_priority_is_bitwise_neutral(dev):
    """sv_gemm_set_priority only raises the waves' issue priority (the lean backward's side-stream
    wgrads): the split-K weight gradient is bit-identical either way."""
    g = torch.Generator().manual_seed(3)
    bf = torch.bfloat16
    dy = torch.randn(8192, 256, generator=g).to(bf).to(dev)
    a = torch.randn(8192, 1024, generator=g).to(bf).to(dev)
    prev_res = nv.value("sv_gemm_set_workgroups_per_cu", 1)  # the backward's residency policy
    try:
        ref = K.linear_wgrad(dy, a)
        prev = nv.value("sv_gemm_set_priority", 1)
        try:
            got = K.linear_wgrad(dy, a)
        finally:
            nv.value("sv_gemm_set_priority", prev)
        torch.cuda.synchronize()
    finally:
        nv.value("sv_gemm_set_workgroups_per_cu", prev_res)
    assert torch.equal(ref, got)


@pytest.mark.parametrize("impl", [0, 3, 9])
def test_gemm_grid_cap_bitwise(dev, impl):
    """sv_gemm_set_grid_cap (the ResNet side stream's weight gradients run under a cap): the kernels are
    persistent over their tiles, so a capped grid computes every tile exactly as the full grid does --
    forward, data-gradient and split-K weight-gradient GEMMs equal bit for bit at caps of 37 and 96."""
    g = torch.Generator().manual_seed(5)
    bf = torch.bfloat16
    M, C = 8192, 256
    y = torch.randn(M, C, generator=g).to(bf).to(dev)
    w1 = (torch.randn(4 * C, C, generator=g) * 0.05).to(bf).to(dev)
    dh = torch.randn(M, 4 * C, generator=g).to(bf).to(dev)

    def run():
        o = torch.empty(M, 4 * C, device=dev, dtype=bf)
        K.linear_fwd(y, w1, out=o)
        d = torch.empty(M, C, device=dev, dtype=bf)
        K.linear_dgrad(dh, w1, out=d, compute_bf16=True)
        wg = K.linear_wgrad(dh, y, compute_bf16=True)
        torch.cuda.synchronize()
        return o.float(), d.float(), wg

    prev_impl = _impl(impl)
    try:
        ref = run()
        for cap in (37, 96):
            prev = nv.value("sv_gemm_set_grid_cap", cap)
            try:
                out = run()
            finally:
                nv.value("sv_gemm_set_grid_cap", prev)
            for a, b in zip(ref, out):
                assert torch.equal(a, b)
    finally:
        _impl(prev_impl)
