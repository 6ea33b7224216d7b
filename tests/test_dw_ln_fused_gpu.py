"""The one-pass depthwise conv + LayerNorm (sv_dwconv7_ln_fwd at C = 128 / 256 / 512 over an f32 input: one workgroup
per strip, timm ConvNeXtBlock conv_dw -> norm) against the two-launch form (depthwise ring kernel, then the vectorised
LayerNorm over the stored z): y, mean and rstd bit for bit without z (the eval forward's save_z=False, which takes the
one pass by default), and z too with z kept (SV_DW_LN_FUSED=1, read once by the library: a child process)."""
import os
import subprocess
import sys

import pytest
import torch

from spine_vision_amd import kernels as K
from spine_vision_amd import native as nv

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# ConvNeXt-base S1 / S2 / S3 strips at a small batch, ragged edges (H, W not multiples of the 16 x 4 strip), bf16 / f32
CASES = [(2, 32, 32, 128, "bf16"), (1, 19, 23, 128, "f32"), (2, 16, 16, 256, "bf16"), (1, 13, 9, 256, "f32"),
         (3, 32, 32, 512, "bf16"), (1, 7, 6, 512, "f32"), (1, 1, 1, 512, "bf16")]

_CHILD = r"""
import sys, torch
sys.path.insert(0, sys.argv[1])
import __graft_entry__
__graft_entry__.load_package()
from spine_vision_amd import kernels as K
out = {}
for i, (B, H, W, C, dts) in enumerate(eval(sys.argv[2])):
    g = torch.Generator().manual_seed(100 + i)
    x = (torch.randn(B, H, W, C, generator=g) * 1.5 + 0.2).cuda()
    w = (torch.randn(C, 49, generator=g) * 0.2).cuda()
    b = (torch.randn(C, generator=g) * 0.1).cuda()
    lw = (torch.rand(C, generator=g) + 0.5).cuda()
    lb = (torch.randn(C, generator=g) * 0.1).cuda()
    act = torch.bfloat16 if dts == "bf16" else torch.float32
    z, y, m, r = K.dwconv7_ln_fwd(x, w, b, lw, lb, act_dtype=act)
    z2, y2, m2, r2 = K.dwconv7_ln_fwd(x, w, b, lw, lb, act_dtype=act, save_z=False)
    assert z2 is None
    out[i] = [t.cpu() for t in (z, y, m, r, y2, m2, r2)]
torch.save(out, sys.argv[3])
"""


def _inputs(i, B, H, W, C):
    g = torch.Generator().manual_seed(100 + i)
    x = (torch.randn(B, H, W, C, generator=g) * 1.5 + 0.2).cuda()
    w = (torch.randn(C, 49, generator=g) * 0.2).cuda()
    b = (torch.randn(C, generator=g) * 0.1).cuda()
    lw = (torch.rand(C, generator=g) + 0.5).cuda()
    lb = (torch.randn(C, generator=g) * 0.1).cuda()
    return x, w, b, lw, lb


def test_dw_ln_fused_matches_two_launches(dev, tmp_path, monkeypatch):
    assert os.environ.get("SV_DW_LN_FUSED") is None
    # the one pass is bitwise the VALU kernels' two launches (f32 taps and x); the training forward's matrix-core
    # depthwise (bf16 operands, K.DW_MFMA) is pinned by tests/test_dw_mfma_gpu.py
    monkeypatch.setattr(K, "DW_MFMA", False)
    refs = []
    for i, (B, H, W, C, dts) in enumerate(CASES):
        code = nv.SV_BF16 if dts == "bf16" else nv.SV_F32
        assert K.value("sv_dwconv7_ln_fused_ok", B, H, W, C, nv.SV_F32, code, code) == 1
        x, w, b, lw, lb = _inputs(i, B, H, W, C)
        act = torch.bfloat16 if dts == "bf16" else torch.float32
        z, y, m, rs = K.dwconv7_ln_fwd(x, w, b, lw, lb, act_dtype=act)  # z kept: the two launches
        z1, y1, m1, rs1 = K.dwconv7_ln_fwd(x, w, b, lw, lb, act_dtype=act, save_z=False)  # the one pass
        torch.cuda.synchronize()
        assert z1 is None
        for name, a, e in (("y", y1, y), ("mean", m1, m), ("rstd", rs1, rs)):
            assert torch.equal(a, e), (B, H, W, C, dts, name, float((a.float() - e.float()).abs().max()))
        refs.append([t.cpu() for t in (z, y, m, rs, y, m, rs)])
    # the one pass with z kept (forced), in a child process
    out_file = tmp_path / "one_pass.pt"
    env = dict(os.environ, SV_DW_LN_FUSED="1", SV_DW_MFMA="0")
    r = subprocess.run([sys.executable, "-c", _CHILD, ROOT, repr(CASES), str(out_file)], env=env, capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    got = torch.load(out_file, weights_only=True)
    for i, (B, H, W, C, dts) in enumerate(CASES):
        for name, a, e in zip(("z", "y", "mean", "rstd", "y (no z)", "mean (no z)", "rstd (no z)"), got[i], refs[i]):
            assert torch.equal(a.reshape(e.shape), e), (B, H, W, C, dts, name,
                                                         float((a.float().reshape(e.shape) - e.float()).abs().max()))


def test_dw_ln_unfused_widths_keep_z(dev, monkeypatch):
    """VALU kernels: C = 64 / 1024 (not the one-pass form) still write z even when the caller keeps none."""
    monkeypatch.setattr(K, "DW_MFMA", False)
    for C in (64, 1024):
        x, w, b, lw, lb = _inputs(7, 1, 8, 8, C)
        assert K.value("sv_dwconv7_ln_fused_ok", 1, 8, 8, C, nv.SV_F32, nv.SV_BF16, nv.SV_BF16) == 0
        z, y, _, _ = K.dwconv7_ln_fwd(x, w, b, lw, lb, act_dtype=torch.bfloat16, save_z=False)
        assert z is not None and z.shape == (1, 8, 8, C) and y.shape == (64, C)


@pytest.mark.parametrize("lanes", [16, 32, 64])
def test_xlane_group_sum_is_the_shuffle_butterfly(dev, lanes):
    """common.h xlane_group_sum (permlane swaps + DPP row rotations, used by the LayerNorm statistics) against the
    ds_bpermute __shfl_xor butterfly on the same lanes: bitwise, over values of mixed sign and magnitude (so every
    addition order would show), denormals, zeros and infinities."""
    g = torch.Generator().manual_seed(lanes)
    n = 256 * 1024
    v = torch.randn(n, generator=g) * torch.exp2(torch.randint(-30, 30, (n,), generator=g).float())
    v[::97] = 0.0
    v[5::101] = 1e-40
    v[7::4099] = float("inf")
    v = v.to(dev)
    xl, sh = torch.empty_like(v), torch.empty_like(v)
    K.call("sv_diag_group_sum", K.ptr(v), K.ptr(xl), K.ptr(sh), n, lanes)
    torch.cuda.synchronize()
    fin = torch.isfinite(sh)
    assert torch.equal(xl[fin], sh[fin]) and torch.equal(torch.isfinite(xl), fin)
    # every lane of a group holds the same sum
    grp = sh.view(-1, lanes)
    ok = torch.isfinite(grp).all(1)
    assert torch.equal(grp[ok], grp[ok][:, :1].expand(-1, lanes))
