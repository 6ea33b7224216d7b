"""fp32 ResNet-50 @256 B=2 teacher-forced block 3 (layer2.0): which kernel carries the dx error?
Each op of the block backward against float64 torch on the same inputs (GPU diagnostic)."""
import sys

import torch

sys.path.insert(0, ".")
import __graft_entry__  # noqa: E402

__graft_entry__.load_package()
import torch.nn.functional as F  # noqa: E402

from spine_vision_amd import kernels as K  # noqa: E402

dev = torch.device("cuda:0")
g = torch.Generator().manual_seed(0)


def rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return float((a - b).norm() / b.norm())


def case(B, H, Cin, Cout, k, stride, pad):
    x = torch.randn(B, Cin, H, H, generator=g)
    w = torch.randn(Cout, Cin, k, k, generator=g) * (2.0 / (Cin * k * k)) ** 0.5
    OH = (H + 2 * pad - k) // stride + 1
    dy = torch.randn(B, Cout, OH, OH, generator=g)
    ref = torch.nn.grad.conv2d_input(x.shape, w.double(), dy.double(), stride=stride, padding=pad)
    cpu32 = torch.nn.grad.conv2d_input(x.shape, w, dy, stride=stride, padding=pad)
    s = K.conv_shape(B, H, H, Cin, Cout, k, stride, pad)
    wp = K.conv_weight_pack(w.to(dev).contiguous(), Cin, torch.float32)
    dyn = dy.permute(0, 2, 3, 1).contiguous().to(dev)
    dx = K.conv_bwd_data(dyn, wp, s).permute(0, 3, 1, 2)
    e = (dx.double().cpu() - ref).abs()
    print(f"dgrad k{k} s{stride} Cin{Cin} Cout{Cout} H{H}: hip rel {rel(dx, ref):.2e} cpu32 rel {rel(cpu32, ref):.2e} "
          f"max abs {float(e.max()):.2e} at {tuple(int(i) for i in (e == e.max()).nonzero()[0])} "
          f"n(>1e-3*max|ref|)={int((e > 1e-3 * ref.abs().max()).sum())}", flush=True)
    # weight gradient too
    refw = torch.nn.grad.conv2d_weight(x.double(), w.shape, dy.double(), stride=stride, padding=pad)
    dw = torch.zeros_like(w).to(dev)
    xn = x.permute(0, 2, 3, 1).contiguous().to(dev)
    K.conv_bwd_weight(dyn, xn, s, dw=dw, accumulate=False)
    print(f"   wgrad: hip rel {rel(dw, refw):.2e}", flush=True)
    # forward
    reff = F.conv2d(x.double(), w.double(), stride=stride, padding=pad)
    y = K.conv_fwd(xn, wp, s, torch.float32).permute(0, 3, 1, 2)
    print(f"   fwd: hip rel {rel(y, reff):.2e}", flush=True)


for args in [(2, 64, 128, 128, 3, 2, 1), (2, 64, 256, 512, 1, 2, 0), (4, 16, 128, 128, 3, 2, 1),
             (2, 32, 128, 128, 3, 1, 1), (2, 64, 64, 64, 3, 1, 1)]:
    case(*args)
