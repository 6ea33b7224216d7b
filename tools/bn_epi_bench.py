"""Standalone timing of the fused BatchNorm-backward statistics against the separate pass, ResNet-50 @256 bs32
inner-BN shapes: conv_bwd_data (bf16 dx) + sv_bn_relu_bwd_stats vs conv_bwd_data_bn (epilogue / split-K finish).
    python tools/bn_epi_bench.py [--iters N]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__  # noqa: E402

__graft_entry__.load_package()
from spine_vision_amd import kernels as K  # noqa: E402
from spine_vision_amd import native as nv  # noqa: E402

SHAPES = {  # name: (B, H, W, Cs, Cout, k)
    "l1_conv3_dgrad_1x1": (32, 64, 64, 64, 256, 1),
    "l1_conv2_dgrad_3x3": (32, 64, 64, 64, 64, 3),
    "l2_conv3_dgrad_1x1": (32, 32, 32, 128, 512, 1),
    "l2_conv2_dgrad_3x3": (32, 32, 32, 128, 128, 3),
    "l3_conv3_dgrad_1x1": (32, 16, 16, 256, 1024, 1),
}


def timeit(fn, iters):
    for _ in range(3):
        fn()
    st = torch.cuda.current_stream()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(st)
    for _ in range(iters):
        fn()
    b.record(st)
    b.synchronize()
    return a.elapsed_time(b) * 1e3 / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    for name, (B, H, W, Cs, Cout, k) in SHAPES.items():
        g = torch.Generator().manual_seed(1)
        s = K.conv_shape(B, H, W, Cs, Cout, k, 1, k // 2)
        wp = K.conv_weight_pack((torch.randn(Cout, Cs, k, k, generator=g) * 0.05).to(dev), Cs, torch.bfloat16)
        dy = torch.randn(B, H, W, Cout, generator=g).to(torch.bfloat16).to(dev)
        rows = B * H * W
        y = torch.randn(rows, Cs, generator=g).to(torch.bfloat16).to(dev)
        gam, bet = (torch.rand(Cs, generator=g) + 0.5).to(dev), (torch.randn(Cs, generator=g) * 0.3).to(dev)
        mean, rstd = K.bn_stats(y)
        P = nv.value("sv_bn_nparts", rows, Cs)
        part = torch.empty(P, 2, Cs, device=dev)

        def sep_dgrad():
            return K.conv_bwd_data(dy, wp, s, dx_dtype=torch.bfloat16)
        dx = sep_dgrad()

        def sep_stats():
            K.call("sv_bn_relu_bwd_stats", K.ptr(dx), K.dt(dx), K.ptr(y), K.dt(y), K.ptr(mean), K.ptr(rstd), K.ptr(gam),
                   K.ptr(bet), rows, Cs, K.ptr(part))
        t_d = timeit(sep_dgrad, args.iters)
        t_s = timeit(sep_stats, args.iters)
        t_f = timeit(lambda: K.conv_bwd_data_bn(dy, wp, s, y.view(B, H, W, Cs), mean, rstd, gam, bet), args.iters)
        print(f"{name:20s} dgrad {t_d:7.1f} us  stats {t_s:7.1f} us  sum {t_d + t_s:7.1f}  fused {t_f:7.1f} us")


if __name__ == "__main__":
    main()
