"""Standalone timing of the ResNet-50 @256 bs32 convolution passes (bf16) on the kernel library:
    python tools/conv_bench.py [--iters N]
Prints one line per (shape, pass): mean us per call over N calls (HIP events on the current stream)."""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__  # noqa: E402

__graft_entry__.load_package()
from spine_vision_amd import kernels as K  # noqa: E402

SHAPES = {  # name: (B, H, W, Cs, Cin, Cout, k, stride, pad)
    "stem7x7s2": (32, 256, 256, 8, 3, 64, 7, 2, 3),
    "l1_3x3": (32, 64, 64, 64, 64, 64, 3, 1, 1),
    "l1_1x1in": (32, 64, 64, 256, 256, 64, 1, 1, 0),
    "l1_1x1out": (32, 64, 64, 64, 64, 256, 1, 1, 0),
    "l2_3x3s2": (32, 64, 64, 128, 128, 128, 3, 2, 1),
    "l2_3x3": (32, 32, 32, 128, 128, 128, 3, 1, 1),
    "l3_3x3s2": (32, 32, 32, 256, 256, 256, 3, 2, 1),
    "l3_3x3": (32, 16, 16, 256, 256, 256, 3, 1, 1),
    "l4_3x3": (32, 8, 8, 512, 512, 512, 3, 1, 1),
    "l2_ds1x1s2": (32, 64, 64, 256, 256, 512, 1, 2, 0),
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
    ap.add_argument("--only", default="")
    ap.add_argument("--split", type=int, default=0, help="force the fwd / stride-1 dgrad split-K depth (0: dispatch's)")
    args = ap.parse_args()
    if args.split:
        K._conv_split = lambda M, N, Kd: args.split
    dev = torch.device("cuda:0")
    tag = " ".join(f"{k}={v}" for k, v in os.environ.items() if k.startswith("SV_")) + (f" split={args.split}" if args.split else "")
    for name, (B, H, W, Cs, Cin, Cout, k, s, p) in SHAPES.items():
        if args.only and args.only not in name:
            continue
        shape = K.conv_shape(B, H, W, Cs, Cout, k, s, p, Cin)
        OH, OW = K.conv_out_hw(H, W, k, s, p)
        x = torch.randn(B, H, W, Cs, device=dev).to(torch.bfloat16)
        dy = torch.randn(B, OH, OW, Cout, device=dev).to(torch.bfloat16)
        w = torch.randn(Cout, Cin, k, k, device=dev) * 0.05
        wp = K.conv_weight_pack(w, Cs, torch.bfloat16)
        dw = torch.zeros_like(w)
        t_w = timeit(lambda: K.conv_bwd_weight(dy, x, shape, dw=dw, accumulate=True), args.iters)
        t_f = timeit(lambda: K.conv_fwd(x, wp, shape, torch.bfloat16), args.iters)
        gf = 2.0 * B * OH * OW * Cout * Cin * k * k / 1e9
        line = (f"{name:12s} {gf:6.2f} GF  wgrad {t_w:8.1f} us {gf / t_w * 1e3:6.0f} TF  "
                f"fwd {t_f:8.1f} us {gf / t_f * 1e3:6.0f} TF")
        if Cin == Cs:
            t_d = timeit(lambda: K.conv_bwd_data(dy, wp, shape, dx_dtype=torch.bfloat16), args.iters)
            line += f"  dgrad {t_d:8.1f} us {gf / t_d * 1e3:6.0f} TF"
        print(line + f"  [{tag}]", flush=True)


if __name__ == "__main__":
    main()
