"""Standalone timing of the ConvNeXt-base @512 bs32 downsample LayerNorm + 2x2 patch gather (forward, bf16
patches) and its backward (f32 dx + bf16 copy) through the C ABI (HIP events).

    python tools/ds_bench.py [--iters 20]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import __graft_entry__  # noqa: E402

__graft_entry__.load_package()
from spine_vision_amd import kernels as K  # noqa: E402

SHAPES = {"S1->S2": (128, 128), "S2->S3": (64, 256), "S3->S4": (32, 512)}


def timeit(fn, iters):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    B = 32
    for name, (S, C) in SHAPES.items():
        x = torch.randn(B, S, S, C, device=dev)
        lnw = torch.rand(C, device=dev) + 0.5
        lnb = torch.randn(C, device=dev) * 0.1
        patches, mean, rstd = K.downsample_fwd(x, lnw, lnb, act_dtype=torch.bfloat16)
        dp = torch.randn(patches.shape, device=dev)
        dlnw, dlnb = torch.zeros(C, device=dev), torch.zeros(C, device=dev)
        n = B * S * S * C
        fwd = timeit(lambda: K.downsample_fwd(x, lnw, lnb, act_dtype=torch.bfloat16), args.iters)
        bwd = timeit(lambda: K.downsample_bwd(dp, x, mean, rstd, lnw, dlnw=dlnw, dlnb=dlnb, with_bf16=True), args.iters)
        print(f"{name} fwd {fwd:7.1f} us {6 * n / fwd / 1e3:7.1f} GB/s | bwd {bwd:7.1f} us {18 * n / bwd / 1e3:7.1f} GB/s",
              flush=True)


if __name__ == "__main__":
    main()
