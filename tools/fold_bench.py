"""Standalone timing of the split-K fold passes of the ConvNeXt-base bs32 weight gradients (HIP events):
the fc2 layer-scale finish (sv_layerscale_wgrad_reduce: slabs -> dW2, dgamma, db2) and the fc1 slab fold
(sv_reduce_partials_multi wide segment), at each stage's split depth -- their rate alone, to set against their
in-step rate beside the main stream.

    python tools/fold_bench.py [--iters 20]
"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__  # noqa: E402

__graft_entry__.load_package()
from spine_vision_amd import kernels as K  # noqa: E402
from spine_vision_amd import native as nv  # noqa: E402

STAGES = {"S1": (524288, 128), "S2": (131072, 256), "S3": (32768, 512), "S4": (8192, 1024)}


def timeit(fn, iters):
    for _ in range(3):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    for st, (M, C) in STAGES.items():
        K4 = 4 * C
        split = K._wgrad_split_for(C, K4, M)
        slab = torch.randn(split * C * K4, device=dev)
        cs = torch.randn(split * C, device=dev)
        w2, dw2 = torch.randn(C, K4, device=dev), torch.zeros(C, K4, device=dev)
        gam, b2 = torch.rand(C, device=dev), torch.randn(C, device=dev)
        dg, db = torch.zeros(C, device=dev), torch.zeros(C, device=dev)

        def ls():
            nv.call("sv_layerscale_wgrad_reduce", nv.ptr(slab), nv.ptr(cs), split, nv.ptr(w2), nv.ptr(gam),
                    nv.ptr(b2), nv.ptr(dw2), nv.ptr(dg), nv.ptr(db), None, C, K4)

        out = torch.zeros(K4 * C, device=dev)
        bias_out = torch.zeros(K4, device=dev)
        cs1 = torch.randn(split * K4, device=dev)

        def multi():
            K.reduce_multi([(slab, out, split, True), (cs1, bias_out, split, True)])

        nbytes_ls = 4.0 * ((split + 2) * C * K4 + (split + 4) * C)
        nbytes_m = 4.0 * ((split + 2) * C * K4 + (split + 2) * K4)
        t_ls, t_m = timeit(ls, args.iters), timeit(multi, args.iters)
        print(f"{st} C={C:5d} split={split:3d}  layerscale_reduce {t_ls:7.1f} us {nbytes_ls / t_ls / 1e6:6.2f} TB/s"
              f"  reduce_multi(fc1 slab + bias) {t_m:7.1f} us {nbytes_m / t_m / 1e6:6.2f} TB/s", flush=True)


if __name__ == "__main__":
    main()
