"""Standalone timing of the fused ConvNeXt MLP forward (sv_mlp_fwd) against the two-GEMM path it replaces, at the
production shapes (HIP events, back-to-back launches on random data).

    python tools/mlp_bench.py [--iters 30] [--shapes base-S1,base-S2,large-S1]
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
from spine_vision_amd import native as nv  # noqa: E402

SHAPES = {"base-S1": (524288, 128), "base-S2": (131072, 256), "large-S1": (1048576, 192), "large-S2": (262144, 384),
          "base-S3": (32768, 512)}
HBM = 6.3e12  # B/s the chip sustains (MI355X_MICROARCH.md: 6.29 TB/s float4 copy)


def timed(fn, iters):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--shapes", default="base-S1,base-S2,large-S1,base-S3")
    ap.add_argument("--bwd", action="store_true", help="also the fused backward (C = 128) against its three kernels")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    bf = torch.bfloat16
    for name in args.shapes.split(","):
        M, C = SHAPES[name]
        H = 4 * C
        y = torch.randn(M, C, device=dev).to(bf)
        w1 = (torch.randn(H, C, device=dev) * 0.08).to(bf)
        w2 = (torch.randn(C, H, device=dev) * 0.05).to(bf)
        b1 = torch.randn(H, device=dev) * 0.1
        b2 = torch.randn(C, device=dev) * 0.1
        gam = torch.rand(C, device=dev) * 0.25 + 0.05
        x = torch.randn(M, C, device=dev)
        xo = torch.empty(M, C, device=dev)
        gh = torch.empty(M, H, device=dev, dtype=bf)
        a = torch.empty(M, H, device=dev, dtype=bf)
        if args.bwd and C in K.MLP_BWD_FUSED_C:
            bwd_case(name, M, C, args.iters, dev)
        for train in (True, False):
            nb = M * C * 10 + (2 * M * H * 2 if train else 0)
            floor = nb / HBM * 1e6
            fl = 4.0 * M * C * H
            if C in K.MLP_FUSED_C:
                tf = timed(lambda: K.mlp_fwd(y, w1, b1, w2, b2, gam, x, out=xo, gelu_grad=gh if train else None,
                                             gelu_out=a if train else None), args.iters)
            else:
                tf = float("nan")
            epi = nv.SV_EPI_BIAS_GELU_DUAL if train else nv.SV_EPI_BIAS_GELU
            t1 = timed(lambda: K.linear_fwd(y, w1, out=gh if train else a, out2=a if train else None, bias=b1,
                                            epilogue=epi), args.iters)
            t2 = timed(lambda: K.linear_fwd(a, w2, out=xo, bias=b2, gamma=gam, residual=x,
                                            epilogue=nv.SV_EPI_BIAS_GAMMA_RES), args.iters)
            print(f"{name:9s} {'train' if train else 'eval ':5s} fused {tf:7.1f} us ({nb / tf / 1e3:6.0f} GB/s, "
                  f"{fl / tf / 1e6:6.0f} TF/s) | fc1 {t1:6.1f} + fc2 {t2:6.1f} = {t1 + t2:6.1f} us | HBM floor "
                  f"{floor:6.1f} us", flush=True)


def bwd_case(name, M, C, iters, dev):
    bf = torch.bfloat16
    H = 4 * C
    d = (torch.randn(M, C, device=dev) * 0.1).to(bf)
    w1 = torch.randn(H, C, device=dev) * 0.08
    w2 = torch.randn(C, H, device=dev) * 0.05
    gam = torch.rand(C, device=dev) * 0.25 + 0.05
    gh = (torch.rand(M, H, device=dev) * 1.2 - 0.1).to(bf)
    z = torch.randn(M, C, device=dev).to(bf)
    mean = z.float().mean(1)
    rstd = 1.0 / torch.sqrt(z.float().var(1, unbiased=False) + 1e-6)
    lnw = torch.rand(C, device=dev) + 0.5
    w2t, w1t = K.transpose_scale_bf16(w2, gam), K.transpose_scale_bf16(w1)
    w2g, w1b = K.scale_rows_bf16(w2, gam), K.cast_bf16(w1)
    dh = torch.empty(M, H, device=dev, dtype=bf)
    dz = torch.empty(M, C, device=dev, dtype=bf)
    dy = torch.empty(M, C, device=dev, dtype=bf)
    dw, db = torch.zeros(C, device=dev), torch.zeros(C, device=dev)
    tf = timed(lambda: K.mlp_bwd(d, w2t, gh, w1t, z, mean, rstd, lnw, dh=dh, dz=dz), iters)
    t1 = timed(lambda: K.linear_dgrad(d, w2g, out=dh, epilogue=nv.SV_EPI_MUL_AUX, aux=gh), iters)
    t2 = timed(lambda: K.linear_dgrad(dh, w1b, out=dy), iters)
    t3 = timed(lambda: K.layernorm_bwd(dy, z, mean, rstd, lnw, dw=dw, db=db, out_dtype=bf), iters)
    nb = M * (C * 2 + H * 2 + C * 2 + H * 2 + C * 2 + 8)
    print(f"{name:9s} bwd   fused {tf:7.1f} us ({nb / tf / 1e3:6.0f} GB/s) | fc2 dgrad {t1:6.1f} + fc1 dgrad {t2:6.1f} + "
          f"ln bwd {t3:6.1f} = {t1 + t2 + t3:6.1f} us | HBM floor {nb / HBM * 1e6:6.1f} us", flush=True)


if __name__ == "__main__":
    main()
