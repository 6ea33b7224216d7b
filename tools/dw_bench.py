"""Standalone timing of the depthwise-conv kernels at the ConvNeXt-base @512 bs32 stage shapes
(HIP events).

    python tools/dw_bench.py [--stages S1,S3] [--iters 20]
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

STAGES = {"S1": (128, 128), "S2": (64, 256), "S3": (32, 512), "S4": (16, 1024)}


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
    ap.add_argument("--stages", default="S1,S2,S3,S4")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--batch", type=int, default=32)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    tag = "ring"
    B = args.batch
    for st in args.stages.split(","):
        S, C = STAGES[st]
        x = torch.randn(B, S, S, C, device=dev)
        w = torch.randn(C, 49, device=dev) * 0.1
        bias = torch.zeros(C, device=dev)
        z = torch.empty(B, S, S, C, device=dev, dtype=torch.bfloat16)
        dz = torch.randn(B, S, S, C, device=dev)
        dzb = dz.to(torch.bfloat16)
        dx = torch.zeros(B, S, S, C, device=dev)
        dxb = torch.empty(B, S, S, C, device=dev, dtype=torch.bfloat16)
        n = B * S * S * C
        P = nv.value("sv_dwconv7_bwd_weight_nparts", B, S, S, C)
        pw = torch.empty(P * C * 49, device=dev)
        pb = torch.empty(P * C, device=dev)

        def fwd():  # dwconv only (the LN half of sv_dwconv7_ln_fwd is timed by ln below)
            nv.call("sv_dwconv7_bwd_data", nv.ptr(x), nv.SV_F32, nv.ptr(w), nv.ptr(dx), None, 0, B, S, S, C)

        cases = [
            ("bwd_data f32 acc+bf16", 4 * n + 4 * n + 4 * n + 2 * n,
             lambda: K.dwconv7_bwd_data(dz, w, dx, accumulate=True, dx_bf16=dxb)),
            ("bwd_data bf16dz acc+bf16", 2 * n + 4 * n + 4 * n + 2 * n,
             lambda: K.dwconv7_bwd_data(dzb, w, dx, accumulate=True, dx_bf16=dxb)),
            ("conv f32->f32 (no acc)", 8 * n, fwd),
            ("wgrad f32 (kernel only)", 8 * n,
             lambda: nv.call("sv_dwconv7_bwd_weight", nv.ptr(dz), nv.SV_F32, nv.ptr(x), nv.SV_F32, nv.ptr(pw),
                             nv.ptr(pb), B, S, S, C)),
            ("wgrad bf16dz (kernel only)", 6 * n,
             lambda: nv.call("sv_dwconv7_bwd_weight", nv.ptr(dzb), nv.SV_BF16, nv.ptr(x), nv.SV_F32, nv.ptr(pw),
                             nv.ptr(pb), B, S, S, C)),
        ]
        lnw = torch.ones(C, device=dev)
        y = torch.empty(B * S * S, C, device=dev, dtype=torch.bfloat16)
        mean = torch.empty(B * S * S, device=dev)
        rstd = torch.empty_like(mean)
        cases.append(("fwd f32->bf16 + LN", 4 * n + 2 * n + 2 * n + 2 * n,
                      lambda: nv.call("sv_dwconv7_ln_fwd", nv.ptr(x), nv.SV_F32, nv.ptr(w), nv.ptr(bias), nv.ptr(lnw),
                                      nv.ptr(bias), 1e-6, nv.ptr(z), nv.SV_BF16, nv.ptr(y), nv.SV_BF16, nv.ptr(mean),
                                      nv.ptr(rstd), B, S, S, C)))
        if nv.value("sv_dwconv7_ln_fused_ok", B, S, S, C, nv.SV_F32, nv.SV_BF16, nv.SV_BF16):
            cases.append(("one-pass f32->bf16 y (eval)", 4 * n + 2 * n,
                          lambda: nv.call("sv_dwconv7_ln_fwd", nv.ptr(x), nv.SV_F32, nv.ptr(w), nv.ptr(bias), nv.ptr(lnw),
                                          nv.ptr(bias), 1e-6, None, nv.SV_BF16, nv.ptr(y), nv.SV_BF16, nv.ptr(mean),
                                          nv.ptr(rstd), B, S, S, C)))
        # the matrix-core kernels (csrc/dwmfma.hip, round 6): bf16 operands
        cases.append(("mfma fwd f32->bf16", 6 * n,
                      lambda: nv.call("sv_dwconv7_fwd_mfma", nv.ptr(x), nv.SV_F32, nv.ptr(w), nv.ptr(bias), nv.ptr(z),
                                      B, S, S, C)))

        def mfma_fwd_ln():
            nv.call("sv_dwconv7_fwd_mfma", nv.ptr(x), nv.SV_F32, nv.ptr(w), nv.ptr(bias), nv.ptr(z), B, S, S, C)
            nv.call("sv_layernorm_fwd", nv.ptr(z), nv.SV_BF16, nv.ptr(lnw), nv.ptr(bias), nv.ptr(y), nv.SV_BF16,
                    nv.ptr(mean), nv.ptr(rstd), B * S * S, C, 1e-6)
        cases.append(("mfma fwd f32->bf16 + LN", 4 * n + 2 * n + 2 * n + 2 * n, mfma_fwd_ln))
        cases.append(("mfma bwd_data bf16dz acc+bf16", 2 * n + 4 * n + 4 * n + 2 * n,
                      lambda: nv.call("sv_dwconv7_bwd_data_mfma", nv.ptr(dzb), nv.ptr(w), nv.ptr(dx), nv.ptr(dxb), 1,
                                      B, S, S, C)))
        Pm = nv.value("sv_dwconv7_bwd_weight_mfma_nparts", B, S, S, C)
        pwm = torch.empty(Pm * C * 49, device=dev)
        pbm = torch.empty(Pm * C, device=dev)
        cases.append(("mfma wgrad bf16dz (kernel only)", 6 * n,
                      lambda: nv.call("sv_dwconv7_bwd_weight_mfma", nv.ptr(dzb), nv.ptr(x), nv.SV_F32, nv.ptr(pwm),
                                      nv.ptr(pbm), B, S, S, C)))
        for name, nbytes, fn in cases:
            us = timeit(fn, args.iters)
            print(f"{tag} {st} {name:28s} {us:8.1f} us  {nbytes / us / 1e3:7.1f} GB/s", flush=True)


if __name__ == "__main__":
    main()
