"""Standalone timing of the ConvNeXt-base @512 bs32 GEMM shapes through sv_gemm (HIP events).

    python tools/gemm_bench.py [--stages S3] [--iters 20]
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

STAGES = {"S1": (524288, 128), "S2": (131072, 256), "S3": (32768, 512), "S4": (8192, 1024),
          "BIG": (16384, 2048)}  # BIG: a long-K calibration shape (fc1 dgrad K 8192), not in the model


def cases(M, C, dev, P):
    """P: a one-element list holding the per-call GEMM policy the lambdas pass (set per impl by main)."""
    bf = torch.bfloat16
    y = torch.randn(M, C, device=dev).to(bf)
    w1 = (torch.randn(4 * C, C, device=dev) * 0.05).to(bf)
    w2 = (torch.randn(C, 4 * C, device=dev) * 0.05).to(bf)
    b1 = torch.zeros(4 * C, device=dev)
    b2 = torch.zeros(C, device=dev)
    gam = torch.ones(C, device=dev)
    h = torch.randn(M, 4 * C, device=dev).to(bf)
    a = torch.randn(M, 4 * C, device=dev).to(bf)
    x = torch.randn(M, C, device=dev)
    d = torch.randn(M, C, device=dev).to(bf)
    dh = torch.randn(M, 4 * C, device=dev).to(bf)
    outh = torch.empty(M, 4 * C, device=dev, dtype=bf)
    outa = torch.empty_like(outh)
    out = torch.empty(M, C, device=dev)
    fl = 2.0 * M * C * 4 * C
    return [
        ("fc1_fwd(gelu2)", fl, lambda: K.linear_fwd(y, w1, out=outh, out2=outa, bias=b1, epilogue=nv.SV_EPI_BIAS_GELU2, policy=P[0])),
        ("fc1_fwd(dual)", fl, lambda: K.linear_fwd(y, w1, out=outh, out2=outa, bias=b1,
                                                  epilogue=nv.SV_EPI_BIAS_GELU_DUAL, policy=P[0])),
        ("fc1_fwd(store)", fl, lambda: K.linear_fwd(y, w1, out=outh, bias=b1, policy=P[0])),
        ("fc2_fwd(res)", fl, lambda: K.linear_fwd(a, w2, out=out, bias=b2, gamma=gam, residual=x,
                                                 epilogue=nv.SV_EPI_BIAS_GAMMA_RES, policy=P[0])),
        ("fc2_dgrad(gelu')", fl, lambda: K.linear_dgrad(d, w2, out=outh, epilogue=nv.SV_EPI_GELU_GRAD, aux=h, policy=P[0])),
        ("fc2_dgrad(mul)", fl, lambda: K.linear_dgrad(d, w2, out=outh, epilogue=nv.SV_EPI_MUL_AUX, aux=h, policy=P[0])),
        ("fc1_dgrad", fl, lambda: K.linear_dgrad(dh, w1, out=out, policy=P[0])),
        ("fc2_wgrad", fl, lambda: K.linear_wgrad(d, a, policy=P[0])),
        ("fc2_wgrad+bias", fl, lambda: K.linear_wgrad(d, a, bias_out=b2, bias_accumulate=False, policy=P[0])),
        ("fc1_wgrad", fl, lambda: K.linear_wgrad(dh, y, policy=P[0])),
        # calibration: the vendor library (hipBLASLt via torch.matmul) on the same shapes, plain store
        ("torch_fc1_fwd", fl, lambda: torch.matmul(y, w1.t(), out=outh)),
        ("torch_fc2_fwd", fl, lambda: torch.matmul(a, w2.t())),
        ("torch_fc1_dgrad", fl, lambda: torch.matmul(dh, w1)),
        ("torch_fc1_wgrad", fl, lambda: torch.matmul(dh.t(), y)),
    ]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--stages", default="S1,S2,S3,S4")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--cases", default="", help="comma-separated case-name substrings to run")
    ap.add_argument("--impls", default="0", help="comma-separated sv_gemm_policy.impl values, timed interleaved")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    for st in args.stages.split(","):
        M, C = STAGES[st]
        P = [None]
        for name, fl, fn in cases(M, C, dev, P):
            if args.cases and not any(c in name for c in args.cases.split(",")):
                continue
            impls = [int(x) for x in args.impls.split(",")] if not name.startswith("torch") else [0]
            res = {i: [] for i in impls}
            for rnd in range(2):
                for impl in impls:
                    P[0] = nv.policy(impl=impl)
                    for _ in range(3):
                        fn()
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    torch.cuda.synchronize()
                    e0.record()
                    for _ in range(args.iters):
                        fn()
                    e1.record()
                    torch.cuda.synchronize()
                    res[impl].append(e0.elapsed_time(e1) / args.iters * 1e3)
            line = " | ".join(f"impl{i} {min(v):7.1f} us {fl / min(v) / 1e6:7.1f} TF" for i, v in res.items())
            print(f"{st} M={M:7d} C={C:5d} {name:18s} {line}", flush=True)


if __name__ == "__main__":
    main()
