"""Does a comm-stream kernel find a free CU while the backward's GEMMs run?  (DESIGN.md "Multi-GPU", VERDICT r3
weak 6.)  A high-priority "comm" stream launches a small LDS-using proxy (a torch column reduction, as RCCL's
kernels use LDS) the moment a GEMM on a compute stream completes, while more persistent v9 GEMMs stay queued
behind it; the proxy's start latency is (its end - the GEMM's completion event) - its standalone time.

Schedules:
  full        one compute stream, grids on every CU
  cap         one compute stream, every grid capped at CUs - reserve (the round-3 mechanism)
  cap2        TWO compute streams (data + weight gradients, as the lean backward runs them), each capped
  mask*       compute stream(s) created with hipExtStreamCreateWithCUMask excluding `reserve` CUs (and the grids
              capped to the unmasked count), in two bit patterns: the last `reserve` bits, or every k-th bit

    python tools/cu_mask_probe.py [--reserve 32] [--reps 20]
"""

import argparse
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import __graft_entry__  # noqa: E402

__graft_entry__.load_package()
from spine_vision_amd import kernels as K  # noqa: E402
from spine_vision_amd import native as nv  # noqa: E402
from spine_vision_amd.training.cumask import masked_stream, reserve_bits  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reserve", type=int, default=32)
    ap.add_argument("--reps", type=int, default=20)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    ncu = torch.cuda.get_device_properties(dev).multi_processor_count
    bf = torch.bfloat16
    M, C = 524288 // 4, 128  # S1 fc1 (GELU dual) at bs8: 1024 v9 tiles, ~80 us
    y = torch.randn(M, C, device=dev).to(bf)
    w1 = (torch.randn(4 * C, C, device=dev) * 0.05).to(bf)
    b1 = torch.zeros(4 * C, device=dev)
    o1 = torch.empty(M, 4 * C, device=dev, dtype=bf)
    o2 = torch.empty_like(o1)
    o3 = torch.empty_like(o1)
    o4 = torch.empty_like(o1)
    comm = torch.cuda.Stream(device=dev, priority=-1)
    buf = torch.randn(1024, 1024, device=dev)
    red = torch.empty(1024, device=dev)
    with torch.cuda.stream(comm):
        for _ in range(3):
            torch.sum(buf, dim=0, out=red)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            torch.sum(buf, dim=0, out=red)
        e1.record()
    torch.cuda.synchronize()
    alone = e0.elapsed_time(e1) * 1e3 / 20

    def gemm(out, pol):
        K.linear_fwd(y, w1, out=out, out2=o2 if out is o1 else o4, bias=b1, epilogue=nv.SV_EPI_BIAS_GELU_DUAL,
                     policy=pol)

    def run(streams, cap):
        pol = nv.policy(grid_cap=cap)
        lat, gem = [], []
        for rep in range(args.reps):
            torch.cuda.synchronize()
            evs = []
            for si, s in enumerate(streams):
                with torch.cuda.stream(s):
                    out = o1 if si == 0 else o3
                    g0 = torch.cuda.Event(enable_timing=True)
                    g0.record()
                    gemm(out, pol)
                    ready = torch.cuda.Event(enable_timing=True)
                    ready.record()
                    for _ in range(4):  # more persistent GEMMs queued behind the reported one
                        gemm(out, pol)
                    g1 = torch.cuda.Event(enable_timing=True)
                    g1.record()
                    evs.append((g0, ready, g1))
            comm.wait_event(evs[0][1])
            with torch.cuda.stream(comm):
                b = torch.cuda.Event(enable_timing=True)
                torch.sum(buf, dim=0, out=red)
                b.record()
            torch.cuda.synchronize()
            lat.append(evs[0][1].elapsed_time(b) * 1e3 - alone)
            gem.append(evs[0][0].elapsed_time(evs[0][2]) * 1e3 / 5)
        lat = np.array(lat[2:])
        return np.median(lat), np.percentile(lat, 90), lat.max(), np.median(gem[2:])

    default = torch.cuda.current_stream()
    side = torch.cuda.Stream(device=dev)
    keep = ncu - args.reserve
    cases = [("full", [default], 0), ("cap", [default], keep), ("cap2", [default, side], keep),
             ("cap2 halves", [default, side], keep // 2)]
    for pat in ("tail", "strided"):
        bits = reserve_bits(ncu, args.reserve, pat)
        m1, m2 = masked_stream(dev, bits), masked_stream(dev, bits)
        cases += [(f"mask {pat}", [m1], keep), (f"mask2 {pat}", [m1, m2], keep)]
    print(f"proxy alone {alone:.1f} us; {ncu} CUs, reserve {args.reserve}")
    for name, streams, cap in cases:
        med, p90, mx, g = run(streams, cap)
        print(f"{name:18s} grid cap {cap:3d}: start latency median {med:8.1f} us  p90 {p90:8.1f}  max {mx:8.1f}; "
              f"GEMM {g:7.1f} us per launch", flush=True)


if __name__ == "__main__":
    main()
