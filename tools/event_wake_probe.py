"""How fast does a high-priority stream wake on an event recorded on a busy stream?  (DESIGN.md "Multi-GPU":
the comm-stream start latency tail follows readiness reports recorded on the backward's MAIN stream.)

A producer stream runs a chain of N kernels (the ConvNeXt backward's v9 data-gradient GEMM at S3, or a short
elementwise kernel); after kernel k an event is recorded and a consumer stream (priority high / normal) waits
on it and runs a small reduction.  Latency = consumer end - event timestamp - consumer alone.  Variants: the
producer chain with a side stream also busy, the event timing-enabled or not (measured through a second
timing event recorded right after it).

    python tools/event_wake_probe.py
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import __graft_entry__  # noqa: E402

__graft_entry__.load_package()
from spine_vision_amd import kernels as K  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    bf = torch.bfloat16
    M, C = 32768, 512
    dh = torch.randn(M, 4 * C, device=dev).to(bf)
    w1 = (torch.randn(4 * C, C, device=dev) * 0.05).to(bf)
    dy = torch.empty(M, C, device=dev, dtype=bf)
    small = torch.randn(1 << 20, device=dev)
    buf = torch.randn(1024, 1024, device=dev)
    red = torch.empty(1024, device=dev)

    def gemm():
        K.linear_dgrad(dh, w1, out=dy)

    def elem():
        small.mul_(1.0000001)

    for prio in (-1, 0):
        comm = torch.cuda.Stream(device=dev, priority=prio)
        with torch.cuda.stream(comm):
            for _ in range(5):
                torch.sum(buf, dim=0, out=red)
            a0, a1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a0.record()
            for _ in range(20):
                torch.sum(buf, dim=0, out=red)
            a1.record()
        torch.cuda.synchronize()
        alone = a0.elapsed_time(a1) * 1e3 / 20
        for kname, kern, n in (("v9 dgrad S3", gemm, 60), ("elementwise 4 MB", elem, 400)):
            for timing in (True, False):
                lat = []
                for rep in range(6):
                    torch.cuda.synchronize()
                    marks = []
                    for i in range(n):
                        kern()
                        if i % (n // 6) == n // 12:
                            ev = torch.cuda.Event(enable_timing=timing)
                            ev.record()
                            t = torch.cuda.Event(enable_timing=True)
                            t.record()  # the producer's timestamp right after ev
                            comm.wait_event(ev)
                            with torch.cuda.stream(comm):
                                torch.sum(buf, dim=0, out=red)
                                b = torch.cuda.Event(enable_timing=True)
                                b.record()
                            marks.append((t, b))
                    torch.cuda.synchronize()
                    if rep:
                        lat += [t.elapsed_time(b) * 1e3 - alone for t, b in marks]
                lat = np.array(lat)
                print(f"comm prio {prio:2d}  producer {kname:18s} event timing={timing!s:5s}: latency median "
                      f"{np.median(lat):7.1f} us  p90 {np.percentile(lat, 90):7.1f}  max {lat.max():7.1f}  (n={len(lat)})",
                      flush=True)


if __name__ == "__main__":
    main()
