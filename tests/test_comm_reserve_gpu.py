"""Data-parallel readiness on one GPU: RCCL's all-reduce kernels run on a comm
stream beside the backward, whose persistent v9 GEMM workgroups hold a whole CU's LDS for the entire launch, on
TWO streams at once (data gradients on the main stream, weight gradients on the side stream).

The test stands in for RCCL with a proxy kernel (a torch reduction, which needs LDS like RCCL's kernels) on a
high-priority comm stream, launched the moment each block's gradients are reported ready in the ConvNeXt-base
bs32 512x512 backward.  It records, per launch, the time from the ready event to the proxy's completion minus
the proxy's standalone duration (its start latency), for the default data-parallel setup (no CU reserve) and
for a 32-CU reserve by grid caps (round 3's mechanism, printed only), and bounds the default's median AND maximum.

Measured (profiles/round4/r7b_* .. r7h_*; rocprofv3 trace of this test, tools/comm_trace.py): the worst waits
follow readiness reports recorded on the MAIN stream -- the stage-transition downsample gradients -- and the
kernels that run meanwhile are the two streams' GEMMs, depthwise and fold kernels, with idle gaps on both compute
queues, so no single kernel class holds the CUs for the whole wait: a high-priority queue does not overtake
workgroups already handed to the dispatcher.  On a single busy stream the comm stream wakes in 14-19 us
(tools/event_wake_probe.py).  Grid caps (32 CUs) lower the median but not the tail (up to 2.9 ms) and cost
0.6-0.7 % of the step; CU-masked step streams (training/cumask.py) were worse (-12..-24 % step).  The default
reserves nothing; the median and the maximum are bounded here, and bench.py's data-parallel prediction charges
every bucket ready during the backward the measured worst latency.  Reference path: accelerate DDP
(spine_vision/training/trainers/base.py:253-266), NCCL/RCCL kernels on their own stream."""

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

# bounds on the default (no reserve) schedule; measured on MI355X over five boxes (the print below): median
# 36.7-186 us, p90 49.5-213 us, max 0.20-1.75 ms (the 128-workgroup weight gradients of round 4 included); with the
# optional 32-CU cap reserve median 22-30 us, max 0.26-2.9 ms
DEFAULT_MEDIAN_US = 300.0
DEFAULT_MAX_US = 5000.0


def _latencies(dev, reserve):
    from spine_vision_amd.training import CoordinateRegressor, StepEngine

    torch.manual_seed(0)
    model = CoordinateRegressor("convnext_base", pretrained=False, precision="bf16").to(dev).train()
    eng = StepEngine(model, dev, comm_reserve_cus=reserve)  # world 1, with the data-parallel CU reserve
    assert model.backbone.comm_reserve_cus == reserve
    comm = torch.cuda.Stream(device=dev, priority=-1)
    buf = torch.randn(1024, 1024, device=dev)
    out = torch.empty(1024, device=dev)
    with torch.cuda.stream(comm):  # standalone duration of the proxy
        for _ in range(3):
            torch.sum(buf, dim=0, out=out)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            torch.sum(buf, dim=0, out=out)
        e1.record()
    torch.cuda.synchronize()
    alone_us = e0.elapsed_time(e1) * 1e3 / 20
    marks = []

    names = {id(p): n for n, p in model.named_parameters()}

    def hook(params):
        ev = torch.cuda.Event(enable_timing=True)
        ev.record()  # on the stream that made the gradients final
        comm.wait_event(ev)
        with torch.cuda.stream(comm):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            torch.sum(buf, dim=0, out=out)
            b.record()
        marks.append((ev, b, names.get(id(params[0]), "?")))

    img = torch.randn(32, 3, 512, 512, device=dev)
    coords = torch.rand(32, 5, 2, device=dev)
    mask = torch.ones(32, 5, device=dev)
    for step in range(3):
        model.backbone.grad_ready_hook = hook if step == 2 else None
        eng.step_localization(img, coords, mask)
    torch.cuda.synchronize()
    lat = np.array([ev.elapsed_time(b) * 1e3 - alone_us for ev, b, _ in marks])
    worst = sorted(range(len(lat)), key=lambda i: -lat[i])[:3]
    print(f"[comm] reserve {reserve}: worst launches " + ", ".join(f"#{i} {marks[i][2]} {lat[i]:.0f} us" for i in worst))
    return alone_us, lat


def test_comm_stream_start_latency_default_no_reserve(dev):
    """Bounds the comm-stream kernel's start latency of the DEFAULT data-parallel schedule (no CU reserve: median and
    max); the 32-CU grid-cap reserve is measured and printed beside it for DESIGN.md, not asserted.  The default run's
    per-launch latencies are written to gpurun_out/comm_latency.json, which bench.py's dp_rehearsal reads (from
    profiles/, once committed) to charge every bucket the expected MAX over the ranks' draws."""
    import json
    import os

    res = {}
    for reserve in (0, 32):
        alone, lat = _latencies(dev, reserve)
        res[reserve] = (alone, lat)
        print(f"[comm] reserve {reserve:2d} CUs: proxy alone {alone:.1f} us; start latency over {len(lat)} "
              f"launches: median {np.median(lat):.1f} us, p90 {np.percentile(lat, 90):.1f} us, max {lat.max():.1f} us")
    lat0 = res[0][1]
    os.makedirs("gpurun_out", exist_ok=True)
    with open(os.path.join("gpurun_out", "comm_latency.json"), "w") as f:
        json.dump({"source": "tests/test_comm_reserve_gpu.py, ConvNeXt-base bs32 512x512 backward, reserve 0",
                   "proxy_alone_us": round(res[0][0], 2), "latency_us": [round(float(v), 2) for v in lat0]}, f)
    assert len(lat0) > 30
    assert np.median(lat0) < DEFAULT_MEDIAN_US and lat0.max() < DEFAULT_MAX_US, (np.median(lat0), lat0.max())
