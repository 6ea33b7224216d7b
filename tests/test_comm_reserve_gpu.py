"""Data-parallel readiness on one GPU: RCCL's all-reduce kernels run on a comm stream
beside the backward, whose persistent v9 GEMM workgroups hold a whole CU's LDS for the entire launch.  With
world > 1 StepEngine sets ``comm_reserve_cus`` (SV_COMM_RESERVE_CUS, default 32) and the backward's GEMM
grids leave that many CUs free.

The test stands in for RCCL with a proxy kernel (a torch reduction, which needs LDS like RCCL's kernels) on a
high-priority comm stream, launched the moment each block's gradients are reported ready in the ConvNeXt-base
bs32 512x512 backward.  It records, per launch, the time from the ready event to the proxy's completion minus
the proxy's standalone duration (its start latency), with every CU available to the GEMMs and with 32
reserved, and asserts the reserved schedule's p90 latency stays within the bound below.  Reference path:
accelerate DDP (spine_vision/training/trainers/base.py:253-266), NCCL/RCCL kernels on their own stream."""

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

RESERVED_P90_US = 60.0  # measured on MI355X: see DESIGN.md "Multi-GPU" (the print below)


def _latencies(dev, reserve):
    from spine_vision_amd.training import CoordinateRegressor, StepEngine

    torch.manual_seed(0)
    model = CoordinateRegressor("convnext_base", pretrained=False, precision="bf16").to(dev).train()
    eng = StepEngine(model, dev)
    model.backbone.comm_reserve_cus = reserve
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

    def hook(params):
        ev = torch.cuda.Event(enable_timing=True)
        ev.record()  # on the stream that made the gradients final
        comm.wait_event(ev)
        with torch.cuda.stream(comm):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            torch.sum(buf, dim=0, out=out)
            b.record()
        marks.append((ev, b))

    img = torch.randn(32, 3, 512, 512, device=dev)
    coords = torch.rand(32, 5, 2, device=dev)
    mask = torch.ones(32, 5, device=dev)
    for step in range(3):
        model.backbone.grad_ready_hook = hook if step == 2 else None
        eng.step_localization(img, coords, mask)
    torch.cuda.synchronize()
    lat = np.array([ev.elapsed_time(b) * 1e3 - alone_us for ev, b in marks])
    return alone_us, lat


def test_comm_stream_kernel_starts_with_reserved_cus(dev):
    res = {}
    for reserve in (0, 32):
        alone, lat = _latencies(dev, reserve)
        res[reserve] = (alone, lat)
        print(f"[comm] reserve {reserve:2d} CUs: proxy alone {alone:.1f} us; start latency over {len(lat)} "
              f"launches: median {np.median(lat):.1f} us, p90 {np.percentile(lat, 90):.1f} us, max {lat.max():.1f} us")
    assert len(res[32][1]) > 30
    assert np.percentile(res[32][1], 90) < RESERVED_P90_US
