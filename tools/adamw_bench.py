"""GPU time of the flat AdamW update at ConvNeXt-base's parameter count (88.6 M), graph-replayed (no host cost),
(r11p: 550-555 us = 4.8 TB/s of the 2.66 GB it moves; two float4 groups per lane per round with non-temporal
stores measured the same, 545-553 us, and the step no different: not kept).
    python tools/adamw_bench.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__  # noqa: E402

__graft_entry__.load_package()
from spine_vision_amd import kernels as K  # noqa: E402

if not torch.cuda.is_available():
    sys.exit("no GPU")
dev = torch.device("cuda", 0)
n = 88_591_464
g = torch.Generator(device=dev).manual_seed(0)
p = torch.randn(n, device=dev, generator=g)
gr = torch.randn(n, device=dev, generator=g) * 1e-2
m = torch.randn(n, device=dev, generator=g) * 1e-3
v = torch.rand(n, device=dev, generator=g) * 1e-5
pb = torch.empty(n, device=dev, dtype=torch.bfloat16)


def step():
    K.adamw_flat(p, gr, m, v, pb, lr=1e-4, beta1=0.9, beta2=0.999, eps=1e-8, weight_decay=1e-5, step=10)


s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    step()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph, stream=s):
        for _ in range(10):
            step()
torch.cuda.current_stream().wait_stream(s)
ts = []
for _ in range(5):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    graph.replay()
    b.record()
    b.synchronize()
    ts.append(a.elapsed_time(b) * 100)
ts.sort()
us = ts[2]
nbytes = n * (16 + 12 + 2)
print(f"adamw_flat: {us:.1f} us per update, {nbytes / us / 1e3:.0f} GB/s "
      f"(algorithmic {nbytes / 1e9:.2f} GB)", flush=True)
