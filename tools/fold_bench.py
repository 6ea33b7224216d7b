"""Per-launch time of the BatchNorm fold kernels against the separate fold + apply launches (HIP events, median of
repeats of a graph of 20 launches), at the ResNet-50 bs32 256^2 shapes.  Knobs read by the library: SV_FOLD_MAX_GRID, SV_FOLD_DIAG.
    python tools/fold_bench.py"""
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


def timed(fn, n=20, reps=5):
    """GPU time per call: n calls captured in one graph, replayed (no host launch cost in the figure)"""
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph, stream=s):
            for _ in range(n):
                fn()
    torch.cuda.current_stream().wait_stream(s)
    graph.replay()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        graph.replay()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1e3 / n)
    ts.sort()
    return ts[len(ts) // 2]


g = torch.Generator().manual_seed(0)
for rows, C in [(524288, 64), (131072, 64), (131072, 256), (32768, 128), (32768, 512), (8192, 1024), (2048, 2048)]:
    y = torch.randn(rows, C, generator=g).to(dev, torch.bfloat16)
    P = (rows + 63) // 64
    part = torch.rand(P, 2, C, generator=g).to(dev)
    prm = ((torch.rand(C, generator=g) + 0.5).to(dev), torch.zeros(C, device=dev), 1e-5, 0.1, torch.zeros(C, device=dev),
           torch.ones(C, device=dev), torch.zeros((), dtype=torch.int64, device=dev))
    tf = timed(lambda: K.bn_act_fold(y, part, prm, relu=True, out_dtype=torch.bfloat16))

    def sep():
        m, r = K.bn_stats_from_partials(part, rows, running_mean=prm[4], running_var=prm[5], num_batches_tracked=prm[6])
        K.bn_act(y, m, r, prm[0], prm[1], relu=True, out_dtype=torch.bfloat16)

    ts = timed(sep)
    print(f"rows {rows:7d} C {C:5d} P {P:5d}: fold {tf:7.1f} us   finish+act {ts:7.1f} us", flush=True)
