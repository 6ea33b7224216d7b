"""Host-side cost of the ResNet-50 bf16 forward + backward kernel sequence, profiled in the main thread
(the autograd engine runs the backward on its device thread, out of cProfile's sight): times one
_forward_impl(save=True) + _backward_impl without device syncs, then a cProfile of the same.
    python tools/host_profile_resnet.py"""
import cProfile
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import __graft_entry__  # noqa: E402

__graft_entry__.load_package()
from spine_vision_amd.backbone import create_resnet  # noqa: E402

dev = torch.device("cuda:0")
m = create_resnet("resnet50", precision="bf16").to(dev).train()
x = torch.rand(32, 3, 256, 256, device=dev)


def once():
    with torch.no_grad():
        feat, tape = m._forward_impl(x, save=True)
        m._backward_impl(tape, torch.ones_like(feat))


for _ in range(3):
    once()
torch.cuda.synchronize()
for _ in range(3):
    t0 = time.perf_counter()
    once()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"host enqueue {1e3 * (t1 - t0):7.2f} ms   synced {1e3 * (t2 - t0):7.2f} ms")
pr = cProfile.Profile()
pr.enable()
once()
pr.disable()
torch.cuda.synchronize()
pstats.Stats(pr).sort_stats("tottime").print_stats(30)
