"""cProfile of the host side of one backbone forward (tape) + explicit backward, both on the calling
thread (autograd would run the backward on its device thread, invisible to cProfile).

    python tools/host_profile.py [--backbone resnet50|convnext_base] [--top 30]
"""

import argparse
import cProfile
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import __graft_entry__  # noqa: E402
import bench  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--backbone", default="resnet50")
ap.add_argument("--top", type=int, default=30)
args = ap.parse_args()
__graft_entry__.load_package()
from spine_vision_amd.training.models.backbone import BackboneFactory  # noqa: E402

dev = torch.device("cuda:0")
bb, F = BackboneFactory.create(args.backbone, False)
bb = bb.to(dev).train()
if args.backbone.startswith("resnet"):
    img, _ = bench.synthetic_cls_batch(32, 256, 256, dev, 1234)
else:
    img, _, _ = bench.synthetic_batch(32, 512, 512, dev, 1234)
dfeat = torch.randn(32, F, device=dev)


def once():
    feat, tape = bb._forward_impl(img, save=True)
    t1 = time.perf_counter()
    bb._backward_impl(tape, dfeat)
    return t1


for _ in range(3):
    once()
torch.cuda.synchronize()
for _ in range(3):
    t0 = time.perf_counter()
    t1 = once()
    t2 = time.perf_counter()
    torch.cuda.synchronize()
    print(f"host forward {1e3 * (t1 - t0):6.2f} ms  backward {1e3 * (t2 - t1):6.2f} ms  "
          f"device {1e3 * (time.perf_counter() - t0):6.2f} ms", flush=True)
pr = cProfile.Profile()
pr.enable()
once()
pr.disable()
torch.cuda.synchronize()
pstats.Stats(pr).sort_stats("tottime").print_stats(args.top)
