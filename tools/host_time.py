"""Host enqueue cost of one training step (ConvNeXt-base localization, bs32 @512): wall time of the
Python step call without a device sync vs the synced step time, plus a cProfile of one step.

    python tools/host_time.py [--batch 32] [--profile]
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
ap.add_argument("--batch", type=int, default=32)
ap.add_argument("--profile", action="store_true")
args = ap.parse_args()
__graft_entry__.load_package()
from spine_vision_amd.training import CoordinateRegressor, StepEngine  # noqa: E402

dev = torch.device("cuda:0")
model = CoordinateRegressor("convnext_base", pretrained=False).to(dev).train()
eng = StepEngine(model, dev, lr=1e-4, weight_decay=1e-5, grad_clip=1.0)
img, coords, mask = bench.synthetic_batch(args.batch, 512, 512, dev, 1234)
for _ in range(3):
    eng.step_localization(img, coords, mask)
torch.cuda.synchronize()
for _ in range(3):
    t0 = time.perf_counter()
    eng.step_localization(img, coords, mask)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"host enqueue {1e3 * (t1 - t0):7.2f} ms   step (synced) {1e3 * (t2 - t0):7.2f} ms", flush=True)
if args.profile:
    pr = cProfile.Profile()
    pr.enable()
    eng.step_localization(img, coords, mask)
    pr.disable()
    torch.cuda.synchronize()
    pstats.Stats(pr).sort_stats("tottime").print_stats(25)
