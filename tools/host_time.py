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
ap.add_argument("--workload", default="localization", choices=["localization", "classification"])
args = ap.parse_args()
__graft_entry__.load_package()
from spine_vision_amd.training import Classifier, CoordinateRegressor, StepEngine  # noqa: E402

dev = torch.device("cuda:0")
if args.workload == "classification":
    from spine_vision_amd.training.trainers.classification import _create_tasks_for_training  # noqa: E402

    tasks = _create_tasks_for_training(target_labels=bench.CLS_TASKS, label_smoothing=0.1)
    model = Classifier("resnet50", tasks=tasks, pretrained=False, dropout=0.3).to(dev).train()
    img, targets = bench.synthetic_cls_batch(args.batch, 256, 256, dev, 1234)
else:
    model = CoordinateRegressor("convnext_base", pretrained=False).to(dev).train()
    img, coords, mask = bench.synthetic_batch(args.batch, 512, 512, dev, 1234)
eng = StepEngine(model, dev, lr=1e-4, weight_decay=1e-5, grad_clip=1.0)


def one_step():
    if args.workload == "classification":
        return eng.step_classification(img, targets)
    return eng.step_localization(img, coords, mask)


for _ in range(3):
    one_step()
torch.cuda.synchronize()
for _ in range(3):
    t0 = time.perf_counter()
    one_step()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"host enqueue {1e3 * (t1 - t0):7.2f} ms   step (synced) {1e3 * (t2 - t0):7.2f} ms", flush=True)
if args.profile:
    pr = cProfile.Profile()
    pr.enable()
    one_step()
    pr.disable()
    torch.cuda.synchronize()
    pstats.Stats(pr).sort_stats("tottime").print_stats(25)
