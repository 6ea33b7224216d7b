"""Run the classification StepEngine trajectory (7 steps, ResNet) twice per mode (eager, graphed) and
report the first step whose loss differs and the worst final-parameter difference, within and across modes.
    python tools/graph_determinism.py [--backbone resnet18]"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import __graft_entry__  # noqa: E402

__graft_entry__.load_package()
from spine_vision_amd.training import Classifier, StepEngine  # noqa: E402
from spine_vision_amd.training.trainers.classification import _create_tasks_for_training  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--backbone", default="resnet18")
ap.add_argument("--steps", type=int, default=7)
args = ap.parse_args()
dev = torch.device("cuda:0")
tasks = _create_tasks_for_training(target_labels=["pfirrmann", "modic", "herniation"], label_smoothing=0.1)


def traj(graphed):
    torch.manual_seed(7)
    model = Classifier(args.backbone, tasks=tasks, pretrained=False, dropout=0.0, precision="bf16").to(dev).train()
    eng = StepEngine(model, dev, lr=1e-4, weight_decay=1e-5, grad_clip=1.0, cuda_graph=graphed)
    g = torch.Generator().manual_seed(3)
    losses, grads = [], []
    for step in range(args.steps):
        img = torch.rand(4, 3, 64, 64, generator=g).to(dev)
        tg = {"pfirrmann": torch.randint(0, 5, (4,), generator=g).to(dev),
              "modic": torch.randint(0, 4, (4,), generator=g).to(dev),
              "herniation": torch.randint(0, 2, (4,), generator=g).float().to(dev)}
        losses.append(float(eng.step_classification(img, tg)))
        torch.cuda.synchronize()
        grads.append({n: p.grad.detach().cpu().clone() for n, p in model.named_parameters()})
    return losses, grads


def cmp(tag, a, b):
    la, ga = a
    lb, gb = b
    first = next((i for i, (x, y) in enumerate(zip(la, lb)) if x != y), None)
    gfirst = None
    for i in range(len(ga)):
        errs = {n: ((ga[i][n] - gb[i][n]).norm() / (ga[i][n].norm() + 1e-30)).item() for n in ga[i]}
        w = max(errs.items(), key=lambda kv: kv[1])
        if w[1] > 0:
            gfirst = (i, w)
            break
    print(f"{tag}: first loss diff at step {first}; first gradient diff {gfirst}")


e1, e2 = traj(False), traj(False)
g1, g2 = traj(True), traj(True)
cmp("eager vs eager", e1, e2)
cmp("graph vs graph", g1, g2)
cmp("eager vs graph", e1, g1)
