"""Digest of the model after a few training steps (bench.py's synthetic workload and engine), for bitwise A/B checks
between two builds of the kernel library (SV_LIB_PATH): every parameter, after AdamW has applied every gradient, as
one sha256.  Two runs of one build must agree (the step is deterministic); a build that claims the same arithmetic must
agree with them.
    python tools/step_digest.py [--workload classification|localization] [--steps 3]"""
import argparse
import hashlib
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__  # noqa: E402
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="classification", choices=["classification", "localization"])
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--batch", type=int, default=None)
    a = ap.parse_args()
    __graft_entry__.load_package()
    from spine_vision_amd.training import Classifier, CoordinateRegressor, StepEngine

    dev = torch.device("cuda", 0)
    torch.manual_seed(42)
    cls = a.workload == "classification"
    if cls:
        from spine_vision_amd.training.trainers.classification import _create_tasks_for_training
        tasks = _create_tasks_for_training(target_labels=bench.CLS_TASKS, label_smoothing=0.1)
        model = Classifier("resnet50", tasks=tasks, pretrained=False, dropout=0.0, precision="bf16")
        B, S = a.batch or 32, 256
    else:
        model = CoordinateRegressor("convnext_base", pretrained=False, precision="bf16")
        B, S = a.batch or 8, 512
    model = model.to(dev).train()
    eng = StepEngine(model, dev, lr=1e-4, weight_decay=1e-5, grad_clip=1.0)
    losses = []
    if cls:
        img, tg = bench.synthetic_cls_batch(B, S, S, dev, 1234)
        for _ in range(a.steps):
            losses.append(float(eng.step_classification(img, tg)))
    else:
        img, co, mk = bench.synthetic_batch(B, S, S, dev, 1234)
        for _ in range(a.steps):
            losses.append(float(eng.step_localization(img, co, mk)))
    torch.cuda.synchronize()
    h = hashlib.sha256()
    for n, p in sorted(model.state_dict().items()):
        h.update(n.encode())
        h.update(p.detach().contiguous().cpu().reshape(-1).view(torch.uint8).numpy().tobytes() if p.numel() else b"")
    print(json.dumps({"lib": os.environ.get("SV_LIB_PATH", "default"), "workload": a.workload, "losses": losses,
                      "digest": h.hexdigest()}))


if __name__ == "__main__":
    main()
