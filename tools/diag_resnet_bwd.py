"""bf16 ResNet gradient error vs the fp32 oracle at two batch/resolution sizes (diagnostic, GPU)."""
import sys

import torch

sys.path.insert(0, ".")
import __graft_entry__  # noqa: E402

__graft_entry__.load_package()
from oracle import resnet as orn  # noqa: E402
from oracle import weights as ow  # noqa: E402
from spine_vision_amd.backbone import create_resnet  # noqa: E402


def rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return float((a - b).norm() / (b.norm() + 1e-30))


for name, B, R in [("resnet18", 4, 64), ("resnet18", 16, 128), ("resnet18", 32, 224)]:
    for prec in ("fp32", "bf16"):
        ref = ow.fill_module(orn.create(name)).train()
        hip = create_resnet(name, precision=prec)
        hip.load_state_dict(ref.state_dict())
        hip = hip.cuda().train()
        img, _ = ow.classification_batch(B, R, R)
        f_ref = ref(img)
        f_hip = hip(img.cuda())
        dfeat = torch.from_numpy(ow.uniform("dfeat", f_ref.numel(), -1, 1).reshape(f_ref.shape))
        f_ref.backward(dfeat)
        f_hip.backward(dfeat.cuda())
        hp = dict(hip.named_parameters())
        errs = [(n, rel(hp[n].grad, p.grad)) for n, p in ref.named_parameters()]
        by_layer = {}
        for n, e in errs:
            k = n.split(".")[0]
            by_layer[k] = max(by_layer.get(k, 0), e)
        print(name, B, R, prec, f"feat {rel(f_hip, f_ref):.2e}", {k: f"{v:.1e}" for k, v in by_layer.items()}, flush=True)
