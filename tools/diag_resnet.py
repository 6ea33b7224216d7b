"""Per-block relative error of the HIP ResNet vs the fp32 oracle (diagnostic, GPU)."""
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


for name, B, R in [("resnet50", 4, 64), ("resnet50", 8, 128), ("resnet18", 4, 64)]:
    for prec in ("fp32", "bf16"):
        ref = ow.fill_module(orn.create(name)).train()
        hip = create_resnet(name, precision=prec)
        hip.load_state_dict(ref.state_dict())
        hip = hip.cuda().train()
        outs = []
        hooks = [b.register_forward_hook(lambda m, i, o: outs.append(o.detach())) for b in ref.modules()
                 if isinstance(b, (orn.BasicBlock, orn.Bottleneck))]
        stem = []
        ref.maxpool.register_forward_hook(lambda m, i, o: stem.append(o.detach()))
        img, _ = ow.classification_batch(B, R, R)
        with torch.no_grad():
            f_ref = ref(img)
            f_hip, tape = hip._forward_impl(img.cuda(), save=True)
        errs = [rel(tape.blocks[0][0].permute(0, 3, 1, 2), stem[0])]
        for (x_in, saved, ds, out), o in zip(tape.blocks, outs):
            errs.append(rel(out.permute(0, 3, 1, 2), o))
        print(name, B, R, prec, "feat", f"{rel(f_hip, f_ref):.2e}", "stem+blocks", " ".join(f"{e:.1e}" for e in errs),
              flush=True)
