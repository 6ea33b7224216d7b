"""Teacher-forced per-block backward: HIP block backward vs the fp32 oracle block fed the same input
and the same output gradient (diagnostic, GPU)."""
import copy
import sys

import torch

sys.path.insert(0, ".")
import __graft_entry__  # noqa: E402

__graft_entry__.load_package()
from oracle import resnet as orn  # noqa: E402
from oracle import weights as ow  # noqa: E402
from spine_vision_amd.backbone import create_resnet  # noqa: E402


def rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return float((a - b).norm() / (b.norm() + 1e-30))


for name, B, R in [("resnet18", 4, 64), ("resnet18", 16, 128), ("resnet50", 8, 128)]:
    for prec in ("fp32", "bf16"):
        ref = ow.fill_module(orn.create(name)).train()
        hip = create_resnet(name, precision=prec)
        hip.load_state_dict(ref.state_dict())
        hip = hip.cuda().train()
        img, _ = ow.classification_batch(B, R, R)
        with torch.no_grad():
            _, tape = hip._forward_impl(img.cuda(), save=True)
        rblocks = [b for b in ref.modules() if isinstance(b, (orn.BasicBlock, orn.Bottleneck))]
        line = []
        for i, (rb, hb, sb) in enumerate(zip(rblocks, hip.blocks(), tape.blocks)):
            x_in, out = sb[0], sb[3]
            xr = x_in.float().permute(0, 3, 1, 2).cpu().clone().requires_grad_(True)
            rbc = copy.deepcopy(rb)
            o = rbc(xr)
            d = torch.randn(o.shape, generator=torch.Generator().manual_seed(i))
            o.backward(d)
            for p in hb.parameters():
                p.grad = torch.zeros_like(p)
            dx = hip._block_backward(hb, sb, d.permute(0, 2, 3, 1).contiguous().cuda().to(hip.grad_dtype))
            e_dx = rel(dx.permute(0, 3, 1, 2), xr.grad)
            hp = dict(hb.named_parameters())
            e_p = {n: rel(hp[n].grad, p.grad) for n, p in rbc.named_parameters()}
            wn = max(e_p, key=e_p.get)
            line.append(f"b{i}: dx {e_dx:.1e} worst {wn} {e_p[wn]:.1e}")
        print(name, B, R, prec, " | ".join(line), flush=True)
