"""Uninitialised-read check for the HIP backward: run the same ResNet forward+backward twice, after filling
the caching allocator's free memory with NaN and with zeros; any gradient that differs (or is NaN) was
computed from memory no kernel wrote.
    python tools/poison_check.py [--backbone resnet18] [--size 64] [--batch 4]"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import __graft_entry__  # noqa: E402

__graft_entry__.load_package()
from spine_vision_amd.backbone import create_resnet, create_convnext  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--backbone", default="resnet18")
ap.add_argument("--size", type=int, default=64)
ap.add_argument("--batch", type=int, default=4)
ap.add_argument("--side", type=int, default=1)
args = ap.parse_args()
dev = torch.device("cuda:0")


def poison(val):
    torch.cuda.synchronize()
    big = [torch.full((1 << 28,), val, device=dev) for _ in range(8)]  # 8 GiB of large-pool blocks
    small = [torch.full((1 << 16,), val, device=dev) for _ in range(4096)]  # small-pool blocks
    torch.cuda.synchronize()
    del big, small


def run(val):
    torch.manual_seed(1)
    if args.backbone.startswith("resnet"):
        m = create_resnet(args.backbone, precision="bf16").to(dev).train()
        m.overlap_wgrad = bool(args.side)
    else:
        m = create_convnext(args.backbone, precision="bf16").to(dev).train()
    g = torch.Generator().manual_seed(2)
    x = torch.rand(args.batch, 3, args.size, args.size, generator=g).to(dev)
    poison(val)
    f = m(x)
    f.backward(torch.rand(f.shape, generator=g).to(dev) - 0.5)
    torch.cuda.synchronize()
    return {n: p.grad.detach().cpu().clone() for n, p in m.named_parameters()}


a = run(float("nan"))
b = run(0.0)
bad = []
for n in a:
    na = torch.isnan(a[n]).sum().item()
    d = ((a[n] - b[n]).norm() / (b[n].norm() + 1e-30)).item()
    if na or d > 0:
        bad.append((n, na, d))
print(f"{args.backbone} @{args.size} B{args.batch} side={args.side}: {len(bad)} of {len(a)} gradients differ")
for r in bad[:40]:
    print("  ", r)
