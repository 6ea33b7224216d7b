"""Benchmark of the north-star hot path: one LocalizationTrainer training step
(forward -> backward -> RCCL gradient all-reduce -> clip(1.0) -> AdamW) of CoordinateRegressor
(ConvNeXt-base, 512x512, batch 32 per GPU, default head, masked SmoothL1) on synthetic uint8
images normalised like the reference's transforms, inputs already resident in HBM.

    python bench.py --gpus N --steps K --warmup W
    (N > 1: python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench.py)

Rank 0 prints ONE JSON line.  ``roofline`` times every launch of one GEMM class (the dominant
kernel) with HIP events on its own stream inside the timed region; ``cpu_baseline``
times the fp32 CPU restatement of the same step (oracle/, TEST INFRASTRUCTURE) on the host cores
over a bounded sample, rank 0 at N=1 only.
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import __graft_entry__  # noqa: E402

METRIC = "images/sec training, ConvNeXt-base 512x512 loc, bs32, at 1/2/4/8 MI355X"
PEAK_BF16_TFLOPS = 2516.6  # 256 CU x 4 SIMD x 1024 FLOP/clk (v_mfma_f32_32x32x16_bf16) x 2.4 GHz
PEAK_F32_MFMA_TFLOPS = 157.3
PROBE_KEYS = {"fwd": (True, True), "dgrad": (True, False), "wgrad": (False, False)}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=32, help="images per GPU")
    ap.add_argument("--image-size", type=int, default=512)
    ap.add_argument("--backbone", default="convnext_base")
    ap.add_argument("--precision", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--probe", default="fwd", choices=sorted(PROBE_KEYS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=15.0, help="bounded CPU sample budget")
    ap.add_argument("--traffic-file", default=os.path.join(ROOT, "profiles", "traffic.json"))
    return ap.parse_args()


def synthetic_batch(B, H, W, device, seed):
    """uint8 grayscale -> RGB replicate -> /255 -> ImageNet normalise (training/datasets/
    localization.py:196-254 of the reference), coords U(0.05,0.95), ~10% masked levels."""
    g = torch.Generator(device=device).manual_seed(seed)
    u8 = torch.randint(0, 256, (B, 1, H, W), generator=g, device=device, dtype=torch.uint8)
    x = (u8.float() / 255.0).expand(B, 3, H, W)
    mean = torch.tensor([0.485, 0.456, 0.406], device=device).view(1, 3, 1, 1)
    std = torch.tensor([0.229, 0.224, 0.225], device=device).view(1, 3, 1, 1)
    img = ((x - mean) / std).contiguous()
    coords = torch.rand(B, 5, 2, generator=g, device=device) * 0.9 + 0.05
    mask = (torch.rand(B, 5, generator=g, device=device) >= 0.1).float()
    return img, coords, mask


def cpu_baseline(args):
    """fp32 CPU restatement of the same training step (oracle/: TEST INFRASTRUCTURE, baseline only)."""
    from oracle import convnext as oc
    from oracle import heads as oh
    from oracle import step as ostep

    threads = min(16, os.cpu_count() or 1)
    torch.set_num_threads(threads)
    B = 4
    model = oh.CoordinateRegressor(oc.create(args.backbone), 1024 if args.backbone == "convnext_base" else 1536)
    model.train()
    opt = ostep.make_optimizer(model)
    img, coords, mask = synthetic_batch(B, args.image_size, args.image_size, "cpu", 7)
    ostep.train_step_localization(model, opt, img, coords, mask)  # warmup
    n, t0 = 0, time.perf_counter()
    while True:
        ostep.train_step_localization(model, opt, img, coords, mask)
        n += 1
        el = time.perf_counter() - t0
        if el >= args.cpu_seconds or n >= 8:
            break
    try:
        cpu_name = [ln.split(":", 1)[1].strip() for ln in open("/proc/cpuinfo") if ln.startswith("model name")][0]
    except Exception:  # pragma: no cover
        cpu_name = "unknown"
    return {
        "value": round(B * n / el, 4),
        "unit": "images/sec",
        "cores": threads,
        "kind": "port",
        "sample": f"{n} timed fp32 train steps (after 1 warmup) of {args.backbone} {args.image_size}x"
                  f"{args.image_size} bs{B} on {cpu_name}, torch eager CPU, oracle/ restatement",
    }


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    device = torch.device("cuda", local)

    pkg = __graft_entry__.load_package()
    from spine_vision_amd import kernels as K
    from spine_vision_amd.training import CoordinateRegressor, StepEngine

    torch.manual_seed(42)
    model = CoordinateRegressor(args.backbone, pretrained=False, precision=args.precision).to(device)
    model.train()
    engine = StepEngine(model, device, lr=1e-4, weight_decay=1e-5, grad_clip=1.0)
    img, coords, mask = synthetic_batch(args.batch, args.image_size, args.image_size, device, 1234 + rank)

    for _ in range(args.warmup):
        engine.step_localization(img, coords, mask)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()

    bf = args.precision == "bf16"
    probe = K.GemmProbe(PROBE_KEYS[args.probe] + (bf,))
    K.PROBE = probe
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = engine.step_localization(img, coords, mask)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    K.PROBE = None
    if world > 1:
        t = torch.tensor([elapsed], device=device, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    final_loss = float(loss.item())
    assert final_loss == final_loss, "loss is NaN"

    probe_ms = probe.elapsed_ms()
    avg_launch_ms = probe_ms / max(probe.launches, 1)
    flops_per_launch = probe.flops / max(probe.launches, 1)
    achieved = flops_per_launch / (avg_launch_ms * 1e-3) / 1e12 if probe.launches else 0.0
    peak = PEAK_BF16_TFLOPS if bf else PEAK_F32_MFMA_TFLOPS
    traffic = None
    if os.path.exists(args.traffic_file):
        try:
            traffic = json.load(open(args.traffic_file)).get(f"{args.probe}_bytes_per_launch")
        except Exception:
            traffic = None

    ms = elapsed / args.steps * 1e3
    value = world * args.batch * args.steps / elapsed
    step_tflops = 481.3 * args.batch / (ms * 1e-3) / 1e3 if args.backbone == "convnext_base" else None
    result = {
        "metric": METRIC,
        "value": round(value, 3),
        "unit": "images/sec",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": args.precision,
        "data": "synthetic uint8 512x512 grayscale->RGB, ImageNet-normalised, resident in HBM; random-init weights",
        "config": {
            "workload": f"CoordinateRegressor({args.backbone}) localization train step fwd+bwd+allreduce+clip+AdamW",
            "image_size": args.image_size,
            "batch_per_gpu": args.batch,
            "global_batch": args.batch * world,
            "parallelism": f"dp{world}",
        },
        "roofline": {
            "bound": "mfma",
            "kernel": f"gemm_kernel {args.probe} ({'bf16' if bf else 'f32'} MFMA)",
            "achieved": round(achieved, 2),
            "peak": peak,
            "unit": "TFLOP/s",
            "frac": round(achieved / peak, 4),
            "traffic": traffic,
            "launches_timed": probe.launches,
            "avg_launch_us": round(avg_launch_ms * 1e3, 2),
            "algorithmic_gflop_per_launch": round(flops_per_launch / 1e9, 3),
            "algorithmic_bytes_per_launch": int(probe.bytes / max(probe.launches, 1)),
            "step_tflops_per_gpu": round(step_tflops, 1) if step_tflops else None,
        },
        "loss": round(final_loss, 6),
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(args)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
