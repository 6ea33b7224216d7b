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
PEAK_HBM_GBS = 8000.0  # MI355X HBM3E (guide: ~8 TB/s)
PROBE_KEYS = {"fwd": (True, True), "dgrad": (True, False), "wgrad": (False, False)}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="localization", choices=["localization", "classification"],
                    help="localization = the BASELINE metric (ConvNeXt-base 512); classification = ResNet-50 "
                         "256x256 3-head ClassificationTrainer step (configs[3], secondary line)")
    ap.add_argument("--batch", type=int, default=32, help="images per GPU")
    ap.add_argument("--image-size", type=int, default=None, help="default 512 (localization) / 256 (classification)")
    ap.add_argument("--backbone", default=None, help="default convnext_base / resnet50")
    ap.add_argument("--precision", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--probe", default="fwd", choices=sorted(PROBE_KEYS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--inference", action="store_true",
                    help="secondary line (row f2): the validation / predict forward (eval mode, no tape) instead "
                         "of the training step")
    ap.add_argument("--cpu-seconds", type=float, default=15.0, help="bounded CPU sample budget")
    ap.add_argument("--traffic-file", default=os.path.join(ROOT, "profiles", "traffic.json"))
    args = ap.parse_args()
    cls = args.workload == "classification"
    if args.image_size is None:
        args.image_size = 256 if cls else 512
    if args.backbone is None:
        args.backbone = "resnet50" if cls else "convnext_base"
    return args


# fwd+bwd GFLOP per image (counted with torch.utils.flop_counter)
STEP_GFLOP = {("convnext_base", 512): 481.3, ("convnext_large", 512): 1077.0, ("resnet50", 256): 31.7,
              ("resnet18", 256): 13.9}
CLS_TASKS = ["pfirrmann", "modic", "herniation"]


def synthetic_cls_batch(B, H, W, device, seed):
    """[T2, T1, T2] uint8 planes -> /255 -> ImageNet normalise (reference datasets/classification.py
    crops), labels pfirrmann U{0..4}, modic U{0..3}, herniation Bernoulli(0.3)."""
    g = torch.Generator(device=device).manual_seed(seed)
    u8 = torch.randint(0, 256, (B, 2, H, W), generator=g, device=device, dtype=torch.uint8)
    x = (u8.float() / 255.0)[:, [0, 1, 0]]
    mean = torch.tensor([0.485, 0.456, 0.406], device=device).view(1, 3, 1, 1)
    std = torch.tensor([0.229, 0.224, 0.225], device=device).view(1, 3, 1, 1)
    img = ((x - mean) / std).contiguous()
    targets = {"pfirrmann": torch.randint(0, 5, (B,), generator=g, device=device),
               "modic": torch.randint(0, 4, (B,), generator=g, device=device),
               "herniation": (torch.rand(B, generator=g, device=device) < 0.3).float()}
    return img, targets


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
    if args.workload == "classification":
        from oracle import resnet as orn

        model = oh.Classifier(orn.create(args.backbone), 2048 if args.backbone == "resnet50" else 512, dropout=0.3)
        img, targets = synthetic_cls_batch(B, args.image_size, args.image_size, "cpu", 7)
        opt = ostep.make_optimizer(model)

        def one():
            ostep.train_step_classification(model, opt, img, targets)
    else:
        model = oh.CoordinateRegressor(oc.create(args.backbone), 1024 if args.backbone == "convnext_base" else 1536)
        img, coords, mask = synthetic_batch(B, args.image_size, args.image_size, "cpu", 7)
        opt = ostep.make_optimizer(model)

        def one():
            ostep.train_step_localization(model, opt, img, coords, mask)
    model.train()
    one()  # warmup
    n, t0 = 0, time.perf_counter()
    while True:
        one()
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
    from spine_vision_amd.training import Classifier, CoordinateRegressor, StepEngine

    torch.manual_seed(42)
    cls = args.workload == "classification"
    if cls:
        from spine_vision_amd.training.trainers.classification import _create_tasks_for_training

        tasks = _create_tasks_for_training(target_labels=CLS_TASKS, label_smoothing=0.1)
        model = Classifier(args.backbone, tasks=tasks, pretrained=False, dropout=0.3, precision=args.precision)
    else:
        model = CoordinateRegressor(args.backbone, pretrained=False, precision=args.precision)
    model = model.to(device).train()
    engine = StepEngine(model, device, lr=1e-4, weight_decay=1e-5, grad_clip=1.0)
    if cls:
        img, targets = synthetic_cls_batch(args.batch, args.image_size, args.image_size, device, 1234 + rank)

        def run_step():
            return engine.step_classification(img, targets)
    else:
        img, coords, mask = synthetic_batch(args.batch, args.image_size, args.image_size, device, 1234 + rank)

        def run_step():
            return engine.step_localization(img, coords, mask)

    if args.inference:  # row f2: trainers' _validate_epoch / predict forward, no autograd tape
        model.eval()
        train_step = run_step

        def run_step():
            with torch.no_grad():
                out = model(img)
            return out.float().mean() if not isinstance(out, dict) else sum(v.float().mean() for v in out.values())

        del train_step
    for _ in range(args.warmup):
        run_step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()

    bf = args.precision == "bf16"
    probe = K.GemmProbe(PROBE_KEYS[args.probe] + (bf,))
    # The probe's HIP events bracket every launch of the class in the LAST timed step: each timing event
    # is a release packet that writes back L2, and probing all K steps cost 2.3% of the step
    # (tools/gpu_probe_ab.sh).  The classification line reports the whole-step rate and takes no probe;
    # SV_BENCH_PROBE=0 leaves the roofline fields empty and SV_BENCH_PROBE=all probes every step.
    probe_mode = os.environ.get("SV_BENCH_PROBE", "1")
    use_probe = not cls and probe_mode != "0"
    t0 = time.perf_counter()
    for i in range(args.steps):
        K.PROBE = probe if use_probe and (probe_mode == "all" or i == args.steps - 1) else None
        loss = run_step()
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
    gflop = STEP_GFLOP.get((args.backbone, args.image_size))
    step_tflops = gflop * args.batch / (ms * 1e-3) / 1e3 if gflop else None
    if args.inference:
        metric = f"images/sec inference (eval forward), {args.backbone} {args.image_size}x{args.image_size}, bs{args.batch}"
        workload = f"{'Classifier' if cls else 'CoordinateRegressor'}({args.backbone}) eval forward (validation / predict)"
        data = "synthetic, resident in HBM; random-init weights"
        gflop = STEP_GFLOP.get((args.backbone, args.image_size))
        step_tflops = (gflop / 3.0) * args.batch / (ms * 1e-3) / 1e3 if gflop else None  # fwd = 1/3 of fwd+bwd
    elif cls:
        metric = f"images/sec training, {args.backbone} {args.image_size}x{args.image_size} 3-head cls, bs{args.batch}"
        workload = f"Classifier({args.backbone}, pfirrmann+modic+herniation) train step fwd+bwd+allreduce+clip+AdamW"
        data = (f"synthetic uint8 {args.image_size}x{args.image_size} [T2,T1,T2] crops, ImageNet-normalised, "
                "resident in HBM; random-init weights")
    else:
        metric = METRIC
        if (args.backbone, args.image_size, args.batch) != ("convnext_base", 512, 32):
            metric = f"images/sec training, {args.backbone} {args.image_size}x{args.image_size} loc, bs{args.batch}"
        workload = f"CoordinateRegressor({args.backbone}) localization train step fwd+bwd+allreduce+clip+AdamW"
        data = "synthetic uint8 512x512 grayscale->RGB, ImageNet-normalised, resident in HBM; random-init weights"
    if cls:
        # the conv kernels are not GEMM-probed: report the whole-step model FLOP rate against the peak
        roof = {"bound": "mfma", "kernel": "whole training step (implicit-GEMM conv + BN), model FLOPs",
                "achieved": round(step_tflops, 2) if step_tflops else None, "peak": peak, "unit": "TFLOP/s",
                "frac": round(step_tflops / peak, 4) if step_tflops else None, "traffic": None}
    else:
        # which roof binds the probed kernel class: its algorithmic FLOPs at the MFMA peak, or its
        # algorithmic bytes (A, B read once; C, C2, residual/aux once) at the HBM peak
        bytes_per_launch = probe.bytes / max(probe.launches, 1)
        t_mfma = flops_per_launch / (peak * 1e12)
        t_hbm = bytes_per_launch / (PEAK_HBM_GBS * 1e9)
        gbs = bytes_per_launch / (avg_launch_ms * 1e-3) / 1e9 if probe.launches else 0.0
        hbm_bound = t_hbm > t_mfma
        roof = {
            "bound": "hbm" if hbm_bound else "mfma",
            "kernel": f"gemm {args.probe} class ({'bf16' if bf else 'f32'} MFMA): fc1/fc2/downsample",
            "achieved": round(gbs, 1) if hbm_bound else round(achieved, 2),
            "peak": PEAK_HBM_GBS if hbm_bound else peak,
            "unit": "GB/s" if hbm_bound else "TFLOP/s",
            "frac": round((gbs / PEAK_HBM_GBS) if hbm_bound else (achieved / peak), 4),
            "traffic": traffic,
            "launches_timed": probe.launches,
            "avg_launch_us": round(avg_launch_ms * 1e3, 2),
            "algorithmic_gflop_per_launch": round(flops_per_launch / 1e9, 3),
            "algorithmic_bytes_per_launch": int(bytes_per_launch),
            "mfma_tflops": round(achieved, 2),
            "mfma_frac": round(achieved / peak, 4),
            "hbm_gbs": round(gbs, 1),
            "hbm_frac": round(gbs / PEAK_HBM_GBS, 4),
            "step_tflops_per_gpu": round(step_tflops, 1) if step_tflops else None,
            "step_mfma_frac": round(step_tflops / peak, 4) if step_tflops else None,
        }
    result = {
        "metric": metric,
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
        "data": data,
        "config": {
            "workload": workload,
            "image_size": args.image_size,
            "batch_per_gpu": args.batch,
            "global_batch": args.batch * world,
            "parallelism": f"dp{world}",
        },
        "roofline": roof,
        "loss": round(final_loss, 6),
        "hbm_reserved_gb": round(torch.cuda.max_memory_reserved(device) / 2**30, 1),
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(args)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
