"""Benchmark of the north-star hot path: one LocalizationTrainer training step
(forward -> backward -> RCCL gradient all-reduce -> clip(1.0) -> AdamW) of CoordinateRegressor
(ConvNeXt-base, 512x512, batch 32 per GPU, default head, masked SmoothL1) on synthetic uint8
images normalised like the reference's transforms, inputs already resident in HBM.

    python bench.py --gpus N --steps K --warmup W

N > 1: when launched without torch.distributed.run (no WORLD_SIZE in the environment) bench.py starts
``python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1`` on itself as a CHILD
process before touching the GPU, and exits with its code; launched by torch.distributed.run it is one
rank (RANK / LOCAL_RANK / WORLD_SIZE from the environment; rank 0 checks WORLD_SIZE == --gpus).

Rank 0 prints ONE JSON line.  ``roofline`` is the dominant GEMM class of the step (the one with the
most device time): every launch of each probed class is timed with HIP events on its launching
stream in the last timed step; ``roofline.kernels`` carries every probed class (split-K weight
gradients, the fc2 data gradient, the forward GEMMs) and ``step_mfma_frac`` the whole-step model-FLOP
rate against the bf16 MFMA peak (the north-star quantity).  ``comm`` (N > 1) carries the RCCL
all-reduce bus bandwidth and the fraction of it hidden under the backward.  ``cpu_baseline`` times
the fp32 CPU restatement of the same step (oracle/, TEST INFRASTRUCTURE) on the host cores over a
bounded sample, rank 0 at N=1 only.
"""

from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
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
# f32 VALU FMA peak: 256 CUs x 4 SIMDs x 32 FMA per cycle x 2.4 GHz = 78.6 T FMA/s (the guide's 157 TFLOP/s f32
# vector peak); tools/valu_rate.hip: v_fma_f32 reaches 27.7 and v_pk_fma_f32 29.7 FMA/cycle/SIMD at 8 waves per SIMD
# (profiles/round3/r5i_valu_rate.txt), so packing does not raise it
PEAK_VALU_TFMA = 1024 * 32 * 2.4e9 / 1e12
SV_EPI_STORE, SV_EPI_SLAB, SV_EPI_MUL_AUX, SV_EPI_LN_BWD = 0, 4, 6, 10  # include/sv_kernels.h (checked at run time)
# probed GEMM classes: (a_kmajor, b_kmajor[, epilogue])
PROBE_KEYS = {"wgrad": (False, False, SV_EPI_SLAB), "fc2_dgrad": (True, False, SV_EPI_MUL_AUX),
              "dgrad": (True, False, SV_EPI_STORE), "dgrad_ln": (True, False, SV_EPI_LN_BWD), "fwd": (True, True)}
PROBE_NAMES = {"wgrad": "split-K weight gradients dW = dY^T X (fc1, fc2, downsample, stem; side stream)",
               "fc2_dgrad": "fc2 data gradient dh = (dY (W2 gamma)) * GELU'(h) (critical path)",
               "dgrad": "fc1 / downsample data gradients dX = dY W (plain store)",
               "dgrad_ln": "fc1 data gradient with the block LayerNorm backward in its epilogue (SV_EPI_LN_BWD: "
                           "dz from dy = dh W1 kept on chip, C = 512 / 1024)",
               "fwd": "forward GEMMs: fc1 (+GELU), fc2 (+gamma, residual), stem, downsample",
               "dw_fwd": "depthwise 7x7 + LayerNorm forward (sv_dwconv7_ln_fwd)",
               "dw_bwd_data": "depthwise 7x7 backward-data (sv_dwconv7_bwd_data, gradient stream += and bf16 copy)",
               "dw_wgrad": "depthwise 7x7 weight gradient (sv_dwconv7_bwd_weight, partials only)",
               "ln_bwd": "block LayerNorm backward (sv_layernorm_bwd)",
               "adamw": "fused AdamW over the flat buffers (+ bf16 shadow refresh)",
               "mlp_fused": "fused narrow-stage MLP forward (sv_mlp_fwd: fc1 -> GELU -> fc2 -> gamma -> + x, S1 / S2)",
               "mlp_bwd_fused": "fused S1 MLP backward (sv_mlp_bwd: fc2 dgrad x GELU' -> fc1 dgrad -> LayerNorm "
                                "backward + its weight / bias partials, C = 128)",
               "fold": "split-K / partial-sum folds (reduce_multi, reduce_pair, layer-scale fold): bytes = the slab "
                       "bytes they move, overhead of split-K rather than algorithmic work"}
# step-time cost of the data-parallel CU reserve (SV_COMM_RESERVE_CUS, default 0 = none) measured at world 1
# (SV_BENCH_RESERVE A/B, interleaved on one box; DESIGN.md "Multi-GPU": 32 CUs by grid caps 0.6-0.7 %, by CU masks
# 12-24 %), and the start latency of a comm-stream kernel after a readiness report (tests/test_comm_reserve_gpu.py
# over five boxes: worst 0.2-2.9 ms during the backward; at its end, with nothing else queued, the 14-19 us of an
# idle wake-up, tools/event_wake_probe.py -- charged as 0.05 ms): folded into dp_rehearsal's predicted scaling
RESERVE_COST = float(os.environ.get("SV_RESERVE_COST", "0.0"))
HBM_SUSTAINED_GBS = 6300.0  # MI355X_MICROARCH.md: 6.29 TB/s measured (float4 copy)


def comm_latency_samples():
    """Measured comm-kernel start latencies (ms) of the default schedule, committed from tests/test_comm_reserve_gpu.py
    (profiles/comm_latency.json), and their source; None when absent."""
    p = os.path.join(ROOT, "profiles", "comm_latency.json")
    try:
        d = json.load(open(p))
        return [v * 1e-3 for v in d["latency_us"]], d.get("source", p)
    except Exception:
        return None
COMM_DELAY_MS = (float(os.environ.get("SV_COMM_DELAY_MS", "2.9")), float(os.environ.get("SV_COMM_DELAY_END_MS", "0.05")))
# HBM-bound kernel classes timed by kernels.OpProbe (reported separately against 8 TB/s)
OP_PROBE_KEYS = ("dw_fwd", "dw_bwd_data", "dw_wgrad", "ln_bwd", "adamw", "mlp_fused", "mlp_bwd_fused", "fold")


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None, help="ranks (default: WORLD_SIZE, or 1)")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="localization", choices=["localization", "classification"],
                    help="localization = the BASELINE metric (ConvNeXt-base 512); classification = ResNet-50 "
                         "256x256 3-head ClassificationTrainer step (configs[3], secondary line)")
    ap.add_argument("--batch", type=int, default=32, help="images per GPU")
    ap.add_argument("--image-size", type=int, default=None, help="default 512 (localization) / 256 (classification)")
    ap.add_argument("--backbone", default=None, help="default convnext_base / resnet50")
    ap.add_argument("--precision", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--selftest", action="store_true",
                    help="launcher / all-reduce plumbing check on CPU (gloo, a small torch model): no GPU, no "
                         "measurement -- used by tests/test_bench_launcher.py")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--inference", action="store_true",
                    help="secondary line (row f2): the validation / predict forward (eval mode, no tape) instead "
                         "of the training step")
    ap.add_argument("--graph", default="off", choices=["on", "off"],
                    help="replay the training step as a captured HIP graph (StepEngine(cuda_graph=True), "
                         "classification only: ConvNeXt's lean side-stream release queries events).  Measured "
                         "(profiles/r3/graph_ab.txt): ResNet-50 3197-3228 img/s replayed vs 3395-3443 eager with "
                         "the side-stream weight gradients, 3300 single-stream replayed -- off by default")
    ap.add_argument("--trainer", action="store_true",
                    help="secondary line (row f1): LocalizationTrainer._train_epoch fed by its DataLoader from "
                         "synthetic grayscale PNGs on disk (decode in the workers, resize / augment / normalise on "
                         "the GPU with --transform device) instead of HBM-resident batches")
    ap.add_argument("--transform", default="device", choices=["device", "host"],
                    help="--trainer: device = device_transform (GPU resize + augment + normalise), host = the "
                         "reference's PIL / torchvision chain in the workers")
    ap.add_argument("--workers", type=int, default=4, help="--trainer: DataLoader workers per rank (reference: 4)")
    ap.add_argument("--native", type=int, default=640, help="--trainer: side of the PNGs on disk (resized to 512)")
    ap.add_argument("--cpu-seconds", type=float, default=15.0, help="bounded CPU sample budget")
    ap.add_argument("--traffic-file", default=os.path.join(ROOT, "profiles", "traffic.json"))
    ap.add_argument("--rocprof-file", default=os.path.join(ROOT, "profiles", "rocprof_avg.json"),
                    help="per-class rocprofv3 average launch durations (tools/rocprof_avg.py) for frac_rocprof")
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

    threads = host_threads()
    torch.set_num_threads(threads)
    B = args.batch  # the same batch as the GPU line
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
    # at least 3 timed steps (the median: the first carries the allocator's warm-up), more while the budget lasts
    times = []
    t0 = time.perf_counter()
    while True:
        t1 = time.perf_counter()
        one()
        times.append(time.perf_counter() - t1)
        if len(times) >= 3 and (time.perf_counter() - t0 >= args.cpu_seconds or len(times) >= 8):
            break
    med = sorted(times)[len(times) // 2]
    try:
        cpu_name = [ln.split(":", 1)[1].strip() for ln in open("/proc/cpuinfo") if ln.startswith("model name")][0]
    except Exception:  # pragma: no cover
        cpu_name = "unknown"
    return {
        "value": round(B / med, 4),
        "unit": "images/sec",
        "cores": threads,
        "kind": "port",
        "sample": f"median of {len(times)} timed fp32 train steps ({', '.join(f'{t:.1f}' for t in times)} s) of "
                  f"{args.backbone} {args.image_size}x{args.image_size} bs{B} on {cpu_name}, torch eager CPU, "
                  "oracle/ restatement",
    }


def host_threads() -> int:
    """Host threads for the CPU baseline: the CPUs this process may run on, capped by the cgroup CPU
    quota when there is one (a GPU box's share of a large host: affinity shows every CPU)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if quota != "max":
            n = min(n, max(1, int(int(quota) // int(period))))
    except (OSError, ValueError):
        pass
    omp = os.environ.get("OMP_NUM_THREADS")
    if omp and omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
    return max(1, n)


def cpu_baseline_config0():
    """configs[0] (plumbing): ResNet18 256x256 classification, bs4, 2 epochs over 32 synthetic crops, fp32
    CPU restatement of the step (oracle/, baseline only)."""
    from oracle import heads as oh
    from oracle import resnet as orn
    from oracle import step as ostep

    threads = host_threads()
    torch.set_num_threads(threads)
    model = oh.Classifier(orn.create("resnet18"), 512, dropout=0.3)
    opt = ostep.make_optimizer(model)
    model.train()
    crops = [synthetic_cls_batch(4, 256, 256, "cpu", 100 + i) for i in range(8)]
    t0 = time.perf_counter()
    for _epoch in range(2):
        for img, targets in crops:
            ostep.train_step_classification(model, opt, img, targets)
    el = time.perf_counter() - t0
    return {"value": round(64 / el, 3), "unit": "images/sec", "cores": threads, "kind": "port",
            "sample": "configs[0]: ResNet18 256x256 bs4, 2 epochs x 8 steps (32 synthetic crops), fp32 oracle/ "
                      "restatement, end to end"}


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(args) -> int:
    """N ranks of this script under torch.distributed.run, started as a child process BEFORE any GPU
    call in this process (never an exec); returns the child's exit code."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("OMP_NUM_THREADS", "1")
    return subprocess.call(cmd, env=env)


def classification_line(args) -> dict:
    """BASELINE configs[3] per GPU (ResNet-50 3-head classification 256x256, bs32) beside the headline line, so the
    driver's own N=1 run times it too (VERDICT r5 missing 5).  A child process of this script (never an exec), run
    after the headline's timed region; its JSON line is condensed here.  SV_BENCH_CLS=0 skips it."""
    steps, warmup = max(args.steps, 20), max(args.warmup, 5)
    cmd = [sys.executable, os.path.abspath(__file__), "--workload", "classification", "--steps", str(steps),
           "--warmup", str(warmup), "--no-cpu-baseline", "--precision", args.precision]
    env = dict(os.environ, SV_BENCH_CLS="0")
    t0 = time.perf_counter()
    try:
        r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
    except subprocess.TimeoutExpired:
        return {"error": "timed out after 300 s"}
    wall = time.perf_counter() - t0
    lines = [ln for ln in r.stdout.strip().splitlines() if ln.startswith("{")]
    if r.returncode != 0 or not lines:
        return {"error": f"exit {r.returncode}", "stderr_tail": r.stderr[-800:]}
    d = json.loads(lines[-1])
    return {"metric": d["metric"], "value": d["value"], "unit": d["unit"], "n_gpus": 1, "steps": d["steps"],
            "warmup": d["warmup"], "ms_per_step": d["ms_per_step"], "dtype": d["dtype"], "config": d["config"],
            "step_mfma_frac": d["roofline"].get("step_mfma_frac"), "main_queue": d.get("main_queue"),
            "loss": d.get("loss"), "child_wall_s": round(wall, 1),
            "baseline_config": "BASELINE.json configs[3] (ResNet50 multi-task classification 256x256), per GPU"}


def selftest(args, world: int, rank: int) -> None:
    """--selftest: the multi-rank plumbing of this script on CPU (gloo) -- launcher, rank env, the flat
    bucketed all-reduce and the max-over-ranks timing -- on a small torch model.  Not a measurement."""
    import torch.nn as nn

    pkg = __graft_entry__.load_package()  # noqa: F841
    from spine_vision_amd.training.comm import GradBucketer, broadcast_parameters
    from spine_vision_amd.training.flat import FlatArena

    if world > 1:
        dist.init_process_group("gloo")
    torch.manual_seed(rank)
    model = nn.Sequential(nn.Linear(64, 256), nn.GELU(), nn.Linear(256, 64))
    arena = FlatArena(model, "cpu", with_shadow=False)
    buck = None
    if world > 1:
        broadcast_parameters(arena, model)
        buck = GradBucketer(arena, bucket_mb=16 * 1024 * 4 / 2**20)
        buck.attach(model)
    x = torch.randn(args.batch, 64, generator=torch.Generator().manual_seed(1234 + rank))
    for _ in range(args.warmup):
        arena.zero_grad()
        model(x).pow(2).mean().backward()
        if buck is not None:
            buck.finish()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        arena.zero_grad()
        model(x).pow(2).mean().backward()
        if buck is not None:
            buck.finish()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    g = arena.grad_flat.clone()
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t)
        allg = [torch.empty_like(g) for _ in range(world)]
        dist.all_gather(allg, g)
        same = all(torch.equal(allg[0], a) for a in allg)
    else:
        same = True
    if rank == 0:
        print(json.dumps({"metric": "selftest (launcher / all-reduce plumbing, CPU gloo; not a measurement)",
                          "value": round(world * args.batch * args.steps / el, 3), "unit": "samples/sec",
                          "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
                          "ms_per_step": round(el / args.steps * 1e3, 3), "higher_is_better": True, "scaling": "weak",
                          "vs_baseline": None, "dtype": "f32", "data": "synthetic",
                          "config": {"workload": "selftest", "parallelism": f"dp{world}",
                                     "buckets": len(buck.buckets) if buck else 0},
                          "grads_identical_across_ranks": same}), flush=True)
    if world > 1:
        dist.destroy_process_group()


def _write_pngs(root: str, n: int, side: int) -> None:
    """n synthetic grayscale MRI-like PNGs (smooth anatomy-scale structure + noise, side x side) and the
    reference's annotations.csv layout (image_path, level, relative_x, relative_y, series_type, source)."""
    import csv
    from concurrent.futures import ThreadPoolExecutor

    import numpy as np
    from PIL import Image

    os.makedirs(os.path.join(root, "img"), exist_ok=True)
    yy, xx = np.meshgrid(np.linspace(0, 1, side), np.linspace(0, 1, side), indexing="ij")

    def one(i):
        rng = np.random.default_rng(i)
        base = 110 + 70 * np.sin(9 * xx + 4 * yy + i) * np.cos(5 * yy - 3 * xx)
        img = np.clip(base + rng.normal(0, 12, (side, side)), 0, 255).astype(np.uint8)
        Image.fromarray(img, "L").save(os.path.join(root, "img", f"s{i}.png"))

    with ThreadPoolExecutor(16) as ex:
        list(ex.map(one, range(n)))
    levels = ("L1/L2", "L2/L3", "L3/L4", "L4/L5", "L5/S1")
    with open(os.path.join(root, "annotations.csv"), "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=["image_path", "level", "relative_x", "relative_y", "series_type", "source"])
        w.writeheader()
        for i in range(n):
            for k, lv in enumerate(levels):
                w.writerow({"image_path": f"img/s{i}.png", "level": lv, "relative_x": 0.45 + 0.01 * k,
                            "relative_y": 0.2 + 0.15 * k, "series_type": "sag_t2", "source": "synthetic"})


def trainer_line(args) -> dict:
    """--trainer: images/sec of LocalizationTrainer._train_epoch (the reference's epoch loop, base.py:547-569)
    fed by its own DataLoader over PNGs on disk: decode (+ host transform) in ``--workers`` worker processes,
    then the MI355X step.  The second epoch is timed (the first starts the workers and warms the kernels).
    Also times the per-image host work of one worker alone, which bounds the loader at workers / that."""
    import shutil
    import tempfile

    pkg = __graft_entry__.load_package()  # noqa: F841
    from spine_vision_amd.training import LocalizationConfig, LocalizationTrainer
    from spine_vision_amd.training.datasets import LocalizationCollator, LocalizationDataset

    steps = max(args.steps, 10)
    root = tempfile.mkdtemp(prefix="sv_trainer_")
    try:
        n = int(args.batch * steps / 0.95) + args.batch  # the dataset's test split keeps 5% aside
        _write_pngs(root, n, args.native)
        dev_t = args.transform == "device"
        cfg = LocalizationConfig(data_path=root, output_path=os.path.join(root, "out"), batch_size=args.batch,
                                 num_epochs=1, num_workers=args.workers, pin_memory=True, device_transform=dev_t,
                                 augment=True, image_size=(512, 512), pretrained=False, val_split=0.0,
                                 log_frequency=10**9, save_frequency=10**9, early_stopping=False,
                                 visualize_predictions=False, use_trackio=False, precision=args.precision)
        tr = LocalizationTrainer(cfg)
        nb = len(tr.train_loader)
        stamps: list = []
        step0 = tr._train_step

        def stamped(batch):  # host time after each step is enqueued (InflightLimiter: <= 2 steps ahead)
            out = step0(batch)
            stamps.append(time.perf_counter())
            return out

        tr._train_step = stamped
        tr._train_epoch()
        torch.cuda.synchronize()
        stamps.clear()
        t0 = time.perf_counter()
        tr._train_epoch()
        torch.cuda.synchronize()
        t_end = time.perf_counter()
        el = t_end - t0
        # steady state: from the 5th step of the timed epoch to its end (worker start-up and the first
        # batches' decode excluded -- the reference's DataLoader restarts its workers every epoch)
        skip = min(5, nb - 2)
        steady = (nb - skip) * args.batch / (t_end - stamps[skip - 1]) if nb > skip + 1 else None
        # one worker's host cost per image (decode + the dataset's host work + collation), single process
        ds = LocalizationDataset(root, split="train", image_size=(512, 512), augment=True, device_transform=dev_t,
                                 val_ratio=0.0)
        col = LocalizationCollator()
        k = min(len(ds), 4 * args.batch)
        h0 = time.perf_counter()
        for j in range(0, k, args.batch):
            col([ds[i] for i in range(j, min(k, j + args.batch))])
        per_img = (time.perf_counter() - h0) / k
    finally:
        shutil.rmtree(root, ignore_errors=True)
    imgs = nb * args.batch
    return {"metric": "images/sec training, LocalizationTrainer epoch over PNGs on disk (DataLoader-fed), "
                      f"{args.backbone} 512x512, bs{args.batch}",
            "value": round(imgs / el, 3), "unit": "images/sec", "n_gpus": 1, "steps": nb, "warmup": nb,
            "ms_per_step": round(el / nb * 1e3, 3), "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": args.precision,
            "data": f"synthetic {args.native}x{args.native} grayscale PNGs on local disk, decoded by the loader",
            "config": {"workload": "LocalizationTrainer._train_epoch (+ its DataLoader)", "transform": args.transform,
                       "workers": args.workers, "native_side": args.native, "image_size": 512,
                       "batch_per_gpu": args.batch, "augment": True},
            "steady_state_img_s": round(steady, 1) if steady else None,
            "first_batch_s": round(stamps[0] - t0, 3) if stamps else None,
            "host_ms_per_image_one_worker": round(per_img * 1e3, 3),
            "host_bound_img_s": round(args.workers / per_img, 1)}


def kernel_roofline(name: str, probe, steps_probed: int, peak: float, traffic: dict) -> dict:
    """Roofline of one probed kernel class: algorithmic FLOPs / bytes (/ f32 VALU FMAs) per launch against the
    mean launch duration from HIP events; the binding roof is the largest of FLOPs / MFMA peak, bytes / HBM
    peak and, for the depthwise convolutions, FMAs / VALU peak (1024 SIMDs x 16 FMA/clk x 2.4 GHz)."""
    n = max(probe.launches, 1)
    avg_ms = probe.elapsed_ms() / n
    flops, nbytes, fma = probe.flops / n, probe.bytes / n, getattr(probe, "fma", 0.0) / n
    tflops = flops / (avg_ms * 1e-3) / 1e12 if probe.launches else 0.0
    gbs = nbytes / (avg_ms * 1e-3) / 1e9 if probe.launches else 0.0
    tfma = fma / (avg_ms * 1e-3) / 1e12 if probe.launches else 0.0
    t_roof = {"hbm": nbytes / (PEAK_HBM_GBS * 1e9), "mfma": flops / (peak * 1e12), "valu": fma / (PEAK_VALU_TFMA * 1e12)}
    bound = max(t_roof, key=t_roof.get)
    ach, pk, unit = {"hbm": (gbs, PEAK_HBM_GBS, "GB/s"), "mfma": (tflops, peak, "TFLOP/s"),
                     "valu": (tfma, PEAK_VALU_TFMA, "T FMA/s")}[bound]
    tr = traffic.get(f"{name}_bytes_per_launch")  # None unless a PMC pass of THIS configuration exists
    out = {
        "kernel": PROBE_NAMES[name],
        "bound": bound,
        "achieved": round(ach, 2 if bound != "hbm" else 1),
        "peak": pk,
        "unit": unit,
        "frac": round(ach / pk, 4),
        "traffic": tr,
        "traffic_ratio": round(tr / nbytes, 3) if tr and nbytes else None,
        "launches_per_step": round(probe.launches / max(steps_probed, 1), 1),
        "ms_per_step": round(avg_ms * probe.launches / max(steps_probed, 1), 3),
        "avg_launch_us": round(avg_ms * 1e3, 2),
        "algorithmic_gflop_per_launch": round(flops / 1e9, 3),
        "algorithmic_bytes_per_launch": int(nbytes),
        "mfma_tflops": round(tflops, 2),
        "mfma_frac": round(tflops / peak, 4),
        "hbm_gbs": round(gbs, 1),
        "hbm_frac": round(gbs / PEAK_HBM_GBS, 4),
    }
    shares = getattr(probe, "shares", None)
    if shares and len(shares) == len(probe.events):
        durs = [a.elapsed_time(b) for a, b in probe.events]
        share = sum(d * s for d, s in zip(durs, shares)) / max(sum(durs), 1e-30)
        out.update({"granted_cu_share": round(share, 3), "frac_of_granted_cus": round(ach / (pk * share), 4)})
    if fma:
        out.update({"valu_gfma_per_launch": round(fma / 1e9, 3), "valu_tfma": round(tfma, 2),
                    "valu_frac": round(tfma / PEAK_VALU_TFMA, 4)})
    return out


def rocprof_frac(path: str, key: str, cls: str, kr: dict, peak: float) -> dict:
    """The dominant class's roofline fraction from the profiler's average launch duration of the same kernels
    (profiles/rocprof_avg.json, tools/rocprof_avg.py) beside the HIP-event probe's: roof time per launch (this line's
    algorithmic bytes / FLOPs) / rocprof's average.  {} when no profile of this configuration is committed."""
    try:
        ent = json.load(open(path))["configs"][key][cls]
    except Exception:
        return {}
    t_roof = max(kr["algorithmic_bytes_per_launch"] / (PEAK_HBM_GBS * 1e9),
                 kr["algorithmic_gflop_per_launch"] * 1e9 / (peak * 1e12))
    avg = ent["avg_launch_us"] * 1e-6
    return {"frac_rocprof": round(t_roof / avg, 4), "rocprof_avg_launch_us": ent["avg_launch_us"],
            "rocprof_source": ent["source"], "frac_probe": kr["frac"]}


def step_floor(kern: dict, ms: float, peak: float) -> dict:
    """The step against its own floor: for every probed class of algorithmic work, launches x max(algorithmic
    bytes / 8 TB/s, FLOPs / bf16 peak) per launch, summed (the split-K folds are overhead, not algorithmic,
    and count zero).  Kernels outside the probed classes (stem / downsample LayerNorms, pooling, head, loss,
    clip) add to the step but not to this floor, so ``frac`` is a lower bound of the step's distance from it."""
    floor_ms, work_ms = 0.0, 0.0
    for k, v in kern.items():
        if k == "fold":
            continue
        n = v["launches_per_step"]
        floor_ms += n * max(v["algorithmic_bytes_per_launch"] / (PEAK_HBM_GBS * 1e9),
                            v["algorithmic_gflop_per_launch"] * 1e9 / (peak * 1e12),
                            v.get("valu_gfma_per_launch", 0.0) * 1e9 / (PEAK_VALU_TFMA * 1e12)) * 1e3
        work_ms += v["ms_per_step"]
    return {"ms": round(floor_ms, 3), "frac": round(floor_ms / ms, 4) if ms else None,
            "classes": sorted(k for k in kern if k != "fold"),
            "classes_ms_per_step": round(work_ms, 3),
            "fold_ms_per_step": kern["fold"]["ms_per_step"] if "fold" in kern else None,
            "note": "sum over the probed classes of max(algorithmic bytes / 8 TB/s, FLOPs / bf16 peak, depthwise f32 "
                    "FMAs / VALU peak) per launch; "
                    "classes_ms_per_step adds their in-step durations, which overlap across the two streams"}


def main():
    args = parse()
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and (args.gpus or 1) > 1:
        sys.exit(launch_ranks(args))  # before any GPU call in this process
    world = int(env_world or "1")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus is not None and args.gpus != world:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    if args.selftest:
        return selftest(args, world, rank)
    if args.trainer:
        if world != 1:
            raise SystemExit("bench.py --trainer runs on one GPU")
        print(json.dumps(trainer_line(args)), flush=True)
        return
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        assert dist.get_world_size() == world
    device = torch.device("cuda", local)

    pkg = __graft_entry__.load_package()  # noqa: F841
    from spine_vision_amd import kernels as K
    from spine_vision_amd import native as nv
    from spine_vision_amd.training import Classifier, CoordinateRegressor, StepEngine

    assert (nv.SV_EPI_STORE, nv.SV_EPI_SLAB, nv.SV_EPI_MUL_AUX, nv.SV_EPI_LN_BWD) == (SV_EPI_STORE, SV_EPI_SLAB,
                                                                                   SV_EPI_MUL_AUX, SV_EPI_LN_BWD)
    torch.manual_seed(42)
    cls = args.workload == "classification"
    if cls:
        from spine_vision_amd.training.trainers.classification import _create_tasks_for_training

        tasks = _create_tasks_for_training(target_labels=CLS_TASKS, label_smoothing=0.1)
        model = Classifier(args.backbone, tasks=tasks, pretrained=False, dropout=0.3, precision=args.precision)
    else:
        model = CoordinateRegressor(args.backbone, pretrained=False, precision=args.precision)
    model = model.to(device).train()
    # SV_BENCH_RESERVE (A/B at world 1): the CU reserve a multi-GPU run applies (CU-masked step streams + capped
    # GEMM grids, training/cumask.py); world > 1 takes SV_COMM_RESERVE_CUS (default 32)
    reserve = int(os.environ["SV_BENCH_RESERVE"]) if os.environ.get("SV_BENCH_RESERVE") else None
    graphed = args.graph == "on" and cls and world == 1
    engine = StepEngine(model, device, lr=1e-4, weight_decay=1e-5, grad_clip=1.0,
                        cuda_graph=graphed and not args.inference, comm_reserve_cus=reserve)
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

        def run_step():  # noqa: F811
            with torch.no_grad():
                out = model(img)
            return out.float().mean() if not isinstance(out, dict) else sum(v.float().mean() for v in out.values())

    for _ in range(args.warmup):
        run_step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    torch.cuda.reset_peak_memory_stats(device)
    retries0 = torch.cuda.memory_stats(device).get("num_alloc_retries", 0)

    bf = args.precision == "bf16"
    probes = {k: K.GemmProbe(v[:2] + (bf,) + v[2:], k) for k, v in PROBE_KEYS.items()}
    op_probes = {k: K.OpProbe(k) for k in OP_PROBE_KEYS}
    # The probes' HIP events bracket every launch of their classes in the LAST timed step: each timing
    # event is a release packet that writes back L2, and probing all K steps cost 2.3% of the step
    # (tools/gpu_probe_ab.sh).  The classification line reports the whole-step rate and takes no probe;
    # SV_BENCH_PROBE=0 leaves the per-kernel fields empty and SV_BENCH_PROBE=all probes every step.
    probe_mode = os.environ.get("SV_BENCH_PROBE", "1")
    use_probe = not cls and not args.inference and probe_mode != "0"
    bucketer = engine.bucketer
    # world 1: rehearse the data-parallel exchange -- when each 64 MB bucket's gradients become final in
    # the last timed step, and a prediction of the exposed all-reduce at N ranks (comm.BucketTimeline)
    timeline = None
    tl_ev: dict = {}
    if world == 1 and not args.inference and os.environ.get("SV_BENCH_TIMELINE", "1") != "0":
        from spine_vision_amd.training.comm import BucketTimeline

        timeline = BucketTimeline(engine.arena, model, bucket_mb=64.0)

        def _bwd_end():
            if timeline.active:
                tl_ev["bwd_end"] = torch.cuda.Event(enable_timing=True)
                tl_ev["bwd_end"].record()

        engine.after_backward = _bwd_end
    t0 = time.perf_counter()
    for i in range(args.steps):
        last = i == args.steps - 1
        if timeline is not None:
            timeline.reset()
            timeline.active = last
            if last:
                tl_ev["start"] = torch.cuda.Event(enable_timing=True)
                tl_ev["start"].record()
        probing = use_probe and (probe_mode == "all" or last)
        K.PROBES = list(probes.values()) if probing else []
        K.OP_PROBES = dict(op_probes) if probing else {}
        if bucketer is not None:
            bucketer.timing = last
        loss = run_step()
        if timeline is not None and last:
            tl_ev["end"] = torch.cuda.Event(enable_timing=True)
            tl_ev["end"].record()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    K.PROBES = []
    K.OP_PROBES = {}
    if world > 1:
        t = torch.tensor([elapsed], device=device, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    # the main queue's busy time: the critical path of the two-stream backward is the stream the
    # step runs on, not the dominant-by-time side-stream class.  One extra, untimed step with HIP events around every
    # sv_* launch on that stream (torch's own kernels there -- head, loss -- are not bracketed)
    main_queue = None
    if not args.inference and os.environ.get("SV_BENCH_MAINQ", "1") != "0":
        mstream = engine._stream if getattr(engine, "_stream", None) is not None else torch.cuda.current_stream()
        nv.STREAM_PROBE = nv.StreamProbe(mstream)
        try:
            run_step()
            torch.cuda.synchronize()
            sp = nv.STREAM_PROBE
            main_queue = {"busy_ms_per_step": round(sp.busy_ms(), 3), "launches_per_step": len(sp.events),
                          "span_ms": round(sp.span_ms(), 3),
                          "source": "HIP events around every sv_* launch on the step's stream, one extra untimed "
                                    "step (torch's head / loss kernels excluded)"}
        finally:
            nv.STREAM_PROBE = None
    final_loss = float(loss.item())
    # (a diagnostic SV_DIAG_SKIP run skips launches on purpose: its loss is garbage and its line says so)
    assert final_loss == final_loss or K._DIAG_SKIP, "loss is NaN"
    mstats = torch.cuda.memory_stats(device)

    peak = PEAK_BF16_TFLOPS if bf else PEAK_F32_MFMA_TFLOPS
    # PMC traffic per launch, keyed by the exact configuration it was measured on (profiles/traffic.json
    # "configs"): a line without a matching pass reports traffic null, never another configuration's bytes
    traffic_key = f"{args.backbone}/{args.image_size}/bs{args.batch}/{args.precision}"
    traffic = {}
    if os.path.exists(args.traffic_file):
        try:
            traffic = json.load(open(args.traffic_file)).get("configs", {}).get(traffic_key, {})
        except Exception:
            traffic = {}

    ms = elapsed / args.steps * 1e3
    value = world * args.batch * args.steps / elapsed
    gflop = STEP_GFLOP.get((args.backbone, args.image_size))
    step_tflops = gflop * args.batch / (ms * 1e-3) / 1e3 if gflop else None
    if args.inference:
        metric = f"images/sec inference (eval forward), {args.backbone} {args.image_size}x{args.image_size}, bs{args.batch}"
        workload = f"{'Classifier' if cls else 'CoordinateRegressor'}({args.backbone}) eval forward (validation / predict)"
        data = "synthetic, resident in HBM; random-init weights"
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
    step_frac = round(step_tflops / peak, 4) if step_tflops else None
    if use_probe:
        nprobed = args.steps if probe_mode == "all" else 1
        kern = {k: kernel_roofline(k, p_, nprobed, peak, traffic) for k, p_ in probes.items() if p_.launches}
        dominant = max(kern, key=lambda k: kern[k]["ms_per_step"])
        kern.update({k: kernel_roofline(k, p_, nprobed, peak, traffic) for k, p_ in op_probes.items() if p_.launches})
        roof = dict(kern[dominant])
        roof["kernel"] = f"{dominant}: {roof['kernel']} (dominant GEMM class by device time)"
        roof["step_tflops_per_gpu"] = round(step_tflops, 1) if step_tflops else None
        roof["step_mfma_frac"] = step_frac
        roof["traffic_config"] = traffic_key if traffic else None
        roof["step_floor"] = step_floor(kern, ms, peak)
        rp = rocprof_frac(args.rocprof_file, traffic_key, dominant, kern[dominant], peak)
        if rp:
            roof.update(rp)
        roof["kernels"] = kern
    else:
        # no per-kernel probe: report the whole-step model FLOP rate against the peak
        roof = {"bound": "mfma", "kernel": "whole training step, model FLOPs" if not args.inference
                else "whole eval forward, model FLOPs",
                "achieved": round(step_tflops, 2) if step_tflops else None, "peak": peak, "unit": "TFLOP/s",
                "frac": step_frac, "traffic": None, "step_mfma_frac": step_frac}
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
            "hip_graph": bool(engine.cuda_graph),
        },
        "roofline": roof,
        "main_queue": main_queue,
        "loss": round(final_loss, 6) if final_loss == final_loss else None,
        **({"diag_skip": sorted(K._DIAG_SKIP)} if K._DIAG_SKIP else {}),
        "hbm_reserved_gb": round(torch.cuda.max_memory_reserved(device) / 2**30, 1),
        "hbm_peak_allocated_gb": round(torch.cuda.max_memory_allocated(device) / 2**30, 1),
        "num_alloc_retries": int(mstats.get("num_alloc_retries", 0) - retries0),
    }
    if bucketer is not None:
        comm = bucketer.timing_stats()
        # the whole gradient buffer once more, alone, for the bus bandwidth of one large all-reduce
        g = engine.arena.grad_flat
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        dist.barrier()
        e0.record()
        for _ in range(3):
            dist.all_reduce(g)
        e1.record()
        torch.cuda.synchronize()
        t_ar = e0.elapsed_time(e1) / 3 * 1e-3
        comm["allreduce_full_mb"] = round(g.numel() * 4 / 2**20, 1)
        comm["allreduce_full_busbw_gbs"] = round(2.0 * (world - 1) / world * g.numel() * 4 / t_ar / 1e9, 1)
        result["comm"] = comm
    if timeline is not None and "bwd_end" in tl_ev:
        timeline.active = False
        ready = timeline.ready_ms(tl_ev["start"])
        bwd_end = tl_ev["start"].elapsed_time(tl_ev["bwd_end"])
        step_last = tl_ev["start"].elapsed_time(tl_ev["end"])
        # xGMI bus bandwidth of RCCL's ring all-reduce on 8 MI355X: not measurable on a 1-GPU box; the
        # prediction is given at 200 / 300 / 400 GB/s (DESIGN.md "Multi-GPU": 7 links x ~153 GB/s per GPU)
        samples = comm_latency_samples()
        result["dp_rehearsal"] = {
            "buckets_mb_ready_ms": ready,
            "backward_end_ms": round(bwd_end, 3), "step_ms_last": round(step_last, 3),
            # the reserve's own cost (32 of 256 CUs masked from the step under data parallelism), measured at
            # world 1 as an interleaved A/B (SV_BENCH_RESERVE, DESIGN.md "Multi-GPU"), stretches every time
            "reserve_cost_frac": RESERVE_COST,
            "comm_launch_delay_ms": list(COMM_DELAY_MS),
            # every bucket charged the worst start latency ever measured, plus RCCL's own HBM traffic beside the
            # backward at the HBM rate the chip sustains (comm.BucketTimeline.predict)
            "predictions": [timeline.predict(ready, bwd_end, ms, 8, bw, reserve_cost=RESERVE_COST,
                                             launch_delay_ms=COMM_DELAY_MS, hbm_gbs=HBM_SUSTAINED_GBS)
                            for bw in (200.0, 300.0, 400.0)],
        }
        if samples:
            # each bucket waits for the slowest of 8 ranks: the expected max of 8 draws from the measured latencies
            result["dp_rehearsal"]["comm_latency_source"] = samples[1]
            result["dp_rehearsal"]["predictions_max_over_ranks"] = [
                timeline.predict(ready, bwd_end, ms, 8, bw, reserve_cost=RESERVE_COST, launch_delay_ms=COMM_DELAY_MS,
                                 latency_samples_ms=samples[0], hbm_gbs=HBM_SUSTAINED_GBS) for bw in (200.0, 300.0, 400.0)]
    if world > 1:
        result["config"]["comm_reserve_cus"] = engine.comm_reserve_cus
    if (rank == 0 and world == 1 and not cls and not args.inference and args.backbone == "convnext_base"
            and os.environ.get("SV_BENCH_CLS", "1") != "0"):
        result["configs3_classification"] = classification_line(args)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(args)
        if not cls and not args.inference:
            result["cpu_baseline_configs0"] = cpu_baseline_config0()
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
