"""GPU: the data-parallel step end to end (StepEngine with distributed=True: rank-0 parameter broadcast,
bucketed gradient all-reduce launched from the backbone's per-block grad_ready_hook on the comm stream,
finish() joining it before clip + AdamW) with two ranks on the box's one GPU over gloo (RCCL needs one
GPU per rank; the bucket/stream logic is backend-agnostic).

Two ranks on B images each must reproduce a single process on the 2B-image batch: the reference's DDP
semantics -- mean loss per rank, gradients averaged over ranks.  fp32 parity mode,
all-valid masks (so every rank's masked mean has the same denominator)."""

import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

B, S = 2, 64


def _batch():
    from oracle import weights as ow

    img, coords, mask = ow.localization_batch(2 * B, S, S)
    return img, coords, torch.ones_like(mask)


def _model(dev, precision="fp32"):
    from oracle import weights as ow
    from spine_vision_amd.training import CoordinateRegressor

    m = CoordinateRegressor("convnext_base", pretrained=False, dropout=0.0, precision=precision)
    ow.fill_module(m)
    return m.to(dev).train()


def _rank(rank, world, port, out):
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    import __graft_entry__

    __graft_entry__.load_package()
    import torch.distributed as dist

    from spine_vision_amd.training import StepEngine

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda:0")
    m = _model(dev)
    if rank == 1:  # the broadcast must overwrite a diverged replica
        with torch.no_grad():
            m.head[5].bias.add_(1.0)
    eng = StepEngine(m, dev, lr=1e-4, weight_decay=1e-5, grad_clip=1.0, distributed=True, bucket_mb=16.0)
    img, coords, mask = _batch()
    sl = slice(rank * B, (rank + 1) * B)
    loss = eng.step_localization(img[sl].to(dev), coords[sl].to(dev), mask[sl].to(dev))
    torch.cuda.synchronize()
    out[rank] = (float(loss), float(eng.last_grad_norm), eng.arena.grad_flat.cpu().clone(),
                 eng.arena.param_flat.cpu().clone(), len(eng.bucketer.buckets))
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_two_rank_step_matches_single_process(dev):
    from spine_vision_amd.training import StepEngine

    ctx = mp.get_context("spawn")
    mgr = ctx.Manager()
    out = mgr.dict()
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, 2, port, out)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=300)
        assert p.exitcode == 0, f"rank exited with {p.exitcode}"
    (l0, n0, g0, p0, nb), (l1, n1, g1, p1, _) = out[0], out[1]
    assert nb > 1, "expected several gradient buckets"
    # every rank holds the all-reduced gradient and the same updated parameters
    assert torch.equal(g0, g1) and n0 == n1
    assert torch.equal(p0, p1)
    # == one process over the whole batch
    m = _model(dev)
    eng = StepEngine(m, dev, lr=1e-4, weight_decay=1e-5, grad_clip=1.0, distributed=False)
    img, coords, mask = _batch()
    l_ref = float(eng.step_localization(img.to(dev), coords.to(dev), mask.to(dev)))
    g_ref = eng.arena.grad_flat.cpu()
    assert float((g0 - g_ref).norm() / g_ref.norm()) < 1e-4
    assert abs(n0 - float(eng.last_grad_norm)) / float(eng.last_grad_norm) < 1e-4
    assert abs(0.5 * (l0 + l1) - l_ref) / l_ref < 1e-5
    dp = (p0 - eng.arena.param_flat.cpu()).abs().max()
    assert float(dp) <= 2e-4 * 1.001  # first AdamW step: each element moves by ~lr*sign(g)


def _rccl_rank(port, out):
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    import __graft_entry__

    __graft_entry__.load_package()
    import torch.distributed as dist

    from spine_vision_amd.training import StepEngine

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    m = _model(dev)
    eng = StepEngine(m, dev, lr=1e-4, weight_decay=1e-5, grad_clip=1.0, distributed=True, bucket_mb=16.0)
    eng.bucketer.timing = True
    img, coords, mask = _batch()
    loss = eng.step_localization(img.to(dev), coords.to(dev), mask.to(dev))
    torch.cuda.synchronize()
    stats = eng.bucketer.timing_stats()
    out["r"] = (dist.get_backend(), float(loss), eng.arena.grad_flat.cpu().clone(), eng.arena.param_flat.cpu().clone(),
                len(eng.bucketer.buckets), stats)
    dist.destroy_process_group()


def test_rccl_bucketer_world1_matches_single_process(dev):
    """The RCCL ("nccl") branch of GradBucketer -- ReduceOp.AVG issued on the high-priority comm stream,
    the comm stream joined to RCCL's stream per bucket, the compute stream joined before clip/AdamW --
    executed at world 1 (the box has one GPU): gradients and the AdamW update equal the non-distributed
    step bit for bit, and the timing hooks report every bucket."""
    from spine_vision_amd.training import StepEngine

    ctx = mp.get_context("spawn")
    mgr = ctx.Manager()
    out = mgr.dict()
    p = ctx.Process(target=_rccl_rank, args=(_free_port(), out))
    p.start()
    p.join(timeout=300)
    assert p.exitcode == 0, f"rank exited with {p.exitcode}"
    backend, loss, g, prm, nb, stats = out["r"]
    assert backend == "nccl" and nb > 1
    m = _model(dev)
    eng = StepEngine(m, dev, lr=1e-4, weight_decay=1e-5, grad_clip=1.0, distributed=False)
    img, coords, mask = _batch()
    l_ref = float(eng.step_localization(img.to(dev), coords.to(dev), mask.to(dev)))
    assert loss == l_ref
    assert torch.equal(g, eng.arena.grad_flat.cpu())
    assert torch.equal(prm, eng.arena.param_flat.cpu())
    assert stats["buckets"] == nb and stats["allreduce_ms_per_step"] > 0


def _resnet_rank(rank, world, port, backend, out):
    """3 classification steps per rank (eager warm-up, forward capture + replay, replay) with the DDP
    bucketer, the BN-buffer broadcast and the side-stream weight gradients; graph_forward on, then off."""
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    import __graft_entry__

    __graft_entry__.load_package()
    import torch.distributed as dist

    from spine_vision_amd.training import Classifier, StepEngine
    from spine_vision_amd.training.trainers.classification import _create_tasks_for_training

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    if backend == "nccl":
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
    else:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    tasks = _create_tasks_for_training(target_labels=["pfirrmann", "modic", "herniation"], label_smoothing=0.1)
    res = []
    for gf in (True, False):
        torch.manual_seed(11)
        m = Classifier("resnet50", tasks=tasks, pretrained=False, dropout=0.0, precision="bf16").to(dev).train()
        m.backbone.graph_forward = gf
        eng = StepEngine(m, dev, lr=1e-4, weight_decay=1e-5, grad_clip=1.0, distributed=True, bucket_mb=16.0)
        g = torch.Generator().manual_seed(100 + rank)
        losses = []
        for _ in range(3):
            img = torch.rand(2, 3, 64, 64, generator=g).to(dev)
            tg = {"pfirrmann": torch.randint(0, 5, (2,), generator=g).to(dev),
                  "modic": torch.randint(0, 4, (2,), generator=g).to(dev),
                  "herniation": torch.randint(0, 2, (2,), generator=g).float().to(dev)}
            losses.append(float(eng.step_classification(img, tg)))
        torch.cuda.synchronize()
        res.append((losses, eng.arena.param_flat.cpu().clone(), len(m.backbone._fgraphs)))
    out[rank] = res
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_resnet_graph_forward(dev):
    """Data-parallel ResNet-50 steps with the graph-replayed forward (two ranks on the box's GPU, gloo):
    the replicas stay identical (bucketed all-reduce from the side-stream grad-ready events, rank-0 BN
    buffer broadcast before each forward replay), and the trajectory equals the eager forward's bit for bit."""
    ctx = mp.get_context("spawn")
    mgr = ctx.Manager()
    out = mgr.dict()
    port = _free_port()
    procs = [ctx.Process(target=_resnet_rank, args=(r, 2, port, "gloo", out)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=300)
        assert p.exitcode == 0, f"rank exited with {p.exitcode}"
    (g0, e0), (g1, e1) = out[0], out[1]
    assert g0[2] == 1 and e0[2] == 0  # the graphed run captured its forward
    assert torch.equal(g0[1], g1[1]) and torch.equal(e0[1], e1[1])  # replicas in sync
    assert g0[0] == e0[0] and g1[0] == e1[0]  # per-rank losses: graph == eager
    assert torch.equal(g0[1], e0[1])


# the bf16 data-parallel ConvNeXt path: 512x512, 4 images per rank, so the backward's GEMM
# grids exceed the 224 CUs the comm reserve leaves them (S1 fc1: 512 tiles) and the cap is exercised
B16, S16 = 4, 512


def _bf16_batch():
    from oracle import weights as ow

    img, coords, mask = ow.localization_batch(2 * B16, S16, S16)
    return img, coords, torch.ones_like(mask)


def _bf16_rank(rank, world, port, out, bucket_mb=16.0):
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    import __graft_entry__

    __graft_entry__.load_package()
    import torch.distributed as dist

    from spine_vision_amd.training import StepEngine

    # the optional 32-CU comm reserve (grid caps on every backward GEMM; the default reserves nothing): caps are
    # bitwise neutral, so the reference below runs without them
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), SV_COMM_RESERVE_CUS="32")
    os.environ.pop("SV_COMM_CU_MASK", None)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda:0")
    m = _model(dev, "bf16")
    if rank == 1:  # the broadcast must overwrite a diverged replica
        with torch.no_grad():
            m.backbone.stages[2].blocks[5].mlp.fc1.bias.add_(1.0)
    eng = StepEngine(m, dev, lr=1e-4, weight_decay=1e-5, grad_clip=1.0, distributed=True, bucket_mb=bucket_mb)
    bb = m.backbone
    ds = bb.stages[3].downsample[0].weight
    first_ends_on_ds = eng.arena.params[eng.bucketer.buckets[0][2][-1]] is ds
    setup = (bb.comm_reserve_cus, bb.lean_sync, bb.overlap_wgrad, bb.precision, first_ends_on_ds)
    img, coords, mask = _bf16_batch()
    sl = slice(rank * B16, (rank + 1) * B16)
    loss = eng.step_localization(img[sl].to(dev), coords[sl].to(dev), mask[sl].to(dev))
    torch.cuda.synchronize()
    out[rank] = (float(loss), eng.arena.grad_flat.cpu().clone(), eng.arena.param_flat.cpu().clone(),
                 len(eng.bucketer.buckets), setup)
    dist.barrier()
    dist.destroy_process_group()


def _run_bf16_ranks(bucket_mb):
    ctx = mp.get_context("spawn")
    mgr = ctx.Manager()
    out = mgr.dict()
    port = _free_port()
    procs = [ctx.Process(target=_bf16_rank, args=(r, 2, port, out, bucket_mb)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=500)
        assert p.exitcode == 0, f"rank exited with {p.exitcode}"
    return out[0], out[1]


def _half_batch_average(dev, losses):
    from spine_vision_amd.training import StepEngine

    img, coords, mask = _bf16_batch()
    halves = []
    for r in range(2):
        m = _model(dev, "bf16")
        eng = StepEngine(m, dev, lr=1e-4, weight_decay=1e-5, grad_clip=1.0, distributed=False)
        sl = slice(r * B16, (r + 1) * B16)
        lr_ = float(eng.step_localization(img[sl].to(dev), coords[sl].to(dev), mask[sl].to(dev)))
        torch.cuda.synchronize()
        assert lr_ == losses[r]  # each rank's loss is its half-batch loss
        halves.append(eng.arena.grad_flat.cpu().clone())
        del eng, m
    return (halves[0] + halves[1]) / 2


@pytest.mark.timeout(600)
def test_two_rank_bf16_lean_step_equals_half_batch_average(dev):
    """Two ranks (gloo, the box's one GPU) run the bf16 ConvNeXt-base step exactly as StepEngine sets it up under
    data parallelism: the lean side-stream backward with per-block grad-ready events launching the bucketed
    all-reduce, here with every backward GEMM grid capped by the optional 32-CU comm reserve.  The replicas end bit-identical, and
    the all-reduced gradient equals, bit for bit, the average of two single-process half-batch gradients
    ((g0 + g1) / 2 in f32: a 2-rank SUM is order-free and the halving exact).  Reference: accelerate DDP
    (spine_vision/training/trainers/base.py:253-266), LocalizationTrainer._train_step (localization.py:186-209)."""
    (l0, g0, p0, nb, setup0), (l1, g1, p1, _, setup1) = _run_bf16_ranks(16.0)
    assert setup0[:4] == setup1[:4] == (32, True, True, "bf16"), setup0
    assert nb > 1
    assert torch.equal(g0, g1) and torch.equal(p0, p1)
    avg = _half_batch_average(dev, (l0, l1))
    diff = (g0 - avg).abs().max()
    print(f"[ddp] bf16 world 2: {nb} buckets, max |allreduced - half-batch average| = {float(diff):.3e}")
    assert torch.equal(g0, avg)


@pytest.mark.timeout(600)
def test_two_rank_bucket_ending_on_downsample_waits_for_every_stream(dev):
    """a bucket whose last-reported parameter is a downsample's (reported on the main stream)
    while the same bucket's block weight gradients come from the side stream.  bucket_mb is chosen so the first
    bucket (from the end of the flat buffer: head + stage-4 blocks) closes exactly on stages[3].downsample's first
    parameter; GradBucketer must make the comm stream wait on both streams' events, so the all-reduced gradient is
    still bit for bit the half-batch average."""
    from spine_vision_amd.training.flat import _align

    m = _model(dev, "bf16")
    ds = m.backbone.stages[3].downsample[0].weight
    sizes, seen, i_ds = [], set(), None
    for p in m.parameters():  # FlatArena's order and 64-B aligned offsets
        if id(p) in seen:
            continue
        seen.add(id(p))
        if p is ds:
            i_ds = len(sizes)
        sizes.append(_align(p.numel()))
    bucket_mb = sum(sizes[i_ds:]) * 4 / 2**20
    del m
    (l0, g0, p0, nb, setup0), (l1, g1, p1, _, setup1) = _run_bf16_ranks(bucket_mb)
    assert setup0 == setup1 == (32, True, True, "bf16", True), setup0
    assert torch.equal(g0, g1) and torch.equal(p0, p1)
    avg = _half_batch_average(dev, (l0, l1))
    print(f"[ddp] bucket_mb {bucket_mb:.2f}: {nb} buckets, first ends on the stage-4 downsample, "
          f"max |allreduced - half-batch average| = {float((g0 - avg).abs().max()):.3e}")
    assert torch.equal(g0, avg)
