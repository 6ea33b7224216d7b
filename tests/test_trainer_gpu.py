"""GPU: the product trainer end to end -- LocalizationTrainer with the HIP ConvNeXt-base backbone,
flat fused AdamW, device-side clip; two epochs on synthetic 64x64 data, checkpoint round trip."""

import pytest
import torch

from spine_vision_amd.backbone import create_resnet
from spine_vision_amd.training import Classifier, CoordinateRegressor, LocalizationConfig, LocalizationTrainer
from spine_vision_amd.training.datasets import SyntheticLocalizationDataset

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("precision", ["bf16", "fp32"])
def test_localization_trainer_gpu(dev, tmp_path, precision):
    cfg = LocalizationConfig(output_path=tmp_path, batch_size=4, num_epochs=2, num_workers=0, image_size=(64, 64),
                             pretrained=False, precision=precision, save_frequency=1, early_stopping=False)
    tr = LocalizationTrainer(cfg, train_dataset=SyntheticLocalizationDataset(8, (64, 64), seed=1),
                             val_dataset=SyntheticLocalizationDataset(4, (64, 64), seed=2))
    assert isinstance(tr.model, CoordinateRegressor)
    before = tr.model.backbone.stem[0].weight.detach().clone()
    res = tr.train()
    assert res.final_train_loss == res.final_train_loss and res.final_train_loss > 0
    assert not torch.equal(before, tr.model.backbone.stem[0].weight.detach())
    assert (tmp_path / "best_model.pt").exists() and (tmp_path / "checkpoint_epoch_2.pt").exists()
    ck = torch.load(tmp_path / "checkpoint_epoch_2.pt", weights_only=False)
    assert "backbone.stages.2.blocks.26.mlp.fc1.weight" in ck["model_state_dict"]
    assert len(ck["optimizer_state_dict"]["state"]) == len(list(tr.model.parameters()))


@pytest.mark.parametrize("precision", ["bf16", "fp32"])
def test_device_transform_matches_host_transform(dev, precision):
    """Row f1: uint8 batches normalised on the device (inside the stem gather in bf16, by
    sv_normalize_u8_gray in fp32) give the SAME training step as the reference's host transform:
    identical stem input bits, so identical loss, gradients and updated weights."""
    from oracle import weights as ow
    from spine_vision_amd.training import StepEngine
    from spine_vision_amd.training.datasets import LocalizationCollator

    ds_u8 = SyntheticLocalizationDataset(4, (64, 64), seed=3, device_transform=True)
    ds_f = SyntheticLocalizationDataset(4, (64, 64), seed=3)
    col = LocalizationCollator()
    b_u8 = col([ds_u8[i] for i in range(4)])
    b_f = col([ds_f[i] for i in range(4)])
    assert b_u8["image"].dtype == torch.uint8 and b_u8["image"].shape == (4, 64, 64)
    out = []
    for batch in (b_u8, b_f):
        m = CoordinateRegressor("convnext_base", pretrained=False, dropout=0.0, precision=precision)
        ow.fill_module(m)
        m = m.to(dev).train()
        eng = StepEngine(m, dev, lr=1e-4, weight_decay=1e-5, grad_clip=1.0)
        loss = eng.step_localization(batch["image"].to(dev), batch["coords"].to(dev), batch["mask"].to(dev))
        out.append((float(loss), float(eng.last_grad_norm), m.backbone.stem[0].weight.detach().cpu(),
                    m.head[5].weight.detach().cpu()))
    (l0, n0, w0, h0), (l1, n1, w1, h1) = out
    assert l0 == l1 and n0 == n1
    assert torch.equal(w0, w1) and torch.equal(h0, h1)


@pytest.mark.parametrize("precision", ["bf16", "fp32"])
def test_classification_device_transform_matches_host_transform(dev, precision):
    """Row f1, classification: uint8 [H,W,3] crops normalised inside the ResNet stem's NHWC conversion
    give the SAME training step as the host ToTensor/Normalize batch (identical loss, grad norm, weights)."""
    from oracle import weights as ow
    from spine_vision_amd.training import StepEngine
    from spine_vision_amd.training.datasets import ClassificationCollator, SyntheticClassificationDataset
    from spine_vision_amd.training.trainers.classification import _create_tasks_for_training

    ds_u8 = SyntheticClassificationDataset(4, (64, 64), seed=3, device_transform=True)
    ds_f = SyntheticClassificationDataset(4, (64, 64), seed=3)
    col = ClassificationCollator()
    b_u8 = col([ds_u8[i] for i in range(4)])
    b_f = col([ds_f[i] for i in range(4)])
    assert b_u8["image"].dtype == torch.uint8 and b_u8["image"].shape == (4, 64, 64, 3)
    out = []
    for batch in (b_u8, b_f):
        tasks = _create_tasks_for_training(target_labels=["pfirrmann", "modic", "herniation"], label_smoothing=0.1)
        m = Classifier("resnet18", tasks=tasks, pretrained=False, dropout=0.0, precision=precision)
        ow.fill_module(m)
        m = m.to(dev).train()
        eng = StepEngine(m, dev, lr=1e-4, weight_decay=1e-5, grad_clip=1.0)
        tg = {k: v.to(dev) for k, v in batch["targets"].to_dict().items()}
        loss = eng.step_classification(batch["image"].to(dev), tg)
        out.append((float(loss), float(eng.last_grad_norm), m.backbone.conv1.weight.detach().cpu(),
                    m.backbone.bn1.running_mean.detach().cpu()))
    (l0, n0, w0, r0), (l1, n1, w1, r1) = out
    assert l0 == l1 and n0 == n1
    assert torch.equal(w0, w1) and torch.equal(r0, r1)


@pytest.mark.parametrize("backbone,precision", [("resnet18", "bf16"), ("resnet50", "fp32")])
def test_classification_trainer_gpu(dev, tmp_path, backbone, precision):
    from spine_vision_amd.training import ClassificationConfig, ClassificationTrainer
    from spine_vision_amd.training.datasets import SyntheticClassificationDataset

    cfg = ClassificationConfig(output_path=tmp_path, batch_size=4, num_epochs=2, num_workers=0, output_size=(64, 64),
                               backbone=backbone, pretrained=False, precision=precision, save_frequency=1,
                               early_stopping=False)
    tr = ClassificationTrainer(cfg, train_dataset=SyntheticClassificationDataset(8, (64, 64), seed=1),
                               val_dataset=SyntheticClassificationDataset(4, (64, 64), seed=2))
    before = tr.model.backbone.conv1.weight.detach().clone()
    rm_before = tr.model.backbone.bn1.running_mean.detach().clone()
    res = tr.train()
    assert res.final_train_loss == res.final_train_loss and res.final_train_loss > 0
    assert not torch.equal(before, tr.model.backbone.conv1.weight.detach())
    assert not torch.equal(rm_before, tr.model.backbone.bn1.running_mean.detach())
    assert (tmp_path / "best_model.pt").exists()
    ck = torch.load(tmp_path / "best_model.pt", weights_only=False)
    assert "backbone.layer4.1.bn2.running_var" in ck["model_state_dict"]


def test_classification_step_matches_oracle(dev):
    """One full ClassificationTrainer step (ResNet-50, 3 heads, fp32 parity mode) against the CPU
    oracle step (pinned to the reference by tests/golden/classification_resnet50_64.npz): loss and
    gradient norm within 1e-3; every clipped parameter gradient against the oracle run in float64,
    within max(1e-3, 3x the fp32 oracle's own error); the AdamW update bound (2 lr) and the BN running
    statistics.  Input 128x128 (B=4): the train-mode BatchNorm of layer4 then normalises over 64 values
    per channel -- at 64x64 it sees 16 and its gamma gradient is so ill-conditioned that two fp32
    summation orders (CPU oracle vs HIP) land 3e-3 and 1.4e-2 away from float64."""
    import copy

    from oracle import heads as oh
    from oracle import resnet as orn
    from oracle import step as ostep
    from oracle import weights as ow
    from spine_vision_amd.training import Classifier, StepEngine
    from spine_vision_amd.training.trainers.classification import _create_tasks_for_training

    tasks = _create_tasks_for_training(target_labels=["pfirrmann", "modic", "herniation"], label_smoothing=0.1)
    m = Classifier(backbone="resnet50", tasks=tasks, pretrained=False, dropout=0.0, precision="fp32")
    ow.fill_module(m)
    ora = oh.Classifier(orn.create("resnet50"), 2048, dropout=0.0)
    ora.load_state_dict(m.state_dict(), strict=False)
    o64 = copy.deepcopy(ora).double().train()
    m = m.to(dev).train()
    ora.train()
    img, targets = ow.classification_batch(4, 128, 128)
    lr = 1e-4
    before = {k: v.detach().cpu().clone() for k, v in m.state_dict().items()}
    eng = StepEngine(m, dev, lr=lr, weight_decay=1e-5, grad_clip=1.0)
    loss = eng.step_classification(img.to(dev), {k: v.to(dev) for k, v in targets.items()})
    opt = ostep.make_optimizer(ora, lr=lr, weight_decay=1e-5)
    l_ref, _, norm = ostep.train_step_classification(ora, opt, img, targets)
    l64 = o64.get_loss(o64(img.double()), targets)
    l64.backward()
    n64 = torch.nn.utils.clip_grad_norm_(o64.parameters(), 1.0)
    assert abs(float(loss) - l_ref) / abs(l_ref) < 1e-3
    assert abs(float(eng.last_grad_norm) - float(norm)) / float(norm) < 1e-3
    e_norm_ora = abs(float(norm) - float(n64)) / float(n64)
    assert abs(float(eng.last_grad_norm) - float(n64)) / float(n64) < max(1e-3, 3.0 * e_norm_ora)
    # HIP keeps the unclipped gradient (the clip is a scale inside the fused AdamW)
    coef = min(1.0, 1.0 / (float(eng.last_grad_norm) + 1e-6))
    hp = dict(m.named_parameters())
    p64 = dict(o64.named_parameters())
    for n, p in ora.named_parameters():
        g64 = p64[n].grad
        scale = float(g64.norm()) + 1e-30
        e_hip = float((hp[n].grad.cpu().double() * coef - g64).norm()) / scale
        e_ora = float((p.grad.double() - g64).norm()) / scale
        assert e_hip < max(1e-3, 3.0 * e_ora), (n, e_hip, e_ora)
    sd_ref = ora.state_dict()
    for k, v in m.state_dict().items():
        ref = sd_ref[k]
        if not v.is_floating_point():
            assert int(v) == int(ref), k
            continue
        if "running" in k:  # BN running statistics (momentum 0.1, unbiased variance)
            assert float((v.cpu() - ref).norm() / ref.norm()) < 1e-5, k
            continue
        du, dr = (v.cpu() - before[k]).double(), (ref - before[k]).double()
        # first AdamW step moves every element by ~lr*sign(g): a sign that differs for a gradient within
        # fp32 noise of zero can move one element by at most 2 lr, never more
        # (Adam's first step is sign-like, so the update itself is not compared in relative L2)
        assert float((du - dr).abs().max()) <= 2.0 * lr * 1.001 + 1e-7, k


@pytest.mark.parametrize("backbone", ["resnet18", "resnet50"])
def test_graphed_step_matches_eager(dev, backbone):
    """StepEngine(cuda_graph=True): the captured step (zero grads, HIP forward/backward incl. the side-stream
    weight gradients, clip, AdamW with device-side lr / bias corrections) against the eager step over 7 steps
    (eager warm-up, capture + replay, replays, then a second input signature with its own warm-up and
    capture): losses, every gradient and every parameter equal bit for bit.  (A bias correction derived
    from the f64 beta instead of the f32 one the C ABI receives differed by a few ulp: with bf16
    activations, that flipped roundings and moved layer3/4 gradients by 1e-3 two steps later.)"""
    from spine_vision_amd.training import StepEngine
    from spine_vision_amd.training.trainers.classification import _create_tasks_for_training

    tasks = _create_tasks_for_training(target_labels=["pfirrmann", "modic", "herniation"], label_smoothing=0.1)
    runs = []
    for graphed in (False, True):
        torch.manual_seed(7)
        model = Classifier(backbone, tasks=tasks, pretrained=False, dropout=0.0, precision="bf16").to(dev).train()
        eng = StepEngine(model, dev, lr=1e-4, weight_decay=1e-5, grad_clip=1.0, cuda_graph=graphed)
        g = torch.Generator().manual_seed(3)
        losses = []
        grads2 = None
        for step in range(7):
            B = 4 if step < 5 else 2  # a second signature: eager warm-up, then its own capture
            img = torch.rand(B, 3, 64, 64, generator=g).to(dev)
            tg = {"pfirrmann": torch.randint(0, 5, (B,), generator=g).to(dev),
                  "modic": torch.randint(0, 4, (B,), generator=g).to(dev),
                  "herniation": torch.randint(0, 2, (B,), generator=g).float().to(dev)}
            losses.append(eng.step_classification(img, tg))
            if step in (1, 2):  # capture + first replay, second replay: gradients against the eager step's
                torch.cuda.synchronize()
                grads2 = (grads2 or []) + [{n: p.grad.detach().cpu().clone() for n, p in model.named_parameters()}]
        torch.cuda.synchronize()
        assert len(eng._graphs) == (2 if graphed else 0)
        runs.append(([float(x) for x in losses], [p.detach().cpu().clone() for p in model.parameters()], grads2))
    (la, pa, ga), (lb, pb, gb) = runs
    assert la == lb
    for k in range(2):
        assert all(torch.equal(ga[k][n], gb[k][n]) for n in ga[k])
    assert all(torch.equal(x, y) for x, y in zip(pa, pb))


def test_adamw_graph_replay_bitwise(dev):
    """FlatAdamW.step_graph with device [lr, 1-b1^t, sqrt(1-b2^t)] (sv_adamw_flat_dev), captured once and
    replayed with the scalars of each step, equals the eager step() bit for bit (same f32 rounding of the
    bias corrections as sv_adamw_flat derives on the host), including an lr change between steps."""
    from spine_vision_amd.training.flat import FlatArena
    from spine_vision_amd.training.optim import FlatAdamW

    def make():
        torch.manual_seed(5)
        m = torch.nn.Sequential(torch.nn.Linear(64, 96), torch.nn.Linear(96, 10)).to(dev)
        arena = FlatArena(m, dev, with_shadow=True)
        return m, arena, FlatAdamW(arena, lr=1e-3, weight_decay=1e-2)

    grads = [torch.randn(4096, generator=torch.Generator().manual_seed(i)) for i in range(4)]
    (m1, a1, o1), (m2, a2, o2) = make(), make()
    scale = torch.tensor([0.7], device=dev)
    graph = hyper = None
    for i, gr in enumerate(grads):
        lr = 1e-3 if i < 2 else 5e-4
        for o, a in ((o1, a1), (o2, a2)):
            o.param_groups[0]["lr"] = lr
            a.grad_flat.zero_()
            a.grad_flat[: gr.numel()].copy_(gr.to(dev)[: a.grad_flat.numel()])
        o1.step(grad_scale=scale)
        ranges, vals = o2.begin_graph_step()
        if graph is None:
            hyper = torch.zeros(len(ranges), 4, device=dev)
            torch.cuda.synchronize()
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph):
                o2.step_graph(ranges, hyper, grad_scale=scale)
        hyper.copy_(torch.tensor(vals))
        graph.replay()
    torch.cuda.synchronize()
    assert torch.equal(a1.param_flat, a2.param_flat)
    assert torch.equal(o1.exp_avg, o2.exp_avg) and torch.equal(o1.exp_avg_sq, o2.exp_avg_sq)
    assert torch.equal(a1.shadow_flat, a2.shadow_flat)


@pytest.mark.parametrize("backbone", ["resnet18", "resnet50"])
def test_resnet_graph_forward_matches_eager(dev, backbone):
    """ResNetHip.graph_forward (default): the training forward replayed from a captured graph, the backward
    eager from its static tape.  Same kernels as the eager forward: losses, gradients, parameters and BN
    running statistics equal bit for bit over 7 steps (warm-up, capture + replay, replays, a second input
    signature with its own capture), side stream on."""
    from spine_vision_amd.training import StepEngine
    from spine_vision_amd.training.trainers.classification import _create_tasks_for_training

    tasks = _create_tasks_for_training(target_labels=["pfirrmann", "modic", "herniation"], label_smoothing=0.1)
    runs = []
    for gf in (False, True):
        torch.manual_seed(7)
        model = Classifier(backbone, tasks=tasks, pretrained=False, dropout=0.0, precision="bf16").to(dev).train()
        model.backbone.graph_forward = gf
        eng = StepEngine(model, dev, lr=1e-4, weight_decay=1e-5, grad_clip=1.0)
        g = torch.Generator().manual_seed(3)
        losses, grads = [], []
        for step in range(7):
            B = 4 if step < 5 else 2
            img = torch.rand(B, 3, 64, 64, generator=g).to(dev)
            tg = {"pfirrmann": torch.randint(0, 5, (B,), generator=g).to(dev),
                  "modic": torch.randint(0, 4, (B,), generator=g).to(dev),
                  "herniation": torch.randint(0, 2, (B,), generator=g).float().to(dev)}
            losses.append(float(eng.step_classification(img, tg)))
            torch.cuda.synchronize()
            grads.append([p.grad.detach().cpu().clone() for p in model.parameters()])
        assert len(model.backbone._fgraphs) == (2 if gf else 0)
        runs.append((losses, grads, [p.detach().cpu().clone() for p in model.parameters()],
                     [b.detach().cpu().clone() for b in model.buffers()]))
    (la, ga, pa, ba), (lb, gb, pb, bb) = runs
    assert la == lb
    assert all(torch.equal(x, y) for sa, sb in zip(ga, gb) for x, y in zip(sa, sb))
    assert all(torch.equal(x, y) for x, y in zip(pa, pb))
    assert all(torch.equal(x, y) for x, y in zip(ba, bb))


def test_resnet_graph_forward_follows_rebound_storage(dev):
    """a captured forward graph bakes in the weights', buffers' and bf16 shadows' addresses.  After
    the graph is captured, (1) a FlatArena rebinds every parameter and installs a bf16 shadow, (2) a BufferSync
    rebinds the BatchNorm buffers, (3) the new storage is updated in place.  Each time the next forward must
    read the new storage (graphs dropped and re-captured): it equals a graph-less twin's bit for bit."""
    from spine_vision_amd.training.comm import BufferSync
    from spine_vision_amd.training.flat import FlatArena

    torch.manual_seed(0)
    a = create_resnet("resnet18", precision="bf16").to(dev).eval()
    b = create_resnet("resnet18", precision="bf16").to(dev).eval()
    b.load_state_dict(a.state_dict())
    b.graph_forward = False
    x = torch.rand(4, 3, 64, 64, generator=torch.Generator().manual_seed(1)).to(dev)

    def check(n=3):
        with torch.no_grad():
            fa = [a(x) for _ in range(n)]
            fb = b(x)
        torch.cuda.synchronize()
        assert all(torch.equal(f, fb) for f in fa)

    check()
    assert len(a._fgraphs) == 1
    arenas = [FlatArena(net, dev, with_shadow=True) for net in (a, b)]  # (1)
    check()
    for net in (a, b):  # (2)
        BufferSync(net)
    with torch.no_grad():
        for net in (a, b):
            for name, buf in net.named_buffers():
                if name.endswith("running_mean"):
                    buf.add_(0.25)
    check()
    with torch.no_grad():  # (3) in place: the addresses stay, the graphs read the new values
        for ar in arenas:
            ar.param_flat.mul_(0.5)
            ar.refresh_shadow()
    check()
    assert len(a._fgraphs) == 1


def test_resnet_graph_forward_two_forwards_one_backward(dev):
    """two training forwards before one backward (a two-view loss).  The second forward must not
    overwrite the first one's graph-owned tape: every gradient equals the eager model's bit for bit."""
    torch.manual_seed(0)
    a = create_resnet("resnet18", precision="bf16").to(dev).train()
    b = create_resnet("resnet18", precision="bf16").to(dev).train()
    b.load_state_dict(a.state_dict())
    b.graph_forward = False
    g = torch.Generator().manual_seed(2)
    xs = [torch.rand(4, 3, 64, 64, generator=g).to(dev) for _ in range(4)]
    for net in (a, b):  # warm-up + capture for the graph model (single-forward steps)
        for x in xs[:2]:
            net(x).sum().backward()
    grads = []
    for net in (a, b):
        for p in net.parameters():
            p.grad = None
        f1 = net(xs[2])
        f2 = net(xs[3])
        (f1.square().sum() + 0.5 * f2.sum()).backward()
        torch.cuda.synchronize()
        grads.append([p.grad.detach().cpu().clone() for p in net.parameters()])
    assert len(a._fgraphs) == 1
    for ga, gb in zip(*grads):
        assert torch.equal(ga, gb)


@pytest.mark.parametrize("backbone", ["resnet50", "resnet18"])
def test_resnet_deferred_wgrad_flush_bitwise(dev, backbone, monkeypatch):
    """SV_DEFER_WGRAD_FLUSH: each block's side-stream weight gradients enqueued after the next block's first
    BatchNorm backward pass instead of at the block's end.  Same kernels and operands: losses, gradients, parameters
    and BN running statistics equal the in-order enqueue bit for bit over 4 steps (side stream on)."""
    from spine_vision_amd.backbone import resnet as rn
    from spine_vision_amd.training import StepEngine
    from spine_vision_amd.training.trainers.classification import _create_tasks_for_training

    tasks = _create_tasks_for_training(target_labels=["pfirrmann", "modic", "herniation"], label_smoothing=0.1)
    runs = []
    for defer in (False, True):
        monkeypatch.setattr(rn, "_DEFER_FLUSH", defer)
        torch.manual_seed(7)
        model = Classifier(backbone, tasks=tasks, pretrained=False, dropout=0.0, precision="bf16").to(dev).train()
        assert model.backbone.overlap_wgrad
        eng = StepEngine(model, dev, lr=1e-4, weight_decay=1e-5, grad_clip=1.0)
        g = torch.Generator().manual_seed(3)
        losses, grads = [], []
        for _ in range(4):
            img = torch.rand(8, 3, 128, 128, generator=g).to(dev)
            tg = {"pfirrmann": torch.randint(0, 5, (8,), generator=g).to(dev),
                  "modic": torch.randint(0, 4, (8,), generator=g).to(dev),
                  "herniation": torch.randint(0, 2, (8,), generator=g).float().to(dev)}
            losses.append(float(eng.step_classification(img, tg)))
            torch.cuda.synchronize()
            grads.append([p.grad.detach().cpu().clone() for p in model.parameters()])
        runs.append((losses, grads, [p.detach().cpu().clone() for p in model.parameters()],
                     [b.detach().cpu().clone() for b in model.buffers()]))
    (la, ga, pa, ba), (lb, gb, pb, bb) = runs
    assert la == lb
    assert all(torch.equal(x, y) for sa, sb in zip(ga, gb) for x, y in zip(sa, sb))
    assert all(torch.equal(x, y) for x, y in zip(pa, pb))
    assert all(torch.equal(x, y) for x, y in zip(ba, bb))
