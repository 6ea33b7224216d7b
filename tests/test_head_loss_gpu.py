"""The fused multi-task classification loss (sv_head_loss via Classifier.get_loss) against torch's per-task modules
(core/tasks.py create_loss_functions: CrossEntropyLoss(label_smoothing), BCEWithLogitsLoss; the reference's
models/generic.py get_loss): the loss and d(loss)/d(logits) in float32."""
import pytest
import torch

from spine_vision_amd import kernels as K
from spine_vision_amd import native as nv
from spine_vision_amd.core.tasks import TaskConfig, get_task
from spine_vision_amd.training.models import generic

pytestmark = pytest.mark.gpu


def _tasks(smoothing=0.1, weights=(1.0, 1.0, 1.0)):
    ts = [get_task("pfirrmann").with_overrides(label_smoothing=smoothing, loss_weight=weights[0]),
          get_task("modic").with_overrides(label_smoothing=smoothing, loss_weight=weights[1]),
          get_task("herniation").with_overrides(loss_weight=weights[2])]
    return ts


def _targets(B, g, dev, ignore=0):
    t = {"pfirrmann": torch.randint(0, 5, (B,), generator=g), "modic": torch.randint(0, 4, (B,), generator=g),
         "herniation": (torch.rand(B, generator=g) < 0.3).float()}
    if ignore:
        t["pfirrmann"][:ignore] = -100
    return {k: v.to(dev) for k, v in t.items()}


def _loss_and_grad(model, logits, targets, fused):
    x = logits.clone().requires_grad_(True)
    pred = generic._HeadOutputs(zip(["pfirrmann", "modic", "herniation"], x.split([5, 4, 1], dim=1)))
    pred.logits = x
    with pytest.MonkeyPatch.context() as mp:
        mp.setattr(generic, "_FUSED_LOSS", fused)
        loss = model.get_loss(pred, targets)
    (loss * 0.75).backward()
    return loss.detach(), x.grad


@pytest.mark.parametrize("B,ignore,smoothing,weights", [(32, 0, 0.1, (1.0, 1.0, 1.0)), (3, 0, 0.0, (1.0, 1.0, 1.0)),
                                                        (300, 7, 0.1, (0.5, 2.0, 1.5)), (32, 32, 0.2, (1.0, 1.0, 1.0))])
def test_fused_head_loss_matches_torch(dev, B, ignore, smoothing, weights):
    g = torch.Generator().manual_seed(B + ignore)
    model = generic.Classifier("resnet18", tasks=_tasks(smoothing, weights), pretrained=False, dropout=0.0,
                               precision="fp32")
    logits = (torch.randn(B, 10, generator=g) * 3).to(dev)
    targets = _targets(B, g, dev, ignore)
    plain = {"pfirrmann": logits[:, :5], "modic": logits[:, 5:9], "herniation": logits[:, 9:]}
    assert model._fused_loss_specs(plain, targets) is None  # a plain dict (no .logits) takes the torch path
    lf, gf = _loss_and_grad(model.to(dev), logits, targets, True)
    lt, gt = _loss_and_grad(model, logits, targets, False)
    if ignore == B:  # torch: a mean over no valid rows is NaN; the fused loss counts that task as 0
        assert torch.isnan(lt)
        return
    assert abs(float(lf) - float(lt)) <= 2e-6 * abs(float(lt)) + 1e-7, (float(lf), float(lt))
    assert float((gf - gt).abs().max()) <= 1e-6 * float(gt.abs().max()) + 1e-8


def test_fused_head_loss_multilabel_and_kernel_contract(dev):
    """A 3-column BCE task (multilabel) beside a CE task, with bf16 targets, straight through kernels.head_loss;
    logits columns no task covers get a zero gradient."""
    g = torch.Generator().manual_seed(3)
    B = 17
    logits = torch.randn(B, 12, generator=g).to(dev)
    y = torch.randint(0, 6, (B,), generator=g).to(dev)
    t = (torch.rand(B, 3, generator=g) < 0.5).to(dev, torch.bfloat16)
    loss, dl = K.head_loss(logits, [(nv.SV_HEAD_CE, 0, 6, 0.7, 0.05, y), (nv.SV_HEAD_BCE, 8, 3, 1.3, 0.0, t)])
    x = logits.clone().requires_grad_(True)
    ref = 0.7 * torch.nn.functional.cross_entropy(x[:, :6], y, label_smoothing=0.05) + \
        1.3 * torch.nn.functional.binary_cross_entropy_with_logits(x[:, 8:11], t.float())
    ref.backward()
    torch.cuda.synchronize()
    assert abs(float(loss) - float(ref)) <= 2e-6 * abs(float(ref))
    assert float((dl - x.grad).abs().max()) <= 1e-6
    assert float(dl[:, 6:8].abs().max()) == 0.0 and float(dl[:, 11:].abs().max()) == 0.0


def test_classifier_step_uses_fused_loss(dev):
    """The whole Classifier (resnet18 backbone, fused heads): the fused loss path gives torch's loss and the same
    head / backbone gradients to float32 rounding."""
    torch.manual_seed(0)
    tasks = _tasks()
    ms = []
    for _ in range(2):
        m = generic.Classifier("resnet18", tasks=tasks, pretrained=False, dropout=0.0, precision="fp32").to(dev)
        ms.append(m)
    ms[1].load_state_dict(ms[0].state_dict())
    g = torch.Generator().manual_seed(1)
    img = torch.rand(4, 3, 64, 64, generator=g).to(dev)
    targets = _targets(4, g, dev)
    losses = []
    for m, fused in zip(ms, (True, False)):
        m.train()
        with pytest.MonkeyPatch.context() as mp:
            mp.setattr(generic, "_FUSED_LOSS", fused)
            out = m(img)
            assert isinstance(out, generic._HeadOutputs)
            loss = m.get_loss(out, targets)
        loss.backward()
        losses.append(float(loss))
    assert abs(losses[0] - losses[1]) <= 1e-5 * abs(losses[1])
    for (n, p0), p1 in zip(ms[0].named_parameters(), ms[1].parameters()):
        if p0.grad is None:
            continue
        err = float((p0.grad - p1.grad).norm() / (p1.grad.norm() + 1e-30))
        assert err < 1e-4, (n, err)


def test_task_config_with_focal_loss_falls_back(dev):
    """A focal-loss binary task is not the kernel's: get_loss takes torch's modules for the whole set."""
    tasks = _tasks()[:2] + [TaskConfig("herniation", 1, "binary", use_focal_loss=True)]
    m = generic.Classifier("resnet18", tasks=tasks, pretrained=False, dropout=0.0, precision="fp32")
    g = torch.Generator().manual_seed(2)
    logits = torch.randn(8, 10, generator=g).to(dev)
    pred = generic._HeadOutputs(zip(["pfirrmann", "modic", "herniation"], logits.split([5, 4, 1], dim=1)))
    pred.logits = logits
    assert m._fused_loss_specs(pred, _targets(8, g, dev)) is None


@pytest.mark.parametrize("bad", [5, -3], ids=["past-ncls", "negative"])
def test_fused_head_loss_out_of_range_target_is_loud(dev, bad):
    """A CE target outside [0, ncls) that is not ignore_index: torch stops with a device-side assert; the fused loss
    makes the loss and that row's logits gradient NaN instead of silently dropping the one-hot term."""
    g = torch.Generator().manual_seed(11)
    model = generic.Classifier("resnet18", tasks=_tasks(), pretrained=False, dropout=0.0, precision="fp32").to(dev)
    logits = (torch.randn(8, 10, generator=g) * 3).to(dev)
    targets = _targets(8, g, dev)
    targets["pfirrmann"][3] = bad
    lf, gf = _loss_and_grad(model, logits, targets, True)
    assert torch.isnan(lf)
    assert torch.isnan(gf[3, :5]).all()
    assert torch.isfinite(gf[:3]).all() and torch.isfinite(gf[4:]).all() and torch.isfinite(gf[3, 5:]).all()
