"""CPU: trainer host logic (loop, history, scheduler quirk, checkpoints, early stop, sharding).

The product backbone needs the HIP library, so these tests inject a small CPU model and a torch
optimizer through the reference's own override points (``model=`` and ``_create_optimizer``,
spine_vision/training/trainers/base.py:384-390) -- exactly what a reference user can do."""

import pytest
import torch

from oracle import convnext as oc
from oracle import heads as oh
from spine_vision_amd.training.datasets import SyntheticClassificationDataset, SyntheticLocalizationDataset
from spine_vision_amd.training.trainers import (
    ClassificationConfig,
    ClassificationTrainer,
    LocalizationConfig,
    LocalizationTrainer,
    ShardedBatchSampler,
)


class TinyLoc(oh.CoordinateRegressor):
    name = "tiny"

    def __init__(self):
        super().__init__(oc.ConvNeXt((1, 1, 1, 1), (64, 64, 64, 64)), 64, dropout=0.0)

    def get_loss(self, pred, target, mask=None):
        return super().get_loss(pred, target, mask)

    def unfreeze_backbone(self):
        for p in self.backbone.parameters():
            p.requires_grad = True


class CpuLocTrainer(LocalizationTrainer):
    def _create_optimizer(self):
        return torch.optim.AdamW(self.model.parameters(), lr=self.config.learning_rate,
                                 weight_decay=self.config.weight_decay)


def _cfg(tmp_path, **kw):
    base = dict(output_path=tmp_path, batch_size=4, num_epochs=3, num_workers=0, pin_memory=False,
                image_size=(32, 32), pretrained=False, save_frequency=2, log_frequency=1)
    base.update(kw)
    return LocalizationConfig(**base)


def test_localization_trainer_loop(tmp_path):
    cfg = _cfg(tmp_path)
    tr = CpuLocTrainer(cfg, model=TinyLoc(), train_dataset=SyntheticLocalizationDataset(12, (32, 32), seed=1),
                       val_dataset=SyntheticLocalizationDataset(8, (32, 32), seed=2))
    assert len(tr.train_loader) == 3  # drop_last on train
    res = tr.train()
    assert len(res.history["train_loss"]) >= 1 and res.final_train_loss > 0
    assert (tmp_path / "best_model.pt").exists()
    assert (tmp_path / "checkpoint_epoch_2.pt").exists()
    assert (tmp_path / "config.yaml").exists()
    ck = torch.load(tmp_path / "checkpoint_epoch_2.pt", weights_only=False)  # our own file
    assert set(ck) == {"epoch", "model_state_dict", "optimizer_state_dict", "scheduler_state_dict", "best_metric",
                       "best_epoch", "history", "config"}
    assert "med" in res.history and "pck@0.05" in res.history


def test_cosine_scheduler_quirk(tmp_path):
    """T_max counted in steps, stepped once per epoch (reference base.py:397-404 vs 471-478)."""
    cfg = _cfg(tmp_path, num_epochs=2, early_stopping=False)
    tr = CpuLocTrainer(cfg, model=TinyLoc(), train_dataset=SyntheticLocalizationDataset(16, (32, 32)),
                       val_dataset=SyntheticLocalizationDataset(4, (32, 32), seed=9))
    assert tr.scheduler.T_max == len(tr.train_loader) * 2 == 8
    seen = []
    tr.on_epoch_end = lambda epoch, m: seen.append(tr.optimizer.param_groups[0]["lr"])
    res = tr.train()
    lrs = [1e-4] + seen
    assert lrs[0] == pytest.approx(1e-4)  # recorded before the epoch's scheduler step
    import math
    expected = 1e-6 + (1e-4 - 1e-6) * (1 + math.cos(math.pi * 1 / 8)) / 2
    assert lrs[1] == pytest.approx(expected)


def test_resume_from_checkpoint(tmp_path):
    cfg = _cfg(tmp_path, num_epochs=2, early_stopping=False, save_frequency=1)
    val = SyntheticLocalizationDataset(4, (32, 32), seed=9)
    tr = CpuLocTrainer(cfg, model=TinyLoc(), train_dataset=SyntheticLocalizationDataset(8, (32, 32)), val_dataset=val)
    tr.train()
    cfg2 = _cfg(tmp_path / "b", num_epochs=3, checkpoint_path=tmp_path / "checkpoint_epoch_2.pt")
    tr2 = CpuLocTrainer(cfg2, model=TinyLoc(), train_dataset=SyntheticLocalizationDataset(8, (32, 32)),
                        val_dataset=val)
    r = tr2.train()
    assert len(r.history["train_loss"]) == 3


class TinyCls(torch.nn.Module):
    name = "tinycls"

    def __init__(self, tasks):
        super().__init__()
        from spine_vision_amd.core.tasks import create_loss_functions, get_strategy

        self.tasks = tasks
        self.backbone = torch.nn.Sequential(torch.nn.Conv2d(3, 8, 4, 4), torch.nn.AdaptiveAvgPool2d(1),
                                            torch.nn.Flatten())
        self.heads = torch.nn.ModuleDict({t.name: torch.nn.Linear(8, t.num_classes) for t in tasks})
        self.losses, self.weights = create_loss_functions(tasks)
        self._strategy = get_strategy

    def forward(self, x):
        f = self.backbone(x)
        return {k: h(f) for k, h in self.heads.items()}

    def get_loss(self, preds, targets):
        return sum(self.weights[t.name] * self.losses[t.name](preds[t.name], self._strategy(t).format_target(
            targets[t.name])) for t in self.tasks)


def test_classification_trainer_plumbing(tmp_path):
    """BASELINE configs[0] plumbing: 32 synthetic crops, bs4, 2 epochs, weighted sampling, CPU."""
    from spine_vision_amd.training.trainers.classification import _create_tasks_for_training

    class CpuCls(ClassificationTrainer):
        def _create_optimizer(self):
            return torch.optim.AdamW(self.model.parameters(), lr=1e-4, weight_decay=1e-5)

    labels = ["pfirrmann", "modic", "herniation"]
    tasks = _create_tasks_for_training(labels)
    cfg = ClassificationConfig(output_path=tmp_path, batch_size=4, num_epochs=2, num_workers=0, pin_memory=False,
                               target_labels=labels, output_size=(32, 32), pretrained=False)
    tr = CpuCls(cfg, model=TinyCls(tasks), train_dataset=SyntheticClassificationDataset(32, (32, 32), seed=3,
                                                                                       target_labels=labels),
                val_dataset=SyntheticClassificationDataset(8, (32, 32), seed=4, target_labels=labels))
    res = tr.train()
    # reference quirk: history is replaced by the best checkpoint's (base.py:521-524)
    assert len(res.history["train_loss"]) == res.best_epoch + 1
    assert "macro_f1" in res.history


@pytest.mark.parametrize("world,n,bs,drop", [(2, 37, 4, True), (2, 37, 4, False), (4, 64, 8, True), (3, 10, 3, False),
                                           (2, 100, 32, False), (4, 5, 2, False), (3, 12, 4, False), (2, 36, 4, False)])
def test_sharding_matches_accelerate(world, n, bs, drop):
    """Every rank's batches equal accelerate's BatchSamplerShard with its prepare() default
    even_batches=True (validation: the last group padded by cycling from the epoch's start)."""
    from accelerate.data_loader import BatchSamplerShard
    from torch.utils.data import BatchSampler, SequentialSampler

    lens = set()
    one = list(ShardedBatchSampler(SequentialSampler(range(n)), bs, drop, 0, 1))
    assert one == list(BatchSampler(SequentialSampler(range(n)), bs, drop))  # world 1: no sharding, no padding
    for r in range(world):
        ours = list(ShardedBatchSampler(SequentialSampler(range(n)), bs, drop, r, world))
        ref = list(BatchSamplerShard(BatchSampler(SequentialSampler(range(n)), bs, drop), num_processes=world,
                                     process_index=r, split_batches=False, even_batches=True))
        assert ours == ref, (r, ours, ref)
        assert len(ours) == len(ShardedBatchSampler(SequentialSampler(range(n)), bs, drop, r, world))
        if not drop:
            assert all(len(b) == bs for b in ours)  # equal shapes for the per-batch all-gather
        lens.add(len(ours))
    assert len(lens) == 1


def test_cosine_tmax_counts_unsharded_batches():
    """The reference creates the scheduler before accelerator.prepare shards the loader
    (base.py:243-266): T_max = unsharded batches x epochs at any world size."""
    from torch.utils.data import SequentialSampler

    for world in (1, 2, 4):
        bs = ShardedBatchSampler(SequentialSampler(range(37)), 4, True, 0, world)
        assert bs.num_batches() == 9
        assert len(bs) == 9 // world


def test_device_transform_dataset_contract():
    """Row f1 host side: with device_transform the dataset yields the decoded uint8 image and the
    collator stacks [B,H,W] uint8; normalising it gives exactly the host-transform sample."""
    from spine_vision_amd.training.datasets import LocalizationCollator, SyntheticLocalizationDataset
    from spine_vision_amd.training.datasets.localization import normalize_u8

    a = SyntheticLocalizationDataset(3, (32, 32), seed=9, device_transform=True)
    b = SyntheticLocalizationDataset(3, (32, 32), seed=9)
    for i in range(3):
        assert a[i]["image"].dtype == torch.uint8
        assert torch.equal(normalize_u8(a[i]["image"]), b[i]["image"])
        assert torch.equal(a[i]["coords"], b[i]["coords"]) and torch.equal(a[i]["mask"], b[i]["mask"])
    batch = LocalizationCollator()([a[i] for i in range(3)])
    assert batch["image"].shape == (3, 32, 32) and batch["image"].dtype == torch.uint8


def test_classification_device_transform_dataset_contract():
    """Row f1 host side, classification: construct_3channel follows the reference channel layout
    ([T2,T1,T2], else one plane replicated, classification.py:40-68); with device_transform the dataset
    yields that uint8 [H,W,3] crop and normalising it channel-first gives exactly the host sample."""
    from spine_vision_amd.training.datasets import ClassificationCollator
    from spine_vision_amd.training.datasets.classification import construct_3channel
    from spine_vision_amd.training.datasets.localization import normalize_u8

    t2 = torch.randint(0, 256, (4, 5), dtype=torch.uint8)
    t1 = torch.randint(0, 256, (4, 5), dtype=torch.uint8)
    both = construct_3channel(t2, t1)
    assert both.shape == (4, 5, 3)
    assert torch.equal(both[..., 0], t2) and torch.equal(both[..., 1], t1) and torch.equal(both[..., 2], t2)
    assert torch.equal(construct_3channel(t2, None), t2.unsqueeze(-1).expand(4, 5, 3))
    assert torch.equal(construct_3channel(None, t1), t1.unsqueeze(-1).expand(4, 5, 3))
    with pytest.raises(ValueError):
        construct_3channel(None, None)
    a = SyntheticClassificationDataset(3, (16, 16), seed=9, device_transform=True)
    b = SyntheticClassificationDataset(3, (16, 16), seed=9)
    for i in range(3):
        assert a[i]["image"].dtype == torch.uint8 and a[i]["image"].shape == (16, 16, 3)
        assert torch.equal(normalize_u8(a[i]["image"].permute(2, 0, 1)), b[i]["image"])
        assert a[i]["targets"] == b[i]["targets"]
    batch = ClassificationCollator()([a[i] for i in range(3)])
    assert batch["image"].shape == (3, 16, 16, 3) and batch["image"].dtype == torch.uint8


def test_classification_config_device_transform_reaches_datasets(tmp_path):
    """ClassificationConfig(device_transform=True) switches datasets that support it to the uint8 crop."""
    from spine_vision_amd.training.trainers.classification import _create_tasks_for_training

    class CpuCls(ClassificationTrainer):
        def _create_optimizer(self):
            return torch.optim.AdamW(self.model.parameters(), lr=1e-4, weight_decay=1e-5)

    labels = ["pfirrmann", "modic", "herniation"]
    tr_ds = SyntheticClassificationDataset(4, (16, 16), seed=1, target_labels=labels)
    va_ds = SyntheticClassificationDataset(2, (16, 16), seed=2, target_labels=labels)
    cfg = ClassificationConfig(output_path=tmp_path, batch_size=2, num_epochs=1, num_workers=0, pin_memory=False,
                               target_labels=labels, output_size=(16, 16), pretrained=False, device_transform=True)
    CpuCls(cfg, model=TinyCls(_create_tasks_for_training(labels)), train_dataset=tr_ds, val_dataset=va_ds)
    assert tr_ds.device_transform and va_ds.device_transform
    assert tr_ds[0]["image"].dtype == torch.uint8 and tr_ds[0]["image"].shape == (16, 16, 3)


def test_step_engine_refuses_graph_for_unsafe_backbone():
    """ConvNeXt's lean backward polls side-stream events, which a stream capture forbids, so
    StepEngine(cuda_graph=True) must refuse it up front instead of failing at the second step."""
    from spine_vision_amd.backbone import create_convnext, create_resnet
    from spine_vision_amd.training import StepEngine

    assert create_resnet("resnet18").graph_safe is True
    with pytest.raises(ValueError, match="capture-safe"):
        StepEngine(create_convnext("convnext_tiny"), "cpu", cuda_graph=True)
