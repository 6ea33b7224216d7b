"""GPU: the fp32 HIP trainer against fixtures written by the REFERENCE's own trainer code
(tests/golden/make_golden_r2.py):

* one ``ClassificationTrainer._train_step`` (trainers/classification.py:269-290): ResNet-50, 3 heads,
  128x128, B=4 -- loss, updated head weights, BN running statistics, per-tensor update statistics;
* a 3-epoch ``LocalizationTrainer.train()`` (trainers/base.py:420-545) on ConvNeXt-base @64: every
  epoch's train/val loss, MED/MAE/PCK and LR, the best epoch, the best-checkpoint reload that replaces
  ``history`` (base.py:521-524), the optimizer step count in the checkpoint and the final parameters --
  with and without ``freeze_backbone_epochs=1`` (backbone frozen in epoch 0; torch AdamW then starts the
  backbone's own step count at 1, which FlatAdamW's per-parameter counts reproduce);
* the structure of the best_model.pt the reference's ``_save_checkpoint`` (base.py:687-719) writes.

The reference's LocalizationTrainer shuffles with an unseeded loader (its DataLoader has no
generator, trainers/localization.py:163-180), so the fixture records the order it drew and the test
replays that order through the trainer's sampler override point.
"""

import json
import os

import numpy as np
import pytest
import torch

from oracle import weights as ow

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _json(name):
    with open(os.path.join(GOLD, name)) as f:
        return json.load(f)


def _cs(t):
    t = t.detach().double().cpu()
    return [float(t.sum()), float((t * t).sum()), float(t.abs().max())]


def test_classification_step_matches_reference_trainer(dev, tmp_path):
    from spine_vision_amd.training import ClassificationConfig, ClassificationTrainer, Classifier
    from spine_vision_amd.training.datasets.classification import DynamicTargets
    from spine_vision_amd.training.trainers.classification import _create_tasks_for_training

    meta = _json("classification_step_resnet50_128.json")
    g = np.load(os.path.join(GOLD, "classification_step_resnet50_128.npz"))
    labels = ["pfirrmann", "modic", "herniation"]
    tasks = _create_tasks_for_training(target_labels=labels, label_smoothing=0.1)
    m = Classifier(backbone="resnet50", tasks=tasks, pretrained=False, dropout=0.0, precision="fp32")
    ow.fill_module(m)
    before = {k: v.detach().clone() for k, v in m.state_dict().items()}
    img, targets = ow.classification_batch(meta["B"], meta["res"], meta["res"])
    assert np.allclose(_cs(img), meta["img"], rtol=1e-9)

    class _DS(torch.utils.data.Dataset):
        def __len__(self):
            return meta["B"]

        def __getitem__(self, i):
            raise RuntimeError("not iterated")

    cfg = ClassificationConfig(output_path=tmp_path, batch_size=meta["B"], num_workers=0, pin_memory=False,
                               learning_rate=1e-4, weight_decay=1e-5, grad_clip=1.0, backbone="resnet50",
                               pretrained=False, dropout=0.0, target_labels=labels, label_smoothing=0.1,
                               use_weighted_sampling=False, precision="fp32")
    tr = ClassificationTrainer(cfg, model=m, train_dataset=_DS(), val_dataset=_DS())
    loss = float(tr._train_step({"image": img, "targets": DynamicTargets(dict(targets))}))
    torch.cuda.synchronize()
    assert abs(loss - meta["loss"]) / abs(meta["loss"]) < 1e-3, (loss, meta["loss"])
    lr = 1e-4
    sd = {k: v.detach().cpu() for k, v in tr.model.state_dict().items()}
    for k, ref in meta["checksums"].items():
        v = sd[k]
        if not v.is_floating_point():
            assert int(v) == ref, k
            continue
        if "running" in k:  # BatchNorm running statistics: momentum 0.1, unbiased batch variance
            got = _cs(v)  # (the plain sum of a running mean can sit near zero: compare its L2 and max)
            assert abs(got[1] - ref[1]) <= 1e-4 * ref[1] + 1e-12 and abs(got[2] - ref[2]) <= 1e-4 * ref[2] + 1e-9, (
                k, got, ref)
            continue
        # the first AdamW step moves every element by ~lr * sign(g); a gradient within fp32 noise of
        # zero may take the other sign: compare the update's size statistics, and the element-wise update
        # where the reference's tensor is stored
        d_ref = meta["delta_checksums"][k]
        d = _cs(v - before[k])
        assert abs(d[1] - d_ref[1]) <= 0.02 * d_ref[1] + 1e-12, (k, d, d_ref)
        assert d[2] <= 2.0 * lr * 1.001 + 1e-7, k
        if "after_step/" + k in g:
            assert float((v - torch.from_numpy(g["after_step/" + k])).abs().max()) <= 2.0 * lr * 1.001 + 1e-7, k


class _LocDS(torch.utils.data.Dataset):
    def __init__(self, n, seed, res):
        self.img, self.coords, self.mask = ow.localization_batch(n, res, res, seed=seed)

    def __len__(self):
        return self.img.shape[0]

    def __getitem__(self, i):
        return {"image": self.img[i], "coords": self.coords[i], "mask": self.mask[i], "series_type_idx": 0,
                "metadata": {"index": int(i)}}


class _ReplayOrder(torch.utils.data.Sampler):
    def __init__(self, orders):
        self.orders, self.epoch = orders, 0

    def __iter__(self):
        order = self.orders[min(self.epoch, len(self.orders) - 1)]
        self.epoch += 1
        return iter(order)

    def __len__(self):
        return len(self.orders[0])


def _pck_close(a, b, n_valid):
    return abs(a - b) <= 100.0 / n_valid + 1e-9  # one sample may sit within fp32 noise of a threshold


@pytest.mark.parametrize("freeze", [False, True])
def test_localization_trajectory_matches_reference_trainer(dev, tmp_path, freeze):
    from spine_vision_amd.training import CoordinateRegressor, LocalizationConfig, LocalizationTrainer

    meta = _json(f"trajectory_localization{'_freeze' if freeze else ''}.json")
    c = meta["config"]

    class Trainer(LocalizationTrainer):
        def _sampler(self, dataset, shuffle):
            if shuffle:
                return _ReplayOrder(meta["train_order"])
            return super()._sampler(dataset, shuffle)

    model = CoordinateRegressor("convnext_base", pretrained=False, dropout=0.0, freeze_backbone=freeze,
                                precision="fp32")
    ow.fill_module(model)
    cfg = LocalizationConfig(output_path=tmp_path, batch_size=c["batch_size"], num_epochs=c["num_epochs"],
                             num_workers=0, pin_memory=False, learning_rate=c["learning_rate"],
                             weight_decay=c["weight_decay"], grad_clip=c["grad_clip"], pretrained=False, dropout=0.0,
                             early_stopping=False, save_frequency=100, freeze_backbone_epochs=c["freeze_backbone_epochs"],
                             image_size=(c["res"], c["res"]), precision="fp32", seed=42)
    tr = Trainer(cfg, model=model, train_dataset=_LocDS(c["train_n"], c["train_seed"], c["res"]),
                 val_dataset=_LocDS(c["val_n"], c["val_seed"], c["res"]))
    assert tr.scheduler.T_max == meta["scheduler_T_max"]
    live = []
    orig_end = tr.on_epoch_end
    tr.on_epoch_end = lambda e, m: (live.append(dict(m)), orig_end(e, m))
    res = tr.train()
    n_valid = int(sum(float(_LocDS(c["val_n"], c["val_seed"], c["res"]).mask.sum()) for _ in [0]))
    assert len(live) == len(meta["epoch_end_metrics"])
    for ep, (got, ref) in enumerate(zip(live, meta["epoch_end_metrics"])):
        for k, v in ref.items():
            if v is None:
                continue
            if k.startswith("pck"):
                assert _pck_close(got[k], v, n_valid), (ep, k, got[k], v)
            else:
                assert abs(got[k] - v) <= 1e-3 * abs(v) + 1e-7, (ep, k, got[k], v)
    r = meta["result"]
    assert res.best_epoch == r["best_epoch"]
    assert abs(res.best_metric - r["best_metric"]) <= 1e-3 * abs(r["best_metric"])
    assert set(res.history) == set(r["history"])
    assert res.history["lr"] == r["history"]["lr"]  # same scheduler arithmetic, bit for bit
    for k, v in r["history"].items():
        assert len(res.history[k]) == len(v), k  # history replaced by the best checkpoint's
    for k in ("train_loss", "val_loss", "med", "mae"):
        np.testing.assert_allclose(res.history[k], r["history"][k], rtol=1e-3, atol=1e-7, err_msg=k)
    params = dict(tr.model.named_parameters())
    for k, ref in meta["final_param_checksums"].items():
        got = _cs(params[k])
        assert abs(got[1] - ref[1]) <= 1e-3 * ref[1], (k, got, ref)
        assert abs(got[2] - ref[2]) <= 1e-3 * ref[2] + 1e-6, (k, got, ref)
    for k, ref in meta["final_small_params"].items():
        d = float((params[k].detach().cpu().reshape(-1) - torch.tensor(ref)).abs().max())
        assert d <= 2.5 * c["learning_rate"] * 3 + 1e-6, (k, d)  # a few sign-flip steps at most
    ck = torch.load(tmp_path / "best_model.pt", map_location="cpu", weights_only=False)  # our own file
    steps = sorted({int(float(s["step"])) for s in ck["optimizer_state_dict"]["state"].values()})
    assert steps == meta["optimizer_steps_in_checkpoint"]
    assert len(ck["optimizer_state_dict"]["state"]) == meta["optimizer_state_count"]
    assert ck["epoch"] == meta["checkpoint_epoch"]
    if not freeze:
        _check_schema(ck, _json("checkpoint_schema.json"))


def _check_schema(ck, s):
    assert sorted(ck.keys()) == s["top_level_keys"]
    msd = {k: {"tensor": str(v.dtype).replace("torch.", ""), "shape": list(v.shape)}
           for k, v in ck["model_state_dict"].items()}
    assert msd == s["model_state_dict"]
    opt = ck["optimizer_state_dict"]
    assert set(s["optimizer_param_groups_keys"]) <= set(opt["param_groups"][0].keys())
    assert len(opt["state"]) == s["optimizer_state_count"]
    entry = next(iter(opt["state"].values()))
    assert {k: ({"tensor": str(v.dtype).replace("torch.", ""), "shape": list(v.shape)} if torch.is_tensor(v) else
                type(v).__name__) for k, v in entry.items()} == s["optimizer_state_entry"]
    assert sorted(ck["scheduler_state_dict"].keys()) == s["scheduler_state_keys"]
    assert sorted(ck["history"].keys()) == s["history_keys"]
    for k, t in s["config_field_types"].items():
        assert k in ck["config"], k
        assert type(ck["config"][k]).__name__ == t, (k, type(ck["config"][k]).__name__, t)
    for k, t in s["types"].items():
        assert type(ck[k]).__name__ == t, k
