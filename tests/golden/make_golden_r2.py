"""Round-2 golden fixtures, produced by the REFERENCE's own code (imported from /root/reference with
the shims of make_golden.py; run in the build container only -- the GPU box never needs the reference):

    python tests/golden/make_golden_r2.py

  focal_loss.json           FocalLoss (reference training/losses.py:90-139) on fixed logits/targets
  metrics.json              ClassifierMetrics (metrics.py:321-518) and LocalizationMetrics.compute
                            (metrics.py:121-185) on fixed predictions/targets
  classification_step_resnet50_128.npz
                            one ClassificationTrainer._train_step (trainers/classification.py:269-290,
                            accelerate on CPU = fp32, clip 1.0, AdamW): loss, post-step head tensors,
                            post-step checksums of backbone tensors
  trajectory_localization.json / trajectory_localization_freeze.json
                            BaseTrainer.train() (trainers/base.py:420-545) of LocalizationTrainer for 3
                            epochs (ConvNeXt-base @64, 6 train / 3 val images, bs 2): per-epoch history
                            (train/val loss, lr, MED, PCK ...), best epoch, the best-checkpoint reload
                            (history replaced, base.py:521-524), post-training parameter checksums, and
                            the batch order the reference's own (unseeded) shuffle produced.  The freeze
                            variant runs freeze_backbone_epochs=1 (generic.py:419-425 +
                            localization.py:383-389): backbone frozen in epoch 0, AdamW steps it from
                            step 1 afterwards.
  checkpoint_schema.json    the structure of the best_model.pt the reference's _save_checkpoint
                            (base.py:687-719) wrote in that run: top-level keys, every model / optimizer
                            state key with dtype and shape, scheduler state keys, config field types.
                            (The file itself is ~1 GB for ConvNeXt-base and is not committed.)
Inputs are regenerated bit-identically by oracle/weights.py; only outputs are stored.
"""

from __future__ import annotations

import json
import os
import sys
import tempfile

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_golden import ROOT, checksum, fp, import_reference  # noqa: E402

sys.path.insert(0, ROOT)
from oracle import weights as ow  # noqa: E402

torch.set_num_threads(8)
PICKS_LOC = ["backbone.stem.0.weight", "backbone.stages.0.blocks.0.conv_dw.weight",
             "backbone.stages.2.blocks.13.mlp.fc1.weight", "backbone.stages.3.blocks.2.gamma",
             "backbone.head.norm.weight", "head.0.weight", "head.2.weight", "head.5.weight", "head.5.bias"]


def dump(name, obj):
    with open(os.path.join(HERE, name), "w") as f:
        json.dump(obj, f, indent=1, sort_keys=True)


def gold_focal():
    from spine_vision.training.losses import FocalLoss

    logits = torch.from_numpy(ow.uniform("focal.logits", 24, -4.0, 4.0).reshape(12, 2))
    targets = torch.from_numpy((ow.uniform("focal.targets", 24, 0.0, 1.0) > 0.6).astype(np.float32).reshape(12, 2))
    cases = []
    for gamma, alpha, pw, red in [(2.0, None, None, "mean"), (2.0, 0.25, None, "sum"), (1.5, None, 3.0, "none"),
                                  (0.0, 0.75, 2.0, "mean"), (3.0, 0.5, 0.5, "none")]:
        out = FocalLoss(gamma=gamma, alpha=alpha, pos_weight=pw, reduction=red)(logits, targets)
        cases.append({"gamma": gamma, "alpha": alpha, "pos_weight": pw, "reduction": red,
                      "out": out.detach().reshape(-1).tolist()})
    dump("focal_loss.json", {"generator": "tests/golden/make_golden_r2.py", "logits": logits.reshape(-1).tolist(),
                             "targets": targets.reshape(-1).tolist(), "shape": [12, 2], "cases": cases})


def gold_metrics():
    from spine_vision.training.metrics import ClassifierMetrics, LocalizationMetrics

    n = 40
    preds = {"pfirrmann": torch.from_numpy(ow.uniform("m.pf", n * 5, -2, 2).reshape(n, 5)),
             "modic": torch.from_numpy(ow.uniform("m.mo", n * 4, -2, 2).reshape(n, 4)),
             "herniation": torch.from_numpy(ow.uniform("m.he", n, -2, 2).reshape(n, 1))}
    tg = {"pfirrmann": torch.from_numpy((ow.uniform("m.tpf", n, 0, 5)).astype(np.int64) % 5),
          "modic": torch.from_numpy((ow.uniform("m.tmo", n, 0, 4)).astype(np.int64) % 4),
          "herniation": torch.from_numpy((ow.uniform("m.the", n, 0, 1) > 0.6).astype(np.float32).reshape(n, 1))}
    out = {"generator": "tests/golden/make_golden_r2.py", "n": n,
           "preds": {k: v.reshape(-1).tolist() for k, v in preds.items()},
           "targets": {k: v.reshape(-1).tolist() for k, v in tg.items()}, "classifier": {}}
    for labels in (["pfirrmann", "modic", "herniation"], ["herniation"], ["pfirrmann"], ["modic", "herniation"]):
        cm = ClassifierMetrics(target_labels=labels)
        cm.update({k: preds[k][:20] for k in labels}, {k: tg[k][:20] for k in labels})  # two batches
        cm.update({k: preds[k][20:] for k in labels}, {k: tg[k][20:] for k in labels})
        out["classifier"][",".join(labels)] = cm.compute()
    m = 30
    p = ow.uniform("lm.p", m * 2, 0, 1).reshape(m, 2)
    t = ow.uniform("lm.t", m * 2, 0, 1).reshape(m, 2)
    t = np.clip(p + (t - 0.5) * 0.12, 0, 1).astype(np.float32)
    lv = (np.arange(m) % 5).astype(np.int64)
    lm = LocalizationMetrics(pck_thresholds=[0.02, 0.05, 0.10], level_names=["L1/L2", "L2/L3", "L3/L4", "L4/L5",
                                                                               "L5/S1"])
    out["localization"] = {"pred": p.reshape(-1).tolist(), "target": t.reshape(-1).tolist(), "levels": lv.tolist(),
                           "level_names": ["L1/L2", "L2/L3", "L3/L4", "L4/L5", "L5/S1"],
                           "metrics": lm.compute(p, t, lv)}
    dump("metrics.json", out)


def gold_classification_step(generic):
    from spine_vision.training.datasets.classification import DynamicTargets
    from spine_vision.training.trainers.classification import (
        ClassificationConfig,
        ClassificationTrainer,
        _create_tasks_for_training,
    )

    B, R = 4, 128
    img, targets = ow.classification_batch(B, R, R)
    labels = ["pfirrmann", "modic", "herniation"]
    tasks = _create_tasks_for_training(target_labels=labels, label_smoothing=0.1)
    model = generic.Classifier(backbone="resnet50", tasks=tasks, pretrained=False, dropout=0.0)
    ow.fill_module(model)
    before = {k: v.detach().clone() for k, v in model.state_dict().items()}

    class _DS(torch.utils.data.Dataset):
        def __len__(self):
            return B

        def __getitem__(self, i):
            raise RuntimeError("not iterated")

    tmp = tempfile.mkdtemp()
    cfg = ClassificationConfig(output_path=tmp, batch_size=B, num_workers=0, pin_memory=False, use_trackio=False,
                               learning_rate=1e-4, weight_decay=1e-5, grad_clip=1.0, backbone="resnet50",
                               pretrained=False, dropout=0.0, target_labels=labels, label_smoothing=0.1,
                               use_weighted_sampling=False)
    model.train()
    tr = ClassificationTrainer(cfg, model=model, train_dataset=_DS(), val_dataset=_DS())
    loss = tr._train_step({"image": img, "targets": DynamicTargets(dict(targets))})
    m = tr.accelerator.unwrap_model(tr.model)
    sd = m.state_dict()
    out = {"loss": np.array(loss)}
    meta = {"B": B, "res": R, "img": checksum(img), "loss": loss, "checksums": {}, "delta_checksums": {}}
    for k, v in sd.items():
        if not v.is_floating_point():
            meta["checksums"][k] = int(v)
            continue
        if k.startswith("heads.") or "layer4.2.bn3" in k or k == "backbone.bn1.running_mean":
            out["after_step/" + k] = fp(v)
        meta["checksums"][k] = checksum(v)
        meta["delta_checksums"][k] = checksum(v - before[k])
    np.savez_compressed(os.path.join(HERE, "classification_step_resnet50_128.npz"), **out)
    dump("classification_step_resnet50_128.json", meta)


class _LocDS(torch.utils.data.Dataset):
    """Reference LocalizationDataset item layout (training/datasets/localization.py:283-312) over
    oracle/weights.py images; records the order in which the loader asks for samples."""

    def __init__(self, n, seed, res=64):
        self.img, self.coords, self.mask = ow.localization_batch(n, res, res, seed=seed)
        self.log: list[int] = []

    def __len__(self):
        return self.img.shape[0]

    def __getitem__(self, i):
        self.log.append(int(i))
        return {"image": self.img[i], "coords": self.coords[i], "mask": self.mask[i], "series_type_idx": 0,
                "metadata": {"index": int(i)}}

    def get_stats(self):
        return {"n": len(self)}


def _schema(ck):
    def desc(v):
        if isinstance(v, torch.Tensor):
            return {"tensor": str(v.dtype).replace("torch.", ""), "shape": list(v.shape)}
        return type(v).__name__

    opt = ck["optimizer_state_dict"]
    return {
        "top_level_keys": sorted(ck.keys()),
        "model_state_dict": {k: desc(v) for k, v in ck["model_state_dict"].items()},
        "optimizer_param_groups_keys": sorted(opt["param_groups"][0].keys()),
        "optimizer_param_groups_params": opt["param_groups"][0]["params"][:5] + ["..."],
        "optimizer_state_count": len(opt["state"]),
        "optimizer_state_entry": {k: desc(v) for k, v in next(iter(opt["state"].values())).items()},
        "scheduler_state_keys": sorted(ck["scheduler_state_dict"].keys()) if ck["scheduler_state_dict"] else None,
        "history_keys": sorted(ck["history"].keys()),
        "config_field_types": {k: type(v).__name__ for k, v in ck["config"].items()},
        "types": {k: type(ck[k]).__name__ for k in ("epoch", "best_metric", "best_epoch")},
    }


def gold_trajectory(generic, freeze: bool):
    from spine_vision.training.trainers.localization import LocalizationConfig, LocalizationTrainer

    torch.manual_seed(1234)
    model = generic.CoordinateRegressor(backbone="convnext_base", pretrained=False, dropout=0.0,
                                        freeze_backbone=freeze)
    ow.fill_module(model)
    train_ds, val_ds = _LocDS(6, seed=42), _LocDS(3, seed=7)
    tmp = tempfile.mkdtemp()
    cfg = LocalizationConfig(output_path=tmp, batch_size=2, num_epochs=3, num_workers=0, pin_memory=False,
                             use_trackio=False, visualize_predictions=False, learning_rate=1e-3,
                             weight_decay=1e-5, grad_clip=1.0, backbone="convnext_base", pretrained=False,
                             dropout=0.0, early_stopping=False, save_frequency=100,
                             freeze_backbone_epochs=1 if freeze else 0, seed=42)
    tr = LocalizationTrainer(cfg, model=model, train_dataset=train_ds, val_dataset=val_ds)
    tr.on_train_end = lambda result: None  # plots only (seaborn is not installed here)
    # per-epoch train-set order and the LR / loss seen at each epoch's end (before the reload)
    orders, live = [], []
    orig_epoch = tr._train_epoch

    def _epoch():
        n0 = len(train_ds.log)
        loss = orig_epoch()
        orders.append(train_ds.log[n0:])
        return loss

    tr._train_epoch = _epoch
    orig_end = tr.on_epoch_end

    def _end(epoch, metrics):
        live.append({k: (float(v) if v is not None else None) for k, v in metrics.items()})
        return orig_end(epoch, metrics)

    tr.on_epoch_end = _end
    res = tr.train()
    m = tr.accelerator.unwrap_model(tr.model)
    params = dict(m.named_parameters())
    ck = torch.load(os.path.join(tmp, "best_model.pt"), map_location="cpu", weights_only=False)
    meta = {
        "generator": "tests/golden/make_golden_r2.py",
        "config": {"batch_size": 2, "num_epochs": 3, "learning_rate": 1e-3, "weight_decay": 1e-5, "grad_clip": 1.0,
                   "freeze_backbone_epochs": 1 if freeze else 0, "train_n": 6, "train_seed": 42, "val_n": 3,
                   "val_seed": 7, "res": 64, "dropout": 0.0},
        "train_order": orders,
        "epoch_end_metrics": live,
        "result": {"best_epoch": res.best_epoch, "best_metric": res.best_metric,
                   "final_train_loss": res.final_train_loss, "final_val_loss": res.final_val_loss,
                   "history": {k: [float(x) for x in v] for k, v in res.history.items()}},
        "scheduler_T_max": tr.scheduler.scheduler.T_max if hasattr(tr.scheduler, "scheduler") else None,
        "final_param_checksums": {k: checksum(params[k]) for k in PICKS_LOC},
        "final_small_params": {k: fp(params[k]).reshape(-1).tolist() for k in PICKS_LOC
                               if params[k].numel() <= 3000},
        "checkpoint_epoch": ck["epoch"],
        "optimizer_steps_in_checkpoint": sorted({int(float(s["step"])) for s in ck["optimizer_state_dict"]["state"].values()}),
        "optimizer_state_count": len(ck["optimizer_state_dict"]["state"]),
    }
    dump(f"trajectory_localization{'_freeze' if freeze else ''}.json", meta)
    return ck


def main():
    trainers, generic = import_reference()
    gold_focal()
    gold_metrics()
    gold_classification_step(generic)
    ck = gold_trajectory(generic, freeze=False)
    s = _schema(ck)
    s["generator"] = "tests/golden/make_golden_r2.py (best_model.pt of the trajectory_localization run)"
    dump("checkpoint_schema.json", s)
    gold_trajectory(generic, freeze=True)
    print("ok")


if __name__ == "__main__":
    main()
