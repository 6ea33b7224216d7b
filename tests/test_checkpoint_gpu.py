"""GPU, row f3 (checkpoint interchange): a checkpoint in the reference's own layout
(spine_vision/training/trainers/base.py:695-706 -- timm state_dict keys, torch.optim.AdamW state,
epoch / best_metric / best_epoch / history / config) loads into this build's LocalizationTrainer (HIP
ConvNeXt-base + FlatAdamW) through the same ``_load_checkpoint`` the reference has (base.py:721-736), and
the build's checkpoint loads back into the reference-structured model with strict=True.

The "reference" side is the CPU oracle (oracle/, pinned to the reference by tests/golden): same module
tree and key names as the timm model the reference builds, optimizer = torch.optim.AdamW exactly as
base.py:384-390 creates it."""

import pytest
import torch

pytestmark = pytest.mark.gpu


def _oracle_after_one_step():
    from oracle import convnext as oc
    from oracle import heads as oh
    from oracle import step as ostep
    from oracle import weights as ow

    ora = oh.CoordinateRegressor(oc.create("convnext_base"), 1024, dropout=0.0)
    ow.fill_module(ora)
    ora.train()
    opt = ostep.make_optimizer(ora)
    img, coords, mask = ow.localization_batch(2, 64, 64)
    ostep.train_step_localization(ora, opt, img, coords, mask)
    return ora, opt


def test_reference_checkpoint_roundtrip(dev, tmp_path):
    from oracle import heads as oh
    from oracle import convnext as oc
    from oracle import weights as ow
    from spine_vision_amd.training import LocalizationConfig, LocalizationTrainer
    from spine_vision_amd.training.datasets import SyntheticLocalizationDataset

    ora, opt = _oracle_after_one_step()
    ref_ck = {
        "epoch": 3,
        "model_state_dict": ora.state_dict(),
        "optimizer_state_dict": opt.state_dict(),
        "scheduler_state_dict": None,
        "best_metric": 0.125,
        "best_epoch": 2,
        "history": {"train_loss": [0.3, 0.2, 0.15, 0.1], "val_loss": [0.31, 0.21, 0.16, 0.12], "lr": [1e-4] * 4},
        "config": {"backbone": "convnext_base", "image_size": (64, 64), "learning_rate": 1e-4},
    }
    path = tmp_path / "best_model.pt"
    torch.save(ref_ck, path)

    cfg = LocalizationConfig(output_path=tmp_path / "run", batch_size=2, num_epochs=1, num_workers=0,
                             image_size=(64, 64), pretrained=False, precision="fp32", dropout=0.0)
    tr = LocalizationTrainer(cfg, train_dataset=SyntheticLocalizationDataset(4, (64, 64), seed=1),
                             val_dataset=SyntheticLocalizationDataset(2, (64, 64), seed=2))
    tr._load_checkpoint(path)
    assert tr.current_epoch == 4 and tr.best_metric == 0.125 and tr.best_epoch == 2
    assert tr.history["train_loss"] == ref_ck["history"]["train_loss"]
    # weights: bit-exact; Adam moments and step carried into the flat optimizer
    sd = tr.model.state_dict()
    for k, v in ora.state_dict().items():
        assert torch.equal(sd[k].cpu(), v), k
    st = tr.optimizer.state_dict()
    ref_state = opt.state_dict()["state"]
    for i, (name, p) in enumerate(ora.named_parameters()):
        assert torch.equal(st["state"][i]["exp_avg"].cpu(), ref_state[i]["exp_avg"]), name
        assert torch.equal(st["state"][i]["exp_avg_sq"].cpu(), ref_state[i]["exp_avg_sq"]), name
        assert float(st["state"][i]["step"]) == float(ref_state[i]["step"])
    # the resumed HIP model predicts what the reference model predicts (fp32 parity mode)
    img, _, _ = ow.localization_batch(2, 64, 64, seed=7)
    tr.model.eval()
    ora.eval()
    with torch.no_grad():
        p_hip = tr.model(img.to(dev)).cpu()
        p_ref = ora(img)
    assert float((p_hip - p_ref).norm() / p_ref.norm()) < 1e-4

    # and back: the build's checkpoint is a reference checkpoint
    tr.config.output_path.mkdir(parents=True, exist_ok=True)
    tr._save_checkpoint(is_best=True)
    ck = torch.load(tr.config.output_path / "best_model.pt", weights_only=False)  # our own file
    assert set(ck) == set(ref_ck)
    back = oh.CoordinateRegressor(oc.create("convnext_base"), 1024, dropout=0.0)
    missing, unexpected = back.load_state_dict(ck["model_state_dict"], strict=True)
    assert not missing and not unexpected
    topt = torch.optim.AdamW(back.parameters(), lr=1e-4, weight_decay=1e-5)
    topt.load_state_dict(ck["optimizer_state_dict"])
    for i, (name, _) in enumerate(back.named_parameters()):
        assert torch.equal(topt.state_dict()["state"][i]["exp_avg"], ref_state[i]["exp_avg"]), name
