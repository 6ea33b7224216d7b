"""GPU: the product trainer end to end -- LocalizationTrainer with the HIP ConvNeXt-base backbone,
flat fused AdamW, device-side clip; two epochs on synthetic 64x64 data, checkpoint round trip."""

import pytest
import torch

from spine_vision_amd.training import CoordinateRegressor, LocalizationConfig, LocalizationTrainer
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
