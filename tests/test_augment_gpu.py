"""GPU: sv_augment_u8 (csrc/augment.hip) against Pillow -- the library torchvision calls for the
reference's RandomHorizontalFlip / RandomAffine / ColorJitter on PIL images -- bit for bit, on
grayscale planes and RGB crops, over random torchvision-drawn parameters (plus the diagonal-matrix
Pillow path and both colour-jitter orders); and the device-transform training step equal to the
host-transform one when both draw the same parameters."""

import numpy as np
import pytest
import torch
from PIL import Image

from spine_vision_amd import kernels as K
from spine_vision_amd.training.datasets.augment import apply_pil, inverse_affine_matrix, sample_params

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("C,H,W,B", [(1, 64, 48, 16), (3, 40, 56, 16), (1, 512, 512, 4), (3, 256, 256, 4)])
def test_augment_kernel_matches_pillow(dev, C, H, W, B):
    rng = np.random.default_rng(C * 1000 + H)
    torch.manual_seed(H + W)
    arr = rng.integers(0, 256, (B, H, W) if C == 1 else (B, H, W, C), dtype=np.uint8)
    params = torch.stack([sample_params(H, W, flip=C == 1) for _ in range(B)])
    params[0, 1:7] = torch.tensor(inverse_affine_matrix([W * 0.5, H * 0.5], 0.0, (2, -1), 1.04), dtype=torch.float64)
    params[1, 7] = 1.19  # brightness > 1 (clipping branch)
    params[2, 9], params[3, 9] = 0.0, 1.0  # both colour orders
    got = K.augment_u8(torch.from_numpy(arr).to(dev), params.to(dev)).cpu().numpy()
    mode = "L" if C == 1 else "RGB"
    for b in range(B):
        ref = np.asarray(apply_pil(Image.fromarray(arr[b], mode), params[b]))
        assert np.array_equal(got[b], ref), (b, int((got[b] != ref).sum()))


@pytest.mark.parametrize("precision", ["fp32", "bf16"])
def test_device_augmented_step_matches_host_augmented_step(dev, precision):
    """Localization, augment on: the uint8 batch augmented + normalised on the GPU trains exactly like
    the PIL-augmented, host-normalised batch with the same torchvision draws."""
    from oracle import weights as ow
    from spine_vision_amd.training import CoordinateRegressor, StepEngine
    from spine_vision_amd.training.datasets import LocalizationCollator, SyntheticLocalizationDataset

    col = LocalizationCollator()
    torch.manual_seed(21)
    b_dev = col([SyntheticLocalizationDataset(4, (64, 64), seed=3, device_transform=True, augment=True)[i]
                 for i in range(4)])
    torch.manual_seed(21)
    b_host = col([SyntheticLocalizationDataset(4, (64, 64), seed=3, augment=True)[i] for i in range(4)])
    img_dev = K.augment_u8(b_dev["image"].to(dev), b_dev["augment"].to(dev))
    assert torch.equal(K.normalize_u8_gray(img_dev).cpu(), b_host["image"])
    out = []
    for image in (img_dev, b_host["image"].to(dev)):
        m = CoordinateRegressor("convnext_base", pretrained=False, dropout=0.0, precision=precision)
        ow.fill_module(m)
        m = m.to(dev).train()
        eng = StepEngine(m, dev, lr=1e-4, weight_decay=1e-5, grad_clip=1.0)
        loss = eng.step_localization(image, b_host["coords"].to(dev), b_host["mask"].to(dev))
        out.append((float(loss), m.backbone.stem[0].weight.detach().cpu()))
    assert out[0][0] == out[1][0] and torch.equal(out[0][1], out[1][1])


def test_classification_trainer_device_augment(dev, tmp_path):
    """ClassificationTrainer with device_transform + augment: uint8 crops and their parameters
    travel, the trainer augments on the GPU, the step trains."""
    from spine_vision_amd.training import ClassificationConfig, ClassificationTrainer
    from spine_vision_amd.training.datasets import SyntheticClassificationDataset

    labels = ["pfirrmann", "modic", "herniation"]
    cfg = ClassificationConfig(output_path=tmp_path, batch_size=4, num_epochs=1, num_workers=0, pin_memory=False,
                               target_labels=labels, output_size=(64, 64), pretrained=False, backbone="resnet18",
                               device_transform=True)
    tr = ClassificationTrainer(cfg, train_dataset=SyntheticClassificationDataset(8, (64, 64), seed=1,
                                                                               target_labels=labels, augment=True),
                               val_dataset=SyntheticClassificationDataset(4, (64, 64), seed=2, target_labels=labels))
    batch = next(iter(tr.train_loader))
    assert batch["image"].dtype == torch.uint8 and batch["augment"].shape == (4, 10)
    res = tr.train()
    assert res.final_train_loss == res.final_train_loss
