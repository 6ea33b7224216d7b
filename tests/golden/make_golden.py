"""Generate the golden fixtures that pin the CPU oracle (oracle/) to the reference itself.

Run in the build container (needs /root/reference, read-only; never needed on the GPU box):
    python tests/golden/make_golden.py

What it does
  1. Imports the reference's own Python (spine_vision, /root/reference) with shims for the modules
     absent here (loguru, tyro, torchmetrics, seaborn, timm, torchvision, iterstrat) and the
     circular-import workaround recorded in SURVEY.md §8(c).  ``timm.create_model`` is routed to the
     oracle's restatement of timm ConvNeXt / ResNet (timm is not installed), so the reference's
     CoordinateRegressor / Classifier wrap exactly the oracle backbone.
  2. Loads identical generated weights (oracle/weights.py) into the reference model and the oracle
     model and records, from the REFERENCE code path: forward outputs, masked loss, and one full
     ``LocalizationTrainer._train_step`` / ``ClassificationTrainer._train_step`` (accelerate on CPU =
     fp32, clip 1.0, AdamW) -- loss and post-step parameter checksums.
  3. Cross-checks the oracle backbones against HF transformers' independent ConvNext / ResNet
     implementations (key remap) and records the max deviation.
Outputs: tests/golden/*.npz (small) + golden_meta.json.  Inputs are not stored: they are regenerated
bit-identically by oracle/weights.py on any machine (a checksum of each input is stored to verify).
"""

from __future__ import annotations

import json
import os
import sys
import tempfile
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.path.insert(0, ROOT)

from oracle import convnext as oc  # noqa: E402
from oracle import heads as oh  # noqa: E402
from oracle import resnet as orn  # noqa: E402
from oracle import step as ostep  # noqa: E402
from oracle import weights as ow  # noqa: E402

torch.set_num_threads(8)


# ------------------------------------------------------------------------------------ shims
def _stub(name, **attrs):
    m = types.ModuleType(name)
    for k, v in attrs.items():
        setattr(m, k, v)
    sys.modules[name] = m
    return m


class _Meta(type):
    def __iter__(cls):
        return iter(())

    def __getattr__(cls, name):
        if name.startswith("__"):
            raise AttributeError(name)
        return _Anything


class _Anything(metaclass=_Meta):
    def __init__(self, *a, **k):
        pass

    def __call__(self, *a, **k):
        return self

    def __getattr__(self, name):
        return _Anything()


def _module_getattr(name):
    if name.startswith("__"):
        raise AttributeError(name)
    return _Anything


class _StubFinder:
    """Meta-path finder that materialises any submodule of a stubbed root package."""

    roots: set = set()

    def find_spec(self, fullname, path=None, target=None):
        import importlib.machinery

        if fullname.split(".")[0] in self.roots and fullname not in sys.modules:
            return importlib.machinery.ModuleSpec(fullname, self, is_package=True)
        return None

    def create_module(self, spec):
        m = types.ModuleType(spec.name)
        m.__path__ = []
        m.__getattr__ = _module_getattr
        return m

    def exec_module(self, module):
        pass


def install_shims():
    # third-party packages that probe optional deps with importlib.util.find_spec: import them
    # before the stubs exist so their availability caches see the real (absent) packages
    import accelerate  # noqa: F401
    import transformers  # noqa: F401
    from transformers import ConvNextModel, ResNetModel  # noqa: F401

    class _Logger:
        def __getattr__(self, name):
            return lambda *a, **k: None

    _stub("loguru", logger=_Logger())
    tyro = _stub("tyro", cli=lambda *a, **k: None)
    tyro.conf = _stub("tyro.conf", arg=lambda *a, **k: None, subcommand=lambda *a, **k: None,
                      Suppress=None, FlagConversionOff=None, OmitArgPrefixes=None)
    tm = _stub("torchmetrics")
    tm.__getattr__ = _module_getattr
    _stub("seaborn").__getattr__ = _module_getattr
    tv = _stub("torchvision")
    tv.transforms = _stub("torchvision.transforms")
    tv.transforms.__getattr__ = _module_getattr
    _StubFinder.roots |= {"cv2", "SimpleITK", "fitz", "paddleocr", "vietocr", "rapidfuzz", "unidecode", "openpyxl"}
    sys.meta_path.insert(0, _StubFinder())
    _stub("iterstrat")
    _stub("iterstrat.ml_stratifiers", MultilabelStratifiedShuffleSplit=_Anything)

    def create_model(name, pretrained=False, num_classes=0, **kw):
        assert not pretrained and num_classes == 0
        base = name.split(".")[0]
        return oc.create(base) if base.startswith("convnext") else orn.create(base)

    _stub("timm", create_model=create_model)


def import_reference():
    install_shims()
    sys.path.insert(0, REF)
    # circular import workaround: skip spine_vision/training/__init__.py
    pkg = types.ModuleType("spine_vision.training")
    pkg.__path__ = [os.path.join(REF, "spine_vision", "training")]
    import spine_vision  # noqa: F401

    sys.modules["spine_vision.training"] = pkg
    import spine_vision.training.trainers as trainers  # noqa: F401
    from spine_vision.training.models import generic

    return trainers, generic


def fp(t):
    return t.detach().cpu().float().numpy()


def checksum(t):
    t = t.detach().double()
    return [float(t.sum()), float((t * t).sum()), float(t.abs().max())]


# ---------------------------------------------------------------------------------- goldens
def gold_localization(trainers, generic, meta):
    from spine_vision.training.trainers.localization import LocalizationConfig, LocalizationTrainer

    B, R = 2, 64
    img, coords, mask = ow.localization_batch(B, R, R)
    meta["loc_inputs"] = {"img": checksum(img), "coords": checksum(coords), "mask": checksum(mask), "B": B, "res": R}
    ref_model = generic.CoordinateRegressor(backbone="convnext_base", pretrained=False, dropout=0.0)
    ow.fill_module(ref_model)
    ora = oh.CoordinateRegressor(oc.create("convnext_base"), 1024, dropout=0.0)
    ora.load_state_dict(ref_model.state_dict(), strict=False)
    ref_model.eval()
    ora.eval()
    with torch.no_grad():
        p_ref = ref_model(img)
        p_ora = ora(img)
        loss_ref = ref_model.get_loss(p_ref, coords, mask=mask)
        loss_ora = ora.get_loss(p_ora, coords, mask)
    meta["loc_forward_ref_vs_oracle_maxabs"] = float((p_ref - p_ora).abs().max())
    meta["loc_loss_ref_vs_oracle_abs"] = float((loss_ref - loss_ora).abs())
    out = {"pred": fp(p_ref), "loss": np.array(float(loss_ref))}

    # one reference training step (trainer API, CPU -> fp32, clip 1.0, AdamW(lr, wd))
    class _DS(torch.utils.data.Dataset):
        def __len__(self):
            return B

        def __getitem__(self, i):
            return {"image": img[i], "coords": coords[i], "mask": mask[i], "series_type_idx": 0, "metadata": {}}

    tmp = tempfile.mkdtemp()
    cfg = LocalizationConfig(output_path=tmp, batch_size=B, num_workers=0, pin_memory=False, mixed_precision=True,
                             use_trackio=False, visualize_predictions=False, learning_rate=1e-4,
                             weight_decay=1e-5, grad_clip=1.0, backbone="convnext_base", pretrained=False,
                             dropout=0.0)
    ref_model.train()
    tr = LocalizationTrainer(cfg, model=ref_model, train_dataset=_DS(), val_dataset=_DS())
    batch = {"image": img, "coords": coords, "mask": mask}
    step_loss = tr._train_step(batch)
    params = dict(tr.accelerator.unwrap_model(tr.model).named_parameters())
    out["step_loss"] = np.array(step_loss)
    picks = ["backbone.stem.0.weight", "backbone.stages.2.blocks.13.mlp.fc1.weight",
             "backbone.stages.3.blocks.2.gamma", "head.2.weight", "head.5.bias"]
    for k in picks:
        if params[k].numel() <= 300_000:  # keep the fixture small; big tensors pinned by checksum
            out["after_step/" + k] = fp(params[k])
    meta["loc_after_step_checksums"] = {k: checksum(params[k]) for k in picks}
    # the same step through the oracle restatement
    ora2 = oh.CoordinateRegressor(oc.create("convnext_base"), 1024, dropout=0.0)
    ow.fill_module(ora2)
    ora2.train()
    opt = ostep.make_optimizer(ora2)
    l2, _, _ = ostep.train_step_localization(ora2, opt, img, coords, mask)
    meta["loc_step_loss_ref_vs_oracle_abs"] = abs(l2 - step_loss)
    p2 = dict(ora2.named_parameters())
    meta["loc_step_param_ref_vs_oracle_maxabs"] = max(float((p2[k] - params[k]).detach().abs().max()) for k in picks)
    np.savez_compressed(os.path.join(HERE, "localization_convnext_base_64.npz"), **out)


def gold_classification(trainers, generic, meta, backbone="resnet50"):
    from spine_vision.core.tasks import get_task
    from spine_vision.training.trainers.classification import _create_tasks_for_training

    B, R = 4, 64
    img, targets = ow.classification_batch(B, R, R)
    meta[f"cls_inputs_{backbone}"] = {"img": checksum(img), "B": B, "res": R}
    tasks = _create_tasks_for_training(target_labels=["pfirrmann", "modic", "herniation"], label_smoothing=0.1)
    ref_model = generic.Classifier(backbone=backbone, tasks=tasks, pretrained=False, dropout=0.0)
    ow.fill_module(ref_model)
    nf = 2048 if backbone == "resnet50" else 512
    ora = oh.Classifier(orn.create(backbone), nf, dropout=0.0)
    ora.load_state_dict(ref_model.state_dict(), strict=False)
    ref_model.train()  # BN in train mode: batch statistics (what the training step uses)
    ora.train()
    with torch.no_grad():
        o_ref = ref_model(img)
        o_ora = ora(img)
        l_ref = ref_model.get_loss(o_ref, targets)
        l_ora = ora.get_loss(o_ora, targets)
    meta[f"cls_{backbone}_forward_ref_vs_oracle_maxabs"] = max(float((o_ref[k] - o_ora[k]).abs().max()) for k in o_ref)
    meta[f"cls_{backbone}_loss_ref_vs_oracle_abs"] = float((l_ref - l_ora).abs())
    out = {f"logits/{k}": fp(v) for k, v in o_ref.items()}
    out["loss"] = np.array(float(l_ref))
    for k in ("pfirrmann", "modic", "herniation"):
        assert get_task(k).name == k
    np.savez_compressed(os.path.join(HERE, f"classification_{backbone}_64.npz"), **out)


def hf_crosscheck(meta):
    """Oracle backbones vs HF transformers (independent implementations of the timm architectures)."""
    from transformers import ConvNextConfig, ConvNextModel, ResNetConfig, ResNetModel

    # ConvNeXt-base
    ora = ow.fill_module(oc.create("convnext_base")).eval()
    cfg = ConvNextConfig(depths=[3, 3, 27, 3], hidden_sizes=[128, 256, 512, 1024], layer_norm_eps=1e-6,
                         layer_scale_init_value=1e-6)
    hf = ConvNextModel(cfg).eval()
    sd = {}
    for k, v in ora.state_dict().items():
        k2 = k.replace("head.norm.", "layernorm.")
        k2 = k2.replace("stem.0.", "embeddings.patch_embeddings.").replace("stem.1.", "embeddings.layernorm.")
        k2 = k2.replace("stages.", "encoder.stages.").replace(".downsample.0.", ".downsampling_layer.0.")
        k2 = k2.replace(".downsample.1.", ".downsampling_layer.1.").replace(".blocks.", ".layers.")
        k2 = k2.replace(".conv_dw.", ".dwconv.").replace(".norm.", ".layernorm.").replace(".mlp.fc1.", ".pwconv1.")
        k2 = k2.replace(".mlp.fc2.", ".pwconv2.").replace(".gamma", ".layer_scale_parameter")
        sd[k2] = v
    missing, unexpected = hf.load_state_dict(sd, strict=False)
    assert not unexpected, unexpected
    assert not [m for m in missing if "num_batches" not in m], missing
    img, _, _ = ow.localization_batch(2, 64, 64)
    with torch.no_grad():
        a = ora(img)
        b = hf(img).pooler_output
    meta["hf_convnext_base_pooled_maxabs"] = float((a - b).abs().max())
    meta["hf_convnext_base_pooled_scale"] = float(a.abs().max())
    # ResNet-50
    orr = ow.fill_module(orn.create("resnet50")).train()
    rcfg = ResNetConfig(depths=[3, 4, 6, 3], hidden_sizes=[256, 512, 1024, 2048], layer_type="bottleneck",
                        downsample_in_first_stage=False)
    hr = ResNetModel(rcfg).train()
    hsd = {}
    for k, v in orr.state_dict().items():
        k2 = k.replace("conv1.", "embedder.embedder.convolution.", 1) if k.startswith("conv1.") else k
        k2 = k2.replace("bn1.", "embedder.embedder.normalization.", 1) if k.startswith("bn1.") else k2
        if k.startswith("layer"):
            li = int(k[5]) - 1
            rest = k.split(".", 1)[1]
            bi, rest = rest.split(".", 1)
            rest = rest.replace("conv1.", "layer.0.convolution.").replace("bn1.", "layer.0.normalization.")
            rest = rest.replace("conv2.", "layer.1.convolution.").replace("bn2.", "layer.1.normalization.")
            rest = rest.replace("conv3.", "layer.2.convolution.").replace("bn3.", "layer.2.normalization.")
            rest = rest.replace("downsample.0.", "shortcut.convolution.").replace("downsample.1.", "shortcut.normalization.")
            k2 = f"encoder.stages.{li}.layers.{bi}.{rest}"
        hsd[k2] = v
    missing, unexpected = hr.load_state_dict(hsd, strict=False)
    assert not unexpected, unexpected
    img2, _ = ow.classification_batch(4, 64, 64)
    with torch.no_grad():
        a = orr(img2)
        b = hr(img2).pooler_output.flatten(1)
    meta["hf_resnet50_pooled_maxabs"] = float((a - b).abs().max())
    meta["hf_resnet50_pooled_scale"] = float(a.abs().max())


def main():
    meta = {"generator": "tests/golden/make_golden.py", "weights": "oracle/weights.py seed 42"}
    trainers, generic = import_reference()
    gold_localization(trainers, generic, meta)
    gold_classification(trainers, generic, meta, "resnet50")
    gold_classification(trainers, generic, meta, "resnet18")
    hf_crosscheck(meta)
    with open(os.path.join(HERE, "golden_meta.json"), "w") as f:
        json.dump(meta, f, indent=1, sort_keys=True)
    print(json.dumps(meta, indent=1, sort_keys=True))


if __name__ == "__main__":
    main()
