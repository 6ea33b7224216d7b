"""Backbone constructor -- drop-in for ``BackboneFactory`` (spine_vision/training/models/backbone.py:
137-225), whose ``create`` calls ``timm.create_model(BACKBONES[name], pretrained, num_classes=0)``
(backbone.py:166-170) and returns ``(module, module.num_features)``.

Here ``create`` returns the MI355X-native module (HIP kernels, timm module tree and state_dict keys)
for the backbones on the north-star path -- ConvNeXt-base/large (localization) and ResNet-18/50
(classification).  Every other name of the reference registry is recognised (``list_backbones``
returns the reference's full list) but raises: those families are outside this build's scope.
``pretrained=True`` cannot download weights offline; pass ``pretrained=False`` or load a timm
state_dict with ``load_state_dict`` (keys match).
"""

from __future__ import annotations

import torch.nn as nn

# reference name -> timm model id (backbone.py:25-85), grouped by family
_FAMILIES: dict[str, dict[str, str]] = {
    "resnet": {
        "resnet18": "resnet18.a1_in1k", "resnet34": "resnet34.a1_in1k", "resnet50": "resnet50.a1_in1k",
        "resnet101": "resnet101.a1_in1k", "resnet152": "resnet152.a1_in1k", "resnet50_a2": "resnet50.a2_in1k",
        "resnet50_b": "resnet50.b1k_in1k", "resnet50_c": "resnet50.c1_in1k", "resnet50_d": "resnet50.d_in1k",
        "resnext50": "resnext50_32x4d.a1h_in1k", "resnext101": "resnext101_32x8d.fb_wsl_ig1b_ft_in1k",
        "wide_resnet50": "wide_resnet50_2.racm_in1k", "wide_resnet101": "wide_resnet101_2.tv2_in1k",
        "resnetrs50": "resnetrs50.tf_in1k", "resnetrs101": "resnetrs101.tf_in1k",
        "resnetrs152": "resnetrs152.tf_in1k",
    },
    "convnext": {
        f"convnext_{s}": f"convnext_{s}.fb_in22k_ft_in1k" for s in ("tiny", "small", "base", "large", "xlarge")
    },
    "convnextv2": {
        "convnextv2_tiny": "convnextv2_tiny.fcmae_ft_in22k_in1k", "convnextv2_small": "convnextv2_small.fcmae",
        "convnextv2_base": "convnextv2_base.fcmae_ft_in22k_in1k",
        "convnextv2_large": "convnextv2_large.fcmae_ft_in22k_in1k",
        "convnextv2_huge": "convnextv2_huge.fcmae_ft_in22k_in1k",
    },
    "vit": {
        "vit_tiny": "vit_tiny_patch16_224.augreg_in21k_ft_in1k", "vit_small": "vit_small_patch16_224.augreg_in21k_ft_in1k",
        "vit_base": "vit_base_patch16_224.augreg2_in21k_ft_in1k", "vit_large": "vit_large_patch16_224.augreg_in21k_ft_in1k",
        "deit_tiny": "deit3_small_patch16_224.fb_in22k_ft_in1k", "deit_small": "deit3_small_patch16_224.fb_in22k_ft_in1k",
        "deit_base": "deit3_base_patch16_224.fb_in22k_ft_in1k",
        "swin_tiny": "swin_tiny_patch4_window7_224.ms_in22k_ft_in1k",
        "swin_small": "swin_small_patch4_window7_224.ms_in22k_ft_in1k",
        "swin_base": "swin_base_patch4_window7_224.ms_in22k_ft_in1k",
    },
    "efficient": {
        **{f"efficientnet_b{i}": f"efficientnet_b{i}.ra_in1k" for i in range(5)},
        **{f"efficientnetv2_{s}": f"efficientnetv2_{s}.ra_in1k" for s in ("s", "m", "l")},
        "mobilenetv3_small": "mobilenetv3_small_100.lamb_in1k", "mobilenetv3_large": "mobilenetv3_large_100.ra_in1k",
    },
}
BACKBONES: dict[str, str] = {k: v for fam in _FAMILIES.values() for k, v in fam.items()}

# names built natively on MI355X (the north-star backbones)
NATIVE = ("convnext_base", "convnext_large", "resnet18", "resnet50")
_FEATURE_DIMS = {"convnext_base": 1024, "convnext_large": 1536, "resnet18": 512, "resnet50": 2048}


class BackboneFactory:
    _feature_dims: dict[str, int] = {}
    precision: str = "bf16"  # default compute precision of created backbones ("bf16" | "fp32")

    @classmethod
    def create(cls, name: str, pretrained: bool = True, precision: str | None = None) -> tuple[nn.Module, int]:
        if name not in BACKBONES:
            raise ValueError(f"Unknown backbone: {name}. Available: {', '.join(sorted(BACKBONES))}")
        if name not in NATIVE:
            raise ValueError(
                f"Backbone {name!r} is not on the MI355X training path (supported: {', '.join(NATIVE)})"
            )
        prec = precision or cls.precision
        if name.startswith("convnext"):
            from ...backbone.convnext import create_convnext

            model = create_convnext(name, precision=prec)
        else:
            from ...backbone.resnet import create_resnet

            model = create_resnet(name, precision=prec)
        if pretrained:
            import warnings

            warnings.warn(
                f"pretrained weights for {BACKBONES[name]} cannot be downloaded offline; using random init "
                "(load a timm state_dict with load_state_dict to use pretrained weights)",
                stacklevel=2,
            )
        cls._feature_dims[name] = model.num_features
        return model, model.num_features

    @classmethod
    def get_feature_dim(cls, name: str) -> int:
        if name in cls._feature_dims:
            return cls._feature_dims[name]
        if name in _FEATURE_DIMS:
            return _FEATURE_DIMS[name]
        return cls.create(name, pretrained=False)[1]

    @classmethod
    def list_backbones(cls, family: str | None = None) -> list[str]:
        names = sorted(BACKBONES)
        return names if family is None else [n for n in names if n.startswith(family.lower())]

    @classmethod
    def get_timm_name(cls, name: str) -> str:
        if name not in BACKBONES:
            raise ValueError(f"Unknown backbone: {name}")
        return BACKBONES[name]
