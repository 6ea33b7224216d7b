"""HIP-backed backbones with timm module trees and state_dict keys."""

from .convnext import CONVNEXT_CFGS, ConvNeXtHip, create_convnext
from .resnet import RESNET_CFGS, ResNetHip, create_resnet

__all__ = ["CONVNEXT_CFGS", "ConvNeXtHip", "create_convnext", "RESNET_CFGS", "ResNetHip", "create_resnet"]
