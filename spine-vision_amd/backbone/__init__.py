"""HIP-backed backbones with timm module trees and state_dict keys."""

from .convnext import CONVNEXT_CFGS, ConvNeXtHip, create_convnext

__all__ = ["CONVNEXT_CFGS", "ConvNeXtHip", "create_convnext"]
