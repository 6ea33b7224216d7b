"""fp32 CPU restatement of timm 1.0.22 ConvNeXt with num_classes=0 (TEST INFRASTRUCTURE ONLY).

Follows the call at spine_vision/training/models/backbone.py:166-170
(``timm.create_model(BACKBONES[name], pretrained, num_classes=0)``; ids at backbone.py:50-51).
timm itself is not vendored in the reference; its published ConvNeXt structure is restated:

  stem      Conv2d(3, d0, 4, stride 4) -> LayerNorm2d(d0, eps 1e-6)
  stage i   downsample (i > 0): LayerNorm2d(d_{i-1}) -> Conv2d(d_{i-1}, d_i, 2, stride 2)
            blocks: x + gamma * fc2(GELU(fc1(LN(dwconv7x7(x)))))   (LN channels-last, eps 1e-6)
  head      global avg pool -> LayerNorm2d(d3) -> flatten (fc = Identity)      -> [B, d3]

The state_dict keys equal timm's, so one generated state dict feeds this module, the HIP backbone
and (after a key remap) HF transformers' ConvNextModel.
"""

from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

CFGS = {
    "convnext_tiny": ((3, 3, 9, 3), (96, 192, 384, 768)),
    "convnext_base": ((3, 3, 27, 3), (128, 256, 512, 1024)),
    "convnext_large": ((3, 3, 27, 3), (192, 384, 768, 1536)),
}


class LayerNorm2d(nn.LayerNorm):
    """LayerNorm over C of an NCHW tensor."""

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        x = x.permute(0, 2, 3, 1)
        x = F.layer_norm(x, self.normalized_shape, self.weight, self.bias, self.eps)
        return x.permute(0, 3, 1, 2)


class Mlp(nn.Module):
    def __init__(self, dim: int, hidden: int) -> None:
        super().__init__()
        self.fc1 = nn.Linear(dim, hidden)
        self.act = nn.GELU()
        self.fc2 = nn.Linear(hidden, dim)

    def forward(self, x):
        return self.fc2(self.act(self.fc1(x)))


class Block(nn.Module):
    def __init__(self, dim: int) -> None:
        super().__init__()
        self.conv_dw = nn.Conv2d(dim, dim, 7, padding=3, groups=dim)
        self.norm = nn.LayerNorm(dim, eps=1e-6)
        self.mlp = Mlp(dim, 4 * dim)
        self.gamma = nn.Parameter(1e-6 * torch.ones(dim))

    def forward(self, x):
        shortcut = x
        x = self.conv_dw(x)
        x = x.permute(0, 2, 3, 1)
        x = self.norm(x)
        x = self.mlp(x)
        x = x.permute(0, 3, 1, 2)
        x = x.mul(self.gamma.reshape(1, -1, 1, 1))
        return x + shortcut


class Stage(nn.Module):
    def __init__(self, cin: int, cout: int, depth: int, downsample: bool) -> None:
        super().__init__()
        self.downsample = (
            nn.Sequential(LayerNorm2d(cin, eps=1e-6), nn.Conv2d(cin, cout, 2, stride=2)) if downsample else nn.Identity()
        )
        self.blocks = nn.Sequential(*[Block(cout) for _ in range(depth)])

    def forward(self, x):
        return self.blocks(self.downsample(x))


class Head(nn.Module):
    def __init__(self, dim: int) -> None:
        super().__init__()
        self.norm = LayerNorm2d(dim, eps=1e-6)

    def forward(self, x):
        x = x.mean((2, 3), keepdim=True)
        return self.norm(x).flatten(1)


class ConvNeXt(nn.Module):
    def __init__(self, depths=(3, 3, 27, 3), dims=(128, 256, 512, 1024)) -> None:
        super().__init__()
        self.stem = nn.Sequential(nn.Conv2d(3, dims[0], 4, stride=4), LayerNorm2d(dims[0], eps=1e-6))
        stages, prev = [], dims[0]
        for i, (d, c) in enumerate(zip(depths, dims)):
            stages.append(Stage(prev, c, d, downsample=i > 0))
            prev = c
        self.stages = nn.Sequential(*stages)
        self.head = Head(prev)
        self.num_features = prev

    def forward_features(self, x):
        return self.stages(self.stem(x))

    def forward(self, x):
        return self.head(self.forward_features(x))


def create(name: str) -> ConvNeXt:
    depths, dims = CFGS[name.split(".")[0]]
    return ConvNeXt(depths, dims)
