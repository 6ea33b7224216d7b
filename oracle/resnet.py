"""fp32 CPU restatement of timm 1.0.22 ResNet-18/50 with num_classes=0 (TEST INFRASTRUCTURE ONLY).

Follows spine_vision/training/models/backbone.py:27,29 (``resnet18.a1_in1k``, ``resnet50.a1_in1k``)
-> timm ``timm/models/resnet.py`` default ResNet (not vendored):
  conv1 7x7/2 (no bias) -> bn1 -> ReLU -> maxpool 3x3/2 pad 1 -> layer1..4 -> global avg pool
  BasicBlock  (resnet18, [2,2,2,2]): conv3x3(stride) bn relu conv3x3 bn (+downsample) relu
  Bottleneck  (resnet50, [3,4,6,3]): conv1x1 bn relu conv3x3(stride) bn relu conv1x1 bn (+ds) relu
  downsample: Conv2d 1x1 stride s (no bias) + BN when stride != 1 or channels change.
BatchNorm: eps 1e-5, momentum 0.1, train-mode batch statistics.  state_dict keys equal timm's.
"""

from __future__ import annotations

import torch.nn as nn

CFGS = {"resnet18": ("basic", (2, 2, 2, 2)), "resnet50": ("bottleneck", (3, 4, 6, 3))}


class BasicBlock(nn.Module):
    expansion = 1

    def __init__(self, inplanes, planes, stride=1, downsample=None):
        super().__init__()
        self.conv1 = nn.Conv2d(inplanes, planes, 3, stride=stride, padding=1, bias=False)
        self.bn1 = nn.BatchNorm2d(planes)
        self.act1 = nn.ReLU(inplace=True)
        self.conv2 = nn.Conv2d(planes, planes, 3, padding=1, bias=False)
        self.bn2 = nn.BatchNorm2d(planes)
        self.act2 = nn.ReLU(inplace=True)
        self.downsample = downsample

    def forward(self, x):
        sc = x if self.downsample is None else self.downsample(x)
        x = self.act1(self.bn1(self.conv1(x)))
        x = self.bn2(self.conv2(x))
        return self.act2(x + sc)


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, inplanes, planes, stride=1, downsample=None):
        super().__init__()
        self.conv1 = nn.Conv2d(inplanes, planes, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(planes)
        self.act1 = nn.ReLU(inplace=True)
        self.conv2 = nn.Conv2d(planes, planes, 3, stride=stride, padding=1, bias=False)
        self.bn2 = nn.BatchNorm2d(planes)
        self.act2 = nn.ReLU(inplace=True)
        self.conv3 = nn.Conv2d(planes, planes * 4, 1, bias=False)
        self.bn3 = nn.BatchNorm2d(planes * 4)
        self.act3 = nn.ReLU(inplace=True)
        self.downsample = downsample

    def forward(self, x):
        sc = x if self.downsample is None else self.downsample(x)
        x = self.act1(self.bn1(self.conv1(x)))
        x = self.act2(self.bn2(self.conv2(x)))
        x = self.bn3(self.conv3(x))
        return self.act3(x + sc)


class ResNet(nn.Module):
    def __init__(self, kind: str, layers) -> None:
        super().__init__()
        block = BasicBlock if kind == "basic" else Bottleneck
        self.conv1 = nn.Conv2d(3, 64, 7, stride=2, padding=3, bias=False)
        self.bn1 = nn.BatchNorm2d(64)
        self.act1 = nn.ReLU(inplace=True)
        self.maxpool = nn.MaxPool2d(3, stride=2, padding=1)
        inplanes = 64
        for i, (planes, n) in enumerate(zip((64, 128, 256, 512), layers)):
            stride = 1 if i == 0 else 2
            blocks = []
            for j in range(n):
                s = stride if j == 0 else 1
                ds = None
                if j == 0 and (s != 1 or inplanes != planes * block.expansion):
                    ds = nn.Sequential(nn.Conv2d(inplanes, planes * block.expansion, 1, stride=s, bias=False),
                                       nn.BatchNorm2d(planes * block.expansion))
                blocks.append(block(inplanes, planes, s, ds))
                inplanes = planes * block.expansion
            setattr(self, f"layer{i + 1}", nn.Sequential(*blocks))
        self.num_features = inplanes

    def forward(self, x):
        x = self.maxpool(self.act1(self.bn1(self.conv1(x))))
        x = self.layer4(self.layer3(self.layer2(self.layer1(x))))
        return x.mean((2, 3))


def create(name: str) -> ResNet:
    kind, layers = CFGS[name.split(".")[0]]
    return ResNet(kind, layers)
