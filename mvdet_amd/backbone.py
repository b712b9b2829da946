"""Backbones feeding the hot path (producer side, stock MIOpen convs).

The reference builds ``nn.Sequential(*list(resnet18(replace_stride_with_dilation=
[False, True, True]).children())[:-2])`` and splits it at index 7
(``persp_trans_detector.py:40-45``; its ResNet copy is
``multiview_detector/models/resnet.py:117-230``), or VGG-11 features with the
last and fourth-from-last layers blanked, split at 10 (``:32-39``).  Written
here from the architecture definitions so the ``state_dict`` keys match
(``base_pt1.0.weight`` … ``base_pt2.7.1.conv2.weight``); weights are random-init
(``pretrained=False`` in the reference; no network here).

Quirk reproduced from ``resnet.py:43-55,170-192``: with dilation enabled only a
block's ``conv1`` is dilated (``conv2`` keeps dilation 1), and the first block
of a dilated stage uses the *previous* stage's dilation.
"""
from __future__ import annotations

from typing import List, Tuple

import torch.nn as nn


def _conv3x3(cin: int, cout: int, stride: int = 1, dilation: int = 1) -> nn.Conv2d:
    return nn.Conv2d(cin, cout, 3, stride=stride, padding=dilation, dilation=dilation, bias=False)


class BasicBlock(nn.Module):
    def __init__(self, cin: int, cout: int, stride: int, dilation: int, downsample: bool):
        super().__init__()
        self.conv1 = _conv3x3(cin, cout, stride, dilation)
        self.bn1 = nn.BatchNorm2d(cout)
        self.relu = nn.ReLU(inplace=True)
        self.conv2 = _conv3x3(cout, cout)
        self.bn2 = nn.BatchNorm2d(cout)
        self.downsample = (nn.Sequential(nn.Conv2d(cin, cout, 1, stride=stride, bias=False), nn.BatchNorm2d(cout))
                           if downsample else None)

    def forward(self, x):
        identity = x if self.downsample is None else self.downsample(x)
        out = self.relu(self.bn1(self.conv1(x)))
        out = self.bn2(self.conv2(out))
        return self.relu(out + identity)


def resnet18_trunk(replace_stride_with_dilation=(False, True, True)) -> nn.Sequential:
    """ResNet-18 without avgpool/fc: children conv1, bn1, relu, maxpool, layer1-4."""
    mods: List[nn.Module] = [nn.Conv2d(3, 64, 7, stride=2, padding=3, bias=False), nn.BatchNorm2d(64),
                             nn.ReLU(inplace=True), nn.MaxPool2d(3, stride=2, padding=1)]
    cin, dilation = 64, 1
    for planes, stride, dilate in ((64, 1, False), (128, 2, replace_stride_with_dilation[0]),
                                   (256, 2, replace_stride_with_dilation[1]),
                                   (512, 2, replace_stride_with_dilation[2])):
        prev = dilation
        if dilate:
            dilation *= stride
            stride = 1
        blocks = [BasicBlock(cin, planes, stride, prev, stride != 1 or cin != planes),
                  BasicBlock(planes, planes, 1, dilation, False)]
        cin = planes
        mods.append(nn.Sequential(*blocks))
    trunk = nn.Sequential(*mods)
    for m in trunk.modules():
        if isinstance(m, nn.Conv2d):
            nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
        elif isinstance(m, nn.BatchNorm2d):
            nn.init.constant_(m.weight, 1)
            nn.init.constant_(m.bias, 0)
    return trunk


def vgg11_features() -> nn.Sequential:
    """torchvision ``vgg11().features`` layout (indices 0..20)."""
    layers: List[nn.Module] = []
    cin = 3
    for v in (64, "M", 128, "M", 256, 256, "M", 512, 512, "M", 512, 512, "M"):
        if v == "M":
            layers.append(nn.MaxPool2d(2, 2))
        else:
            conv = nn.Conv2d(cin, v, 3, padding=1)
            nn.init.kaiming_normal_(conv.weight, mode="fan_out", nonlinearity="relu")
            nn.init.constant_(conv.bias, 0)
            layers += [conv, nn.ReLU(inplace=True)]
            cin = v
    return nn.Sequential(*layers)


def build_backbone(arch: str) -> Tuple[nn.Sequential, nn.Sequential, int]:
    """(base_pt1, base_pt2, out_channel) as ``persp_trans_detector.py:32-47``."""
    if arch == "vgg11":
        base = vgg11_features()
        base[-1] = nn.Sequential()
        base[-4] = nn.Sequential()
        split = 10
    elif arch == "resnet18":
        base = resnet18_trunk((False, True, True))
        split = 7
    else:
        raise Exception("architecture currently support [vgg11, resnet18]")
    return base[:split], base[split:], 512
