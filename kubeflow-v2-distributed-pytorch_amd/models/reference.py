"""Plain-PyTorch reference definitions of the model zoo.

These modules use only ``torch.nn`` layers and exist for two purposes:

1. numerics oracles: tests compare mipipe's fused HIP-kernel models against them
   parameter-for-parameter (same ``state_dict`` keys), and
2. the *stock PyTorch-ROCm comparator* that BASELINE.md asks for (torch DDP +
   MIOpen/hipBLASLt + RCCL on the same MI355X, same model/batch/dtype).

The layer structure and ``state_dict`` key names follow torchvision's ResNet, which
the reference instantiates through ``models.__dict__[arch]()`` (task.py:50-52,
task.py:166-171).  torchvision is not installed in this image, so the layouts are
written from the published architecture (He et al. 2015, ResNet v1.5 with the
stride on the 3x3 conv).
"""
from __future__ import annotations

from typing import List, Optional, Type, Union

import torch
import torch.nn as nn


def conv3x3(cin: int, cout: int, stride: int = 1) -> nn.Conv2d:
    return nn.Conv2d(cin, cout, 3, stride=stride, padding=1, bias=False)


def conv1x1(cin: int, cout: int, stride: int = 1) -> nn.Conv2d:
    return nn.Conv2d(cin, cout, 1, stride=stride, bias=False)


class RefBasicBlock(nn.Module):
    expansion = 1

    def __init__(self, inplanes: int, planes: int, stride: int = 1,
                 downsample: Optional[nn.Module] = None):
        super().__init__()
        self.conv1 = conv3x3(inplanes, planes, stride)
        self.bn1 = nn.BatchNorm2d(planes)
        self.relu = nn.ReLU(inplace=True)
        self.conv2 = conv3x3(planes, planes)
        self.bn2 = nn.BatchNorm2d(planes)
        self.downsample = downsample
        self.stride = stride

    def forward(self, x):
        identity = x
        out = self.relu(self.bn1(self.conv1(x)))
        out = self.bn2(self.conv2(out))
        if self.downsample is not None:
            identity = self.downsample(x)
        return self.relu(out + identity)


class RefBottleneck(nn.Module):
    expansion = 4

    def __init__(self, inplanes: int, planes: int, stride: int = 1,
                 downsample: Optional[nn.Module] = None):
        super().__init__()
        self.conv1 = conv1x1(inplanes, planes)
        self.bn1 = nn.BatchNorm2d(planes)
        self.conv2 = conv3x3(planes, planes, stride)
        self.bn2 = nn.BatchNorm2d(planes)
        self.conv3 = conv1x1(planes, planes * 4)
        self.bn3 = nn.BatchNorm2d(planes * 4)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = downsample
        self.stride = stride

    def forward(self, x):
        identity = x
        out = self.relu(self.bn1(self.conv1(x)))
        out = self.relu(self.bn2(self.conv2(out)))
        out = self.bn3(self.conv3(out))
        if self.downsample is not None:
            identity = self.downsample(x)
        return self.relu(out + identity)


class RefResNet(nn.Module):
    def __init__(self, block: Type[Union[RefBasicBlock, RefBottleneck]], layers: List[int],
                 num_classes: int = 1000, in_chans: int = 3):
        super().__init__()
        self.inplanes = 64
        self.conv1 = nn.Conv2d(in_chans, 64, 7, stride=2, padding=3, bias=False)
        self.bn1 = nn.BatchNorm2d(64)
        self.relu = nn.ReLU(inplace=True)
        self.maxpool = nn.MaxPool2d(3, stride=2, padding=1)
        self.layer1 = self._make_layer(block, 64, layers[0])
        self.layer2 = self._make_layer(block, 128, layers[1], stride=2)
        self.layer3 = self._make_layer(block, 256, layers[2], stride=2)
        self.layer4 = self._make_layer(block, 512, layers[3], stride=2)
        self.avgpool = nn.AdaptiveAvgPool2d((1, 1))
        self.fc = nn.Linear(512 * block.expansion, num_classes)
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, nn.BatchNorm2d):
                nn.init.ones_(m.weight)
                nn.init.zeros_(m.bias)

    def _make_layer(self, block, planes, blocks, stride=1):
        downsample = None
        if stride != 1 or self.inplanes != planes * block.expansion:
            downsample = nn.Sequential(conv1x1(self.inplanes, planes * block.expansion, stride),
                                       nn.BatchNorm2d(planes * block.expansion))
        layers = [block(self.inplanes, planes, stride, downsample)]
        self.inplanes = planes * block.expansion
        for _ in range(1, blocks):
            layers.append(block(self.inplanes, planes))
        return nn.Sequential(*layers)

    def forward(self, x):
        x = self.maxpool(self.relu(self.bn1(self.conv1(x))))
        x = self.layer4(self.layer3(self.layer2(self.layer1(x))))
        x = torch.flatten(self.avgpool(x), 1)
        return self.fc(x)


_RESNET_CFG = {
    "resnet18": (RefBasicBlock, [2, 2, 2, 2]),
    "resnet34": (RefBasicBlock, [3, 4, 6, 3]),
    "resnet50": (RefBottleneck, [3, 4, 6, 3]),
    "resnet101": (RefBottleneck, [3, 4, 23, 3]),
    "resnet152": (RefBottleneck, [3, 8, 36, 3]),
}


def ref_resnet(arch: str, num_classes: int = 1000, in_chans: int = 3) -> RefResNet:
    block, layers = _RESNET_CFG[arch]
    return RefResNet(block, layers, num_classes=num_classes, in_chans=in_chans)


class RefMnistCNN(nn.Module):
    """Small CNN for the MNIST-shape correctness config (BASELINE config 1)."""

    def __init__(self, num_classes: int = 10, in_chans: int = 1):
        super().__init__()
        self.conv1 = nn.Conv2d(in_chans, 32, 3, padding=1, bias=False)
        self.bn1 = nn.BatchNorm2d(32)
        self.conv2 = nn.Conv2d(32, 64, 3, stride=2, padding=1, bias=False)
        self.bn2 = nn.BatchNorm2d(64)
        self.conv3 = nn.Conv2d(64, 128, 3, stride=2, padding=1, bias=False)
        self.bn3 = nn.BatchNorm2d(128)
        self.fc1 = nn.Linear(128, 128)
        self.fc2 = nn.Linear(128, num_classes)

    def forward(self, x):
        x = torch.relu(self.bn1(self.conv1(x)))
        x = torch.relu(self.bn2(self.conv2(x)))
        x = torch.relu(self.bn3(self.conv3(x)))
        x = x.mean(dim=(2, 3))
        return self.fc2(torch.relu(self.fc1(x)))
