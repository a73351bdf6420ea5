"""SqueezeNet 1.0 / 1.1 (torchvision layouts) on mipipe's NHWC kernels.

An ``--arch`` choice of the reference through its torchvision registry scan (task.py:50-52).
Every conv carries a bias and a ReLU, so each is ONE MFMA implicit-GEMM launch with bias + ReLU
in the epilogue (the classifier conv falls back to the direct kernel when the class count is
not a multiple of 8); max-pools use torch's ``ceil_mode`` output size.
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.nn as tnn

from mipipe import nn as mnn

from . import register_model
from ._zoo import ZooModel, run_seq

__all__ = ["SqueezeNet", "squeezenet1_0", "squeezenet1_1"]


class Fire(tnn.Module):
    def __init__(self, inplanes: int, squeeze_planes: int, expand1x1_planes: int,
                 expand3x3_planes: int):
        super().__init__()
        self.inplanes = inplanes
        self.squeeze = mnn.XConv2d(inplanes, squeeze_planes, kernel_size=1)
        self.squeeze_activation = tnn.ReLU(inplace=True)
        self.expand1x1 = mnn.XConv2d(squeeze_planes, expand1x1_planes, kernel_size=1)
        self.expand1x1_activation = tnn.ReLU(inplace=True)
        self.expand3x3 = mnn.XConv2d(squeeze_planes, expand3x3_planes, kernel_size=3, padding=1)
        self.expand3x3_activation = tnn.ReLU(inplace=True)

    def forward(self, x):  # torchvision semantics: NCHW, plain torch
        x = self.squeeze_activation(self.squeeze(x))
        return torch.cat([self.expand1x1_activation(self.expand1x1(x)),
                          self.expand3x3_activation(self.expand3x3(x))], 1)

    def run(self, x, ex):
        s = self.squeeze.run(x, "relu")
        return torch.cat((self.expand1x1.run(s, "relu"), self.expand3x3.run(s, "relu")), dim=-1)


class SqueezeNet(ZooModel):
    def __init__(self, version: str = "1_0", num_classes: int = 1000, dropout: float = 0.5,
                 compute_dtype: Optional[torch.dtype] = None, **_):
        super().__init__()
        self.num_classes = num_classes
        if version == "1_0":
            self.features = tnn.Sequential(
                mnn.XConv2d(3, 96, kernel_size=7, stride=2), tnn.ReLU(inplace=True),
                tnn.MaxPool2d(kernel_size=3, stride=2, ceil_mode=True),
                Fire(96, 16, 64, 64), Fire(128, 16, 64, 64), Fire(128, 32, 128, 128),
                tnn.MaxPool2d(kernel_size=3, stride=2, ceil_mode=True),
                Fire(256, 32, 128, 128), Fire(256, 48, 192, 192), Fire(384, 48, 192, 192),
                Fire(384, 64, 256, 256),
                tnn.MaxPool2d(kernel_size=3, stride=2, ceil_mode=True),
                Fire(512, 64, 256, 256))
        elif version == "1_1":
            self.features = tnn.Sequential(
                mnn.XConv2d(3, 64, kernel_size=3, stride=2), tnn.ReLU(inplace=True),
                tnn.MaxPool2d(kernel_size=3, stride=2, ceil_mode=True),
                Fire(64, 16, 64, 64), Fire(128, 16, 64, 64),
                tnn.MaxPool2d(kernel_size=3, stride=2, ceil_mode=True),
                Fire(128, 32, 128, 128), Fire(256, 32, 128, 128),
                tnn.MaxPool2d(kernel_size=3, stride=2, ceil_mode=True),
                Fire(256, 48, 192, 192), Fire(384, 48, 192, 192), Fire(384, 64, 256, 256),
                Fire(512, 64, 256, 256))
        else:
            raise ValueError(f"Unsupported SqueezeNet version {version}: 1_0 or 1_1 expected")
        final_conv = mnn.XConv2d(512, self.num_classes, kernel_size=1)
        self.classifier = tnn.Sequential(tnn.Dropout(p=dropout), final_conv,
                                         tnn.ReLU(inplace=True), tnn.AdaptiveAvgPool2d((1, 1)))
        self.compute_dtype = compute_dtype
        for m in self.modules():
            if isinstance(m, tnn.Conv2d):
                if m is final_conv:
                    tnn.init.normal_(m.weight, mean=0.0, std=0.01)
                else:
                    tnn.init.kaiming_uniform_(m.weight)
                if m.bias is not None:
                    tnn.init.constant_(m.bias, 0)

    def run_model(self, x, ex):
        x = run_seq(self.classifier, run_seq(self.features, x, ex), ex)
        return x.reshape(x.shape[0], -1)

    def reference_forward(self, x):
        return torch.flatten(self.classifier(self.features(x)), 1)


def squeezenet1_0(**kw) -> SqueezeNet:
    kw.pop("pretrained", None)
    return SqueezeNet("1_0", **kw)


def squeezenet1_1(**kw) -> SqueezeNet:
    kw.pop("pretrained", None)
    return SqueezeNet("1_1", **kw)


register_model("squeezenet1_0", squeezenet1_0)
register_model("squeezenet1_1", squeezenet1_1)
