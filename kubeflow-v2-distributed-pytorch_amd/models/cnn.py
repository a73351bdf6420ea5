"""Small CNN for the MNIST-shape correctness config (BASELINE.json config 1/2).

Same topology/keys as :class:`mipipe.models.reference.RefMnistCNN`: three conv-BN-ReLU
stages (28x28 -> 14x14 -> 7x7), global average pool, two Linear layers.
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.nn as tnn

from mipipe import nn as mnn
from mipipe.ops import kernels as K

__all__ = ["MnistCNN", "mnist_cnn"]


class _PaddedConv(mnn.Conv2d):
    CIN_PAD = 8

    def compute_weight(self, dtype):
        w = self.weight.detach().permute(0, 2, 3, 1)
        ci = w.shape[-1]
        if ci % self.CIN_PAD:
            w = torch.nn.functional.pad(w, (0, self.CIN_PAD - ci % self.CIN_PAD))
        return w.to(dtype).contiguous()


class MnistCNN(tnn.Module):
    def __init__(self, num_classes: int = 10, in_chans: int = 1,
                 compute_dtype: Optional[torch.dtype] = None):
        super().__init__()
        self.compute_dtype = compute_dtype
        self.conv1 = _PaddedConv(in_chans, 32, 3, padding=1)
        self.bn1 = mnn.BatchNorm2d(32)
        self.conv2 = mnn.Conv2d(32, 64, 3, stride=2, padding=1)
        self.bn2 = mnn.BatchNorm2d(64)
        self.conv3 = mnn.Conv2d(64, 128, 3, stride=2, padding=1)
        self.bn3 = mnn.BatchNorm2d(128)
        self.pool = mnn.AdaptiveAvgPool2d((1, 1))
        self.fc1 = mnn.Linear(128, 128)
        self.fc2 = mnn.Linear(128, num_classes)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        dt = self.compute_dtype or (torch.bfloat16 if x.is_cuda else torch.float32)
        x = K.nchw_to_nhwc(x, dt, _PaddedConv.CIN_PAD)
        x = mnn.conv_bn_act(x, self.conv1, self.bn1, relu=True)
        x = mnn.conv_bn_act(x, self.conv2, self.bn2, relu=True)
        x = mnn.conv_bn_act(x, self.conv3, self.bn3, relu=True)
        x = self.pool(x)
        x = self.fc1(x, act="relu")
        return self.fc2(x)


def mnist_cnn(**kw) -> MnistCNN:
    kw.pop("pretrained", None)
    return MnistCNN(**kw)
