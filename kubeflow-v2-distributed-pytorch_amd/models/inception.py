"""GoogLeNet and Inception-v3 (torchvision layouts, auxiliary heads included) on mipipe's kernels.

Both are ``--arch`` choices of the reference through its torchvision registry scan
(task.py:50-52).  In training mode they return torchvision's ``GoogLeNetOutputs`` /
``InceptionOutputs`` named tuples; mipipe's ``CrossEntropyLoss`` (train/task.py) adds the
auxiliary losses — the reference would hand the tuple to ``nn.CrossEntropyLoss`` and crash.

Every BasicConv2d is conv -> BN(eps 1e-3) -> ReLU: square convs run on the MFMA implicit-GEMM
kernel with BN statistics in the epilogue, Inception-v3's 1x7 / 7x1 / 1x3 / 3x1 convs on the
direct kernel of ``vision.hip``; pools on the NHWC pool kernels.  Each Inception block's data
flow is written once (``_branches``) and executed either with plain torch ops on NCHW
(``forward``, the reference) or with mipipe's kernels on NHWC (``run``).
"""
from __future__ import annotations

from collections import namedtuple
from typing import Optional

import torch
import torch.nn as tnn
import torch.nn.functional as F

from mipipe import nn as mnn
from mipipe.ops import functional as MF

from . import register_model
from ._zoo import ZooModel, adaptive_avg_pool, conv_bn, global_pool, ref_linear, run_module

__all__ = ["GoogLeNet", "Inception3", "GoogLeNetOutputs", "InceptionOutputs", "googlenet",
           "inception_v3"]

GoogLeNetOutputs = namedtuple("GoogLeNetOutputs", ["logits", "aux_logits2", "aux_logits1"])
InceptionOutputs = namedtuple("InceptionOutputs", ["logits", "aux_logits"])


class _TorchOps:
    """Plain-torch NCHW execution of a block's data flow (the numerics oracle)."""
    cat_dim = 1

    @staticmethod
    def mod(m, x):
        return m(x)

    @staticmethod
    def avg(x, k, s, p=0):
        return F.avg_pool2d(x, k, s, p)

    @staticmethod
    def max(x, k, s, p=0):
        return F.max_pool2d(x, k, s, p)


class _MipipeOps:
    """NHWC execution on mipipe's kernels."""
    cat_dim = -1

    def __init__(self, ex):
        self.ex = ex

    def mod(self, m, x):
        return run_module(m, x, self.ex)

    @staticmethod
    def avg(x, k, s, p=0):
        return MF.avg_pool2d(x, k, s, p)

    @staticmethod
    def max(x, k, s, p=0):
        return MF.max_pool2d(x, k, s, p)


class _Block(tnn.Module):
    def forward(self, x):
        return torch.cat(self._branches(x, _TorchOps), 1)

    def run(self, x, ex):
        return torch.cat(self._branches(x, _MipipeOps(ex)), -1)


class BasicConv2d(tnn.Module):
    def __init__(self, in_channels: int, out_channels: int, **kwargs):
        super().__init__()
        self.conv = mnn.XConv2d(in_channels, out_channels, bias=False, **kwargs)
        self.bn = tnn.BatchNorm2d(out_channels, eps=0.001)

    def forward(self, x):
        return F.relu(self.bn(self.conv(x)), inplace=True)

    def run(self, x, ex):
        return conv_bn(x, self.conv, self.bn, "relu")


def _trunc_normal_init(module: tnn.Module, default_std: float) -> None:
    """torchvision's init: truncated normal (±2σ) weights for Conv2d / Linear (σ from a
    ``stddev`` attribute on the layer itself, else ``default_std``), BN weight 1 / bias 0."""
    for m in module.modules():
        if isinstance(m, (tnn.Conv2d, tnn.Linear)):
            std = float(getattr(m, "stddev", default_std))
            with torch.no_grad():
                tnn.init.trunc_normal_(m.weight, 0.0, std, -2 * std, 2 * std)
        elif isinstance(m, tnn.BatchNorm2d):
            tnn.init.constant_(m.weight, 1)
            tnn.init.constant_(m.bias, 0)


def _transform_input(x: torch.Tensor, enabled: bool) -> torch.Tensor:
    if not enabled:
        return x
    x0 = x[:, 0:1] * (0.229 / 0.5) + (0.485 - 0.5) / 0.5
    x1 = x[:, 1:2] * (0.224 / 0.5) + (0.456 - 0.5) / 0.5
    x2 = x[:, 2:3] * (0.225 / 0.5) + (0.406 - 0.5) / 0.5
    return torch.cat((x0, x1, x2), 1)


# ----------------------------------------------------------------------------------- GoogLeNet
class Inception(_Block):
    def __init__(self, in_channels, ch1x1, ch3x3red, ch3x3, ch5x5red, ch5x5, pool_proj):
        super().__init__()
        self.branch1 = BasicConv2d(in_channels, ch1x1, kernel_size=1)
        self.branch2 = tnn.Sequential(BasicConv2d(in_channels, ch3x3red, kernel_size=1),
                                      BasicConv2d(ch3x3red, ch3x3, kernel_size=3, padding=1))
        # kernel_size=3 instead of 5: torchvision's historical layout, kept for state_dict parity
        self.branch3 = tnn.Sequential(BasicConv2d(in_channels, ch5x5red, kernel_size=1),
                                      BasicConv2d(ch5x5red, ch5x5, kernel_size=3, padding=1))
        self.branch4 = tnn.Sequential(
            tnn.MaxPool2d(kernel_size=3, stride=1, padding=1, ceil_mode=True),
            BasicConv2d(in_channels, pool_proj, kernel_size=1))

    def _branches(self, x, ops):
        return [ops.mod(b, x) for b in (self.branch1, self.branch2, self.branch3, self.branch4)]


class InceptionAux(tnn.Module):
    def __init__(self, in_channels: int, num_classes: int, dropout: float = 0.7):
        super().__init__()
        self.conv = BasicConv2d(in_channels, 128, kernel_size=1)
        self.fc1 = mnn.Linear(2048, 1024)
        self.fc2 = mnn.Linear(1024, num_classes)
        self.p = dropout

    def forward(self, x):
        x = torch.flatten(self.conv(F.adaptive_avg_pool2d(x, (4, 4))), 1)
        x = F.relu(ref_linear(self.fc1, x), inplace=True)
        x = F.dropout(x, self.p, training=self.training)
        return ref_linear(self.fc2, x)

    def run(self, x, ex):
        h = self.conv.run(adaptive_avg_pool(x, (4, 4)), ex)
        h = h.permute(0, 3, 1, 2).reshape(h.shape[0], -1)  # torchvision flatten order (C, H, W)
        h = self.fc1(h, act="relu")
        h = MF.dropout(h, self.p, ex.seed(), self.training)
        return self.fc2(h)


class GoogLeNet(ZooModel):
    def __init__(self, num_classes: int = 1000, aux_logits: bool = True,
                 transform_input: bool = False, init_weights: Optional[bool] = True,
                 dropout: float = 0.2, dropout_aux: float = 0.7,
                 compute_dtype: Optional[torch.dtype] = None, **_):
        super().__init__()
        self.aux_logits = aux_logits
        self.transform_input = transform_input
        self.conv1 = BasicConv2d(3, 64, kernel_size=7, stride=2, padding=3)
        self.maxpool1 = tnn.MaxPool2d(3, stride=2, ceil_mode=True)
        self.conv2 = BasicConv2d(64, 64, kernel_size=1)
        self.conv3 = BasicConv2d(64, 192, kernel_size=3, padding=1)
        self.maxpool2 = tnn.MaxPool2d(3, stride=2, ceil_mode=True)
        self.inception3a = Inception(192, 64, 96, 128, 16, 32, 32)
        self.inception3b = Inception(256, 128, 128, 192, 32, 96, 64)
        self.maxpool3 = tnn.MaxPool2d(3, stride=2, ceil_mode=True)
        self.inception4a = Inception(480, 192, 96, 208, 16, 48, 64)
        self.inception4b = Inception(512, 160, 112, 224, 24, 64, 64)
        self.inception4c = Inception(512, 128, 128, 256, 24, 64, 64)
        self.inception4d = Inception(512, 112, 144, 288, 32, 64, 64)
        self.inception4e = Inception(528, 256, 160, 320, 32, 128, 128)
        self.maxpool4 = tnn.MaxPool2d(2, stride=2, ceil_mode=True)
        self.inception5a = Inception(832, 256, 160, 320, 32, 128, 128)
        self.inception5b = Inception(832, 384, 192, 384, 48, 128, 128)
        if aux_logits:
            self.aux1 = InceptionAux(512, num_classes, dropout_aux)
            self.aux2 = InceptionAux(528, num_classes, dropout_aux)
        else:
            self.aux1 = None
            self.aux2 = None
        self.avgpool = tnn.AdaptiveAvgPool2d((1, 1))
        self.dropout = tnn.Dropout(dropout)
        self.fc = mnn.Linear(1024, num_classes)
        self.compute_dtype = compute_dtype
        if init_weights or init_weights is None:
            _trunc_normal_init(self, 0.01)

    def forward(self, x):
        return self.run_model(*self.begin(_transform_input(x, self.transform_input)))

    def _flow(self, x, ops, aux_fn, head):
        x = ops.mod(self.maxpool1, ops.mod(self.conv1, x))
        x = ops.mod(self.maxpool2, ops.mod(self.conv3, ops.mod(self.conv2, x)))
        x = ops.mod(self.maxpool3, ops.mod(self.inception3b, ops.mod(self.inception3a, x)))
        x = ops.mod(self.inception4a, x)
        use_aux = self.training and self.aux1 is not None
        aux1 = aux_fn(self.aux1, x) if use_aux else None
        for m in (self.inception4b, self.inception4c, self.inception4d):
            x = ops.mod(m, x)
        aux2 = aux_fn(self.aux2, x) if use_aux else None
        x = ops.mod(self.maxpool4, ops.mod(self.inception4e, x))
        x = ops.mod(self.inception5b, ops.mod(self.inception5a, x))
        x = head(x)
        if self.training and self.aux_logits:
            return GoogLeNetOutputs(x, aux2, aux1)
        return x

    def run_model(self, x, ex):
        ops = _MipipeOps(ex)
        return self._flow(x, ops, lambda a, h: a.run(h, ex),
                          lambda h: self.fc(run_module(self.dropout, global_pool(h), ex)))

    def reference_forward(self, x):
        x = _transform_input(x, self.transform_input)
        return self._flow(x, _TorchOps, lambda a, h: a(h),
                          lambda h: ref_linear(self.fc, self.dropout(torch.flatten(self.avgpool(h), 1))))


# -------------------------------------------------------------------------------- Inception-v3
class InceptionA(_Block):
    def __init__(self, in_channels: int, pool_features: int):
        super().__init__()
        self.branch1x1 = BasicConv2d(in_channels, 64, kernel_size=1)
        self.branch5x5_1 = BasicConv2d(in_channels, 48, kernel_size=1)
        self.branch5x5_2 = BasicConv2d(48, 64, kernel_size=5, padding=2)
        self.branch3x3dbl_1 = BasicConv2d(in_channels, 64, kernel_size=1)
        self.branch3x3dbl_2 = BasicConv2d(64, 96, kernel_size=3, padding=1)
        self.branch3x3dbl_3 = BasicConv2d(96, 96, kernel_size=3, padding=1)
        self.branch_pool = BasicConv2d(in_channels, pool_features, kernel_size=1)

    def _branches(self, x, ops):
        b1 = ops.mod(self.branch1x1, x)
        b5 = ops.mod(self.branch5x5_2, ops.mod(self.branch5x5_1, x))
        b3 = x
        for m in (self.branch3x3dbl_1, self.branch3x3dbl_2, self.branch3x3dbl_3):
            b3 = ops.mod(m, b3)
        bp = ops.mod(self.branch_pool, ops.avg(x, 3, 1, 1))
        return [b1, b5, b3, bp]


class InceptionB(_Block):
    def __init__(self, in_channels: int):
        super().__init__()
        self.branch3x3 = BasicConv2d(in_channels, 384, kernel_size=3, stride=2)
        self.branch3x3dbl_1 = BasicConv2d(in_channels, 64, kernel_size=1)
        self.branch3x3dbl_2 = BasicConv2d(64, 96, kernel_size=3, padding=1)
        self.branch3x3dbl_3 = BasicConv2d(96, 96, kernel_size=3, stride=2)

    def _branches(self, x, ops):
        b3 = ops.mod(self.branch3x3, x)
        bd = x
        for m in (self.branch3x3dbl_1, self.branch3x3dbl_2, self.branch3x3dbl_3):
            bd = ops.mod(m, bd)
        return [b3, bd, ops.max(x, 3, 2)]


class InceptionC(_Block):
    def __init__(self, in_channels: int, channels_7x7: int):
        super().__init__()
        c7 = channels_7x7
        self.branch1x1 = BasicConv2d(in_channels, 192, kernel_size=1)
        self.branch7x7_1 = BasicConv2d(in_channels, c7, kernel_size=1)
        self.branch7x7_2 = BasicConv2d(c7, c7, kernel_size=(1, 7), padding=(0, 3))
        self.branch7x7_3 = BasicConv2d(c7, 192, kernel_size=(7, 1), padding=(3, 0))
        self.branch7x7dbl_1 = BasicConv2d(in_channels, c7, kernel_size=1)
        self.branch7x7dbl_2 = BasicConv2d(c7, c7, kernel_size=(7, 1), padding=(3, 0))
        self.branch7x7dbl_3 = BasicConv2d(c7, c7, kernel_size=(1, 7), padding=(0, 3))
        self.branch7x7dbl_4 = BasicConv2d(c7, c7, kernel_size=(7, 1), padding=(3, 0))
        self.branch7x7dbl_5 = BasicConv2d(c7, 192, kernel_size=(1, 7), padding=(0, 3))
        self.branch_pool = BasicConv2d(in_channels, 192, kernel_size=1)

    def _branches(self, x, ops):
        b1 = ops.mod(self.branch1x1, x)
        b7 = x
        for m in (self.branch7x7_1, self.branch7x7_2, self.branch7x7_3):
            b7 = ops.mod(m, b7)
        bd = x
        for m in (self.branch7x7dbl_1, self.branch7x7dbl_2, self.branch7x7dbl_3,
                  self.branch7x7dbl_4, self.branch7x7dbl_5):
            bd = ops.mod(m, bd)
        bp = ops.mod(self.branch_pool, ops.avg(x, 3, 1, 1))
        return [b1, b7, bd, bp]


class InceptionD(_Block):
    def __init__(self, in_channels: int):
        super().__init__()
        self.branch3x3_1 = BasicConv2d(in_channels, 192, kernel_size=1)
        self.branch3x3_2 = BasicConv2d(192, 320, kernel_size=3, stride=2)
        self.branch7x7x3_1 = BasicConv2d(in_channels, 192, kernel_size=1)
        self.branch7x7x3_2 = BasicConv2d(192, 192, kernel_size=(1, 7), padding=(0, 3))
        self.branch7x7x3_3 = BasicConv2d(192, 192, kernel_size=(7, 1), padding=(3, 0))
        self.branch7x7x3_4 = BasicConv2d(192, 192, kernel_size=3, stride=2)

    def _branches(self, x, ops):
        b3 = ops.mod(self.branch3x3_2, ops.mod(self.branch3x3_1, x))
        b7 = x
        for m in (self.branch7x7x3_1, self.branch7x7x3_2, self.branch7x7x3_3, self.branch7x7x3_4):
            b7 = ops.mod(m, b7)
        return [b3, b7, ops.max(x, 3, 2)]


class InceptionE(_Block):
    def __init__(self, in_channels: int):
        super().__init__()
        self.branch1x1 = BasicConv2d(in_channels, 320, kernel_size=1)
        self.branch3x3_1 = BasicConv2d(in_channels, 384, kernel_size=1)
        self.branch3x3_2a = BasicConv2d(384, 384, kernel_size=(1, 3), padding=(0, 1))
        self.branch3x3_2b = BasicConv2d(384, 384, kernel_size=(3, 1), padding=(1, 0))
        self.branch3x3dbl_1 = BasicConv2d(in_channels, 448, kernel_size=1)
        self.branch3x3dbl_2 = BasicConv2d(448, 384, kernel_size=3, padding=1)
        self.branch3x3dbl_3a = BasicConv2d(384, 384, kernel_size=(1, 3), padding=(0, 1))
        self.branch3x3dbl_3b = BasicConv2d(384, 384, kernel_size=(3, 1), padding=(1, 0))
        self.branch_pool = BasicConv2d(in_channels, 192, kernel_size=1)

    def _branches(self, x, ops):
        b1 = ops.mod(self.branch1x1, x)
        b3 = ops.mod(self.branch3x3_1, x)
        bd = ops.mod(self.branch3x3dbl_2, ops.mod(self.branch3x3dbl_1, x))
        bp = ops.mod(self.branch_pool, ops.avg(x, 3, 1, 1))
        # torchvision concatenates (2a, 2b) and (3a, 3b) first; the flat order is identical
        return [b1, ops.mod(self.branch3x3_2a, b3), ops.mod(self.branch3x3_2b, b3),
                ops.mod(self.branch3x3dbl_3a, bd), ops.mod(self.branch3x3dbl_3b, bd), bp]


class InceptionAuxV3(tnn.Module):
    def __init__(self, in_channels: int, num_classes: int):
        super().__init__()
        self.conv0 = BasicConv2d(in_channels, 128, kernel_size=1)
        self.conv1 = BasicConv2d(128, 768, kernel_size=5)
        self.conv1.stddev = 0.01  # set on the block, so (as in torchvision) init ignores it
        self.fc = mnn.Linear(768, num_classes)
        self.fc.stddev = 0.001

    def forward(self, x):
        x = self.conv1(self.conv0(F.avg_pool2d(x, kernel_size=5, stride=3)))
        return ref_linear(self.fc, torch.flatten(F.adaptive_avg_pool2d(x, (1, 1)), 1))

    def run(self, x, ex):
        x = self.conv1.run(self.conv0.run(MF.avg_pool2d(x, 5, 3, 0), ex), ex)
        return self.fc(global_pool(x))


class Inception3(ZooModel):
    def __init__(self, num_classes: int = 1000, aux_logits: bool = True,
                 transform_input: bool = False, init_weights: Optional[bool] = True,
                 dropout: float = 0.5, compute_dtype: Optional[torch.dtype] = None, **_):
        super().__init__()
        self.aux_logits = aux_logits
        self.transform_input = transform_input
        self.Conv2d_1a_3x3 = BasicConv2d(3, 32, kernel_size=3, stride=2)
        self.Conv2d_2a_3x3 = BasicConv2d(32, 32, kernel_size=3)
        self.Conv2d_2b_3x3 = BasicConv2d(32, 64, kernel_size=3, padding=1)
        self.maxpool1 = tnn.MaxPool2d(kernel_size=3, stride=2)
        self.Conv2d_3b_1x1 = BasicConv2d(64, 80, kernel_size=1)
        self.Conv2d_4a_3x3 = BasicConv2d(80, 192, kernel_size=3)
        self.maxpool2 = tnn.MaxPool2d(kernel_size=3, stride=2)
        self.Mixed_5b = InceptionA(192, pool_features=32)
        self.Mixed_5c = InceptionA(256, pool_features=64)
        self.Mixed_5d = InceptionA(288, pool_features=64)
        self.Mixed_6a = InceptionB(288)
        self.Mixed_6b = InceptionC(768, channels_7x7=128)
        self.Mixed_6c = InceptionC(768, channels_7x7=160)
        self.Mixed_6d = InceptionC(768, channels_7x7=160)
        self.Mixed_6e = InceptionC(768, channels_7x7=192)
        self.AuxLogits = InceptionAuxV3(768, num_classes) if aux_logits else None
        self.Mixed_7a = InceptionD(768)
        self.Mixed_7b = InceptionE(1280)
        self.Mixed_7c = InceptionE(2048)
        self.avgpool = tnn.AdaptiveAvgPool2d((1, 1))
        self.dropout = tnn.Dropout(dropout)
        self.fc = mnn.Linear(2048, num_classes)
        self.compute_dtype = compute_dtype
        if init_weights or init_weights is None:
            _trunc_normal_init(self, 0.1)

    def forward(self, x):
        return self.run_model(*self.begin(_transform_input(x, self.transform_input)))

    def _stages(self):
        pre = (self.Conv2d_1a_3x3, self.Conv2d_2a_3x3, self.Conv2d_2b_3x3, self.maxpool1,
               self.Conv2d_3b_1x1, self.Conv2d_4a_3x3, self.maxpool2, self.Mixed_5b,
               self.Mixed_5c, self.Mixed_5d, self.Mixed_6a, self.Mixed_6b, self.Mixed_6c,
               self.Mixed_6d, self.Mixed_6e)
        return pre, (self.Mixed_7a, self.Mixed_7b, self.Mixed_7c)

    def _flow(self, x, ops, aux_fn, head):
        pre, post = self._stages()
        for m in pre:
            x = ops.mod(m, x)
        aux = aux_fn(self.AuxLogits, x) if self.AuxLogits is not None and self.training else None
        for m in post:
            x = ops.mod(m, x)
        x = head(x)
        if self.training and self.aux_logits:
            return InceptionOutputs(x, aux)
        return x

    def run_model(self, x, ex):
        return self._flow(x, _MipipeOps(ex), lambda a, h: a.run(h, ex),
                          lambda h: self.fc(run_module(self.dropout, global_pool(h), ex)))

    def reference_forward(self, x):
        x = _transform_input(x, self.transform_input)
        return self._flow(x, _TorchOps, lambda a, h: a(h),
                          lambda h: ref_linear(self.fc, torch.flatten(self.dropout(self.avgpool(h)), 1)))


def googlenet(**kw) -> GoogLeNet:
    kw.pop("pretrained", None)  # no network: pretrained weights cannot be fetched
    return GoogLeNet(**kw)


def inception_v3(**kw) -> Inception3:
    kw.pop("pretrained", None)
    return Inception3(**kw)


register_model("googlenet", googlenet)
register_model("inception_v3", inception_v3)
