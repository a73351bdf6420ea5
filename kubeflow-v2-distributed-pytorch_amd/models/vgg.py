"""VGG (11/13/16/19, with and without BatchNorm) and AlexNet on mipipe's fused kernels.

The reference's ``--arch`` choices are torchvision's model registry (task.py:50-52, 63-67) and
its DataParallel branch special-cases ``alexnet*`` / ``vgg*`` (task.py:201-205), so these two
families are part of the model zoo.  ``state_dict`` keys and layouts follow torchvision
(``features.<i>.*`` / ``classifier.<i>.*``), so checkpoints interchange.

Execution: NHWC bf16 activations; conv + bias + ReLU in one implicit-GEMM kernel (epilogue);
conv + BN + ReLU through the fused BN path; max-pool kernel; the classifier runs on the MFMA GEMM
with bias/ReLU epilogues and hash-keyed dropout.  The flatten keeps torchvision's NCHW order so
``classifier.0.weight`` matches.
"""
from __future__ import annotations

from typing import List, Optional, Union

import torch
import torch.nn as tnn
import torch.nn.functional as F

from mipipe import nn as mnn
from mipipe.ops import functional as MF
from mipipe.ops import kernels as K

from . import register_model

_CFGS = {
    "A": [64, "M", 128, "M", 256, 256, "M", 512, 512, "M", 512, 512, "M"],
    "B": [64, 64, "M", 128, 128, "M", 256, 256, "M", 512, 512, "M", 512, 512, "M"],
    "D": [64, 64, "M", 128, 128, "M", 256, 256, 256, "M", 512, 512, 512, "M", 512, 512, 512, "M"],
    "E": [64, 64, "M", 128, 128, "M", 256, 256, 256, 256, "M", 512, 512, 512, 512, "M",
          512, 512, 512, 512, "M"],
}

CIN_PAD = 8  # first conv: input channels zero-padded 3 -> 8 (16-byte operand rows)


class _PaddedConv(mnn.Conv2d):
    """torch.nn.Conv2d state; compute weight padded along Cin to a multiple of 8."""

    def compute_weight(self, dtype):
        w = self.weight.detach().permute(0, 2, 3, 1)
        ci = w.shape[-1]
        if ci % CIN_PAD:
            return F.pad(w, (0, CIN_PAD - ci % CIN_PAD)).to(dtype).contiguous()
        return super().compute_weight(dtype)


def _run_features(features: tnn.Sequential, x: torch.Tensor) -> torch.Tensor:
    """Walk a torchvision-indexed ``features`` Sequential, fusing Conv[+BN]+ReLU groups."""
    mods = list(features)
    i = 0
    while i < len(mods):
        m = mods[i]
        if isinstance(m, mnn.Conv2d):
            nxt = mods[i + 1] if i + 1 < len(mods) else None
            if isinstance(nxt, mnn.BatchNorm2d):
                relu = i + 2 < len(mods) and isinstance(mods[i + 2], tnn.ReLU)
                x = mnn.conv_bn_act(x, m, nxt, relu=relu)
                i += 3 if relu else 2
                continue
            relu = isinstance(nxt, tnn.ReLU)
            w_c = m.compute_weight(x.dtype)
            x = MF.conv2d_bias_act(x, m.weight, w_c, m.bias, m.stride[0], m.padding[0], relu)
            i += 2 if relu else 1
            continue
        if isinstance(m, tnn.MaxPool2d):
            k = m.kernel_size if isinstance(m.kernel_size, int) else m.kernel_size[0]
            st = m.stride if isinstance(m.stride, int) else m.stride[0]
            p = m.padding if isinstance(m.padding, int) else m.padding[0]
            x = MF.max_pool2d(x, k, st, p)
        elif isinstance(m, tnn.ReLU):
            x = torch.relu(x)
        else:
            raise TypeError(f"unsupported feature layer {type(m).__name__}")
        i += 1
    return x


def _adaptive_flatten(x: torch.Tensor, size) -> torch.Tensor:
    """NHWC -> adaptive average pool to ``size`` -> flatten in torchvision's (C, H, W) order."""
    N, H, W, C = x.shape
    if (H, W) != tuple(size):
        xc = x.permute(0, 3, 1, 2)
        xc = xc.float() if xc.dtype in (torch.bfloat16, torch.float16) else xc
        x = F.adaptive_avg_pool2d(xc, size).to(x.dtype)
        return x.reshape(N, -1)
    return x.permute(0, 3, 1, 2).reshape(N, -1)


class _Classifier(tnn.Sequential):
    """torchvision classifier (Dropout/Linear/ReLU ...) on the GEMM kernel."""

    def run(self, x: torch.Tensor, training: bool, seed: int) -> torch.Tensor:
        mods = list(self)
        i = 0
        while i < len(mods):
            m = mods[i]
            if isinstance(m, tnn.Dropout):
                x = MF.dropout(x, m.p, seed + i, training)
                i += 1
            elif isinstance(m, mnn.Linear):
                relu = i + 1 < len(mods) and isinstance(mods[i + 1], tnn.ReLU)
                x = m(x, act="relu" if relu else "none")
                i += 2 if relu else 1
            elif isinstance(m, tnn.ReLU):
                x = torch.relu(x)
                i += 1
            else:
                raise TypeError(f"unsupported classifier layer {type(m).__name__}")
        return x


class VGG(tnn.Module):
    def __init__(self, cfg: List[Union[int, str]], batch_norm: bool = False,
                 num_classes: int = 1000, dropout: float = 0.5, in_chans: int = 3,
                 compute_dtype: Optional[torch.dtype] = None, **_):
        super().__init__()
        layers: List[tnn.Module] = []
        c = in_chans
        first = True
        for v in cfg:
            if v == "M":
                layers.append(tnn.MaxPool2d(2, 2))
                continue
            conv_cls = _PaddedConv if first else mnn.Conv2d
            layers.append(conv_cls(c, v, 3, padding=1, bias=True))
            if batch_norm:
                layers.append(mnn.BatchNorm2d(v))
            layers.append(tnn.ReLU(inplace=True))
            c, first = v, False
        self.features = tnn.Sequential(*layers)
        self.avgpool = tnn.AdaptiveAvgPool2d((7, 7))
        self.classifier = _Classifier(
            mnn.Linear(512 * 7 * 7, 4096), tnn.ReLU(True), tnn.Dropout(dropout),
            mnn.Linear(4096, 4096), tnn.ReLU(True), tnn.Dropout(dropout),
            mnn.Linear(4096, num_classes))
        self.compute_dtype = compute_dtype
        self._step = 0
        for m in self.modules():  # torchvision VGG init
            if isinstance(m, mnn.Conv2d):
                tnn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
                if m.bias is not None:
                    tnn.init.zeros_(m.bias)
            elif isinstance(m, mnn.BatchNorm2d):
                tnn.init.ones_(m.weight)
                tnn.init.zeros_(m.bias)
            elif isinstance(m, mnn.Linear):
                tnn.init.normal_(m.weight, 0, 0.01)
                tnn.init.zeros_(m.bias)

    def activation_dtype(self, x):
        if self.compute_dtype is not None:
            return self.compute_dtype
        return torch.bfloat16 if x.is_cuda else torch.float32

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if self.training:
            self._step += 1
        x = K.nchw_to_nhwc(x, self.activation_dtype(x), CIN_PAD)
        x = _run_features(self.features, x)
        x = _adaptive_flatten(x, (7, 7))
        return self.classifier.run(x, self.training, self._step * 16)


class AlexNet(tnn.Module):
    """torchvision AlexNet (the 'one weird trick' variant torchvision ships)."""

    def __init__(self, num_classes: int = 1000, dropout: float = 0.5,
                 compute_dtype: Optional[torch.dtype] = None, **_):
        super().__init__()
        self.features = tnn.Sequential(
            _PaddedConv(3, 64, 11, stride=4, padding=2, bias=True), tnn.ReLU(True),
            tnn.MaxPool2d(3, 2),
            mnn.Conv2d(64, 192, 5, padding=2, bias=True), tnn.ReLU(True),
            tnn.MaxPool2d(3, 2),
            mnn.Conv2d(192, 384, 3, padding=1, bias=True), tnn.ReLU(True),
            mnn.Conv2d(384, 256, 3, padding=1, bias=True), tnn.ReLU(True),
            mnn.Conv2d(256, 256, 3, padding=1, bias=True), tnn.ReLU(True),
            tnn.MaxPool2d(3, 2))
        self.avgpool = tnn.AdaptiveAvgPool2d((6, 6))
        self.classifier = _Classifier(
            tnn.Dropout(dropout), mnn.Linear(256 * 6 * 6, 4096), tnn.ReLU(True),
            tnn.Dropout(dropout), mnn.Linear(4096, 4096), tnn.ReLU(True),
            mnn.Linear(4096, num_classes))
        self.compute_dtype = compute_dtype
        self._step = 0

    activation_dtype = VGG.activation_dtype

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if self.training:
            self._step += 1
        x = K.nchw_to_nhwc(x, self.activation_dtype(x), CIN_PAD)
        x = _run_features(self.features, x)
        x = _adaptive_flatten(x, (6, 6))
        return self.classifier.run(x, self.training, self._step * 16)


def _vgg(cfg, bn):
    def make(**kw):
        kw.pop("pretrained", None)
        return VGG(_CFGS[cfg], batch_norm=bn, **kw)
    return make


for _name, _cfg in (("vgg11", "A"), ("vgg13", "B"), ("vgg16", "D"), ("vgg19", "E")):
    register_model(_name, _vgg(_cfg, False))
    register_model(_name + "_bn", _vgg(_cfg, True))


def alexnet(**kw) -> AlexNet:
    kw.pop("pretrained", None)
    return AlexNet(**kw)


register_model("alexnet", alexnet)
