"""MobileNetV2 and MNASNet (torchvision layouts) on mipipe's NHWC kernels.

Both are ``--arch`` choices of the reference through its torchvision registry scan
(task.py:50-52, 63-67).  Depthwise 3x3 / 5x5 convolutions run on the 8-channel vector direct
kernels of ``vision.hip``, the 1x1 expansions / projections on the MFMA implicit-GEMM conv with
BatchNorm statistics in its epilogue; ReLU6 is fused into the BN apply pass and the
inverted-residual add into the projection's BN apply.  ``state_dict`` keys and shapes follow
torchvision (``features.1.conv.0.0.weight``, ``layers.8.0.layers.3.weight`` ...).
"""
from __future__ import annotations

from typing import List, Optional

import torch
import torch.nn as tnn
import torch.nn.functional as F

from mipipe import nn as mnn

from . import register_model
from ._zoo import ZooModel, conv_bn, global_pool, ref_linear, run_seq

__all__ = ["MobileNetV2", "MNASNet", "mobilenet_v2", "mnasnet0_5", "mnasnet0_75", "mnasnet1_0",
           "mnasnet1_3"]


def _make_divisible(v: float, divisor: int, min_value: Optional[int] = None) -> int:
    if min_value is None:
        min_value = divisor
    new_v = max(min_value, int(v + divisor / 2) // divisor * divisor)
    if new_v < 0.9 * v:  # never round down by more than 10 %
        new_v += divisor
    return new_v


class ConvBNReLU(tnn.Sequential):
    def __init__(self, in_planes: int, out_planes: int, kernel_size: int = 3, stride: int = 1,
                 groups: int = 1):
        padding = (kernel_size - 1) // 2
        super().__init__(
            mnn.XConv2d(in_planes, out_planes, kernel_size, stride, padding, groups=groups,
                        bias=False),
            tnn.BatchNorm2d(out_planes), tnn.ReLU6(inplace=True))


class InvertedResidual(tnn.Module):
    def __init__(self, inp: int, oup: int, stride: int, expand_ratio: int):
        super().__init__()
        if stride not in (1, 2):
            raise ValueError(f"stride must be 1 or 2, got {stride}")
        hidden_dim = int(round(inp * expand_ratio))
        self.use_res_connect = stride == 1 and inp == oup
        layers: List[tnn.Module] = []
        if expand_ratio != 1:
            layers.append(ConvBNReLU(inp, hidden_dim, kernel_size=1))
        layers.extend([
            ConvBNReLU(hidden_dim, hidden_dim, stride=stride, groups=hidden_dim),
            mnn.XConv2d(hidden_dim, oup, 1, 1, 0, bias=False),
            tnn.BatchNorm2d(oup),
        ])
        self.conv = tnn.Sequential(*layers)

    def forward(self, x):  # torchvision semantics: NCHW, plain torch
        return x + self.conv(x) if self.use_res_connect else self.conv(x)

    def run(self, x, ex):
        mods = list(self.conv)
        h = run_seq(mods[:-2], x, ex)
        return conv_bn(h, mods[-2], mods[-1], "none", residual=x if self.use_res_connect else None)


class MobileNetV2(ZooModel):
    def __init__(self, num_classes: int = 1000, width_mult: float = 1.0,
                 inverted_residual_setting=None, round_nearest: int = 8, dropout: float = 0.2,
                 compute_dtype: Optional[torch.dtype] = None, **_):
        super().__init__()
        input_channel, last_channel = 32, 1280
        if inverted_residual_setting is None:
            inverted_residual_setting = [
                # t, c, n, s
                [1, 16, 1, 1], [6, 24, 2, 2], [6, 32, 3, 2], [6, 64, 4, 2],
                [6, 96, 3, 1], [6, 160, 3, 2], [6, 320, 1, 1]]
        input_channel = _make_divisible(input_channel * width_mult, round_nearest)
        self.last_channel = _make_divisible(last_channel * max(1.0, width_mult), round_nearest)
        features: List[tnn.Module] = [ConvBNReLU(3, input_channel, stride=2)]
        for t, c, n, s in inverted_residual_setting:
            output_channel = _make_divisible(c * width_mult, round_nearest)
            for i in range(n):
                features.append(InvertedResidual(input_channel, output_channel,
                                                 s if i == 0 else 1, expand_ratio=t))
                input_channel = output_channel
        features.append(ConvBNReLU(input_channel, self.last_channel, kernel_size=1))
        self.features = tnn.Sequential(*features)
        self.classifier = tnn.Sequential(tnn.Dropout(dropout),
                                         mnn.Linear(self.last_channel, num_classes))
        self.compute_dtype = compute_dtype
        for m in self.modules():
            if isinstance(m, tnn.Conv2d):
                tnn.init.kaiming_normal_(m.weight, mode="fan_out")
                if m.bias is not None:
                    tnn.init.zeros_(m.bias)
            elif isinstance(m, tnn.BatchNorm2d):
                tnn.init.ones_(m.weight)
                tnn.init.zeros_(m.bias)
            elif isinstance(m, tnn.Linear):
                tnn.init.normal_(m.weight, 0, 0.01)
                tnn.init.zeros_(m.bias)

    def run_model(self, x, ex):
        x = run_seq(self.features, x, ex)
        return run_seq(self.classifier, global_pool(x), ex)

    def reference_forward(self, x):
        x = self.features(x)
        x = F.adaptive_avg_pool2d(x, (1, 1)).reshape(x.shape[0], -1)
        return ref_linear(self.classifier[1], self.classifier[0](x))


# ------------------------------------------------------------------------------------ MNASNet
_BN_MOMENTUM = 1 - 0.9997  # TensorFlow's batch-norm decay, as torchvision uses


class _MnasInvertedResidual(tnn.Module):
    def __init__(self, in_ch: int, out_ch: int, kernel_size: int, stride: int,
                 expansion_factor: int, bn_momentum: float = 0.1):
        super().__init__()
        if stride not in (1, 2) or kernel_size not in (3, 5):
            raise ValueError("MNASNet blocks use stride 1/2 and kernel 3/5")
        mid_ch = in_ch * expansion_factor
        self.apply_residual = in_ch == out_ch and stride == 1
        self.layers = tnn.Sequential(
            mnn.XConv2d(in_ch, mid_ch, 1, bias=False),
            tnn.BatchNorm2d(mid_ch, momentum=bn_momentum), tnn.ReLU(inplace=True),
            mnn.XConv2d(mid_ch, mid_ch, kernel_size, padding=kernel_size // 2, stride=stride,
                        groups=mid_ch, bias=False),
            tnn.BatchNorm2d(mid_ch, momentum=bn_momentum), tnn.ReLU(inplace=True),
            mnn.XConv2d(mid_ch, out_ch, 1, bias=False),
            tnn.BatchNorm2d(out_ch, momentum=bn_momentum))

    def forward(self, x):
        return self.layers(x) + x if self.apply_residual else self.layers(x)

    def run(self, x, ex):
        mods = list(self.layers)
        h = run_seq(mods[:-2], x, ex)
        return conv_bn(h, mods[-2], mods[-1], "none", residual=x if self.apply_residual else None)


def _stack(in_ch, out_ch, kernel_size, stride, exp_factor, repeats, bn_momentum):
    first = _MnasInvertedResidual(in_ch, out_ch, kernel_size, stride, exp_factor, bn_momentum)
    rest = [_MnasInvertedResidual(out_ch, out_ch, kernel_size, 1, exp_factor, bn_momentum)
            for _ in range(1, repeats)]
    return tnn.Sequential(first, *rest)


def _round_to_multiple_of(val: float, divisor: int, round_up_bias: float = 0.9) -> int:
    new_val = max(divisor, int(val + divisor / 2) // divisor * divisor)
    return new_val if new_val >= round_up_bias * val else new_val + divisor


def _get_depths(alpha: float) -> List[int]:
    return [_round_to_multiple_of(d * alpha, 8) for d in (32, 16, 24, 40, 80, 96, 192, 320)]


class MNASNet(ZooModel):
    def __init__(self, alpha: float, num_classes: int = 1000, dropout: float = 0.2,
                 compute_dtype: Optional[torch.dtype] = None, **_):
        super().__init__()
        if alpha <= 0.0:
            raise ValueError(f"alpha should be greater than 0.0 instead of {alpha}")
        self.alpha = alpha
        d = _get_depths(alpha)
        m = _BN_MOMENTUM
        self.layers = tnn.Sequential(
            # first layer: regular conv
            mnn.XConv2d(3, d[0], 3, padding=1, stride=2, bias=False),
            tnn.BatchNorm2d(d[0], momentum=m), tnn.ReLU(inplace=True),
            # depthwise separable, no skip
            mnn.XConv2d(d[0], d[0], 3, padding=1, stride=1, groups=d[0], bias=False),
            tnn.BatchNorm2d(d[0], momentum=m), tnn.ReLU(inplace=True),
            mnn.XConv2d(d[0], d[1], 1, padding=0, stride=1, bias=False),
            tnn.BatchNorm2d(d[1], momentum=m),
            # MNASNet blocks: stacks of inverted residuals
            _stack(d[1], d[2], 3, 2, 3, 3, m), _stack(d[2], d[3], 5, 2, 3, 3, m),
            _stack(d[3], d[4], 5, 2, 6, 3, m), _stack(d[4], d[5], 3, 1, 6, 2, m),
            _stack(d[5], d[6], 5, 2, 6, 4, m), _stack(d[6], d[7], 3, 1, 6, 1, m),
            # final mapping to classifier input
            mnn.XConv2d(d[7], 1280, 1, padding=0, stride=1, bias=False),
            tnn.BatchNorm2d(1280, momentum=m), tnn.ReLU(inplace=True))
        self.classifier = tnn.Sequential(tnn.Dropout(p=dropout, inplace=True),
                                         mnn.Linear(1280, num_classes))
        self.compute_dtype = compute_dtype
        for mod in self.modules():
            if isinstance(mod, tnn.Conv2d):
                tnn.init.kaiming_normal_(mod.weight, mode="fan_out", nonlinearity="relu")
                if mod.bias is not None:
                    tnn.init.zeros_(mod.bias)
            elif isinstance(mod, tnn.BatchNorm2d):
                tnn.init.ones_(mod.weight)
                tnn.init.zeros_(mod.bias)
            elif isinstance(mod, tnn.Linear):
                tnn.init.kaiming_uniform_(mod.weight, mode="fan_out", nonlinearity="sigmoid")
                tnn.init.zeros_(mod.bias)

    def run_model(self, x, ex):
        return run_seq(self.classifier, global_pool(run_seq(self.layers, x, ex)), ex)

    def reference_forward(self, x):
        x = self.layers(x).mean([2, 3])
        return ref_linear(self.classifier[1], self.classifier[0](x))


def mobilenet_v2(**kw) -> MobileNetV2:
    kw.pop("pretrained", None)  # no network: pretrained weights cannot be fetched
    return MobileNetV2(**kw)


def _mnasnet(alpha: float):
    def make(**kw) -> MNASNet:
        kw.pop("pretrained", None)
        return MNASNet(alpha, **kw)
    return make


mnasnet0_5, mnasnet0_75 = _mnasnet(0.5), _mnasnet(0.75)
mnasnet1_0, mnasnet1_3 = _mnasnet(1.0), _mnasnet(1.3)

register_model("mobilenet_v2", mobilenet_v2)
for _name, _fn in (("mnasnet0_5", mnasnet0_5), ("mnasnet0_75", mnasnet0_75),
                   ("mnasnet1_0", mnasnet1_0), ("mnasnet1_3", mnasnet1_3)):
    register_model(_name, _fn)
