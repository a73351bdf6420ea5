"""ShuffleNetV2 (torchvision layouts x0.5 / x1.0 / x1.5 / x2.0) on mipipe's NHWC kernels.

An ``--arch`` choice of the reference through its torchvision registry scan (task.py:50-52).
Branch channel counts are not multiples of 8 for x1.0 / x2.0 (58, 122 ...), so those layers run
on the any-channel direct conv and BatchNorm kernels of ``vision.hip``; x0.5 / x1.5 take the
vector depthwise and MFMA paths.  The split / concat / channel-shuffle of each unit is one
interleaving copy on NHWC data (``cat`` followed by ``channel_shuffle(., 2)`` interleaves the
two branches channel by channel).
"""
from __future__ import annotations

from typing import List, Optional

import torch
import torch.nn as tnn

from mipipe import nn as mnn

from . import register_model
from ._zoo import ZooModel, global_pool, ref_linear, run_module, run_seq

__all__ = ["ShuffleNetV2", "shufflenet_v2_x0_5", "shufflenet_v2_x1_0", "shufflenet_v2_x1_5",
           "shufflenet_v2_x2_0"]


def channel_shuffle(x: torch.Tensor, groups: int) -> torch.Tensor:
    b, c, h, w = x.size()
    x = x.view(b, groups, c // groups, h, w).transpose(1, 2).contiguous()
    return x.view(b, -1, h, w)


def cat_shuffle_nhwc(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """``channel_shuffle(cat((a, b), C), 2)`` on NHWC tensors in one copy: a0 b0 a1 b1 ..."""
    return torch.stack((a, b), dim=-1).reshape(*a.shape[:-1], a.shape[-1] * 2)


class InvertedResidual(tnn.Module):
    def __init__(self, inp: int, oup: int, stride: int):
        super().__init__()
        if not 1 <= stride <= 3:
            raise ValueError("illegal stride value")
        self.stride = stride
        bf = oup // 2
        if self.stride == 1 and inp != bf << 1:
            raise ValueError("stride-1 units need inp == oup")
        if self.stride > 1:
            self.branch1 = tnn.Sequential(
                self.depthwise_conv(inp, inp, kernel_size=3, stride=self.stride, padding=1),
                tnn.BatchNorm2d(inp),
                mnn.XConv2d(inp, bf, kernel_size=1, stride=1, padding=0, bias=False),
                tnn.BatchNorm2d(bf), tnn.ReLU(inplace=True))
        else:
            self.branch1 = tnn.Sequential()
        self.branch2 = tnn.Sequential(
            mnn.XConv2d(inp if self.stride > 1 else bf, bf, kernel_size=1, stride=1, padding=0,
                        bias=False),
            tnn.BatchNorm2d(bf), tnn.ReLU(inplace=True),
            self.depthwise_conv(bf, bf, kernel_size=3, stride=self.stride, padding=1),
            tnn.BatchNorm2d(bf),
            mnn.XConv2d(bf, bf, kernel_size=1, stride=1, padding=0, bias=False),
            tnn.BatchNorm2d(bf), tnn.ReLU(inplace=True))

    @staticmethod
    def depthwise_conv(i: int, o: int, kernel_size: int, stride: int = 1, padding: int = 0,
                       bias: bool = False) -> mnn.XConv2d:
        return mnn.XConv2d(i, o, kernel_size, stride, padding, bias=bias, groups=i)

    def forward(self, x):  # torchvision semantics: NCHW, plain torch
        if self.stride == 1:
            x1, x2 = x.chunk(2, dim=1)
            out = torch.cat((x1, self.branch2(x2)), dim=1)
        else:
            out = torch.cat((self.branch1(x), self.branch2(x)), dim=1)
        return channel_shuffle(out, 2)

    def run(self, x, ex):
        if self.stride == 1:
            c = x.shape[-1] // 2
            return cat_shuffle_nhwc(x[..., :c], run_seq(self.branch2, x[..., c:].contiguous(), ex))
        return cat_shuffle_nhwc(run_seq(self.branch1, x, ex), run_seq(self.branch2, x, ex))


class ShuffleNetV2(ZooModel):
    def __init__(self, stages_repeats: List[int], stages_out_channels: List[int],
                 num_classes: int = 1000, compute_dtype: Optional[torch.dtype] = None, **_):
        super().__init__()
        if len(stages_repeats) != 3 or len(stages_out_channels) != 5:
            raise ValueError("expected 3 stage repeats and 5 stage output channel counts")
        self._stage_out_channels = stages_out_channels
        input_channels = 3
        output_channels = self._stage_out_channels[0]
        self.conv1 = tnn.Sequential(
            mnn.XConv2d(input_channels, output_channels, 3, 2, 1, bias=False),
            tnn.BatchNorm2d(output_channels), tnn.ReLU(inplace=True))
        input_channels = output_channels
        self.maxpool = tnn.MaxPool2d(kernel_size=3, stride=2, padding=1)
        for name, repeats, output_channels in zip(("stage2", "stage3", "stage4"), stages_repeats,
                                                  self._stage_out_channels[1:]):
            seq = [InvertedResidual(input_channels, output_channels, 2)]
            seq += [InvertedResidual(output_channels, output_channels, 1)
                    for _ in range(repeats - 1)]
            setattr(self, name, tnn.Sequential(*seq))
            input_channels = output_channels
        output_channels = self._stage_out_channels[-1]
        self.conv5 = tnn.Sequential(
            mnn.XConv2d(input_channels, output_channels, 1, 1, 0, bias=False),
            tnn.BatchNorm2d(output_channels), tnn.ReLU(inplace=True))
        self.fc = mnn.Linear(output_channels, num_classes)
        self.compute_dtype = compute_dtype

    def _trunk(self):
        return (self.conv1, self.maxpool, self.stage2, self.stage3, self.stage4, self.conv5)

    def run_model(self, x, ex):
        for m in self._trunk():
            x = run_module(m, x, ex)
        return self.fc(global_pool(x))

    def reference_forward(self, x):
        for m in self._trunk():
            x = m(x)
        return ref_linear(self.fc, x.mean([2, 3]))


def _shufflenet(repeats, channels):
    def make(**kw) -> ShuffleNetV2:
        kw.pop("pretrained", None)
        return ShuffleNetV2(repeats, channels, **kw)
    return make


shufflenet_v2_x0_5 = _shufflenet([4, 8, 4], [24, 48, 96, 192, 1024])
shufflenet_v2_x1_0 = _shufflenet([4, 8, 4], [24, 116, 232, 464, 1024])
shufflenet_v2_x1_5 = _shufflenet([4, 8, 4], [24, 176, 352, 704, 1024])
shufflenet_v2_x2_0 = _shufflenet([4, 8, 4], [24, 244, 488, 976, 2048])

for _name, _fn in (("shufflenet_v2_x0_5", shufflenet_v2_x0_5),
                   ("shufflenet_v2_x1_0", shufflenet_v2_x1_0),
                   ("shufflenet_v2_x1_5", shufflenet_v2_x1_5),
                   ("shufflenet_v2_x2_0", shufflenet_v2_x2_0)):
    register_model(_name, _fn)
