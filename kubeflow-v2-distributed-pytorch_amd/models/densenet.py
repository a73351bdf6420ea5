"""DenseNet-121 / 161 / 169 / 201 (torchvision layouts) on mipipe's NHWC kernels.

An ``--arch`` choice of the reference through its torchvision registry scan (task.py:50-52).
Each dense layer is BN+ReLU (any-channel BN pass over the concatenated features) -> 1x1 conv on
the MFMA kernel with BN2's statistics in its epilogue -> BN2+ReLU in one pass -> 3x3 conv;
concatenation is along the contiguous NHWC channel axis.  ``state_dict`` keys follow torchvision
(``features.denseblock1.denselayer1.norm1.weight`` ...).
"""
from __future__ import annotations

from collections import OrderedDict
from typing import List, Optional, Tuple

import torch
import torch.nn as tnn
import torch.nn.functional as F

from mipipe import nn as mnn
from mipipe.ops import functional as MF

from . import register_model
from ._zoo import ZooModel, conv_bn, global_pool, ref_linear, run_seq

__all__ = ["DenseNet", "densenet121", "densenet161", "densenet169", "densenet201"]


class _DenseLayer(tnn.Module):
    def __init__(self, num_input_features: int, growth_rate: int, bn_size: int,
                 drop_rate: float, memory_efficient: bool = False):
        super().__init__()
        self.add_module("norm1", tnn.BatchNorm2d(num_input_features))
        self.add_module("relu1", tnn.ReLU(inplace=True))
        self.add_module("conv1", mnn.XConv2d(num_input_features, bn_size * growth_rate,
                                             kernel_size=1, stride=1, bias=False))
        self.add_module("norm2", tnn.BatchNorm2d(bn_size * growth_rate))
        self.add_module("relu2", tnn.ReLU(inplace=True))
        self.add_module("conv2", mnn.XConv2d(bn_size * growth_rate, growth_rate, kernel_size=3,
                                             stride=1, padding=1, bias=False))
        self.drop_rate = float(drop_rate)
        self.memory_efficient = memory_efficient  # accepted for API parity; no checkpointing

    def forward(self, inputs):  # torchvision semantics: NCHW, plain torch
        prev = [inputs] if isinstance(inputs, torch.Tensor) else inputs
        h = self.conv1(self.relu1(self.norm1(torch.cat(prev, 1))))
        new = self.conv2(self.relu2(self.norm2(h)))
        if self.drop_rate > 0:
            new = F.dropout(new, p=self.drop_rate, training=self.training)
        return new

    def run(self, feats: List[torch.Tensor], ex) -> torch.Tensor:
        x = feats[0] if len(feats) == 1 else torch.cat(feats, dim=-1)
        h = MF.bn_act(x, self.norm1, "relu")
        h = conv_bn(h, self.conv1, self.norm2, "relu")
        new = self.conv2.run(h)
        if self.drop_rate > 0:
            new = MF.dropout(new, self.drop_rate, ex.seed(), self.training)
        return new


class _DenseBlock(tnn.ModuleDict):
    _version = 2

    def __init__(self, num_layers: int, num_input_features: int, bn_size: int, growth_rate: int,
                 drop_rate: float, memory_efficient: bool = False):
        super().__init__()
        for i in range(num_layers):
            self.add_module("denselayer%d" % (i + 1),
                            _DenseLayer(num_input_features + i * growth_rate, growth_rate,
                                        bn_size, drop_rate, memory_efficient))

    def forward(self, init_features):
        features = [init_features]
        for _, layer in self.items():
            features.append(layer(features))
        return torch.cat(features, 1)

    def run(self, x, ex):
        feats = [x]
        for _, layer in self.items():
            feats.append(layer.run(feats, ex))
        return torch.cat(feats, dim=-1)


class _Transition(tnn.Sequential):
    def __init__(self, num_input_features: int, num_output_features: int):
        super().__init__()
        self.add_module("norm", tnn.BatchNorm2d(num_input_features))
        self.add_module("relu", tnn.ReLU(inplace=True))
        self.add_module("conv", mnn.XConv2d(num_input_features, num_output_features,
                                            kernel_size=1, stride=1, bias=False))
        self.add_module("pool", tnn.AvgPool2d(kernel_size=2, stride=2))


class DenseNet(ZooModel):
    def __init__(self, growth_rate: int = 32, block_config: Tuple[int, ...] = (6, 12, 24, 16),
                 num_init_features: int = 64, bn_size: int = 4, drop_rate: float = 0,
                 num_classes: int = 1000, memory_efficient: bool = False,
                 compute_dtype: Optional[torch.dtype] = None, **_):
        super().__init__()
        self.features = tnn.Sequential(OrderedDict([
            ("conv0", mnn.XConv2d(3, num_init_features, kernel_size=7, stride=2, padding=3,
                                  bias=False)),
            ("norm0", tnn.BatchNorm2d(num_init_features)),
            ("relu0", tnn.ReLU(inplace=True)),
            ("pool0", tnn.MaxPool2d(kernel_size=3, stride=2, padding=1)),
        ]))
        num_features = num_init_features
        for i, num_layers in enumerate(block_config):
            block = _DenseBlock(num_layers, num_features, bn_size, growth_rate, drop_rate,
                                memory_efficient)
            self.features.add_module("denseblock%d" % (i + 1), block)
            num_features = num_features + num_layers * growth_rate
            if i != len(block_config) - 1:
                self.features.add_module("transition%d" % (i + 1),
                                         _Transition(num_features, num_features // 2))
                num_features = num_features // 2
        self.features.add_module("norm5", tnn.BatchNorm2d(num_features))
        self.classifier = mnn.Linear(num_features, num_classes)
        self.compute_dtype = compute_dtype
        for m in self.modules():
            if isinstance(m, tnn.Conv2d):
                tnn.init.kaiming_normal_(m.weight)
            elif isinstance(m, tnn.BatchNorm2d):
                tnn.init.constant_(m.weight, 1)
                tnn.init.constant_(m.bias, 0)
            elif isinstance(m, tnn.Linear):
                tnn.init.constant_(m.bias, 0)

    def run_model(self, x, ex):
        mods = list(self.features)
        x = run_seq(mods[:-1], x, ex)
        x = MF.bn_act(x, mods[-1], "relu")  # norm5 + the functional ReLU after it
        return self.classifier(global_pool(x))

    def reference_forward(self, x):
        out = F.relu(self.features(x))
        return ref_linear(self.classifier, torch.flatten(F.adaptive_avg_pool2d(out, (1, 1)), 1))


def _densenet(growth_rate, block_config, num_init_features):
    def make(**kw) -> DenseNet:
        kw.pop("pretrained", None)
        return DenseNet(growth_rate, block_config, num_init_features, **kw)
    return make


densenet121 = _densenet(32, (6, 12, 24, 16), 64)
densenet161 = _densenet(48, (6, 12, 36, 24), 96)
densenet169 = _densenet(32, (6, 12, 32, 32), 64)
densenet201 = _densenet(32, (6, 12, 48, 32), 64)

for _name, _fn in (("densenet121", densenet121), ("densenet161", densenet161),
                   ("densenet169", densenet169), ("densenet201", densenet201)):
    register_model(_name, _fn)
