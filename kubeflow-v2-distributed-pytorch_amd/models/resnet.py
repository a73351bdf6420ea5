"""ResNet family on mipipe's fused NHWC kernels, torchvision-compatible ``state_dict``.

The reference builds ``torchvision.models.__dict__[arch]()`` (task.py:166-171; default
``resnet18``, 1000-class head).  Parameter/buffer names and shapes here match torchvision's
(``conv1.weight``, ``bn1.running_mean``, ``layer2.0.downsample.0.weight``, ``fc.bias`` ...)
so checkpoints load either way.

Execution is fused per conv: ``conv -> BN -> [+identity | +BN(downsample conv)] -> ReLU`` is
one implicit-GEMM launch (BN statistics accumulated in its epilogue), a tiny finalize and one
elementwise pass; the downsample branch is normalised inside the residual pass.
"""
from __future__ import annotations

from typing import List, Optional, Type, Union

import torch
import torch.nn as tnn

from mipipe import nn as mnn
from mipipe.ops import kernels as K
from mipipe.ops import functional as MF

__all__ = ["ResNet", "BasicBlock", "Bottleneck", "resnet18", "resnet34", "resnet50",
           "resnet101", "resnet152", "wide_resnet50_2", "wide_resnet101_2", "resnext50_32x4d",
           "resnext101_32x8d"]


def _conv3x3(cin, cout, stride=1):
    return mnn.Conv2d(cin, cout, 3, stride=stride, padding=1, bias=False)


def _conv1x1(cin, cout, stride=1):
    return mnn.Conv2d(cin, cout, 1, stride=stride, padding=0, bias=False)


class BasicBlock(tnn.Module):
    expansion = 1

    def __init__(self, inplanes, planes, stride=1, downsample=None, base_width=64, groups=1):
        super().__init__()
        if groups != 1 or base_width != 64:
            raise ValueError("BasicBlock only supports groups=1 and base_width=64")
        self.conv1 = _conv3x3(inplanes, planes, stride)
        self.bn1 = mnn.BatchNorm2d(planes)
        self.relu = mnn.ReLU(inplace=True)
        self.conv2 = _conv3x3(planes, planes)
        self.bn2 = mnn.BatchNorm2d(planes)
        self.downsample = downsample
        self.stride = stride

    def forward(self, x):
        slot = MF.ResidualSlot()
        out = mnn.conv_bn_act(x, self.conv1, self.bn1, relu=True, res_take=slot, fuse_prev=True)
        if self.downsample is not None:
            ds_conv, ds_bn = self.downsample[0], self.downsample[1]
            return mnn.conv_bn_act(out, self.conv2, self.bn2, relu=True, fuse_prev=True,
                                   branch=(x, ds_conv, ds_bn), res_give=slot)
        return mnn.conv_bn_act(out, self.conv2, self.bn2, relu=True, residual=x, fuse_prev=True,
                               res_give=slot)


class Bottleneck(tnn.Module):
    expansion = 4

    def __init__(self, inplanes, planes, stride=1, downsample=None, base_width=64, groups=1):
        super().__init__()
        width = int(planes * (base_width / 64.0)) * groups
        self.conv1 = _conv1x1(inplanes, width)
        self.bn1 = mnn.BatchNorm2d(width)
        # ResNeXt: the grouped 3x3 runs on the direct grouped-conv kernel (vision.hip)
        self.conv2 = (_conv3x3(width, width, stride) if groups == 1 else
                      mnn.XConv2d(width, width, 3, stride=stride, padding=1, groups=groups,
                                  bias=False))
        self.bn2 = mnn.BatchNorm2d(width)
        self.conv3 = _conv1x1(width, planes * self.expansion)
        self.bn3 = mnn.BatchNorm2d(planes * self.expansion)
        self.relu = mnn.ReLU(inplace=True)
        self.downsample = downsample
        self.stride = stride

    def forward(self, x):
        # conv2 / conv3 are the only consumers of their inputs: BN1 / BN2 backward reductions
        # run in their dgrad epilogues; conv1's dgrad adds the identity/downsample gradient
        slot = MF.ResidualSlot()
        # fuse_prev on conv1: if x is the previous block's BN+residual+ReLU output, its BN
        # backward reductions run in conv1's dgrad epilogue once the identity gradient is added
        out = mnn.conv_bn_act(x, self.conv1, self.bn1, relu=True, res_take=slot, fuse_prev=True)
        if isinstance(self.conv2, mnn.XConv2d):  # grouped: direct kernel + any-C BN/ReLU pass
            out = MF.bn_act(self.conv2.run(out), self.bn2, "relu")
        else:
            # conv3 (dense 1x1) is the only consumer: BN2's apply + ReLU folds into it
            out = mnn.conv_bn_act(out, self.conv2, self.bn2, relu=True, fuse_prev=True,
                                  fold_next=True)
        if self.downsample is not None:
            ds_conv, ds_bn = self.downsample[0], self.downsample[1]
            return mnn.conv_bn_act(out, self.conv3, self.bn3, relu=True, fuse_prev=True,
                                   branch=(x, ds_conv, ds_bn), res_give=slot)
        return mnn.conv_bn_act(out, self.conv3, self.bn3, relu=True, residual=x, fuse_prev=True,
                               res_give=slot)


class _StemConv(mnn.Conv2d):
    """7x7/2, pad 3 stem on 3-channel images, run as a "super-pixel" convolution: the image is
    packed (``stem_pack``) into 8-channel super-pixels of 2 horizontally adjacent padded pixels x
    4 channels, and the filter into [Co, 7, 4, 8]; the conv then has vertical stride 2,
    horizontal stride 1 and no padding, with K = 7*4*8 = 224 instead of the 7*7*8 = 392 a
    channel-padded NHWC stem needs (1.75x fewer MFMA operations, every 16-byte load one tap).
    Parameter layout/state stay torchvision's [64, 3, 7, 7]."""

    CIN_PAD = 8

    def packed_geometry(self, H: int, W: int):
        k, s, p = self.kernel_size[0], self.stride[0], self.padding[0]
        Ho, Wo = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
        return Ho, Wo, s * (Ho - 1) + k, Wo + (k + 1) // 2 - 1

    def packable(self) -> bool:
        return (self.in_channels <= 4 and self.kernel_size[0] == self.kernel_size[1]
                and self.stride[0] == 2 and self.stride[1] == 2)

    def pack_input(self, x: torch.Tensor, dtype) -> torch.Tensor:
        _, _, Hp, Wsp = self.packed_geometry(x.shape[2], x.shape[3])
        w = self.weight.detach()
        if K.use_native(x) and w.is_cuda and w.dtype == torch.float32:
            # the packing launch also packs this step's filter (consumed once by compute_weight)
            xp, wp = K.stem_pack(x, dtype, self.padding[0], Hp, Wsp, w=w)
            self.__dict__["_mipipe_wpack"] = wp
            return xp
        return K.stem_pack(x, dtype, self.padding[0], Hp, Wsp)

    def compute_weight(self, dtype):
        wp = self.__dict__.pop("_mipipe_wpack", None)
        if wp is not None and wp.dtype == dtype:
            return wp
        w = self.weight.detach()
        Co, C, k, _ = w.shape
        kw2 = (k + 1) // 2
        wp = w.new_zeros(Co, k, 2 * kw2, 4)            # [co, kh, kw(padded), c(padded)]
        wp[:, :, :k, :C] = w.permute(0, 2, 3, 1)
        # super-tap j holds kw = 2j + p at channels p*4 + c
        return wp.reshape(Co, k, kw2, 8).to(dtype).contiguous()

    def _ensure_wgrad_map(self):
        if getattr(self.weight, "_mipipe_wgrad_map", None) is None:
            k, C = self.kernel_size[0], self.in_channels

            def unpack(dw, k=k, C=C):  # [Co, k, k2, 8] (kernel layout) -> [Co, C, k, k]
                Co = dw.shape[0]
                d = dw.reshape(Co, k, -1, 4)[:, :, :k, :C]
                return d.permute(0, 3, 1, 2).contiguous()

            def unpack_into(dw, g):  # native: accumulate straight into g (the flat grad view)
                if dw.is_cuda and dw.dtype == torch.float32 and g.dtype == torch.float32:
                    K.stem_wgrad_unpack(dw.contiguous(), g)
                    return True
                return False
            unpack.accumulate_into = unpack_into
            self.weight._mipipe_wgrad_map = unpack

    def forward(self, x, stats_shift=None, slabs=None, prev=None, res_take=None, res_give=None):
        """x: packed super-pixels from :meth:`pack_input`."""
        w_c = self.compute_weight(x.dtype)
        self._ensure_wgrad_map()
        y, ps, pss = MF.conv2d(x, self.weight, w_c, (self.stride[0], 1), 0, stats_shift, slabs,
                               prev, res_take, res_give)
        return y if stats_shift is None else (y, ps, pss)

    def fused_bn_relu_maxpool(self, xp, bn, k: int, s: int, p: int):
        """maxpool(relu(bn(conv(xp)))) on the recompute-fused stem kernels (stem.hip), or None
        when they do not apply (other geometry / dtype / pool, eval with autograd on)."""
        if (k, s, p) != (3, 2, 1) or self.bias is not None or self.kernel_size[0] != 7:
            return None
        if not bn.training and torch.is_grad_enabled():
            return None
        w_c = self.compute_weight(xp.dtype)
        if not MF.stem_fused_ok(xp, w_c, bn):
            return None
        self._ensure_wgrad_map()
        return MF.stem_conv_bn_relu_maxpool(xp, self.weight, w_c, bn)


class _PaddedStemConv(mnn.Conv2d):
    """Generic stem for > 4 input channels: channels zero-padded to a multiple of 8."""

    CIN_PAD = 8

    def packable(self) -> bool:
        return False

    def pack_input(self, x: torch.Tensor, dtype) -> torch.Tensor:
        return K.nchw_to_nhwc(x, dtype, self.CIN_PAD)

    def compute_weight(self, dtype):
        w = self.weight.detach().permute(0, 2, 3, 1)
        ci = w.shape[-1]
        if ci % self.CIN_PAD:
            w = torch.nn.functional.pad(w, (0, self.CIN_PAD - ci % self.CIN_PAD))
        return w.to(dtype).contiguous()


class ResNet(tnn.Module):
    def __init__(self, block: Type[Union[BasicBlock, Bottleneck]], layers: List[int],
                 num_classes: int = 1000, zero_init_residual: bool = False,
                 width_per_group: int = 64, in_chans: int = 3,
                 compute_dtype: Optional[torch.dtype] = None, groups: int = 1):
        super().__init__()
        self.inplanes = 64
        self.groups = groups
        self.base_width = width_per_group
        self.in_chans = in_chans
        self.compute_dtype = compute_dtype
        stem_cls = _StemConv if in_chans <= 4 else _PaddedStemConv
        self.conv1 = stem_cls(in_chans, 64, 7, stride=2, padding=3, bias=False)
        self.bn1 = mnn.BatchNorm2d(64)
        self.relu = mnn.ReLU(inplace=True)
        self.maxpool = mnn.MaxPool2d(kernel_size=3, stride=2, padding=1)
        self.layer1 = self._make_layer(block, 64, layers[0])
        self.layer2 = self._make_layer(block, 128, layers[1], stride=2)
        self.layer3 = self._make_layer(block, 256, layers[2], stride=2)
        self.layer4 = self._make_layer(block, 512, layers[3], stride=2)
        self.avgpool = mnn.AdaptiveAvgPool2d((1, 1))
        self.fc = mnn.Linear(512 * block.expansion, num_classes)
        for m in self.modules():
            if isinstance(m, (mnn.Conv2d, mnn.XConv2d)):
                tnn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, tnn.BatchNorm2d):
                tnn.init.ones_(m.weight)
                tnn.init.zeros_(m.bias)
        if zero_init_residual:
            for m in self.modules():
                if isinstance(m, Bottleneck):
                    tnn.init.zeros_(m.bn3.weight)
                elif isinstance(m, BasicBlock):
                    tnn.init.zeros_(m.bn2.weight)

    def _make_layer(self, block, planes, blocks, stride=1):
        downsample = None
        if stride != 1 or self.inplanes != planes * block.expansion:
            downsample = tnn.Sequential(_conv1x1(self.inplanes, planes * block.expansion, stride),
                                        mnn.BatchNorm2d(planes * block.expansion))
        layers = [block(self.inplanes, planes, stride, downsample, self.base_width, self.groups)]
        self.inplanes = planes * block.expansion
        for _ in range(1, blocks):
            layers.append(block(self.inplanes, planes, base_width=self.base_width,
                                groups=self.groups))
        return tnn.Sequential(*layers)

    def activation_dtype(self, x: torch.Tensor) -> torch.dtype:
        if self.compute_dtype is not None:
            return self.compute_dtype
        return torch.bfloat16 if x.is_cuda else torch.float32

    def forward_features(self, x: torch.Tensor) -> torch.Tensor:
        """NCHW float input -> NHWC features of layer4."""
        x = self.conv1.pack_input(x, self.activation_dtype(x))
        x = mnn.conv_bn_relu_maxpool(x, self.conv1, self.bn1, self.maxpool)
        x = self.layer1(x)
        x = self.layer2(x)
        x = self.layer3(x)
        return self.layer4(x)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        x = self.forward_features(x)
        x = self.avgpool(x)
        return self.fc(x)


def _resnet(block, layers, **kw) -> ResNet:
    kw.pop("pretrained", None)  # no network: pretrained weights cannot be fetched
    return ResNet(block, layers, **kw)


def resnet18(**kw) -> ResNet:
    return _resnet(BasicBlock, [2, 2, 2, 2], **kw)


def resnet34(**kw) -> ResNet:
    return _resnet(BasicBlock, [3, 4, 6, 3], **kw)


def resnet50(**kw) -> ResNet:
    return _resnet(Bottleneck, [3, 4, 6, 3], **kw)


def resnet101(**kw) -> ResNet:
    return _resnet(Bottleneck, [3, 4, 23, 3], **kw)


def resnet152(**kw) -> ResNet:
    return _resnet(Bottleneck, [3, 8, 36, 3], **kw)


def wide_resnet50_2(**kw) -> ResNet:
    return _resnet(Bottleneck, [3, 4, 6, 3], width_per_group=128, **kw)


def wide_resnet101_2(**kw) -> ResNet:
    return _resnet(Bottleneck, [3, 4, 23, 3], width_per_group=128, **kw)


def resnext50_32x4d(**kw) -> ResNet:
    return _resnet(Bottleneck, [3, 4, 6, 3], groups=32, width_per_group=4, **kw)


def resnext101_32x8d(**kw) -> ResNet:
    return _resnet(Bottleneck, [3, 4, 23, 3], groups=32, width_per_group=8, **kw)
