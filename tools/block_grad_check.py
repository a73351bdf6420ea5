#!/usr/bin/env python3
"""Localise a gradient error to a ResNet building block: each block runs fwd + bwd on the GPU
(mipipe kernels, --dtype) and in float64 on the CPU (plain torch ops on the same module tree);
prints the relative error of the output, the input gradient and every parameter gradient."""
from __future__ import annotations

import argparse
import copy
import os
import sys

import torch
import torch.nn as tnn

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).abs().max() / (b.abs().max() + 1e-30)).item()


class Wrap(tnn.Module):
    """NHWC block under test with the model's compute dtype for the input conversion."""

    def __init__(self, body, dtype):
        super().__init__()
        self.body = body
        self.dtype = dtype

    def forward(self, x):  # x: NHWC float
        return self.body(x.to(self.dtype))


def run(name, body, x_shape, dtype, dev="cuda", seed=0):
    torch.manual_seed(seed)
    ref = copy.deepcopy(body).double()
    gpu = body.to(dev)
    x = torch.randn(*x_shape)
    xg = x.to(dev).to(dtype).detach().clone().requires_grad_(True)
    xr = x.double().detach().clone().requires_grad_(True)
    yg = gpu(xg)
    yr = ref(xr)
    w = torch.randn(yr.shape, dtype=torch.float64)
    (yg.double() * w.to(dev)).sum().backward()
    (yr * w).sum().backward()
    print(f"{name}: out {rel(yg, yr):.2e}  dx {rel(xg.grad, xr.grad):.2e}")
    pr = dict(ref.named_parameters())
    for n, p in gpu.named_parameters():
        e = rel(p.grad, pr[n].grad)
        flag = "  <-- " if e > 1e-3 else ""
        print(f"    {n:32s} {e:.2e}{flag}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dtype", default="fp32", choices=["fp32", "bf16"])
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--device", default="cuda")
    ap.add_argument("--only", default="")
    a = ap.parse_args()
    dt = torch.float32 if a.dtype == "fp32" else torch.bfloat16
    from mipipe import nn as mnn
    from mipipe.models.resnet import BasicBlock, Bottleneck, _conv1x1
    N = a.batch

    class ConvBN(tnn.Module):
        def __init__(self, cin, cout, k, s, relu):
            super().__init__()
            self.conv = mnn.Conv2d(cin, cout, k, stride=s, padding=k // 2)
            self.bn = mnn.BatchNorm2d(cout)
            self.relu = relu

        def forward(self, x):
            return mnn.conv_bn_act(x, self.conv, self.bn, relu=self.relu)

    class TwoConvBN(tnn.Module):  # second conv fuses the first BN's backward reductions
        def __init__(self, c):
            super().__init__()
            self.a = ConvBN(c, c, 3, 1, True)
            self.conv = mnn.Conv2d(c, c, 3, stride=1, padding=1)
            self.bn = mnn.BatchNorm2d(c)

        def forward(self, x):
            h = self.a(x)
            return mnn.conv_bn_act(h, self.conv, self.bn, relu=True, fuse_prev=True)

    def ds(cin, cout, s):
        return tnn.Sequential(_conv1x1(cin, cout, s), mnn.BatchNorm2d(cout))

    cases = [
        ("conv3x3+bn (no relu)", ConvBN(64, 64, 3, 1, False), (N, 8, 8, 64)),
        ("conv3x3+bn+relu", ConvBN(64, 64, 3, 1, True), (N, 8, 8, 64)),
        ("conv1x1 64->128 +bn+relu", ConvBN(64, 128, 1, 1, True), (N, 8, 8, 64)),
        ("conv1x1 64->128 +bn", ConvBN(64, 128, 1, 1, False), (N, 8, 8, 64)),
        ("conv1x1 64->64 +bn+relu", ConvBN(64, 64, 1, 1, True), (N, 8, 8, 64)),
        ("conv1x1 128->128 +bn+relu", ConvBN(128, 128, 1, 1, True), (N, 8, 8, 128)),
        ("conv3x3 64->128 +bn+relu", ConvBN(64, 128, 3, 1, True), (N, 8, 8, 64)),
        ("two conv+bn (fused dgrad BN)", TwoConvBN(64), (N, 8, 8, 64)),
        ("BasicBlock identity", BasicBlock(64, 64), (N, 8, 8, 64)),
        ("BasicBlock downsample", BasicBlock(64, 128, 2, ds(64, 128, 2)), (N, 8, 8, 64)),
        ("BasicBlock 1x1 spatial", BasicBlock(512, 512), (N, 1, 1, 512)),
        ("Bottleneck identity", Bottleneck(256, 64), (N, 8, 8, 256)),
        ("two BasicBlocks", tnn.Sequential(BasicBlock(64, 64), BasicBlock(64, 64)), (N, 8, 8, 64)),
    ]
    for name, body, shp in cases:
        if a.only and a.only not in name:
            continue
        for mod in body.modules():
            if isinstance(mod, tnn.BatchNorm2d):
                mod.train()
        run(name, body, shp, dt, a.device)


if __name__ == "__main__":
    main()
