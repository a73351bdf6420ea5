#!/usr/bin/env python3
"""Fused vs unfused stem: per-output relative differences (out, running stats, dW, dγ, dβ)."""
import copy
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    from mipipe import nn as mnn
    from mipipe.models.resnet import _StemConv
    from mipipe.ops import functional as MF
    torch.manual_seed(3)
    conv = _StemConv(3, 64, kernel_size=7, stride=2, padding=3, bias=False).cuda()
    bn = mnn.BatchNorm2d(64).cuda()
    pool = mnn.MaxPool2d(3, 2, 1)
    conv2, bn2 = copy.deepcopy(conv), copy.deepcopy(bn)
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    x = torch.randn(N, 3, 224, 224, device="cuda")
    dp = torch.randn(N, 56, 56, 64, device="cuda").to(torch.bfloat16)
    outs = []
    for c, b, fused in ((conv, bn, True), (conv2, bn2, False)):
        MF.set_stem_fused(fused)
        xp = c.pack_input(x, torch.bfloat16)
        o = mnn.conv_bn_relu_maxpool(xp, c, b, pool)
        o.backward(dp)
        torch.cuda.synchronize()
        outs.append((o, b.running_mean, b.running_var, c.weight.grad, b.weight.grad, b.bias.grad))

    def rel(a, b):
        return ((a.float() - b.float()).abs().max() / b.float().abs().max().clamp_min(1e-12)).item()
    for name, a, b in zip(["out", "rmean", "rvar", "dW", "dgamma", "dbeta"], outs[0], outs[1]):
        print(f"{name:8s} rel {rel(a, b):.3e}")
    dw_f, dw_u = outs[0][3], outs[1][3]
    print("dW per (c, kh) rel:")
    for c in range(3):
        print("  c", c, " ".join(f"{rel(dw_f[:, c, kh], dw_u[:, c, kh]):.1e}" for kh in range(7)))
    print("dW per kw:", " ".join(f"{rel(dw_f[..., kw], dw_u[..., kw]):.1e}" for kw in range(7)))


if __name__ == "__main__":
    main()
