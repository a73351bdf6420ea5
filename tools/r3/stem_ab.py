#!/usr/bin/env python3
"""ResNet stem forward+backward time, recompute-fused (stem.hip) vs unfused (packed conv +
pool_bn kernels), at the bench batch (b256, 224 px, bf16)."""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--modes", default="0,1,0,1", help="comma list of fused flags to time in order")
    a = ap.parse_args()
    from mipipe import nn as mnn
    from mipipe.models.resnet import _StemConv
    from mipipe.ops import functional as MF
    torch.manual_seed(0)
    conv = _StemConv(3, 64, kernel_size=7, stride=2, padding=3, bias=False).cuda()
    bn = mnn.BatchNorm2d(64).cuda()
    pool = mnn.MaxPool2d(3, 2, 1)
    x = torch.randn(a.batch, 3, 224, 224, device="cuda")
    xp = conv.pack_input(x, torch.bfloat16)
    dp = torch.randn(a.batch, 56, 56, 64, device="cuda").to(torch.bfloat16)
    for fused in (bool(int(v)) for v in a.modes.split(",")):
        MF.set_stem_fused(fused)
        for _ in range(3):
            mnn.conv_bn_relu_maxpool(xp, conv, bn, pool).backward(dp)
        torch.cuda.synchronize()
        e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
        tf = tb = 0.0
        for _ in range(a.iters):
            e0.record()
            out = mnn.conv_bn_relu_maxpool(xp, conv, bn, pool)
            e1.record()
            out.backward(dp)
            e2.record()
            torch.cuda.synchronize()
            tf += e0.elapsed_time(e1)
            tb += e1.elapsed_time(e2)
        print(f"fused={int(fused)} fwd {1e3 * tf / a.iters:8.1f} us  bwd {1e3 * tb / a.iters:8.1f} us"
              f"  total {1e3 * (tf + tb) / a.iters:8.1f} us", flush=True)


if __name__ == "__main__":
    main()
