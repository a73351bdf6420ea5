#!/usr/bin/env python3
"""Where does the ~15 us of bn_bwd_collect come from?  Times, with device events, loops of
  (a) fused dgrad (BN-backward partials -> replica slab) + collect,
  (b) the fused dgrad alone,
  (c) collect alone,
  (d) fused dgrad + a tiny unrelated kernel + collect
for a layer-1 and a layer-4 ResNet-50 b256 shape.
"""
from __future__ import annotations

import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from mipipe.ops import kernels as K  # noqa: E402


def timed(fn, iters=50):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters * 1e3  # us


def main():
    dev = torch.device("cuda")
    R = K.native().STAT_REPLICAS
    out = []
    for name, (N, H, Co, Ci) in {"l1.c3": (256, 56, 256, 64), "l4.c3": (256, 7, 2048, 512),
                                 "l2.c3": (256, 28, 512, 128)}.items():
        dy = torch.randn(N, H, H, Co, device=dev).to(torch.bfloat16)
        w = (torch.randn(Co, 1, 1, Ci, device=dev) * 0.05).to(torch.bfloat16)
        y = torch.randn(N, H, H, Ci, device=dev).to(torch.bfloat16)
        mean = torch.zeros(Ci, device=dev)
        invstd = torch.ones(Ci, device=dev)
        scale = torch.ones(Ci, device=dev)
        bias = torch.zeros(Ci, device=dev)
        rep = torch.zeros(3, R, Ci, device=dev)
        dg = torch.zeros(Ci, device=dev)
        db = torch.zeros(Ci, device=dev)
        tiny = torch.zeros(16, device=dev)
        bnr = (y, mean, invstd, scale, bias, rep)
        shp = (N, H, H, Ci)

        def dgrad():
            return K.conv_dgrad(dy, w, shp, 1, 0, bnr=bnr)

        def collect():
            return K.bn_bwd_collect(rep, Ci, (dg, db))

        def both():
            dgrad()
            collect()

        def plain():
            return K.conv_dgrad(dy, w, shp, 1, 0)

        def plain_collect():
            plain()
            collect()

        def fused_plain():
            dgrad()
            plain()

        def both_gap():
            dgrad()
            tiny.add_(1.0)
            collect()

        r = {"shape": name, "dgrad+collect_us": round(timed(both), 1),
             "dgrad_us": round(timed(dgrad), 1), "collect_us": round(timed(collect), 1),
             "dgrad+tiny+collect_us": round(timed(both_gap), 1),
             "tiny_us": round(timed(lambda: tiny.add_(1.0)), 1),
             "plain_us": round(timed(plain), 1),
             "plain+collect_us": round(timed(plain_collect), 1),
             "fused+plain_us": round(timed(fused_plain), 1)}
        print(json.dumps(r), flush=True)
        out.append(r)


if __name__ == "__main__":
    main()
