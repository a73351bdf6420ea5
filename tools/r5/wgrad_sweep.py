#!/usr/bin/env python3
"""Weight-grad plan sweep (tile x split count x atomic / workspace) on ResNet-50's 1x1 shapes.

python tools/r5/wgrad_sweep.py [--iters 10]   (one JSON line per shape: every plan's us)"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from mipipe.ops._native import native  # noqa: E402
from tools.bench_kernels import timeit  # noqa: E402

SHAPES = [  # name, N, H, Ci, Co, k, s, p
    ("l1.0.c3", 256, 56, 64, 256, 1, 1, 0), ("l1.1.c1", 256, 56, 256, 64, 1, 1, 0),
    ("l2.0.c3", 256, 28, 128, 512, 1, 1, 0), ("l2.1.c1", 256, 28, 512, 128, 1, 1, 0),
    ("l3.0.c3", 256, 14, 256, 1024, 1, 1, 0), ("l3.1.c1", 256, 14, 1024, 256, 1, 1, 0),
    ("l4.0.c3", 256, 7, 512, 2048, 1, 1, 0), ("l4.1.c1", 256, 7, 2048, 512, 1, 1, 0),
    ("l3.1.c2", 256, 14, 256, 256, 3, 1, 1),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--tiles", default="0,1,2,3,4,5,7,8,9,10,14,15")
    a = ap.parse_args()
    C = native()
    tiles = [int(t) for t in a.tiles.split(",")]
    for (name, N, H, Ci, Co, k, s, p) in SHAPES:
        Ho = (H + 2 * p - k) // s + 1
        x = torch.randn(N, H, H, Ci, device="cuda").to(torch.bfloat16)
        dy = torch.randn(N, Ho, Ho, Co, device="cuda").to(torch.bfloat16)
        dw = torch.zeros(Co, k, k, Ci, device="cuda")
        flops = 2.0 * N * Ho * Ho * Co * Ci * k * k
        res = {}
        for t in tiles:
            for sp in (0, 4, 8, 16, 24, 32, 48):
                for ws in (0, 1024):
                    if ws and sp in (0,):
                        continue
                    plan = (t + 16 * sp) | ws
                    res[f"{t}/{sp}{'w' if ws else ''}"] = timeit(
                        lambda: C.conv_wgrad(dy, x, k, k, s, p, out=dw, cfg=plan), a.iters)
        d = timeit(lambda: C.conv_wgrad(dy, x, k, k, s, p, out=dw, cfg=-1), a.iters)
        best = min(res, key=res.get)
        top = sorted(res.items(), key=lambda kv: kv[1])[:8]
        print(json.dumps({"layer": name, "default_us": round(d, 1), "best": best,
                          "best_us": round(res[best], 1),
                          "best_tflops": round(flops / res[best] / 1e6, 1),
                          "top": [(k_, round(v, 1)) for k_, v in top]}), flush=True)


if __name__ == "__main__":
    main()
