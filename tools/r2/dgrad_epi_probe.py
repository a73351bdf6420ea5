#!/usr/bin/env python3
"""Fused data-grad epilogue cost on the ResNet-50 layer-1 shapes: plain dgrad vs + residual
addend vs + BN-backward reduction (mask from y, from stored z, from 1-bit mask) for every tile
config.  Prints one JSON line per (shape, variant) with the best / per-config times and the
achieved HBM bandwidth of the ideal traffic."""
from __future__ import annotations

import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from mipipe.ops._native import native  # noqa: E402


def timed(fn, iters=20):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters * 1e3


# tiles-per-block sweep of a looping-grid build (round-2 experiment, reverted: not faster)
KS = [int(v) for v in os.environ.get("LOOPS", "1").split(",")]


def main():
    dev = torch.device("cuda")
    nat = native()
    R = nat.STAT_REPLICAS
    cfgs = list(range(nat.CONV_TILE_CONFIGS))
    shapes = {"l1.conv1(256->64)": (256, 56, 64, 256), "l1.conv3(64->256)": (256, 56, 256, 64),
              "l3.conv1(1024->256)": (256, 14, 256, 1024)}
    for name, (N, H, Co, Ci) in shapes.items():
        bf = lambda *s: torch.randn(*s, device=dev).to(torch.bfloat16)  # noqa: E731
        dy = bf(N, H, H, Co)
        w = (torch.randn(Co, 1, 1, Ci, device=dev) * 0.05).to(torch.bfloat16)
        y, add, z = bf(N, H, H, Ci), bf(N, H, H, Ci), bf(N, H, H, Ci)
        mask = torch.randint(0, 255, (N * H * H * Ci // 8,), device=dev, dtype=torch.uint8)
        mean, invstd = torch.zeros(Ci, device=dev), torch.ones(Ci, device=dev)
        scale, bias = torch.ones(Ci, device=dev), torch.zeros(Ci, device=dev)
        rep = torch.zeros(3, R, Ci, device=dev)
        shp = [N, H, H, Ci]
        E = N * H * H * Ci * 2  # bytes of one dx-sized bf16 tensor
        shift = torch.zeros(Co, device=dev)
        variants = {
            "fwd_stats": (lambda c: nat.conv_fwd(y, w, 1, 0, shift, cfg=c), E + E // Ci * Co),
            "plain": (lambda c: nat.conv_dgrad(dy, w, shp, 1, 0, cfg=c), E // Ci * Co + E),
            "addend": (lambda c: nat.conv_dgrad(dy, w, shp, 1, 0, add, cfg=c), E // Ci * Co + 2 * E),
            "bn_y": (lambda c: nat.conv_dgrad(dy, w, shp, 1, 0, None, y, mean, invstd, scale, bias,
                                              rep, cfg=c), E // Ci * Co + 2 * E),
            "bn_mask_addend": (lambda c: nat.conv_dgrad(dy, w, shp, 1, 0, add, y, mean, invstd,
                                                        scale, bias, rep, None, cfg=c,
                                                        bn_mask=mask), E // Ci * Co + 3 * E + E // 16),
        }
        for vn, (fn, bytes_) in variants.items():
          for k in (KS if vn in ("fwd_stats", "bn_y", "bn_mask_addend") else (1,)):
            if hasattr(nat, "set_stat_loop"):
                nat.set_stat_loop(k)
            t = {}
            for c in cfgs:
                try:
                    t[c] = round(timed(lambda: fn(c)), 1)
                except RuntimeError as ex:  # config not valid for this op
                    t[c] = str(ex)[:40]
            num = {c: v for c, v in t.items() if isinstance(v, float)}
            best = min(num, key=num.get)
            print(json.dumps({"shape": name, "variant": vn, "loop": k, "best_cfg": best,
                              "best_us": num[best],
                              "TBps": round(bytes_ / num[best] / 1e6, 2), "us": t}), flush=True)
            rep.zero_()


if __name__ == "__main__":
    main()
