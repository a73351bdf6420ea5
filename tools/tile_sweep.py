#!/usr/bin/env python3
"""Time every conv tile config (csrc/kernels/conv_common.hpp table) on every distinct ResNet-50
@224 conv shape (fwd / dgrad / wgrad) and report the per-shape best against the heuristic
default.  This is the offline view of what benchmark mode (mipipe.ops.tuning) does online.

python tools/tile_sweep.py [--batch 256] [--iters 10] [--dtype bf16|fp32] [--model resnet50]
Prints one JSON line per (layer, op) and a totals line (count-weighted, us per step).
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mipipe.ops._native import native  # noqa: E402
from tools.bench_kernels import resnet50_convs, timeit  # noqa: E402


def resnet18_convs(B, res):
    H = res // 4
    out = [("stem", B, res, res, 8, 64, 7, 2, 3, 1)]
    inpl = 64
    for li, (planes, stride) in enumerate([(64, 1), (128, 2), (256, 2), (512, 2)]):
        for b in range(2):
            s = stride if b == 0 else 1
            Hout = (H + 2 - 3) // s + 1
            out.append((f"l{li+1}.{b}.c1", B, H, H, inpl, planes, 3, s, 1, 1))
            out.append((f"l{li+1}.{b}.c2", B, Hout, Hout, planes, planes, 3, 1, 1, 1))
            if b == 0 and (s != 1 or inpl != planes):
                out.append((f"l{li+1}.{b}.ds", B, H, H, inpl, planes, 1, s, 0, 1))
            inpl = planes
            H = Hout
    merged = {}
    for (n, *shape) in out:
        key = tuple(shape[:-1])
        merged.setdefault(key, [n, 0])[1] += 1
    return [(v[0], *k, v[1]) for k, v in merged.items()]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--res", type=int, default=224)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--model", default="resnet50", choices=["resnet50", "resnet18"])
    a = ap.parse_args()
    dev = "cuda"
    dt = torch.bfloat16 if a.dtype == "bf16" else torch.float32
    C = native()
    cfgs = list(range(C.CONV_TILE_CONFIGS)) if a.dtype == "bf16" else [0, 2, 8]
    shapes = resnet50_convs(a.batch) if a.model == "resnet50" else resnet18_convs(a.batch, a.res)
    tot_def = {"fwd": 0.0, "dgrad": 0.0, "wgrad": 0.0}
    tot_best = {"fwd": 0.0, "dgrad": 0.0, "wgrad": 0.0}
    for (name, N, H, W, Ci, Co, k, s, p, cnt) in shapes:
        Ho, Wo = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
        x = torch.randn(N, H, W, Ci, device=dev).to(dt)
        w = (torch.randn(Co, k, k, Ci, device=dev) / (Ci * k * k) ** 0.5).to(dt)
        dy = torch.randn(N, Ho, Wo, Co, device=dev).to(dt)
        shift = torch.zeros(Co, device=dev)
        flops = 2.0 * N * Ho * Wo * Co * Ci * k * k
        dw = torch.zeros(Co, k, k, Ci, device=dev)
        ops = {
            "fwd": lambda c: C.conv_fwd(x, w, s, p, shift, cfg=c),
            "dgrad": lambda c: C.conv_dgrad(dy, w, [N, H, W, Ci], s, p, cfg=c),
            "wgrad": lambda c: C.conv_wgrad(dy, x, k, k, s, p, out=dw, cfg=c),
        }
        for op, fn in ops.items():
            if op == "dgrad" and name == "stem":
                continue
            times = {}
            for c in cfgs:
                if op == "wgrad" and c == 6:
                    continue
                times[c] = timeit(lambda: fn(c), a.iters)
            t_def = timeit(lambda: fn(-1), a.iters)
            best = min(times, key=times.get)
            tot_def[op] += t_def * cnt
            tot_best[op] += times[best] * cnt
            print(json.dumps({"layer": name, "op": op, "shape": [N, H, W, Ci, Co, k, s, p],
                              "count": cnt, "default_us": round(t_def, 1), "best_cfg": best,
                              "best_us": round(times[best], 1),
                              "best_tflops": round(flops / times[best] / 1e6, 1),
                              "us": {str(c): round(v, 1) for c, v in times.items()}}), flush=True)
    print(json.dumps({"totals_us_default": {k: round(v, 1) for k, v in tot_def.items()},
                      "totals_us_best": {k: round(v, 1) for k, v in tot_best.items()},
                      "sum_default": round(sum(tot_def.values()), 1),
                      "sum_best": round(sum(tot_best.values()), 1)}), flush=True)


if __name__ == "__main__":
    main()
