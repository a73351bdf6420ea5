#!/usr/bin/env python3
"""Per-shape conv roofline table for ResNet-50 b256 bf16: runs one eager training step with the
tile tuner in verbose mode (every candidate plan timed on scratch outputs) and prints, per
(op, shape), the best time, its TFLOP/s and the fraction of the 2.5 PFLOP/s dense bf16 peak.

usage: python tools/r2/tune_dump.py [--batch 256]   (GPU)
       python tools/r2/tune_dump.py --parse log.txt  (summarise a saved stderr log)
"""
from __future__ import annotations

import argparse
import os
import re
import subprocess
import sys

PEAK = 2.5e15
LINE = re.compile(r"\[mipipe tune\] (\w+)\|([\d,\-]+)\|(\w+) -> (-?\d+)\s+\(us:(.*)\)")


def flops(op: str, shp: list) -> float:
    N, H, W, Ci, Co, KH, KW, S, P = shp[:9]
    Ho = (H + 2 * P - KH) // S + 1
    Wo = (W + 2 * P - KW) // S + 1
    return 2.0 * N * Ho * Wo * Co * Ci * KH * KW


def parse(text: str) -> None:
    rows = []
    for m in LINE.finditer(text):
        op, shp, dt, best, times = m.groups()
        shp = [int(v) for v in shp.split(",")]
        if len(shp) < 9:  # GEMM keys
            continue
        ts = {}
        for tok in times.split():
            k, v = tok.split(":")
            ts[int(k)] = float(v)
        if not ts:
            continue
        bt = min(ts.values())
        f = flops(op, shp)
        rows.append((bt, op, shp, int(best), f / (bt * 1e-6) / 1e12))
    rows.sort(reverse=True)
    tot = sum(r[0] for r in rows)
    print(f"{'op':6s} {'N,H,W,Ci,Co,KH,KW,S,P':34s} {'best':>5s} {'us':>8s} {'TF/s':>7s} {'%peak':>6s}")
    for bt, op, shp, best, tf in rows:
        print(f"{op:6s} {','.join(map(str, shp[:9])):34s} {best:5d} {bt:8.1f} {tf:7.0f} {100 * tf * 1e12 / PEAK:5.1f}%")
    print(f"sum of best times over distinct shapes: {tot:.0f} us")


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--parse")
    ap.add_argument("--batch", type=int, default=256)
    a = ap.parse_args()
    if a.parse:
        parse(open(a.parse).read())
        return 0
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
    import torch
    from mipipe.models import create_model
    from mipipe.ops import tuning
    from mipipe.ops.functional import cross_entropy
    from mipipe.optim import SGD
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    model = create_model("resnet50", num_classes=1000).to(dev)
    model.compute_dtype = torch.bfloat16
    opt = SGD(model.parameters(), 0.1, momentum=0.9, weight_decay=1e-4)
    x = torch.randn(a.batch, 3, 224, 224, device=dev)
    y = torch.randint(0, 1000, (a.batch,), device=dev)
    tuning.set_benchmark(True, verbose=True, reps=5)
    opt.zero_grad()
    cross_entropy(model(x), y).backward()
    opt.step()
    torch.cuda.synchronize()
    return 0


if __name__ == "__main__":
    sys.exit(main())
