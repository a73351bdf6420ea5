"""Per-layer microbenchmark: mipipe conv kernels vs MIOpen (stock torch, channels_last bf16)
on the ResNet-50 @224, batch 256 conv shapes.  Prints one JSON line per shape.

python tools/bench_kernels.py [--batch 256] [--iters 10] [--only fwd|dgrad|wgrad]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mipipe.ops._native import native  # noqa: E402


def resnet50_convs(B):
    """(name, N, H, W, Ci, Co, k, s, p, count) for every distinct conv of ResNet-50 @224."""
    out = [("stem", B, 224, 224, 8, 64, 7, 2, 3, 1)]
    H = 56
    inpl = 64
    for li, (planes, blocks, stride) in enumerate([(64, 3, 1), (128, 4, 2), (256, 6, 2), (512, 3, 2)]):
        for b in range(blocks):
            s = stride if b == 0 else 1
            Hin = H
            Hout = H // s
            out.append((f"l{li+1}.{b}.c1", B, Hin, Hin, inpl, planes, 1, 1, 0, 1))
            out.append((f"l{li+1}.{b}.c2", B, Hin, Hin, planes, planes, 3, s, 1, 1))
            out.append((f"l{li+1}.{b}.c3", B, Hout, Hout, planes, planes * 4, 1, 1, 0, 1))
            if b == 0:
                out.append((f"l{li+1}.{b}.ds", B, Hin, Hin, inpl, planes * 4, 1, s, 0, 1))
            inpl = planes * 4
            H = Hout
    # merge identical shapes
    merged = {}
    for (n, *shape) in out:
        key = tuple(shape[:-1])
        if key in merged:
            merged[key][1] += 1
        else:
            merged[key] = [n, 1]
    return [(v[0], *k, v[1]) for k, v in merged.items()]


def timeit(fn, iters):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--no-torch", action="store_true")
    a = ap.parse_args()
    dev = "cuda"
    torch.backends.cudnn.benchmark = True
    C = native()
    tot = {"ours_fwd": 0.0, "ours_dgrad": 0.0, "ours_wgrad": 0.0, "torch_fwd": 0.0, "torch_bwd": 0.0}
    for (name, N, H, W, Ci, Co, k, s, p, cnt) in resnet50_convs(a.batch):
        Ho, Wo = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
        x = torch.randn(N, H, W, Ci, device=dev).to(torch.bfloat16)
        w = (torch.randn(Co, k, k, Ci, device=dev) / (Ci * k * k) ** 0.5).to(torch.bfloat16)
        dy = torch.randn(N, Ho, Wo, Co, device=dev).to(torch.bfloat16)
        shift = torch.zeros(Co, device=dev)
        flops = 2.0 * N * Ho * Wo * Co * Ci * k * k
        r = {"layer": name, "shape": [N, H, W, Ci, Co, k, s, p], "count": cnt}
        t = timeit(lambda: C.conv_fwd(x, w, s, p, shift), a.iters)
        r["fwd_us"] = round(t, 1)
        r["fwd_tflops"] = round(flops / t / 1e6, 1)
        if name != "stem":
            t2 = timeit(lambda: C.conv_dgrad(dy, w, [N, H, W, Ci], s, p), a.iters)
            r["dgrad_us"] = round(t2, 1)
            r["dgrad_tflops"] = round(flops / t2 / 1e6, 1)
            tot["ours_dgrad"] += t2 * cnt
        t3 = timeit(lambda: C.conv_wgrad(dy, x, k, k, s, p), a.iters)
        r["wgrad_us"] = round(t3, 1)
        r["wgrad_tflops"] = round(flops / t3 / 1e6, 1)
        tot["ours_fwd"] += t * cnt
        tot["ours_wgrad"] += t3 * cnt
        if not a.no_torch:
            xt = x.permute(0, 3, 1, 2).contiguous(memory_format=torch.channels_last)
            wt = w.permute(0, 3, 1, 2).contiguous(memory_format=torch.channels_last)
            tf = timeit(lambda: F.conv2d(xt, wt, stride=s, padding=p), a.iters)
            xt.requires_grad_(True)
            wt.requires_grad_(True)
            yt = F.conv2d(xt, wt, stride=s, padding=p)
            dyt = dy.permute(0, 3, 1, 2).contiguous(memory_format=torch.channels_last)
            tb = timeit(lambda: torch.autograd.grad(yt, [xt, wt], dyt, retain_graph=True), a.iters)
            r["torch_fwd_us"] = round(tf, 1)
            r["torch_bwd_us"] = round(tb, 1)
            tot["torch_fwd"] += tf * cnt
            tot["torch_bwd"] += tb * cnt
        print(json.dumps(r), flush=True)
    print(json.dumps({"totals_us": {k: round(v, 1) for k, v in tot.items()}}), flush=True)


if __name__ == "__main__":
    main()
