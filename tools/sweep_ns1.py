"""Sweep the K threshold below which dense (1x1) conv fwd/dgrad use the single-LDS-stage
kernels (more blocks per CU, serial k-steps).  Interleaved rounds, medians."""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mipipe.ops._native import native  # noqa: E402

C = native()
dev = "cuda"


def t_us(fn, iters=10):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


B = 256
shapes = [(56, 64, 256), (56, 256, 64), (28, 128, 512), (28, 512, 128), (14, 256, 1024),
          (14, 1024, 256), (7, 512, 2048), (7, 2048, 512), (56, 256, 128)]
cases = []
for (H, Ci, Co) in shapes:
    x = torch.randn(B, H, H, Ci, device=dev).to(torch.bfloat16)
    w = (torch.randn(Co, 1, 1, Ci, device=dev) * 0.05).to(torch.bfloat16)
    dy = torch.randn(B, H, H, Co, device=dev).to(torch.bfloat16)
    sh = torch.zeros(Co, device=dev)
    cases.append((f"fwd {H}x{Ci}->{Co}", lambda x=x, w=w, sh=sh: C.conv_fwd(x, w, 1, 0, sh)))
    cases.append((f"dgrad {H}x{Ci}->{Co}",
                  lambda dy=dy, w=w, H=H, Ci=Ci: C.conv_dgrad(dy, w, [B, H, H, Ci], 1, 0)))
ths = [64, 128, 256, 512, 1024]
res = {(t, n): [] for t in ths for n, _ in cases}
for _ in range(3):
    for t in ths:
        C.set_ns1_max_k(t)
        for n, fn in cases:
            res[(t, n)].append(t_us(fn))
C.set_ns1_max_k(512)
for n, _ in cases:
    print(json.dumps({"case": n, **{str(t): round(statistics.median(res[(t, n)]), 1) for t in ths}}),
          flush=True)
