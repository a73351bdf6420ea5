"""Sweep the split-K workgroup target for the atomically-accumulated weight-gradient GEMMs
(conv wgrad on ResNet-50 shapes, Linear wgrad on BERT-base shapes).  Interleaved rounds in one
process (guide §5.4 rule 24); prints one JSON line per (target, shape) with the median time."""
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


cases = []
B = 256
for (H, Ci, Co, k, st, p) in [(56, 64, 64, 3, 1, 1), (56, 64, 256, 1, 1, 0), (28, 128, 128, 3, 1, 1),
                              (14, 256, 256, 3, 1, 1), (7, 512, 512, 3, 1, 1), (14, 1024, 256, 1, 1, 0),
                              (7, 2048, 512, 1, 1, 0), (224, 8, 64, 7, 2, 3)]:
    Ho = (H + 2 * p - k) // st + 1
    x = torch.randn(B, H, H, Ci, device=dev).to(torch.bfloat16)
    dy = torch.randn(B, Ho, Ho, Co, device=dev).to(torch.bfloat16)
    out = torch.zeros(Co, k, k, Ci, device=dev)
    cases.append((f"conv{H}x{Ci}->{Co}k{k}s{st}",
                  lambda x=x, dy=dy, k=k, st=st, p=p, out=out: C.conv_wgrad(dy, x, k, k, st, p, out)))
for (T, fin, fout) in [(4096, 768, 2304), (4096, 768, 768), (4096, 768, 3072), (4096, 3072, 768)]:
    x = torch.randn(T, fin, device=dev).to(torch.bfloat16)
    dy = torch.randn(T, fout, device=dev).to(torch.bfloat16)
    g = torch.zeros(fout, fin, device=dev)
    cases.append((f"linear{T}x{fin}->{fout}",
                  lambda x=x, dy=dy, g=g: C.gemm(dy, x, True, False, None, "none", torch.float32, g, 1.0)))

targets = [int(v) for v in (sys.argv[1:] or ["128", "256", "512", "768", "1024", "2048"])]
res = {(t, n): [] for t in targets for n, _ in cases}
for rnd in range(3):
    for t in targets:
        C.set_splitk_target(t)
        for n, fn in cases:
            res[(t, n)].append(t_us(fn))
C.set_splitk_target(512)
for n, _ in cases:
    row = {"shape": n}
    for t in targets:
        row[str(t)] = round(statistics.median(res[(t, n)]), 1)
    print(json.dumps(row), flush=True)
