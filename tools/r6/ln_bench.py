"""LayerNorm kernel families timed on BERT-base shapes (4096 x 768 rows, residual + dropout
forward; dropout + bias-sum backward): mode 0 = generic kernels, 4 / 8 / 16 = exact-width."""
import json
import sys

import torch

from mipipe.ops._native import native

dev = "cuda"
N = native()


def timeit(fn, iters=200):
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters * 1e3


out = []
for R, H in [(4096, 768), (640, 768), (4096, 1024), (16384, 768)]:
    x = torch.randn(R, H, device=dev).to(torch.bfloat16)
    res = torch.randn(R, H, device=dev).to(torch.bfloat16)
    dy = torch.randn(R, H, device=dev).to(torch.bfloat16)
    g, b = torch.rand(H, device=dev) + 0.5, torch.randn(H, device=dev)
    ga, ba, da = torch.zeros(H, device=dev), torch.zeros(H, device=dev), torch.zeros(H, device=dev)
    for mode in (0, 4, 8, 16):
        N.set_layernorm_mode(mode)
        y, m, r, xs = N.layernorm_fwd(x, g, b, 1e-12, res, 0.1, 7)
        tf = timeit(lambda: N.layernorm_fwd(x, g, b, 1e-12, res, 0.1, 7))
        tb = timeit(lambda: N.layernorm_bwd(dy, xs, m, r, g, ga, ba, 0.1, 7, None, da))
        rec = {"R": R, "H": H, "mode": mode, "fwd_us": round(tf, 2), "bwd_us": round(tb, 2)}
        out.append(rec)
        print(json.dumps(rec), flush=True)
N.set_layernorm_mode(16)
