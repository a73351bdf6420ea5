"""Where does a memory-bound 1x1 conv forward spend its time?  Times conv_fwd with / without the
fused BN-statistics epilogue and with the single- vs double-buffered main loop, next to the
stock conv and a plain copy of the same bytes."""
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mipipe.ops.kernels import native  # noqa: E402


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


C = native()
for (N, H, W, Ci, Co, k, s, p) in [(256, 56, 56, 64, 256, 1, 1, 0), (256, 56, 56, 256, 64, 1, 1, 0),
                                   (256, 28, 28, 128, 512, 1, 1, 0), (256, 56, 56, 64, 64, 3, 1, 1),
                                   (256, 14, 14, 256, 1024, 1, 1, 0)]:
    x = torch.randn(N, H, W, Ci, device="cuda").to(torch.bfloat16)
    w = (torch.randn(Co, k, k, Ci, device="cuda") / (Ci * k * k) ** 0.5).to(torch.bfloat16)
    shift = torch.zeros(Co, device="cuda")
    Ho, Wo = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
    out_b = N * Ho * Wo * Co * 2
    r = {"shape": [N, H, W, Ci, Co, k], "bytes_MB": round((x.numel() * 2 + out_b) / 1e6, 1)}
    for ns1 in (512, 0):
        C.set_ns1_max_k(ns1)
        r[f"stats_ns1max{ns1}"] = round(timeit(lambda: C.conv_fwd(x, w, s, p, shift)), 1)
        r[f"nostats_ns1max{ns1}"] = round(timeit(lambda: C.conv_fwd(x, w, s, p)), 1)
    C.set_ns1_max_k(512)
    xt = x.permute(0, 3, 1, 2)
    wt = w.permute(0, 3, 1, 2)
    r["torch"] = round(timeit(lambda: F.conv2d(xt, wt, stride=s, padding=p)), 1)
    y = torch.empty(N * Ho * Wo * Co, dtype=torch.bfloat16, device="cuda")
    r["fill_out_us"] = round(timeit(lambda: y.fill_(1.0)), 1)
    src = torch.empty_like(y)
    r["copy_out_us"] = round(timeit(lambda: y.copy_(src)), 1)
    print(json.dumps(r), flush=True)
