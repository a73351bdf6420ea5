"""How many replica rows should the BN-statistics atomics spread over?  Times the 1x1/3x3 conv
forward with the fused BN-statistics epilogue and the dgrad with the fused BN-backward reduction
at several ``set_stat_rows`` values (the slab layout is always STAT_REPLICAS rows)."""
import json
import os
import sys

import torch

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
R = C.STAT_REPLICAS
for (N, H, W, Ci, Co, k, s, p) in [(256, 56, 56, 64, 256, 1, 1, 0), (256, 56, 56, 256, 64, 1, 1, 0),
                                   (256, 28, 28, 128, 512, 1, 1, 0), (256, 56, 56, 64, 64, 3, 1, 1),
                                   (256, 14, 14, 256, 1024, 1, 1, 0), (256, 7, 7, 512, 2048, 1, 1, 0)]:
    x = torch.randn(N, H, W, Ci, device="cuda").to(torch.bfloat16)
    w = (torch.randn(Co, k, k, Ci, device="cuda") / (Ci * k * k) ** 0.5).to(torch.bfloat16)
    shift = torch.zeros(Co, device="cuda")
    Ho, Wo = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
    dy = torch.randn(N, Ho, Wo, Co, device="cuda").to(torch.bfloat16)
    mean = torch.zeros(Ci, device="cuda")
    invstd = torch.ones(Ci, device="cuda")
    scale = torch.ones(Ci, device="cuda")
    bias = torch.zeros(Ci, device="cuda")
    rep = torch.zeros(3, R, Ci, device="cuda")
    s1 = torch.zeros(R, Co, device="cuda")
    s2 = torch.zeros(R, Co, device="cuda")
    r = {"shape": [N, H, W, Ci, Co, k]}
    for rows in (16, 32, 64):
        C.set_stat_rows(rows)
        r[f"fwd_stats_R{rows}"] = round(timeit(lambda: C.conv_fwd(x, w, s, p, shift, s1, s2)), 1)
        r[f"dgrad_bnr_R{rows}"] = round(timeit(
            lambda: C.conv_dgrad(dy, w, [N, H, W, Ci], s, p, None, x, mean, invstd, scale, bias,
                                 rep, None, -1)), 1)
    r["fwd_nostats"] = round(timeit(lambda: C.conv_fwd(x, w, s, p)), 1)
    r["dgrad_plain"] = round(timeit(lambda: C.conv_dgrad(dy, w, [N, H, W, Ci], s, p, None)), 1)
    print(json.dumps(r), flush=True)
C.set_stat_rows(R)
