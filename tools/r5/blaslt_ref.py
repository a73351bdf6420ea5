#!/usr/bin/env python3
"""hipBLASLt (torch.mm, bf16) on the GEMM equivalents of ResNet-50's 1x1 convs: the library's
time for the same M, N, K and operand layouts as mipipe's fwd / dgrad / wgrad kernels — what a
plain GEMM achieves on this GPU, as the comparator for the hand-written kernels."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from tools.bench_kernels import timeit  # noqa: E402

SHAPES = [("l1.0.c3", 256, 56, 64, 256), ("l1.1.c1", 256, 56, 256, 64), ("l2.0.c3", 256, 28, 128, 512),
          ("l2.1.c1", 256, 28, 512, 128), ("l3.0.c3", 256, 14, 256, 1024),
          ("l3.1.c1", 256, 14, 1024, 256), ("l4.0.c3", 256, 7, 512, 2048),
          ("l4.1.c1", 256, 7, 2048, 512)]
for name, N, H, Ci, Co in SHAPES:
    M = N * H * H
    x = torch.randn(M, Ci, device="cuda").to(torch.bfloat16)
    dy = torch.randn(M, Co, device="cuda").to(torch.bfloat16)
    w = torch.randn(Co, Ci, device="cuda").to(torch.bfloat16)
    fl = 2.0 * M * Ci * Co
    out = {"layer": name}
    for op, fn in (("fwd", lambda: torch.mm(x, w.t())), ("dgrad", lambda: torch.mm(dy, w)),
                   ("wgrad", lambda: torch.mm(dy.t(), x))):
        us = timeit(fn, 20)
        out[op] = [round(us, 1), round(fl / us / 1e6, 1)]
    print(json.dumps(out), flush=True)
a = torch.randn(4096, 4096, device="cuda").to(torch.bfloat16)
us = timeit(lambda: torch.mm(a, a), 20)
print(json.dumps({"gemm4096": [round(us, 1), round(2 * 4096 ** 3 / us / 1e6, 1)]}))
