"""ResNet-50 conv shapes (b256): forward / data-grad / weight-grad median us with operands warm
(resident in the memory-side cache) vs cold (after a 512 MB sweep) vs cold with each operand
re-read.  Does the GEMM-prefetch lever (ops/prefetch.py) carry over to the convolutions?"""
import json

import torch

from mipipe.ops._native import native

C = native()
dev = "cuda"
junk = torch.empty(512 << 20, dtype=torch.uint8, device=dev)
scratch = torch.empty(256 << 20, dtype=torch.uint8, device=dev)


def touch(t):
    C.touch([t])


def run(fn, setup, iters=30):
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(iters)]
    for i in range(iters + 3):
        setup()
        e = ev[i - 3] if i >= 3 else None
        if e:
            e[0].record()
        fn()
        if e:
            e[1].record()
    torch.cuda.synchronize()
    t = sorted(s.elapsed_time(f) * 1e3 for s, f in ev)
    return round(t[len(t) // 2], 1)


# (N, H, Ci, Co, k, s, p): layer1..4 3x3, a layer-3 / layer-4 1x1
for (N, H, Ci, Co, k, s, p) in [(256, 56, 64, 64, 3, 1, 1), (256, 28, 128, 128, 3, 1, 1),
                                (256, 14, 256, 256, 3, 1, 1), (256, 7, 512, 512, 3, 1, 1),
                                (256, 14, 1024, 256, 1, 1, 0), (256, 7, 512, 2048, 1, 1, 0)]:
    Ho = (H + 2 * p - k) // s + 1
    x = torch.randn(N, H, H, Ci, device=dev).to(torch.bfloat16)
    w = (torch.randn(Co, k, k, Ci, device=dev) * 0.05).to(torch.bfloat16)
    dy = torch.randn(N, Ho, Ho, Co, device=dev).to(torch.bfloat16)
    sh = torch.zeros(Co, device=dev)
    out = torch.zeros(Co, k, k, Ci, device=dev)
    ops = {"fwd": (lambda: C.conv_fwd(x, w, s, p, sh), x, w),
           "dgrad": (lambda: C.conv_dgrad(dy, w, [N, H, H, Ci], s, p), dy, w),
           "wgrad": (lambda: C.conv_wgrad(dy, x, k, k, s, p, out), dy, x)}
    for name, (fn, a, b) in ops.items():
        rec = {"shape": [N, H, Ci, Co, k], "op": name, "MB": [a.numel() * 2 >> 20, b.numel() * 2 >> 20],
               "warm": run(fn, lambda: None),
               "cold": run(fn, lambda: junk.fill_(1)),
               "cold_touch_a": run(fn, lambda: (junk.fill_(1), touch(a))),
               "cold_touch_b": run(fn, lambda: (junk.fill_(1), touch(b)))}
        print(json.dumps(rec), flush=True)
