"""Sweep the single-stage threshold for gathered convs (3x3 im2col fwd, dgrad classes)."""
import json, os, statistics, sys
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
cases = []
for (H, Ci, Co, st) in [(56, 64, 64, 1), (28, 128, 128, 1), (14, 256, 256, 1), (7, 512, 512, 1),
                        (56, 128, 128, 2), (28, 256, 256, 2), (56, 256, 512, 2)]:
    k, p = (3, 1) if Ci == Co else (1, 0)
    Ho = (H + 2 * p - k) // st + 1
    x = torch.randn(B, H, H, Ci, device=dev).to(torch.bfloat16)
    w = (torch.randn(Co, k, k, Ci, device=dev) * 0.05).to(torch.bfloat16)
    dy = torch.randn(B, Ho, Ho, Co, device=dev).to(torch.bfloat16)
    sh = torch.zeros(Co, device=dev)
    cases.append((f"fwd {H}x{Ci}->{Co} k{k}s{st}", lambda x=x, w=w, sh=sh, st=st, p=p: C.conv_fwd(x, w, st, p, sh)))
    cases.append((f"dgrad {H}x{Ci}->{Co} k{k}s{st}",
                  lambda dy=dy, w=w, H=H, Ci=Ci, st=st, p=p: C.conv_dgrad(dy, w, [B, H, H, Ci], st, p)))
ths = [0, 1152, 2304, 4608]
res = {(t, n): [] for t in ths for n, _ in cases}
for _ in range(3):
    for t in ths:
        C.set_ns1_max_k_gather(t)
        for n, fn in cases:
            res[(t, n)].append(t_us(fn))
C.set_ns1_max_k_gather(1152)
for n, _ in cases:
    print(json.dumps({"case": n, **{str(t): round(statistics.median(res[(t, n)]), 1) for t in ths}}), flush=True)
