"""FFN-out GEMM cold-cache probe, part 2: after a 512 MB sweep, which operand's re-warming
restores the warm time — the weight (B) or the activation (A)?"""
import json

import torch

from mipipe.ops._native import native

N = native()
dev = "cuda"
junk = torch.empty(512 << 20, dtype=torch.uint8, device=dev)
scratch = torch.empty(64 << 20, dtype=torch.uint8, device=dev)


def touch(t):
    b = t.view(torch.uint8).reshape(-1)
    scratch[: b.numel()].copy_(b)


def run(a, w, bias, plan, setup, iters=40):
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(iters)]
    for i in range(iters + 5):
        setup()
        e = ev[i - 5] if i >= 5 else None
        if e:
            e[0].record()
        N.gemm(a, w, False, True, bias, "none", torch.bfloat16, None, 0.0, plan)
        if e:
            e[1].record()
    torch.cuda.synchronize()
    t = sorted(s.elapsed_time(f) * 1e3 for s, f in ev)
    return round(t[len(t) // 2], 2)


for name, (M, Nn, K), plans in [("ffn_out", (4096, 768, 3072), (8, 2)),
                                ("attn_out", (4096, 768, 768), (8,)),
                                ("ffn_in", (4096, 3072, 768), (1,)),
                                ("qkv", (4096, 2304, 768), (1,))]:
    a = torch.randn(M, K, device=dev).to(torch.bfloat16)
    w = (torch.randn(Nn, K, device=dev) / K ** 0.5).to(torch.bfloat16)
    bias = torch.randn(Nn, device=dev)
    for plan in plans:
        rec = {"gemm": name, "plan": plan,
               "warm": run(a, w, bias, plan, lambda: None),
               "cold": run(a, w, bias, plan, lambda: junk.fill_(1)),
               "cold_touch_w": run(a, w, bias, plan, lambda: (junk.fill_(1), touch(w))),
               "cold_touch_a": run(a, w, bias, plan, lambda: (junk.fill_(1), touch(a))),
               "cold_touch_both": run(a, w, bias, plan, lambda: (junk.fill_(1), touch(a), touch(w)))}
        print(json.dumps(rec), flush=True)
