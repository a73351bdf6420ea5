"""Does warming the FFN-out weight help the FFN-out GEMM inside the forward sequence
(FFN-in GEMM -> GELU -> FFN-out)?  Median us of the FFN-out GEMM after each setup."""
import json

import torch

from mipipe.ops._native import native

N = native()
dev = "cuda"
junk = torch.empty(512 << 20, dtype=torch.uint8, device=dev)
x1 = torch.randn(4096, 768, device=dev).to(torch.bfloat16)
w1 = (torch.randn(3072, 768, device=dev) / 28).to(torch.bfloat16)
w2 = (torch.randn(768, 3072, device=dev) / 55).to(torch.bfloat16)
b1, b2 = torch.randn(3072, device=dev), torch.randn(768, device=dev)
st = {}


def fc1(pf=None):
    st["h"] = N.gemm(x1, w1, False, True, b1, "none", torch.bfloat16, None, 0.0, -1, None, pf)


def gelu():
    st["a"] = N.gelu_fwd(st["h"])


fc1()
gelu()


def run(setup, iters=40):
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(iters)]
    for i in range(iters + 5):
        setup()
        e = ev[i - 5] if i >= 5 else None
        if e:
            e[0].record()
        N.gemm(st["a"], w2, False, True, b2, "none", torch.bfloat16, None, 0.0)
        if e:
            e[1].record()
    torch.cuda.synchronize()
    t = sorted(s.elapsed_time(f) * 1e3 for s, f in ev)
    return round(t[len(t) // 2], 2)


cold = lambda: junk.fill_(1)  # noqa: E731
rec = {
    "warm": run(lambda: None),
    "cold_fc1_gelu": run(lambda: (cold(), fc1(), gelu())),
    "cold_fc1pf_gelu": run(lambda: (cold(), fc1([w2]), gelu())),
    "cold_fc1_gelu_touchw": run(lambda: (cold(), fc1(), gelu(), N.touch([w2]))),
    "cold_touchw_fc1_gelu": run(lambda: (cold(), N.touch([w2]), fc1(), gelu())),
    "cold_fc1_gelu_copyw": run(lambda: (cold(), fc1(), gelu(), w2.clone())),
    "cold_fc1_gelu_sumw": run(lambda: (cold(), fc1(), gelu(), w2.sum())),
}
print(json.dumps(rec), flush=True)
