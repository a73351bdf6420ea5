"""Time single conv ops (fwd / dgrad / wgrad) per plan with CUDA events; one JSON line each.
usage: python tools/r5/conv_time.py TAG op:N,H,Ci,Co,k,s,p:cfg [...]"""
import json
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402
from mipipe.ops._native import native  # noqa: E402

C = native()
tag = sys.argv[1]
for spec in sys.argv[2:]:
    op, shape, cfg = spec.split(":")
    N, H, Ci, Co, k, s, p = [int(v) for v in shape.split(",")]
    cfg = int(cfg)
    Ho = (H + 2 * p - k) // s + 1
    x = torch.randn(N, H, H, Ci, device="cuda").to(torch.bfloat16)
    w = (torch.randn(Co, k, k, Ci, device="cuda") * 0.05).to(torch.bfloat16)
    dy = torch.randn(N, Ho, Ho, Co, device="cuda").to(torch.bfloat16)
    sh = torch.zeros(Co, device="cuda")
    out = torch.zeros(Co, k, k, Ci, device="cuda")

    def run():
        if op == "fwd":
            C.conv_fwd(x, w, s, p, sh, cfg=cfg)
        elif op == "dgrad":
            C.conv_dgrad(dy, w, [N, H, H, Ci], s, p, cfg=cfg)
        else:
            C.conv_wgrad(dy, x, k, k, s, p, out, cfg=cfg)
    for _ in range(5):
        run()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 30
    e0.record()
    for _ in range(reps):
        run()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / reps
    fl = 2.0 * N * Ho * Ho * Co * k * k * Ci
    print(json.dumps({"tag": tag, "op": op, "shape": [N, H, Ci, Co, k, s, p], "cfg": cfg,
                      "us": round(us, 2), "tflops": round(fl / us / 1e6, 1)}), flush=True)
