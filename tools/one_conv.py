"""Run one conv shape's fwd (and optionally dgrad/wgrad) N times for PMC profiling."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from mipipe.ops._native import native
C = native()
N, H, Ci, Co, k, s, p = [int(v) for v in (sys.argv[1:8] if len(sys.argv) > 7 else [256, 14, 256, 256, 3, 1, 1])]
which = sys.argv[8] if len(sys.argv) > 8 else "fwd"
cfg = int(sys.argv[9]) if len(sys.argv) > 9 else -1
Ho = (H + 2 * p - k) // s + 1
x = torch.randn(N, H, H, Ci, device="cuda").to(torch.bfloat16)
w = (torch.randn(Co, k, k, Ci, device="cuda") * 0.05).to(torch.bfloat16)
dy = torch.randn(N, Ho, Ho, Co, device="cuda").to(torch.bfloat16)
sh = torch.zeros(Co, device="cuda")
out = torch.zeros(Co, k, k, Ci, device="cuda")
for _ in range(20):
    if which == "fwd":
        C.conv_fwd(x, w, s, p, sh, cfg=cfg)
    elif which == "dgrad":
        C.conv_dgrad(dy, w, [N, H, H, Ci], s, p, cfg=cfg)
    else:
        C.conv_wgrad(dy, x, k, k, s, p, out, cfg=cfg)
torch.cuda.synchronize()
print("done", which)
