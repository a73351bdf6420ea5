"""colsum (bias-gradient column sum) grid sweep on BERT shapes: row-block count and one- vs
two-pass (partials + fixed-order sum)."""
import json
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
from mipipe.ops._native import native

N = native()
for rows, cols in [(4096, 768), (4096, 2304), (640, 30528)]:
    x = torch.randn(rows, cols, device="cuda").to(torch.bfloat16)
    ref = x.float().sum(0)
    for two in (False, True):
        for G in (0, 32, 64, 96, 128, 192, 256):
            N.set_colsum_row_blocks(G)
            out = torch.zeros(cols, device="cuda")
            for _ in range(3):
                N.colsum(x, out, two)
            torch.cuda.synchronize()
            # hipGraph replay (launch cost excluded, as in the graphed training step)
            gr = torch.cuda.CUDAGraph()
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                N.colsum(x, out, two)
            torch.cuda.current_stream().wait_stream(s)
            with torch.cuda.graph(gr):
                for _ in range(50):
                    N.colsum(x, out, two)
            gr.replay()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            gr.replay()
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) / 50 * 1e3
            o = torch.zeros(cols, device="cuda")
            N.colsum(x, o, two)
            err = ((o - ref).abs().max() / ref.abs().max()).item()
            print(json.dumps({"rows": rows, "cols": cols, "two_pass": two, "G": G,
                              "us": round(us, 2), "GBps": round(rows * cols * 2 / us / 1e3, 1),
                              "err": err}), flush=True)
N.set_colsum_row_blocks(0)

# LayerNorm backward on BERT-base shapes
for rows in (4096, 616, 16384):
    H = 768
    x = torch.randn(rows, H, device="cuda").to(torch.bfloat16)
    dy = torch.randn(rows, H, device="cuda").to(torch.bfloat16)
    g = torch.rand(H, device="cuda") + 0.5
    b = torch.zeros(H, device="cuda")
    from mipipe.ops import kernels as K
    y, mean, rstd, _ = K.layernorm_fwd(x, g, b, 1e-12, None)
    for _ in range(3):
        K.layernorm_bwd(dy, x, mean, rstd, g, None)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(50):
        K.layernorm_bwd(dy, x, mean, rstd, g, None)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / 50 * 1e3
    print(json.dumps({"op": "layernorm_bwd", "rows": rows, "H": H, "us": round(us, 2),
                      "GBps": round(rows * H * 2 * 3 / us / 1e3, 1)}), flush=True)
