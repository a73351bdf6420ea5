#!/usr/bin/env python3
"""Every GEMM plan (MFMA tile x split-K x workspace split) on the GEMM shapes of one BERT-base
32x128 step, timed by hipGraph replay (launch cost excluded, as in the graphed training step),
against the same product through hipBLASLt (torch.mm / addmm — a comparator only: no library
GEMM runs in the training step).  Prints one JSON line per shape: the best MFMA plan, the
library time, their ratio, and the five fastest plans.

python tools/gemm_plans.py [--reps 20] [--shapes KEY ...]
KEY = "M,N,K,a_kc,b_kc,mode[,bias]" as in the tuning table (mode 0 bf16 out, 2 fp32 accumulate,
3 bf16 out + addend; bias 1: the call carries a bias, as BERT's forward projections do).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mipipe.ops._native import native  # noqa: E402

BERT_32x128 = [
    "4096,2304,768,1,1,0,1", "4096,768,768,1,1,0,1", "4096,3072,768,1,1,0,1",
    "4096,768,3072,1,1,0,1", "640,768,768,1,1,0,1", "640,30528,768,1,1,0,1",
    "4096,768,2304,1,0,3", "4096,768,768,1,0,0", "4096,3072,768,1,0,0", "4096,768,3072,1,0,3",
    "640,768,30528,1,0,0", "640,768,768,1,0,0",
    "2304,768,4096,0,0,2", "768,768,4096,0,0,2", "3072,768,4096,0,0,2", "768,3072,4096,0,0,2",
    "30528,768,640,0,0,2", "768,768,640,0,0,2",
]
SPLIT, WS = 16, 1024


def t_graph(fn, reps):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr):
        for _ in range(reps):
            fn()
    gr.replay()
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(3):
        t = time.perf_counter()
        gr.replay()
        torch.cuda.synchronize()
        best = min(best, (time.perf_counter() - t) / reps * 1e6)
    return best


def plans(C, mode, K, all_ws=False):
    """``all_ws``: workspace split-K plans at every K (the training-step tuner offers them from
    K >= 1024 / 2048 only)."""
    if all_ws:
        K = 1 << 30
    tiles = list(range(C.CONV_TILE_CONFIGS))
    out = []
    if mode == 2:
        for t in tiles:
            for sp in (1, 2, 4):
                out.append(t + SPLIT * sp)
            if K >= 1024:
                for sp in (2, 3, 4, 6, 8):
                    out.append((t + SPLIT * sp) | WS)
    else:
        out += tiles
        if K >= 2048:  # bf16 output with a bias (mode 0) or an addend (mode 3)
            for t in tiles:
                for sp in (2, 3, 4, 6, 8):
                    out.append((t + SPLIT * sp) | WS)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--shapes", nargs="*", default=BERT_32x128)
    ap.add_argument("--all-ws", action="store_true", help="workspace split plans at every K")
    a = ap.parse_args()
    C = native()
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    for key in a.shapes:
        f = [int(v) for v in key.split(",")]
        M, N, K, akc, bkc, mode = f[:6]
        has_bias = len(f) > 6 and f[6] == 1
        A = (torch.randn(M, K, device=dev) if akc else torch.randn(K, M, device=dev)).bfloat16()
        B = (torch.randn(N, K, device=dev) if bkc else torch.randn(K, N, device=dev)).bfloat16() * 0.05
        add = torch.randn(M, N, device=dev).bfloat16() if mode == 3 else None
        acc = torch.zeros(M, N, device=dev) if mode == 2 else None
        bias = torch.randn(N, device=dev) if has_bias else None

        def run(p):
            if mode == 2:
                return C.gemm(A, B, not akc, bool(bkc), None, "none", torch.float32, acc, 1.0, p)
            return C.gemm(A, B, not akc, bool(bkc), bias, "none", torch.bfloat16, None, 0.0, p,
                          add)

        At = A if akc else A.t()
        Bt = B.t() if bkc else B

        def lib():
            if mode == 2:
                return torch.addmm(acc, At, Bt, out_dtype=torch.float32, out=acc)
            if mode == 3:
                return torch.addmm(add, At, Bt)
            if bias is not None:
                return torch.addmm(bias.bfloat16(), At, Bt)
            return torch.mm(At, Bt)

        res = {}
        for p in plans(C, mode, K, a.all_ws):
            res[p] = t_graph(lambda: run(p), a.reps)
        t_lib = t_graph(lib, a.reps)
        best = min(res, key=res.get)
        fl = 2.0 * M * N * K
        print(json.dumps({"shape": key, "best_mfma_plan": best, "best_mfma_us": round(res[best], 2),
                          "lib_us": round(t_lib, 2), "mfma_over_lib": round(res[best] / t_lib, 3),
                          "best_tflops": round(fl / res[best] / 1e6, 1),
                          "top5": {str(p): round(v, 2) for p, v in sorted(res.items(), key=lambda x: x[1])[:5]}}),
              flush=True)


if __name__ == "__main__":
    main()
