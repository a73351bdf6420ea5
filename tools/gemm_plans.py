#!/usr/bin/env python3
"""Every GEMM plan (MFMA tile x split-K x workspace split, and the library plan) on the GEMM
shapes of one BERT-base 32x128 step, timed by hipGraph replay (launch cost excluded, as in the
graphed training step).  Prints one JSON line per shape: the best MFMA plan, the library plan,
their ratio, and the five fastest plans — the evidence for (or against) keeping a library plan.

python tools/gemm_plans.py [--reps 20] [--shapes KEY ...]
KEY = "M,N,K,a_kc,b_kc,mode" as in the tuning table (mode 0 bf16 out, 2 fp32 accumulate,
3 bf16 out + addend).
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
    "4096,2304,768,1,1,0", "4096,768,768,1,1,0", "4096,3072,768,1,1,0", "4096,768,3072,1,1,0",
    "640,768,768,1,1,0", "640,30528,768,1,1,0",
    "4096,768,2304,1,0,3", "4096,768,768,1,0,0", "4096,3072,768,1,0,0", "4096,768,3072,1,0,3",
    "640,768,30528,1,0,0", "640,768,768,1,0,0",
    "2304,768,4096,0,0,2", "768,768,4096,0,0,2", "3072,768,4096,0,0,2", "768,3072,4096,0,0,2",
    "30528,768,640,0,0,2", "768,768,640,0,0,2",
]
LIB, SPLIT, WS = 4096, 16, 1024


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


def plans(C, mode, K):
    tiles = list(range(C.CONV_TILE_CONFIGS))
    out = []
    if mode == 2:
        for t in tiles:
            for sp in (1, 2, 4):
                out.append(t + SPLIT * sp)
            if K >= 1024:
                for sp in (2, 4, 8):
                    out.append((t + SPLIT * sp) | WS)
    else:
        out += tiles
        if mode == 0 and K >= 4096:
            for t in tiles:
                for sp in (2, 4, 8):
                    out.append(t + SPLIT * sp)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--shapes", nargs="*", default=BERT_32x128)
    a = ap.parse_args()
    C = native()
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    for key in a.shapes:
        M, N, K, akc, bkc, mode = (int(v) for v in key.split(","))
        A = (torch.randn(M, K, device=dev) if akc else torch.randn(K, M, device=dev)).bfloat16()
        B = (torch.randn(N, K, device=dev) if bkc else torch.randn(K, N, device=dev)).bfloat16() * 0.05
        add = torch.randn(M, N, device=dev).bfloat16() if mode == 3 else None
        acc = torch.zeros(M, N, device=dev) if mode == 2 else None

        def run(p):
            if mode == 2:
                return C.gemm(A, B, not akc, bool(bkc), None, "none", torch.float32, acc, 1.0, p)
            return C.gemm(A, B, not akc, bool(bkc), None, "none", torch.bfloat16, None, 0.0, p,
                          add)

        res = {}
        for p in plans(C, mode, K) + [LIB]:
            try:
                res[p] = t_graph(lambda: run(p), a.reps)
            except RuntimeError as e:  # a plan a shape cannot take
                res[p] = float("inf")
                print(f"# {key} plan {p}: {str(e)[:80]}", file=sys.stderr)
        mf = {p: v for p, v in res.items() if p != LIB}
        best = min(mf, key=mf.get)
        fl = 2.0 * M * N * K
        print(json.dumps({"shape": key, "best_mfma_plan": best, "best_mfma_us": round(mf[best], 2),
                          "lib_us": round(res[LIB], 2), "mfma_over_lib": round(mf[best] / res[LIB], 3),
                          "best_tflops": round(fl / mf[best] / 1e6, 1),
                          "top5": {str(p): round(v, 2) for p, v in sorted(mf.items(), key=lambda x: x[1])[:5]}}),
              flush=True)


if __name__ == "__main__":
    main()
