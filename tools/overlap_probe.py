#!/usr/bin/env python3
"""Does a collective on the process group's stream run CONCURRENTLY with compute, eagerly and
when replayed from a captured hipGraph?  (VERDICT r2 Missing #1: the rocprofv3 trace showed 0.0 %
overlap; this measures it by wall clock, which does not depend on the tracer.)

World 1 over RCCL (``nccl`` backend): the all-reduce is RCCL's one-rank kernel (reads and
writes the whole buffer: a real HBM-bound kernel on the PG stream).  Compute = a chain of bf16
matmuls on the current stream.  For each mode we time
    A  = compute alone,  B = collective alone,  AB = both issued together
and report overlap = (A + B - AB) / min(A, B)  (1.0 = fully hidden, 0.0 = serialised).
Also a control with no RCCL: a side-stream copy kernel vs the same matmuls.

usage: python tools/overlap_probe.py [--mb 512] [--gemms 12]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, reps=9):
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    ts.sort()
    return ts[len(ts) // 2] * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mb", type=int, default=512)
    ap.add_argument("--gemms", type=int, default=12)
    ap.add_argument("--n", type=int, default=8192)
    ap.add_argument("--prio", type=int, default=0, help="side-stream priority (-1 = high)")
    ap.add_argument("--compute", default="conv", choices=["conv", "matmul"],
                    help="conv = mipipe 3x3 conv forwards (many workgroups, like a training "
                         "step); matmul = torch/hipBLASLt GEMMs")
    a = ap.parse_args()
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29533")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    n = a.n
    xa = torch.randn(n, n, device=dev, dtype=torch.bfloat16)
    xb = torch.randn(n, n, device=dev, dtype=torch.bfloat16)
    out = torch.empty(n, n, device=dev, dtype=torch.bfloat16)
    buf = torch.randn(a.mb * 2 ** 20 // 4, device=dev)
    src = torch.randn_like(buf)
    side = torch.cuda.Stream(dev, priority=a.prio)

    from mipipe.ops import kernels as K
    cx = torch.randn(256, 28, 28, 128, device=dev, dtype=torch.bfloat16)
    cw = torch.randn(128, 3, 3, 128, device=dev, dtype=torch.bfloat16) * 0.05

    def compute():
        for _ in range(a.gemms):
            if a.compute == "matmul":
                torch.matmul(xa, xb, out=out)
            else:
                K.conv_fwd(cx, cw, 1, 1)

    def comm():
        dist.all_reduce(buf, op=dist.ReduceOp.AVG, async_op=True).wait()

    def both():
        w = dist.all_reduce(buf, op=dist.ReduceOp.AVG, async_op=True)
        compute()
        w.wait()

    def copy_side():
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            buf.copy_(src)
        torch.cuda.current_stream().wait_stream(side)

    def both_copy():
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            buf.copy_(src)
        compute()
        torch.cuda.current_stream().wait_stream(side)

    res = {}
    for _ in range(2):
        compute(); comm(); both(); copy_side(); both_copy()
    for name, (fa, fb, fab) in {"eager_rccl": (compute, comm, both),
                                "eager_copy": (compute, copy_side, both_copy)}.items():
        A, B, AB = timeit(fa), timeit(fb), timeit(fab)
        res[name] = {"A_ms": round(A, 3), "B_ms": round(B, 3), "AB_ms": round(AB, 3),
                     "overlap": round((A + B - AB) / min(A, B), 3)}
        print(json.dumps({name: res[name]}), flush=True)

    # the same three workloads captured into hipGraphs and replayed
    graphs = {}
    for key, fn in (("A", compute), ("B", comm), ("AB", both), ("Bc", copy_side), ("ABc", both_copy)):
        s = torch.cuda.Stream(dev)
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            fn()
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, capture_error_mode="thread_local"):
            fn()
        graphs[key] = g
    torch.cuda.synchronize()
    for name, (ka, kb, kab) in {"graph_rccl": ("A", "B", "AB"), "graph_copy": ("A", "Bc", "ABc")}.items():
        A = timeit(graphs[ka].replay)
        B = timeit(graphs[kb].replay)
        AB = timeit(graphs[kab].replay)
        res[name] = {"A_ms": round(A, 3), "B_ms": round(B, 3), "AB_ms": round(AB, 3),
                     "overlap": round((A + B - AB) / min(A, B), 3)}
        print(json.dumps({name: res[name]}), flush=True)
    print(json.dumps({"overlap_probe": res, "mb": a.mb, "gemms": a.gemms, "n": n,
                      "env": {k: os.environ.get(k) for k in ("GPU_MAX_HW_QUEUES", "HIP_FORCE_QUEUE_PROFILING",
                                                              "DEBUG_HIP_FORCE_GRAPH_QUEUES", "TORCH_NCCL_HIGH_PRIORITY")},
                      "prio": a.prio, "compute": a.compute}))
    dist.destroy_process_group()


if __name__ == "__main__":
    sys.exit(main())
