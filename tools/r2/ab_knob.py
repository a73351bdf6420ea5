"""A/B a runtime kernel knob on the ResNet-50 b256 training step in ONE process (interleaved
rounds, guide rule 24); eager steps so the knob reaches every launch: python tools/r2/ab_knob.py <setter> <valueA> <valueB> [rounds]
e.g. set_colsum_row_blocks 0 64, or py:mipipe.ops.functional._RELU_BITMASK 0 1"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch

import bench
from mipipe.ops import tuning
from mipipe.ops._native import native


def main():
    setter, va, vb = sys.argv[1], float(sys.argv[2]), float(sys.argv[3])
    rounds = int(sys.argv[4]) if len(sys.argv) > 4 else 4
    a = argparse.Namespace(model="resnet50", batch=256, res=224, classes=1000, impl="mipipe",
                           graph="off", device="cuda", dtype="bf16", distributed=False,
                           bucket_cap_mb=32.0, force_reduce=False, warmup=3, seq=128)
    torch.cuda.set_device(0)
    tuning.set_benchmark(True, verbose=False)
    step, model, batches = bench.build_cnn(a, 1, 0, torch.device("cuda", 0), 0)
    model.train()
    if setter.startswith("py:"):  # a module attribute, e.g. py:mipipe.ops.functional._RELU_BITMASK
        import importlib
        mod, attr = setter[3:].rsplit(".", 1)
        m = importlib.import_module(mod)

        def fn(v):
            setattr(m, attr, type(getattr(m, attr))(v))
    else:
        fn = getattr(native(), setter)
    res = {va: [], vb: []}
    for r in range(rounds):
        for v in (va, vb) if r % 2 == 0 else (vb, va):
            fn(v)
            for i in range(3):
                step(*batches[i % 2])
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for i in range(10):
                step(*batches[i % 2])
            torch.cuda.synchronize()
            res[v].append((time.perf_counter() - t0) / 10 * 1e3)
    for v, ts in res.items():
        print(f"{setter}({v:g}): ms/step " + " ".join(f"{t:.3f}" for t in ts) +
              f"  min {min(ts):.3f}", flush=True)


if __name__ == "__main__":
    main()
