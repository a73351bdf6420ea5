"""mipipe's MFMA GEMM (tuned per shape) vs torch.matmul (hipBLASLt) on the BERT-base 32x128
shapes: forward (x @ W^T), data-grad (dy @ W), weight-grad (dy^T @ x, fp32 out)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from mipipe.ops import kernels as K
from mipipe.ops._native import native


def t_ms(fn, reps=50):
    """Device time per call: ``reps`` calls captured in one hipGraph and replayed (host launch
    cost excluded, as in the graphed training step)."""
    for _ in range(5):
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
        best = min(best, (time.perf_counter() - t) / reps * 1e3)
    return best


def main():
    dev = torch.device("cuda", 0)
    native().set_benchmark(True, False, 5)
    M = 4096
    rows = []
    for (N, Kd, name) in [(2304, 768, "qkv"), (768, 768, "proj"), (3072, 768, "ffn1"),
                          (768, 3072, "ffn2"), (30528, 768, "mlm")]:
        x = torch.randn(M, Kd, device=dev, dtype=torch.bfloat16)
        w = torch.randn(N, Kd, device=dev, dtype=torch.bfloat16) * 0.02
        dy = torch.randn(M, N, device=dev, dtype=torch.bfloat16)
        g = torch.zeros(N, Kd, device=dev)
        fl = 2.0 * M * N * Kd
        for kind, f_mi, f_bl in [
            ("fwd", lambda: K.gemm(x, w, False, True, None, "none", torch.bfloat16),
             lambda: torch.mm(x, w.t())),
            ("dgrad", lambda: K.gemm(dy, w, False, False, None, "none", torch.bfloat16),
             lambda: torch.mm(dy, w)),
            ("wgrad", lambda: K.gemm(dy, x, True, False, None, "none", torch.float32, g, 1.0),
             lambda: torch.mm(dy.t(), x)),
            # the training step's contract: fp32 accumulate into the flat gradient (beta = 1)
            ("wgrad32", lambda: K.gemm(dy, x, True, False, None, "none", torch.float32, g, 1.0),
             lambda: torch.addmm(g, dy.t(), x, out_dtype=torch.float32, out=g)),
        ]:
            a, b = t_ms(f_mi), t_ms(f_bl)
            rows.append((name, kind, a, b))
            print(f"{name:5s} {kind:5s} M={M} N={N} K={Kd}: mipipe {a*1e3:7.1f} us ({fl/a/1e9:6.0f} TF)"
                  f"  hipBLASLt {b*1e3:7.1f} us ({fl/b/1e9:6.0f} TF)", flush=True)
    lib = sorted(k for k, v in native().tune_table().items() if k.startswith("gemm") and v >= 0 and v & 4096)
    print("shapes the tuner gave to the library plan:", lib)
    print(f"sum: mipipe {sum(r[2] for r in rows)*1e3:.0f} us, hipBLASLt {sum(r[3] for r in rows)*1e3:.0f} us")


if __name__ == "__main__":
    main()
