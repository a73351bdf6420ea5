"""Does hipGraph replay run independent branches concurrently on this ROCm?  Two chains of
work that each underfill the GPU (small GEMMs) and a memory-bound chain, captured (a) on one
stream, (b) forked onto two streams with event joins; eager timings for both too."""
import time

import torch


def chains(a, b, x, y, n=20):
    for _ in range(n):
        torch.mm(a, b, out=x)          # compute chain (underfills: 1024x1024 bf16)
    for _ in range(n):
        y.mul_(1.0001)                  # memory chain (256 MB)


def run_serial(a, b, x, y):
    chains(a, b, x, y)


def run_forked(a, b, x, y, s2):
    cur = torch.cuda.current_stream()
    s2.wait_stream(cur)
    with torch.cuda.stream(s2):
        for _ in range(20):
            y.mul_(1.0001)
    for _ in range(20):
        torch.mm(a, b, out=x)
    cur.wait_stream(s2)


def timeit(fn, reps=20):
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps * 1e3


def main():
    dev = torch.device("cuda", 0)
    a = torch.randn(1024, 1024, device=dev, dtype=torch.bfloat16)
    b = torch.randn(1024, 1024, device=dev, dtype=torch.bfloat16)
    x = torch.empty(1024, 1024, device=dev, dtype=torch.bfloat16)
    y = torch.randn(64 << 20, device=dev)
    s2 = torch.cuda.Stream(dev)
    for _ in range(3):
        run_serial(a, b, x, y)
        run_forked(a, b, x, y, s2)
    print(f"eager serial {timeit(lambda: run_serial(a, b, x, y)):.3f} ms")
    print(f"eager forked {timeit(lambda: run_forked(a, b, x, y, s2)):.3f} ms")
    cs = torch.cuda.Stream(dev)
    g1, g2 = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
    with torch.cuda.graph(g1, stream=cs):
        run_serial(a, b, x, y)
    with torch.cuda.graph(g2, stream=cs):
        run_forked(a, b, x, y, s2)
    print(f"graph serial {timeit(g1.replay):.3f} ms")
    print(f"graph forked {timeit(g2.replay):.3f} ms")
    # each chain alone, for reference
    g3 = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g3, stream=cs):
        for _ in range(20):
            torch.mm(a, b, out=x)
    g4 = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g4, stream=cs):
        for _ in range(20):
            y.mul_(1.0001)
    print(f"graph mm chain alone {timeit(g3.replay):.3f} ms, mul chain alone {timeit(g4.replay):.3f} ms")


if __name__ == "__main__":
    main()
