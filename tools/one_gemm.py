"""Run one GEMM shape with one plan N times for PMC profiling (tools/r4/pmc_gemm.sh).
usage: one_gemm.py M,N,K,a_kc,b_kc,mode PLAN   (keys as in tools/gemm_plans.py)"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from mipipe.ops._native import native  # noqa: E402

C = native()
M, N, K, akc, bkc, mode = [int(v) for v in sys.argv[1].split(",")[:6]]
plan = int(sys.argv[2]) if len(sys.argv) > 2 else -1
A = (torch.randn(M, K, device="cuda") if akc else torch.randn(K, M, device="cuda")).bfloat16()
B = (torch.randn(N, K, device="cuda") if bkc else torch.randn(K, N, device="cuda")).bfloat16() * 0.05
acc = torch.zeros(M, N, device="cuda") if mode == 2 else None
for _ in range(20):
    if mode == 2:
        C.gemm(A, B, not akc, bool(bkc), None, "none", torch.float32, acc, 1.0, plan)
    else:
        C.gemm(A, B, not akc, bool(bkc), None, "none", torch.bfloat16, None, 0.0, plan)
torch.cuda.synchronize()
print("done", sys.argv[1], plan)
