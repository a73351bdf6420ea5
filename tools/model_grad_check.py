#!/usr/bin/env python3
"""Per-parameter gradient error of one mipipe training step on the GPU vs the same module tree
evaluated in float64 on the CPU (plain torch ops).  Used to validate the fp32 path and to
localise a wrong gradient to a layer.

usage: python tools/model_grad_check.py --arch resnet18 --res 32 --batch 64 --dtype fp32
"""
from __future__ import annotations

import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).abs().max() / (b.abs().max() + 1e-30)).item()


def rel2(a, b):
    """relative L2 error (robust to the rare ReLU / max-pool decision that flips between two
    precisions when a pre-activation lies within rounding of zero)"""
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).norm() / (b.norm() + 1e-30)).item()


def stock_errors(a, x, y):
    """The same check for stock PyTorch-ROCm on the GPU (MIOpen / hipBLASLt, fp32 or bf16
    autocast) vs float64 on the CPU: the calibration for what "fp32" means on this GPU."""
    from mipipe.models.reference import ref_resnet
    torch.manual_seed(0)
    m = ref_resnet(a.arch, num_classes=a.classes)
    r = ref_resnet(a.arch, num_classes=a.classes).double()
    r.load_state_dict(m.state_dict())
    m = m.cuda()
    with torch.autocast("cuda", dtype=torch.bfloat16, enabled=a.dtype == "bf16"):
        out = m(x.cuda())
    torch.nn.functional.cross_entropy(out.float(), y.cuda()).backward()
    torch.nn.functional.cross_entropy(r(x.double()), y).backward()
    pr = dict(r.named_parameters())
    e2 = sorted(rel2(p.grad, pr[n].grad) for n, p in m.named_parameters())
    return e2[len(e2) // 2], e2[-1]


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--arch", default="resnet18")
    ap.add_argument("--res", type=int, default=32)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--classes", type=int, default=10)
    ap.add_argument("--dtype", default="fp32", choices=["fp32", "bf16"])
    ap.add_argument("--top", type=int, default=12)
    a = ap.parse_args()
    from mipipe.models import create_model
    from mipipe.train.task import CrossEntropyLoss
    torch.manual_seed(0)
    m = create_model(a.arch, num_classes=a.classes)
    ref = create_model(a.arch, num_classes=a.classes, compute_dtype=torch.float64).double()
    ref.load_state_dict(m.state_dict())
    m = m.cuda()
    m.compute_dtype = torch.float32 if a.dtype == "fp32" else torch.bfloat16
    x = torch.randn(a.batch, 3, a.res, a.res)
    y = torch.randint(0, a.classes, (a.batch,))
    out = m(x.cuda())
    loss = CrossEntropyLoss()(out, y.cuda())
    loss.backward()
    out_r = ref(x.double())
    loss_r = torch.nn.functional.cross_entropy(out_r, y)
    loss_r.backward()
    print(f"{a.arch} {a.dtype} batch {a.batch} res {a.res}: logits rel err {rel(out, out_r):.3e}, "
          f"loss {loss.item():.6f} vs {loss_r.item():.6f}")
    pr = dict(ref.named_parameters())
    errs = sorted(((rel2(p.grad, pr[n].grad), rel(p.grad, pr[n].grad), n)
                   for n, p in m.named_parameters()), reverse=True)
    print("  rel L2 err   max-abs rel err   parameter")
    for e2, e, n in errs[: a.top]:
        print(f"  {e2:10.3e}  {e:10.3e}  {n}")
    print(f"  mipipe {a.dtype}: median rel-L2 grad err {errs[len(errs) // 2][0]:.3e}, "
          f"max {errs[0][0]:.3e} over {len(errs)} tensors")
    if a.arch.startswith("resnet"):
        med, mx = stock_errors(a, x, y)
        print(f"  stock torch {a.dtype}: median rel-L2 grad err {med:.3e}, max {mx:.3e}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
