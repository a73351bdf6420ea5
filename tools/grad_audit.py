"""Per-parameter gradient audit of a registry model on the GPU against the fp64 CPU path.

For each parameter (backward order) prints cos(gpu, fp64 truth) and cos(gpu run 1, gpu run 2)
(run-to-run agreement: fp32 atomics make bf16 gradients nondeterministic at the ulp level, a
race shows up as a large disagreement).  Flags the first parameter whose gradient goes bad.

python tools/grad_audit.py --arch mobilenet_v2 [--res 64] [--batch 16]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mipipe.models import create_model  # noqa: E402
from mipipe.optim import SGD  # noqa: E402
from mipipe.train.task import CrossEntropyLoss  # noqa: E402


def cos(a, b):
    a, b = a.flatten().double().cpu(), b.flatten().double().cpu()
    return float(a @ b / (a.norm() * b.norm() + 1e-30))


def make(arch, **kw):
    for extra in ({"dropout": 0.0, "dropout_aux": 0.0}, {"dropout": 0.0}, {}):
        try:
            m = create_model(arch, num_classes=16, **kw, **extra)
            break
        except TypeError:
            continue
    for mod in m.modules():
        if isinstance(mod, torch.nn.Dropout):
            mod.p = 0.0
    return m


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--arch", default="mobilenet_v2")
    ap.add_argument("--res", type=int, default=64)
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--flat", action="store_true", help="give the GPU model a flat optimizer "
                    "space (direct-to-bucket weight gradients)")
    ap.add_argument("--all", action="store_true", help="print every parameter")
    ap.add_argument("--stock", action="store_true", help="also audit stock torch (the same "
                    "module tree through reference_forward / ref_resnet, bf16 autocast)")
    a = ap.parse_args(argv)
    ce = CrossEntropyLoss()
    torch.manual_seed(0)
    truth = make(a.arch, compute_dtype=torch.float64).double()
    gm = make(a.arch).cuda()
    gm.load_state_dict(truth.state_dict())
    opt = SGD(gm.parameters(), 0.0) if a.flat else None
    x = torch.randn(a.batch, 3, a.res, a.res, dtype=torch.float64)
    y = torch.randint(0, 16, (a.batch,))
    lt = truth(x)
    ce(lt, y).backward()
    runs, logits = [], []
    for _ in range(2):
        if opt is not None:
            opt.zero_grad()
        else:
            for p in gm.parameters():
                p.grad = None
        out = gm(x.float().cuda())
        logits.append((out[0] if isinstance(out, tuple) else out).detach().float())
        ce(out, y.cuda()).backward()
        torch.cuda.synchronize()
        runs.append([p.grad.detach().clone() for p in gm.parameters()])
    lt0 = lt[0] if isinstance(lt, tuple) else lt
    print(f"train-mode logits: cos_truth {cos(logits[0], lt0):.5f} run2run {cos(logits[0], logits[1]):.6f}")
    names = [n for n, _ in gm.named_parameters()]
    tg = [p.grad for p in truth.parameters()]
    gmax = max(float(t.norm()) for t in tg)
    first_bad = None
    rows = []
    for i in reversed(range(len(names))):
        if float(tg[i].norm()) < 1e-4 * gmax:
            continue
        ct, cr = cos(runs[0][i], tg[i]), cos(runs[0][i], runs[1][i])
        bad = ct < 0.95 or cr < 0.99
        if bad and first_bad is None:
            first_bad = names[i]
        rows.append((names[i], ct, cr, bad))
    for n, ct, cr, bad in rows:
        if a.all or bad:
            print(f"{'BAD ' if bad else '    '}{n:55s} cos_truth {ct:.5f} run2run {cr:.5f}")
    whole = lambda gs: torch.cat([g.flatten().double().cpu() for g in gs])  # noqa: E731
    print(f"AUDIT {a.arch} res {a.res} b{a.batch} flat={a.flat}: whole-model cos_truth "
          f"{cos(whole(runs[0]), whole(tg)):.5f} run2run {cos(whole(runs[0]), whole(runs[1])):.5f}; "
          f"first bad (backward order): {first_bad}", flush=True)
    if a.stock:
        import copy
        if a.arch.startswith(("resnet", "resnext", "wide_resnet")):
            from mipipe.models.reference import ref_resnet
            sm = ref_resnet(a.arch, num_classes=16).cuda().to(memory_format=torch.channels_last)
            sm.load_state_dict(truth.state_dict())
            fwd = sm.forward
        else:
            sm = copy.deepcopy(truth).float().cuda()
            fwd = sm.reference_forward
        sr = []
        for _ in range(2):
            for p in sm.parameters():
                p.grad = None
            with torch.autocast("cuda", dtype=torch.bfloat16):
                out = fwd(x.float().cuda())
            ce(out, y.cuda()).backward()
            torch.cuda.synchronize()
            sr.append([p.grad.detach().clone() for p in sm.parameters()])
        print(f"STOCK {a.arch}: whole-model cos_truth {cos(whole(sr[0]), whole(tg)):.5f} run2run "
              f"{cos(whole(sr[0]), whole(sr[1])):.5f}", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
