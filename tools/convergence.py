#!/usr/bin/env python3
"""Convergence parity: the reference's recipe (SGD lr 0.1, momentum 0.9, wd 1e-4, CE loss —
/root/reference/task.py:210-214, 303-312) trained on the SAME learnable synthetic batches from
the SAME initial weights by (a) mipipe's kernels and (b) stock PyTorch-ROCm (MIOpen convs, ATen
BN / CE, torch.optim.SGD; bf16 autocast when --dtype bf16).  Prints a JSON line per logging
interval (mean loss over the interval, both implementations) and a final summary with held-out
accuracy.  Loss curves of two correct implementations agree to within run-to-run noise; a
kernel bug shows up as a systematic gap.

python tools/convergence.py --arch resnet18 --res 32 --batch 256 --steps 400 --dtype bf16
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--arch", default="resnet18")
    ap.add_argument("--res", type=int, default=32)
    ap.add_argument("--classes", type=int, default=10)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--steps", type=int, default=400)
    ap.add_argument("--lr", type=float, default=0.1)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--log-every", type=int, default=20)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--eval-batches", type=int, default=8)
    ap.add_argument("--impls", default="mipipe,stock")
    a = ap.parse_args()
    dev = torch.device("cuda")
    from mipipe.data.synthetic import synthetic_batch
    from mipipe.models import create_model
    from mipipe.models.reference import ref_resnet
    from mipipe.optim import SGD
    from mipipe.train.task import CrossEntropyLoss
    from mipipe.ops import tuning
    tuning.set_benchmark(True)

    torch.manual_seed(a.seed)
    init = create_model(a.arch, num_classes=a.classes).state_dict()
    shape = (3, a.res, a.res)
    bf16 = a.dtype == "bf16"

    def batch(step, offset=0):
        idx = torch.arange(step * a.batch, (step + 1) * a.batch, device=dev) + offset
        return synthetic_batch(idx, shape, a.classes, seed=a.seed)

    impls = a.impls.split(",")
    models, opts, steps_fn = {}, {}, {}
    if "mipipe" in impls:
        m = create_model(a.arch, num_classes=a.classes)
        m.load_state_dict(init)
        m = m.to(dev)
        m.compute_dtype = torch.bfloat16 if bf16 else torch.float32
        opt = SGD(m.parameters(), a.lr, momentum=0.9, weight_decay=1e-4,
                  shadow_dtype="auto" if bf16 else None)
        crit = CrossEntropyLoss()

        def step_m(x, y, m=m, opt=opt, crit=crit):
            opt.zero_grad()
            loss = crit(m(x), y)
            loss.backward()
            opt.step()
            return loss.detach()
        models["mipipe"], steps_fn["mipipe"] = m, step_m
    if "stock" in impls:
        r = ref_resnet(a.arch, num_classes=a.classes)
        r.load_state_dict(init)
        r = r.to(dev).to(memory_format=torch.channels_last)
        ropt = torch.optim.SGD(r.parameters(), a.lr, momentum=0.9, weight_decay=1e-4)
        torch.backends.cudnn.benchmark = True

        def step_s(x, y, r=r, ropt=ropt):
            ropt.zero_grad(set_to_none=True)
            with torch.autocast("cuda", dtype=torch.bfloat16, enabled=bf16):
                loss = torch.nn.functional.cross_entropy(
                    r(x.contiguous(memory_format=torch.channels_last)), y)
            loss.backward()
            ropt.step()
            return loss.detach().float()
        models["stock"], steps_fn["stock"] = r, step_s

    hist = {k: [] for k in steps_fn}
    t0 = time.time()
    for s in range(a.steps):
        x, y = batch(s)
        for k, fn in steps_fn.items():
            hist[k].append(fn(x, y))
        if (s + 1) % a.log_every == 0:
            rec = {"step": s + 1, "t": round(time.time() - t0, 1)}
            for k in hist:
                rec[k] = round(float(torch.stack(hist[k][-a.log_every:]).mean()), 4)
            print(json.dumps(rec), flush=True)

    @torch.no_grad()
    def accuracy(k):
        m = models[k]
        m.eval()
        correct = 0
        for b in range(a.eval_batches):
            x, y = batch(b, offset=10_000_000)  # held-out indices
            with torch.autocast("cuda", dtype=torch.bfloat16, enabled=bf16 and k == "stock"):
                out = m(x if k == "mipipe" else x.contiguous(memory_format=torch.channels_last))
            correct += int((out.float().argmax(1) == y).sum())
        m.train()
        return correct / (a.eval_batches * a.batch)

    summary = {"summary": True, "arch": a.arch, "res": a.res, "batch": a.batch,
               "steps": a.steps, "lr": a.lr, "dtype": a.dtype}
    for k in hist:
        L = torch.stack(hist[k]).float().cpu()
        summary[k] = {"loss_first20": round(float(L[:20].mean()), 4),
                      "loss_last50": round(float(L[-50:].mean()), 4),
                      "loss_max": round(float(L.max()), 3),
                      "step_of_max": int(L.argmax()) + 1,
                      "heldout_acc": round(accuracy(k), 4)}
    print(json.dumps(summary), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
