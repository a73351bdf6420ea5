"""Stock PyTorch-ROCm comparator ("the bar is a measured comparator").

Runs the task.py-style training step (forward, CrossEntropy, backward, SGD-momentum
step) with *stock* torch ops only: MIOpen convs/BN, hipBLASLt GEMMs, ATen elementwise,
torch DDP over RCCL when launched with torchrun.  Synthetic data, random init.

Usage (1 GPU):  python tools/stock_baseline.py --model resnet50 --batch 256 --dtype bf16
Prints one JSON line per config.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch
import torch.nn as nn

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mipipe.models.reference import ref_resnet, RefMnistCNN  # noqa: E402


def run(model_name: str, batch: int, res: int, dtype: str, steps: int, warmup: int,
        channels_last: bool) -> dict:
    dist = int(os.environ.get("WORLD_SIZE", "1")) > 1
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dev = torch.device("cuda", local_rank)
    torch.cuda.set_device(dev)
    if dist and not torch.distributed.is_initialized():
        torch.distributed.init_process_group("nccl")
    torch.manual_seed(0)
    if model_name == "mnist_cnn":
        model = RefMnistCNN()
        x = torch.randn(batch, 1, 28, 28, device=dev)
        y = torch.randint(0, 10, (batch,), device=dev)
    else:
        model = ref_resnet(model_name)
        x = torch.randn(batch, 3, res, res, device=dev)
        y = torch.randint(0, 1000, (batch,), device=dev)
    model = model.to(dev)
    if channels_last:
        model = model.to(memory_format=torch.channels_last)
        x = x.contiguous(memory_format=torch.channels_last)
    if dist:
        model = torch.nn.parallel.DistributedDataParallel(model, device_ids=[local_rank])
    crit = nn.CrossEntropyLoss()
    opt = torch.optim.SGD(model.parameters(), 0.1, momentum=0.9, weight_decay=1e-4)
    torch.backends.cudnn.benchmark = True
    amp = dtype == "bf16"

    def step():
        opt.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=amp):
            out = model(x)
            loss = crit(out, y)
        loss.backward()
        opt.step()
        return loss

    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    if dist:
        torch.distributed.barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        loss = step()
    torch.cuda.synchronize()
    if dist:
        torch.distributed.barrier()
    dt = time.perf_counter() - t0
    world = torch.distributed.get_world_size() if dist else 1
    return {"impl": "stock-torch", "model": model_name, "batch_per_gpu": batch, "res": res,
            "dtype": dtype, "channels_last": channels_last, "n_gpus": world,
            "ms_per_step": dt / steps * 1e3, "samples_per_s": batch * world * steps / dt,
            "loss": float(loss)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--res", type=int, default=224)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--no-channels-last", action="store_true")
    a = ap.parse_args()
    r = run(a.model, a.batch, a.res, a.dtype, a.steps, a.warmup, not a.no_channels_last)
    if int(os.environ.get("RANK", "0")) == 0:
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
