"""Rehearse the multi-GPU DDP path on a ONE-GPU box: 2 ranks share cuda:0 over gloo (RCCL
refuses two ranks on one device), exercising the real flat-bucket hooks, direct-to-bucket
weight gradients, fused BN paths and the buffer broadcast with GPU tensors.

Checks after one backward: (1) the all-reduced gradient equals the average of the per-rank
gradients computed by two independent single-process replicas (cosine per parameter, compared
with the replicas' own run-to-run agreement: fp32 atomics make bf16 training nondeterministic
at the ulp level); (2) after 3 optimizer steps the parameters are bit-identical across ranks.

torchrun --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 tools/ddp_gpu_check.py
"""
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mipipe.models import create_model  # noqa: E402
from mipipe.optim import SGD  # noqa: E402
from mipipe.ops.functional import cross_entropy  # noqa: E402
from mipipe.parallel import DistributedDataParallel  # noqa: E402


def cos(a, b):
    a, b = a.flatten().double(), b.flatten().double()
    return float(a @ b / (a.norm() * b.norm() + 1e-30))


def main():
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    base = create_model("resnet18", num_classes=16).to(dev)
    refs = []
    for _ in range(2):
        r = create_model("resnet18", num_classes=16).to(dev)
        r.load_state_dict(base.state_dict())
        refs.append((r, SGD(r.parameters(), 0.05, momentum=0.9, weight_decay=1e-4)))
    model = DistributedDataParallel(base, device_ids=[0], bucket_cap_mb=4, first_bucket_mb=0.5,
                                    check_collectives=True, check_every=1)
    opt = SGD(model.parameters(), 0.05, momentum=0.9, weight_decay=1e-4)
    g = torch.Generator(device=dev)
    g.manual_seed(123)
    B = 16
    for step in range(3):
        xs = torch.randn(world * B, 3, 32, 32, device=dev, generator=g)
        ys = torch.randint(0, 16, (world * B,), device=dev, generator=g)
        x, y = xs[rank * B:(rank + 1) * B], ys[rank * B:(rank + 1) * B]
        opt.zero_grad()
        cross_entropy(model(x), y).backward()
        if step == 0:
            for r, ro in refs:  # replicas: average of the per-rank gradients
                ro.zero_grad()
                for k in range(world):
                    (cross_entropy(r(xs[k * B:(k + 1) * B]), ys[k * B:(k + 1) * B]) / world).backward()
            torch.cuda.synchronize()
            worst = (1.0, "")
            for (n, p), (_, q1), (_, q2) in zip(base.named_parameters(), refs[0][0].named_parameters(),
                                                refs[1][0].named_parameters()):
                c_ddp, c_self = cos(p.grad, q1.grad), cos(q2.grad, q1.grad)
                if c_ddp - c_self < worst[0] - 1.0 or worst[1] == "":
                    worst = (1.0 + c_ddp - c_self, n)
                assert c_ddp > min(0.999, c_self - 0.01), (n, c_ddp, c_self)
            if rank == 0:
                print(f"step0 gradient check OK (worst cos gap {1.0 - worst[0]:.2e} at {worst[1]})",
                      flush=True)
        opt.step()
    torch.cuda.synchronize()
    flat = model.space.flat.detach().clone()
    gathered = [torch.empty_like(flat) for _ in range(world)]
    dist.all_gather(gathered, flat)
    assert all(torch.equal(gathered[0], t) for t in gathered), "ranks diverged"
    if rank == 0:
        print(f"DDP gpu check OK: world={world}, parameters bit-identical across ranks after 3 "
              f"steps, collectives={model._clog.count}", flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
