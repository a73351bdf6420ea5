"""Rehearse the multi-GPU DDP path on a ONE-GPU box: 2 ranks share cuda:0 over gloo (RCCL
refuses two ranks on one device), exercising the real flat-bucket hooks, direct-to-bucket
weight gradients, fused BN paths and the buffer broadcast with GPU tensors.

Checks on the first backward, with ``dist.all_reduce`` intercepted (each bucket's collective is
deferred to its ``wait()``): (1) no gradient is written into a bucket after the bucket's
all-reduce was launched (launch-time snapshot == end-of-backward contents: the "ready before
written" race of direct-to-bucket kernels), (2) the reduced bucket equals the sum/average of
the ranks' local buckets.  Then, informative unless the model is well conditioned: the
all-reduced gradient is as close to the fp64 CPU ground truth as a single-process replica is
(random-init BN nets at 16 samples/rank are chaotic in bf16: stock torch autocast lands just as
far from fp64, see tools/grad_audit.py).  Finally (3) after 3 optimizer steps the parameters are
bit-identical across ranks.

torchrun --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 tools/ddp_gpu_check.py
    [--arch resnet18] [--res 32]      (any registry arch; dropout is disabled for the check)
"""
import argparse
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mipipe.models import create_model  # noqa: E402
from mipipe.optim import SGD  # noqa: E402
from mipipe.train.task import CrossEntropyLoss  # noqa: E402  (sums aux-head losses too)

cross_entropy = CrossEntropyLoss()
from mipipe.parallel import DistributedDataParallel  # noqa: E402


def cos(a, b):
    a, b = a.flatten().double().cpu(), b.flatten().double().cpu()
    return float(a @ b / (a.norm() * b.norm() + 1e-30))


class _DeferredAllReduce:
    """Work handle: snapshot the bucket at launch, run the real collective at wait()."""
    real = dist.all_reduce
    log = []

    def __init__(self, t, op, group):
        self.t, self.op, self.group = t, op, group
        self.snap = t.detach().clone()

    def wait(self):
        late = not torch.equal(self.t, self.snap)
        local = self.t.detach().clone()
        _DeferredAllReduce.real(self.t, op=self.op, group=self.group)
        parts = [torch.empty_like(local) for _ in range(dist.get_world_size(self.group))]
        dist.all_gather(parts, local, group=self.group)
        exp = torch.stack([q.double() for q in parts]).sum(0)
        if self.op == dist.ReduceOp.AVG:
            exp = exp / len(parts)
        err = float((self.t.double() - exp).abs().max() / (exp.abs().max() + 1e-30))
        _DeferredAllReduce.log.append((late, err, self.t.numel()))
        return True


def _intercept(t, op=dist.ReduceOp.SUM, group=None, async_op=False):
    w = _DeferredAllReduce(t, op, group)
    if not async_op:
        w.wait()
        return None
    return w


def _make(arch, **kw):
    kw["num_classes"] = 16
    for extra in ({"dropout": 0.0, "dropout_aux": 0.0}, {"dropout": 0.0}, {}):
        try:
            m = create_model(arch, **kw, **extra)
            break
        except TypeError:
            continue
    for mod in m.modules():  # no dropout anywhere: replicas must see identical math
        if isinstance(mod, torch.nn.Dropout):
            mod.p = 0.0
    return m


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--arch", default="resnet18")
    ap.add_argument("--res", type=int, default=32)
    ap.add_argument("--device", default="cuda", help="cpu: the same check on the CPU path")
    ap.add_argument("--reducer", default="python", choices=["python", "native"],
                    help="python: the interceptable reducer (checks (1)/(2) per bucket); native: "
                         "mipipe._C.Reducer (collectives issued from C++: checks (1)/(2) are "
                         "replaced by the replica comparison and check (3))")
    a = ap.parse_args()
    os.environ["MIPIPE_NATIVE_REDUCER"] = "1" if a.reducer == "native" else "0"
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    dev = torch.device(a.device, 0) if a.device == "cuda" else torch.device("cpu")
    sync = torch.cuda.synchronize if dev.type == "cuda" else (lambda: None)
    torch.manual_seed(0)
    base = _make(a.arch).to(dev)
    refs = []
    for _ in range(2):
        r = _make(a.arch).to(dev)
        r.load_state_dict(base.state_dict())
        refs.append((r, SGD(r.parameters(), 0.05, momentum=0.9, weight_decay=1e-4)))
    # ground truth for the gradient: the same replica on the fp64 CPU path.  Random-init deep
    # nets on tiny per-rank batches are ill-conditioned (BN backward cancellation: a 1e-6 input
    # perturbation moves the fp32 gradient by ~1-2%), so "DDP equals the replica" is judged
    # relative to how far a single-process replica itself lies from this truth.
    truth = _make(a.arch, compute_dtype=torch.float64).double()
    truth.load_state_dict({k: v.cpu() for k, v in base.state_dict().items()})
    model = DistributedDataParallel(base, device_ids=[0] if dev.type == "cuda" else None,
                                    bucket_cap_mb=4, first_bucket_mb=0.5,
                                    check_collectives=True, check_every=1)
    opt = SGD(model.parameters(), 0.05, momentum=0.9, weight_decay=1e-4)
    g = torch.Generator(device=dev)
    g.manual_seed(123)
    B = 16
    for step in range(3):
        xs = torch.randn(world * B, 3, a.res, a.res, device=dev, generator=g)
        ys = torch.randint(0, 16, (world * B,), device=dev, generator=g)
        x, y = xs[rank * B:(rank + 1) * B], ys[rank * B:(rank + 1) * B]
        opt.zero_grad()
        if step == 0:
            dist.all_reduce = _intercept
        try:
            cross_entropy(model(x), y).backward()
        finally:
            dist.all_reduce = _DeferredAllReduce.real
        if step == 0:
            assert model.native_reducer == (a.reducer == "native")
        if step == 0 and a.reducer == "native":
            assert not _DeferredAllReduce.log  # nothing went through the Python collective API
            if rank == 0:
                print(f"step0 native reducer: {len(model.buckets)} buckets issued from C++", flush=True)
        if step == 0 and a.reducer == "python":
            log = _DeferredAllReduce.log
            assert len(log) == len(model.buckets), (len(log), len(model.buckets))
            late = [i for i, (lt, _, _) in enumerate(log) if lt]
            assert not late, f"gradients written after their bucket's all-reduce launched: {late}"
            worst_err = max(e for _, e, _ in log)
            assert worst_err < 1e-5, worst_err
            if rank == 0:
                print(f"step0 bucket check OK: {len(log)} buckets, no late writes, reduced == "
                      f"sum of local gradients (max rel err {worst_err:.1e})", flush=True)
        if step == 0:
            # replicas (and the fp64 truth): average of the per-rank gradients
            for r in [ro[0] for ro in refs] + [truth]:
                rd = next(r.parameters()).device
                for q in r.parameters():
                    q.grad = None
                for k in range(world):
                    xk, yk = xs[k * B:(k + 1) * B].to(rd), ys[k * B:(k + 1) * B].to(rd)
                    if r is truth:
                        xk = xk.double()
                    (cross_entropy(r(xk), yk) / world).backward()
            sync()
            flat_g = lambda m: torch.cat([q.grad.flatten().double().cpu() for q in m.parameters()])  # noqa: E731
            gt, gd, g1, g2 = flat_g(truth), flat_g(base), flat_g(refs[0][0]), flat_g(refs[1][0])
            # the all-reduced gradient must be about as close to the fp64 truth as a
            # single-process replica is, and the replicas must agree with each other
            c_ddp, c_rep, c_self = cos(gd, gt), cos(g1, gt), cos(g1, g2)
            if os.environ.get("DDP_CHECK_VERBOSE") and rank == 0:  # per tensor, backward order
                for (n, p), (_, q) in reversed(list(zip(base.named_parameters(),
                                                        refs[0][0].named_parameters()))):
                    e = float((p.grad.double().cpu() - q.grad.double().cpu()).norm()
                              / (q.grad.double().norm() + 1e-30))
                    print(f"rel err ddp vs replica {e:.3e}  {n}", flush=True)
            conditioned = c_self > 0.99 and c_rep > 0.9
            if conditioned:
                assert 1 - c_ddp <= 3 * (1 - c_rep) + 1e-4, (c_ddp, c_rep, c_self)
            worst = (1.0, "")
            gmax = max(float(q.grad.norm()) for q in truth.parameters())
            for (n, p), (_, q1), (_, t) in zip(base.named_parameters(), refs[0][0].named_parameters(),
                                               truth.named_parameters()):
                if float(t.grad.norm()) < 1e-4 * gmax:
                    continue  # (near-)zero true gradient, e.g. a BN bias feeding conv -> BN
                cd, cr = cos(p.grad, t.grad), cos(q1.grad, t.grad)
                if cd - cr < worst[0] - 1.0 or worst[1] == "":
                    worst = (1.0 + cd - cr, n)
                assert not conditioned or 1 - cd <= 3 * (1 - cr) + 2e-3, (n, cd, cr)
            if rank == 0:
                print(f"step0 gradient vs truth {'OK' if conditioned else '(ill-conditioned: info)'}: cos to fp64 truth ddp {c_ddp:.5f} replica {c_rep:.5f} "
                      f"replica-vs-replica {c_self:.5f}; worst per-tensor gap {1.0 - worst[0]:.2e} "
                      f"at {worst[1]}", flush=True)
        opt.step()
    sync()
    flat = model.space.flat.detach().clone()
    gathered = [torch.empty_like(flat) for _ in range(world)]
    dist.all_gather(gathered, flat)
    assert all(torch.equal(gathered[0], t) for t in gathered), "ranks diverged"
    if rank == 0:
        print(f"DDP gpu check OK ({a.arch}): world={world}, parameters bit-identical across ranks after 3 "
              f"steps, collectives={model._clog.count} oneshot={model._oneshot is not None}",
              flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
