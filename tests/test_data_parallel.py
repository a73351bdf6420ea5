"""mipipe's native DataParallel (reference task.py:201-208, path (d)).

Replicas share a device here (``["cpu", "cpu", "cpu"]`` on CPU, ``[0, 0]`` on the 1-GPU box):
that exercises replicate -> scatter -> threaded apply -> gather -> gradient reduction exactly as
with distinct GPUs, except that the collectives take the copy+add tree instead of in-process
RCCL.  The oracle is the unwrapped module run chunk by chunk (per-chunk BatchNorm statistics, as
in torch's DataParallel), concatenated, with the same loss.
"""
import copy

import pytest
import torch

from mipipe.models import create_model
from mipipe.optim import SGD
from mipipe.ops.functional import cross_entropy
from mipipe.parallel import DataParallel
from mipipe.train.task import _unwrap


def _chunked_reference(model, x, y, n):
    out = torch.cat([model(c) for c in x.chunk(n)])
    return out, cross_entropy(out, y)


def _grads(model):
    return [p.grad.detach().clone() for p in model.parameters()]


@pytest.mark.parametrize("flat", [True, False], ids=["mipipe_sgd", "torch_sgd"])
def test_dp_cpu_matches_chunked_module(flat):
    torch.manual_seed(0)
    model = create_model("resnet18", num_classes=10)
    ref = copy.deepcopy(model)
    dp = DataParallel(model, device_ids=["cpu", "cpu", "cpu"])
    mk = (lambda ps: SGD(ps, 0.05, momentum=0.9, weight_decay=1e-4)) if flat else \
        (lambda ps: torch.optim.SGD(ps, 0.05, momentum=0.9, weight_decay=1e-4))
    opt, ropt = mk(dp.parameters()), mk(ref.parameters())
    assert len(list(dp.parameters())) == len(list(model.parameters()))  # replicas not registered
    x = torch.randn(12, 3, 32, 32)
    y = torch.randint(0, 10, (12,))
    for step in range(3):
        # lock-step oracle: BN normalises with a running-mean shift, so replicas (which start
        # from the master's buffers) differ from a sequential chunk loop at ~1e-5, and a
        # batch-4 BN net amplifies that ~100x per SGD step; re-syncing the oracle each step
        # keeps the check exact while still requiring replicas to pick up updated weights
        with torch.no_grad():
            for a, b in zip(ref.state_dict().values(), model.state_dict().values()):
                a.copy_(b)
        opt.zero_grad()
        ropt.zero_grad()
        out = dp(x)
        loss = cross_entropy(out, y)
        loss.backward()
        rout, rloss = _chunked_reference(ref, x, y, 3)
        rloss.backward()
        torch.testing.assert_close(out, rout, rtol=1e-4, atol=1e-4)
        for g, rg in zip(_grads(model), _grads(ref)):
            torch.testing.assert_close(g, rg, rtol=1e-3, atol=1e-3 * float(rg.abs().max()))
        opt.step()
        ropt.step()
    # replica gradient buffers were drained into the master
    for rep in dp._replicas:
        for p in rep.parameters():
            assert p.grad is None or float(p.grad.abs().max()) == 0.0
    assert _unwrap(dp) is model
    assert set(dp.state_dict()) == {"module." + k for k in model.state_dict()}


def test_dp_cpu_uneven_batch_and_eval():
    torch.manual_seed(1)
    model = torch.nn.Sequential(torch.nn.Linear(8, 16), torch.nn.ReLU(), torch.nn.Linear(16, 3))
    ref = copy.deepcopy(model)
    dp = DataParallel(model, device_ids=["cpu"] * 4)
    x = torch.randn(3, 8)  # fewer rows than devices: 3 active replicas
    out = dp(x)
    out.sum().backward()
    ref(x).sum().backward()
    for p, rp in zip(model.parameters(), ref.parameters()):
        torch.testing.assert_close(p.grad, rp.grad)
    with torch.no_grad():
        torch.testing.assert_close(dp(x), ref(x))


def test_dp_single_device_passthrough():
    inner = torch.nn.Sequential(torch.nn.Linear(8, 4), torch.nn.ReLU(), torch.nn.Linear(4, 3))
    dp = DataParallel(inner, device_ids=["cpu"])
    x = torch.randn(5, 8)
    torch.testing.assert_close(dp(x), inner(x))
    assert dp._replicas == []


@pytest.mark.gpu
def test_dp_gpu_replicas_match_per_chunk_copies():
    """bf16 HIP-kernel ResNet-18 under DataParallel([0, 0]) vs one deep copy of the module per
    chunk (what DataParallel computes; deterministic kernels, copies re-synced each step): the
    replica reads its own flat bf16 shadow, writes its own flat gradients, and the reduction sums
    them into the master's.  (A single module looped over both chunks is not the oracle in bf16:
    its second chunk normalises around the running mean the first chunk just moved, and batch-8
    bf16 BatchNorm gradients are sensitive to that at the 10 % level — fp32 agrees to 1e-5;
    measured in round 2.)"""
    from mipipe.ops.determinism import deterministic
    torch.manual_seed(0)
    dev = torch.device("cuda", 0)
    model = create_model("resnet18", num_classes=10).to(dev)
    model.compute_dtype = torch.bfloat16
    copies = [copy.deepcopy(model) for _ in range(2)]
    dp = DataParallel(model, device_ids=[0, 0])
    opt = SGD(dp.parameters(), 0.05, momentum=0.9)
    keep = [SGD(c.parameters(), 0.05) for c in copies]
    x = torch.randn(16, 3, 32, 32, device=dev)
    y = torch.randint(0, 10, (16,), device=dev)
    with deterministic(True):
        for _ in range(3):
            with torch.no_grad():
                for c in copies:
                    for a, b in zip(c.state_dict().values(), model.state_dict().values()):
                        a.copy_(b)
            opt.zero_grad()
            for o in keep:
                o.zero_grad()
            loss = cross_entropy(dp(x), y)
            loss.backward()
            rloss = cross_entropy(torch.cat([c(xc) for c, xc in zip(copies, x.chunk(2))]), y)
            rloss.backward()
            torch.cuda.synchronize()
            lv, rv = float(loss.detach()), float(rloss.detach())
            assert abs(lv - rv) < 1e-4 * max(1.0, abs(rv)), (lv, rv)
            g = torch.cat([p.grad.flatten() for p in model.parameters()])
            rg = sum(torch.cat([p.grad.flatten() for p in c.parameters()]) for c in copies)
            err = float((g - rg).norm() / rg.norm())
            assert err < 1e-3, err
            opt.step()
    rs = dp._rep_spaces[0]
    assert rs is not None and rs.shadow is not None and rs.flat.device == dev
    assert float(rs.flat_grad.abs().max()) == 0.0  # drained into the master
