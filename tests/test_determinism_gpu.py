"""Deterministic mode (reference task.py:25-26 ``cudnn.deterministic = True``): identical runs give
bit-identical parameters; the deterministic reductions agree with the atomic ones numerically."""
import math

import pytest
import torch

from mipipe.ops import determinism
from mipipe.ops import _ref
from mipipe.ops._native import native, native_available

pytestmark = pytest.mark.gpu
dev = "cuda"


@pytest.fixture(autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    assert native_available()
    yield
    determinism.set_deterministic(False)


def _train(arch, dtype, steps=3, batch=32, res=64, seed=0):
    from mipipe.models import create_model
    from mipipe.optim import SGD
    from mipipe.train.task import CrossEntropyLoss
    torch.manual_seed(seed)
    m = create_model(arch, num_classes=10).to(dev)
    m.compute_dtype = dtype
    opt = SGD(m.parameters(), 0.1, momentum=0.9, weight_decay=1e-4,
              shadow_dtype=None if dtype == torch.float32 else "auto")
    g = torch.Generator(device=dev)
    g.manual_seed(123)
    crit = CrossEntropyLoss()
    losses = []
    for _ in range(steps):
        x = torch.randn(batch, 3, res, res, device=dev, generator=g)
        y = torch.randint(0, 10, (batch,), device=dev, generator=g)
        opt.zero_grad()
        loss = crit(m(x), y)
        loss.backward()
        opt.step()
        losses.append(loss.detach().clone())
    torch.cuda.synchronize()
    flat = torch.cat([p.detach().reshape(-1) for p in m.parameters()] +
                     [b.detach().float().reshape(-1) for b in m.buffers()])
    return flat, torch.stack(losses)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("arch", ["resnet18", "resnet50"])
def test_identical_runs_bit_identical(arch, dtype):
    determinism.set_deterministic(True)
    a, la = _train(arch, dtype)
    b, lb = _train(arch, dtype)
    assert torch.equal(la, lb), (la, lb)
    assert torch.equal(a, b), f"{(a != b).sum().item()} of {a.numel()} values differ"


def test_det_reductions_match_atomic():
    torch.manual_seed(7)
    x = torch.randn(16, 28, 28, 64, device=dev).to(torch.bfloat16)
    dy = torch.randn(16, 28, 28, 64, device=dev).to(torch.bfloat16)
    w = (torch.randn(64, 3, 3, 64, device=dev) / 24).to(torch.bfloat16)
    shift = torch.zeros(64, device=dev)
    ref_dw = _ref.conv_wgrad(dy.float(), x.float(), 3, 3, 1, 1)
    determinism.set_deterministic(True)
    dw1 = native().conv_wgrad(dy, x, 3, 3, 1, 1)
    dw2 = native().conv_wgrad(dy, x, 3, 3, 1, 1)
    _, s1, q1 = native().conv_fwd(x, w, 1, 1, shift)
    _, s2, q2 = native().conv_fwd(x, w, 1, 1, shift)
    determinism.set_deterministic(False)
    dw3 = native().conv_wgrad(dy, x, 3, 3, 1, 1)
    _, s3, q3 = native().conv_fwd(x, w, 1, 1, shift)
    assert torch.equal(dw1, dw2) and torch.equal(s1, s2) and torch.equal(q1, q2)
    rel = lambda a, b: ((a - b).abs().max() / b.abs().max()).item()  # noqa: E731
    assert rel(dw1, ref_dw) < 5e-3 and rel(dw1, dw3) < 1e-4
    assert rel(s1.sum(0), s3.sum(0)) < 1e-4 and rel(q1.sum(0), q3.sum(0)) < 1e-4


def test_identical_runs_with_benchmark_mode_on():
    """task.py's default is deterministic AND cudnn.benchmark-style tuning on (reference
    task.py:25 + :244).  Timing-based plan selection would let two runs pick different reduction
    partitions; in deterministic mode the plan must come from a table or the heuristic, so two
    runs that each start from an empty tuning table still agree bit for bit."""
    from mipipe.ops import tuning
    determinism.set_deterministic(True)
    try:
        tuning.clear()
        tuning.set_benchmark(True)
        a, la = _train("resnet18", torch.bfloat16)
        assert not tuning.table(), "deterministic mode must not time-tune"
        tuning.clear()
        b, lb = _train("resnet18", torch.bfloat16)
    finally:
        tuning.set_benchmark(False)
        tuning.clear()
    assert torch.equal(la, lb), (la, lb)
    assert torch.equal(a, b), f"{(a != b).sum().item()} of {a.numel()} values differ"
