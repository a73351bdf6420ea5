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


def _det_rows_sum(rows):
    """det_sum_rows' fixed order on the CPU in fp32 (IEEE adds, no FMA): long columns (> 256
    rows) as 64-row chunk sums first (4 interleaved groups, then ((g0+g1)+g2)+g3), then 16
    interleaved row groups each summed in row order, then the 16 group sums in index order."""
    rows = rows.float().cpu()
    if rows.shape[0] > 256:
        chunks = []
        for r0 in range(0, rows.shape[0], 64):
            ch = rows[r0:r0 + 64]
            gs = []
            for g in range(4):
                a = torch.zeros(rows.shape[1])
                for p in range(g, ch.shape[0], 4):
                    a = a + ch[p]
                gs.append(a)
            chunks.append(((gs[0] + gs[1]) + gs[2]) + gs[3])
        rows = torch.stack(chunks)
    parts = []
    for g in range(16):
        a = torch.zeros(rows.shape[1])
        for p in range(g, rows.shape[0], 16):
            a = a + rows[p]
        parts.append(a)
    s = torch.zeros(rows.shape[1])
    for a in parts:
        s = s + a
    return s


@pytest.mark.parametrize("P", [5, 16 * 8 + 3, 128, 300, 2048])
@pytest.mark.parametrize("C", [64, 200])
def test_bn_finalize_partial_rows_fixed_order(P, C):
    """Deterministic-mode bn_finalize of P per-tile partial rows (one launch, no det_sum_rows
    into the slab first): the same bits as the slab route — the rows summed in det_sum_rows'
    order into replica row 0 of a zeroed [16, C] slab, then the replica finalize — and within
    fp32 rounding of a float64 evaluation."""
    torch.manual_seed(P + C)
    count = 4096
    s1 = torch.randn(P, C, device=dev) * 3.0
    s2 = torch.rand(P, C, device=dev) * 20.0 + 40.0
    shift = torch.randn(C, device=dev) * 0.1
    gamma, beta = torch.rand(C, device=dev) + 0.5, torch.randn(C, device=dev)
    outs = []
    for route in ("rows", "slab"):
        rm, rv = torch.zeros(C, device=dev), torch.ones(C, device=dev)
        if route == "rows":
            a, b = s1.clone(), s2.clone()
        else:
            R = native().STAT_REPLICAS
            a, b = torch.zeros(R, C, device=dev), torch.zeros(R, C, device=dev)
            a[0], b[0] = _det_rows_sum(s1).to(dev), _det_rows_sum(s2).to(dev)
        outs.append(native().bn_finalize(a, b, count, shift, gamma, beta, rm, rv, 0.1, 1e-5, True,
                                         None) + (rm, rv))
    for x, y in zip(outs[0], outs[1]):
        assert torch.equal(x, y), (x - y).abs().max()
    mean, invstd = outs[0][0].double(), outs[0][1].double()
    ms = s1.double().sum(0) / count
    var = s2.double().sum(0) / count - ms * ms
    assert torch.allclose(mean, ms + shift.double(), rtol=1e-5, atol=1e-5)
    assert torch.allclose(invstd, torch.rsqrt(var + 1e-5), rtol=1e-5)
