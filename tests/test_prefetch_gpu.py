"""GEMM operand prefetch (mipipe/ops/prefetch.py): a GEMM warming other tensors computes the same
bits; the standalone touch kernel reads and writes nothing visible; the weight order is recorded
over one step and replayed; training results are bit-identical with and without it, eager and
replayed from a captured hipGraph."""
import copy

import pytest
import torch

from mipipe.ops import prefetch
from mipipe.ops._native import native, native_available

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    assert native_available()
    prefetch.reset()
    old = prefetch._MODE
    yield
    prefetch._MODE = old
    prefetch.reset()


def test_touch_kernel_reads_only():
    ts = [torch.randn(n, device="cuda").to(dt) for n, dt in
          [(7, torch.float32), (4096, torch.bfloat16), (1 << 20, torch.float32), (33, torch.bfloat16),
           (3 << 18, torch.bfloat16), (64, torch.float32)]]
    before = [t.clone() for t in ts]
    native().touch(ts)
    torch.cuda.synchronize()
    for a, b in zip(ts, before):
        assert torch.equal(a, b)


@pytest.mark.parametrize("M,N,K,ta,tb", [(4096, 768, 3072, False, True), (640, 768, 768, False, False),
                                         (768, 3072, 512, True, False)])
def test_gemm_with_prefetch_same_bits(M, N, K, ta, tb):
    a = torch.randn(K if ta else M, M if ta else K, device="cuda").to(torch.bfloat16)
    b = torch.randn(N if tb else K, K if tb else N, device="cuda").to(torch.bfloat16)
    warm = [torch.randn(3 << 20, device="cuda").to(torch.bfloat16), torch.randn(999, device="cuda")]
    for odt in (torch.bfloat16, torch.float32):
        y0 = native().gemm(a, b, ta, tb, None, "none", odt, None, 0.0)
        y1 = native().gemm(a, b, ta, tb, None, "none", odt, None, 0.0, -1, None, warm)
        y2 = native().gemm(a, b, ta, tb, None, "none", odt, None, 0.0, -1, None, warm[:1])
        assert torch.equal(y0, y1) and torch.equal(y0, y2)


def _step_fn(m, opt):
    def step(ids, am, pos, labels):
        opt.zero_grad()
        loss = m(ids, am, masked_positions=pos, labels=labels)
        loss.backward()
        opt.step()
        return loss
    return step


def _batch(V, B=2, S=128, P=20):
    g = torch.Generator(device="cuda")
    g.manual_seed(3)
    ids = torch.randint(0, V, (B, S), device="cuda", generator=g)
    am = torch.ones(B, S, device="cuda", dtype=torch.int64)
    pos = torch.stack([torch.randperm(S, device="cuda", generator=g)[:P] for _ in range(B)])
    labels = torch.randint(0, V, (B, P), device="cuda", generator=g)
    return ids, am, pos, labels


def test_prefetch_bit_identical_eager_and_graphed():
    from mipipe.models import create_model
    from mipipe.ops.determinism import deterministic
    from mipipe.optim import AdamW
    from mipipe.train.graph import GraphedStep
    with deterministic(True):
        torch.manual_seed(0)
        a = create_model("bert_tiny").cuda()
        b, c = copy.deepcopy(a), copy.deepcopy(a)
        opts = [AdamW(m.parameters(), lr=1e-3, weight_decay=0.01) for m in (a, b, c)]
        batch = _batch(a.config.vocab_size)
        prefetch._MODE = "0"
        la = [_step_fn(a, opts[0])(*batch).item() for _ in range(4)]
        prefetch.reset()
        prefetch._MODE = "1"  # record (step 1), then prefetch
        lc = [_step_fn(c, opts[2])(*batch).item() for _ in range(4)]
        assert prefetch._S.armed and len(prefetch._S.order) >= 2 * 4  # fwd + data-grad GEMMs
        # (the deep-copied model's tied decoder weight is a per-step cast: a volatile slot)
        assert len(prefetch._S.volatile) <= 2
        assert prefetch._S.cursor == len(prefetch._S.order)
        prefetch.reset()
        gs = GraphedStep(_step_fn(b, opts[1]), batch, warmup=2, inputs=[batch])
        assert prefetch._S.armed
        lb = [gs.warmup_loss.item()] + [gs.replay(0).item() for _ in range(2)]
        torch.cuda.synchronize()
    assert la == lc, (la, lc)
    assert la[1:] == lb, (la, lb)
    for (n, p), (_, q), (_, r) in zip(a.named_parameters(), b.named_parameters(),
                                       c.named_parameters()):
        assert torch.equal(p, r), n  # prefetch off vs on, eager
        assert torch.equal(p, q), n  # vs graph replay with prefetch
